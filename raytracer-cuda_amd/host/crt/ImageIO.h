// ImageIO.h — frame output for the headless renderer.
//
// The reference shows its RGBA8 framebuffer in an SFML window: WindowManager::drawFrame
// (WindowManager.h:79-93) copies the device image to the host and flips it vertically,
// because row 0 of the framebuffer is the BOTTOM row (Camera::getRay, Camera.cuh:32-44,
// maps y = 0 to the lower-left corner).  Headless, the same bytes go to a file instead:
// flipVertically = true reproduces what the window shows.  Alpha (always 255,
// CRTUtility.cuh:34-38) is dropped; the files are 8-bit RGB.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace CRT {

// PNG (colour type 2, 8 bit): per-row adaptive filter (None/Sub/Up/Average/Paeth, minimum
// sum of absolute residuals), zlib stream of fixed-Huffman deflate blocks with greedy LZ77.
std::vector<uint8_t> encodePNG(const uint8_t* rgba, int width, int height, bool flipVertically = true);
// Binary PPM (P6).
std::vector<uint8_t> encodePPM(const uint8_t* rgba, int width, int height, bool flipVertically = true);
// Writes PNG or PPM by the file extension (.png / .ppm); throws std::runtime_error.
void writeImage(const std::string& path, const uint8_t* rgba, int width, int height, bool flipVertically = true);

}  // namespace CRT
