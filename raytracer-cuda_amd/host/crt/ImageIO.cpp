// ImageIO.cpp — PNG / PPM encoders for the framebuffer (see ImageIO.h).
#include "ImageIO.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace CRT {
namespace {

// ---- checksums (PNG chunk CRC-32, zlib Adler-32) ----
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0) {
    static uint32_t table[256];
    static bool ready = false;
    if (!ready) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xedb88320u ^ (v >> 1) : v >> 1;
            table[i] = v;
        }
        ready = true;
    }
    c = ~c;
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}

uint32_t adler32(const uint8_t* p, size_t n) {
    uint32_t a = 1, b = 0;
    while (n) {
        size_t k = n < 5552 ? n : 5552;   // largest block before the sums can overflow 32 bits
        n -= k;
        while (k--) { a += *p++; b += a; }
        a %= 65521u;
        b %= 65521u;
    }
    return (b << 16) | a;
}

// ---- deflate, fixed Huffman codes (RFC 1951 §3.2.6) ----
class BitWriter {
public:
    explicit BitWriter(std::vector<uint8_t>& out) : out_(out) {}
    void bits(uint32_t v, int n) {          // LSB first
        acc_ |= (uint64_t)v << nacc_;
        nacc_ += n;
        while (nacc_ >= 8) { out_.push_back((uint8_t)acc_); acc_ >>= 8; nacc_ -= 8; }
    }
    void huff(uint32_t code, int n) {       // Huffman codes are packed MSB first
        uint32_t r = 0;
        for (int i = 0; i < n; ++i) r |= ((code >> i) & 1u) << (n - 1 - i);
        bits(r, n);
    }
    void flush() { if (nacc_) { out_.push_back((uint8_t)acc_); acc_ = 0; nacc_ = 0; } }

private:
    std::vector<uint8_t>& out_;
    uint64_t acc_ = 0;
    int nacc_ = 0;
};

void putLiteralLength(BitWriter& bw, int sym) {
    if (sym < 144) bw.huff(0x30 + sym, 8);
    else if (sym < 256) bw.huff(0x190 + (sym - 144), 9);
    else if (sym < 280) bw.huff(sym - 256, 7);
    else bw.huff(0xc0 + (sym - 280), 8);
}

const int kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                          35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const int kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const int kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                           257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const int kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

void putMatch(BitWriter& bw, int len, int dist) {
    int li = 28;
    while (kLenBase[li] > len) --li;
    putLiteralLength(bw, 257 + li);
    if (kLenExtra[li]) bw.bits(len - kLenBase[li], kLenExtra[li]);
    int di = 29;
    while (kDistBase[di] > dist) --di;
    bw.huff(di, 5);
    if (kDistExtra[di]) bw.bits(dist - kDistBase[di], kDistExtra[di]);
}

// One final fixed-Huffman block; greedy LZ77 over a 32 KiB window with short hash chains.
std::vector<uint8_t> zlibCompress(const std::vector<uint8_t>& in) {
    std::vector<uint8_t> out = {0x78, 0x01};    // CM 8, 32 KiB window, FCHECK: 0x7801 % 31 == 0
    BitWriter bw(out);
    bw.bits(1, 1);   // BFINAL
    bw.bits(1, 2);   // BTYPE 01 = fixed Huffman
    constexpr int WINDOW = 32768, HBITS = 15, CHAIN = 16, MAXLEN = 258;
    std::vector<int32_t> head(1 << HBITS, -1), prev(in.size() > 0 ? in.size() : 1, -1);
    const size_t n = in.size();
    auto hash = [&](size_t i) {
        return (uint32_t)(((in[i] << 16) | (in[i + 1] << 8) | in[i + 2]) * 2654435761u) >> (32 - HBITS);
    };
    auto insert = [&](size_t i) {
        if (i + 2 >= n) return;
        uint32_t h = hash(i);
        prev[i] = head[h];
        head[h] = (int32_t)i;
    };
    size_t i = 0;
    while (i < n) {
        int best = 0, bestDist = 0;
        if (i + 2 < n) {
            int32_t cand = head[hash(i)];
            const int maxLen = (int)std::min<size_t>(MAXLEN, n - i);
            for (int c = 0; c < CHAIN && cand >= 0 && (int)(i - cand) <= WINDOW; ++c, cand = prev[cand]) {
                int l = 0;
                while (l < maxLen && in[cand + l] == in[i + l]) ++l;
                if (l > best) { best = l; bestDist = (int)(i - cand); if (l == maxLen) break; }
            }
        }
        if (best >= 3) {
            putMatch(bw, best, bestDist);
            for (int k = 0; k < best; ++k) insert(i + k);
            i += best;
        } else {
            putLiteralLength(bw, in[i]);
            insert(i);
            ++i;
        }
    }
    putLiteralLength(bw, 256);   // end of block
    bw.flush();
    const uint32_t a = adler32(in.data(), in.size());
    for (int s = 24; s >= 0; s -= 8) out.push_back((uint8_t)(a >> s));
    return out;
}

void putU32BE(std::vector<uint8_t>& v, uint32_t x) {
    for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}

void putChunk(std::vector<uint8_t>& png, const char type[4], const std::vector<uint8_t>& data) {
    putU32BE(png, (uint32_t)data.size());
    const size_t at = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), data.begin(), data.end());
    putU32BE(png, crc32(png.data() + at, png.size() - at));
}

uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (uint8_t)((pa <= pb && pa <= pc) ? a : pb <= pc ? b : c);
}

void checkArgs(const uint8_t* rgba, int w, int h) {
    if (!rgba || w <= 0 || h <= 0) throw std::runtime_error("image: bad arguments");
}

}  // namespace

std::vector<uint8_t> encodePNG(const uint8_t* rgba, int w, int h, bool flip) {
    checkArgs(rgba, w, h);
    const size_t stride = (size_t)w * 3;
    std::vector<uint8_t> raw;
    raw.reserve((stride + 1) * h);
    std::vector<uint8_t> cur(stride), up(stride, 0), trial(stride), best(stride);
    for (int r = 0; r < h; ++r) {
        const int src = flip ? h - 1 - r : r;   // WindowManager.h:88 flipVertically
        const uint8_t* p = rgba + (size_t)src * w * 4;
        for (int x = 0; x < w; ++x)
            for (int c = 0; c < 3; ++c) cur[3 * x + c] = p[4 * x + c];
        long bestCost = -1;
        int bestType = 0;
        for (int type = 0; type < 5; ++type) {
            long cost = 0;
            for (size_t i = 0; i < stride; ++i) {
                const int a = i >= 3 ? cur[i - 3] : 0, b = up[i], c = i >= 3 ? up[i - 3] : 0;
                int pred = 0;
                switch (type) {
                    case 1: pred = a; break;
                    case 2: pred = b; break;
                    case 3: pred = (a + b) >> 1; break;
                    case 4: pred = paeth(a, b, c); break;
                    default: break;
                }
                trial[i] = (uint8_t)(cur[i] - pred);
                cost += trial[i] < 128 ? trial[i] : 256 - trial[i];
            }
            if (bestCost < 0 || cost < bestCost) { bestCost = cost; bestType = type; best.swap(trial); }
        }
        raw.push_back((uint8_t)bestType);
        raw.insert(raw.end(), best.begin(), best.end());
        up.swap(cur);
    }
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    putU32BE(ihdr, (uint32_t)w);
    putU32BE(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit RGB, deflate, adaptive filtering, no interlace
    putChunk(png, "IHDR", ihdr);
    putChunk(png, "IDAT", zlibCompress(raw));
    putChunk(png, "IEND", {});
    return png;
}

std::vector<uint8_t> encodePPM(const uint8_t* rgba, int w, int h, bool flip) {
    checkArgs(rgba, w, h);
    char hdr[64];
    const int k = std::snprintf(hdr, sizeof hdr, "P6\n%d %d\n255\n", w, h);
    std::vector<uint8_t> out(hdr, hdr + k);
    out.reserve(k + (size_t)w * h * 3);
    for (int r = 0; r < h; ++r) {
        const uint8_t* p = rgba + (size_t)(flip ? h - 1 - r : r) * w * 4;
        for (int x = 0; x < w; ++x) out.insert(out.end(), p + 4 * x, p + 4 * x + 3);
    }
    return out;
}

void writeImage(const std::string& path, const uint8_t* rgba, int w, int h, bool flip) {
    const auto dot = path.find_last_of('.');
    std::string ext = dot == std::string::npos ? "" : path.substr(dot + 1);
    for (char& c : ext) c = (char)std::tolower((unsigned char)c);
    std::vector<uint8_t> bytes;
    if (ext == "png") bytes = encodePNG(rgba, w, h, flip);
    else if (ext == "ppm") bytes = encodePPM(rgba, w, h, flip);
    else throw std::runtime_error("image: unsupported extension (use .png or .ppm): " + path);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("image: cannot open " + path);
    const size_t wrote = std::fwrite(bytes.data(), 1, bytes.size(), f);
    const int closed = std::fclose(f);
    if (wrote != bytes.size() || closed != 0) throw std::runtime_error("image: short write to " + path);
}

}  // namespace CRT
