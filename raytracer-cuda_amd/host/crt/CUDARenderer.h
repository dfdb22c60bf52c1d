// CUDARenderer.h — the reference's renderer facade (CudaRayTracer/src/CUDARenderer.cuh:9-60)
// with the same method names, implemented over the C ABI of libcrt_hip.so.
// `HIPRenderer` is the class; `CUDARenderer` is kept as an alias so reference host code
// (Raytracer.h:77-102) compiles unchanged.
#pragma once
#include <cstdint>
#include <vector>

#include "Camera.h"
#include "CUDAHelpers.h"
#include "crt_hip.h"

class HIPRenderer {
public:
    HIPRenderer(int width, int height, int device = 0) : m_Width(width), m_Height(height), m_Device(device) {}
    ~HIPRenderer() { if (m_R) crt_renderer_destroy(m_R); }
    HIPRenderer(const HIPRenderer&) = delete;
    HIPRenderer& operator=(const HIPRenderer&) = delete;

    // CUDARenderer::initialize (CUDARenderer.cuh:39-49): allocate image + RNG, curand_init per pixel.
    // The reference seeds with rand() (41 on MSVC, the reference platform); the seed is explicit here.
    void initialize(const CUDAHelpers::RenderConfig& config, unsigned long long seed = 41ull,
                    unsigned long long subsequenceBase = 0ull) {
        m_Config = config;
        if (!m_R) CRT_CHECK(crt_renderer_create(m_Width, m_Height, m_Device, &m_R));
        CRT_CHECK(crt_renderer_init_rand(m_R, seed, subsequenceBase, nullptr));
        CRT_CHECK(crt_renderer_synchronize(m_R, nullptr));
    }
    // CUDARenderer::updateCamera (:51-53)
    void updateCamera(const CRT::Camera& camera) {
        m_Camera = camera.toDesc();
        CRT_CHECK(crt_renderer_set_camera(m_R, &m_Camera));
    }
    // CUDARenderer::render (:55-60): one frame, camera spp, 20 bounces, synchronous.
    void render(crt_scene* bvhNodes, crt_scene* world) {
        (void)world;
        CRT_CHECK(crt_renderer_render_frame(m_R, bvhNodes, nullptr));
    }
    // Device pointers, like getImageData()/getRandState() (:16-17).
    uint8_t* getImageData() const { return crt_renderer_rgba_device_ptr(m_R); }
    uint32_t* getRandState() const { return crt_renderer_rng_device_ptr(m_R); }
    float* getLinearSum() const { return crt_renderer_linear_device_ptr(m_R); }
    crt_renderer* handle() const { return m_R; }

    std::vector<uint8_t> readImage() const {
        std::vector<uint8_t> img((size_t)m_Width * m_Height * 4);
        CRT_CHECK(crt_renderer_read_rgba8(m_R, img.data()));
        return img;
    }

private:
    int m_Width, m_Height, m_Device;
    CUDAHelpers::RenderConfig m_Config;
    crt_camera_desc m_Camera{};
    crt_renderer* m_R = nullptr;
};

using CUDARenderer = HIPRenderer;
