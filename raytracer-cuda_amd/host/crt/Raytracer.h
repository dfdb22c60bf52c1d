// Raytracer.h — the reference's application loop (CudaRayTracer/src/Raytracer.h:9-102), headless.
//
// The reference polls an SFML window each frame: handleEvents → updateAndRender(deltaTime,
// isRightMousePressed) → drawFrame, sleeping to 60 fps (Raytracer.h:52-71).  updateAndRender moves
// the camera (Camera::updateCamera), uploads it (CUDARenderer::updateCamera) and renders one frame
// with the camera's spp: 1 while idle or moving, 2000 in high-quality mode (F).  Every pixel's
// curandState persists across frames (CUDAKernels.h:165 stores it back), so consecutive 1-spp frames
// continue the same per-pixel random streams.
//
// Here the window is replaced by an InputState per frame (a script or an FFI caller) and drawFrame by
// the renderer's RGBA8 buffer (CUDARenderer::getImageData; ImageIO writes files).  Frames are timed
// instead of throttled.  `accumulate` is an addition the reference does not have: while the camera is
// still, 1-spp frames add into the linear sum and resolve with 1/(samples so far), so the image
// converges progressively; any camera motion (or a high-quality frame) restarts the sum.  K
// accumulated 1-spp frames equal one K-spp frame bit for bit (same per-pixel sample order).
#pragma once
#include <chrono>
#include <string>
#include <vector>

#include "CUDARenderer.h"
#include "Camera.h"
#include "SceneManager.h"

namespace CRT {

struct RaytracerOptions {
    std::vector<std::string> modelFiles;   // empty = SceneManager's default list
    crt_scene_options scene{};             // CRT_BVH_REFERENCE (bit-exact) by default
    unsigned long long seed = 41;          // the reference seeds with rand() (41 under MSVC)
    int device = 0;
    // Camera pose.  The reference's initializeScene puts the camera at (0,4,4) with focus |pos - target| and
    // yaw -90 (Raytracer.h:77-86), which frames only sky and ground for the Cornell scene.
    bool hasPose = false;
    Vec3 position{0.f, 4.f, 4.f};
    float focusDist = 0.f;                  // <= 0: |position - (0,0,0)|, the reference's rule
    bool accumulate = false;
    int meshBuildDevice = -1;              // >= 0: mesh BVHs built on that GPU (same trees, SceneManager)
    // variant 7 (the < 64-spp frames of the loop) dispatches its tiles most expensive first by the previous frame's rays
    // per pixel (crt_renderer_set_temporal_order): consecutive frames share the cost map; results never depend on it
    bool temporalOrder = true;
    // variant 7's regeneration threshold once its pixel queue is empty (crt_renderer_set_drain_threshold; 0 = unchanged)
    int drainThreshold = 0;
};

struct FrameInfo {
    long long frame = 0;        // frames rendered so far, this one included
    int spp = 0;                // samples traced this frame (Camera::m_SamplesPerPixel)
    int accumulated = 0;        // samples in the displayed image (== spp unless accumulating)
    bool moving = false;        // Camera::isCameraInMotion
    bool highQuality = false;
    float kernelMs = 0.f;       // render kernel, HIP events
    double frameMs = 0.0;       // updateAndRender wall clock (camera update + upload + render + resolve + sync)
};

class Raytracer {
public:
    // Raytracer::Raytracer + initializeScene (Raytracer.h:38-47, :77-92)
    Raytracer(int width, int height, float aspectRatio, float verticalFOV, float aperture,
              const RaytracerOptions& opts = RaytracerOptions())
        : m_Width(width), m_Height(height), m_AspectRatio(aspectRatio), m_VerticalFOV(verticalFOV),
          m_Aperture(aperture), m_Options(opts), m_SceneManager(width, height, opts.device),
          m_Renderer(width, height, opts.device) {
        initializeScene();
        CRT_CHECK(crt_renderer_set_temporal_order(m_Renderer.handle(), opts.temporalOrder ? 1 : 0));
        CRT_CHECK(crt_renderer_set_drain_threshold(m_Renderer.handle(), opts.drainThreshold));
    }

    // Raytracer::updateAndRender (Raytracer.h:94-102) for one frame of input.
    FrameInfo updateAndRender(float deltaTime, const InputState& in) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < in.focusSteps; ++k) m_Camera.adjustFocusDistance(0.1f);    // WindowManager.h:64-67
        for (int k = 0; k > in.focusSteps; --k) m_Camera.adjustFocusDistance(-0.1f);
        m_Camera.updateCamera(deltaTime, m_Width, m_Height, in);
        m_Renderer.updateCamera(m_Camera);
        FrameInfo fi;
        fi.spp = m_Camera.m_SamplesPerPixel;
        fi.moving = m_Camera.isCameraInMotion();
        fi.highQuality = m_Camera.isHighQuality();
        crt_renderer* r = m_Renderer.handle();
        const bool keep = m_Options.accumulate && !fi.moving && !fi.highQuality && in.focusSteps == 0 && m_Accumulated > 0;
        if (!m_Options.accumulate) {
            m_Renderer.render(m_SceneManager.getBVHNodes(), m_SceneManager.getWorld());   // CUDARenderer::render
            m_Accumulated = fi.spp;
        } else {
            const bool still = !fi.moving && !fi.highQuality;
            CRT_CHECK(crt_renderer_render(r, m_SceneManager.getBVHNodes(), fi.spp, 20, keep ? CRT_RENDER_ACCUMULATE : 0u,
                                          nullptr));
            m_Accumulated = keep ? m_Accumulated + fi.spp : fi.spp;
            CRT_CHECK(crt_renderer_resolve(r, 1.f / (float)m_Accumulated, nullptr));
            CRT_CHECK(crt_renderer_synchronize(r, nullptr));
            if (!still) m_Accumulated = 0;   // a moving / high-quality frame is shown once, never added to
        }
        fi.accumulated = m_Accumulated > 0 ? m_Accumulated : fi.spp;
        fi.kernelMs = crt_renderer_last_kernel_ms(r);
        fi.frame = ++m_Frame;
        fi.frameMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return fi;
    }

    // Raytracer::run (Raytracer.h:52-71) without the window: `input(frame)` supplies each frame's
    // deltaTime and InputState, `display(info)` stands in for drawFrame.
    template <class InputFn, class DisplayFn>
    void run(long long frames, InputFn input, DisplayFn display) {
        for (long long f = 0; f < frames; ++f) {
            float dt = 0.f;
            InputState in = input(f, &dt);
            display(updateAndRender(dt, in));
        }
    }

    const Camera& camera() const { return m_Camera; }
    HIPRenderer& renderer() { return m_Renderer; }
    SceneManager& sceneManager() { return m_SceneManager; }
    int width() const { return m_Width; }
    int height() const { return m_Height; }

private:
    void initializeScene() {
        const Vec3 target(0, 0, 0), worldY(0, 1, 0);
        const Vec3 pos = m_Options.hasPose ? m_Options.position : Vec3(0, 4, 4);
        const float focus = m_Options.focusDist > 0.f ? m_Options.focusDist : (pos - target).length();
        m_Camera = Camera(m_AspectRatio, m_VerticalFOV, pos, target, worldY, m_Aperture, focus);
        auto config = CUDAHelpers::createRenderConfig(m_Width, m_Height);
        m_Renderer.initialize(config, m_Options.seed);
        if (!m_Options.modelFiles.empty()) m_SceneManager.setModelFiles(m_Options.modelFiles);
        m_SceneManager.setSceneOptions(m_Options.scene);
        m_SceneManager.setMeshBuildDevice(m_Options.meshBuildDevice);
        m_SceneManager.initializeScene(config, m_Renderer.getRandState());
    }

    int m_Width, m_Height;
    float m_AspectRatio, m_VerticalFOV, m_Aperture;
    RaytracerOptions m_Options;
    Camera m_Camera;
    SceneManager m_SceneManager;
    HIPRenderer m_Renderer;
    long long m_Frame = 0;
    int m_Accumulated = 0;
};

}  // namespace CRT
