// crt_render — headless equivalent of the reference's EntryPoint.cu:14-42 + Raytracer.h:77-102:
// build the scene with SceneManager, set the camera, render one frame with CUDARenderer and
// write it as PNG or binary PPM by extension (rows flipped like WindowManager::drawFrame's flipVertically).
//
//   crt_render [-w W] [-h H] [-spp N] [-seed S] [-o out.ppm] [-pos x y z] [-fov deg] [-bvh reference|rebuilt]
//              [-leaf N] [-sbvh] model.obj...       (-sbvh: rebuilt tree with spatial splits)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "crt/CUDARenderer.h"
#include "crt/Camera.h"
#include "crt/ImageIO.h"
#include "crt/SceneManager.h"

int main(int argc, char** argv) {
    try {
        int W = 2560, spp = 1;
        int H = -1;
        unsigned long long seed = 41;
        float fov = 80.0f, aperture = 0.000001f;
        float pos[3] = {0.f, 0.f, 0.3f};
        std::string out = "frame.png";
        std::vector<std::string> files;
        crt_scene_options opts{};
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            auto need = [&](int k) { if (i + k >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); } };
            if (a == "-w") { need(1); W = std::atoi(argv[++i]); }
            else if (a == "-h") { need(1); H = std::atoi(argv[++i]); }
            else if (a == "-spp") { need(1); spp = std::atoi(argv[++i]); }
            else if (a == "-seed") { need(1); seed = std::strtoull(argv[++i], nullptr, 10); }
            else if (a == "-o") { need(1); out = argv[++i]; }
            else if (a == "-fov") { need(1); fov = (float)std::atof(argv[++i]); }
            else if (a == "-pos") { need(3); for (float& p : pos) p = (float)std::atof(argv[++i]); }
            else if (a == "-bvh") { need(1); std::string m = argv[++i]; opts.bvh = m == "rebuilt" ? CRT_BVH_REBUILT : CRT_BVH_REFERENCE; }
            else if (a == "-leaf") { need(1); opts.leaf_size = std::atoi(argv[++i]); }
            else if (a == "-sbvh") { opts.bvh = CRT_BVH_REBUILT; opts.spatial_splits = 1; }
            else files.push_back(a);
        }
        const float ASPECT_RATIO = 16.0f / 9.0f;                 // EntryPoint.cu:16-20
        if (H < 0) H = static_cast<int>(W / ASPECT_RATIO);
        if (files.empty()) files = {"assets/models/CornellBox-Original.obj", "assets/models/bunny.obj"};

        CRT::Camera camera(ASPECT_RATIO, fov, CRT::Vec3(pos[0], pos[1], pos[2]), CRT::Vec3(0, 0, 0), CRT::Vec3(0, 1, 0),
                           aperture, 0.3f);
        camera.setSamplesPerPixel(spp);
        auto config = CUDAHelpers::createRenderConfig(W, H);
        SceneManager scene(W, H);
        scene.setModelFiles(files);
        scene.setSceneOptions(opts);
        CUDARenderer renderer(W, H);
        auto t0 = std::chrono::steady_clock::now();
        renderer.initialize(config, seed);
        scene.initializeScene(config, renderer.getRandState());
        auto t1 = std::chrono::steady_clock::now();
        renderer.updateCamera(camera);
        renderer.render(scene.getBVHNodes(), scene.getWorld());
        auto t2 = std::chrono::steady_clock::now();
        crt_work_counters c{};
        CRT_CHECK(crt_renderer_get_counters(renderer.handle(), &c));
        std::vector<uint8_t> img = renderer.readImage();
        CRT::writeImage(out, img.data(), W, H, true);   // flipVertically (WindowManager.h:88); .png or .ppm
        double setup = std::chrono::duration<double>(t1 - t0).count();
        double frame = std::chrono::duration<double>(t2 - t1).count();
        std::printf("{\"width\": %d, \"height\": %d, \"spp\": %d, \"rays\": %llu, \"setup_s\": %.4f, \"frame_s\": %.4f, "
                    "\"kernel_ms\": %.3f, \"mrays_per_s\": %.2f, \"out\": \"%s\"}\n",
                    W, H, spp, (unsigned long long)c.rays, setup, frame, crt_renderer_last_kernel_ms(renderer.handle()),
                    c.rays / frame / 1e6, out.c_str());
        return EXIT_SUCCESS;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n", e.what());
        return EXIT_FAILURE;
    }
}
