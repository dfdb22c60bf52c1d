// crt_viewer — the reference's interactive loop (EntryPoint.cu:14-42 → Raytracer::run, Raytracer.h:52-102)
// without a window: a scripted input stream drives Raytracer::updateAndRender frame after frame and the
// frame times are reported (the reference throttles to 60 fps; here frames run back to back).
//
//   crt_viewer [-w W] [-h H] [-frames N] [-script still|walk|orbit|hq] [-bvh reference|rebuilt]
//              [-accumulate] [-no-temporal] [-drain LANES] [-seed S] [-o last.png] model.obj...
//
// Scripts: still = no input (1 spp per frame, RNG continues); walk = W held; orbit = right mouse dragged
// in a circle; hq = F pressed once, then still (2000 spp frames).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "crt/ImageIO.h"
#include "crt/Raytracer.h"

int main(int argc, char** argv) {
    try {
        int W = 2560, H = -1;
        long long frames = 240;
        std::string script = "still", out;
        CRT::RaytracerOptions opts;
        opts.hasPose = true;                          // the bench pose that frames the Cornell box
        opts.position = CRT::Vec3(0.f, 0.f, 0.3f);
        opts.focusDist = 0.3f;
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            auto need = [&](int k) { if (i + k >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); } };
            if (a == "-w") { need(1); W = std::atoi(argv[++i]); }
            else if (a == "-h") { need(1); H = std::atoi(argv[++i]); }
            else if (a == "-frames") { need(1); frames = std::atoll(argv[++i]); }
            else if (a == "-script") { need(1); script = argv[++i]; }
            else if (a == "-seed") { need(1); opts.seed = std::strtoull(argv[++i], nullptr, 10); }
            else if (a == "-o") { need(1); out = argv[++i]; }
            else if (a == "-accumulate") opts.accumulate = true;
            else if (a == "-no-temporal") opts.temporalOrder = false;
            else if (a == "-drain") { need(1); opts.drainThreshold = std::atoi(argv[++i]); }
            else if (a == "-bvh") {
                need(1);
                std::string m = argv[++i];
                opts.scene.bvh = m == "rebuilt" ? CRT_BVH_REBUILT : CRT_BVH_REFERENCE;
            }
            else opts.modelFiles.push_back(a);
        }
        const float ASPECT_RATIO = 16.0f / 9.0f;      // EntryPoint.cu:16-20
        if (H < 0) H = static_cast<int>(W / ASPECT_RATIO);
        if (opts.modelFiles.empty()) opts.modelFiles = {"assets/models/CornellBox-Original.obj", "assets/models/bunny.obj"};
        if (script != "still" && script != "walk" && script != "orbit" && script != "hq")
            throw std::runtime_error("unknown script " + script);

        CRT::Raytracer rt(W, H, ASPECT_RATIO, 80.0f, 0.000001f, opts);
        const float dt = 1.0f / 60.0f;
        auto input = [&](long long f, float* dtOut) {
            *dtOut = dt;
            CRT::InputState in;
            if (script == "walk") in.keyW = (f / 60) % 2 == 0;           // walk 1 s, stand 1 s
            else if (script == "orbit") {
                const float a = 0.05f * (float)f;
                in.rightMouse = true;
                in.mouseX = W * 0.5f + 40.f * std::cos(a);
                in.mouseY = H * 0.5f + 40.f * std::sin(a);
            } else if (script == "hq") in.keyF = f == 0;
            return in;
        };
        std::vector<double> frameMs, kernelMs;
        long long samples = 0;
        CRT::FrameInfo last;
        rt.run(frames, input, [&](const CRT::FrameInfo& fi) {
            frameMs.push_back(fi.frameMs);
            kernelMs.push_back(fi.kernelMs);
            samples += fi.spp;
            last = fi;
        });
        if (!out.empty()) {
            std::vector<uint8_t> img = rt.renderer().readImage();
            CRT::writeImage(out, img.data(), W, H, true);
        }
        std::vector<double> s = frameMs;
        std::sort(s.begin(), s.end());
        double tot = 0, ktot = 0;
        for (double v : frameMs) tot += v;
        for (double v : kernelMs) ktot += v;
        const size_t n = s.size();
        auto pct = [&](double p) { return n ? s[std::min(n - 1, (size_t)(p * (n - 1) + 0.5))] : 0.0; };
        std::printf("{\"width\": %d, \"height\": %d, \"script\": \"%s\", \"bvh\": \"%s\", \"accumulate\": %s, "
                    "\"temporal\": %s, \"drain\": %d, \"frames\": %lld, \"fps\": %.1f, \"frame_ms_mean\": %.3f, \"frame_ms_p50\": %.3f, "
                    "\"frame_ms_p99\": %.3f, \"kernel_ms_mean\": %.3f, \"samples_per_pixel_total\": %lld, "
                    "\"paths_per_s\": %.4g, \"last_accumulated\": %d}\n",
                    W, H, script.c_str(), opts.scene.bvh == CRT_BVH_REBUILT ? "rebuilt" : "reference",
                    opts.accumulate ? "true" : "false", opts.temporalOrder ? "true" : "false", opts.drainThreshold, frames, n ? 1000.0 * n / tot : 0.0, n ? tot / n : 0.0,
                    pct(0.5), pct(0.99), n ? ktot / n : 0.0, samples,
                    tot > 0 ? (double)W * H * samples / (tot / 1e3) : 0.0, last.accumulated);
        return EXIT_SUCCESS;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n", e.what());
        return EXIT_FAILURE;
    }
}
