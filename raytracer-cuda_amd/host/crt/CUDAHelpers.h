// CUDAHelpers.h — the reference's launch-config / error helpers (CudaRayTracer/src/CUDAHelpers.h:9-35)
// kept under the same names so reference host code compiles unchanged.  Errors from the
// C ABI are reported like CUDA_CHECK: print, then throw std::runtime_error.
#pragma once
#include <iostream>
#include <stdexcept>
#include <string>

#include "crt_hip.h"

#define CRT_CHECK(val) CUDAHelpers::checkCrt((val), #val, __FILE__, __LINE__)
#define CUDA_CHECK(val) CRT_CHECK(val)

namespace CUDAHelpers {

struct Dim3 {
    unsigned x = 1, y = 1, z = 1;
    Dim3() = default;
    Dim3(unsigned a, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};

struct RenderConfig {   // CUDAHelpers.h:10-14
    Dim3 threads;
    Dim3 blocks;
    int totalThreads = 0;
};

inline void checkCrt(int result, char const* const func, const char* const file, int const line) {
    if (result != CRT_OK) {
        std::cerr << "CRT error = " << result << " at " << file << ":" << line << " '" << func << "': "
                  << crt_last_error() << "\n";
        throw std::runtime_error(std::string("CRT error: ") + crt_last_error());
    }
}

constexpr int THREADS_PER_BLOCK = 16;   // CUDAHelpers.h:28
inline RenderConfig createRenderConfig(int width, int height) {
    RenderConfig c;
    c.threads = Dim3(THREADS_PER_BLOCK, THREADS_PER_BLOCK);
    c.blocks = Dim3((width + THREADS_PER_BLOCK - 1) / THREADS_PER_BLOCK, (height + THREADS_PER_BLOCK - 1) / THREADS_PER_BLOCK);
    c.totalThreads = (int)(c.blocks.x * c.blocks.y * c.threads.x * c.threads.y);
    return c;
}

}  // namespace CUDAHelpers
