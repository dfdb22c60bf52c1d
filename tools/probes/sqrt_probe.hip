// Exhaustive probe: which short sqrt sequences equal the correctly rounded sqrtf (-fhip-fp32-correctly-rounded-divide-sqrt)
// for every positive float?  Prints the mismatch count per range for each candidate.  Investigation tool only (not part
// of the library).
//   raw : v_sqrt_f32 alone (round 1: ~16 % of inputs differ in every binade, profiles/r01k)
//   rsq : r = v_rsq_f32(x); s0 = x * r; s = fma(fma(-s0, s0, x), 0.5 * r, s0)         (one correction step)
//   rcp : s0 = v_sqrt_f32(x); s = fma(fma(-s0, s0, x), v_rcp_f32(s0 + s0), s0)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float cand(int k, float x) {
    if (k == 0) return __builtin_amdgcn_sqrtf(x);
    if (k == 1) {
        const float r = __builtin_amdgcn_rsqf(x);
        const float s0 = x * r;
        return __builtin_fmaf(__builtin_fmaf(-s0, s0, x), 0.5f * r, s0);
    }
    const float s0 = __builtin_amdgcn_sqrtf(x);
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, x), __builtin_amdgcn_rcpf(s0 + s0), s0);
}

__global__ void probe(int k, uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long n = 0;
    for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi && b >= lo; b += stride) {
        const float x = __uint_as_float(b);
        if (__float_as_uint(cand(k, x)) != __float_as_uint(sqrtf(x))) {
            ++n;
            atomicMin(first, b);
        }
        if (b > 0xffffffffu - stride) break;
    }
    if (n) atomicAdd(bad, n);
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 1;
    const struct { const char* name; uint32_t lo, hi; } R[] = {
        {"denormal", 0x00000001u, 0x00800000u},
        {"[2^-126, 2^-100)", 0x00800000u, 0x0d800000u},
        {"[2^-100, 2^-64)", 0x0d800000u, 0x1f800000u},
        {"[2^-64, 2^64)", 0x1f800000u, 0x5f800000u},
        {"[2^64, 2^100)", 0x5f800000u, 0x71800000u},
        {"[2^100, inf)", 0x71800000u, 0x7f800000u},
    };
    const char* names[3] = {"raw", "rsq", "rcp"};
    for (int k = 0; k < 3; ++k)
        for (const auto& r : R) {
            (void)hipMemset(bad, 0, 8);
            (void)hipMemset(first, 0xff, 4);
            hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, k, r.lo, r.hi, bad, first);
            unsigned long long h = 0;
            uint32_t f = 0;
            (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
            std::printf("%s %-18s mismatches %llu first 0x%08x\n", names[k], r.name, h, f);
        }
    return 0;
}
