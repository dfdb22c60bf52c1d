// Exhaustive probe: is raw v_sqrt_f32 (__builtin_amdgcn_sqrtf) correctly rounded on this GPU, i.e. equal to the
// compiler's correctly rounded sqrtf (-fhip-fp32-correctly-rounded-divide-sqrt) for every positive float?
// Prints the mismatch count per binade range.  Investigation tool only (not part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long n = 0;
    for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi && b >= lo; b += stride) {
        const float x = __uint_as_float(b);
        if (__float_as_uint(__builtin_amdgcn_sqrtf(x)) != __float_as_uint(sqrtf(x))) {
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
        {"[2^-126, 2^-64)", 0x00800000u, 0x1f800000u},
        {"[2^-64, 2^64)", 0x1f800000u, 0x5f800000u},
        {"[2^64, inf)", 0x5f800000u, 0x7f800000u},
    };
    for (const auto& r : R) {
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(first, 0xff, 4);
        hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, r.lo, r.hi, bad, first);
        unsigned long long h = 0;
        uint32_t f = 0;
        (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
        std::printf("%-18s mismatches %llu first 0x%08x\n", r.name, h, f);
    }
    return 0;
}
