// l1_probe.hip — vector-L1 (TCP) calibration micro-benchmark for the render kernel's roofline.
//
// The render kernel's per-lane node and triangle gathers are served by the vector L1 / L2, not HBM.
// Its binding resource is therefore read from TCP_TOTAL_CACHE_ACCESSES (tag lookups) per CU-cycle, and that needs a
// peak: this probe issues global_load_dwordx4 wave-instructions of known shapes against an L1-resident table (16 KiB
// per workgroup region) and reports, per kernel, the load instructions issued and the time; rocprofv3 --pmc on the
// same binary gives the lookups (TCP_TOTAL_CACHE_ACCESSES) and cycles (GRBM_GUI_ACTIVE), so
//   lookups per instruction  -> the L1 line size and how lookups count for each access shape;
//   lookups per CU-cycle     -> the peak rate of the fully divergent shape (the render kernel's shape).
// Shapes (64 lanes, 16 B each; the record shapes are in main()):
//   coalesced : lane l reads bytes [16 l, 16 l + 16) of a 1 KiB row           (1 KiB contiguous per instruction)
//   stride64  : lane l reads 16 B at 64 l                                      (4 KiB span, 2 lanes per 128-B line)
//   stride128 : lane l reads 16 B at 128 l                                     (64 distinct 128-B lines)
//   random    : lane l reads 16 B at a pseudo-random 16-B slot of the 16 KiB table
//   node128   : lanes read the 7 x 16 B of a pseudo-random 128-B record (the 4-wide node load, 7 instructions)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/l1_probe tools/probes/l1_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                           \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int TABLE_F4 = 1024;      // 16 KiB per workgroup region (L1 is 32 KiB per CU)
constexpr int ITERS = 2048;

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int SHAPE>
__global__ __launch_bounds__(256) void l1_probe_kernel(const float4* __restrict__ table, float* __restrict__ out) {
    const float4* t = table + (blockIdx.x % 64) * TABLE_F4;   // 64 regions: 1 MiB, L2-resident, L1-resident per CU
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t h = hash(blockIdx.x * 256u + threadIdx.x);
#pragma unroll 8
    for (int i = 0; i < ITERS; ++i) {
        uint32_t idx;
        if (SHAPE == 0) idx = ((uint32_t)i * 64u + lane) & (TABLE_F4 - 1);            // coalesced
        else if (SHAPE == 1) idx = ((uint32_t)i * 4u + lane * 4u + wave) & (TABLE_F4 - 1);   // stride 64 B
        else if (SHAPE == 2) idx = ((uint32_t)i * 8u + lane * 8u + wave) & (TABLE_F4 - 1);   // stride 128 B
        else {                                                                           // random slot
            h = h * 1664525u + 1013904223u;
            idx = (h >> 8) & (TABLE_F4 - 1);
        }
        const float4 v = t[idx];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

// R-row records of REC bytes, one pseudo-random record per lane per iteration, R dwordx4 loads per record.
// ROT = 0: row k at byte 16 k of the record (every lane's load k at the same offset inside its line);
// ROT = 1: row k at slot (k + record) mod (REC / 16) (the offset varies with the record);
// ROT = 2: load k reads slot 0 of record (record + 37 k): random lines, every lane at offset 0.
template <int REC, int R, int ROT>
__global__ __launch_bounds__(256) void l1_probe_rec(const float4* __restrict__ table, float* __restrict__ out) {
    const float4* t = table + (blockIdx.x % 64) * TABLE_F4;
    constexpr int SLOTS = REC / 16, NREC = TABLE_F4 / SLOTS;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t h = hash(blockIdx.x * 256u + threadIdx.x);
#pragma unroll 2
    for (int i = 0; i < ITERS / R; ++i) {
        h = h * 1664525u + 1013904223u;
        const uint32_t rec = (h >> 8) & (NREC - 1);
        const float4* q = t + SLOTS * rec;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint32_t slot = ROT == 0 ? (uint32_t)k : ROT == 1 ? ((uint32_t)k + rec) & (SLOTS - 1) : 0u;
            const float4 v = ROT == 2 ? t[SLOTS * ((rec + 37u * k) & (NREC - 1))] : q[slot];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 8;                     // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    std::vector<float> h(64 * TABLE_F4 * 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i % 97) * 0.01f;
    float4* d_table;
    float* d_out;
    CHECK(hipMalloc(&d_table, h.size() * 4));
    CHECK(hipMalloc(&d_out, (size_t)blocks * 256 * 4));
    CHECK(hipMemcpy(d_table, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct Shape { const char* name; void (*k)(const float4*, float*); int per_iter; };
    const Shape shapes[] = {
        {"coalesced", l1_probe_kernel<0>, 1},
        {"stride64", l1_probe_kernel<1>, 1},
        {"stride128", l1_probe_kernel<2>, 1},
        {"random", l1_probe_kernel<3>, 1},
        {"node128", l1_probe_rec<128, 7, 0>, 7},          // the 4-wide node today: 7 rows at fixed offsets
        {"node128_rot", l1_probe_rec<128, 7, 1>, 7},      // rows rotated by the record index
        {"line128_slot0", l1_probe_rec<128, 7, 2>, 7},    // random lines, all lanes at offset 0
        {"node64", l1_probe_rec<64, 4, 0>, 4},            // a 64-B node: 4 rows at fixed offsets
        {"node64_rot", l1_probe_rec<64, 4, 1>, 4},
        {"tri48", l1_probe_rec<64, 3, 0>, 3},             // 3 rows of a 64-B-aligned record (48-B triangle padded)
    };
    for (const Shape& sh : shapes) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(sh.k, dim3(blocks), dim3(256), 0, 0, d_table, d_out);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double insts = (double)blocks * 4 * (ITERS / sh.per_iter) * sh.per_iter;   // wave-level load insts
        std::printf("{\"shape\": \"%s\", \"cus\": %d, \"blocks\": %d, \"wave_load_insts\": %.0f, \"best_ms\": %.4f, "
                    "\"cycles_per_inst_at_2p4GHz\": %.2f}\n",
                    sh.name, cus, blocks, insts, best, best * 1e6 * 2.4 / (insts / cus));
    }
    CHECK(hipFree(d_table));
    CHECK(hipFree(d_out));
    return 0;
}
