// crt_hip.hip — MI355X (gfx950) render layer: kernels + the C ABI of include/crt_hip.h.
//
// Hot path: crt_render_kernel — one lane per pixel (8x8 pixel tile per wave64,
// 16x16 per 256-thread workgroup), the pixel's samples traced strictly in order
// so each pixel's XORWOW stream is consumed exactly as in the reference
// (CUDAKernels.h:147-166).  Inside a wave, lanes are decoupled at PATH-SEGMENT
// granularity: a lane whose path ends (miss, light, absorption, Russian
// roulette, max bounces) immediately starts its next sample, so every loop
// iteration traces one ray per live lane instead of idling until the longest
// path of the wave finishes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "crt_hip.h"
#include "crt_device.h"
#include "crt_sah.h"
#include "crt/ParallelFor.h"

using namespace crt;

// ------------------------------------------------------------------ errors
static thread_local std::string g_last_error;
static int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
int crtx_set_error(int code, const std::string& msg) { return set_error(code, msg); }   // crt_bvh_build.hip
int crtx_build_sah_gpu(int device, const std::vector<crt_sah::Item>& items, int leaf_size, float trav_cost,
                       std::vector<crt_sah::Node>* nodes_out, std::vector<int>* order_out, int* max_depth);
#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return set_error(CRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------ kernels
struct RenderParams {
    const float4* __restrict__ nodes;
    const float4* __restrict__ prims;
    const float4* __restrict__ mats;
    const float4* __restrict__ shade;     // per reference DFS rank: shading record (crt_device.h)
    int n_nodes, n_mats, n_prims;         // n_nodes: nodes of ONE threaded layout
    int n_layouts;                        // 1, or 6 direction-ordered layouts (CRT_BVH_REBUILT)
    uint32_t* __restrict__ ovf;           // variant 4: traversal-stack entries beyond the LDS part
    int stack_cap;                        // variant 4: stack entries a ray can need (host bound)
    int stack_lds;                        // variant 4: entries kept in LDS (<= STACK_LDS; rest in ovf)
    int sphere_first, n_ray_spheres;      // variant 4: spheres tested per ray at generation (not in the BVH)
    int tree_spheres;                     // variant 4: the 4-wide tree's leaves hold spheres too
    const float4* __restrict__ sphere_chain;   // their reference scene-level leaf boxes (see ray_spheres)
    int n_chain;                                // boxes in sphere_chain
    // exactly two per-ray spheres (every reference scene: SceneManager's ground + metal sphere): their data
    // by value; the kernels stage it in LDS once, so a pass reads it with uniform LDS loads instead of two
    // dependent vector loads.  Per sphere: center.xyz, radius^2, rank bits, box lo.xyz, box hi.xyz, pad
    float sph2[2][12];
    unsigned* err;                // device error flag (bit 0: primitive index out of range)
    int width, height, spp, max_bounces;
    float rcp_w, rcp_h;           // next_ray's u = (x + U) / width by uv_div when fast_uv (crt_renderer_create)
    int fast_uv;
    int accumulate;
    int regen_threshold;          // variant 2: parked lanes needed before a shading/regeneration pass
    uint32_t* __restrict__ rng;   // W*H*6 (v0..v4, d)
    float* __restrict__ sum;      // W*H*3
    unsigned long long* __restrict__ counters;  // crt_work_counters layout
    crt_camera_desc cam;
    // variant 7 (persistent, 4-wide scenes): lanes take pixels from a global queue
    const uint32_t* __restrict__ order;   // slot -> pixel index (most expensive first, from the probe); ~0 = none
    uint32_t* __restrict__ queue;         // next unclaimed slot
    int n_slots;
    int tiles_x;                          // variant 8: 8x8 tiles per row (order[] holds tile indices)
    uint32_t* __restrict__ probe_cost;    // probe launch (variant 4): rays per pixel; nothing else is written
    int probe_stride;                     // probe launch (variant 4): lanes take every probe_stride-th pixel in x and y
    uint32_t* __restrict__ pix_rays;      // variant 7: rays each pixel took this frame (the next frame's tile order)
    int crit_tiles, crit_threshold;       // variant 8: the first crit_tiles tiles of the cost order regenerate at
                                          // crit_threshold parked lanes instead of regen_threshold
    int drain_threshold;                  // variant 7: the threshold once the pixel queue is empty
    int wave_drain;                       // variants 4/8: sixty-fourths of the live lanes a draining wave passes at
    int top_levels;                       // 4-wide variants: a new ray's first node steps taken from LDS (<= CRT_TOP_LEVELS)
};

#ifdef CRT_PROFILE_LIVE
// profiling build (tools/live_histogram.py): variant 8's wave time by the number of lanes that still have samples,
// s_memtime cycles summed over waves in 9 buckets of 8 lanes (the last: 64)
__device__ unsigned long long g_live_hist[16];
#endif
#ifdef CRT_PROFILE_PAIRS
__device__ unsigned long long g_pair_hist[32];   // [0, 16): log2 buckets of leaf pairs per wave step; [16, 25): lanes / 8
#endif

struct TraceCounts {
    uint32_t boxes, tris, spheres, step_slots, round_slots, trace_calls;
    // COUNT-mode section profile (variant 4; wave-uniform shader-clock cycles, s_memtime)
    uint64_t cyc_regen, cyc_step, cyc_round, passes;
    uint64_t cyc_shade, cyc_next;   // inside the regen pass: ray_spheres() + shade(), next_ray(); the rest is ray init
    uint64_t cyc_sph;               // of cyc_shade: the per-ray spheres (ray_spheres)
    uint64_t cyc_setup, cyc_top, cyc_head;   // CRT_PROFILE_PASS: new-ray set-up, LDS root step, loop head
#ifdef CRT_PROFILE_ROWS
    uint64_t cyc_rows, cyc_prims;            // node-row and primitive-record load-to-data cycles (profiling build)
#endif
};
__device__ __forceinline__ uint64_t shader_clock() { return __builtin_amdgcn_s_memtime(); }
// Profiling build only (tools/build_profile_lib.sh pass -DCRT_PROFILE_PASS, tools/pass_profile.py): the section timers
// the counting kernel keeps (s_memtime per section) also in the timed kernel, with the regeneration pass split into
// its parts.  g_pass_prof, summed over variant 8's waves: [0] step, [1] rounds, [2] pass total, [3] finish_ray (spheres
// + shade), [4] of which the per-ray spheres, [5] next_ray, [6] new-ray set-up (1/d, rows, LDS ray record), [7] the
// LDS root step (top_steps), [8] loop head (live / parked ballots, the drain rule), [9] passes, [10] waves, [11] wave
// lifetime (first to last instruction), [12] node steps, [13] leaf rounds, [14] rays.  -DCRT_PROFILE_PASS_FIRST=K keeps
// only the first K workgroups of the tile order (K = 1: the most expensive tile, config B's critical chain).  With
// -DCRT_PROFILE_ROWS as well: [15] the node step's wait for its seven rows and [16] the leaf round's wait for its
// primitive records (the loads issued, then an explicit vmcnt(0) between two timers)
// a 64-bit value of one lane, to every lane (the profiling builds' timer accumulators)
__device__ __forceinline__ uint64_t bcast64(uint64_t v, int lane) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), lane) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
}
#ifdef CRT_PROFILE_PASS
constexpr bool kProfilePass = true;
__device__ unsigned long long g_pass_prof[20];
#ifndef CRT_PROFILE_PASS_FIRST
#define CRT_PROFILE_PASS_FIRST 0x7fffffff
#endif
#else
constexpr bool kProfilePass = false;
#endif

// Hit rule shared by every variant and both BVH modes: a candidate (t, rank) replaces the current hit
// when t < closest, or t == closest and its reference DFS rank is higher.  In CRT_BVH_REFERENCE mode the
// traversal visits primitives in rank order, so this is exactly the reference's closed-interval
// acceptance (ties go to the later primitive); in CRT_BVH_REBUILT mode it reproduces that choice in
// any visiting order.
__device__ __forceinline__ bool better(float t, int rank, float closest, int hit) {
    return t < closest || (t == closest && rank > hit);
}

// Node array offset (in float4) of the threaded layout a ray walks: layout 2*axis + (d[axis] < 0) for the
// dominant axis of d when six direction-ordered layouts are resident, else 0.
__device__ __forceinline__ int layout_base(V3 d, int n_layouts, int n_nodes) {
    if (n_layouts == 1) return 0;
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const int l = (ax >= ay && ax >= az) ? (d.x < 0.f) : (ay >= az ? 2 + (d.y < 0.f) : 4 + (d.z < 0.f));
    return 2 * l * n_nodes;
}

// Closest hit over the threaded scene+mesh BVH.  Returns the reference DFS rank of the hit primitive
// or -1; `closest` = IntersectionTime of the accepted hit.
// Semantics: BVHNode::hit (BVHNode.cuh:115-156), Mesh::hit (Mesh.cuh:55-110),
// AABB::hit (AABB.cuh:123-146), rayTriangleIntersect (Mesh.cuh:266-308),
// Sphere::hit (Sphere.cuh:27-47); closed-interval acceptance so ties go to the
// later primitive, exactly as in the reference order.
template <bool COUNT>
__device__ __forceinline__ int trace(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                     int n_nodes, int nbase, V3 o, V3 d, float& closest, TraceCounts& cnt) {
    const float INF = __builtin_inff();
    // AABB::hit computes 1/d per node visit; the value is the same every time.
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    closest = INF;
    int hit = -1;
    int node = 0;
    while (node < n_nodes) {
        const float4 A = nodes[nbase + 2 * node];
        const float4 B = nodes[nbase + 2 * node + 1];
        const int a = __float_as_int(B.z);
        const int b = __float_as_int(B.w);
        const bool scene_level = (b == NODE_SCENE_INNER) || (b >= SPHERE_BIT);
        const float tcl = scene_level ? INF : closest;
        if (COUNT) cnt.boxes++;
        const float t0x = (A.x - o.x) * inv.x, t0y = (A.y - o.y) * inv.y, t0z = (A.z - o.z) * inv.z;
        const float t1x = (A.w - o.x) * inv.x, t1y = (B.x - o.y) * inv.y, t1z = (B.y - o.z) * inv.z;
        float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
        float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
        tmin = fmaxf(tmin, 0.001f);
        tmax = fminf(tmax, tcl);
        const bool box_hit = !(tmax <= tmin);
        int next = node + 1;
        if (b < 0) {
            if (!box_hit) next = a;
        } else if (box_hit) {
            if (b >= SPHERE_BIT) {
                const int p = b - SPHERE_BIT;
                if (COUNT) cnt.spheres++;
                const float4 f0 = prims[3 * p], f1 = prims[3 * p + 1];
                const V3 oc = o - v3(f0.x, f0.y, f0.z);
                const float qa = dot(d, d);
                const float hb = dot(oc, d);
                const float qc = dot(oc, oc) - f1.x;
                const float disc = hb * hb - qa * qc;
                if (!(disc < 0)) {
                    const float sq = sqrt_exact_wave(disc);
                    float root = (-hb - sq) / qa;
                    bool ok = true;
                    if (root < 0.001f || root > closest) {
                        root = (-hb + sq) / qa;
                        if (root < 0.001f || root > closest) ok = false;
                    }
                    const int rank = __float_as_int(f1.z);
                    if (ok && better(root, rank, closest, hit)) { closest = root; hit = rank; }
                }
            } else {
                for (int k = 0; k < a; ++k) {
                    const int p = b + k;
                    if (COUNT) cnt.tris++;
                    const float4 f0 = prims[3 * p], f1 = prims[3 * p + 1], f2 = prims[3 * p + 2];
                    const V3 e1 = v3(f0.w, f1.x, f1.y);
                    const V3 e2 = v3(f1.z, f1.w, f2.x);
                    const V3 h = cross(d, e2);
                    const float det = dot(e1, h);
                    if (fabsf(det) < 1e-8f) continue;
                    const float f = 1.f / det;
                    const V3 s = o - v3(f0.x, f0.y, f0.z);
                    const float u = f * dot(s, h);
                    if (u < 0.f || u > 1.f) continue;
                    const V3 q = cross(s, e1);
                    const float v = f * dot(d, q);
                    if (v < 0.f || (u + v) > 1.f) continue;
                    const float t = f * dot(e2, q);
                    if (t < 0.001f || t > closest) continue;
                    const int rank = __float_as_int(f2.z);
                    if (!better(t, rank, closest, hit)) continue;
                    closest = t;
                    hit = rank;
                }
            }
        }
        node = next;
    }
    return hit;
}

// Lanes of the wave (active lanes only) whose predicate holds.  HIP's __ballot widens the predicate to an int and
// compares it again (two VALU per ballot); the builtin takes the compare's lane mask as it is.
__device__ __forceinline__ uint64_t wave_ballot(bool pred) { return __builtin_amdgcn_ballot_w64(pred); }

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    return x;
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Wave64 inclusive scans with DPP (no LDS traffic): Kogge-Stone inside each 16-lane row
// (row_shr 1,2,4,8 with identity fill), then row_bcast15 / row_bcast31 carry the row totals.
// Same sequence as LLVM's AMDGPU atomic optimizer uses on gfx9.
#define CRT_DPP_ROW_SHR(n) (0x110 | (n))
#define CRT_DPP_BCAST15 0x142
#define CRT_DPP_BCAST31 0x143
// bound_ctrl: a lane whose source is out of range reads 0 (the identity), so LLVM's DPP combiner can fold
// each step into one v_add_u32_dpp / v_max_u32_dpp instead of v_mov (identity) + v_mov_dpp + the op.
__device__ __forceinline__ int wave_inclusive_scan(int x, int /*lane*/) {
    x += __builtin_amdgcn_update_dpp(0, x, CRT_DPP_ROW_SHR(1), 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, CRT_DPP_ROW_SHR(2), 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, CRT_DPP_ROW_SHR(4), 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, CRT_DPP_ROW_SHR(8), 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, CRT_DPP_BCAST15, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, CRT_DPP_BCAST31, 0xc, 0xf, false);
    return x;
}
// The same scan as six in-place v_add_u32_dpp.  In traverse_step4 the combiner leaves the builtin form as v_mov_dpp +
// v_add pairs (it reuses the partial sums for the exclusive prefix): 14 VALU instead of 6.  The s_nops are the
// VALU-write -> DPP-read wait states, which the compiler does not insert inside an asm block.
__device__ __forceinline__ int wave_inclusive_scan_dpp(int x) {
    __asm__ volatile(
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(x));
    return x;
}
// Inclusive max-scan of non-negative values (0 = none) with the same structure.
__device__ __forceinline__ uint32_t wave_inclusive_max_scan_u(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CRT_DPP_ROW_SHR(1), 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CRT_DPP_ROW_SHR(2), 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CRT_DPP_ROW_SHR(4), 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CRT_DPP_ROW_SHR(8), 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CRT_DPP_BCAST15, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CRT_DPP_BCAST31, 0xc, 0xf, false));
    return x;
}
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
// Reference (ds_bpermute) form, used by the scan self-test.
__device__ __forceinline__ int wave_inclusive_scan_shfl(int x, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    return x;
}

// Per-wave LDS for the cooperative leaf step.
struct WaveLds {
    float4 ray0[64];                 // o.x, o.y, o.z, d.x of each lane's ray
    float4 ray1[64];                 // d.y, d.z, closest at leaf entry, first prim (int bits)
    unsigned long long key[64];      // per owner: (t bits << 32) | (0xffffffff - rank), min-reduced
    int prefix[64];                  // first pair index of each owner's leaf
    unsigned char owner_at[64];      // owner lane of the pair that starts at each slot of a round
};
// The 4-wide kernels' per-wave LDS (traverse_step4): WaveLds without the owners' pair prefixes, which the fast build
// keeps in the ray records (ray1.w), so the 256 B go to the top nodes (CRT_TOP_LEVELS) within occupancy 6.
struct WaveLdsWide {
    float4 ray0[64];
    float4 ray1[64];
    unsigned long long key[64];
    unsigned char owner_at[64];
    uint32_t rays;                   // variant 8: the wave's ray count (in LDS, not a VGPR live across the loop)
#ifdef CRT_CHECKED
    int prefix[64];                  // checked build: each owner's first pair index and pair count
    int span_n[64];
#endif
};

// Möller–Trumbore (Mesh.cuh:266-308) on a triangle record; returns t or -1 when rejected (any accepted
// t >= 0.001).
__device__ __forceinline__ float tri_test_rec(float4 f0, float4 f1, float4 f2, V3 o, V3 d, float tmax) {
    const V3 e1 = v3(f0.w, f1.x, f1.y);
    const V3 e2 = v3(f1.z, f1.w, f2.x);
    const V3 h = cross(d, e2);
    const float det = dot(e1, h);
    if (fabsf(det) < 1e-8f) return -1.f;
    const float f = recip_exact(det);          // == 1.f / det bit for bit (see crt_device.h)
    const V3 s = o - v3(f0.x, f0.y, f0.z);
    const float u = f * dot(s, h);
    if (u < 0.f || u > 1.f) return -1.f;
    const V3 q = cross(s, e1);
    const float v = f * dot(d, q);
    if (v < 0.f || (u + v) > 1.f) return -1.f;
    const float t = f * dot(e2, q);
    if (t < 0.001f || t > tmax) return -1.f;
    return t;
}
// The same test without early exits, for the leaf rounds: u, v and t are pure functions of the record and the ray, so
// computing them on every lane and rejecting once returns the same value (the reject predicate keeps the reference's
// comparisons, NaN included).  1/det by rcp_newton when every active lane's |det| is below 2^126 (a wave-uniform
// choice; lanes with |det| < 1e-8 are rejected whatever f is), else by IEEE division.
__device__ __forceinline__ float tri_test_flat(float4 f0, float4 f1, float4 f2, V3 o, V3 d, float tmax) {
    const V3 e1 = v3(f0.w, f1.x, f1.y);
    const V3 e2 = v3(f1.z, f1.w, f2.x);
    const V3 h = cross(d, e2);
    const float det = dot(e1, h);
    const float a = fabsf(det);
    float f;
    if (__builtin_amdgcn_ballot_w64(!(a < RCP_FAST_MAX)) == 0) {
        f = rcp_newton(det);
    } else {
        __asm__ volatile("");
        f = 1.0f / det;
    }
    const V3 s = o - v3(f0.x, f0.y, f0.z);
    const float u = f * dot(s, h);
    const V3 q = cross(s, e1);
    const float v = f * dot(d, q);
    const float t = f * dot(e2, q);
    const bool rej = (a < 1e-8f) | (u < 0.f) | (u > 1.f) | (v < 0.f) | ((u + v) > 1.f) | (t < 0.001f) | (t > tmax);
    return rej ? -1.f : t;
}
__device__ __forceinline__ float tri_test(const float4* __restrict__ prims, int p, V3 o, V3 d, float tmax, int& rank) {
    const float4 f0 = prims[3 * p], f1 = prims[3 * p + 1], f2 = prims[3 * p + 2];
    rank = __float_as_int(f2.z);
    return tri_test_rec(f0, f1, f2, o, d, tmax);
}

// Sphere::hit (Sphere.cuh:27-47) as a candidate: the root it would accept against any closest >= the
// result (the near root if >= 0.001, else the far one), or -1.  Independent of the visiting order, so
// it can enter the same min-reduction as triangles.
__device__ __forceinline__ float sphere_candidate(float4 f0, float4 f1, V3 o, V3 d, float tmax) {
    const V3 oc = o - v3(f0.x, f0.y, f0.z);
    const float qa = dot(d, d);
    const float hb = dot(oc, d);
    const float qc = dot(oc, oc) - f1.x;
    const float disc = hb * hb - qa * qc;
    if (disc < 0) return -1.f;
    const float sq = sqrt_exact_wave(disc);
    float root = (-hb - sq) / qa;
    if (root < 0.001f || root > tmax) {
        root = (-hb + sq) / qa;
        if (root < 0.001f || root > tmax) return -1.f;
    }
    return root;
}

// Any primitive of a CRT_BVH_REBUILT leaf: triangle, or sphere (record word 11 == 1; only when the tree
// holds spheres — a uniform flag, so triangle-only trees skip the branch).
// Record at a 32-bit byte offset from a uniform base: the load takes the SGPR base + VGPR offset form, no
// 64-bit address arithmetic per lane (the host keeps primitive and 4-wide node arrays below 4 GiB).
__device__ __forceinline__ const float4* rec_at(const float4* base, uint32_t byte_off) {
    return reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + byte_off);
}

// (Storing the records as three planes of float4, for contiguous 16-B words per load, measured 2.7 % slower: the three
// planes are three cache lines per triangle where the 48-B record mostly sits in one, profiles/r02c.)
__device__ __forceinline__ float prim_test(const float4* __restrict__ prims, int p, V3 o, V3 d, float tmax, int& rank,
                                           bool tree_spheres = true) {
    // 24-bit multiply (full rate; v_mul_lo_u32 is quarter rate): the 4-wide tree holds < 2^24 primitives (emit4)
    const float4* r = rec_at(prims, __umul24((uint32_t)p, 48u));
    const float4 f0 = r[0], f1 = r[1], f2 = r[2];
    // keep the unused word: the third row then loads as one dwordx4 instead of a dword + a dwordx2 (one vector-L1
    // lookup set less per pair; -0.7 %, profiles/r02s)
    __asm__ volatile("" : : "v"(f2.y));
    rank = __float_as_int(f2.z);
    if (tree_spheres && __float_as_int(f2.w) == 1) return sphere_candidate(f0, f1, o, d, tmax);
    // without early exits: the leaf rounds are full of lanes, so the exits only cost branches (-0.75 %, profiles/r02ap)
    return tri_test_flat(f0, f1, f2, o, d, tmax);
}

// Sphere::hit (Sphere.cuh:27-47) against [0.001, closest]; updates closest/hit (= rank) on acceptance.
__device__ __forceinline__ void sphere_test(const float4* __restrict__ prims, int b, V3 o, V3 d, float& closest, int& hit) {
    const int p = b - SPHERE_BIT;
    const float4 f0 = prims[3 * p], f1 = prims[3 * p + 1];
    const V3 oc = o - v3(f0.x, f0.y, f0.z);
    const float qa = dot(d, d);
    const float hb = dot(oc, d);
    const float qc = dot(oc, oc) - f1.x;
    const float disc = hb * hb - qa * qc;
    if (disc < 0) return;
    const float sq = sqrt_exact_wave(disc);
    float root = (-hb - sq) / qa;
    if (root < 0.001f || root > closest) {
        root = (-hb + sq) / qa;
        if (root < 0.001f || root > closest) return;
    }
    const int rank = __float_as_int(f1.z);
    if (!better(root, rank, closest, hit)) return;
    closest = root;
    hit = rank;
}

// Variant 1: per-lane threaded traversal, leaf triangles tested cooperatively by the whole wave.
// Every lane that reaches a mesh leaf in a step contributes its (lane, triangle) pairs; the wave
// tests 64 pairs per round and min-reduces (t, later-index-wins) per owner in LDS.  Within one
// leaf a triangle's acceptance depends only on the closest hit at leaf entry, so the result is
// the same closest hit (ties to the later triangle) as Mesh::hit's sequential loop.
// MUST be called by all 64 lanes (inactive lanes pass active=false).
template <bool COUNT>
__device__ int trace_coop(const float4* __restrict__ nodes, const float4* __restrict__ prims, int n_nodes, int nbase,
                          int n_prims, unsigned* err, V3 o, V3 d, bool active, float& closest, TraceCounts& cnt,
                          WaveLds& L, int lane) {
    const float INF = __builtin_inff();
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    closest = INF;
    int hit = -1;
    int node = active ? 0 : n_nodes;
    L.ray0[lane] = make_float4(o.x, o.y, o.z, d.x);
    L.owner_at[lane] = 0;      // owner + 1, 0 = none
    if (COUNT) cnt.trace_calls++;
    while (wave_ballot(node < n_nodes)) {
        if (COUNT) cnt.step_slots++;        // one traversal step of the wave (x64 lanes)
        int leaf_n = 0, leaf_first = 0;
        if (node < n_nodes) {
            const float4 A = nodes[nbase + 2 * node];
            const float4 B = nodes[nbase + 2 * node + 1];
            const int a = __float_as_int(B.z);
            const int b = __float_as_int(B.w);
            const bool scene_level = (b == NODE_SCENE_INNER) || (b >= SPHERE_BIT);
            const float tcl = scene_level ? INF : closest;
            if (COUNT) cnt.boxes++;
            const float t0x = (A.x - o.x) * inv.x, t0y = (A.y - o.y) * inv.y, t0z = (A.z - o.z) * inv.z;
            const float t1x = (A.w - o.x) * inv.x, t1y = (B.x - o.y) * inv.y, t1z = (B.y - o.z) * inv.z;
            float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
            float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
            tmin = fmaxf(tmin, 0.001f);
            tmax = fminf(tmax, tcl);
            const bool box_hit = !(tmax <= tmin);
            int next = node + 1;
            if (b < 0) {
                if (!box_hit) next = a;
            } else if (box_hit) {
                if (b >= SPHERE_BIT) {
                    if (COUNT) cnt.spheres++;
                    sphere_test(prims, b, o, d, closest, hit);
                } else {
                    leaf_n = a;
                    leaf_first = b;
                }
            }
            node = next;
        }
        if (!wave_ballot(leaf_n > 0)) continue;
        const int incl = wave_inclusive_scan(leaf_n, lane);
        const int total = __builtin_amdgcn_readlane(incl, 63);
        const int pfx = incl - leaf_n;
        if (leaf_n > 0) {
            L.ray1[lane] = make_float4(d.y, d.z, closest, __int_as_float(leaf_first));
            L.prefix[lane] = pfx;
            L.key[lane] = ~0ull;
        }
        uint32_t carry = 0;   // owner + 1 of the last pair of the previous round
        for (int base = 0; base < total; base += 64) {
            if (COUNT) cnt.round_slots++;
            // owner of pair (base + lane): lanes whose leaf starts in this round mark their start slot,
            // then an inclusive max-scan over slots (owners are increasing in slot order) fills the gaps;
            // slots before the first start of the round belong to the previous round's last owner.
            if (leaf_n > 0 && pfx >= base && pfx < base + 64) L.owner_at[pfx - base] = (unsigned char)(lane + 1);
            wave_sync();
            const uint32_t mark = L.owner_at[lane];
            L.owner_at[lane] = 0;                     // reset own slot for the next round
            const uint32_t owner1 = max(wave_inclusive_max_scan_u(mark), carry);
            const int owner = (int)owner1 - 1;
            const int j = base + lane;
            if (j < total) {
                const float4 r0 = L.ray0[owner], r1 = L.ray1[owner];
                const int k = j - L.prefix[owner];
                const int p = __float_as_int(r1.w) + k;
                if (COUNT) cnt.tris++;
                if ((unsigned)p < (unsigned)n_prims && (unsigned)k < 0xffffffffu) {
                    int rank;
                    const float t = tri_test(prims, p, v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y), r1.z, rank);
                    if (t >= 0.f)
                        atomicMin(&L.key[owner], ((unsigned long long)__float_as_uint(t) << 32) | (0xffffffffu - (unsigned)rank));
                } else {
                    atomicOr(err, 1u);                // indexing bug: report instead of faulting
                }
            }
            carry = __builtin_amdgcn_readlane(owner1, 63);
            wave_sync();
        }
        if (leaf_n > 0) {
            const unsigned long long kk = L.key[lane];
            const float t = __uint_as_float((unsigned)(kk >> 32));
            const int rank = (int)(0xffffffffu - (unsigned)kk);
            if (kk != ~0ull && better(t, rank, closest, hit)) {
                closest = t;
                hit = rank;
            }
        }
    }
    return hit;
}

// One wave traversal step (variant 2): every lane with node < n_nodes tests one node; the leaves
// reached in this step are intersected cooperatively (same rounds as trace_coop).  All 64 lanes call it.
// PREFETCH: the caller keeps the current node's 32 B in (pA, pB); the next node is loaded right after
// the box test so its latency overlaps this step's leaf rounds.
template <bool COUNT, bool PREFETCH>
__device__ __forceinline__ void traverse_step(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                              int n_nodes, int nbase, int n_prims, unsigned* err, V3 o, V3 d,
                                              V3 inv, int& node, float& closest, int& hit, TraceCounts& cnt,
                                              WaveLds& L, int lane, float4& pA, float4& pB) {
    const float INF = __builtin_inff();
    if (COUNT) cnt.step_slots++;
    int leaf_n = 0, leaf_first = 0;
    if (node < n_nodes) {
        const float4 A = PREFETCH ? pA : nodes[nbase + 2 * node];
        const float4 B = PREFETCH ? pB : nodes[nbase + 2 * node + 1];
        const int a = __float_as_int(B.z);
        const int b = __float_as_int(B.w);
        const bool scene_level = (b == NODE_SCENE_INNER) || (b >= SPHERE_BIT);
        const float tcl = scene_level ? INF : closest;
        if (COUNT) cnt.boxes++;
        const float t0x = (A.x - o.x) * inv.x, t0y = (A.y - o.y) * inv.y, t0z = (A.z - o.z) * inv.z;
        const float t1x = (A.w - o.x) * inv.x, t1y = (B.x - o.y) * inv.y, t1z = (B.y - o.z) * inv.z;
        float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
        float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
        tmin = fmaxf(tmin, 0.001f);
        tmax = fminf(tmax, tcl);
        const bool box_hit = !(tmax <= tmin);
        int next = node + 1;
        if (b < 0) {
            if (!box_hit) next = a;
        } else if (box_hit) {
            if (b >= SPHERE_BIT) {
                if (COUNT) cnt.spheres++;
                sphere_test(prims, b, o, d, closest, hit);
            } else {
                leaf_n = a;
                leaf_first = b;
            }
        }
        node = next;
        if (PREFETCH && next < n_nodes) {
            pA = nodes[nbase + 2 * next];
            pB = nodes[nbase + 2 * next + 1];
        }
    }
    if (!wave_ballot(leaf_n > 0)) return;
    const int incl = wave_inclusive_scan_dpp(leaf_n);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    const int pfx = incl - leaf_n;
    if (leaf_n > 0) {
        L.ray1[lane] = make_float4(d.y, d.z, closest, __int_as_float(leaf_first));
        L.prefix[lane] = pfx;
        L.key[lane] = ~0ull;
    }
    uint32_t carry = 0;   // owner + 1 of the last pair of the previous round
    for (int base = 0; base < total; base += 64) {
        if (COUNT || kProfilePass) cnt.round_slots++;
        if (leaf_n > 0 && pfx >= base && pfx < base + 64) L.owner_at[pfx - base] = (unsigned char)(lane + 1);
        wave_sync();
        const uint32_t mark = L.owner_at[lane];
        L.owner_at[lane] = 0;
        const uint32_t owner1 = max(wave_inclusive_max_scan_u(mark), carry);
        const int owner = (int)owner1 - 1;
        const int j = base + lane;
        if (j < total) {
            const float4 r0 = L.ray0[owner], r1 = L.ray1[owner];
            const int k = j - L.prefix[owner];
            const int p = __float_as_int(r1.w) + k;
            if (COUNT) cnt.tris++;
            if ((unsigned)p < (unsigned)n_prims) {
                int rank;
                const float t = tri_test(prims, p, v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y), r1.z, rank);
                if (t >= 0.f)
                    atomicMin(&L.key[owner], ((unsigned long long)__float_as_uint(t) << 32) | (0xffffffffu - (unsigned)rank));
            } else {
                atomicOr(err, 1u);
            }
        }
        carry = __builtin_amdgcn_readlane(owner1, 63);
        wave_sync();
    }
    if (leaf_n > 0) {
        const unsigned long long kk = L.key[lane];
        const float t = __uint_as_float((unsigned)(kk >> 32));
        const int rank = (int)(0xffffffffu - (unsigned)kk);
        if (kk != ~0ull && better(t, rank, closest, hit)) {
            closest = t;
            hit = rank;
        }
    }
}

// ------------------------------------------------------------------ 4-wide BVH (CRT_BVH_REBUILT)
// Node = 8 x float4 (128 B): child boxes as SoA rows (lo.x[4], hi.x[4], lo.y[4], hi.y[4], lo.z[4],
// hi.z[4]), then meta = (first_child, n_internal | n_slots << 8, leaf_first, 8-bit triangle count per
// slot), then padding.  Slots [0, n_internal) are internal children at node first_child + slot; the
// following slots are leaves whose primitives are consecutive from leaf_first in slot order; empty slots
// have a zero-thickness box far away (never hit).
// crt_render: variant 8 below 4 tiles per wave slot runs at occupancy 4 with the row prefetch when the probe's largest
// tile work exceeds CRT_CHAIN_RHO times the mean work per occupancy-6 wave slot (a chain-bound frame), else at 6
#ifndef CRT_CHAIN_RHO
#define CRT_CHAIN_RHO 1.6   // profiles/r06y: occupancy 4 won at rho 1.62-6.4 and lost at 0.79-1.55 (one exception, -2 % at 1.54)
#endif
constexpr int STACK_LDS = 16;   // per-lane traversal-stack entries kept in LDS; deeper entries go to P.ovf
#ifndef CRT_STACK6
#define CRT_STACK6 12           // entries at occupancy 6 (6 one-wave workgroups per SIMD within 160 KiB: <= 6144 B each)
#endif
#ifndef CRT_STACK7
#define CRT_STACK7 8            // entries at occupancy 7: LDS is allocated in 1-KiB steps, so 28 one-wave workgroups per
                                // CU need <= 5,120 B each (variant 8: 5,024 B; 9 entries, 5,280 B, stay at 6 per SIMD,
                                // profiles/r03ah)
#endif

struct Wide4 {
    float tmin[4];
    bool hit[4];
};

// Slab test of the four child boxes against [0.001, tmax]: plane * inv - o * inv as one fma per plane (one operation
// where (lo - o) * inv takes two; measured -2.1 %, profiles/r01at).  Its error, about ulp(o) * |inv|
// in t, is of the same order as that of (lo - o) * inv and far inside the boxes' 1e-5 * max(1, |coord|) padding
// (DESIGN.md §2b).  inv must be finite AND o * inv / lo * inv must not overflow: an infinite product makes
// lo * inv - o * inv = inf - inf = NaN on a plane, and the min/max would then cull a box the ray runs inside of.
// The traversal's 1/d is therefore the exact 1/d clamped to +-2^64 (box_inv): a plane keeps its sign and a magnitude
// >= padding * 2^64, far above the rounding, and |coord| * 2^64 stays finite for every |coord| < 2^60, the bound
// crt_scene_create_ex enforces on the rebuilt tree's boxes (every later ray origin is a hit point inside them) and
// crt_renderer_set_camera on the primary rays' origins (camera origin + lens offset, below 2^59 + 2^58).
constexpr float BOX_INV_CLAMP = 0x1p64f;
__device__ __forceinline__ V3 box_inv(V3 inv) {
    return v3(__builtin_amdgcn_fmed3f(inv.x, -BOX_INV_CLAMP, BOX_INV_CLAMP),
              __builtin_amdgcn_fmed3f(inv.y, -BOX_INV_CLAMP, BOX_INV_CLAMP),
              __builtin_amdgcn_fmed3f(inv.z, -BOX_INV_CLAMP, BOX_INV_CLAMP));
}
// 1/d of a new ray, each component == 1.f / x bit for bit: rcp_newton when every active lane's three components lie in
// its verified range (a wave-uniform branch), else recip_exact_any per component (-0.33 %, profiles/r02av).
__device__ __forceinline__ V3 recip3_exact(V3 d) {
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const bool ok = ax >= RCP_FAST_MIN && ax < RCP_FAST_MAX && ay >= RCP_FAST_MIN && ay < RCP_FAST_MAX &&
                    az >= RCP_FAST_MIN && az < RCP_FAST_MAX;
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) return v3(rcp_newton(d.x), rcp_newton(d.y), rcp_newton(d.z));
    __asm__ volatile("");
    return v3(recip_exact_any(d.x), recip_exact_any(d.y), recip_exact_any(d.z));
}
// The per-ray spheres' exact 1/d (their reference box test) from the traversal's box_inv: recomputed only when a
// component was clamped.
__device__ __forceinline__ V3 sphere_inv(V3 d, V3 binv) {
    if (fabsf(binv.x) == BOX_INV_CLAMP || fabsf(binv.y) == BOX_INV_CLAMP || fabsf(binv.z) == BOX_INV_CLAMP)
        return v3(recip_exact_any(d.x), recip_exact_any(d.y), recip_exact_any(d.z));
    return binv;
}
// Row k of 4-wide node n sits at 16-B slot k ^ (n & 7) of the node's 128-B record (swizzled at upload,
// crt_scene_create_ex).  One wave instruction loads row k of up to 64 different nodes; at a fixed slot every lane reads
// the same 16-B offset of its line, and the vector L1 then serves about one lane per cycle (tools/probes/l1_probe,
// profiles/r02c: 62 cycles per instruction for that shape against 38 for random offsets).  b = node_base(n).
__device__ __forceinline__ uint32_t node_base(int node) { return ((uint32_t)node << 7) | (((uint32_t)node & 7u) << 4); }
__device__ __forceinline__ float4 node_row(const float4* __restrict__ nodes, uint32_t b, uint32_t k) {
    return *rec_at(nodes, b ^ (k << 4));
}
// The slab test by the ray's direction signs: for axis a, the row of the four child planes the ray enters first (lo
// for inv >= 0, hi for inv < 0) is row 2a ^ sign_a, and the row it leaves by is the other one.  fma(plane, inv, -o*inv)
// is monotone in the plane, so the entry row's t values are exactly min(t_lo, t_hi) and the exit row's exactly
// max(t_lo, t_hi): the same box hits and tmin as the min/max form, bit for bit, without its 24 min/max per node.  The
// row choice is an address bit (the sign of inv, shifted to the row's 16-B slot), not a select.
__device__ __forceinline__ uint32_t sign_row(float inv) { return (__float_as_uint(inv) >> 27) & 16u; }
// The ray's entry-row offsets for the three axes, one byte each (row 2a ^ sign, in 16-B units), computed once per
// ray: a node step then needs one xor per row address instead of re-deriving the signs.
__device__ __forceinline__ uint32_t ray_rows(V3 inv) {
    return sign_row(inv.x) | ((32u ^ sign_row(inv.y)) << 8) | ((64u ^ sign_row(inv.z)) << 16);
}
__device__ __forceinline__ Wide4 wide_boxes_of(const float4& nxr, const float4& fxr, const float4& nyr, const float4& fyr,
                                               const float4& nzr, const float4& fzr, V3 o, V3 inv, float tmax);
__device__ __forceinline__ Wide4 wide_boxes(const float4* __restrict__ nodes, uint32_t b, uint32_t rows, V3 o, V3 inv,
                                            float tmax) {
    const uint32_t ex = b ^ (rows & 0xffu), ey = b ^ ((rows >> 8) & 0xffu), ez = b ^ (rows >> 16);
    const float4 nxr = *rec_at(nodes, ex), fxr = *rec_at(nodes, ex ^ 16u);
    const float4 nyr = *rec_at(nodes, ey), fyr = *rec_at(nodes, ey ^ 16u);
    const float4 nzr = *rec_at(nodes, ez), fzr = *rec_at(nodes, ez ^ 16u);
    return wide_boxes_of(nxr, fxr, nyr, fyr, nzr, fzr, o, inv, tmax);
}
// The rows of node b for the row prefetch of variant 8 at occupancy 4 (traverse_step4<.., true>): pf[0..5] = the ray's
// entry / exit rows per axis (the order wide_boxes_of takes), pf[6] = the link row.
__device__ __forceinline__ void load_node_rows(const float4* __restrict__ nodes, uint32_t b, uint32_t rows, float4* pf) {
    const uint32_t ex = b ^ (rows & 0xffu), ey = b ^ ((rows >> 8) & 0xffu), ez = b ^ (rows >> 16);
    pf[0] = *rec_at(nodes, ex); pf[1] = *rec_at(nodes, ex ^ 16u);
    pf[2] = *rec_at(nodes, ey); pf[3] = *rec_at(nodes, ey ^ 16u);
    pf[4] = *rec_at(nodes, ez); pf[5] = *rec_at(nodes, ez ^ 16u);
    pf[6] = *rec_at(nodes, b ^ (6u << 4));
}
__device__ __forceinline__ Wide4 wide_boxes_of(const float4& nxr, const float4& fxr, const float4& nyr, const float4& fyr,
                                               const float4& nzr, const float4& fzr, V3 o, V3 inv, float tmax) {
    // one v_fma_f32 per plane: a v_pk_fma_f32 costs the SIMD the same cycles as two (MI355X_MICROARCH.md) and needs
    // {inv, inv} / {-o*inv, -o*inv} register pairs, which made the persistent variant 7 spill in this step (the
    // scalar form: variant 8 -1.7 %, variant 7 -18 %, profiles/r02aa)
    const float nx = -(o.x * inv.x), ny = -(o.y * inv.y), nz = -(o.z * inv.z);
    Wide4 w;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const float ax = __builtin_fmaf((&nxr.x)[s], inv.x, nx), bx = __builtin_fmaf((&fxr.x)[s], inv.x, nx);
        const float ay = __builtin_fmaf((&nyr.x)[s], inv.y, ny), by = __builtin_fmaf((&fyr.x)[s], inv.y, ny);
        const float az = __builtin_fmaf((&nzr.x)[s], inv.z, nz), bz = __builtin_fmaf((&fzr.x)[s], inv.z, nz);
        const float t0 = fmaxf(fmaxf(ax, ay), fmaxf(az, 0.001f));
        const float t1 = fminf(fminf(bx, by), fminf(bz, tmax));
        w.tmin[s] = t0;
        w.hit[s] = t0 < t1;
    }
    return w;
}

// Spheres kept out of a 4-wide BVH (scenes with few spheres) are tested once per ray, before the traversal;
// the hit rule is order-independent, so this is the same closest hit.  A sphere is reached only if the
// reference's scene-level boxes on its path pass AABB::hit against [0.001, inf) with the exact 1/d: the
// reference never tests a sphere whose box the ray's interval misses, and f32 roots of large spheres can
// land outside the sphere's own box (a ray leaving the radius-999 ground sphere at t just above 0.001).
// Every ancestor box contains the sphere's leaf box and AABB::hit is monotone in the box (f32 subtraction
// and multiplication are monotone), so the leaf box alone decides: record word 7 = its index in chain.
__device__ __forceinline__ bool ref_scene_box(float4 A, float4 B, V3 o, V3 inv) {
    const float t0x = (A.x - o.x) * inv.x, t0y = (A.y - o.y) * inv.y, t0z = (A.z - o.z) * inv.z;
    const float t1x = (A.w - o.x) * inv.x, t1y = (B.x - o.y) * inv.y, t1z = (B.y - o.z) * inv.z;
    float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    tmin = fmaxf(tmin, 0.001f);
    tmax = fminf(tmax, __builtin_inff());
    return !(tmax <= tmin);
}
// Sphere::hit's candidate root from its discriminant terms (Sphere.cuh:27-47 with closest = inf).
__device__ __forceinline__ float sphere_root(float qa, float hb, float disc) {
    if (disc < 0) return -1.f;
    const float sq = sqrt_exact_wave(disc);
    float root = (-hb - sq) / qa;
    if (root < 0.001f) {
        root = (-hb + sq) / qa;
        if (root < 0.001f) return -1.f;
    }
    return root;
}

// The per-ray spheres of the 4-wide variants are tested after the trace, against the trace's closest hit (the hit
// rule is order-independent, so the result is the same as testing them first).  A sphere whose near root is
// provably beyond that hit then skips the correctly rounded sqrt and division: with su >= sqrtf(disc) (raw
// v_sqrt_f32 is within 1 ulp, so 4 ulp of margin), fl(-hb - su) <= fl(-hb - sqrtf(disc)) by monotone rounding, and
// fl(-hb - su) > fl(closest * qa) * (1 + 1e-5) puts the exact root above nextafter(closest).  The far root is
// larger still.  (Testing them at ray start instead measured +2.1 %, profiles/r01ag.)
__device__ __forceinline__ bool sphere_beyond(float qa, float hb, float disc, float closest) {
    if (!(disc > 1e-30f) || !(closest < __builtin_inff())) return false;
    const float su = __builtin_amdgcn_sqrtf(disc) * (1.0f + 0x1p-21f);
    const float lb = -hb - su;
    return lb > (closest * qa) * (1.0f + 1e-5f);
}

// Two spheres at once (data from the kernel arguments): the reference box tests and the discriminant
// arithmetic (IEEE, the reference's operation order: (x*x + y*y) + z*z), roots and divisions per sphere.  In scalar
// f32: the packed form (v_pk_*) takes the same SIMD cycles and its register pairs cost the hot loop two spilled
// VGPRs (-1.2 % without, profiles/r02ab).
template <bool LATE = false>
__device__ __forceinline__ void ray_spheres2(const float* sa, const float* sb, V3 o, V3 d, V3 inv,
                                             float& closest, int& hit) {
    const float* sp[2] = {sa, sb};
    bool reach[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const float* q = sp[s];
        const float4 lo = *reinterpret_cast<const float4*>(q + 4), hi = *reinterpret_cast<const float4*>(q + 8);
        const float t0x = (lo.x - o.x) * inv.x, t1x = (lo.w - o.x) * inv.x;
        const float t0y = (lo.y - o.y) * inv.y, t1y = (hi.x - o.y) * inv.y;
        const float t0z = (lo.z - o.z) * inv.z, t1z = (hi.y - o.z) * inv.z;
        float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
        float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
        tmin = fmaxf(tmin, 0.001f);
        reach[s] = !(tmax <= tmin);
    }
    if (!(reach[0] || reach[1])) return;
    const float qa = dot(d, d);
    float t[2];
    // (a wave-uniform skip of a sphere no lane reaches measured +0.9 % on config C and -0.8 % on B, profiles/r05e)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const float4 c = *reinterpret_cast<const float4*>(sp[s]);
        const float ocx = o.x - c.x, ocy = o.y - c.y, ocz = o.z - c.z;
        const float hb = (ocx * d.x + ocy * d.y) + ocz * d.z;
        const float qc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - c.w;
        const float disc = hb * hb - qa * qc;
        t[s] = reach[s] && !(LATE && sphere_beyond(qa, hb, disc, closest)) ? sphere_root(qa, hb, disc) : -1.f;
    }
    const int ra = __float_as_int(sa[10]), rb = __float_as_int(sb[10]);
    if (t[0] >= 0.f && better(t[0], ra, closest, hit)) { closest = t[0]; hit = ra; }
    if (t[1] >= 0.f && better(t[1], rb, closest, hit)) { closest = t[1]; hit = rb; }
}

// inv: AABB::hit's 1/d, bit-exact (recip_exact_any), shared with the traversal.
template <bool LATE = false>
__device__ __forceinline__ void ray_spheres(const float4* __restrict__ prims, const float4* __restrict__ chain,
                                            int n_chain, int first, int n, V3 o, V3 d, V3 inv, float& closest,
                                            int& hit, const float* sph2 = nullptr) {
    if (n == 0) return;
    if (n == 2 && sph2) {
        ray_spheres2<LATE>(sph2, sph2 + 16, o, d, inv, closest, hit);
        return;
    }
    for (int s = 0; s < n; ++s) {
        const int p = first + s;
        const float4 f0 = prims[3 * p], f1 = prims[3 * p + 1];
        const int k = __float_as_int(f1.w);
        if (!ref_scene_box(chain[2 * k], chain[2 * k + 1], o, inv)) continue;
        const float t = sphere_candidate(f0, f1, o, d, __builtin_inff());
        const int rank = __float_as_int(f1.z);
        if (t >= 0.f && better(t, rank, closest, hit)) {
            closest = t;
            hit = rank;
        }
    }
}

__device__ __forceinline__ void cas(uint32_t& a, uint32_t& b) {
    const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Per-lane closest hit over a 4-wide BVH (diagnostic path: crt_scene_compare).  Returns the rank or -1.
__device__ int trace4(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                      const float4* __restrict__ chain, int n_chain, int sphere_first, int n_spheres, V3 o, V3 d,
                      float& closest) {
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    closest = __builtin_inff();
    int hit = -1, node = 0, sp = 0;
    ray_spheres(prims, chain, n_chain, sphere_first, n_spheres, o, d, inv, closest, hit);
    int stack[64];
    while (node >= 0) {
        const uint32_t b = node_base(node);
        const Wide4 w = wide_boxes(nodes, b, ray_rows(box_inv(inv)), o, box_inv(inv), closest);
        const float4 mf = node_row(nodes, b, 6);
        const int first_child = __float_as_int(mf.x), n_int = __float_as_int(mf.y) & 0xff;
        const uint32_t counts = __float_as_uint(mf.w);
        int off = 0;
        const float entry = closest;
        for (int s = 0; s < 4; ++s) {
            const int c = (counts >> (8 * s)) & 0xff;
            if (s >= n_int && c > 0 && w.hit[s]) {
                for (int k = 0; k < c; ++k) {
                    int rank;
                    const float t = prim_test(prims, __float_as_int(mf.z) + off + k, o, d, entry, rank);
                    if (t >= 0.f && better(t, rank, closest, hit)) { closest = t; hit = rank; }
                }
            }
            off += c;
        }
        uint32_t k[4];
        for (int s = 0; s < 4; ++s) k[s] = (s < n_int && w.hit[s]) ? ((__float_as_uint(w.tmin[s]) & ~3u) | s) : ~0u;
        cas(k[0], k[1]); cas(k[2], k[3]); cas(k[0], k[2]); cas(k[1], k[3]); cas(k[1], k[2]);
        if (k[0] != ~0u) {
            node = first_child + (int)(k[0] & 3);
            for (int s = 3; s >= 1; --s)
                if (k[s] != ~0u && sp < 64) stack[sp++] = first_child + (int)(k[s] & 3);
        } else {
            node = sp > 0 ? stack[--sp] : -1;
        }
    }
    return hit;
}

// One wave traversal step over a 4-wide BVH (variant 4).  Every lane with a node tests its four child
// boxes; hit internal children are ordered near-first (u32 sort of (tmin bits | slot) keys), the nearest
// becomes the lane's next node and the others go onto its stack as ONE entry (children are consecutive
// nodes): first_child << 8 | remaining << 6 | slot0 << 4 | slot1 << 2 | slot2, slots in pop order.  A pop
// takes slot0 and rewrites the entry while slots remain, so the stack holds at most one entry per
// branching ancestor.  The primitives of the hit leaf children (one consecutive range) join this step's
// cooperative leaf rounds.  All 64 lanes call it.
// Overflow stack entry `at` of pixel `pix`: a 32-bit byte offset from the uniform base (the host keeps the
// region below 4 GiB), so the address is SGPR base + VGPR offset and nothing 64-bit stays live per lane.
__device__ __forceinline__ uint32_t* ovf_slot(const RenderParams& P, int at, size_t pix, size_t n_pix) {
    const uint32_t byte = ((uint32_t)(at - P.stack_lds) * (uint32_t)n_pix + (uint32_t)pix) << 2;
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(P.ovf) + byte);
}

// The lane id recomputed at the point of use (two VALU ops, no register kept across the loop): at the 80-VGPR
// budget of 6 waves/SIMD the allocator otherwise spills the lane's stack address and reloads it from scratch on
// every push and pop.
__device__ __forceinline__ int lane_fresh() {
    int l;
    __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

template <bool COUNT, bool PF = false>
__device__ __forceinline__ void node_step4(const RenderParams& P, V3 o, V3 inv, uint32_t rows, int& node, int& sp, float closest,
                                           TraceCounts& cnt, uint32_t* __restrict__ stk, int lane, size_t pix,
                                           size_t n_pix, int& leaf_first, int& leaf_n, float4* pf = nullptr,
                                           bool have_pf = false) {
    leaf_n = 0;
    leaf_first = 0;
#ifdef CRT_PROFILE_ROWS
    uint64_t row_wait = 0;
#endif
    if (node >= 0) {
        const uint32_t b = node_base(node);
#ifdef CRT_PROFILE_ROWS
        // profiling build: the seven rows issued, then waited for between two timers
        const uint32_t ex = b ^ (rows & 0xffu), ey = b ^ ((rows >> 8) & 0xffu), ez = b ^ (rows >> 16);
        const uint64_t ra = shader_clock();
        const float4 mf = node_row(P.nodes, b, 6);
        const float4 nxr = *rec_at(P.nodes, ex), fxr = *rec_at(P.nodes, ex ^ 16u);
        const float4 nyr = *rec_at(P.nodes, ey), fyr = *rec_at(P.nodes, ey ^ 16u);
        const float4 nzr = *rec_at(P.nodes, ez), fzr = *rec_at(P.nodes, ez ^ 16u);
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
        __asm__ volatile("" : : "v"(mf.x), "v"(nxr.x), "v"(fxr.x), "v"(nyr.x), "v"(fyr.x), "v"(nzr.x), "v"(fzr.x) : "memory");
        row_wait = shader_clock() - ra;
        const Wide4 w = wide_boxes_of(nxr, fxr, nyr, fyr, nzr, fzr, o, inv, closest);
#else
        // PF: the rows are in pf when the previous step's first leaf round loaded them for this node (have_pf), else
        // they load here as without the prefetch
        if (PF && !have_pf) load_node_rows(P.nodes, b, rows, pf);
        const float4 mf = PF ? pf[6] : node_row(P.nodes, b, 6);
        const Wide4 w = PF ? wide_boxes_of(pf[0], pf[1], pf[2], pf[3], pf[4], pf[5], o, inv, closest)
                           : wide_boxes(P.nodes, b, rows, o, inv, closest);
#endif
        // keep the whole link row in the node's loads: left to itself the compiler loads leaf_first / counts
        // only inside the leaf branch, one more dependent load on a leaf step's critical path.  Pinned after the
        // box tests, so the wait it implies is the one the boxes need anyway (pinned before them, it made the six
        // box loads wait for the link row's round trip)
        __asm__ volatile("" : : "v"(mf.z), "v"(mf.w));
        const int first_child = __float_as_int(mf.x);
        const int meta = __float_as_int(mf.y);
        const uint32_t counts = __float_as_uint(mf.w);
        const int n_int = meta & 0xff;
        if (COUNT) cnt.boxes += (uint32_t)(meta >> 8);
        // leaf children: consecutive primitives; test the span from the first to the last hit leaf.  Slots
        // [n_int, n_slots) are leaves (count >= 1), empty slots are never hit, so the hit leaves are the hit bits
        // above n_int; counts * 0x01010101 holds the running ends in its bytes (at most 255 primitives per node,
        // checked by the builder).
        uint32_t hm = 0;
#pragma unroll
        for (int s = 0; s < 4; ++s) hm |= w.hit[s] ? (1u << s) : 0u;
        const uint32_t lm = hm & (0xfu << n_int);
        if (lm) {
            // counts * 0x01010101 (byte-wise running sums) as shift-adds: a 32-bit multiply is quarter rate (the empty
            // asm keeps the compiler from folding the shifts back into one)
            uint32_t c2 = counts + (counts << 8);
            __asm__("" : "+v"(c2));
            uint32_t ends = c2 + (c2 << 16);
            __asm__("" : "+v"(ends));
            const uint32_t first = (uint32_t)__builtin_ctz(lm), last = 31u - (uint32_t)__builtin_clz(lm);
            const int lo = (int)(((ends << 8) >> (8u * first)) & 0xffu);
            const int hi = (int)((ends >> (8u * last)) & 0xffu);
            leaf_n = hi - lo;
            leaf_first = __float_as_int(mf.z) + lo;
#ifdef CRT_CHECKED
            // the span must lie inside the primitive array.  emit4 guarantees it for every node it writes (checked there
            // on the host, once per node), so the fast build trusts the tree; the checked build re-checks it here once per
            // lane and step (before round 5 the fast build did too: one kernel-argument reload and wait per leaf step)
            if ((unsigned)leaf_first > (unsigned)P.n_prims || (unsigned)leaf_n > (unsigned)(P.n_prims - leaf_first)) {
                atomicOr(P.err, 1u);
                leaf_n = 0;
            }
#endif
        }
        uint32_t k[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) k[s] = (s < n_int && w.hit[s]) ? ((__float_as_uint(w.tmin[s]) & ~3u) | s) : ~0u;
        cas(k[0], k[1]); cas(k[2], k[3]); cas(k[0], k[2]); cas(k[1], k[3]); cas(k[1], k[2]);
        // sp counts stored entries only: an entry beyond the host's bound is dropped (and reported through P.err, the
        // frame is wrong) without advancing sp, so a pop never reads an entry that was not stored (reading one made
        // the traversal restart at the root, forever)
        auto store = [&](int at, uint32_t v) -> bool {
            if (at < P.stack_lds) stk[at * 64 + lane_fresh()] = v;
            else if (at < P.stack_cap) *ovf_slot(P, at, pix, n_pix) = v;
            else { atomicOr(P.err, 2u); return false; }
            return true;
        };
        if (k[0] != ~0u) {
            node = first_child + (int)(k[0] & 3);
            // the hit internal children but the nearest (k[s] != ~0u exactly for the hit slots below n_int), as one
            // popcount (-1.0 %, profiles/r02ap)
            const uint32_t n_rest = (uint32_t)__popc(hm & ((1u << n_int) - 1u)) - 1u;
            if (n_rest && store(sp, ((uint32_t)first_child << 8) | (n_rest << 6) | ((k[1] & 3) << 4) |
                                        ((k[2] & 3) << 2) | (k[3] & 3)))
                ++sp;
        } else if (sp > 0) {
            const int at = sp - 1;
            const uint32_t top = at < P.stack_lds ? stk[at * 64 + lane_fresh()]
                                                  : (at < P.stack_cap ? *ovf_slot(P, at, pix, n_pix) : 0u);
            const uint32_t rest = (top >> 6) & 3;
            node = (int)(top >> 8) + (int)((top >> 4) & 3);
            if (rest <= 1) sp = at;
            else store(at, (top & ~0xffu) | ((rest - 1) << 6) | ((top & 0xfu) << 2));
        } else {
            node = -1;
        }
    }
#ifdef CRT_PROFILE_ROWS
    {   // the wait of a lane that stepped (uniform among them: the timers are scalar)
        const uint64_t st = wave_ballot(row_wait != 0);
        if (st) cnt.cyc_rows += bcast64(row_wait, __builtin_ctzll(st));
    }
#endif
}

template <bool COUNT, bool PF = false>
__device__ __forceinline__ void traverse_step4(const RenderParams& P, V3 o, V3 d, V3 inv, uint32_t rows, int& node, int& sp,
                                               float& closest, int& hit, TraceCounts& cnt, WaveLdsWide& L,
                                               uint32_t* __restrict__ stk, int lane, size_t pix, size_t n_pix,
                                               float4* pf = nullptr, int* pf_node = nullptr) {
    constexpr bool TIME = COUNT || kProfilePass;
    if (COUNT || kProfilePass) cnt.step_slots++;
    const uint64_t c0 = TIME ? shader_clock() : 0;
    int leaf_n, leaf_first;
    if constexpr (PF) {
        // pf holds node *pf_node's rows when the previous step's first leaf round loaded them (profiles/r06r)
        node_step4<COUNT, true>(P, o, inv, rows, node, sp, closest, cnt, stk, lane, pix, n_pix, leaf_first, leaf_n, pf,
                                *pf_node == node);
        *pf_node = -1;
    } else
    node_step4<COUNT>(P, o, inv, rows, node, sp, closest, cnt, stk, lane, pix, n_pix, leaf_first, leaf_n);
    const uint64_t c1 = TIME ? shader_clock() : 0;
    if (TIME) cnt.cyc_step += c1 - c0;
#ifdef CRT_PROFILE_PAIRS
    // profiling build (tools/pair_histogram.py): per wave step, the lanes stepping and the leaf pairs, log2 buckets
    {
        const uint32_t n_step = (uint32_t)__popcll(wave_ballot(node >= 0 || leaf_n > 0));
        const int tot = __builtin_amdgcn_readlane(wave_inclusive_scan(leaf_n, lane), 63);
        if (lane_fresh() == 0) {
            atomicAdd(&g_pair_hist[tot == 0 ? 0 : 1 + min(31 - __clz(tot), 14)], 1ull);
            atomicAdd(&g_pair_hist[16 + min(n_step >> 3, 8u)], 1ull);
        }
    }
#endif
    if (!wave_ballot(leaf_n > 0)) return;
    const int incl = wave_inclusive_scan_dpp(leaf_n);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    const int pfx = incl - leaf_n;
    {   // every lane writes its own slots, only the owners' are read: no branch (-0.8 %, profiles/r02ar)
        // leaf_first - prefix: a pair's primitive is ray1.w + its index j (-0.27 %, profiles/r02aq; round 1 measured
        // this +2.2 %, profiles/r01aj, before the round-2 changes to the round's code)
        L.ray1[lane] = make_float4(d.y, d.z, closest, __int_as_float(leaf_first - pfx));
#ifdef CRT_CHECKED
        L.prefix[lane] = pfx;
        L.span_n[lane] = leaf_n;
#endif
        // the empty key, materialised here: as a plain constant the register allocator keeps ~0ull live across
        // the loop and spills it (a scratch reload and a vmcnt(0) wait on every leaf step)
        uint32_t ones;
        __asm__ volatile("v_mov_b32 %0, -1" : "=v"(ones));
        L.key[lane] = ((unsigned long long)ones << 32) | ones;
    }
    uint32_t carry = 0;   // owner + 1 of the last pair of the previous round
    if constexpr (PF) {
        // The row prefetch (variant 8 at occupancy 4, profiles/r06r): the lane's next node is known before the leaf
        // rounds, and their hits only lower `closest`, which the rows do not depend on.  The first round loads every
        // lane's pair record (slots past the end: record 0), THEN the lane's next node's seven rows (node 0 for a lane
        // without one): vector-memory loads retire in order, so the round waits for its records only (rows loaded
        // before the records made the round wait for them too: +3.6 %, profiles/r06o).  The next node step finds the
        // rows in registers (28 VGPRs, which is why this needs occupancy 4's budget).
        auto round = [&](int base, auto first) {
            if (COUNT || kProfilePass) cnt.round_slots++;
            if (leaf_n > 0 && pfx >= base && pfx < base + 64) L.owner_at[pfx - base] = (unsigned char)(lane + 1);
            wave_sync();
            const uint32_t mark = L.owner_at[lane];
            L.owner_at[lane] = 0;
            const uint32_t owner1 = max(wave_inclusive_max_scan_u(mark), carry);
            const int owner = (int)owner1 - 1;   // >= 0 on every lane: slot 0 of round 0 carries a mark
            const int j = base + lane;
            const float4 r0 = L.ray0[owner], r1 = L.ray1[owner];
#ifdef CRT_CHECKED
            // checked build: the fast path's per-pair bounds re-checked, as in the rounds below
            const bool bad = j < total && ((unsigned)owner >= 64u || j < L.prefix[owner] ||
                                           j >= L.prefix[owner] + L.span_n[owner] ||
                                           (unsigned)(__float_as_int(r1.w) + j) >= (unsigned)P.n_prims);
            if (bad) atomicOr(P.err, 4u);
            const bool act = j < total && !bad;
#else
            const bool act = j < total;
#endif
            const int pp = act ? __float_as_int(r1.w) + j : 0;
            const float4* rr = rec_at(P.prims, __umul24((uint32_t)pp, 48u));
            const float4 f0 = rr[0], f1 = rr[1], f2 = rr[2];
            if constexpr (decltype(first)::value) {
                __asm__ volatile("" : : : "memory");   // the rows after the records
                load_node_rows(P.nodes, node_base(node >= 0 ? node : 0), rows, pf);
            }
            if (act) {
                if (COUNT) cnt.tris++;
                __asm__ volatile("" : : "v"(f2.y));   // the third row as one dwordx4 (prim_test)
                const V3 ro = v3(r0.x, r0.y, r0.z), rd = v3(r0.w, r1.x, r1.y);
                const int rank = __float_as_int(f2.z);
                const float t = (P.tree_spheres != 0 && __float_as_int(f2.w) == 1) ? sphere_candidate(f0, f1, ro, rd, r1.z)
                                                                                  : tri_test_flat(f0, f1, f2, ro, rd, r1.z);
                const unsigned long long kp = ((unsigned long long)__float_as_uint(t) << 32) | (0xffffffffu - (unsigned)rank);
                atomicMin(&L.key[owner], t >= 0.f ? kp : ~0ull);
            }
            carry = __builtin_amdgcn_readlane(owner1, 63);
            wave_sync();
        };
        round(0, std::true_type{});
        *pf_node = node;
        for (int base = 64; base < total; base += 64) round(base, std::false_type{});
    } else
    for (int base = 0; base < total; base += 64) {
        if (COUNT || kProfilePass) cnt.round_slots++;
        if (leaf_n > 0 && pfx >= base && pfx < base + 64) L.owner_at[pfx - base] = (unsigned char)(lane + 1);
        wave_sync();
        const uint32_t mark = L.owner_at[lane];
        L.owner_at[lane] = 0;
        const uint32_t owner1 = max(wave_inclusive_max_scan_u(mark), carry);
        const int owner = (int)owner1 - 1;
        const int j = base + lane;
#ifdef CRT_PROFILE_ROWS
        uint64_t prim_wait = 0;
#endif
        if (j < total) {
            const float4 r0 = L.ray0[owner], r1 = L.ray1[owner];
            const int p = __float_as_int(r1.w) + j;   // leaf_first - prefix + j: inside the owner's checked span
            if (COUNT) cnt.tris++;
            int rank;
#ifdef CRT_PROFILE_ROWS
            {   // profiling build: the pair's record loaded and waited for between two timers (prim_test reloads it
                // from the vector L1)
                const float4* rr = rec_at(P.prims, __umul24((uint32_t)p, 48u));
                const uint64_t pa = shader_clock();
                const float4 g0 = rr[0], g1 = rr[1], g2 = rr[2];
                __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
                __asm__ volatile("" : : "v"(g0.x), "v"(g1.x), "v"(g2.x) : "memory");
                prim_wait = shader_clock() - pa;
            }
#endif
#ifdef CRT_CHECKED
            // checked build (-DCRT_CHECKED, lib/checked/): the per-pair bounds the fast path proves once per lane and
            // step (node_step4), re-checked here with the owner lookup itself, so a stale LDS owner mark or a wrong
            // prefix reports through P.err instead of loading outside the primitive array
            const bool bad = (unsigned)owner >= 64u || j < L.prefix[owner] || j >= L.prefix[owner] + L.span_n[owner] ||
                             (unsigned)p >= (unsigned)P.n_prims;
            if (bad) atomicOr(P.err, 4u);
            rank = -1;
            const float t = bad ? -1.f : prim_test(P.prims, p, v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y), r1.z, rank,
                                                   P.tree_spheres != 0);
#else
            const float t = prim_test(P.prims, p, v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y), r1.z, rank,
                                      P.tree_spheres != 0);
#endif
            // a rejected pair offers the empty key (no effect on the min): one LDS atomic per pair, no branch
            // (-0.75 %, profiles/r02ar)
            const unsigned long long kp = ((unsigned long long)__float_as_uint(t) << 32) | (0xffffffffu - (unsigned)rank);
            atomicMin(&L.key[owner], t >= 0.f ? kp : ~0ull);
        }
#ifdef CRT_PROFILE_ROWS
        cnt.cyc_prims += bcast64(prim_wait, 0);   // lane 0's slot base + 0 < total is always tested
#endif
        carry = __builtin_amdgcn_readlane(owner1, 63);
        wave_sync();
    }
    {
        const unsigned long long kk = L.key[lane];
        const float t = __uint_as_float((unsigned)(kk >> 32));
        const int rank = (int)(0xffffffffu - (unsigned)kk);
        if (leaf_n > 0 && kk != ~0ull && better(t, rank, closest, hit)) {
            closest = t;
            hit = rank;
        }
    }
    if (TIME) cnt.cyc_round += shader_clock() - c1;
}

// The tree's top nodes held in LDS (CRT_TOP_LEVELS): the root and, at level 2, its internal children, copied once
// per workgroup with their rows unswizzled (row k at 16-B slot k).  Every ray starts at the root, and its first node
// steps are the same for every ray up to the direction signs, so a new ray takes them in the regeneration pass from
// LDS instead of in traversal steps that wait for L1/L2: the same box tests with the same operands (closest = inf,
// no leaf was tested yet), the same near-first order and stack entries, hence the same traversal bit for bit.
#ifndef CRT_TOP_LEVELS
#define CRT_TOP_LEVELS 1
#endif
constexpr int TOP_NODES = CRT_TOP_LEVELS >= 2 ? 5 : CRT_TOP_LEVELS >= 1 ? 1 : 0;

// One node step of node_step4 on an LDS record, for a lane whose ray has tested no leaf yet (closest = inf).  Returns
// false, changing nothing, when a leaf child is hit: the lane then takes this node through the regular step, whose
// leaf rounds test it.
template <bool COUNT>
__device__ __forceinline__ bool top_step4(const RenderParams& P, const float4* rec, V3 o, V3 inv, uint32_t rows,
                                          int& node, int& sp, TraceCounts& cnt, uint32_t* __restrict__ stk,
                                          size_t pix, size_t n_pix) {
    const Wide4 w = wide_boxes(rec, 0u, rows, o, inv, __builtin_inff());
    const float4 mf = rec[6];
    const int first_child = __float_as_int(mf.x);
    const int meta = __float_as_int(mf.y);
    const int n_int = meta & 0xff;
    uint32_t hm = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) hm |= w.hit[s] ? (1u << s) : 0u;
    if (hm & (0xfu << n_int)) return false;
    if (COUNT) cnt.boxes += (uint32_t)(meta >> 8);
    uint32_t k[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) k[s] = (s < n_int && w.hit[s]) ? ((__float_as_uint(w.tmin[s]) & ~3u) | s) : ~0u;
    cas(k[0], k[1]); cas(k[2], k[3]); cas(k[0], k[2]); cas(k[1], k[3]); cas(k[1], k[2]);
    auto store = [&](int at, uint32_t v) -> bool {
        if (at < P.stack_lds) stk[at * 64 + lane_fresh()] = v;
        else if (at < P.stack_cap) *ovf_slot(P, at, pix, n_pix) = v;
        else { atomicOr(P.err, 2u); return false; }
        return true;
    };
    if (k[0] != ~0u) {
        node = first_child + (int)(k[0] & 3);
        const uint32_t n_rest = (uint32_t)__popc(hm & ((1u << n_int) - 1u)) - 1u;
        if (n_rest && store(sp, ((uint32_t)first_child << 8) | (n_rest << 6) | ((k[1] & 3) << 4) |
                                    ((k[2] & 3) << 2) | (k[3] & 3)))
            ++sp;
    } else if (sp > 0) {
        const int at = sp - 1;
        const uint32_t top = at < P.stack_lds ? stk[at * 64 + lane_fresh()]
                                              : (at < P.stack_cap ? *ovf_slot(P, at, pix, n_pix) : 0u);
        const uint32_t rest = (top >> 6) & 3;
        node = (int)(top >> 8) + (int)((top >> 4) & 3);
        if (rest <= 1) sp = at;
        else store(at, (top & ~0xffu) | ((rest - 1) << 6) | ((top & 0xfu) << 2));
    } else {
        node = -1;
    }
    return true;
}

// A new ray's first node steps from the LDS top nodes: the root, then (TOPN = 5) the internal child it continues to.
template <bool COUNT, int TOPN>
__device__ __forceinline__ void top_steps(const RenderParams& P, const float4* top, V3 o, V3 inv, uint32_t rows,
                                          int& node, int& sp, TraceCounts& cnt, uint32_t* __restrict__ stk, size_t pix,
                                          size_t n_pix) {
    if (P.top_levels <= 0) return;   // uniform
    if (!top_step4<COUNT>(P, top, o, inv, rows, node, sp, cnt, stk, pix, n_pix) || TOPN < 5 || P.top_levels < 2 ||
        node < 0)
        return;
    const int m = node - __float_as_int(top[6].x);   // node is an internal child of the root: slot m < 4
    if ((unsigned)m < 4u) top_step4<COUNT>(P, top + 8 * (1 + m), o, inv, rows, node, sp, cnt, stk, pix, n_pix);
}

// Per-lane path state of one pixel (rayColor's locals, CUDAKernels.h:102-145, plus the sample loop).
struct PathState {
    Rng s;
    V3 pixel, o, d, thr;
    int remaining, bounce;
    bool need_new;
    uint32_t rays, paths;
#ifdef CRT_PROFILE_LOOPS
    uint32_t k1, k2, kr;   // this pass: unit-sphere candidates, unit-disk candidates, Russian-roulette draws
#endif
};
#ifdef CRT_PROFILE_LOOPS
// Profiling build only (tools/build_profile_lib.sh loops -DCRT_PROFILE_LOOPS, tools/loop_fusion_count.py): the
// regeneration pass's two rejection loops, counted from the XORWOW draw counter (d advances by 362437 per draw;
// 945708813 is its inverse mod 2^32).  Summed over variant 8's passes: [0] passes, [1] sum of the wave's max unit-sphere
// candidates, [2] max unit-disk candidates, [3] max over lanes of (sphere + disk candidates), the iteration count of
// one fused loop, [4] max over lanes of (sphere + RR + disk) draws-steps, [5] lane sum of sphere candidates, [6] lane
// sum of disk candidates, [7] parked lanes
__device__ unsigned long long g_loop_prof[8];
__device__ __forceinline__ uint32_t draws_since(uint32_t d0, uint32_t d1) { return (d1 - d0) * 945708813u; }
#endif

struct CamRegs {
    V3 pos, llc, hor, ver, right, up;
    float lens, fw, fh;
    float rfw, rfh;   // RN(1 / fw), RN(1 / fh) (host IEEE division)
    int fast_uv;      // uv_div is verified exact for this frame size (crt_renderer_create): no IEEE division
};

// Phase 1: give the lane a ray to trace — Camera::getRay for a new sample, the bounce-limit exit and
// Russian roulette (CUDAKernels.h:110-121).  Returns false when the pixel has no samples left.
__device__ __forceinline__ bool next_ray(PathState& S, const CamRegs& C, int x, int y, int max_bounces) {
    for (;;) {
        if (S.need_new) {
            if (S.remaining == 0) return false;
            --S.remaining;
            float da, db;                                    // Utility::randomPointInUnitDisk
#ifdef CRT_PROFILE_LOOPS
            const uint32_t pd0 = S.s.d;
#endif
            for (;;) {
                da = rand_pm1(S.s);
                db = rand_pm1(S.s);
                if (len2(v3(da, db, 0)) >= 1) continue;
                break;
            }
#ifdef CRT_PROFILE_LOOPS
            S.k2 += draws_since(pd0, S.s.d) / 2u;
#endif
            const V3 rd = C.lens * v3(da, db, 0);
            const V3 off = v3(C.right.x * rd.x, C.right.y * rd.x, C.right.z * rd.x) +
                           v3(C.up.x * rd.y, C.up.y * rd.y, C.up.z * rd.y);
            const float au = (float)x + uniform(S.s);
            const float av = (float)y + uniform(S.s);
            float u, v;
            if (C.fast_uv) {
                u = uv_div(au, C.fw, C.rfw);
                v = uv_div(av, C.fh, C.rfh);
            } else {
                __asm__ volatile("");   // a real branch: no if-conversion that would run both divisions
                u = au / C.fw;
                v = av / C.fh;
            }
            S.o = C.pos + off;
            S.d = (((C.llc + u * C.hor) + v * C.ver) - C.pos) - off;
            S.thr = v3(1.0f, 1.0f, 1.0f);
            S.bounce = 0;
            S.need_new = false;
        }
        if (S.bounce >= max_bounces) {                      // loop exhausted: final_color = 0
            S.pixel = S.pixel + v3(0.0f, 0.0f, 0.0f);
            ++S.paths;
            S.need_new = true;
            continue;
        }
        if (S.bounce >= 3) {
            float p = fmaxf(S.thr.x, fmaxf(S.thr.y, S.thr.z));
            p = fminf(p, 0.95f);
#ifdef CRT_PROFILE_LOOPS
            S.kr += 1u;
#endif
            if (uniform(S.s) > p) {
                S.pixel = S.pixel + v3(0.0f, 0.0f, 0.0f);
                ++S.paths;
                S.need_new = true;
                continue;
            }
            S.thr = recip_exact_wave(p) * S.thr;   // 1 / p, exact (crt_device.h)
        }
        return true;
    }
}

// Dielectric::scatter's total-internal-reflection test in double, as the reference computes it (Material.cuh:115-118):
//   cannot = RN(ri * RN(sqrt(y))) > 1,   y = RN(1 - c * c)   (c * c is exact in double: two 24-bit factors).
// sqrt and the product are correctly rounded and monotone, so ri^2 * y decides the outcome unless it is within a hair
// of 1.  z = RN(RN(ri * ri) * y) is within a relative 2^-52 of ri^2 * y.  If z > 1 + 2^-40, then ri * sqrt(y) >
// 1 + 2^-43, and the two roundings (a relative 2^-53 each) keep RN(ri * RN(sqrt(y))) above 1 + 2^-53, so it rounds
// above 1.  If z < 1 - 2^-40, the product stays below 1.  Only a wave with a lane in between (or a NaN) runs the
// reference's f64 sqrt; the f64 sqrt sequence is otherwise the most expensive part of the glass shading.
__device__ __forceinline__ bool cannot_refract_exact(float cos_theta, float ri) {
    const double c = cos_theta, r = ri;
    const double y = __builtin_fma(-c, c, 1.0);          // == RN(1.0 - c * c): the product is exact
    const double z = (r * r) * y;
    const bool above = z > 1.0 + 0x1p-40, below = z < 1.0 - 0x1p-40;
    if (__builtin_amdgcn_ballot_w64(!(above || below)) == 0) return above;
    // keeps the f64 sqrt behind the branch: without it the compiler if-converts the uniform branch and computes the
    // sqrt sequence in every wave with a glass hit, then selects
    __asm__ volatile("");
    return r * sqrt(y) > 1.0;
}

// Phase 3: material scatter / emit / sky (CUDAKernels.h:123-142, Material.cuh:66-146).  The hit's normal and
// material come from its shading record (crt_device.h): one pair of independent loads per hit.
// shade_rec: the same with the hit's shading record rows 0-1 already loaded (r0, m); a sphere's row 2 (1 / radius) is
// inv_r when `staged`, else loaded here.
__device__ __forceinline__ void shade_rec(PathState& S, const RenderParams& P, int hit_rank, float t, float4 r0,
                                          float4 m, bool staged, float inv_r);
__device__ __forceinline__ void shade(PathState& S, const RenderParams& P, int hit_rank, float t) {
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), m = r0;
    if (hit_rank >= 0) {
        const float4* R = P.shade + 3u * (uint32_t)hit_rank;   // 32-bit index (ranks < 2^30): no 64-bit multiply
        r0 = R[0];
        m = R[1];
    }
    shade_rec(S, P, hit_rank, t, r0, m, false, 0.f);
}
__device__ __forceinline__ void shade_rec(PathState& S, const RenderParams& P, int hit_rank, float t, float4 r0,
                                          float4 m, bool staged, float inv_r) {
    if (hit_rank < 0) {                                  // :137-142
        S.pixel = S.pixel + S.thr * sky(S.d);
        ++S.paths;
        S.need_new = true;
        return;
    }
    const uint32_t kind = __float_as_uint(r0.w);
    const V3 hp = S.o + t * S.d;                         // Ray::pointAtDistance
    V3 outward = v3(r0.x, r0.y, r0.z);                   // triangle: unit(cross(e1, e2)), Mesh.cuh:303-304
    if (kind & SHADE_SPHERE) {                           // Sphere.cuh:44: (1 / radius) * (p - center)
        const float ir = staged ? inv_r : P.shade[3u * (uint32_t)hit_rank + 2u].x;
        outward = ir * (hp - outward);
    }
    const bool front = dot(S.d, outward) < 0;            // HitInfo::setFaceNormal
    const V3 n = front ? outward : -outward;
    const uint32_t code = kind & 15u;
    if (code == SHADE_INVALID) {                         // :127 invalid material: same ray again
        ++S.bounce;
        return;
    }
    // Lambertian and Metal both draw one randomUnitVector first (their only draws): one rejection loop for
    // both, so a wave holding both materials does not run the loop twice.
    V3 ruv;
#ifdef CRT_PROFILE_LOOPS
    const uint32_t pd0 = S.s.d;
#endif
    if (code == SHADE_LAMBERT || code == SHADE_METAL) ruv = rand_unit_vector(S.s);
#ifdef CRT_PROFILE_LOOPS
    S.k1 += draws_since(pd0, S.s.d) / 3u;
#endif
    if (code == SHADE_LAMBERT) {                         // Material.cuh:66-77
        V3 sd = n + ruv;
        if (fabsf(sd.x) < 1e-8f && fabsf(sd.y) < 1e-8f && fabsf(sd.z) < 1e-8f) sd = n;
        S.thr = S.thr * v3(m.x, m.y, m.z);
        S.o = hp;
        S.d = sd;
        ++S.bounce;
    } else if (code == SHADE_METAL) {                    // :89-96
        V3 refl = reflect(S.d, n);
        refl = unit(refl) + (m.w * ruv);
        if (dot(refl, n) > 0) {
            S.thr = S.thr * v3(m.x, m.y, m.z);
            S.o = hp;
            S.d = refl;
            ++S.bounce;
        } else {                                         // absorbed: return Material::emit() = 0
            S.pixel = S.pixel + v3(0.0f, 0.0f, 0.0f);
            ++S.paths;
            S.need_new = true;
        }
    } else if (code == SHADE_DIELECTRIC) {               // :109-128
        const float ri = front ? m.y : m.x;              // 1.0f / ior (front face) or ior, from the shading record
        const float r0 = front ? m.z : m.w;              // Schlick's r0 for that ri
        const V3 ud = unit(S.d);
        const float cos_theta = fminf(dot(-ud, n), 1.0f);
        const bool cannot_refract = cannot_refract_exact(cos_theta, ri);
        V3 dir;
        if (cannot_refract || schlick_r0(cos_theta, r0) > uniform(S.s))
            dir = reflect(ud, n);
        else
            dir = refract(ud, n, ri);
        S.o = hp;
        S.d = dir;
        ++S.bounce;   // attenuation (1,1,1): thr unchanged (x*1 == x)
    } else {                                             // DiffuseLight: return emit() raw
        const V3 em = code == SHADE_LIGHT ? v3(m.x, m.y, m.z) : v3(0.0f, 0.0f, 0.0f);
        S.pixel = S.pixel + em;
        ++S.paths;
        S.need_new = true;
    }
}

// A parked lane's end of trace in the regeneration pass (4-wide variants): the per-ray spheres (Sphere::hit behind the
// reference's sphere box, ray_spheres) and then shade.  The trace's own hit record is loaded before the sphere test,
// behind a compiler barrier, so its latency hides behind that test (-0.6 %, profiles/r03aa); when a per-ray sphere
// wins, its record comes from the LDS copy of the two per-ray spheres' records (or from HBM for other sphere counts).
template <bool COUNT>
__device__ __forceinline__ void finish_ray(PathState& S, const RenderParams& P, V3 inv, float closest, int hit,
                                           const float* sph_lds, const float4* shd_lds, TraceCounts& cnt, uint64_t s0) {
    const int h0 = hit;
    float4 e0 = make_float4(0.f, 0.f, 0.f, 0.f), e1 = e0;
    if (h0 >= 0) {
        const float4* Rh = P.shade + 3u * (uint32_t)h0;
        e0 = Rh[0];
        e1 = Rh[1];
    }
    __asm__ volatile("" : : : "memory");   // keep the loads ahead of the sphere test
    ray_spheres<true>(P.prims, P.sphere_chain, P.n_chain, P.sphere_first, P.n_ray_spheres, S.o, S.d,
                      sphere_inv(S.d, inv), closest, hit, sph_lds);
    if (COUNT || kProfilePass) cnt.cyc_sph += shader_clock() - s0;
    bool staged = false;
    float inv_r = 0.f;
    if (hit != h0 && hit >= 0) {   // a per-ray sphere won: its record from LDS (two spheres) or HBM
        if (P.n_ray_spheres == 2) {
            const int k = hit == __float_as_int(sph_lds[26]) ? 3 : 0;
            e0 = shd_lds[k];
            e1 = shd_lds[k + 1];
            inv_r = shd_lds[k + 2].x;
            staged = true;
        } else {
            const float4* Rh = P.shade + 3u * (uint32_t)hit;
            e0 = Rh[0];
            e1 = Rh[1];
        }
    }
    shade_rec(S, P, hit, closest, e0, e1, staged, inv_r);
}

// VARIANT 0: per-lane traversal (leaf loops inside the lane).  VARIANT 1: cooperative leaves.
// VARIANT 2: cooperative leaves + traversal-step scheduling.  MINW: occupancy target (waves per SIMD)
// handed to the register allocator through __launch_bounds__.
#ifdef CRT_PROFILE_WAVE_TIMES
// Profiling build only (tools/build_profile_lib.sh): per-wave start/end of the last render launch
// (s_memrealtime, 100 MHz), read with crt_profile_wave_times — the occupancy timeline of the launch.
__device__ unsigned long long g_wave_prof[2 * 4 * 65536];
#endif
#ifdef CRT_PROFILE_CRIT_TRACE
// Profiling build only (tools/crit_trace.py): the first workgroup of a variant-8 launch (the most expensive tile) logs
// s_memrealtime and its live / parked lane counts every 16 loop iterations, and every wave logs where it ran (HW_ID,
// XCC_ID), so the critical wave's iteration rate can be set against the waves sharing its SIMD over time
__device__ unsigned long long g_crit_trace[2 * 16384];
__device__ unsigned g_wave_hw[2 * 4 * 65536];
#endif

// Waves per workgroup: 4 (16x16 pixels), or 1 for variant 8 (one 8x8 tile per workgroup, so a finished wave frees
// its slot at once instead of holding it until its three siblings end).
template <int VARIANT> struct KernelShape { static constexpr int waves = VARIANT == 8 || VARIANT == 10 ? 1 : 4; };

template <bool COUNT, int VARIANT, int MINW>
__global__ __launch_bounds__(64 * KernelShape<VARIANT>::waves, MINW) void crt_render_kernel(RenderParams P) {
#ifdef CRT_PROFILE_WAVE_TIMES
    const unsigned long long prof_t0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef CRT_PROFILE_PASS
    const uint64_t prof_life0 = shader_clock();
#endif
    constexpr int WGW = KernelShape<VARIANT>::waves;
    // variant 4: 16 LDS stack entries per lane at 5 waves/SIMD; 12 at 6+ so 6 workgroups fit the 160 KiB
    constexpr bool PERSIST = VARIANT == 7;
    constexpr bool TILED = VARIANT == 8;    // variant 4 with one wave per workgroup and a tile order
    constexpr bool TILES = TILED || VARIANT == 10;   // one 8x8 tile per one-wave workgroup (variant 10: variant 3's program)
    constexpr bool WIDE = VARIANT == 4 || PERSIST || TILED;
    using Lds = std::conditional_t<WIDE, WaveLdsWide, WaveLds>;
    __shared__ Lds lds[VARIANT >= 1 ? WGW : 1];
    constexpr int SD = WIDE ? (MINW >= 7 ? CRT_STACK7 : MINW >= 6 ? CRT_STACK6 : STACK_LDS) : 1;
    __shared__ uint32_t stack_lds[WIDE ? WGW * SD * 64 : 1];
    // the two per-ray spheres in 16-B rows, so every read is one ds_read_b128 at a fixed offset: per sphere
    // (center.xyz, radius^2) (box lo.xyz, box hi.x) (box hi.yz, rank, 0) (unused)
    __shared__ __attribute__((aligned(16))) float sph_lds[32];
    constexpr int TOPN = WIDE ? TOP_NODES : 0;
    // the two per-ray spheres' shading records (3 rows each), so a pass whose sphere test overrides the trace's hit
    // reads the record from LDS (the trace's own hit record is loaded at the pass start)
    __shared__ float4 shd_lds[WIDE ? 6 : 1];
    __shared__ float4 top_lds[TOPN > 0 ? 8 * TOPN : 1];   // CRT_TOP_LEVELS: root, then its internal children
    __shared__ uint32_t rays0_lds[PERSIST ? 64 * WGW : 1];   // variant 7: the lane's ray count when its pixel started
    if (WIDE) {
        if (threadIdx.x < 32) {
            const int k = threadIdx.x & 15;
            const int src = k < 4 ? k : k < 9 ? k + 1 : k == 9 ? 10 : k == 10 ? 4 : -1;
            sph_lds[threadIdx.x] = src < 0 ? 0.f : P.sph2[threadIdx.x >> 4][src];
        }
        if (threadIdx.x >= 32 && threadIdx.x < 38 && P.n_ray_spheres == 2) {
            const uint32_t q = threadIdx.x - 32, sp = q / 3;
            shd_lds[q] = P.shade[3u * (uint32_t)__float_as_int(P.sph2[sp][4]) + q % 3];
        }
        if (TOPN > 0 && threadIdx.x < 8u * TOPN) {
            const uint32_t m = threadIdx.x >> 3, k = threadIdx.x & 7;
            int n = 0;
            if (m > 0) {   // internal child m - 1 of the root (BFS emission: consecutive from first_child)
                const float4 rm = node_row(P.nodes, node_base(0), 6);
                n = (int)(m - 1) < (__float_as_int(rm.y) & 0xff) ? __float_as_int(rm.x) + (int)(m - 1) : -1;
            }
            if (n >= 0 && n < P.n_nodes) top_lds[threadIdx.x] = node_row(P.nodes, node_base(n), k);
        }
        __syncthreads();
    }
    // 16x16 pixel tile per workgroup, 8x8 per wave64.
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: LDS bases stay scalar
    int x, y;
    if (TILES) {                               // workgroup b renders 8x8 tile order[b]
        const uint32_t t = P.order ? P.order[blockIdx.x] : blockIdx.x;
        x = (int)(t % (uint32_t)P.tiles_x) * 8 + (lane & 7);
        y = (int)(t / (uint32_t)P.tiles_x) * 8 + (lane >> 3);
    } else {
        x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
        y = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
        if (VARIANT == 4 && P.probe_cost) {   // a subsampled cost probe (crt_renderer_set_schedule's stride)
            x *= P.probe_stride;
            y *= P.probe_stride;
        }
    }
    const bool valid = x < P.width && y < P.height;
    const int pix = valid ? y * P.width + x : 0;

    PathState S;
    S.s = Rng{0, 0, 0, 0, 0, 0};
    S.pixel = v3(0.f, 0.f, 0.f);
    S.o = v3(0, 0, 0); S.d = v3(0, 0, 1); S.thr = v3(1, 1, 1);
    S.remaining = 0; S.bounce = 0; S.need_new = true; S.rays = 0; S.paths = 0;
#ifdef CRT_PROFILE_LOOPS
    S.k1 = S.k2 = S.kr = 0;
    unsigned long long lp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    if (valid && !PERSIST) {
        const uint32_t* r = P.rng + 6 * (size_t)pix;
        S.s.v0 = r[0]; S.s.v1 = r[1]; S.s.v2 = r[2]; S.s.v3 = r[3]; S.s.v4 = r[4]; S.s.d = r[5];
        if (P.accumulate) S.pixel = v3(P.sum[3 * (size_t)pix], P.sum[3 * (size_t)pix + 1], P.sum[3 * (size_t)pix + 2]);
        S.remaining = P.spp;
    }
    const crt_camera_desc& Cd = P.cam;
    CamRegs C;
    C.pos = v3(Cd.origin[0], Cd.origin[1], Cd.origin[2]);
    C.llc = v3(Cd.lower_left[0], Cd.lower_left[1], Cd.lower_left[2]);
    C.hor = v3(Cd.horizontal[0], Cd.horizontal[1], Cd.horizontal[2]);
    C.ver = v3(Cd.vertical[0], Cd.vertical[1], Cd.vertical[2]);
    C.right = v3(Cd.right[0], Cd.right[1], Cd.right[2]);
    C.up = v3(Cd.up[0], Cd.up[1], Cd.up[2]);
    C.lens = Cd.lens_radius;
    C.fw = (float)P.width;
    C.fh = (float)P.height;
    C.rfw = P.rcp_w;
    C.rfh = P.rcp_h;
    C.fast_uv = P.fast_uv;
    TraceCounts cnt{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t wave_rays = 0;    // variant 8: rays of the wave (uniform); the other variants count per lane

    if constexpr (VARIANT == 0) {
        for (;;) {
            if (!next_ray(S, C, x, y, P.max_bounces)) break;
            ++S.rays;
            float t;
            const int hit = trace<COUNT>(P.nodes, P.prims, P.n_nodes, layout_base(S.d, P.n_layouts, P.n_nodes), S.o,
                                         S.d, t, cnt);
            shade(S, P, hit, t);
        }
    } else if constexpr (PERSIST) {
        // Variant 4's scheduling, but a lane whose pixel has no samples left stores it and takes the next
        // pixel slot from the global queue (8x8 tiles in `order`, most expensive first), so lanes never wait
        // for their wave's slowest pixel and waves never wait for their workgroup or the launch's last tiles.
        // Each pixel is still traced by ONE lane, samples in order, from its own RNG stream: same results.
        auto& L = lds[wave];
        uint32_t* stk = stack_lds + wave * SD * 64;
        const float INF = __builtin_inff();
        const size_t n_pix = (size_t)P.width * P.height;
        const uint32_t total_slots = (uint32_t)P.n_slots;
        const uint64_t below = (1ull << lane) - 1ull;
        bool live = false, has_result = false, have = false;
        int node = -1, sp = 0, hit = -1, px = 0, py = 0, ppix = 0;
        float closest = INF;
        V3 inv = v3(0.f, 0.f, 0.f);
        uint32_t rows = 0;         // ray_rows(inv)
        uint32_t pool = 0, used = 64;    // wave-uniform: first slot of the reserved block, slots handed out
        bool exhausted = false;
        L.owner_at[lane] = 0;
        for (;;) {
            const bool parked = live && node < 0;
            const int n_parked = __popcll(wave_ballot(parked));
            const int n_live = __popcll(wave_ballot(live));
            const uint64_t c0 = COUNT ? shader_clock() : 0;
            // once the queue is empty the wave only drains: its last paths no longer wait for many parked lanes
            // (crt_renderer_set_drain_threshold)
            const int regen_t = exhausted ? P.drain_threshold : P.regen_threshold;
            if (n_parked >= regen_t || n_parked == n_live) {
                if (COUNT) cnt.passes++;
                if (parked) {
                    if (has_result) finish_ray<COUNT>(S, P, inv, closest, hit, sph_lds, shd_lds, cnt, c0);
                    live = next_ray(S, C, px, py, P.max_bounces);
                    has_result = false;
                }
                if (have && !live) {     // the pixel's samples are done: store it (CUDAKernels.h:162-165)
                    uint32_t* r = P.rng + 6 * (size_t)ppix;
                    r[0] = S.s.v0; r[1] = S.s.v1; r[2] = S.s.v2; r[3] = S.s.v3; r[4] = S.s.v4; r[5] = S.s.d;
                    P.sum[3 * (size_t)ppix] = S.pixel.x;
                    P.sum[3 * (size_t)ppix + 1] = S.pixel.y;
                    P.sum[3 * (size_t)ppix + 2] = S.pixel.z;
                    if (P.pix_rays) P.pix_rays[ppix] = S.rays - rays0_lds[threadIdx.x];
                    have = false;
                }
                while (!exhausted) {                // lanes without a pixel take the next slots
                    const uint64_t need = wave_ballot(!have);
                    if (need == 0) break;
                    if (used >= 64u) {
                        uint32_t b = 0;
                        if (lane == 0) b = atomicAdd(P.queue, 64u);
                        pool = __builtin_amdgcn_readfirstlane(b);
                        used = 0;
                        if (pool >= total_slots) { exhausted = true; break; }
                    }
                    const uint32_t take = min((uint32_t)__popcll(need), 64u - used);
                    const uint32_t rank = (uint32_t)__popcll(need & below);
                    if (!have && rank < take && pool + used + rank < total_slots) {
                        const uint32_t pixel = P.order[pool + used + rank];
                        if (pixel != 0xffffffffu) {
                            ppix = (int)pixel;
                            px = ppix % P.width;
                            py = ppix / P.width;
                            const uint32_t* r = P.rng + 6 * (size_t)ppix;
                            S.s.v0 = r[0]; S.s.v1 = r[1]; S.s.v2 = r[2]; S.s.v3 = r[3]; S.s.v4 = r[4]; S.s.d = r[5];
                            S.pixel = P.accumulate ? v3(P.sum[3 * (size_t)ppix], P.sum[3 * (size_t)ppix + 1],
                                                        P.sum[3 * (size_t)ppix + 2])
                                                   : v3(0.f, 0.f, 0.f);
                            S.remaining = P.spp;
                            S.need_new = true;
                            have = true;
                            rays0_lds[threadIdx.x] = S.rays;
                            live = next_ray(S, C, px, py, P.max_bounces);
                            if (!live) {         // spp == 0: nothing to trace, store as is
                                uint32_t* w = P.rng + 6 * (size_t)ppix;
                                w[0] = S.s.v0; w[1] = S.s.v1; w[2] = S.s.v2; w[3] = S.s.v3; w[4] = S.s.v4; w[5] = S.s.d;
                                P.sum[3 * (size_t)ppix] = S.pixel.x;
                                P.sum[3 * (size_t)ppix + 1] = S.pixel.y;
                                P.sum[3 * (size_t)ppix + 2] = S.pixel.z;
                                if (P.pix_rays) P.pix_rays[ppix] = 0;
                                have = false;
                            }
                        }
                    }
                    used += take;
                }
                if (live && node < 0) {          // a new ray: the parked lanes' next ray or a new pixel's first
                    ++S.rays;
                    has_result = true;
                    node = 0;
                    sp = 0;
                    closest = INF;
                    hit = -1;
                    inv = recip3_exact(S.d);
                    inv = box_inv(inv);   // the traversal's 1/d (wide_boxes)
                    rows = ray_rows(inv);
                    if (COUNT) cnt.spheres += P.n_ray_spheres;
                    L.ray0[lane] = make_float4(S.o.x, S.o.y, S.o.z, S.d.x);
                    if (COUNT) cnt.trace_calls++;
                    if (TOPN > 0) top_steps<COUNT, TOPN>(P, top_lds, S.o, inv, rows, node, sp, cnt, stk, (size_t)ppix, n_pix);
                }
                if (!wave_ballot(live)) break;      // the queue is empty and every lane is done
            }
            if (COUNT) cnt.cyc_regen += shader_clock() - c0;
            traverse_step4<COUNT>(P, S.o, S.d, inv, rows, node, sp, closest, hit, cnt, L, stk, lane, (size_t)ppix, n_pix);
        }
    } else if constexpr (WIDE) {
        // Same scheduling as variant 3 over a 4-wide BVH: node < 0 = no node left (lane parked).
        auto& L = lds[wave];
        uint32_t* stk = stack_lds + wave * SD * 64;
        const float INF = __builtin_inff();
        const size_t n_pix = (size_t)P.width * P.height;
        // Lane masks instead of per-lane bools for the per-step tests: a ballot of a bool the compiler keeps as a lane
        // mask costs two VALU (widen, compare), a ballot of a compare none.  Every lane starts live (a pixel without
        // samples ends at the first pass); after a pass the live lanes are exactly those with a ray (has_result).
        uint64_t live_mask = wave_ballot(true);
        bool has_result = false;
        int node = -1, sp = 0, hit = -1;
        float closest = INF;
        V3 inv = v3(0.f, 0.f, 0.f);
        uint32_t rows = 0;         // ray_rows(inv)
        L.owner_at[lane] = 0;      // traverse_step4: owner + 1, 0 = none
        if (TILED && lane == 0) L.rays = 0;
        // variant 8: the most expensive tiles of the cost order bound the frame when it has few tiles per wave slot
        // (their pixels' sample chains are sequential); they regenerate sooner (profiles/r02h)
        const int regen_t = (TILED && (int)blockIdx.x < P.crit_tiles) ? P.crit_threshold : P.regen_threshold;
        bool first_pass = true;    // uniform
        // variant 8 at occupancy 4 (frames of few tiles per wave slot, bound by their most expensive tiles' sample
        // chains): the next node's rows load during the leaf round (traverse_step4<.., true>, profiles/r06r, r06s)
        constexpr bool PFV = TILED && MINW <= 4;
        float4 pf[PFV ? 7 : 1];
        int pf_node = -1;   // the node whose rows pf holds
#ifdef CRT_PROFILE_CRIT_TRACE
        uint32_t crit_iter = 0;
#endif
#ifdef CRT_PROFILE_LIVE
        uint64_t lh0 = 0, lh1 = 0, lh2 = 0, lh3 = 0, lh4 = 0, lh5 = 0, lh6 = 0, lh7 = 0, lh8 = 0;
        uint64_t lt_prev = shader_clock();
        int lb_prev = 8;
#endif
        constexpr bool TIME = COUNT || kProfilePass;
        for (;;) {
            const uint64_t h0 = kProfilePass ? shader_clock() : 0;
            const uint64_t parked_mask = live_mask & wave_ballot(node < 0);
            const int n_parked = __popcll(parked_mask);
            const int n_live = __popcll(live_mask);
#ifdef CRT_PROFILE_LIVE
            if (TILED) {
                const uint64_t lt = shader_clock(), dt = lt - lt_prev;
                lt_prev = lt;
                lh0 += lb_prev == 0 ? dt : 0; lh1 += lb_prev == 1 ? dt : 0; lh2 += lb_prev == 2 ? dt : 0;
                lh3 += lb_prev == 3 ? dt : 0; lh4 += lb_prev == 4 ? dt : 0; lh5 += lb_prev == 5 ? dt : 0;
                lh6 += lb_prev == 6 ? dt : 0; lh7 += lb_prev == 7 ? dt : 0; lh8 += lb_prev == 8 ? dt : 0;
                lb_prev = n_live >> 3;
                if (n_live == 0 && lane == 0) {
                    atomicAdd(&g_live_hist[0], lh0); atomicAdd(&g_live_hist[1], lh1); atomicAdd(&g_live_hist[2], lh2);
                    atomicAdd(&g_live_hist[3], lh3); atomicAdd(&g_live_hist[4], lh4); atomicAdd(&g_live_hist[5], lh5);
                    atomicAdd(&g_live_hist[6], lh6); atomicAdd(&g_live_hist[7], lh7); atomicAdd(&g_live_hist[8], lh8);
                }
            }
#endif
#ifdef CRT_PROFILE_CRIT_TRACE
            if (TILED && blockIdx.x == 0) {
                if ((crit_iter & 15u) == 0 && (crit_iter >> 4) < 16384u && lane == 0) {
                    g_crit_trace[2 * (crit_iter >> 4)] = __builtin_amdgcn_s_memrealtime();
                    g_crit_trace[2 * (crit_iter >> 4) + 1] = (unsigned long long)n_live | ((unsigned long long)n_parked << 8) |
                                                             ((unsigned long long)crit_iter << 16);
                }
                ++crit_iter;
            }
#endif
            if (n_live == 0) break;
            const uint64_t c0 = TIME ? shader_clock() : 0;
            if (kProfilePass) cnt.cyc_head += c0 - h0;
            // once fewer than regen_t lanes still have samples, waiting for every live lane to park before a pass makes
            // each of them wait for the slowest path of the others at every bounce; a pass at wave_drain/64 of them
            // (crt_renderer_set_wave_drain; 64 = all) shortens the wave's own drain (profiles/r04n)
            const bool drain_pass = n_live < regen_t && n_parked * 64 >= n_live * P.wave_drain;
            if (n_parked >= regen_t || n_parked == n_live || drain_pass) {
                if (COUNT || kProfilePass) cnt.passes++;
#ifdef CRT_PROFILE_LOOPS
                uint32_t pk1 = 0, pk2 = 0, pkr = 0;
#endif
                if (__builtin_amdgcn_inverse_ballot_w64(parked_mask)) {
                    const uint64_t s0 = TIME ? shader_clock() : 0;
                    // (loading the shading record before this sphere test, to overlap its latency, measured +0.7 %:
                    // profiles/r01ar)
                    // after the first pass every parked lane holds a result (parked_mask is within live_mask, which is
                    // the lanes with a ray): a uniform test instead of a divergent branch on has_result (-0.38 %,
                    // profiles/r02av)
                    if (!first_pass) {
                        finish_ray<COUNT>(S, P, inv, closest, hit, sph_lds, shd_lds, cnt, s0);
                    }
                    const uint64_t s1 = TIME ? shader_clock() : 0;
                    const bool live = next_ray(S, C, x, y, P.max_bounces);
                    if (TIME) {
                        const uint64_t s2 = shader_clock();
                        cnt.cyc_shade += s1 - s0;
                        cnt.cyc_next += s2 - s1;
                    }
#ifdef CRT_PROFILE_LOOPS
                    pk1 = S.k1; pk2 = S.k2; pkr = S.kr;
                    S.k1 = S.k2 = S.kr = 0;
#endif
                    has_result = false;
                    if (live) {
                        if (!TILED) ++S.rays;
                        has_result = true;
                        node = 0;
                        sp = 0;
                        closest = INF;
                        hit = -1;
                        // exact 1/d: the per-ray spheres' reference box tests need it (the padded traversal
                        // would do with rcp)
                        inv = recip3_exact(S.d);
                        inv = box_inv(inv);   // the traversal's 1/d (wide_boxes)
                        rows = ray_rows(inv);
                        if (COUNT) cnt.spheres += P.n_ray_spheres;
                        L.ray0[lane] = make_float4(S.o.x, S.o.y, S.o.z, S.d.x);
                        if (COUNT) cnt.trace_calls++;
                        const uint64_t s3 = kProfilePass ? shader_clock() : 0;
                        if (TOPN > 0) top_steps<COUNT, TOPN>(P, top_lds, S.o, inv, rows, node, sp, cnt, stk, (size_t)pix, n_pix);
                        if (kProfilePass) {
                            const uint64_t s4 = shader_clock();
                            cnt.cyc_top += s4 - s3;
                            cnt.cyc_setup += s3 - s1;   // next_ray and the set-up; next_ray's share is subtracted below
                        }
                    }
                }
#ifdef CRT_PROFILE_LOOPS
                {
                    uint32_t m1 = pk1, m2 = pk2, m12 = pk1 + pk2, m1r2 = pk1 + pkr + pk2, s1 = pk1, s2 = pk2;
                    for (int off = 32; off > 0; off >>= 1) {
                        m1 = max(m1, (uint32_t)__shfl_xor((int)m1, off));
                        m2 = max(m2, (uint32_t)__shfl_xor((int)m2, off));
                        m12 = max(m12, (uint32_t)__shfl_xor((int)m12, off));
                        m1r2 = max(m1r2, (uint32_t)__shfl_xor((int)m1r2, off));
                        s1 += (uint32_t)__shfl_xor((int)s1, off);
                        s2 += (uint32_t)__shfl_xor((int)s2, off);
                    }
                    lp[0] += 1; lp[1] += m1; lp[2] += m2; lp[3] += m12; lp[4] += m1r2; lp[5] += s1; lp[6] += s2;
                    lp[7] += (unsigned long long)n_parked;
                }
#endif
                live_mask = wave_ballot(has_result);
                if constexpr (kProfilePass) {
                    // the pass's section timers ran in divergent code, so each lane's accumulators hold only the passes
                    // it took part in (lane 0 alone was reported before): every lane adopts the accumulators of a lane
                    // that ran this pass's innermost timed section, which keeps them wave-uniform
                    const uint64_t ran = parked_mask & live_mask;
                    const int src = __builtin_ctzll(ran ? ran : parked_mask);
                    cnt.cyc_shade = bcast64(cnt.cyc_shade, src);
                    cnt.cyc_sph = bcast64(cnt.cyc_sph, src);
                    cnt.cyc_next = bcast64(cnt.cyc_next, src);
                    cnt.cyc_setup = bcast64(cnt.cyc_setup, src);
                    cnt.cyc_top = bcast64(cnt.cyc_top, src);
                }
                first_pass = false;
                // variant 8 counts the wave's rays in LDS (one VGPR less in the hot loop); (an LDS add without return
                // instead of the read-modify-write measured +0.4 % on config C, profiles/r05e)
                if (TILED && lane == 0) L.rays += (uint32_t)__popcll(parked_mask & live_mask);
            }
            if (TIME) cnt.cyc_regen += shader_clock() - c0;
            if constexpr (PFV) {
                traverse_step4<COUNT, true>(P, S.o, S.d, inv, rows, node, sp, closest, hit, cnt, L, stk, lane, (size_t)pix,
                                            n_pix, pf, &pf_node);
            } else
            traverse_step4<COUNT>(P, S.o, S.d, inv, rows, node, sp, closest, hit, cnt, L, stk, lane, (size_t)pix, n_pix);
        }
    } else if constexpr (VARIANT == 2 || VARIANT == 3 || VARIANT == 10) {
        constexpr bool PF = VARIANT == 3 || VARIANT == 10;
        float4 pA = make_float4(0.f, 0.f, 0.f, 0.f), pB = pA;
        // One wave iteration = one traversal step.  A lane whose trace ends parks until at least
        // `regen_threshold` lanes (or every live lane) are parked; the parked lanes then shade, start
        // their next ray and rejoin traversal while the others keep stepping.
        auto& L = lds[wave];
        const float INF = __builtin_inff();
        bool live = true, has_result = false;
        int node = P.n_nodes, hit = -1, nbase = 0;
        float closest = INF;
        V3 inv = v3(0.f, 0.f, 0.f);
        L.owner_at[lane] = 0;      // owner + 1, 0 = none
        for (;;) {
            const bool parked = live && node >= P.n_nodes;
            const int n_parked = __popcll(wave_ballot(parked));
            const int n_live = __popcll(wave_ballot(live));
            if (n_live == 0) break;
            if (n_parked >= P.regen_threshold || n_parked == n_live) {
                if (parked) {
                    if (has_result) shade(S, P, hit, closest);
                    live = next_ray(S, C, x, y, P.max_bounces);
                    has_result = false;
                    if (live) {
                        ++S.rays;
                        has_result = true;
                        node = 0;
                        closest = INF;
                        hit = -1;
                        inv = v3(1.0f / S.d.x, 1.0f / S.d.y, 1.0f / S.d.z);
                        nbase = layout_base(S.d, P.n_layouts, P.n_nodes);
                        L.ray0[lane] = make_float4(S.o.x, S.o.y, S.o.z, S.d.x);
                        if (PF) {
                            pA = P.nodes[nbase];
                            pB = P.nodes[nbase + 1];
                        }
                        if (COUNT) cnt.trace_calls++;
                    }
                }
            }
            traverse_step<COUNT, PF>(P.nodes, P.prims, P.n_nodes, nbase, P.n_prims, P.err, S.o, S.d, inv, node,
                                     closest, hit, cnt, L, lane, pA, pB);
        }
    } else {
        bool live = true;
        for (;;) {
            if (live) live = next_ray(S, C, x, y, P.max_bounces);
            if (!wave_ballot(live)) break;
            float t;
            const int hit = trace_coop<COUNT>(P.nodes, P.prims, P.n_nodes, layout_base(S.d, P.n_layouts, P.n_nodes),
                                              P.n_prims, P.err, S.o, S.d, live, t, cnt, lds[wave], lane);
            if (live) {
                ++S.rays;
                shade(S, P, hit, t);
            }
        }
    }

    if (((WIDE && !PERSIST) || VARIANT == 3) && P.probe_cost) {   // probe launch: work of this pixel; no state is written
        // counting probe: a ray's shading + generation costs about as much as 16 child-box tests, a triangle
        // test about 4 (section profile, profiles/r01h); plain probe: rays
        if (valid) P.probe_cost[pix] = COUNT ? (16u * S.rays + cnt.boxes + 4u * cnt.tris) >> 3 : S.rays;
        return;
    }
    if (valid && !PERSIST) {
        uint32_t* r = P.rng + 6 * (size_t)pix;
        r[0] = S.s.v0; r[1] = S.s.v1; r[2] = S.s.v2; r[3] = S.s.v3; r[4] = S.s.v4; r[5] = S.s.d;
        P.sum[3 * (size_t)pix] = S.pixel.x;
        P.sum[3 * (size_t)pix + 1] = S.pixel.y;
        P.sum[3 * (size_t)pix + 2] = S.pixel.z;
    }
    if constexpr (TILED) wave_rays = lds[0].rays;
    const uint64_t wr = TILED ? (uint64_t)wave_rays : wave_sum_u64(S.rays);
    if (COUNT) {
        const uint64_t wb = wave_sum_u64(cnt.boxes), wt = wave_sum_u64(cnt.tris);
        const uint64_t ws = wave_sum_u64(cnt.spheres), wp = wave_sum_u64(S.paths);
        if (lane == 0) {
            atomicAdd(&P.counters[1], (unsigned long long)wb);
            atomicAdd(&P.counters[2], (unsigned long long)wt);
            atomicAdd(&P.counters[3], (unsigned long long)ws);
            atomicAdd(&P.counters[4], (unsigned long long)wp);
            // scheduling diagnostics (variant 1): lane-slots offered by traversal steps / leaf rounds,
            // and wave-level trace calls (all uniform per wave)
            atomicAdd(&P.counters[5], 64ull * cnt.step_slots);
            atomicAdd(&P.counters[6], 64ull * cnt.round_slots + ((unsigned long long)cnt.trace_calls << 40));
            atomicAdd(&P.counters[8], (unsigned long long)cnt.cyc_regen);
            atomicAdd(&P.counters[9], (unsigned long long)cnt.cyc_step);
            atomicAdd(&P.counters[10], (unsigned long long)cnt.cyc_round);
            atomicAdd(&P.counters[11], (unsigned long long)cnt.passes);
            atomicAdd(&P.counters[12], 1ull);
            atomicAdd(&P.counters[13], (unsigned long long)cnt.cyc_shade);
            atomicAdd(&P.counters[14], (unsigned long long)cnt.cyc_next);
            atomicAdd(&P.counters[7], (unsigned long long)cnt.cyc_sph);
        }
    }
    if (lane == 0) atomicAdd(&P.counters[0], (unsigned long long)wr);
#ifdef CRT_PROFILE_PASS
    if (!COUNT && TILED && lane == 0 && (int)blockIdx.x < CRT_PROFILE_PASS_FIRST) {
        const unsigned long long v[17] = {cnt.cyc_step, cnt.cyc_round, cnt.cyc_regen, cnt.cyc_shade, cnt.cyc_sph,
                                          cnt.cyc_next, cnt.cyc_setup, cnt.cyc_top, cnt.cyc_head, cnt.passes, 1ull,
                                          shader_clock() - prof_life0, cnt.step_slots, cnt.round_slots, wave_rays,
#ifdef CRT_PROFILE_ROWS
                                          cnt.cyc_rows, cnt.cyc_prims
#else
                                          0ull, 0ull
#endif
        };
        for (int k = 0; k < 17; ++k) atomicAdd(&g_pass_prof[k], v[k]);
    }
#endif
#ifdef CRT_PROFILE_LOOPS
    if (lane == 0 && !P.probe_cost)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_loop_prof[k], lp[k]);
#endif
#ifdef CRT_PROFILE_WAVE_TIMES
    {
        const unsigned wid = (blockIdx.y * gridDim.x + blockIdx.x) * (unsigned)WGW + (threadIdx.x >> 6);
        if (lane == 0 && wid < 4u * 65536u) {
            g_wave_prof[2 * wid] = prof_t0;
            g_wave_prof[2 * wid + 1] = __builtin_amdgcn_s_memrealtime();
#ifdef CRT_PROFILE_CRIT_TRACE
            g_wave_hw[2 * wid] = __builtin_amdgcn_s_getreg(4 | (31 << 11));        // HW_REG_HW_ID
            g_wave_hw[2 * wid + 1] = __builtin_amdgcn_s_getreg(20 | (3 << 11));    // HW_REG_XCC_ID [3:0]
#endif
        }
    }
#endif
}

struct CompareParams {
    RenderParams A;
    const float4* __restrict__ nodes_b;
    const float4* __restrict__ prims_b;
    int n_nodes_b, n_layouts_b;
    int width_a, width_b;
    int sphere_first_b, n_spheres_b;
    const float4* chain_b;
    int n_chain_b;
    float* dump;          // optional: up to max_dump differing rays, 10 floats each
    int max_dump;
};

__global__ __launch_bounds__(256) void crt_compare_kernel(CompareParams Q) {
    const RenderParams& P = Q.A;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int y = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (x >= P.width || y >= P.height) return;
    const int pix = y * P.width + x;
    PathState S;
    const uint32_t* r = P.rng + 6 * (size_t)pix;
    S.s = Rng{r[0], r[1], r[2], r[3], r[4], r[5]};
    S.pixel = v3(0.f, 0.f, 0.f);
    S.o = v3(0, 0, 0); S.d = v3(0, 0, 1); S.thr = v3(1, 1, 1);
    S.remaining = P.spp; S.bounce = 0; S.need_new = true; S.rays = 0; S.paths = 0;
    const crt_camera_desc& Cd = P.cam;
    CamRegs C;
    C.pos = v3(Cd.origin[0], Cd.origin[1], Cd.origin[2]);
    C.llc = v3(Cd.lower_left[0], Cd.lower_left[1], Cd.lower_left[2]);
    C.hor = v3(Cd.horizontal[0], Cd.horizontal[1], Cd.horizontal[2]);
    C.ver = v3(Cd.vertical[0], Cd.vertical[1], Cd.vertical[2]);
    C.right = v3(Cd.right[0], Cd.right[1], Cd.right[2]);
    C.up = v3(Cd.up[0], Cd.up[1], Cd.up[2]);
    C.lens = Cd.lens_radius;
    C.fw = (float)P.width;
    C.fh = (float)P.height;
    C.rfw = P.rcp_w;
    C.rfh = P.rcp_h;
    C.fast_uv = P.fast_uv;
    TraceCounts cnt{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long n_rank = 0, n_t = 0, n_bmiss = 0, n_amiss = 0;
    while (next_ray(S, C, x, y, P.max_bounces)) {
        ++S.rays;
        float ta, tb;
        const int ha = Q.width_a == 4 ? trace4(P.nodes, P.prims, P.sphere_chain, P.n_chain, P.sphere_first, P.n_ray_spheres,
                                               S.o, S.d, ta)
                                      : trace<false>(P.nodes, P.prims, P.n_nodes, layout_base(S.d, P.n_layouts, P.n_nodes),
                                                     S.o, S.d, ta, cnt);
        const int hb = Q.width_b == 4 ? trace4(Q.nodes_b, Q.prims_b, Q.chain_b, Q.n_chain_b, Q.sphere_first_b, Q.n_spheres_b,
                                               S.o, S.d, tb)
                                      : trace<false>(Q.nodes_b, Q.prims_b, Q.n_nodes_b,
                                                     layout_base(S.d, Q.n_layouts_b, Q.n_nodes_b), S.o, S.d, tb, cnt);
        if (ha != hb) {
            ++n_rank;
            n_bmiss += (hb < 0);
            n_amiss += (ha < 0);
            if (Q.dump) {
                const unsigned slot = atomicAdd(reinterpret_cast<unsigned*>(P.counters + 6), 1u);
                if ((int)slot < Q.max_dump) {
                    float* q = Q.dump + 10 * (size_t)slot;
                    q[0] = S.o.x; q[1] = S.o.y; q[2] = S.o.z; q[3] = S.d.x; q[4] = S.d.y; q[5] = S.d.z;
                    q[6] = __int_as_float(ha); q[7] = __int_as_float(hb); q[8] = ta; q[9] = tb;
                }
            }
        } else if (ha >= 0 && __float_as_uint(ta) != __float_as_uint(tb)) {
            ++n_t;
        }
        shade(S, P, ha, ta);
    }
    atomicAdd(&P.counters[0], (unsigned long long)S.rays);
    if (n_rank) atomicAdd(&P.counters[1], n_rank);
    if (n_t) atomicAdd(&P.counters[2], n_t);
    if (n_bmiss) atomicAdd(&P.counters[3], n_bmiss);
    if (n_amiss) atomicAdd(&P.counters[4], n_amiss);
}

// curand_init(seed, subsequence_base + pixel, 0) (CUDAKernels.h:18-26): scrambled seed, then
// v <- A^(2^67 * subsequence) v with seq[k] = A^(2^67 * 4^k) (one base-4 digit per matrix).
__global__ __launch_bounds__(256) void crt_init_rand_kernel(uint32_t* __restrict__ rng, const uint32_t* __restrict__ seq,
                                                            int n_pix, unsigned long long seed,
                                                            unsigned long long subseq_base) {
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= n_pix) return;
    const uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    uint32_t v[5] = {123456789u + t0, 362436069u ^ t0, 521288629u + t1, 88675123u ^ t1, 5783321u + t0};
    const uint32_t dd = 6615241u + t1 + t0;
    unsigned long long n = subseq_base + (unsigned long long)pix;
    for (int k = 0; n; ++k, n >>= 2) {
        const uint32_t reps = (uint32_t)(n & 3u);
        const uint32_t* m = seq + 800 * k;
        for (uint32_t q = 0; q < reps; ++q) {
            uint32_t r[5] = {0, 0, 0, 0, 0};
            for (int i = 0; i < 5; ++i) {
                const uint32_t w = v[i];
#pragma unroll 4
                for (int j = 0; j < 32; ++j) {
                    const uint32_t msk = 0u - ((w >> j) & 1u);
                    const uint32_t* col = m + (i * 32 + j) * 5;
#pragma unroll
                    for (int c = 0; c < 5; ++c) r[c] ^= msk & col[c];
                }
            }
#pragma unroll
            for (int c = 0; c < 5; ++c) v[c] = r[c];
        }
    }
    uint32_t* o = rng + 6 * (size_t)pix;
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3]; o[4] = v[4]; o[5] = dd;
}

// writeColor(data, idx, m_PixelSampleScale * pixel_color) (CUDAKernels.h:164, CRTUtility.cuh:21-32)
__global__ __launch_bounds__(256) void crt_resolve_kernel(const float* __restrict__ sum, uint8_t* __restrict__ rgba,
                                                          int n_pix, float scale) {
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= n_pix) return;
    const float r = scale * sum[3 * (size_t)pix];
    const float g = scale * sum[3 * (size_t)pix + 1];
    const float b = scale * sum[3 * (size_t)pix + 2];
    uchar4 o;
    o.x = to_u8(r); o.y = to_u8(g); o.z = to_u8(b); o.w = 255;
    reinterpret_cast<uchar4*>(rgba)[pix] = o;
}

__global__ void crt_selftest_math_kernel(const float* a, const float* b, int n, float* out, double* out64) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i], y = b[i];
    out[4 * i] = x / y;
    out[4 * i + 1] = sqrtf(fabsf(x));
    out[4 * i + 2] = 1.0f / x;
    const double dx = fabs((double)x * (double)y);
    out[4 * i + 3] = (float)sqrt((double)fabsf(x));
    out64[2 * i] = sqrt(dx);
    out64[2 * i + 1] = 1.0 - dx * dx;
}

// Exhaustive check of rcp_newton against IEEE 1.f/x over bit patterns [lo, hi) of positive floats
// (the negative half is the mirror image: both rcp and the FMAs are sign-symmetric, still checked).
__global__ __launch_bounds__(256) void crt_selftest_rcp_kernel(uint32_t lo, uint32_t hi, unsigned long long* bad,
                                                               uint32_t* first_bad) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi && b >= lo; b += stride) {
        const float x = __uint_as_float(b);
        const float a = rcp_newton(x), c = 1.0f / x;
        const float an = rcp_newton(-x), cn = 1.0f / -x;
        if (__float_as_uint(a) != __float_as_uint(c) || __float_as_uint(an) != __float_as_uint(cn)) {
            ++nbad;
            atomicMin(first_bad, b);
        }
        if (b > 0xffffffffu - stride) break;
    }
    if (nbad) atomicAdd(bad, nbad);
}

__global__ __launch_bounds__(256) void crt_selftest_sqrt_kernel(uint32_t lo, uint32_t hi, unsigned long long* bad,
                                                                uint32_t* first_bad) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi && b >= lo; b += stride) {
        const float x = __uint_as_float(b);
        if (__float_as_uint(sqrt_rsq(x)) != __float_as_uint(sqrtf(x))) {
            ++nbad;
            atomicMin(first_bad, b);
        }
        if (b > 0xffffffffu - stride) break;
    }
    if (nbad) atomicAdd(bad, nbad);
}

// Exhaustive check of next_ray's division for one frame dimension b: every float a in [lo, hi] (all values (x + U) can
// take) through uv_div against IEEE a / b.
__global__ __launch_bounds__(256) void crt_uv_div_check_kernel(float b, float r, uint32_t lo, uint32_t hi,
                                                               unsigned long long* bad) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x; i <= hi && i >= lo; i += stride) {
        const float a = __uint_as_float(i);
        if (__float_as_uint(uv_div(a, b, r)) != __float_as_uint(a / b)) ++nbad;
        if (i > 0xffffffffu - stride) break;
    }
    if (nbad) atomicAdd(bad, nbad);
}

__global__ __launch_bounds__(64) void crt_selftest_scan_kernel(const int* in, int* out, int n_waves) {
    const int w = blockIdx.x;
    if (w >= n_waves) return;
    const int lane = threadIdx.x;
    const int x = in[64 * w + lane];
    out[3 * (64 * w + lane)] = wave_inclusive_scan(x, lane);
    out[3 * (64 * w + lane) + 1] = wave_inclusive_scan_shfl(x, lane);
    // the kernels' max-scan runs on owner + 1 (0 = none); inputs here are >= -1
    out[3 * (64 * w + lane) + 2] = (int)wave_inclusive_max_scan_u((uint32_t)(x + 1)) - 1;
}

// Known-answer self-test of the render path's own primitive functions (tests/golden/primitives.json):
// kind 0 = tri_test_rec (Möller–Trumbore, window [0.001, tmax]), 1 = ref_scene_box (AABB::hit against
// [0.001, inf) with the exact 1/d), 2 = sphere_candidate (Sphere::hit, window [0.001, tmax]), 3 = next_ray's
// Camera::getRay for a new sample.
__global__ void crt_selftest_geometry_kernel(int kind, const float* __restrict__ in, int n, float* __restrict__ out,
                                             uint32_t* __restrict__ rng, crt_camera_desc cam, int w, int h, float rcp_w,
                                             float rcp_h, int fast_uv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (kind == 0) {
        const float* q = in + 17 * i;
        const V3 o = v3(q[0], q[1], q[2]), d = v3(q[3], q[4], q[5]);
        const float e1[3] = {q[9] - q[6], q[10] - q[7], q[11] - q[8]}, e2[3] = {q[12] - q[6], q[13] - q[7], q[14] - q[8]};
        const float4 f0 = make_float4(q[6], q[7], q[8], e1[0]), f1 = make_float4(e1[1], e1[2], e2[0], e2[1]);
        const float4 f2 = make_float4(e2[2], 0.f, 0.f, 0.f);
        out[i] = tri_test_rec(f0, f1, f2, o, d, q[16]);
    } else if (kind == 1) {
        const float* q = in + 14 * i;
        const V3 o = v3(q[0], q[1], q[2]), d = v3(q[3], q[4], q[5]);
        const V3 inv = v3(recip_exact_any(d.x), recip_exact_any(d.y), recip_exact_any(d.z));
        out[i] = ref_scene_box(make_float4(q[6], q[7], q[8], q[9]), make_float4(q[10], q[11], 0.f, 0.f), o, inv) ? 1.f : 0.f;
    } else if (kind == 2) {
        const float* q = in + 12 * i;
        const V3 o = v3(q[0], q[1], q[2]), d = v3(q[3], q[4], q[5]);
        out[i] = sphere_candidate(make_float4(q[6], q[7], q[8], q[9]), make_float4(q[9] * q[9], 0.f, 0.f, 0.f), o, d,
                                  q[11]);
    } else if (kind == 4) {   // the per-ray spheres' skip test (sphere_beyond) against closest = q[10]
        const float* q = in + 12 * i;
        const float ocx = q[0] - q[6], ocy = q[1] - q[7], ocz = q[2] - q[8];
        const float qa = dot(v3(q[3], q[4], q[5]), v3(q[3], q[4], q[5]));
        const float hb = (ocx * q[3] + ocy * q[4]) + ocz * q[5];
        const float qc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - q[9] * q[9];
        const float disc = hb * hb - qa * qc;
        out[i] = sphere_beyond(qa, hb, disc, q[10]) ? 1.f : 0.f;
    } else {
        const int* xy = reinterpret_cast<const int*>(in);
        CamRegs C;
        C.pos = v3(cam.origin[0], cam.origin[1], cam.origin[2]);
        C.llc = v3(cam.lower_left[0], cam.lower_left[1], cam.lower_left[2]);
        C.hor = v3(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
        C.ver = v3(cam.vertical[0], cam.vertical[1], cam.vertical[2]);
        C.right = v3(cam.right[0], cam.right[1], cam.right[2]);
        C.up = v3(cam.up[0], cam.up[1], cam.up[2]);
        C.lens = cam.lens_radius;
        C.fw = (float)w;
        C.fh = (float)h;
        C.rfw = rcp_w;
        C.rfh = rcp_h;
        C.fast_uv = fast_uv;
        PathState S;
        uint32_t* r = rng + 6 * (size_t)i;
        S.s = Rng{r[0], r[1], r[2], r[3], r[4], r[5]};
        S.pixel = v3(0.f, 0.f, 0.f);
        S.thr = v3(1.f, 1.f, 1.f);
        S.remaining = 1; S.bounce = 0; S.need_new = true; S.rays = 0; S.paths = 0;
        next_ray(S, C, xy[2 * i], xy[2 * i + 1], 20);
        r[0] = S.s.v0; r[1] = S.s.v1; r[2] = S.s.v2; r[3] = S.s.v3; r[4] = S.s.v4; r[5] = S.s.d;
        float* o6 = out + 6 * (size_t)i;
        o6[0] = S.o.x; o6[1] = S.o.y; o6[2] = S.o.z; o6[3] = S.d.x; o6[4] = S.d.y; o6[5] = S.d.z;
    }
}

__global__ void crt_selftest_rng_kernel(const uint32_t* st_in, int n, int n_draw, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rng s{st_in[6 * i], st_in[6 * i + 1], st_in[6 * i + 2], st_in[6 * i + 3], st_in[6 * i + 4], st_in[6 * i + 5]};
    for (int k = 0; k < n_draw; ++k) out[(size_t)i * n_draw + k] = uniform(s);
}

// ------------------------------------------------------------------ variant 7: pixel order from the probe
// Most expensive pixels first (longest-processing-time order), so the pixels whose sample sequences take
// longest start at once and the launch ends on cheap ones.  Counting sort of the probe's per-pixel ray
// counts (keys clamped to 1023), descending; within a key the order is arbitrary (scheduling only).
constexpr int ORDER_KEYS = 1024;
constexpr int ORDER_ITEMS = 1024;   // pixels per workgroup of the sort passes
__device__ __forceinline__ uint32_t order_bucket(uint32_t cost) { return ORDER_KEYS - 1 - min(cost, (uint32_t)ORDER_KEYS - 1); }
__global__ __launch_bounds__(256) void crt_order_hist_kernel(const uint32_t* __restrict__ cost, int n,
                                                             uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[ORDER_KEYS];
    for (int i = threadIdx.x; i < ORDER_KEYS; i += 256) h[i] = 0;
    __syncthreads();
    const int b0 = blockIdx.x * ORDER_ITEMS;
    for (int i = b0 + threadIdx.x; i < min(n, b0 + ORDER_ITEMS); i += 256) atomicAdd(&h[order_bucket(cost[i])], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < ORDER_KEYS; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}
__global__ __launch_bounds__(ORDER_KEYS) void crt_order_scan_kernel(uint32_t* __restrict__ hist) {
    __shared__ uint32_t part[ORDER_KEYS];
    const int t = threadIdx.x;
    const uint32_t c = hist[t];
    part[t] = c;
    __syncthreads();
    for (int o = 1; o < ORDER_KEYS; o <<= 1) {
        const uint32_t add = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    hist[t] = part[t] - c;   // exclusive offsets
}
__global__ __launch_bounds__(256) void crt_order_scatter_kernel(const uint32_t* __restrict__ cost, int n,
                                                                uint32_t* __restrict__ hist,
                                                                uint32_t* __restrict__ order, uint32_t base) {
    __shared__ uint32_t h[ORDER_KEYS];
    for (int i = threadIdx.x; i < ORDER_KEYS; i += 256) h[i] = 0;
    __syncthreads();
    const int b0 = blockIdx.x * ORDER_ITEMS;
    uint32_t rank[ORDER_ITEMS / 256];
    for (int k = 0; k < ORDER_ITEMS / 256; ++k) {
        const int i = b0 + threadIdx.x + 256 * k;
        rank[k] = i < n ? atomicAdd(&h[order_bucket(cost[i])], 1u) : 0u;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ORDER_KEYS; i += 256)   // reserve this block's run of every key
        if (h[i]) h[i] = atomicAdd(&hist[i], h[i]);
    __syncthreads();
    for (int k = 0; k < ORDER_ITEMS / 256; ++k) {
        const int i = b0 + threadIdx.x + 256 * k;
        if (i < n) order[h[order_bucket(cost[i])] + rank[k]] = base + (uint32_t)i;
    }
}
// XCD regions (crt_renderer_set_xcd_regions): MI355X deals workgroups round-robin over its 8 XCDs, so blocks b and b + 8
// share an XCD and its 4 MiB L2 (MI355X_MICROARCH.md §Workgroup dispatch; which XCD is not fixed, and nothing depends on
// it for correctness).  This reorders the cost-sorted tile list so that the blocks of one XCD group (b % 8 == k) render
// one screen region: 8 vertical strips of equal probe cost (column sums of the tile keys), each in descending cost
// (a stable partition of the sorted list).  Every group gets n/8 blocks (+1 for the first n % 8 groups): a strip with more
// tiles than that hands its cheapest tail to a shared pool, from which the groups with fewer tiles take their last
// blocks.  One workgroup of 1024 threads; `part` and `pool` are scratch of n entries each.  Results never depend on
// the order (each pixel is one lane's sequential chain).
constexpr int XCD_GROUPS = 8;
__global__ __launch_bounds__(1024) void crt_xcd_order_kernel(uint32_t* __restrict__ order, const uint32_t* __restrict__ key,
                                                             int n, int tiles_x, uint32_t* __restrict__ part,
                                                             uint32_t* __restrict__ pool) {
    __shared__ uint32_t col_region[2048];              // tiles_x <= 2048 (checked by the host)
    __shared__ unsigned long long col_cost[2048];
    __shared__ uint32_t wave_cnt[16][XCD_GROUPS];
    __shared__ uint32_t reg_n[XCD_GROUPS], reg_off[XCD_GROUPS], run[XCD_GROUPS];
    __shared__ uint32_t cap[XCD_GROUPS], exc_off[XCD_GROUPS], def_off[XCD_GROUPS];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int c = t; c < tiles_x; c += 1024) col_cost[c] = 0;
    if (t < XCD_GROUPS) run[t] = 0;
    __syncthreads();
    for (int i = t; i < n; i += 1024)   // a tile weighs its clamped key + 1, as the counting sort sees it
        atomicAdd(&col_cost[i % tiles_x], (unsigned long long)(min(key[i], (uint32_t)ORDER_KEYS - 1) + 1u));
    __syncthreads();
    if (t == 0) {   // strips of equal cost: column c joins the strip its cost midpoint falls in
        unsigned long long tot = 0;
        for (int c = 0; c < tiles_x; ++c) tot += col_cost[c];
        unsigned long long acc = 0;
        for (int c = 0; c < tiles_x; ++c) {
            const unsigned long long mid = acc + col_cost[c] / 2;
            col_region[c] = (uint32_t)min((unsigned long long)XCD_GROUPS - 1, mid * XCD_GROUPS / (tot ? tot : 1));
            acc += col_cost[c];
        }
    }
    __syncthreads();
    // stable partition of the sorted list by strip (ballot ranks inside a wave, wave totals across the workgroup)
    for (int b0 = 0; b0 < n; b0 += 1024) {
        const int i = b0 + t;
        const uint32_t tile = i < n ? order[i] : 0u;
        const uint32_t r = i < n ? col_region[tile % (uint32_t)tiles_x] : 0xffu;
        uint32_t rank = 0;
        for (int g = 0; g < XCD_GROUPS; ++g) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(r == (uint32_t)g);
            if (r == (uint32_t)g) rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (lane == 0) wave_cnt[wv][g] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if (r < (uint32_t)XCD_GROUPS) {
            uint32_t before = run[r];
            for (int w = 0; w < wv; ++w) before += wave_cnt[w][r];
            part[(size_t)r * n + before + rank] = tile;   // strip r's list at part[r * n ...]
        }
        __syncthreads();
        if (t < XCD_GROUPS)
            for (int w = 0; w < 16; ++w) run[t] += wave_cnt[w][t];
        __syncthreads();
    }
    if (t == 0) {
        const uint32_t q = (uint32_t)n / XCD_GROUPS, e = (uint32_t)n % XCD_GROUPS;
        uint32_t eo = 0, dd = 0;
        for (int g = 0; g < XCD_GROUPS; ++g) {
            reg_n[g] = run[g];
            cap[g] = q + ((uint32_t)g < e ? 1u : 0u);
            exc_off[g] = eo;
            def_off[g] = dd;
            if (run[g] > cap[g]) eo += run[g] - cap[g];
            else dd += cap[g] - run[g];
        }
        (void)reg_off;
    }
    __syncthreads();
    for (int g = 0; g < XCD_GROUPS; ++g)   // the strips' tails beyond their group's share, concatenated
        for (uint32_t i = cap[g] + (uint32_t)t; i < reg_n[g]; i += 1024) pool[exc_off[g] + i - cap[g]] = part[(size_t)g * n + i];
    __syncthreads();
    for (int b = t; b < n; b += 1024) {
        const int g = b % XCD_GROUPS;
        const uint32_t i = (uint32_t)(b / XCD_GROUPS);
        order[b] = i < reg_n[g] ? part[(size_t)g * n + i] : pool[def_off[g] + i - reg_n[g]];
    }
}

// Variant 8: the key of an 8x8 tile is its most expensive pixel (the wave ends with its slowest lane);
// key_mode 1 adds the mean pixel (ties between tiles with equal maxima); key_mode 2 raises a tile to 3/4 of
// the largest key among its 8 neighbours (a 4-spp probe underestimates some tiles next to expensive ones, and an
// underestimated tile dispatched late becomes the launch's tail).
// stats (optional, zeroed by the caller): [0] the largest tile work, [1] the sum of the tile works, both in probe cost units
// over the probed pixels (a tile's work = the sum of its probed pixels' costs); the host's occupancy choice (crt_render)
__global__ void crt_tile_cost_kernel(const uint32_t* __restrict__ pix_cost, int width, int height, int tiles_x,
                                     int n_tiles, uint32_t* __restrict__ tile_cost, int key_mode, int stride,
                                     unsigned long long* __restrict__ stats) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const int x0 = (t % tiles_x) * 8, y0 = (t / tiles_x) * 8;
    uint32_t m = 0, sum = 0, k = 0;
    for (int y = y0; y < min(height, y0 + 8); y += stride)   // a subsampled probe wrote pixels with x, y % stride == 0
        for (int x = x0; x < min(width, x0 + 8); x += stride) {
            const uint32_t c = pix_cost[(size_t)y * width + x];
            m = max(m, c);
            sum += c;
            ++k;
        }
    tile_cost[t] = key_mode == 1 ? m + sum / max(1u, k) : m;
    if (stats) {
        atomicMax(&stats[0], (unsigned long long)sum);
        atomicAdd(&stats[1], (unsigned long long)sum);
    }
}
__global__ void crt_tile_neighbour_kernel(const uint32_t* __restrict__ key_in, int tiles_x, int n_tiles,
                                          uint32_t* __restrict__ key_out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const int tx = t % tiles_x, ty = t / tiles_x, tiles_y = (n_tiles + tiles_x - 1) / tiles_x;
    uint32_t nb = 0;
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
            const int x = tx + dx, y = ty + dy;
            if ((dx || dy) && x >= 0 && x < tiles_x && y >= 0 && y < tiles_y && y * tiles_x + x < n_tiles)
                nb = max(nb, key_in[y * tiles_x + x]);
        }
    key_out[t] = max(key_in[t], (nb * 3u) / 4u);
}

// No probe: 8x8 tiles in row order, pixels row-major inside a tile (a wave's first 64 slots are one tile, so
// its primary rays are coherent); slots of partial edge tiles hold ~0.
// Pixel sharding (crt_renderer_set_pixel_shard): the tiles of other shards get key 0 and this shard's keys + 1, so
// the descending cost order puts exactly this shard's tiles first, whatever order the counting sort gives equal keys.
__global__ void crt_tile_shard_mask_kernel(uint32_t* __restrict__ key, int n_tiles, int shard, int shards) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const uint32_t k = key[t];
    key[t] = t % shards == shard ? (k < 0xffffffffu ? k + 1u : k) : 0u;
}

// Pixel sharding without the probe: slot k holds tile k * shards + shard.
__global__ void crt_shard_tiles_kernel(uint32_t* __restrict__ order, int n_tiles, int shard, int shards) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k * shards + shard < n_tiles) order[k] = (uint32_t)(k * shards + shard);
}

// Variant 7 with the temporal order (crt_renderer_set_temporal_order): slots of 8x8 tiles in the order tile_order
// holds (the tiles most expensive first by the previous frame's rays per pixel), pixels row-major inside a tile.
__global__ void crt_expand_tile_order_kernel(const uint32_t* __restrict__ tile_order, uint32_t* __restrict__ order,
                                             int width, int height, int n_slots) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int tiles_x = (width + 7) / 8, tile = (int)tile_order[s >> 6], q = s & 63;
    const int x = (tile % tiles_x) * 8 + (q & 7), y = (tile / tiles_x) * 8 + (q >> 3);
    order[s] = (x < width && y < height) ? (uint32_t)(y * width + x) : 0xffffffffu;
}
__global__ void crt_order_tiles_kernel(uint32_t* __restrict__ order, int width, int height, int n_slots) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int tiles_x = (width + 7) / 8, tile = s >> 6, q = s & 63;
    const int x = (tile % tiles_x) * 8 + (q & 7), y = (tile / tiles_x) * 8 + (q >> 3);
    order[s] = (x < width && y < height) ? (uint32_t)(y * width + x) : 0xffffffffu;
}

// ------------------------------------------------------------------ host side
namespace {

// XORWOW single-step linear map and its 2^67*4^k powers (160 columns x 5 words).
void xw_step(uint32_t v[5]) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}
void mv(const uint32_t* m, uint32_t v[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 160; ++i)
        if (v[i / 32] & (1u << (i % 32)))
            for (int k = 0; k < 5; ++k) r[k] ^= m[i * 5 + k];
    std::memcpy(v, r, sizeof r);
}
void mm(const uint32_t* b, const uint32_t* a, uint32_t* c) {   // c = b o a
    for (int col = 0; col < 160; ++col) {
        uint32_t v[5];
        std::memcpy(v, a + 5 * col, sizeof v);
        mv(b, v);
        std::memcpy(c + 5 * col, v, sizeof v);
    }
}
const std::vector<uint32_t>& seq_tables() {
    static std::vector<uint32_t> tab;
    static std::once_flag once;
    std::call_once(once, [] {
        tab.assign(32 * 800, 0);
        std::vector<uint32_t> m(800), t(800);
        for (int col = 0; col < 160; ++col) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[col / 32] = 1u << (col % 32);
            xw_step(v);
            std::memcpy(&m[5 * col], v, sizeof v);
        }
        for (int s = 0; s < 67; ++s) { mm(m.data(), m.data(), t.data()); m.swap(t); }
        std::memcpy(&tab[0], m.data(), 800 * 4);
        for (int k = 1; k < 32; ++k) {
            mm(&tab[800 * (k - 1)], &tab[800 * (k - 1)], t.data());
            mm(t.data(), t.data(), &tab[800 * k]);
        }
    });
    return tab;
}

inline float i2f(int v) { float f; std::memcpy(&f, &v, 4); return f; }
inline int i2i_host(float f) { int v; std::memcpy(&v, &f, 4); return v; }

inline bool zero_thickness(const float bmin[3], const float bmax[3]) {
    // AABB::hit can never report such a box (the slab of that axis is empty: tmax <= tmin)
    return bmin[0] == bmax[0] || bmin[1] == bmax[1] || bmin[2] == bmax[2];
}

// CRT_SETUP_TRACE=1: the host stages of scene creation timed on stderr (tools/setup_breakdown.py).
struct SetupTrace {
    bool on = std::getenv("CRT_SETUP_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* stage) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[crt setup] %-28s %8.2f ms\n", stage, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// The host loops of scene creation that gather or fill one record per primitive run on up to 16 threads
// (CRT::parallel_ranges; on config E's million triangles they took ~120 ms of its 0.34-s scene creation on one,
// profiles/r05k).
using CRT::parallel_ranges;

// Flattens the reference's scene + mesh BVHs into the threaded layout and records, per primitive,
// its reference DFS rank (the order BVHNode::hit / Mesh::hit visit primitives) and whether any box
// on its path is zero-thickness (then the reference never reports it).
struct Flattener {
    const crt_scene_desc* D;
    std::vector<float4> nodes, prims;
    std::vector<int> mesh_prim_base;
    std::vector<int> rank_of;        // per prim
    std::vector<char> reachable;     // per prim
    std::vector<int> rank_code;      // per rank: prim code
    int max_depth = 0;
    std::string err;

    void visit_prim(int p, int code, bool thin) {
        if (rank_of[p] >= 0) return;
        rank_of[p] = (int)rank_code.size();
        rank_code.push_back(code);
        reachable[p] = !thin;
    }
    // Primitives no leaf references get the remaining ranks (never hit); ranks go into the records.
    void finalize_ranks() {
        const int n = (int)(prims.size() / 3);
        for (int p = 0; p < n; ++p) {
            if (rank_of[p] < 0) {
                rank_of[p] = (int)rank_code.size();
                rank_code.push_back(p);
                reachable[p] = 0;
            }
            const bool sphere = (rank_code[rank_of[p]] & SPHERE_BIT) != 0;
            if (sphere) prims[3 * p + 1].z = i2f(rank_of[p]);
            prims[3 * p + 2].z = i2f(rank_of[p]);
        }
    }

    int push_node(const float bmin[3], const float bmax[3], int a, int b) {
        nodes.push_back(make_float4(bmin[0], bmin[1], bmin[2], bmax[0]));
        nodes.push_back(make_float4(bmax[1], bmax[2], i2f(a), i2f(b)));
        return (int)(nodes.size() / 2) - 1;
    }
    void set_a(int idx, int a) { nodes[2 * idx + 1].z = i2f(a); }
    int count() const { return (int)(nodes.size() / 2); }

    bool emit_mesh(int m, int ni, int depth, bool thin) {
        const crt_mesh_desc& M = D->meshes[m];
        if (ni < 0 || ni >= M.node_count) { err = "mesh node index out of range"; return false; }
        if (depth > 4096) { err = "mesh BVH too deep"; return false; }
        max_depth = std::max(max_depth, depth);
        const crt_bvh_node_desc& N = M.nodes[ni];
        thin = thin || zero_thickness(N.bmin, N.bmax);
        if (!N.is_leaf) {
            int idx = push_node(N.bmin, N.bmax, 0, NODE_MESH_INNER);
            if (!emit_mesh(m, N.left, depth + 1, thin) || !emit_mesh(m, N.right, depth + 1, thin)) return false;
            set_a(idx, count());
        } else {
            if (N.obj_index < 0 || N.obj_count < 0 || N.obj_index % 3 || N.obj_count % 3 ||
                (uint64_t)N.obj_index + N.obj_count > M.index_count) { err = "bad mesh leaf range"; return false; }
            long first = mesh_prim_base[m] + N.obj_index / 3;
            if (first >= SPHERE_BIT) { err = "too many primitives"; return false; }
            push_node(N.bmin, N.bmax, N.obj_count / 3, (int)first);
            for (int k = 0; k < (int)N.obj_count / 3; ++k) visit_prim((int)first + k, (int)first + k, thin);
        }
        return true;
    }
    bool emit_scene(int ni, int depth, bool thin) {
        if (ni < 0 || ni >= D->n_scene_nodes) { err = "scene node index out of range"; return false; }
        if (depth > 4096) { err = "scene BVH too deep"; return false; }
        max_depth = std::max(max_depth, depth);
        const crt_bvh_node_desc& N = D->scene_nodes[ni];
        thin = thin || zero_thickness(N.bmin, N.bmax);
        if (!N.is_leaf) {
            int idx = push_node(N.bmin, N.bmax, 0, NODE_SCENE_INNER);
            if (!emit_scene(N.left, depth + 1, thin) || !emit_scene(N.right, depth + 1, thin)) return false;
            set_a(idx, count());
            return true;
        }
        if (N.obj_index < 0 || N.obj_index >= D->n_objects) { err = "scene leaf object out of range"; return false; }
        const crt_object_desc& O = D->objects[N.obj_index];
        if (O.kind == CRT_OBJECT_MESH) {
            if (O.index < 0 || O.index >= D->n_meshes) { err = "mesh object index out of range"; return false; }
            int idx = push_node(N.bmin, N.bmax, 0, NODE_SCENE_INNER);
            if (D->meshes[O.index].node_count > 0 && !emit_mesh(O.index, 0, depth + 1, thin)) return false;
            set_a(idx, count());
        } else if (O.kind == CRT_OBJECT_SPHERE) {
            if (O.index < 0 || O.index >= D->n_spheres) { err = "sphere object index out of range"; return false; }
            const crt_sphere_desc& S = D->spheres[O.index];
            int p = (int)(prims.size() / 3);
            if (p >= SPHERE_BIT) { err = "too many primitives"; return false; }
            prims.push_back(make_float4(S.center[0], S.center[1], S.center[2], S.radius));
            prims.push_back(make_float4(S.radius * S.radius, i2f(S.material), 0.f, 0.f));   // Sphere.cuh:21
            prims.push_back(make_float4(0.f, i2f(S.material), 0.f, i2f(1)));                  // word 11 = 1: sphere
            rank_of.push_back(-1);
            reachable.push_back(0);
            visit_prim(p, SPHERE_BIT | p, thin);
            push_node(N.bmin, N.bmax, 0, SPHERE_BIT | p);
        } else {
            err = "unknown object kind";
            return false;
        }
        return true;
    }
    bool build_triangles() {
        mesh_prim_base.assign(D->n_meshes, 0);
        size_t total = 0;
        for (int m = 0; m < D->n_meshes; ++m) {
            const crt_mesh_desc& M = D->meshes[m];
            if ((uint64_t)M.index_offset + M.index_count > D->n_indices ||
                (uint64_t)M.vertex_offset + M.vertex_count > D->n_positions ||
                (uint64_t)M.face_offset + M.index_count / 3 > D->n_faces || M.index_count % 3) {
                err = "mesh ranges exceed the scene arrays";
                return false;
            }
            mesh_prim_base[m] = (int)total;
            total += M.index_count / 3;
        }
        prims.reserve(3 * (total + (size_t)std::max(D->n_spheres, 0)));   // emit_scene appends the spheres
        prims.assign(3 * total, make_float4(0.f, 0.f, 0.f, 0.f));
        bool bad_index = false;
        for (int m = 0; m < D->n_meshes; ++m) {
            const crt_mesh_desc& M = D->meshes[m];
            float4* out = prims.data() + 3 * (size_t)mesh_prim_base[m];
            std::atomic<bool> bad{false};
            parallel_ranges(M.index_count / 3, [&](size_t b, size_t e) {
                for (size_t t = b; t < e; ++t) {
                    uint32_t iv[3];
                    for (int c = 0; c < 3; ++c) {
                        iv[c] = D->indices[M.index_offset + 3 * t + c];
                        if (iv[c] >= M.vertex_count) { bad.store(true, std::memory_order_relaxed); iv[c] = 0; }   // reported below
                    }
                    const float* p0 = D->positions + 3 * ((size_t)M.vertex_offset + iv[0]);
                    const float* p1 = D->positions + 3 * ((size_t)M.vertex_offset + iv[1]);
                    const float* p2 = D->positions + 3 * ((size_t)M.vertex_offset + iv[2]);
                    const float e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};   // Mesh.cuh:277
                    const float e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};   // Mesh.cuh:278
                    const uint32_t mat = (uint32_t)(D->face_materials[M.face_offset + t] + (int32_t)M.material_id_offset);
                    out[3 * t] = make_float4(p0[0], p0[1], p0[2], e1[0]);
                    out[3 * t + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
                    out[3 * t + 2] = make_float4(e2[2], i2f((int)mat), 0.f, 0.f);
                }
            });
            bad_index = bad_index || bad.load();
        }
        if (bad_index) { err = "vertex index out of range"; return false; }
        rank_of.assign(prims.size() / 3, -1);
        reachable.assign(prims.size() / 3, 0);
        return true;
    }
};

// CRT_BVH_REBUILT: binned-SAH tree over the reachable primitives of a flattened reference scene,
// emitted as `layouts` threaded arrays (crt_sah.h).  Primitive records keep their rank.
struct Rebuilt {
    std::vector<float4> nodes, prims;
    std::vector<int> rank_code;
    int n_nodes = 0, max_depth = 0;
    long excluded = 0;
    std::string err;

    int width = 2;
    int stack_bound = 0;   // width 4: most stack entries any traversal can hold
    int sphere_first = 0, n_ray_spheres = 0;   // width 4: spheres kept out of the tree (tested per ray)
    std::vector<float4> chain;                 // their reference scene-level leaf boxes (2 float4 per box)
    static constexpr int kMaxRaySpheres = 8;

    // gpu_device >= 0: the binned-SAH tree is built on that GPU (crtx_build_sah_gpu, crt_bvh_build.hip)
    long spatial_splits = 0;   // SBVH: nodes cut by a plane, and primitive references in the leaves
    long references = 0;

    // gpu_device >= 0: the binned-SAH tree is built on that GPU (crtx_build_sah_gpu, crt_bvh_build.hip); spatial:
    // SBVH on the host (crt_sah::SpatialBuilder), width 4 only
    bool build(const Flattener& F, int leaf_size, int layouts, float trav_cost, int wide, int gpu_device = -1,
               bool spatial = false, float alpha = 1e-5f, float max_dup = 1.f) {
        SetupTrace tr;
        width = wide;
        const int n = (int)(F.prims.size() / 3);
        std::vector<crt_sah::Item> items;
        items.reserve(n);
        std::vector<int> ray_sph;
        std::vector<crt_sah::TriVerts> verts;
        if (spatial && width != 4) { err = "spatial splits need width 4"; return false; }
        int n_sph = 0;
        for (int p = 0; p < n; ++p) n_sph += (F.rank_code[F.rank_of[p]] & SPHERE_BIT) != 0;
        const bool spheres_per_ray = width == 4 && n_sph <= kMaxRaySpheres;
        for (int p = 0; p < n; ++p) {
            const bool sphere = (F.rank_code[F.rank_of[p]] & SPHERE_BIT) != 0;
            if (!F.reachable[p]) { excluded += !sphere; continue; }
            const float4 f0 = F.prims[3 * p], f1 = F.prims[3 * p + 1], f2 = F.prims[3 * p + 2];
            if (sphere && spheres_per_ray) {
                // a per-ray sphere's hit point becomes a ray origin too: the same 2^60 bound as the tree's boxes
                // (wide_boxes: |o| * 2^64 must stay finite)
                const float c[3] = {f0.x, f0.y, f0.z}, r = std::fabs(f0.w);
                for (int a = 0; a < 3; ++a)
                    if (!(std::fabs(c[a] - r) < 0x1p60f && std::fabs(c[a] + r) < 0x1p60f)) {
                        err = "sphere bounds non-finite or beyond 2^60";
                        return false;
                    }
                ray_sph.push_back(p);
                continue;
            }
            crt_sah::Item it;
            it.src = p;
            it.sphere = sphere;
            if (sphere) {
                const float c[3] = {f0.x, f0.y, f0.z}, r = std::fabs(f0.w);
                for (int a = 0; a < 3; ++a) { it.lo[a] = c[a] - r; it.hi[a] = c[a] + r; }
            } else {
                const float v0[3] = {f0.x, f0.y, f0.z};
                const float e1[3] = {f0.w, f1.x, f1.y}, e2[3] = {f1.z, f1.w, f2.x};
                for (int a = 0; a < 3; ++a) {
                    const float v1 = v0[a] + e1[a], v2 = v0[a] + e2[a];
                    it.lo[a] = std::min(v0[a], std::min(v1, v2));
                    it.hi[a] = std::max(v0[a], std::max(v1, v2));
                }
            }
            if (spatial && !sphere) {   // the triangle's vertices for clipping, v0 + e1 and v0 + e2 exact in double
                crt_sah::TriVerts T;
                const double v0[3] = {f0.x, f0.y, f0.z};
                const double e1[3] = {f0.w, f1.x, f1.y}, e2[3] = {f1.z, f1.w, f2.x};
                for (int a = 0; a < 3; ++a) {
                    T.v[0][a] = v0[a];
                    T.v[1][a] = v0[a] + e1[a];
                    T.v[2][a] = v0[a] + e2[a];
                }
                it.tri = (int)verts.size();
                verts.push_back(T);
            }
            bool finite = true;
            for (int a = 0; a < 3; ++a) {
                it.c[a] = 0.5f * it.lo[a] + 0.5f * it.hi[a];
                // box_inv's clamp (2^64) keeps |coord| * inv finite only below 2^60 (wide_boxes)
                finite = finite && std::fabs(it.lo[a]) < 0x1p60f && std::fabs(it.hi[a]) < 0x1p60f;
            }
            if (!finite) { err = "primitive bounds non-finite or beyond 2^60"; return false; }
            items.push_back(it);
        }
        rank_code.assign(F.rank_code.size(), 0);
        auto append_ray_spheres = [&]() {
            sphere_first = (int)(prims.size() / 3);
            const int n_ref = F.count();
            for (int p : ray_sph) {
                const int np = (int)(prims.size() / 3);
                for (int q = 0; q < 3; ++q) prims.push_back(F.prims[3 * p + q]);
                rank_code[F.rank_of[p]] = SPHERE_BIT | np;
                // the sphere's leaf in the flattened reference scene and every scene-level node enclosing it
                int leaf = -1;
                for (int i = 0; i < n_ref && leaf < 0; ++i)
                    if (i2i(F.nodes[2 * (size_t)i + 1].w) == (SPHERE_BIT | p)) leaf = i;
                const float4 B = F.nodes[2 * (size_t)leaf + 1];
                prims[3 * (size_t)np + 1].w = i2f((int)(chain.size() / 2));
                chain.push_back(F.nodes[2 * (size_t)leaf]);
                chain.push_back(make_float4(B.x, B.y, 0.f, 0.f));
            }
            n_ray_spheres = (int)ray_sph.size();
        };
        if (items.empty()) {   // nothing hittable: one empty-box node that no ray enters
            const float lo[3] = {0, 0, 0};
            prims.assign(3, make_float4(0, 0, 0, 0));
            for (int l = 0; l < layouts; ++l) {
                nodes.push_back(make_float4(lo[0], lo[1], lo[2], lo[0]));
                nodes.push_back(make_float4(lo[1], lo[2], i2f(1), i2f(NODE_MESH_INNER)));
            }
            n_nodes = 1;
            if (width == 4) {   // a 4-wide root with no slots
                nodes.clear();
                for (int r = 0; r < 6; ++r) nodes.push_back(make_float4(1e30f, 1e30f, 1e30f, 1e30f));
                nodes.push_back(make_float4(i2f(0), i2f(0), i2f(0), i2f(0)));
                nodes.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
                prims.clear();
                append_ray_spheres();
                stack_bound = 1;
            }
            return true;
        }
        tr.lap("  SAH items");
        std::vector<crt_sah::Node> bnv;
        std::vector<crt_sah::Item> its;
        if (spatial) {
            crt_sah::SpatialBuilder B(std::move(items), std::move(verts), leaf_size, trav_cost, alpha, max_dup);
            B.build();
            max_depth = B.max_depth();
            spatial_splits = B.spatial_splits();
            bnv = B.nodes();
            its = B.items();
        } else if (gpu_device >= 0) {
            std::vector<int> order;
            if (crtx_build_sah_gpu(gpu_device, items, leaf_size, trav_cost, &bnv, &order, &max_depth) != CRT_OK) {
                err = std::string("GPU SAH build: ") + crt_last_error();
                return false;
            }
            its.resize(order.size());
            for (size_t i = 0; i < order.size(); ++i) its[i] = items[order[i]];
        } else {
            crt_sah::Builder B(std::move(items), leaf_size, trav_cost);
            B.build();
            max_depth = B.max_depth();
            bnv = B.nodes();
            its = B.items();
        }
        references = (long)its.size();
        tr.lap(gpu_device >= 0 ? "  SAH build (GPU)" : "  SAH build (host)");
        if (width == 4) {
            if (!emit4(F, bnv, its, !spatial)) return false;
            tr.lap("  4-wide collapse + emission");
            append_ray_spheres();
            tr.lap("  per-ray spheres");
            return true;
        }
        prims.resize(3 * its.size());
        for (size_t i = 0; i < its.size(); ++i) {
            const int p = its[i].src;
            for (int q = 0; q < 3; ++q) prims[3 * i + q] = F.prims[3 * p + q];
            rank_code[F.rank_of[p]] = its[i].sphere ? (SPHERE_BIT | (int)i) : (int)i;
        }
        const auto& bn = bnv;
        n_nodes = (int)bn.size();
        nodes.reserve(2 * (size_t)n_nodes * layouts);
        for (int l = 0; l < layouts; ++l) {
            const size_t base = nodes.size() / 2;
            emit(bn, its, 0, l, layouts, base);
        }
        return true;
    }

private:
    // 4-wide nodes in BFS order (internal children of a node consecutive), primitives re-laid out so the
    // leaf children of every node are consecutive in slot order.  See the node format at wide_boxes().
    bool emit4(const Flattener& F, const std::vector<crt_sah::Node>& bn, const std::vector<crt_sah::Item>& its,
               bool unique_items) {
        prims.clear();
        SetupTrace tr;
        // a 4-wide node step costs about one triangle test (the cost probe's weights); node costs 0.5
        // and 2 measured the same (profiles/r02ax)
        const crt_sah::Collapse col(bn, 1.0);
        tr.lap("    collapse DP");
        // BFS one level at a time: the level's cuts (Collapse::open, a few dependent reads of the binary tree each) in
        // parallel, then its child and primitive offsets in order
        std::vector<int> queue{0}, first_child_of, leaf_first_of;
        std::vector<crt_sah::Wide> wide;
        size_t n_items = 0;
        for (size_t lb = 0; lb < queue.size();) {
            const size_t le = queue.size();
            wide.resize(le);
            parallel_ranges(le - lb, [&](size_t b, size_t e) {
                for (size_t qi = lb + b; qi < lb + e; ++qi) wide[qi] = col.open(queue[qi]);
            }, 4096);
            for (size_t qi = lb; qi < le; ++qi) {
                const crt_sah::Wide& w = wide[qi];
                first_child_of.push_back((int)queue.size());
                for (int s = 0; s < w.n_internal; ++s) queue.push_back(w.bin[s]);
                leaf_first_of.push_back((int)n_items);
                int total_leaf = 0;
                for (int s = w.n_internal; s < w.n_slots; ++s) {
                    if (bn[w.bin[s]].count > 255) { err = "leaf too large"; return false; }
                    total_leaf += bn[w.bin[s]].count;
                }
                // node_step4 takes the leaf span from counts * 0x01010101 (byte-wise running sums)
                if (total_leaf > 255) { err = "leaf children of one node hold more than 255 primitives"; return false; }
                n_items += (size_t)total_leaf;
                // prim_test addresses a record as __umul24(index, 48): the 4-wide tree holds fewer than 2^24 primitives
                if (n_items >= ((size_t)1 << 24)) { err = "the 4-wide tree holds at most 2^24 - 1 primitives"; return false; }
            }
            lb = le;
        }
        const size_t n_wide = queue.size();
        tr.lap("    node cuts (BFS)");
        // node records and each primitive position's item (item_at), then the primitive records: every node and every
        // position is written once.  Every span node_step4 can form (leaf_first + the node's leaf counts) lies inside
        // the primitive array by construction; the fast kernel relies on it (the checked build re-checks it on the
        // device).
        nodes.assign(8 * n_wide, make_float4(0.f, 0.f, 0.f, 0.f));
        std::vector<int> item_at(n_items);
        parallel_ranges(n_wide, [&](size_t b, size_t e) {
            for (size_t qi = b; qi < e; ++qi) {
                const crt_sah::Wide& w = wide[qi];
                uint32_t counts = 0;
                int at = leaf_first_of[qi];
                for (int s = w.n_internal; s < w.n_slots; ++s) {
                    const crt_sah::Node& L = bn[w.bin[s]];
                    counts |= (uint32_t)L.count << (8 * s);
                    for (int i = L.first; i < L.first + L.count; ++i) item_at[at++] = i;
                }
                float4* row = nodes.data() + 8 * qi;
                for (int a = 0; a < 3; ++a) {
                    float lo[4], hi[4];
                    for (int s = 0; s < 4; ++s) {
                        lo[s] = hi[s] = 1e30f;   // empty slot: zero-thickness, never hit
                        if (s < w.n_slots) { lo[s] = bn[w.bin[s]].lo[a]; hi[s] = bn[w.bin[s]].hi[a]; }
                    }
                    row[2 * a] = make_float4(lo[0], lo[1], lo[2], lo[3]);
                    row[2 * a + 1] = make_float4(hi[0], hi[1], hi[2], hi[3]);
                }
                row[6] = make_float4(i2f(first_child_of[qi]), i2f(w.n_internal | (w.n_slots << 8)), i2f(leaf_first_of[qi]),
                                     i2f((int)counts));
            }
        }, 4096);
        tr.lap("    node records");
        prims.reserve(3 * (n_items + kMaxRaySpheres));   // append_ray_spheres adds at most kMaxRaySpheres records
        prims.resize(3 * n_items);
        // a primitive referenced by several leaves (spatial splits) keeps the rank code of its last position, as the
        // sequential emission did; unique items (the binned builders) have one position each, so any order will do
        auto gather = [&](size_t b, size_t e) {
            for (size_t np = b; np < e; ++np) {
                const crt_sah::Item& it = its[item_at[np]];
                for (int q = 0; q < 3; ++q) prims[3 * np + q] = F.prims[3 * (size_t)it.src + q];
                rank_code[F.rank_of[it.src]] = it.sphere ? (SPHERE_BIT | (int)np) : (int)np;
            }
        };
        if (unique_items) parallel_ranges(n_items, gather);
        else gather(0, n_items);
        n_nodes = (int)queue.size();
        tr.lap("    primitive gather");
        // stack bound: visiting a node with 2+ hit internal children pushes ONE entry (its remaining children)
        if (n_nodes >= (1 << 24)) { err = "too many nodes for 24-bit stack entries"; return false; }
        std::vector<int> bound(n_nodes, 0);
        for (int n = n_nodes - 1; n >= 0; --n) {
            const int fc = i2i(nodes[8 * (size_t)n + 6].x), m = wide[n].n_internal;
            int b = 0;
            for (int s = 0; s < m; ++s) b = std::max(b, bound[fc + s]);
            bound[n] = b + (m >= 2 ? 1 : 0);
        }
        stack_bound = bound[0] + 1;
        return true;
    }
    static int i2i(float f) { int v; std::memcpy(&v, &f, 4); return v; }

    void emit(const std::vector<crt_sah::Node>& bn, const std::vector<crt_sah::Item>& its, int ni, int layout,
              int layouts, size_t base) {
        const crt_sah::Node& N = bn[ni];
        const size_t idx = nodes.size() / 2;
        int a = 0, b;
        if (N.child[0] < 0) {
            if (its[N.first].sphere) b = SPHERE_BIT | N.first;
            else { a = N.count; b = N.first; }
        } else {
            b = NODE_MESH_INNER;
        }
        nodes.push_back(make_float4(N.lo[0], N.lo[1], N.lo[2], N.hi[0]));
        nodes.push_back(make_float4(N.hi[1], N.hi[2], i2f(a), i2f(b)));
        if (N.child[0] < 0) return;
        int first = N.child[0], second = N.child[1];
        if (layouts == 6) {   // near child first along the layout's direction
            const int ax = layout / 2;
            const bool neg = layout & 1;
            const float c0 = bn[first].lo[ax] + bn[first].hi[ax], c1 = bn[second].lo[ax] + bn[second].hi[ax];
            if (neg ? (c1 > c0) : (c1 < c0)) std::swap(first, second);
        }
        emit(bn, its, first, layout, layouts, base);
        emit(bn, its, second, layout, layouts, base);
        nodes[2 * idx + 1].z = i2f((int)(nodes.size() / 2 - base));   // skip, relative to the layout
    }
};

}  // namespace

struct crt_scene {
    int device = 0;
    float4* d_nodes = nullptr;
    float4* d_prims = nullptr;
    float4* d_mats = nullptr;
    float4* d_chain = nullptr;     // width 4: reference scene-level boxes on the per-ray spheres' paths
    int n_chain = 0;
    float4* d_shade = nullptr;     // shading record per rank (crt_device.h)
    int n_nodes = 0, n_prims = 0, n_mats = 0, n_ranks = 0;   // n_nodes per layout
    int max_depth = 0;
    int bvh = CRT_BVH_REFERENCE, layouts = 1;
    int width = 2;                 // 2: threaded layouts (variants 0-3); 4: 4-wide nodes (variant 4)
    int stack_cap = 0;             // width 4: traversal-stack entries a ray can need
    long spatial_splits = 0, references = 0;   // rebuilt tree: SBVH cuts, leaf references
    int sphere_first = 0, n_ray_spheres = 0;   // width 4: spheres tested per ray, prims [first, first + n)
    float sph2[2][12] = {};                    // width 4 with exactly two per-ray spheres: their kernel-argument copy
    int tree_spheres = 1;                      // width 4: some leaf holds a sphere
    long excluded = 0;
};

constexpr int ERR_WORD = 15;      // d_counters word of the device error flags (RenderParams::err)

struct crt_renderer {
    int device = 0, width = 0, height = 0;
    uint32_t* d_rng = nullptr;
    float* d_sum = nullptr;       // active linear framebuffer (own or attached)
    float* d_sum_own = nullptr;
    uint8_t* d_rgba = nullptr;
    uint32_t* d_seq = nullptr;
    unsigned long long* d_counters = nullptr;
    crt_camera_desc cam{};
    bool has_camera = false;
    // HIP events of the current render: ev0 before the cost probe, ev_main just before the main render kernel (after
    // the probe and the tile sort), ev1 after it.  They point into a ring of CRT_TIMING_RING frames, so a caller that
    // renders K frames back to back without synchronising can read every frame's phases afterwards
    // (crt_renderer_timing_history).  The ring has one slot more than the history reaches: a render records into slot
    // n_timed % (CRT_TIMING_RING + 1), which none of the last CRT_TIMING_RING complete frames occupies, so a render that
    // fails after its first event (an allocation, the overflow-region check) leaves every readable slot intact.
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_main = nullptr;
    hipEvent_t ring[CRT_TIMING_RING + 1][3] = {};
    unsigned long long n_timed = 0;   // renders whose three events were all recorded
    char kernel_name[64] = "";     // instantiation of the last render launch, rocprof's spelling
    // variant 7: pixel order, slot queue, probe costs, sort scratch (allocated on first use)
    uint32_t* d_order = nullptr;
    uint32_t* d_queue = nullptr;
    uint32_t* d_tile_cost = nullptr;   // per-pixel probe costs
    uint32_t* d_order_hist = nullptr;
    uint32_t* d_tile_key = nullptr;    // variant 8: per-tile keys
    unsigned long long* d_probe_stats = nullptr;   // crt_tile_cost_kernel's stats: largest tile work, total work
    unsigned long long* h_probe_stats = nullptr;   // their pinned host copy
    float last_schedule[4] = {0.f, 0.f, 0.f, 0.f};  // crt_renderer_last_schedule
    uint32_t* d_rng_cache = nullptr;   // curand_init result of (rng_cache_seed, rng_cache_base)
    unsigned long long rng_cache_seed = 0, rng_cache_base = 0;
    bool rng_cache_valid = false;
    int probe_spp = -1;            // samples per pixel of the cost probe; 0 = no probe (8x8-tile order),
                                   // -1 = automatic: 4 for renders of >= 1000 spp, else 2 (profiles/r01ad)
    int probe_min_spp = 64;        // renders with fewer samples per pixel skip the probe
    int tile_key_mode = 2;         // variant 8: see crt_tile_cost_kernel (2: measured best, profiles/r01ac)
    int n_cus = 0;
    int variant = -1;              // see crt_renderer_set_kernel_variant; -1 = automatic
    unsigned long long diag[3] = {0, 0, 0};
    unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // COUNT-mode section profile (variant 4)
    int regen_threshold = 24;      // variants 2/3
    int regen_threshold_wide = 44; // variants 4/7/8 (measured: 40 for variant 4, profiles/r01d; 44-48 for 8, r01af)
    int crit_tiles = -1;           // variant 8: leading tiles of the cost order regenerating at crit_threshold; -1 = 4 per CU
    int tile_shard = 0, tile_shards = 1;   // pixel sharding (crt_renderer_set_pixel_shard)
    int crit_threshold = 16;       // (measured: profiles/r02h, r02i)
    int top_levels = -1;           // 4-wide variants: new rays' first node steps from LDS; -1 = CRT_TOP_LEVELS
    int xcd_regions = 0;           // variant 8: XCD groups render screen strips (crt_xcd_order_kernel)
    int probe_stride = 0;          // variant 8's cost probe: every probe_stride-th pixel in x and y (0 = automatic)
    int temporal = 0;              // variant 7: tiles ordered by the previous variant-7 frame's rays per pixel
    int drain_threshold = 0;       // variant 7: regeneration threshold once the pixel queue is empty (0 = unchanged)
    int wave_drain = 48;           // variants 4/8: draining waves pass at 48/64 of their live lanes (profiles/r04n)
    uint32_t* d_pix_rays = nullptr;   // variant 7 with the temporal order: rays per pixel of the last frame
    uint32_t* d_tile_order = nullptr; // its tiles, most expensive first
    bool pix_rays_valid = false;
    int min_waves = 0;             // occupancy target (waves/SIMD); 0 = auto: 7 for variant 8 over >= 4 tiles per wave
                                   // slot, 6 for the other 4-wide launches and variants 3 and 10, 5 for variants 0-2
    uint32_t* d_ovf = nullptr;     // variant 4: stack entries beyond the LDS part, ovf_entries x W*H
    size_t ovf_entries = 0;
    int stack_lds = STACK_LDS;     // variant 4: per-lane stack entries kept in LDS
    float rcp_w = 1.f, rcp_h = 1.f; // RN(1 / width), RN(1 / height)
    int fast_uv = 0;               // next_ray divides by uv_div (verified for this size at creation, uv_div_mismatches)
    // variant 5 (wavefront) state, allocated on first use
};

namespace {
int use_device(int dev) {
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (n <= 0) return set_error(CRT_ERR_NO_DEVICE, "no HIP device visible");
    if (dev < 0 || dev >= n) return set_error(CRT_ERR_INVALID_ARGUMENT, "device ordinal out of range");
    HIP_TRY(hipSetDevice(dev));
    return CRT_OK;
}
}  // namespace

extern "C" {

int crt_abi_version(void) { return CRT_ABI_VERSION; }
int crt_build_flags(void) {
#ifdef CRT_CHECKED
    return CRT_BUILD_CHECKED;
#else
    return 0;
#endif
}
const char* crt_last_error(void) { return g_last_error.c_str(); }

int crt_device_count(int* out) {
    if (!out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *out = (e == hipSuccess) ? n : 0;
    return CRT_OK;
}

int crt_scene_create(const crt_scene_desc* D, int device, crt_scene** out) {
    return crt_scene_create_ex(D, device, nullptr, out);
}

}  // extern "C"

// Host half of scene creation: flatten the reference BVHs (ranks, reachability) and, for CRT_BVH_REBUILT,
// build the SAH tree.  Shared by crt_scene_create_ex and crt_scene_export.
static int build_scene_arrays(const crt_scene_desc* D, const crt_scene_options* opts, crt_scene_options& o,
                              Flattener& F, Rebuilt& RB, int gpu_device) {
    o = crt_scene_options{};
    if (opts) o = *opts;
    if (o.bvh != CRT_BVH_REFERENCE && o.bvh != CRT_BVH_REBUILT) return set_error(CRT_ERR_INVALID_ARGUMENT, "unknown bvh mode");
    if (o.leaf_size == 0) o.leaf_size = 4;
    if (o.layouts == 0) o.layouts = 6;
    if (o.traversal_cost == 0.f) o.traversal_cost = 2.f;   // measured optimum for 4-wide leaves <= 4 (profiles/r01i)
    if (o.width == 0) o.width = 4;
    if (o.width != 2 && o.width != 4) return set_error(CRT_ERR_INVALID_ARGUMENT, "width must be 2 or 4");
    if (!(o.traversal_cost > 0.f && o.traversal_cost <= 64.f)) return set_error(CRT_ERR_INVALID_ARGUMENT, "traversal_cost must be in (0, 64]");
    if (o.leaf_size < 1 || o.leaf_size > 16) return set_error(CRT_ERR_INVALID_ARGUMENT, "leaf_size must be 1..16");
    if (o.layouts != 1 && o.layouts != 6) return set_error(CRT_ERR_INVALID_ARGUMENT, "layouts must be 1 or 6");
    if (D->n_scene_nodes <= 0 || !D->scene_nodes) return set_error(CRT_ERR_INVALID_ARGUMENT, "scene has no BVH nodes");
    if (D->n_materials < 0 || (D->n_materials > 0 && !D->materials)) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad materials");
    SetupTrace tr;
    if (!F.build_triangles()) return set_error(CRT_ERR_INVALID_ARGUMENT, "scene: " + F.err);
    tr.lap("triangle records");
    if (!F.emit_scene(0, 0, false)) return set_error(CRT_ERR_INVALID_ARGUMENT, "scene: " + F.err);
    tr.lap("flatten reference BVHs");
    F.finalize_ranks();
    tr.lap("ranks");
    if (o.bvh == CRT_BVH_REBUILT) {
        if (o.width == 4) o.layouts = 1;
        if (o.spatial_alpha == 0.f) o.spatial_alpha = 1e-5f;
        if (o.spatial_max_dup == 0.f) o.spatial_max_dup = 1.f;
        if (o.spatial_splits != 0 && o.spatial_splits != 1) return set_error(CRT_ERR_INVALID_ARGUMENT, "spatial_splits must be 0 or 1");
        if (!(o.spatial_alpha > 0.f && o.spatial_alpha <= 1.f) || !(o.spatial_max_dup > 0.f && o.spatial_max_dup <= 8.f))
            return set_error(CRT_ERR_INVALID_ARGUMENT, "spatial_alpha must be in (0, 1], spatial_max_dup in (0, 8]");
        if (!RB.build(F, o.leaf_size, o.layouts, o.traversal_cost, o.width, o.gpu_build && !o.spatial_splits ? gpu_device : -1,
                      o.spatial_splits != 0, o.spatial_alpha, o.spatial_max_dup))
            return set_error(CRT_ERR_INVALID_ARGUMENT, "scene: " + RB.err);
        tr.lap("rebuilt tree (all)");
        if ((size_t)RB.n_nodes * o.layouts * (o.width == 4 ? 8 : 2) >= (size_t)1 << 31)
            return set_error(CRT_ERR_INVALID_ARGUMENT, "scene too large");
    }
    return CRT_OK;
}

extern "C" {

int crt_scene_export(const crt_scene_desc* D, const crt_scene_options* opts, float* nodes, float* prims,
                     int32_t* rank_code, int64_t info[10]) {
    if (!D || !info) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    crt_scene_options o;
    Flattener F{D};
    Rebuilt RB;
    if (int rc = build_scene_arrays(D, opts, o, F, RB, 0)) return rc;
    const bool rebuilt = o.bvh == CRT_BVH_REBUILT;
    const std::vector<float4>& N = rebuilt ? RB.nodes : F.nodes;
    const std::vector<float4>& Pr = rebuilt ? RB.prims : F.prims;
    const std::vector<int>& rc = rebuilt ? RB.rank_code : F.rank_code;
    info[0] = (int64_t)N.size();
    info[1] = (int64_t)Pr.size();
    info[2] = (int64_t)rc.size();
    info[3] = rebuilt ? RB.n_nodes : F.count();
    info[4] = rebuilt ? o.layouts : 1;
    info[5] = rebuilt ? RB.width : 2;
    info[6] = rebuilt ? RB.stack_bound : 0;
    info[7] = rebuilt ? RB.excluded : 0;
    info[8] = rebuilt ? RB.sphere_first : 0;
    info[9] = rebuilt ? RB.n_ray_spheres : 0;
    if (nodes) std::memcpy(nodes, N.data(), N.size() * sizeof(float4));
    if (prims) std::memcpy(prims, Pr.data(), Pr.size() * sizeof(float4));
    if (rank_code) std::memcpy(rank_code, rc.data(), rc.size() * sizeof(int));
    return CRT_OK;
}

// Per-rank shading records (layout in crt_device.h).  The triangle normal is unit(cross(e1, e2)) in the
// device's f32 operation order (the library is compiled with -ffp-contract=off and IEEE sqrt / division on
// the host too), so the record holds exactly the value shade() used to compute per hit.
static std::vector<float4> shading_records(const std::vector<int>& rank_code, const std::vector<float4>& prims,
                                           const crt_scene_desc* D) {
    std::vector<float4> out(3 * rank_code.size(), make_float4(0.f, 0.f, 0.f, 0.f));
    parallel_ranges(rank_code.size(), [&](size_t rb, size_t re) {
        for (size_t r = rb; r < re; ++r) {
            const bool sphere = (rank_code[r] & SPHERE_BIT) != 0;
            const size_t p = (size_t)(rank_code[r] & ~SPHERE_BIT);
            const float4 f0 = prims[3 * p], f1 = prims[3 * p + 1], f2 = prims[3 * p + 2];
            const uint32_t mat = (uint32_t)i2i_host(sphere ? f1.y : f2.y);
            uint32_t code = SHADE_INVALID;
            float4 pay = make_float4(0.f, 0.f, 0.f, 0.f);
            if (mat < (uint32_t)D->n_materials) {
                const crt_material_desc& M = D->materials[mat];
                switch (M.type) {
                    case CRT_LAMBERTIAN: code = SHADE_LAMBERT; pay = make_float4(M.albedo[0], M.albedo[1], M.albedo[2], 0.f); break;
                    case CRT_METAL:
                        code = SHADE_METAL;
                        pay = make_float4(M.albedo[0], M.albedo[1], M.albedo[2], M.roughness < 1.f ? M.roughness : 1.f);
                        break;
                    case CRT_DIELECTRIC: {
                        // Material.cuh:113 ri = front ? 1.0f / ior : ior, and Schlick's r0 = ((1 - ri) / (1 + ri))^2
                        // (:133-134) for both faces, in IEEE f32 as the device would compute them per hit
                        code = SHADE_DIELECTRIC;
                        auto r0 = [](float r) { const float x = (1 - r) / (1 + r); return x * x; };
                        const float inv = 1.0f / M.ior;
                        pay = make_float4(M.ior, inv, r0(inv), r0(M.ior));
                        break;
                    }
                    case CRT_DIFFUSE_LIGHT:
                        code = SHADE_LIGHT;
                        pay = make_float4(M.emission[0], M.emission[1], M.emission[2], 0.f);
                        break;
                    default: code = SHADE_NOEMIT; break;
                }
            }
            float4 a;
            if (sphere) {
                a = make_float4(f0.x, f0.y, f0.z, i2f((int)(code | SHADE_SPHERE)));
                out[3 * r + 2] = make_float4(1 / f0.w, 0.f, 0.f, 0.f);
            } else {
                const float ux = f0.w, uy = f1.x, uz = f1.y, vx = f1.z, vy = f1.w, vz = f2.x;
                const float cx = uy * vz - uz * vy, cy = uz * vx - ux * vz, cz = ux * vy - uy * vx;
                const float s = 1.0f / std::sqrt(cx * cx + cy * cy + cz * cz);
                a = make_float4(s * cx, s * cy, s * cz, i2f((int)code));
            }
            out[3 * r] = a;
            out[3 * r + 1] = pay;
        }
    });
    return out;
}

int crt_scene_create_ex(const crt_scene_desc* D, int device, const crt_scene_options* opts, crt_scene** out) {
    if (!D || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    crt_scene_options o;
    Flattener F{D};
    Rebuilt RB;
    if (int rc = build_scene_arrays(D, opts, o, F, RB, device)) return rc;
    SetupTrace tr;
    const bool rebuilt = o.bvh == CRT_BVH_REBUILT;
    std::vector<float4> mats;
    for (int i = 0; i < D->n_materials; ++i) {
        const crt_material_desc& M = D->materials[i];
        mats.push_back(make_float4(i2f(M.type), M.albedo[0], M.albedo[1], M.albedo[2]));
        mats.push_back(make_float4(M.emission[0], M.emission[1], M.emission[2], M.roughness < 1.f ? M.roughness : 1.f));
        mats.push_back(make_float4(M.ior, 0.f, 0.f, 0.f));
    }
    if (int rc = use_device(device)) return rc;
    crt_scene* S = new (std::nothrow) crt_scene;
    if (!S) return set_error(CRT_ERR_OUT_OF_MEMORY, "host allocation failed");
    S->device = device;
    S->bvh = o.bvh;
    S->layouts = rebuilt ? o.layouts : 1;
    S->n_nodes = rebuilt ? RB.n_nodes : F.count();
    S->n_prims = (int)((rebuilt ? RB.prims : F.prims).size() / 3);
    S->n_ranks = (int)F.rank_code.size();
    S->n_mats = D->n_materials;
    S->max_depth = rebuilt ? RB.max_depth : F.max_depth;
    S->excluded = rebuilt ? RB.excluded : 0;
    S->width = rebuilt ? RB.width : 2;
    S->stack_cap = rebuilt ? (o.stack_cap > 0 ? o.stack_cap : RB.stack_bound) : 0;
    S->sphere_first = rebuilt ? RB.sphere_first : 0;
    S->spatial_splits = rebuilt ? RB.spatial_splits : 0;
    S->references = rebuilt ? RB.references : 0;
    {
        int in_tree = 0;   // spheres the 4-wide tree itself holds (not tested per ray)
        if (rebuilt)
            for (int r = 0; r < (int)RB.rank_code.size(); ++r)
                if ((RB.rank_code[r] & SPHERE_BIT) && (RB.rank_code[r] & ~SPHERE_BIT) < RB.sphere_first) ++in_tree;
        S->tree_spheres = in_tree > 0 || !rebuilt;
    }
    if (rebuilt && RB.n_ray_spheres == 2) {
        for (int s = 0; s < 2; ++s) {
            const size_t q = 3 * (size_t)(RB.sphere_first + s);
            const float4 f0 = RB.prims[q], f1 = RB.prims[q + 1];
            const int k = i2i_host(f1.w);
            const float4 A = RB.chain[2 * (size_t)k], B = RB.chain[2 * (size_t)k + 1];
            const float v[12] = {f0.x, f0.y, f0.z, f1.x, f1.z, A.x, A.y, A.z, A.w, B.x, B.y, 0.f};
            std::memcpy(S->sph2[s], v, sizeof v);
        }
    }
    S->n_chain = rebuilt ? (int)(RB.chain.size() / 2) : 0;
    S->n_ray_spheres = rebuilt ? RB.n_ray_spheres : 0;
    auto up = [&](float4** dst, const std::vector<float4>& src) -> hipError_t {
        size_t bytes = std::max<size_t>(src.size(), 1) * sizeof(float4);
        hipError_t e = hipMalloc((void**)dst, bytes);
        if (e != hipSuccess) return e;
        if (!src.empty()) e = hipMemcpy(*dst, src.data(), src.size() * sizeof(float4), hipMemcpyHostToDevice);
        return e;
    };
    const std::vector<int>& rc = rebuilt ? RB.rank_code : F.rank_code;
    std::vector<float4> swizzled;   // width 4: row k of node n at slot k ^ (n & 7) of its record (node_row)
    if (S->width == 4) {
        swizzled.resize(RB.nodes.size());
        for (size_t n = 0; n < RB.nodes.size() / 8; ++n)
            for (size_t k = 0; k < 8; ++k) swizzled[8 * n + (k ^ (n & 7))] = RB.nodes[8 * n + k];
    }
    tr.lap("node swizzle");
    const std::vector<float4> shade = shading_records(rc, rebuilt ? RB.prims : F.prims, D);
    tr.lap("shading records");
    hipError_t e;
    if ((e = up(&S->d_nodes, S->width == 4 ? swizzled : (rebuilt ? RB.nodes : F.nodes))) != hipSuccess ||
        (e = up(&S->d_prims, rebuilt ? RB.prims : F.prims)) != hipSuccess ||
        (e = up(&S->d_mats, mats)) != hipSuccess ||
        (e = up(&S->d_chain, rebuilt ? RB.chain : std::vector<float4>())) != hipSuccess ||
        (e = up(&S->d_shade, shade)) != hipSuccess) {
        crt_scene_destroy(S);
        return set_error(CRT_ERR_HIP, std::string("scene upload: ") + hipGetErrorString(e));
    }
    tr.lap("uploads");
    *out = S;
    return CRT_OK;
}

int crt_scene_get_stats(const crt_scene* S, crt_scene_stats* out) {
    if (!S || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    out->device_nodes = (int64_t)S->n_nodes * S->layouts;
    out->width = S->width;
    out->stack_bound = S->stack_cap;
    out->spatial_splits = S->spatial_splits;
    out->references = S->references;
    out->device_prims = S->n_prims;
    out->device_bytes = (int64_t)S->n_nodes * S->layouts * (S->width == 4 ? 128 : 32) + (int64_t)S->n_prims * 48 + (int64_t)S->n_mats * 48 +
                        (int64_t)S->n_ranks * 48;
    out->max_depth = S->max_depth;
    out->n_materials = S->n_mats;
    out->bvh = S->bvh;
    out->layouts = S->layouts;
    out->excluded_prims = S->excluded;
    return CRT_OK;
}

void crt_scene_destroy(crt_scene* S) {
    if (!S) return;
    (void)hipSetDevice(S->device);
    if (S->d_nodes) (void)hipFree(S->d_nodes);
    if (S->d_prims) (void)hipFree(S->d_prims);
    if (S->d_mats) (void)hipFree(S->d_mats);
    if (S->d_shade) (void)hipFree(S->d_shade);
    if (S->d_chain) (void)hipFree(S->d_chain);
    delete S;
}

namespace {
// Mismatches of uv_div(a, b, RN(1 / b)) against a / b over every a next_ray can form for an image dimension b:
// a = fl(x + U) with x in [0, b - 1] and U = fl(X * 2^-32 + 2^-33) in [2^-33, 1], so a in [2^-33, b].
constexpr uint32_t UV_A_MIN_BITS = 0x2f000000u;   // 2^-33
int uv_div_mismatches(int dim, unsigned long long* out) {
    const float b = (float)dim, r = 1.0f / b;
    uint32_t hi;
    std::memcpy(&hi, &b, 4);
    unsigned long long* d;
    HIP_TRY(hipMalloc((void**)&d, 8));
    hipError_t e = hipMemset(d, 0, 8);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(crt_uv_div_check_kernel, dim3(4096), dim3(256), 0, 0, b, r, UV_A_MIN_BITS, hi, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIP_TRY(e);
    return CRT_OK;
}
}  // namespace

int crt_selftest_uv_div(int dim, unsigned long long* mismatches) {
    if (dim <= 0 || !mismatches) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    return uv_div_mismatches(dim, mismatches);
}

static hipError_t create_timing_ring(crt_renderer* R) {
    for (auto& slot : R->ring)
        for (hipEvent_t& ev : slot)
            if (hipError_t e = hipEventCreate(&ev); e != hipSuccess) return e;
    return hipSuccess;
}

int crt_renderer_create(int width, int height, int device, crt_renderer** out) {
    if (!out || width <= 0 || height <= 0 || (long long)width * height > (1LL << 31) / 6)
        return set_error(CRT_ERR_INVALID_ARGUMENT, "bad renderer size");
    *out = nullptr;
    if (int rc = use_device(device)) return rc;
    crt_renderer* R = new (std::nothrow) crt_renderer;
    if (!R) return set_error(CRT_ERR_OUT_OF_MEMORY, "host allocation failed");
    R->device = device; R->width = width; R->height = height;
    const size_t n = (size_t)width * height;
    const auto& tab = seq_tables();
    hipError_t e;
    if ((e = hipMalloc((void**)&R->d_rng, n * 6 * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&R->d_sum_own, n * 3 * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&R->d_rgba, n * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&R->d_seq, tab.size() * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&R->d_counters, 16 * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipMemcpy(R->d_seq, tab.data(), tab.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(R->d_sum_own, 0, n * 3 * 4)) != hipSuccess ||
        (e = hipMemset(R->d_rgba, 0, n * 4)) != hipSuccess ||
        (e = hipMemset(R->d_counters, 0, 16 * sizeof(unsigned long long))) != hipSuccess ||
        (e = create_timing_ring(R)) != hipSuccess) {
        crt_renderer_destroy(R);
        return set_error(e == hipErrorOutOfMemory ? CRT_ERR_OUT_OF_MEMORY : CRT_ERR_HIP,
                         std::string("renderer allocation: ") + hipGetErrorString(e));
    }
    R->d_sum = R->d_sum_own;
    // next_ray's image-coordinate divisions: uv_div when it equals the IEEE division for every input of this size
    unsigned long long bad_w = 0, bad_h = 0;
    int rc = uv_div_mismatches(width, &bad_w);
    if (rc == CRT_OK) rc = height == width ? CRT_OK : uv_div_mismatches(height, &bad_h);
    if (rc != CRT_OK) {
        crt_renderer_destroy(R);
        return rc;
    }
    R->rcp_w = 1.0f / (float)width;
    R->rcp_h = 1.0f / (float)height;
    R->fast_uv = bad_w == 0 && bad_h == 0;
    *out = R;
    return CRT_OK;
}

int crt_renderer_attach_linear(crt_renderer* R, float* ptr) {
    if (!R) return set_error(CRT_ERR_INVALID_ARGUMENT, "null renderer");
    if (ptr) {
        hipPointerAttribute_t attr;
        HIP_TRY(hipPointerGetAttributes(&attr, ptr));
        if (attr.type != hipMemoryTypeDevice || attr.device != R->device)
            return set_error(CRT_ERR_INVALID_ARGUMENT, "attach_linear: not device memory of the renderer's device");
    }
    R->d_sum = ptr ? ptr : R->d_sum_own;
    return CRT_OK;
}

void crt_renderer_destroy(crt_renderer* R) {
    if (!R) return;
    (void)hipSetDevice(R->device);
    if (R->d_rng) (void)hipFree(R->d_rng);
    if (R->d_sum_own) (void)hipFree(R->d_sum_own);
    if (R->d_rgba) (void)hipFree(R->d_rgba);
    if (R->d_seq) (void)hipFree(R->d_seq);
    if (R->d_counters) (void)hipFree(R->d_counters);
    if (R->d_ovf) (void)hipFree(R->d_ovf);
    if (R->d_order) (void)hipFree(R->d_order);
    if (R->d_queue) (void)hipFree(R->d_queue);
    if (R->d_tile_cost) (void)hipFree(R->d_tile_cost);
    if (R->d_order_hist) (void)hipFree(R->d_order_hist);
    if (R->d_tile_key) (void)hipFree(R->d_tile_key);
    if (R->d_probe_stats) (void)hipFree(R->d_probe_stats);
    if (R->h_probe_stats) (void)hipHostFree(R->h_probe_stats);
    if (R->d_pix_rays) (void)hipFree(R->d_pix_rays);
    if (R->d_tile_order) (void)hipFree(R->d_tile_order);
    if (R->d_rng_cache) (void)hipFree(R->d_rng_cache);
    for (auto& slot : R->ring)
        for (hipEvent_t& ev : slot)
            if (ev) (void)hipEventDestroy(ev);
    delete R;
}

int crt_renderer_init_rand(crt_renderer* R, unsigned long long seed, unsigned long long subseq_base, void* stream) {
    if (!R) return set_error(CRT_ERR_INVALID_ARGUMENT, "null renderer");
    HIP_TRY(hipSetDevice(R->device));
    const int n = R->width * R->height;
    hipStream_t st = (hipStream_t)stream;
    // curand_init is a pure function of (seed, subsequence): keep the initialised array and copy it back for a
    // repeated (seed, base) — 2.8 ms of GF(2) jumps at 2560x1440 become a 35 us device copy, same bits
    if (R->rng_cache_valid && R->rng_cache_seed == seed && R->rng_cache_base == subseq_base) {
        HIP_TRY(hipMemcpyAsync(R->d_rng, R->d_rng_cache, (size_t)n * 24, hipMemcpyDeviceToDevice, st));
        return CRT_OK;
    }
    hipLaunchKernelGGL(crt_init_rand_kernel, dim3((n + 255) / 256), dim3(256), 0, st, R->d_rng,
                       R->d_seq, n, seed, subseq_base);
    HIP_TRY(hipGetLastError());
    R->rng_cache_valid = false;
    if (!R->d_rng_cache) {
        HIP_TRY(hipStreamSynchronize(st));
        if (hipMalloc((void**)&R->d_rng_cache, (size_t)n * 24) != hipSuccess) {   // optional: no cache then
            (void)hipGetLastError();
            R->d_rng_cache = nullptr;
            return CRT_OK;
        }
    }
    HIP_TRY(hipMemcpyAsync(R->d_rng_cache, R->d_rng, (size_t)n * 24, hipMemcpyDeviceToDevice, st));
    R->rng_cache_seed = seed;
    R->rng_cache_base = subseq_base;
    R->rng_cache_valid = true;
    return CRT_OK;
}

int crt_renderer_set_kernel_variant(crt_renderer* R, int variant) {
    if (!R || variant < -1 || variant > 10 || variant == 5 || variant == 6 || variant == 9)
        return set_error(CRT_ERR_INVALID_ARGUMENT, "bad kernel variant (-1 = automatic, 0-4, 7, 8, 10)");
    R->variant = variant;
    return CRT_OK;
}

int crt_renderer_set_schedule(crt_renderer* R, int probe_spp, int min_spp, int flags) {
    if (!R || probe_spp < -1 || probe_spp > 64 || min_spp < 0) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad schedule");
    const int stride = (flags >> 20) & 0xf;   // variant 8's probe subsampling: 0 = automatic, 1 (every pixel), 2, 4
    if (stride != 0 && stride != 1 && stride != 2 && stride != 4)   // checked before any field changes
        return set_error(CRT_ERR_INVALID_ARGUMENT, "probe stride (flags >> 20): 0, 1, 2 or 4");
    R->probe_spp = probe_spp < 0 ? -1 : probe_spp;
    R->probe_min_spp = min_spp;
    R->tile_key_mode = (flags >> 16) & 0xf;   // 0 = slowest pixel (callers that pass 0 get the plain key)
    R->probe_stride = stride;
    return CRT_OK;
}

int crt_renderer_set_pixel_shard(crt_renderer* R, int shard, int shards) {
    if (!R || shards < 1 || shard < 0 || shard >= shards) return set_error(CRT_ERR_INVALID_ARGUMENT, "shard in [0, shards)");
    const int n_tiles = ((R->width + 7) / 8) * ((R->height + 7) / 8);
    if (shards > n_tiles) return set_error(CRT_ERR_INVALID_ARGUMENT, "more shards than 8x8 tiles");
    R->tile_shard = shard;
    R->tile_shards = shards;
    return CRT_OK;
}

int crt_renderer_set_top_levels(crt_renderer* R, int levels) {
    if (!R || levels < -1 || levels > CRT_TOP_LEVELS)
        return set_error(CRT_ERR_INVALID_ARGUMENT, "top levels -1 (default) .. " + std::to_string(CRT_TOP_LEVELS));
    R->top_levels = levels;
    return CRT_OK;
}

int crt_renderer_set_critical_tiles(crt_renderer* R, int tiles, int lanes) {
    if (!R || tiles < -1 || lanes < 1 || lanes > 64) return set_error(CRT_ERR_INVALID_ARGUMENT, "critical tiles >= -1, lanes 1..64");
    R->crit_tiles = tiles;
    R->crit_threshold = lanes;
    return CRT_OK;
}

int crt_renderer_set_occupancy_target(crt_renderer* R, int waves_per_simd) {
    if (!R || waves_per_simd < 0 || waves_per_simd > 8) return set_error(CRT_ERR_INVALID_ARGUMENT, "waves per SIMD 0..8");
    R->min_waves = waves_per_simd;
    return CRT_OK;
}

int crt_renderer_set_stack_lds(crt_renderer* R, int entries) {
    if (!R || entries < 1 || entries > STACK_LDS) return set_error(CRT_ERR_INVALID_ARGUMENT, "stack LDS entries 1..16");
    R->stack_lds = entries;
    return CRT_OK;
}

int crt_renderer_set_regen_threshold(crt_renderer* R, int lanes) {
    if (!R || lanes < 1 || lanes > 64) return set_error(CRT_ERR_INVALID_ARGUMENT, "threshold must be 1..64");
    R->regen_threshold = lanes;
    R->regen_threshold_wide = lanes;
    return CRT_OK;
}

int crt_renderer_set_camera(crt_renderer* R, const crt_camera_desc* cam) {
    if (!R || !cam) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    // primary rays start within lens_radius of the origin (right/up are unit vectors); the 4-wide slab test needs
    // |o| * 2^64 finite (box_inv), the same 2^60 bound the rebuilt tree's boxes are held to
    bool ok = std::isfinite(cam->lens_radius) && std::fabs(cam->lens_radius) < 0x1p58f;
    for (int a = 0; a < 3; ++a) ok = ok && std::isfinite(cam->origin[a]) && std::fabs(cam->origin[a]) < 0x1p59f;
    if (!ok) return set_error(CRT_ERR_INVALID_ARGUMENT, "camera origin or lens radius non-finite or beyond 2^59");
    R->cam = *cam;
    R->has_camera = true;
    return CRT_OK;
}

// Cost-probe samples for a render of `spp` samples per pixel (0 = no probe).
static int probe_spp_for(const crt_renderer* R, int spp) {
    if (spp < R->probe_min_spp || R->probe_spp == 0) return 0;
    return R->probe_spp > 0 ? R->probe_spp : (spp >= 1000 ? 4 : 2);
}

int crt_renderer_render(crt_renderer* R, const crt_scene* S, int spp, int max_bounces, unsigned flags, void* stream) {
    if (!R || !S) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    if (!R->has_camera) return set_error(CRT_ERR_INVALID_ARGUMENT, "camera not set");
    if (spp < 0 || max_bounces < 0) return set_error(CRT_ERR_INVALID_ARGUMENT, "negative spp / bounces");
    if (S->device != R->device) return set_error(CRT_ERR_INVALID_ARGUMENT, "scene and renderer on different devices");
    HIP_TRY(hipSetDevice(R->device));
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(R->d_counters, 0, ERR_WORD * sizeof(unsigned long long), st));   // the error word stays
    RenderParams P{};
    P.nodes = S->d_nodes; P.prims = S->d_prims; P.mats = S->d_mats; P.shade = S->d_shade;
    P.n_nodes = S->n_nodes; P.n_mats = S->n_mats; P.n_prims = S->n_prims; P.n_layouts = S->layouts;
    P.err = reinterpret_cast<unsigned*>(R->d_counters + ERR_WORD);
    P.width = R->width; P.height = R->height; P.spp = spp; P.max_bounces = max_bounces;
    P.accumulate = (flags & CRT_RENDER_ACCUMULATE) ? 1 : 0;
    P.rng = R->d_rng; P.sum = R->d_sum; P.counters = R->d_counters; P.cam = R->cam;
    P.rcp_w = R->rcp_w; P.rcp_h = R->rcp_h; P.fast_uv = R->fast_uv;
    P.probe_stride = 1;
    P.pix_rays = nullptr;
    P.ovf = nullptr;
    P.order = nullptr; P.queue = nullptr; P.n_slots = 0; P.probe_cost = nullptr; P.tiles_x = 0; P.crit_tiles = 0; P.crit_threshold = 64;
    P.top_levels = R->top_levels < 0 ? CRT_TOP_LEVELS : R->top_levels;
    P.stack_cap = S->stack_cap;
    P.sphere_first = S->sphere_first;
    P.n_ray_spheres = S->n_ray_spheres;
    P.sphere_chain = S->d_chain;
    P.n_chain = S->n_chain;
    P.tree_spheres = S->tree_spheres;
    std::memcpy(P.sph2, S->sph2, sizeof P.sph2);
    dim3 grid((R->width + 15) / 16, (R->height + 15) / 16), block(256);
    const bool cnt = (flags & CRT_RENDER_COUNT_WORK) != 0;
    P.regen_threshold = S->width == 4 ? R->regen_threshold_wide : R->regen_threshold;
    P.drain_threshold = R->drain_threshold > 0 ? R->drain_threshold : P.regen_threshold;
    P.wave_drain = R->wave_drain;
    if (R->tile_shards > 1) {
        // pixel sharding: variant 8 renders this shard's tiles; every other pixel of the framebuffer is 0, so the sum
        // of the shards' framebuffers (one collective) is the unsharded frame exactly (x + 0 = x).  Checked and
        // cleared before ev0, so a rejected call leaves the previous frame's timings intact and the clear is not
        // counted as probe/sort time.
        if (S->width != 4) return set_error(CRT_ERR_UNSUPPORTED, "pixel sharding needs a 4-wide rebuilt scene (variant 8)");
        if (P.accumulate) return set_error(CRT_ERR_INVALID_ARGUMENT, "pixel sharding does not accumulate");
        HIP_TRY(hipMemsetAsync(R->d_sum, 0, (size_t)R->width * R->height * 3 * sizeof(float), st));
    }
    {   // this render's slot of the timing ring: the spare slot, which no readable frame occupies (crt_renderer)
        hipEvent_t* slot = R->ring[R->n_timed % (CRT_TIMING_RING + 1)];
        R->ev0 = slot[0]; R->ev_main = slot[1]; R->ev1 = slot[2];
    }
    HIP_TRY(hipEventRecord(R->ev0, st));
#define CRT_LAUNCH(V, W)                                                                     \
    do {                                                                                     \
        std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, %d, %d>", \
                      cnt ? "true" : "false", V, W);                                         \
        HIP_TRY(hipEventRecord(R->ev_main, st));                                             \
        if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, V, W>), grid, block, 0, st, P);  \
        else hipLaunchKernelGGL((crt_render_kernel<false, V, W>), grid, block, 0, st, P);     \
    } while (0)
    // 4-wide scenes: variant 4 / 7 / 8 when selected explicitly; otherwise the measured best (profiles/r01w):
    // 8 (probe-ordered tiles, one wave per workgroup) when the render runs the cost probe, 7 (lanes refill from a
    // pixel queue) for short renders such as the 1-spp interactive frames
    int wv = R->variant;
    if (S->width == 4 && wv != 4 && wv != 7 && wv != 8) wv = probe_spp_for(R, spp) > 0 ? 8 : 7;
    // threaded scenes (the bit-exact reference BVH, rebuilt width 2): variants 0-3 and 10 when selected explicitly;
    // otherwise 10 (variant 3 over probe-ordered 8x8 tiles, one wave per workgroup; -17 %, profiles/r03s) when the
    // render runs the cost probe, else 3
    int tv = R->variant;
    if (S->width != 4 && !(tv >= 0 && tv <= 3) && tv != 10) tv = probe_spp_for(R, spp) > 0 ? 10 : 3;
    // occupancy target (waves per SIMD): variant 8 runs at 7 (72 VGPRs, 8 LDS stack entries so that 28 one-wave
    // workgroups fit a CU's LDS; -2.4 % on config C, profiles/r03aj) when its frame has at least 4 tiles per wave slot,
    // else at 6, or at 4 with the row prefetch when the cost probe shows a chain-bound frame: a frame with few tiles per
    // slot can end with its most expensive tiles' sequential sample chains (config B, 2 tiles per slot: +3.3 % at 7,
    // profiles/r03ak), and the prefetch takes the node rows' wait off every iteration of a chain (B -8 % against
    // occupancy 6, profiles/r06r-r06u; where the frame is not chain-bound the lost waves cost more: the plain Cornell box
    // at 1280x720 +15 %, 1600x900 +17 %, C +24 %; profiles/r06y).  The other 4-wide variants run at 6, threaded scenes
    // at 5.
    // Variants 10 and 3 (threaded, bit-exact) run at 6 (80 VGPRs; -8.0 % and -4.8 % against 5, profiles/r03am, r03as).
    int occ = R->min_waves ? R->min_waves : (S->width == 4 || tv == 10 || tv == 3 ? 6 : 5);
    bool auto_small = false;   // variant 8, automatic occupancy, few tiles per slot: 4 or 6 from the probe's statistics
    R->last_schedule[0] = R->last_schedule[1] = R->last_schedule[2] = R->last_schedule[3] = 0.f;
    if (!R->min_waves && S->width == 4 && (wv == 8 || R->tile_shards > 1)) {
        if (!R->n_cus) HIP_TRY(hipDeviceGetAttribute(&R->n_cus, hipDeviceAttributeMultiprocessorCount, R->device));
        const size_t tiles = (size_t)((R->width + 7) / 8) * ((R->height + 7) / 8) / (size_t)std::max(1, R->tile_shards);
        // at least 4 tiles per wave slot: occupancy 7 (throughput).  Fewer: 6, or 4 when the cost probe's tile works
        // show a chain-bound frame (decided after the sort, below; without the probe there is nothing to decide on,
        // and the tile count alone cannot tell: at 1280x720 the bunny gains 8 % at 4 and the plain Cornell box loses
        // 16 %, profiles/r06x).  (The counting kernel keeps 6: its counts do not depend on the schedule.)
        occ = tiles >= (size_t)4 * R->n_cus * 4 * 7 ? 7 : 6;
        if (occ < 7 && !cnt && probe_spp_for(R, spp) > 0) auto_small = true;
    }
    P.stack_lds = std::min(R->stack_lds, occ >= 7 ? CRT_STACK7 : occ >= 6 ? CRT_STACK6 : STACK_LDS);
    // a stack_cap override below the LDS entries must still report the entries it drops (crt_scene_options.stack_cap)
    if (S->width == 4 && S->stack_cap > 0) P.stack_lds = std::min(P.stack_lds, S->stack_cap);
    if (S->width == 4 && S->stack_cap > P.stack_lds) {
        const size_t need = (size_t)(S->stack_cap - P.stack_lds);
        if (need * R->width * R->height * 4 >= ((size_t)1 << 32))
            return set_error(CRT_ERR_INVALID_ARGUMENT, "traversal-stack overflow region would exceed 4 GiB");
        if (need > R->ovf_entries) {         // grow the overflow stack region (rarely needed)
            HIP_TRY(hipStreamSynchronize(st));
            if (R->d_ovf) (void)hipFree(R->d_ovf);
            R->d_ovf = nullptr;
            R->ovf_entries = 0;
            HIP_TRY(hipMalloc((void**)&R->d_ovf, need * R->width * R->height * 4));
            R->ovf_entries = need;
        }
        P.ovf = R->d_ovf;
    }
    if (R->tile_shards > 1) wv = 8;   // pixel sharding (checked above)
    if (S->width == 4 && wv == 8) {
        const size_t n_pix = (size_t)R->width * R->height;
        const int tiles_x = (R->width + 7) / 8, n_tiles = tiles_x * ((R->height + 7) / 8);
        if (!R->d_tile_key) {
            HIP_TRY(hipStreamSynchronize(st));
            if (!R->d_order) {
                HIP_TRY(hipMalloc((void**)&R->d_order, std::max(n_pix, (size_t)n_tiles * 64) * 4));
                HIP_TRY(hipMalloc((void**)&R->d_queue, 4));
                HIP_TRY(hipMalloc((void**)&R->d_tile_cost, n_pix * 4));
                HIP_TRY(hipMalloc((void**)&R->d_order_hist, ORDER_KEYS * 4));
                HIP_TRY(hipDeviceGetAttribute(&R->n_cus, hipDeviceAttributeMultiprocessorCount, R->device));
            }
            HIP_TRY(hipMalloc((void**)&R->d_tile_key, (size_t)n_tiles * 4));
        }
        P.tiles_x = tiles_x;
        P.order = nullptr;     // no probe: tiles in row order
        if (probe_spp_for(R, spp) > 0) {
            // cost probe (variant 4, read-only) -> per-tile key -> tiles most expensive first
            RenderParams Q = P;
            Q.spp = probe_spp_for(R, spp);
            Q.accumulate = 0;
            Q.probe_cost = R->d_tile_cost;
            // every stride-th pixel in x and y; automatic: 2 below 1000 spp, where the probe is a larger share of the
            // frame (a 250-spp rank share: probe 3.2 -> 1.2 ms, render -0.9 %; at 2000 spp the render is unchanged,
            // profiles/r04f)
            const int pst = R->probe_stride ? R->probe_stride : (spp >= 1000 ? 1 : 2);
            Q.probe_stride = pst;
            const int ps = 16 * pst;
            const dim3 pgrid((R->width + ps - 1) / ps, (R->height + ps - 1) / ps);
            if (occ >= 6) hipLaunchKernelGGL((crt_render_kernel<true, 4, 6>), pgrid, block, 0, st, Q);
            else hipLaunchKernelGGL((crt_render_kernel<true, 4, 5>), pgrid, block, 0, st, Q);
            if (auto_small) {
                if (!R->d_probe_stats) {
                    HIP_TRY(hipMalloc((void**)&R->d_probe_stats, 2 * sizeof(unsigned long long)));
                    HIP_TRY(hipHostMalloc((void**)&R->h_probe_stats, 2 * sizeof(unsigned long long)));
                }
                HIP_TRY(hipMemsetAsync(R->d_probe_stats, 0, 2 * sizeof(unsigned long long), st));
            }
            hipLaunchKernelGGL(crt_tile_cost_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st, R->d_tile_cost,
                               R->width, R->height, tiles_x, n_tiles, R->d_tile_key, R->tile_key_mode, pst,
                               auto_small ? R->d_probe_stats : nullptr);
            if (auto_small) HIP_TRY(hipMemcpyAsync(R->h_probe_stats, R->d_probe_stats, 2 * sizeof(unsigned long long),
                                                   hipMemcpyDeviceToHost, st));
            if (R->tile_key_mode == 2) {   // per-pixel costs are no longer needed: reuse them for the smoothed keys
                hipLaunchKernelGGL(crt_tile_neighbour_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st,
                                   R->d_tile_key, tiles_x, n_tiles, R->d_tile_cost);
                HIP_TRY(hipMemcpyAsync(R->d_tile_key, R->d_tile_cost, (size_t)n_tiles * 4, hipMemcpyDeviceToDevice, st));
            }
            if (R->tile_shards > 1)
                hipLaunchKernelGGL(crt_tile_shard_mask_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st,
                                   R->d_tile_key, n_tiles, R->tile_shard, R->tile_shards);
            const unsigned ob = (unsigned)((n_tiles + ORDER_ITEMS - 1) / ORDER_ITEMS);
            HIP_TRY(hipMemsetAsync(R->d_order_hist, 0, ORDER_KEYS * 4, st));
            hipLaunchKernelGGL(crt_order_hist_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scan_kernel, dim3(1), dim3(ORDER_KEYS), 0, st, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scatter_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles,
                               R->d_order_hist, R->d_order, 0u);
            // XCD regions: the per-pixel costs are dead by now, so they hold the strips' lists and the pool (9 n_tiles)
            if (R->xcd_regions && R->tile_shards == 1 && tiles_x <= 2048 && n_pix >= (size_t)9 * n_tiles)
                hipLaunchKernelGGL(crt_xcd_order_kernel, dim3(1), dim3(1024), 0, st, R->d_order, R->d_tile_key, n_tiles,
                                   tiles_x, R->d_tile_cost, R->d_tile_cost + (size_t)8 * n_tiles);
            P.order = R->d_order;
            P.crit_tiles = R->crit_tiles < 0 ? 4 * R->n_cus : R->crit_tiles;
            P.crit_threshold = R->crit_threshold;
            if (auto_small) {
                // Chain-bound or not, from the probe's tile works: rho = the largest tile's work over the mean work per
                // wave slot at occupancy 6 (this rank's share of the tiles when pixel-sharded).  rho > 1 means the most
                // expensive tile alone outlasts an even spread of the frame over the slots; above CRT_CHAIN_RHO the frame
                // runs at occupancy 4 with the row prefetch, which shortens every chain iteration (-9 %) and gives up a
                // third of the wave slots (profiles/r06x, r06y: config B rho 2.0, -7.6 %; the plain Cornell box at the
                // same size rho 0.8, +15 % at 4).  One host synchronisation after the sort.
                HIP_TRY(hipStreamSynchronize(st));
                const double mx = (double)R->h_probe_stats[0];
                const double mine = (double)R->h_probe_stats[1] / std::max(1, R->tile_shards);
                const double rho = mine > 0 ? mx * (4.0 * R->n_cus * 6) / mine : 0.0;
                if (rho > CRT_CHAIN_RHO) {
                    occ = 4;
                    P.stack_lds = std::min(R->stack_lds, STACK_LDS);
                    if (S->stack_cap > 0) P.stack_lds = std::min(P.stack_lds, S->stack_cap);
                }
                R->last_schedule[0] = (float)rho;
                R->last_schedule[2] = (float)mx;
                R->last_schedule[3] = (float)(mine / std::max(1, n_tiles / std::max(1, R->tile_shards)));
            }
        }
        if (R->tile_shards > 1 && !P.order) {   // pixel shard without the probe: this shard's tiles in row order
            hipLaunchKernelGGL(crt_shard_tiles_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st, R->d_order, n_tiles,
                               R->tile_shard, R->tile_shards);
            P.order = R->d_order;
        }
        if (P.crit_tiles > 0) P.crit_tiles = (P.crit_tiles + R->tile_shards - 1) / R->tile_shards;
        const dim3 tgrid((unsigned)((n_tiles - R->tile_shard + R->tile_shards - 1) / R->tile_shards)), tblock(64);
        R->last_schedule[1] = (float)occ;
        const char* cs = cnt ? "true" : "false";
        HIP_TRY(hipEventRecord(R->ev_main, st));
        if (occ >= 7) {
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 8, 7>", cs);
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 8, 7>), tgrid, tblock, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 8, 7>), tgrid, tblock, 0, st, P);
        } else if (occ >= 6) {
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 8, 6>", cs);
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 8, 6>), tgrid, tblock, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 8, 6>), tgrid, tblock, 0, st, P);
        } else if (occ <= 4 && !cnt) {   // with the row prefetch (profiles/r06r, r06s); the counting kernel runs at 5
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<false, 8, 4>");
            hipLaunchKernelGGL((crt_render_kernel<false, 8, 4>), tgrid, tblock, 0, st, P);
        } else {
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 8, 5>", cs);
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 8, 5>), tgrid, tblock, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 8, 5>), tgrid, tblock, 0, st, P);
        }
    } else if (S->width == 4 && wv == 7) {
        const size_t n_pix = (size_t)R->width * R->height;
        const int tiles_x = (R->width + 7) / 8, tiles_y = (R->height + 7) / 8;
        const size_t n_tile_slots = (size_t)tiles_x * tiles_y * 64;
        const size_t cap = std::max(n_pix, n_tile_slots);
        if (!R->d_order) {
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipMalloc((void**)&R->d_order, cap * 4));
            HIP_TRY(hipMalloc((void**)&R->d_queue, 4));
            HIP_TRY(hipMalloc((void**)&R->d_tile_cost, n_pix * 4));
            HIP_TRY(hipMalloc((void**)&R->d_order_hist, ORDER_KEYS * 4));
            HIP_TRY(hipDeviceGetAttribute(&R->n_cus, hipDeviceAttributeMultiprocessorCount, R->device));
        }
        if (probe_spp_for(R, spp) > 0) {
            // cost probe: variant 4 at probe_spp samples over the same RNG state, read-only: rays per pixel
            RenderParams Q = P;
            Q.spp = probe_spp_for(R, spp);
            Q.accumulate = 0;
            Q.probe_cost = R->d_tile_cost;
            if (occ >= 6) hipLaunchKernelGGL((crt_render_kernel<false, 4, 6>), grid, block, 0, st, Q);
            else hipLaunchKernelGGL((crt_render_kernel<false, 4, 5>), grid, block, 0, st, Q);
            const unsigned ob = (unsigned)((n_pix + ORDER_ITEMS - 1) / ORDER_ITEMS);
            HIP_TRY(hipMemsetAsync(R->d_order_hist, 0, ORDER_KEYS * 4, st));
            hipLaunchKernelGGL(crt_order_hist_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_cost, (int)n_pix, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scan_kernel, dim3(1), dim3(ORDER_KEYS), 0, st, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scatter_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_cost, (int)n_pix,
                               R->d_order_hist, R->d_order, 0u);
            P.n_slots = (int)n_pix;
        } else {
            const int n_tiles = tiles_x * tiles_y;
            if (R->temporal && !R->d_pix_rays) {
                HIP_TRY(hipStreamSynchronize(st));
                HIP_TRY(hipMalloc((void**)&R->d_pix_rays, n_pix * 4));
                HIP_TRY(hipMalloc((void**)&R->d_tile_order, (size_t)n_tiles * 4));
                if (!R->d_tile_key) HIP_TRY(hipMalloc((void**)&R->d_tile_key, (size_t)n_tiles * 4));
                R->pix_rays_valid = false;
            }
            if (R->temporal && R->pix_rays_valid) {
                // the interactive loop's frames repeat the last frame's cost map: its rays per pixel -> tile keys (the
                // slowest pixel, raised to 3/4 of the neighbours', as variant 8's probe keys) -> tiles most expensive
                // first, so the long paths start early and the launch does not end with them (profiles/r04i: a 1-spp
                // frame in row order spends its last 31 % draining)
                hipLaunchKernelGGL(crt_tile_cost_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st, R->d_pix_rays,
                                   R->width, R->height, tiles_x, n_tiles, R->d_tile_order, 0, 1, nullptr);
                hipLaunchKernelGGL(crt_tile_neighbour_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st,
                                   R->d_tile_order, tiles_x, n_tiles, R->d_tile_key);
                const unsigned ob = (unsigned)((n_tiles + ORDER_ITEMS - 1) / ORDER_ITEMS);
                HIP_TRY(hipMemsetAsync(R->d_order_hist, 0, ORDER_KEYS * 4, st));
                hipLaunchKernelGGL(crt_order_hist_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles, R->d_order_hist);
                hipLaunchKernelGGL(crt_order_scan_kernel, dim3(1), dim3(ORDER_KEYS), 0, st, R->d_order_hist);
                hipLaunchKernelGGL(crt_order_scatter_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles,
                                   R->d_order_hist, R->d_tile_order, 0u);
                hipLaunchKernelGGL(crt_expand_tile_order_kernel, dim3((unsigned)((n_tile_slots + 255) / 256)), dim3(256),
                                   0, st, R->d_tile_order, R->d_order, R->width, R->height, (int)n_tile_slots);
            } else {
                hipLaunchKernelGGL(crt_order_tiles_kernel, dim3((unsigned)((n_tile_slots + 255) / 256)), dim3(256), 0, st,
                                   R->d_order, R->width, R->height, (int)n_tile_slots);
            }
            P.n_slots = (int)n_tile_slots;
            if (R->temporal) {
                P.pix_rays = R->d_pix_rays;
                R->pix_rays_valid = true;
            }
        }
        HIP_TRY(hipMemsetAsync(R->d_queue, 0, 4, st));
        P.order = R->d_order;
        P.queue = R->d_queue;
        P.probe_cost = nullptr;
        const int per_cu = occ >= 7 ? 7 : occ >= 6 ? 6 : 5;        // workgroups of 4 waves resident per CU
        const int n_wg = std::max(1, std::min(R->n_cus * per_cu, (int)((n_pix + 255) / 256)));
        const dim3 pgrid(n_wg);
        HIP_TRY(hipEventRecord(R->ev_main, st));
        if (occ >= 7) {
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 7, 7>", cnt ? "true" : "false");
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 7, 7>), pgrid, block, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 7, 7>), pgrid, block, 0, st, P);
        } else if (occ >= 6) {
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 7, 6>", cnt ? "true" : "false");
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 7, 6>), pgrid, block, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 7, 6>), pgrid, block, 0, st, P);
        } else {
            std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 7, 5>", cnt ? "true" : "false");
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 7, 5>), pgrid, block, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 7, 5>), pgrid, block, 0, st, P);
        }
    } else if (S->width == 4) {
        if (occ >= 7) CRT_LAUNCH(4, 7);
        else if (occ >= 6) CRT_LAUNCH(4, 6);
        else if (occ >= 5) CRT_LAUNCH(4, 5);
        else if (occ >= 4) CRT_LAUNCH(4, 4);
        else CRT_LAUNCH(4, 1);
    }
    else if (tv == 10) {
        // variant 3's wave program (threaded BVHs, the bit-exact reference mode) scheduled like variant 8: one 8x8 tile
        // per one-wave workgroup, most expensive first by a cost probe (variant 3's counting kernel, read-only)
        const size_t n_pix = (size_t)R->width * R->height;
        const int tiles_x = (R->width + 7) / 8, n_tiles = tiles_x * ((R->height + 7) / 8);
        if (!R->d_tile_key) {
            HIP_TRY(hipStreamSynchronize(st));
            if (!R->d_order) {
                HIP_TRY(hipMalloc((void**)&R->d_order, std::max(n_pix, (size_t)n_tiles * 64) * 4));
                HIP_TRY(hipMalloc((void**)&R->d_queue, 4));
                HIP_TRY(hipMalloc((void**)&R->d_tile_cost, n_pix * 4));
                HIP_TRY(hipMalloc((void**)&R->d_order_hist, ORDER_KEYS * 4));
                HIP_TRY(hipDeviceGetAttribute(&R->n_cus, hipDeviceAttributeMultiprocessorCount, R->device));
            }
            HIP_TRY(hipMalloc((void**)&R->d_tile_key, (size_t)n_tiles * 4));
        }
        P.tiles_x = tiles_x;
        P.order = nullptr;
        if (probe_spp_for(R, spp) > 0) {
            RenderParams Q = P;
            Q.spp = probe_spp_for(R, spp);
            Q.accumulate = 0;
            Q.probe_cost = R->d_tile_cost;
            hipLaunchKernelGGL((crt_render_kernel<true, 3, 5>), grid, block, 0, st, Q);
            hipLaunchKernelGGL(crt_tile_cost_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st, R->d_tile_cost,
                               R->width, R->height, tiles_x, n_tiles, R->d_tile_key, R->tile_key_mode, 1, nullptr);
            if (R->tile_key_mode == 2) {
                hipLaunchKernelGGL(crt_tile_neighbour_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st,
                                   R->d_tile_key, tiles_x, n_tiles, R->d_tile_cost);
                HIP_TRY(hipMemcpyAsync(R->d_tile_key, R->d_tile_cost, (size_t)n_tiles * 4, hipMemcpyDeviceToDevice, st));
            }
            const unsigned ob = (unsigned)((n_tiles + ORDER_ITEMS - 1) / ORDER_ITEMS);
            HIP_TRY(hipMemsetAsync(R->d_order_hist, 0, ORDER_KEYS * 4, st));
            hipLaunchKernelGGL(crt_order_hist_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scan_kernel, dim3(1), dim3(ORDER_KEYS), 0, st, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scatter_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles,
                               R->d_order_hist, R->d_order, 0u);
            // XCD regions: the per-pixel costs are dead by now, so they hold the strips' lists and the pool (9 n_tiles)
            if (R->xcd_regions && R->tile_shards == 1 && tiles_x <= 2048 && n_pix >= (size_t)9 * n_tiles)
                hipLaunchKernelGGL(crt_xcd_order_kernel, dim3(1), dim3(1024), 0, st, R->d_order, R->d_tile_key, n_tiles,
                                   tiles_x, R->d_tile_cost, R->d_tile_cost + (size_t)8 * n_tiles);
            P.order = R->d_order;
        }
        const dim3 tgrid(n_tiles), tblock(64);
        const int w10 = occ >= 7 ? 7 : occ >= 6 ? 6 : 5;
        std::snprintf(R->kernel_name, sizeof R->kernel_name, "crt_render_kernel<%s, 10, %d>", cnt ? "true" : "false", w10);
        HIP_TRY(hipEventRecord(R->ev_main, st));
        if (w10 == 7) {
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 10, 7>), tgrid, tblock, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 10, 7>), tgrid, tblock, 0, st, P);
        } else if (w10 == 6) {
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 10, 6>), tgrid, tblock, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 10, 6>), tgrid, tblock, 0, st, P);
        } else {
            if (cnt) hipLaunchKernelGGL((crt_render_kernel<true, 10, 5>), tgrid, tblock, 0, st, P);
            else hipLaunchKernelGGL((crt_render_kernel<false, 10, 5>), tgrid, tblock, 0, st, P);
        }
    }
    else if (tv == 0) CRT_LAUNCH(0, 1);
    else if (tv == 1) CRT_LAUNCH(1, 1);
    else if (tv == 3) {
        if (occ >= 6) CRT_LAUNCH(3, 6);
        else if (occ >= 5) CRT_LAUNCH(3, 5);
        else if (occ >= 4) CRT_LAUNCH(3, 4);
        else CRT_LAUNCH(3, 1);
    }
    else if (occ >= 8) CRT_LAUNCH(2, 8);
    else if (occ >= 6) CRT_LAUNCH(2, 6);
    else if (occ >= 5) CRT_LAUNCH(2, 5);
    else CRT_LAUNCH(2, 1);
#undef CRT_LAUNCH
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(R->ev1, st));
    ++R->n_timed;
    return CRT_OK;
}

int crt_scene_compare_dump(crt_renderer* R, const crt_scene* A, const crt_scene* B, int spp, int max_bounces,
                           uint64_t out[5], float* dump, int max_dump);
int crt_scene_compare(crt_renderer* R, const crt_scene* A, const crt_scene* B, int spp, int max_bounces,
                      uint64_t out[5]) {
    return crt_scene_compare_dump(R, A, B, spp, max_bounces, out, nullptr, 0);
}

int crt_scene_compare_dump(crt_renderer* R, const crt_scene* A, const crt_scene* B, int spp, int max_bounces,
                           uint64_t out[5], float* dump, int max_dump) {
    if (!R || !A || !B || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    if (!R->has_camera) return set_error(CRT_ERR_INVALID_ARGUMENT, "camera not set");
    if (A->device != R->device || B->device != R->device)
        return set_error(CRT_ERR_INVALID_ARGUMENT, "scenes and renderer on different devices");
    if (A->n_ranks != B->n_ranks) return set_error(CRT_ERR_INVALID_ARGUMENT, "scenes hold different primitive sets");
    if (spp < 0 || max_bounces < 0) return set_error(CRT_ERR_INVALID_ARGUMENT, "negative spp / bounces");
    HIP_TRY(hipSetDevice(R->device));
    HIP_TRY(hipMemset(R->d_counters, 0, ERR_WORD * sizeof(unsigned long long)));
    CompareParams Q{};
    RenderParams& P = Q.A;
    P.nodes = A->d_nodes; P.prims = A->d_prims; P.mats = A->d_mats; P.shade = A->d_shade;
    P.n_nodes = A->n_nodes; P.n_mats = A->n_mats; P.n_prims = A->n_prims; P.n_layouts = A->layouts;
    P.err = reinterpret_cast<unsigned*>(R->d_counters + ERR_WORD);
    P.width = R->width; P.height = R->height; P.spp = spp; P.max_bounces = max_bounces;
    P.accumulate = 0; P.regen_threshold = 64; P.drain_threshold = 64; P.wave_drain = 64;
    P.rng = R->d_rng; P.sum = R->d_sum; P.counters = R->d_counters; P.cam = R->cam;
    P.rcp_w = R->rcp_w; P.rcp_h = R->rcp_h; P.fast_uv = R->fast_uv;
    P.probe_stride = 1;
    P.pix_rays = nullptr;
    Q.nodes_b = B->d_nodes; Q.prims_b = B->d_prims; Q.n_nodes_b = B->n_nodes; Q.n_layouts_b = B->layouts;
    Q.width_a = A->width; Q.width_b = B->width;
    Q.dump = nullptr;
    Q.max_dump = 0;
    float* d_dump = nullptr;
    if (dump && max_dump > 0) {
        HIP_TRY(hipMalloc((void**)&d_dump, (size_t)max_dump * 10 * sizeof(float)));
        Q.dump = d_dump;
        Q.max_dump = max_dump;
    }
    P.sphere_first = A->sphere_first; P.n_ray_spheres = A->n_ray_spheres; P.sphere_chain = A->d_chain;
    P.n_chain = A->n_chain;
    std::memcpy(P.sph2, A->sph2, sizeof P.sph2);
    Q.sphere_first_b = B->sphere_first; Q.n_spheres_b = B->n_ray_spheres; Q.chain_b = B->d_chain;
    Q.n_chain_b = B->n_chain;
    dim3 grid((R->width + 15) / 16, (R->height + 15) / 16), block(256);
    hipLaunchKernelGGL(crt_compare_kernel, grid, block, 0, 0, Q);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[8];
    HIP_TRY(hipMemcpy(h, R->d_counters, sizeof h, hipMemcpyDeviceToHost));
    for (int i = 0; i < 5; ++i) out[i] = h[i];
    if (d_dump) {
        const size_t n = std::min<size_t>((size_t)max_dump, (size_t)(h[6] & 0xffffffffu));
        hipError_t e = n ? hipMemcpy(dump, d_dump, n * 10 * sizeof(float), hipMemcpyDeviceToHost) : hipSuccess;
        (void)hipFree(d_dump);
        HIP_TRY(e);
    }
    return CRT_OK;
}

int crt_renderer_resolve(crt_renderer* R, float scale, void* stream) {
    if (!R) return set_error(CRT_ERR_INVALID_ARGUMENT, "null renderer");
    HIP_TRY(hipSetDevice(R->device));
    const int n = R->width * R->height;
    hipLaunchKernelGGL(crt_resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, R->d_sum,
                       R->d_rgba, n, scale);
    HIP_TRY(hipGetLastError());
    return CRT_OK;
}

int crt_renderer_render_frame(crt_renderer* R, const crt_scene* S, void* stream) {
    if (!R) return set_error(CRT_ERR_INVALID_ARGUMENT, "null renderer");
    if (!R->has_camera) return set_error(CRT_ERR_INVALID_ARGUMENT, "camera not set");
    if (int rc = crt_renderer_render(R, S, R->cam.samples_per_pixel, 20, 0u, stream)) return rc;
    if (int rc = crt_renderer_resolve(R, R->cam.pixel_sample_scale, stream)) return rc;
    return crt_renderer_synchronize(R, stream);
}

// The device error word (sticky across renders until read here): a render that dropped a traversal-stack entry
// or met an out-of-range primitive index produced a wrong frame.  Reported where the reference reports a kernel
// fault, at the synchronisation after the launch (CUDARenderer.cuh:59, CUDA_CHECK(cudaDeviceSynchronize())).
static int take_device_error(crt_renderer* R, unsigned long long word) {
    if (!word) return CRT_OK;
    HIP_TRY(hipMemset(R->d_counters + ERR_WORD, 0, sizeof(unsigned long long)));
    std::string m = "render kernel reported an internal error:";
    if (word & 1u) m += " primitive index out of range;";
    if (word & 2u) m += " traversal stack deeper than the scene's stack bound (entries dropped);";
    if (word & 4u) m += " leaf-round pair outside its owner's span (checked build);";
    return set_error(CRT_ERR_HIP, m + " the frame is invalid");
}

int crt_renderer_synchronize(crt_renderer* R, void* stream) {
    if (!R) return set_error(CRT_ERR_INVALID_ARGUMENT, "null renderer");
    HIP_TRY(hipSetDevice(R->device));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    unsigned long long word = 0;
    HIP_TRY(hipMemcpy(&word, R->d_counters + ERR_WORD, sizeof word, hipMemcpyDeviceToHost));
    return take_device_error(R, word);
}

static int read_dev(crt_renderer* R, void* dst, const void* src, size_t bytes) {
    if (!R || !dst) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(R->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return CRT_OK;
}
int crt_renderer_read_linear(crt_renderer* R, float* out) {
    return R ? read_dev(R, out, R->d_sum, (size_t)R->width * R->height * 12) : set_error(CRT_ERR_INVALID_ARGUMENT, "null");
}
int crt_renderer_read_rgba8(crt_renderer* R, uint8_t* out) {
    return R ? read_dev(R, out, R->d_rgba, (size_t)R->width * R->height * 4) : set_error(CRT_ERR_INVALID_ARGUMENT, "null");
}
int crt_renderer_read_rng(crt_renderer* R, uint32_t* out) {
    return R ? read_dev(R, out, R->d_rng, (size_t)R->width * R->height * 24) : set_error(CRT_ERR_INVALID_ARGUMENT, "null");
}
int crt_renderer_write_linear(crt_renderer* R, const float* in) {
    if (!R || !in) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(R->device));
    HIP_TRY(hipMemcpy(R->d_sum, in, (size_t)R->width * R->height * 12, hipMemcpyHostToDevice));
    return CRT_OK;
}
int crt_renderer_get_counters(crt_renderer* R, crt_work_counters* out) {
    if (!R || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    unsigned long long c[16];
    if (int rc = read_dev(R, c, R->d_counters, sizeof c)) return rc;
    R->diag[0] = c[5]; R->diag[1] = c[6] & ((1ull << 40) - 1); R->diag[2] = c[6] >> 40;
    for (int i = 0; i < 7; ++i) R->prof[i] = c[8 + i];
    R->prof[7] = c[7];
    out->rays = c[0]; out->box_tests = c[1]; out->tri_tests = c[2]; out->sphere_tests = c[3]; out->paths = c[4];
    return take_device_error(R, c[ERR_WORD]);
}
int crt_renderer_get_section_profile(crt_renderer* R, unsigned long long* out7) {
    if (!R || !out7) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    for (int i = 0; i < 7; ++i) out7[i] = R->prof[i];
    return CRT_OK;
}
int crt_renderer_get_section_profile_ex(crt_renderer* R, unsigned long long* out, int n) {
    if (!R || !out || n < 0) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    for (int i = 0; i < n && i < 8; ++i) out[i] = R->prof[i];
    return CRT_OK;
}
int crt_renderer_get_schedule_stats(crt_renderer* R, unsigned long long* out3) {
    if (!R || !out3) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    out3[0] = R->diag[0]; out3[1] = R->diag[1]; out3[2] = R->diag[2];
    return CRT_OK;
}

float* crt_renderer_linear_device_ptr(crt_renderer* R) { return R ? R->d_sum : nullptr; }
uint8_t* crt_renderer_rgba_device_ptr(crt_renderer* R) { return R ? R->d_rgba : nullptr; }
uint32_t* crt_renderer_rng_device_ptr(crt_renderer* R) { return R ? R->d_rng : nullptr; }

const char* crt_renderer_last_kernel_name(const crt_renderer* R) { return R ? R->kernel_name : ""; }

#ifdef CRT_PROFILE_PAIRS
extern "C" int crt_profile_pair_hist(unsigned long long* out32, int reset) {
    if (!out32) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_pair_hist), 32 * 8, 0, hipMemcpyDeviceToHost));
    if (reset) {
        static const unsigned long long zero[32] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pair_hist), zero, sizeof zero, 0, hipMemcpyHostToDevice));
    }
    return CRT_OK;
}
#endif
#ifdef CRT_PROFILE_LIVE
extern "C" int crt_profile_live_hist(unsigned long long* out16, int reset) {
    if (!out16) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_live_hist), 16 * 8, 0, hipMemcpyDeviceToHost));
    if (reset) {
        static const unsigned long long zero[16] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_live_hist), zero, sizeof zero, 0, hipMemcpyHostToDevice));
    }
    return CRT_OK;
}
#endif
#ifdef CRT_PROFILE_PASS
extern "C" int crt_profile_pass_sections(unsigned long long* out20, int reset) {
    if (!out20) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out20, HIP_SYMBOL(g_pass_prof), 20 * 8, 0, hipMemcpyDeviceToHost));
    if (reset) {
        static const unsigned long long zero[20] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pass_prof), zero, sizeof zero, 0, hipMemcpyHostToDevice));
    }
    return CRT_OK;
}
#endif
#ifdef CRT_PROFILE_LOOPS
extern "C" int crt_profile_loop_counts(unsigned long long* out8, int reset) {
    if (!out8) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_loop_prof), 8 * 8, 0, hipMemcpyDeviceToHost));
    if (reset) {
        static const unsigned long long zero[8] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_loop_prof), zero, sizeof zero, 0, hipMemcpyHostToDevice));
    }
    return CRT_OK;
}
#endif
#ifdef CRT_PROFILE_CRIT_TRACE
// out: 2 x 16384 trace words, then 2 x n_waves HW words
extern "C" int crt_profile_crit_trace(unsigned long long* trace, unsigned* hw, int n_waves) {
    if (!trace || !hw || n_waves <= 0 || n_waves > 4 * 65536) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(trace, HIP_SYMBOL(g_crit_trace), sizeof(unsigned long long) * 2 * 16384, 0,
                                hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_wave_hw), (size_t)n_waves * 8, 0, hipMemcpyDeviceToHost));
    static const unsigned long long zero[2 * 16384] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_crit_trace), zero, sizeof zero, 0, hipMemcpyHostToDevice));
    return CRT_OK;
}
#endif
#ifdef CRT_PROFILE_WAVE_TIMES
extern "C" int crt_profile_wave_times(unsigned long long* out, int n_waves) {
    if (!out || n_waves <= 0 || n_waves > 4 * 65536) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_prof), (size_t)n_waves * 16, 0, hipMemcpyDeviceToHost));
    return CRT_OK;
}
#endif

int crt_renderer_timing_history(crt_renderer* R, int back, float out[3]) {
    if (!R || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    if (back < 0 || back >= CRT_TIMING_RING) return set_error(CRT_ERR_INVALID_ARGUMENT, "back outside [0, CRT_TIMING_RING)");
    if ((unsigned long long)back >= R->n_timed) return set_error(CRT_ERR_INVALID_ARGUMENT, "fewer renders than back + 1");
    hipEvent_t* slot = R->ring[(R->n_timed - 1 - (unsigned long long)back) % (CRT_TIMING_RING + 1)];
    HIP_TRY(hipSetDevice(R->device));
    HIP_TRY(hipEventSynchronize(slot[2]));
    HIP_TRY(hipEventElapsedTime(&out[0], slot[0], slot[2]));
    HIP_TRY(hipEventElapsedTime(&out[1], slot[0], slot[1]));
    HIP_TRY(hipEventElapsedTime(&out[2], slot[1], slot[2]));
    return CRT_OK;
}

int crt_renderer_set_temporal_order(crt_renderer* R, int on) {
    if (!R || on < 0 || on > 1) return set_error(CRT_ERR_INVALID_ARGUMENT, "temporal order: 0 or 1");
    R->temporal = on;
    R->pix_rays_valid = false;
    return CRT_OK;
}

int crt_renderer_set_drain_threshold(crt_renderer* R, int lanes) {
    if (!R || lanes < 0 || lanes > 64) return set_error(CRT_ERR_INVALID_ARGUMENT, "drain threshold 0..64");
    R->drain_threshold = lanes;
    return CRT_OK;
}

int crt_renderer_set_wave_drain(crt_renderer* R, int sixty_fourths) {
    if (!R || sixty_fourths < 1 || sixty_fourths > 64) return set_error(CRT_ERR_INVALID_ARGUMENT, "wave drain 1..64");
    R->wave_drain = sixty_fourths;
    return CRT_OK;
}

int crt_renderer_set_xcd_regions(crt_renderer* R, int on) {
    if (!R || on < 0 || on > 1) return set_error(CRT_ERR_INVALID_ARGUMENT, "xcd regions: 0 or 1");
    R->xcd_regions = on;
    return CRT_OK;
}

// The round-4 leaf-pair carry was measured and not kept (+1.8 % / +15 %); its kernels live on as
// profiles/r04c/leaf_carry.patch.  The entry point stays in the ABI and reports that this build has no carry.
int crt_renderer_set_leaf_carry(crt_renderer* R, int lanes, int max_pairs) {
    if (!R) return set_error(CRT_ERR_INVALID_ARGUMENT, "null renderer");
    (void)lanes;
    (void)max_pairs;
    return set_error(CRT_ERR_UNSUPPORTED, "leaf-pair carry: not in this build (measured and removed, DESIGN.md §8; "
                                          "profiles/r04c/leaf_carry.patch)");
}

int crt_renderer_last_schedule(crt_renderer* R, float out[4]) {
    if (!R || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    for (int k = 0; k < 4; ++k) out[k] = R->last_schedule[k];
    return CRT_OK;
}

int crt_renderer_last_timings(crt_renderer* R, float out[3]) {
    if (!R || !out) return set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    if (!R->n_timed) return set_error(CRT_ERR_INVALID_ARGUMENT, "no render yet");
    return crt_renderer_timing_history(R, 0, out);
}

float crt_renderer_last_kernel_ms(crt_renderer* R) {
    float t[3];
    if (!R || !R->n_timed || crt_renderer_timing_history(R, 0, t) != CRT_OK) return -1.f;
    return t[0];
}

int crt_selftest_math(const float* a, const float* b, int n, float* out, double* out64) {
    if (!a || !b || !out || !out64 || n <= 0) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    float *da, *db, *dout;
    double* d64;
    HIP_TRY(hipMalloc((void**)&da, n * 4));
    HIP_TRY(hipMalloc((void**)&db, n * 4));
    HIP_TRY(hipMalloc((void**)&dout, n * 16));
    HIP_TRY(hipMalloc((void**)&d64, n * 16));
    HIP_TRY(hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(crt_selftest_math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, n, dout, d64);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout, n * 16, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out64, d64, n * 16, hipMemcpyDeviceToHost));
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout); (void)hipFree(d64);
    return CRT_OK;
}

int crt_selftest_rcp(uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches, uint32_t* first_bad) {
    if (!mismatches || !first_bad) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    unsigned long long* dbad;
    uint32_t* dfirst;
    HIP_TRY(hipMalloc((void**)&dbad, 8));
    HIP_TRY(hipMalloc((void**)&dfirst, 4));
    HIP_TRY(hipMemset(dbad, 0, 8));
    HIP_TRY(hipMemset(dfirst, 0xff, 4));
    hipLaunchKernelGGL(crt_selftest_rcp_kernel, dim3(8192), dim3(256), 0, 0, lo_bits, hi_bits, dbad, dfirst);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(mismatches, dbad, 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(first_bad, dfirst, 4, hipMemcpyDeviceToHost));
    (void)hipFree(dbad);
    (void)hipFree(dfirst);
    return CRT_OK;
}

int crt_selftest_sqrt(uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches, uint32_t* first_bad) {
    if (!mismatches || !first_bad) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    unsigned long long* dbad;
    uint32_t* dfirst;
    HIP_TRY(hipMalloc((void**)&dbad, 8));
    HIP_TRY(hipMalloc((void**)&dfirst, 4));
    HIP_TRY(hipMemset(dbad, 0, 8));
    HIP_TRY(hipMemset(dfirst, 0xff, 4));
    hipLaunchKernelGGL(crt_selftest_sqrt_kernel, dim3(8192), dim3(256), 0, 0, lo_bits, hi_bits, dbad, dfirst);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(mismatches, dbad, 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(first_bad, dfirst, 4, hipMemcpyDeviceToHost));
    (void)hipFree(dbad);
    (void)hipFree(dfirst);
    return CRT_OK;
}

int crt_selftest_scan(const int* in, int n_waves, int* out) {
    if (!in || !out || n_waves <= 0) return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    int *din, *dout;
    HIP_TRY(hipMalloc((void**)&din, (size_t)n_waves * 64 * 4));
    HIP_TRY(hipMalloc((void**)&dout, (size_t)n_waves * 64 * 12));
    HIP_TRY(hipMemcpy(din, in, (size_t)n_waves * 64 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(crt_selftest_scan_kernel, dim3(n_waves), dim3(64), 0, 0, din, dout, n_waves);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout, (size_t)n_waves * 64 * 12, hipMemcpyDeviceToHost));
    (void)hipFree(din);
    (void)hipFree(dout);
    return CRT_OK;
}

int crt_selftest_geometry(int kind, const float* in, int n, const crt_camera_desc* cam, int width, int height,
                          uint32_t* rng, float* out) {
    static const int in_words[5] = {17, 14, 12, 2, 12}, out_words[5] = {1, 1, 1, 6, 1};
    if (kind < 0 || kind > 4 || !in || !out || n <= 0 || (kind == 3 && (!cam || !rng || width <= 0 || height <= 0)))
        return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    float *din, *dout;
    uint32_t* drng = nullptr;
    HIP_TRY(hipMalloc((void**)&din, (size_t)n * in_words[kind] * 4));
    HIP_TRY(hipMalloc((void**)&dout, (size_t)n * out_words[kind] * 4));
    if (kind == 3) HIP_TRY(hipMalloc((void**)&drng, (size_t)n * 24));
    hipError_t e = hipMemcpy(din, in, (size_t)n * in_words[kind] * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && kind == 3) e = hipMemcpy(drng, rng, (size_t)n * 24, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        unsigned long long bad_w = 0, bad_h = 0;   // the renderer's choice for this size (crt_renderer_create)
        if (kind == 3 && (uv_div_mismatches(width, &bad_w) != CRT_OK || uv_div_mismatches(height, &bad_h) != CRT_OK))
            e = hipErrorUnknown;
        if (e == hipSuccess) {
            hipLaunchKernelGGL(crt_selftest_geometry_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, kind, din, n, dout,
                               drng, cam ? *cam : crt_camera_desc{}, width, height, kind == 3 ? 1.0f / (float)width : 1.f,
                               kind == 3 ? 1.0f / (float)height : 1.f, (int)(kind == 3 && bad_w == 0 && bad_h == 0));
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * out_words[kind] * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && kind == 3) e = hipMemcpy(rng, drng, (size_t)n * 24, hipMemcpyDeviceToHost);
    (void)hipFree(din);
    (void)hipFree(dout);
    if (drng) (void)hipFree(drng);
    HIP_TRY(e);
    return CRT_OK;
}

int crt_selftest_rng(unsigned long long seed, const unsigned long long* subseq, int n, int n_draw,
                     uint32_t* state_out, float* uniforms_out) {
    if (!subseq || !state_out || !uniforms_out || n <= 0 || n_draw < 0)
        return set_error(CRT_ERR_INVALID_ARGUMENT, "bad argument");
    if (int rc = use_device(0)) return rc;
    const auto& tab = seq_tables();
    uint32_t *dseq, *dst;
    float* du;
    HIP_TRY(hipMalloc((void**)&dseq, tab.size() * 4));
    HIP_TRY(hipMalloc((void**)&dst, (size_t)n * 24));
    HIP_TRY(hipMalloc((void**)&du, (size_t)n * std::max(n_draw, 1) * 4));
    HIP_TRY(hipMemcpy(dseq, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    for (int i = 0; i < n; ++i) {   // one launch per subsequence keeps the kernel identical to the renderer's
        hipLaunchKernelGGL(crt_init_rand_kernel, dim3(1), dim3(64), 0, 0, dst + 6 * i, dseq, 1, seed, subseq[i]);
    }
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(crt_selftest_rng_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, dst, n, n_draw, du);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(state_out, dst, (size_t)n * 24, hipMemcpyDeviceToHost));
    if (n_draw) HIP_TRY(hipMemcpy(uniforms_out, du, (size_t)n * n_draw * 4, hipMemcpyDeviceToHost));
    (void)hipFree(dseq); (void)hipFree(dst); (void)hipFree(du);
    return CRT_OK;
}

}  // extern "C"
