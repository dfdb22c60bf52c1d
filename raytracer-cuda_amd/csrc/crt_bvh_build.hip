// crt_bvh_build.hip — the reference's mesh BVH builder, GPU-parallel and order-exact.
//
// The reference builds each mesh's BVH on the device with ONE thread (Mesh::buildBVHMesh, Mesh.cuh:121-264,
// launched <<<1,1>>> by initMesh, CUDAKernels.h:28-33).  This file computes the same node array and the
// same triangle permutation in parallel, level by level, for the whole mesh at once:
//
//  * Everything the reference computes per node except the partition ORDER is a function of the node's
//    triangle SET: centroid min/max per axis, midpoints, the SAH side counts and boxes (evaluateSAH,
//    :222-240), the chosen axis/position, leaf boxes (computeTrianglesAABB, :258-264), the bottom-up
//    combine (:211-218).  These are segmented reductions (ordered-integer min/max, counts).
//  * The partition (:182-198) is a forward scan that swaps each "less" triangle to `mid`.  Its result is
//    restated exactly (tests/test_parallel_partition.py): the "less" triangles keep their order; right-block
//    position j ends up holding a[root(j)], root following j -> j - m_j (m_j = ">=" triangles before j)
//    through "less" positions.  An exclusive scan plus pointer jumping computes it.
//  * Node indices come from the processing order of the reference's explicit stack (pop, push right, push
//    left): internal node X gets children 1 + 2*rank(X) and 2 + 2*rank(X), rank = X's preorder position
//    among internal nodes, computed from subtree internal-node counts.  The stack-overflow condition of the
//    host restatement (BVHBuild.cpp) is evaluated per node from the same order.
//  * The reference's node cap `(nextNodeIndex + 1) >= maxNodes` (:148) can only fire after a split with an
//    empty side (all three SAH costs NaN; then every later split repeats it).  Such meshes return
//    CRT_ERR_UNSUPPORTED and callers use the sequential host builder.
//
// One difference is representational only: min/max here order -0 below +0 (ordered-integer atomics), while
// fminf/fmaxf in a sequential loop keep whichever zero came first.  Box bounds can then differ in the sign
// of a zero, never in value; no comparison, size or area the render path computes can tell them apart.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "crt_hip.h"

int crtx_set_error(int code, const std::string& msg);   // crt_hip.hip

namespace {

constexpr int LEAF_SPAN_TRIS = 10;   // span <= 30 indices is a leaf (Mesh.cuh:148)
constexpr int MAX_STACK_SIZE = 64;   // BVHNode.cuh:7
constexpr int RED = 48;              // reduction words per level node: cmin[3] cmax[3], then per axis & side 7
constexpr int SCAN_ITEMS = 1024;     // elements per workgroup of the exclusive scan
constexpr unsigned ERR_DEGENERATE = 1u, ERR_STACK = 2u, ERR_JUMP = 4u, ERR_INDEX = 8u;

__device__ __forceinline__ uint32_t ord(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

// AABB::padToMinimums / Interval::expand (AABB.cuh:181-186, Interval.cuh:41-44)
__device__ __forceinline__ void pad_axis(float& lo, float& hi) {
    const float delta = 0.000001f;
    if (hi - lo < delta) {
        const float p = delta / 2.f;
        lo = lo - p;
        hi = hi + p;
    }
}
// AABB::area (AABB.cuh:74-81)
__device__ __forceinline__ float box_area(const float lo[3], const float hi[3]) {
    const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
    return 2.0f * (ex * ey + ey * ez + ez * ex);
}

struct NodeOut {   // crt_bvh_node_desc
    float bmin[3], bmax[3];
    int32_t left, right, obj_index, obj_count, is_leaf;
};
static_assert(sizeof(NodeOut) == sizeof(crt_bvh_node_desc), "node layout");

// Build-time node table, indexed by creation ("tmp") id; level L's nodes are a contiguous tmp range.
struct Nodes {
    int* start;     // first triangle position
    int* count;     // triangles
    int* left;      // tmp id of the left child (right = left + 1), -1 for leaves
    float* lo;      // box, 3 per node
    float* hi;
    int* axis;
    float* pos;
    int* nless;     // triangles on the left of the split
    int* icount;    // internal nodes in the subtree (incl. itself)
    int* rank;      // preorder position among internal nodes
    int* pend;      // reference stack entries below this node when it is popped
    int* fidx;      // final (reference) node index
};

// ---- per-triangle precomputation: centroid (Mesh.cuh:251-256) and vertex bounds ----
__global__ void k_tri_prep(const float* __restrict__ v, uint32_t nv, const uint32_t* __restrict__ idx, int n,
                           float* __restrict__ cen, float* __restrict__ tlo, float* __restrict__ thi,
                           unsigned* err) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t i0 = idx[3 * (size_t)t], i1 = idx[3 * (size_t)t + 1], i2 = idx[3 * (size_t)t + 2];
    if (i0 >= nv || i1 >= nv || i2 >= nv) { atomicOr(err, ERR_INDEX); return; }
    float p[3][3];
    const uint32_t ii[3] = {i0, i1, i2};
    for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a) p[k][a] = v[3 * (size_t)ii[k] + a];
    for (int a = 0; a < 3; ++a) {
        const float s = (p[0][a] + p[1][a]) + p[2][a];      // (p0 + p1 + p2) * (1.f / 3.f)
        cen[(size_t)a * n + t] = s * (1.f / 3.f);
        tlo[(size_t)a * n + t] = fminf(fminf(p[0][a], p[1][a]), p[2][a]);
        thi[(size_t)a * n + t] = fmaxf(fmaxf(p[0][a], p[1][a]), p[2][a]);
    }
}

// Mesh ctor box: unpadded expand over every vertex slot (Mesh.cuh:39-47); box6 holds ordered ints.
__global__ void k_vertex_box(const float* __restrict__ v, uint32_t nv, uint32_t* box6) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        const float x = i < nv ? v[3 * (size_t)i + a] : 0.f;
        lo[a] = i < nv ? ord(x) : 0xffffffffu;
        hi[a] = i < nv ? ord(x) : 0u;
        lo[a] = wave_min(lo[a]);
        hi[a] = wave_max(hi[a]);
    }
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; ++a) { atomicMin(&box6[a], lo[a]); atomicMax(&box6[3 + a], hi[a]); }
}

// Root that is itself a leaf (<= 10 triangles): computeTrianglesAABB over all of them.
__global__ void k_root_leaf_box(const float* __restrict__ tlo, const float* __restrict__ thi, int n, Nodes N) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int a = 0; a < 3; ++a) {
        float lo = INFINITY, hi = -INFINITY;
        for (int t = 0; t < n; ++t) { lo = fminf(lo, tlo[(size_t)a * n + t]); hi = fmaxf(hi, thi[(size_t)a * n + t]); }
        N.lo[a] = lo;
        N.hi[a] = hi;
    }
}

// ---- level step 1: internal-node ranks of the level (single workgroup) ----
// stats: [0] internal nodes, [1] largest internal node (triangles)
__global__ __launch_bounds__(1024) void k_level_scan(Nodes N, int base, int n_lev, int* __restrict__ irank,
                                                     int* __restrict__ stats) {
    __shared__ int part[1024];
    __shared__ int smax;
    const int tid = threadIdx.x;
    if (tid == 0) smax = 0;
    const int per = (n_lev + 1023) / 1024;
    const int b = min(n_lev, tid * per), e = min(n_lev, b + per);
    int c = 0, mx = 0;
    for (int i = b; i < e; ++i) {
        const int cnt = N.count[base + i];
        if (cnt > LEAF_SPAN_TRIS) { ++c; mx = max(mx, cnt); }
    }
    part[tid] = c;
    __syncthreads();
    if (mx) atomicMax(&smax, mx);
    for (int o = 1; o < 1024; o <<= 1) {       // inclusive Hillis-Steele scan
        const int add = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    int r = part[tid] - c;
    for (int i = b; i < e; ++i) irank[i] = N.count[base + i] > LEAF_SPAN_TRIS ? r++ : -1;
    if (tid == 1023) { stats[0] = part[1023]; stats[1] = smax; }
}

__global__ void k_level_reset(uint32_t* __restrict__ red, int n_lev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_lev * RED) return;
    const int w = i % RED;
    uint32_t v;
    if (w < 3) v = ord(1e30f);                          // minPos = 1e30f (Mesh.cuh:166)
    else if (w < 6) v = ord(-1e30f);                    // maxPos = -1e30f
    else {
        const int k = (w - 6) % 7;                      // count, lo[3], hi[3] of an AABB_EMPTY side box
        v = k == 0 ? 0u : k < 4 ? ord(INFINITY) : ord(-INFINITY);
    }
    red[i] = v;
}

// The lane's level node (local index) and whether the wave holds a single node.
struct LaneSeg {
    int s;          // level-local node index, -1 = not in an internal node of this level
    bool uniform;   // every lane with s >= 0 has the same s (and at least one has)
    int s0;
};

// Steps 2 and 3 run per workgroup chunk of LEVEL_CHUNK positions, and only over the level's big nodes (more than
// LEVEL_SMALL triangles).  A node's triangles occupy one contiguous range of positions, so a chunk whose first and last
// positions belong to one node holds that node only (the top levels): it reduces in registers and LDS and adds its
// result with one global atomic per word, where every wave used to (1M triangles: 16k waves on one node's 48 words).
// Nodes of at most LEVEL_SMALL triangles (the deep levels) are reduced by one thread each from their triangles
// (k_level_small), without atomics.  Min, max and add are order-independent: the same words, the same tree.
constexpr int LEVEL_CHUNK = 4096;
constexpr int LEVEL_SMALL = 32;

// The lane's big level node (local index) or -1, and whether the wave holds a single one.
__device__ __forceinline__ LaneSeg lane_seg_big(const int* __restrict__ seg, int p, int n, const Nodes& N, int base) {
    LaneSeg L;
    const int s = p < n ? seg[p] : -1;
    L.s = s >= 0 && N.count[base + s] > LEVEL_SMALL ? s : -1;
    const int hi = wave_max_i(L.s);
    const int lo = wave_min_i(L.s >= 0 ? L.s : 0x7fffffff);
    L.uniform = hi >= 0 && lo == hi;
    L.s0 = hi;
    return L;
}

// block-wide min / max / add of K words per thread into part[K] (thread 0..K-1 then hold the results); op[k]: 0 add,
// 1 min, 2 max
template <int K>
__device__ __forceinline__ uint32_t block_reduce(uint32_t (&v)[K], const int (&op)[K], uint32_t (*part)[K], int k) {
    const int w = threadIdx.x >> 6;
    for (int q = 0; q < K; ++q) {
        uint32_t r = v[q];
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t x = (uint32_t)__shfl_xor((int)r, o, 64);
            r = op[q] == 0 ? r + x : op[q] == 1 ? min(r, x) : max(r, x);
        }
        if ((threadIdx.x & 63) == 0) part[w][q] = r;
    }
    __syncthreads();
    uint32_t r = 0;
    if (k < K) {
        r = part[0][k];
        for (int q = 1; q < 4; ++q) r = op[k] == 0 ? r + part[q][k] : op[k] == 1 ? min(r, part[q][k]) : max(r, part[q][k]);
    }
    return r;
}

// ---- level step 2: centroid bounds per node (Mesh.cuh:164-172) ----
__global__ __launch_bounds__(256) void k_level_bounds(const int* __restrict__ seg, const uint32_t* __restrict__ perm,
                                                      const float* __restrict__ cen, int n, Nodes N, int base,
                                                      uint32_t* __restrict__ red) {
    __shared__ uint32_t part[4][6];
    const int p0 = blockIdx.x * LEVEL_CHUNK, p1 = min(n, p0 + LEVEL_CHUNK);
    const int s_first = seg[p0];
    if (s_first >= 0 && seg[p1 - 1] == s_first && N.count[base + s_first] > LEVEL_SMALL) {   // one big node
        uint32_t v[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
        const int op[6] = {1, 1, 1, 2, 2, 2};
        for (int p = p0 + (int)threadIdx.x; p < p1; p += 256) {
            const uint32_t t = perm[p];
            for (int a = 0; a < 3; ++a) {
                const uint32_t c = ord(cen[(size_t)a * n + t]);
                v[a] = min(v[a], c);
                v[3 + a] = max(v[3 + a], c);
            }
        }
        const int k = threadIdx.x;
        const uint32_t r = block_reduce<6>(v, op, part, k);
        if (k < 3) atomicMin(&red[s_first * RED + k], r);
        else if (k < 6) atomicMax(&red[s_first * RED + k], r);
        return;
    }
    for (int q = p0; q < p1; q += 256) {
        const int p = q + (int)threadIdx.x;
        const LaneSeg L = lane_seg_big(seg, p, p1, N, base);
        if (L.s0 < 0) continue;   // whole wave idle
        const uint32_t t = L.s >= 0 ? perm[p] : 0;
        uint32_t c[3];
        for (int a = 0; a < 3; ++a) c[a] = L.s >= 0 ? ord(cen[(size_t)a * n + t]) : 0;
        if (L.uniform) {
            for (int a = 0; a < 3; ++a) {
                const uint32_t mn = wave_min(L.s >= 0 ? c[a] : 0xffffffffu);
                const uint32_t mx = wave_max(L.s >= 0 ? c[a] : 0u);
                if ((threadIdx.x & 63) == 0) {
                    atomicMin(&red[L.s0 * RED + a], mn);
                    atomicMax(&red[L.s0 * RED + 3 + a], mx);
                }
            }
        } else if (L.s >= 0) {
            for (int a = 0; a < 3; ++a) {
                atomicMin(&red[L.s * RED + a], c[a]);
                atomicMax(&red[L.s * RED + 3 + a], c[a]);
            }
        }
    }
}

__device__ __forceinline__ float node_mid(const uint32_t* __restrict__ r, int a) {
    return 0.5f * (unord(r[a]) + unord(r[3 + a]));   // midPos = 0.5f * (minPos + maxPos) (Mesh.cuh:172)
}

// ---- level step 3: SAH side counts and boxes for the three candidate splits (evaluateSAH) ----
__global__ __launch_bounds__(256) void k_level_sah(const int* __restrict__ seg, const uint32_t* __restrict__ perm,
                                                   const float* __restrict__ cen, const float* __restrict__ tlo,
                                                   const float* __restrict__ thi, int n, Nodes N, int base,
                                                   uint32_t* __restrict__ red) {
    __shared__ uint32_t part[4][42];
    const int p0 = blockIdx.x * LEVEL_CHUNK, p1 = min(n, p0 + LEVEL_CHUNK);
    const int s_first = seg[p0];
    if (s_first >= 0 && seg[p1 - 1] == s_first && N.count[base + s_first] > LEVEL_SMALL) {   // one big node
        uint32_t v[42];   // per axis and side: count, lo[3], hi[3]
        int op[42];
        for (int q = 0; q < 42; ++q) {
            const int k = q % 7;
            v[q] = k == 0 ? 0u : k < 4 ? 0xffffffffu : 0u;
            op[q] = k == 0 ? 0 : k < 4 ? 1 : 2;
        }
        float mid[3];
        for (int a = 0; a < 3; ++a) mid[a] = node_mid(red + (size_t)s_first * RED, a);
        for (int p = p0 + (int)threadIdx.x; p < p1; p += 256) {
            const uint32_t t = perm[p];
            uint32_t lo[3], hi[3];
            for (int k = 0; k < 3; ++k) { lo[k] = ord(tlo[(size_t)k * n + t]); hi[k] = ord(thi[(size_t)k * n + t]); }
            for (int a = 0; a < 3; ++a) {
                const int side = cen[(size_t)a * n + t] < mid[a] ? 0 : 1;   // 0 = left (c[axis] < pos)
                for (int sd = 0; sd < 2; ++sd) {   // unrolled selects: v stays in registers
                    uint32_t* o = v + (a * 2 + sd) * 7;
                    const bool in = side == sd;
                    o[0] += in ? 1u : 0u;
                    for (int k = 0; k < 3; ++k) {
                        o[1 + k] = in ? min(o[1 + k], lo[k]) : o[1 + k];
                        o[4 + k] = in ? max(o[4 + k], hi[k]) : o[4 + k];
                    }
                }
            }
        }
        const int k = threadIdx.x;
        const uint32_t r = block_reduce<42>(v, op, part, k);
        if (k < 42) {
            uint32_t* o = red + (size_t)s_first * RED + 6 + k;
            const int w = k % 7;
            if (w == 0) { if (r) atomicAdd(o, r); }
            else if (w < 4) atomicMin(o, r);
            else atomicMax(o, r);
        }
        return;
    }
    for (int q = p0; q < p1; q += 256) {
        const int p = q + (int)threadIdx.x;
        const LaneSeg L = lane_seg_big(seg, p, p1, N, base);
        if (L.s0 < 0) continue;
        const bool act = L.s >= 0;
        const uint32_t t = act ? perm[p] : 0;
        const int me = act ? L.s : L.s0;
        uint32_t lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = act ? ord(tlo[(size_t)a * n + t]) : 0xffffffffu;
            hi[a] = act ? ord(thi[(size_t)a * n + t]) : 0u;
        }
        for (int a = 0; a < 3; ++a) {
            const float mid = node_mid(red + (size_t)me * RED, a);
            const int side = act ? (cen[(size_t)a * n + t] < mid ? 0 : 1) : -1;   // 0 = left (c[axis] < pos)
            if (L.uniform) {
                for (int sd = 0; sd < 2; ++sd) {
                    const bool in = side == sd;
                    const uint64_t bal = __ballot(in);
                    if (!bal) continue;
                    uint32_t r[6];
                    for (int k = 0; k < 3; ++k) {
                        r[k] = wave_min(in ? lo[k] : 0xffffffffu);
                        r[3 + k] = wave_max(in ? hi[k] : 0u);
                    }
                    if ((threadIdx.x & 63) == 0) {
                        uint32_t* o = red + (size_t)L.s0 * RED + 6 + (a * 2 + sd) * 7;
                        atomicAdd(&o[0], (uint32_t)__popcll(bal));
                        for (int k = 0; k < 3; ++k) { atomicMin(&o[1 + k], r[k]); atomicMax(&o[4 + k], r[3 + k]); }
                    }
                }
            } else if (act) {
                uint32_t* o = red + (size_t)L.s * RED + 6 + (a * 2 + side) * 7;
                atomicAdd(&o[0], 1u);
                for (int k = 0; k < 3; ++k) { atomicMin(&o[1 + k], lo[k]); atomicMax(&o[4 + k], hi[k]); }
            }
        }
    }
}

// Steps 2 and 3 for the level's small internal nodes (LEVEL_SMALL triangles or fewer), one thread each: the words the
// atomics of k_level_bounds / k_level_sah would leave, from the reset values (k_level_reset) and the same ord() minima,
// maxima and counts.
__global__ void k_level_small(Nodes N, int base, int n_lev, const int* __restrict__ irank, const uint32_t* __restrict__ perm,
                              const float* __restrict__ cen, const float* __restrict__ tlo, const float* __restrict__ thi,
                              int n, uint32_t* __restrict__ red) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lev || irank[li] < 0) return;
    const int X = base + li, count = N.count[X], start = N.start[X];
    if (count > LEVEL_SMALL) return;
    uint32_t* r = red + (size_t)li * RED;
    uint32_t cmin[3], cmax[3];
    for (int a = 0; a < 3; ++a) { cmin[a] = r[a]; cmax[a] = r[3 + a]; }   // ord(1e30f), ord(-1e30f)
    for (int k = 0; k < count; ++k) {
        const uint32_t t = perm[start + k];
        for (int a = 0; a < 3; ++a) {
            const uint32_t c = ord(cen[(size_t)a * n + t]);
            cmin[a] = min(cmin[a], c);
            cmax[a] = max(cmax[a], c);
        }
    }
    for (int a = 0; a < 3; ++a) { r[a] = cmin[a]; r[3 + a] = cmax[a]; }
    for (int a = 0; a < 3; ++a) {
        const float mid = node_mid(r, a);
        uint32_t o[2][7];
        for (int sd = 0; sd < 2; ++sd)
            for (int k = 0; k < 7; ++k) o[sd][k] = r[6 + (a * 2 + sd) * 7 + k];
        for (int k = 0; k < count; ++k) {
            const uint32_t t = perm[start + k];
            const int sd = cen[(size_t)a * n + t] < mid ? 0 : 1;
            o[sd][0] += 1u;
            for (int q = 0; q < 3; ++q) {
                o[sd][1 + q] = min(o[sd][1 + q], ord(tlo[(size_t)q * n + t]));
                o[sd][4 + q] = max(o[sd][4 + q], ord(thi[(size_t)q * n + t]));
            }
        }
        for (int sd = 0; sd < 2; ++sd)
            for (int k = 0; k < 7; ++k) r[6 + (a * 2 + sd) * 7 + k] = o[sd][k];
    }
}

// ---- level step 4: choose the split (Mesh.cuh:160-179) and create the children ----
__global__ void k_level_decide(Nodes N, int base, int n_lev, const int* __restrict__ irank,
                               const uint32_t* __restrict__ red, int next_base, unsigned* err) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lev) return;
    const int X = base + li;
    if (irank[li] < 0) { N.left[X] = -1; return; }   // leaf
    const uint32_t* r = red + (size_t)li * RED;
    int bestAxis = 0;
    float bestPos = 0.f, bestCost = 1e30f;
    int lcount[3];
    for (int a = 0; a < 3; ++a) {
        const float mid = node_mid(r, a);
        float blo[2][3], bhi[2][3];
        int cnt[2];
        for (int sd = 0; sd < 2; ++sd) {
            const uint32_t* o = r + 6 + (a * 2 + sd) * 7;
            cnt[sd] = (int)o[0];
            for (int k = 0; k < 3; ++k) { blo[sd][k] = unord(o[1 + k]); bhi[sd][k] = unord(o[4 + k]); }
        }
        float cost = cnt[0] * box_area(blo[0], bhi[0]) + cnt[1] * box_area(blo[1], bhi[1]);
        cost = cost < 1e-8f ? 1e-8f : cost;
        lcount[a] = cnt[0];
        if (cost < bestCost) { bestCost = cost; bestAxis = a; bestPos = mid; }
    }
    const int n = N.count[X], l = lcount[bestAxis];
    if (l == 0 || l == n) atomicOr(err, ERR_DEGENERATE);   // the node cap would take over (see header)
    N.axis[X] = bestAxis;
    N.pos[X] = bestPos;
    N.nless[X] = l;
    const int cl = next_base + 2 * irank[li];
    N.left[X] = cl;
    const int st = N.start[X];
    const int cs[2] = {st, st + l}, cc[2] = {l, n - l};
    const uint32_t* ob = r + 6 + (bestAxis * 2) * 7;
    for (int sd = 0; sd < 2; ++sd) {
        const int c = cl + sd;
        N.start[c] = cs[sd];
        N.count[c] = cc[sd];
        N.left[c] = -1;
        for (int k = 0; k < 3; ++k) {   // exact for leaves (computeTrianglesAABB); internal boxes are refit later
            N.lo[3 * (size_t)c + k] = unord(ob[sd * 7 + 1 + k]);
            N.hi[3 * (size_t)c + k] = unord(ob[sd * 7 + 4 + k]);
        }
    }
}

// ---- level step 5: partition flags (c[bestAxis] < bestPos, Mesh.cuh:185) ----
__global__ void k_level_flags(const int* __restrict__ seg, const uint32_t* __restrict__ perm,
                              const float* __restrict__ cen, int n, Nodes N, int base, uint32_t* __restrict__ flags) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    uint32_t f = 0;
    if (s >= 0) {
        const int X = base + s;
        f = cen[(size_t)N.axis[X] * n + perm[p]] < N.pos[X] ? 1u : 0u;
    }
    flags[p] = f;
}

// ---- exclusive scan of flags (3 passes) ----
__global__ __launch_bounds__(256) void k_scan_blocks(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                     uint32_t* __restrict__ bsum, int n) {
    __shared__ uint32_t part[256];
    const int tid = threadIdx.x;
    const size_t b0 = (size_t)blockIdx.x * SCAN_ITEMS + 4 * tid;
    uint32_t v[4], s = 0;
    for (int k = 0; k < 4; ++k) { v[k] = b0 + k < (size_t)n ? in[b0 + k] : 0u; s += v[k]; }
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const uint32_t add = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    uint32_t run = part[tid] - s;
    for (int k = 0; k < 4; ++k) {
        if (b0 + k < (size_t)n) out[b0 + k] = run;
        run += v[k];
    }
    if (tid == 255) bsum[blockIdx.x] = part[255];
}
__global__ __launch_bounds__(1024) void k_scan_top(uint32_t* __restrict__ bsum, int nb) {
    __shared__ uint32_t part[1024];
    const int tid = threadIdx.x, per = (nb + 1023) / 1024;
    const int b = min(nb, tid * per), e = min(nb, b + per);
    uint32_t s = 0;
    for (int i = b; i < e; ++i) s += bsum[i];
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t add = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    uint32_t run = part[tid] - s;
    for (int i = b; i < e; ++i) { const uint32_t x = bsum[i]; bsum[i] = run; run += x; }
}
__global__ void k_scan_add(uint32_t* __restrict__ out, const uint32_t* __restrict__ bsum, int n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (size_t)n) out[i] += bsum[i / SCAN_ITEMS];
}

// ---- level step 6: right-block sources, then pointer jumping (see header) ----
__global__ void k_level_ptr(const int* __restrict__ seg, const uint32_t* __restrict__ flags,
                            const uint32_t* __restrict__ lb, int n, Nodes N, int base, int* __restrict__ ptr) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    int q = p;
    if (s >= 0 && flags[p]) {
        const int st = N.start[base + s];
        const int ge_before = (p - st) - (int)(lb[p] - lb[st]);
        if (ge_before > 0) q = p - ge_before;   // the queue front this "less" triangle's swap moves to p
    }
    ptr[p] = q;
}
__global__ void k_level_jump(const int* __restrict__ seg, const int* __restrict__ src, int* __restrict__ dst, int n) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int q = src[p];
    dst[p] = seg[p] >= 0 ? src[q] : q;
}

// ---- level step 7: scatter the new order, next level's node of every position ----
__global__ void k_level_scatter(const int* __restrict__ seg, const uint32_t* __restrict__ flags,
                                const uint32_t* __restrict__ lb, const int* __restrict__ ptr,
                                const uint32_t* __restrict__ perm, uint32_t* __restrict__ perm2,
                                int* __restrict__ seg2, int n, Nodes N, int base, int next_base,
                                unsigned* err) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    if (s < 0) { perm2[p] = perm[p]; seg2[p] = -1; return; }
    const int X = base + s;
    const int st = N.start[X], i = p - st, l = N.nless[X];
    if (flags[p]) perm2[st + (int)(lb[p] - lb[st])] = perm[p];   // stable left block
    if (i >= l) {
        const int r = ptr[p];
        if (flags[r]) atomicOr(err, ERR_JUMP);                   // a root is always a ">=" position
        perm2[p] = perm[r];
    }
    const int c = N.left[X] + (i < l ? 0 : 1);
    seg2[p] = N.count[c] > LEAF_SPAN_TRIS ? c - next_base : -1;
}

// ---- final passes over the levels ----
__global__ void k_icount(Nodes N, int b, int e) {
    const int t = b + blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= e) return;
    const int l = N.left[t];
    N.icount[t] = l < 0 ? 0 : 1 + N.icount[l] + N.icount[l + 1];
}
__global__ void k_rank(Nodes N, int b, int e, unsigned* err) {
    const int t = b + blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= e) return;
    const int l = N.left[t];
    if (l < 0) return;
    const int r = N.rank[t], pd = N.pend[t];
    if (pd + 2 > MAX_STACK_SIZE) atomicOr(err, ERR_STACK);   // BVHBuild.cpp's reference-stack check
    N.rank[l] = r + 1;
    N.pend[l] = pd + 1;
    N.rank[l + 1] = r + 1 + N.icount[l];
    N.pend[l + 1] = pd;
    N.fidx[l] = 1 + 2 * r;
    N.fidx[l + 1] = 2 + 2 * r;
}
// AABB::combine (AABB.cuh:91-98): min/max, then padToMinimums
__global__ void k_refit(Nodes N, int b, int e) {
    const int t = b + blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= e) return;
    const int l = N.left[t];
    if (l < 0) return;
    for (int k = 0; k < 3; ++k) {
        float lo = fminf(N.lo[3 * (size_t)l + k], N.lo[3 * (size_t)(l + 1) + k]);
        float hi = fmaxf(N.hi[3 * (size_t)l + k], N.hi[3 * (size_t)(l + 1) + k]);
        pad_axis(lo, hi);
        N.lo[3 * (size_t)t + k] = lo;
        N.hi[3 * (size_t)t + k] = hi;
    }
}
__global__ void k_emit(Nodes N, int total, uint32_t index_count, NodeOut* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    NodeOut o;
    for (int k = 0; k < 3; ++k) { o.bmin[k] = N.lo[3 * (size_t)t + k]; o.bmax[k] = N.hi[3 * (size_t)t + k]; }
    const int l = N.left[t];
    if (l < 0) {                                    // Mesh.cuh:149-154 (indices, not triangles)
        o.left = o.right = 0;
        o.obj_index = 3 * N.start[t];
        o.obj_count = 3 * N.count[t];
        o.is_leaf = 1;
    } else {
        o.left = N.fidx[l];
        o.right = N.fidx[l + 1];
        o.obj_index = 0;                            // root: 0 / m_IndexCount (:134-135); others zeroed
        o.obj_count = t == 0 ? (int)index_count : 0;
        o.is_leaf = 0;
    }
    out[N.fidx[t]] = o;
}
__global__ void k_permute(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ idx_in,
                          const int32_t* __restrict__ fm_in, uint32_t* __restrict__ idx_out,
                          int32_t* __restrict__ fm_out, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t t = perm[k];
    for (int c = 0; c < 3; ++c) idx_out[3 * (size_t)k + c] = idx_in[3 * (size_t)t + c];
    fm_out[k] = fm_in[t];
}
__global__ void k_iota(uint32_t* __restrict__ perm, int* __restrict__ seg, int n) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) { perm[p] = (uint32_t)p; seg[p] = 0; }
}

inline unsigned blocks(size_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

// RAII for the build's device allocations
struct DeviceArena {
    std::vector<void*> ptrs;
    ~DeviceArena() { for (void* p : ptrs) (void)hipFree(p); }
    template <class T>
    hipError_t alloc(T** p, size_t count) {
        hipError_t e = hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
    }
};

#define BTRY(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return crtx_set_error(CRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

extern "C" int crt_build_mesh_bvh(int device, const float* positions, uint32_t vertex_count, uint32_t* indices,
                                  int32_t* face_materials, uint32_t index_count, crt_bvh_node_desc* nodes,
                                  int32_t* node_count, float mesh_box[6], float* build_ms) {
    if (!node_count || !mesh_box || (vertex_count && !positions) || (index_count && (!indices || !face_materials)))
        return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "null argument");
    if (index_count % 3 != 0)
        return crtx_set_error(CRT_ERR_UNSUPPORTED, "index count is not a multiple of 3: use the host builder");
    const int n = (int)(index_count / 3);
    if ((uint64_t)index_count >= (1ull << 31)) return crtx_set_error(CRT_ERR_UNSUPPORTED, "mesh too large");
    if (n > 0 && !nodes) return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "null nodes");
    int ndev = 0;
    BTRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "device ordinal out of range");
    BTRY(hipSetDevice(device));
    DeviceArena A;
    hipStream_t st = nullptr;
    hipEvent_t e0, e1;
    BTRY(hipEventCreate(&e0));
    BTRY(hipEventCreate(&e1));
    struct EvGuard { hipEvent_t a, b; ~EvGuard() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); } } evg{e0, e1};

    // Mesh ctor box (unpadded expand over every slot; AABB() when there are none)
    float* d_v = nullptr;
    BTRY(A.alloc(&d_v, (size_t)vertex_count * 3));
    if (vertex_count) BTRY(hipMemcpy(d_v, positions, (size_t)vertex_count * 12, hipMemcpyHostToDevice));
    uint32_t* d_box6 = nullptr;
    BTRY(A.alloc(&d_box6, 6));
    BTRY(hipEventRecord(e0, st));
    {
        const uint32_t init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
        BTRY(hipMemcpyAsync(d_box6, init, sizeof init, hipMemcpyHostToDevice, st));
        if (vertex_count) hipLaunchKernelGGL(k_vertex_box, dim3(blocks(vertex_count)), dim3(256), 0, st, d_v, vertex_count, d_box6);
    }
    if (n == 0) {   // no triangles: no BVH (BVHBuild.cpp does the same)
        uint32_t b6[6];
        BTRY(hipMemcpy(b6, d_box6, sizeof b6, hipMemcpyDeviceToHost));
        for (int k = 0; k < 6; ++k) {
            uint32_t o = b6[k];
            mesh_box[k] = vertex_count ? (float)__builtin_bit_cast(float, (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o)
                                       : (k < 3 ? INFINITY : -INFINITY);
        }
        *node_count = 0;
        if (build_ms) *build_ms = 0.f;
        return CRT_OK;
    }

    uint32_t *d_idx = nullptr, *d_idx_out = nullptr;
    int32_t *d_fm = nullptr, *d_fm_out = nullptr;
    float *d_cen = nullptr, *d_tlo = nullptr, *d_thi = nullptr;
    uint32_t *d_perm = nullptr, *d_perm2 = nullptr, *d_flags = nullptr, *d_lb = nullptr, *d_bsum = nullptr, *d_red = nullptr;
    int *d_seg = nullptr, *d_seg2 = nullptr, *d_ptr = nullptr, *d_ptr2 = nullptr, *d_irank = nullptr, *d_stats = nullptr;
    unsigned* d_err = nullptr;
    const size_t cap = 2 * (size_t)n + 2;                           // total nodes <= 2n - 1
    const size_t lev_cap = 2 * ((size_t)n / (LEAF_SPAN_TRIS + 1)) + 2;   // nodes of one level
    const int nb = (int)((n + SCAN_ITEMS - 1) / SCAN_ITEMS);
    BTRY(A.alloc(&d_idx, 3 * (size_t)n));
    BTRY(A.alloc(&d_idx_out, 3 * (size_t)n));
    BTRY(A.alloc(&d_fm, n));
    BTRY(A.alloc(&d_fm_out, n));
    BTRY(A.alloc(&d_cen, 3 * (size_t)n));
    BTRY(A.alloc(&d_tlo, 3 * (size_t)n));
    BTRY(A.alloc(&d_thi, 3 * (size_t)n));
    BTRY(A.alloc(&d_perm, n));
    BTRY(A.alloc(&d_perm2, n));
    BTRY(A.alloc(&d_flags, n));
    BTRY(A.alloc(&d_lb, n));
    BTRY(A.alloc(&d_bsum, nb));
    BTRY(A.alloc(&d_seg, n));
    BTRY(A.alloc(&d_seg2, n));
    BTRY(A.alloc(&d_ptr, n));
    BTRY(A.alloc(&d_ptr2, n));
    BTRY(A.alloc(&d_red, lev_cap * RED));
    BTRY(A.alloc(&d_irank, lev_cap));
    BTRY(A.alloc(&d_stats, 2));
    BTRY(A.alloc(&d_err, 1));
    Nodes N;
    BTRY(A.alloc(&N.start, cap));
    BTRY(A.alloc(&N.count, cap));
    BTRY(A.alloc(&N.left, cap));
    BTRY(A.alloc(&N.lo, 3 * cap));
    BTRY(A.alloc(&N.hi, 3 * cap));
    BTRY(A.alloc(&N.axis, cap));
    BTRY(A.alloc(&N.pos, cap));
    BTRY(A.alloc(&N.nless, cap));
    BTRY(A.alloc(&N.icount, cap));
    BTRY(A.alloc(&N.rank, cap));
    BTRY(A.alloc(&N.pend, cap));
    BTRY(A.alloc(&N.fidx, cap));
    NodeOut* d_out = nullptr;
    BTRY(A.alloc(&d_out, cap));

    BTRY(hipMemcpyAsync(d_idx, indices, 12 * (size_t)n, hipMemcpyHostToDevice, st));
    BTRY(hipMemcpyAsync(d_fm, face_materials, 4 * (size_t)n, hipMemcpyHostToDevice, st));
    BTRY(hipMemsetAsync(d_err, 0, 4, st));
    hipLaunchKernelGGL(k_tri_prep, dim3(blocks(n)), dim3(256), 0, st, d_v, vertex_count, d_idx, n, d_cen, d_tlo, d_thi, d_err);
    hipLaunchKernelGGL(k_iota, dim3(blocks(n)), dim3(256), 0, st, d_perm, d_seg, n);
    {   // root (Mesh.cuh:132-138)
        const int zero = 0, one = 1;
        BTRY(hipMemcpyAsync(N.start, &zero, 4, hipMemcpyHostToDevice, st));
        BTRY(hipMemcpyAsync(N.count, &n, 4, hipMemcpyHostToDevice, st));
        BTRY(hipMemsetAsync(N.left, 0xff, 4, st));
        BTRY(hipMemcpyAsync(N.rank, &zero, 4, hipMemcpyHostToDevice, st));
        BTRY(hipMemcpyAsync(N.pend, &zero, 4, hipMemcpyHostToDevice, st));
        BTRY(hipMemcpyAsync(N.fidx, &zero, 4, hipMemcpyHostToDevice, st));
        (void)one;
    }
    if (n <= LEAF_SPAN_TRIS) hipLaunchKernelGGL(k_root_leaf_box, dim3(1), dim3(64), 0, st, d_tlo, d_thi, n, N);

    std::vector<int> level_off = {0, 1};   // level L = tmp ids [level_off[L], level_off[L+1])
    int stats[2];
    unsigned err = 0;
    for (;;) {
        const int base = level_off[level_off.size() - 2], n_lev = level_off.back() - base;
        hipLaunchKernelGGL(k_level_scan, dim3(1), dim3(1024), 0, st, N, base, n_lev, d_irank, d_stats);
        BTRY(hipMemcpyAsync(stats, d_stats, sizeof stats, hipMemcpyDeviceToHost, st));
        BTRY(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
        BTRY(hipStreamSynchronize(st));
        const int n_int = stats[0], maxc = stats[1];
        if (n_int == 0 || err) break;   // done, or a degenerate split / bad index: reported below
        const int next_base = level_off.back();
        hipLaunchKernelGGL(k_level_reset, dim3(blocks((size_t)n_lev * RED)), dim3(256), 0, st, d_red, n_lev);
        const int lchunks = (n + LEVEL_CHUNK - 1) / LEVEL_CHUNK;
        hipLaunchKernelGGL(k_level_bounds, dim3(lchunks), dim3(256), 0, st, d_seg, d_perm, d_cen, n, N, base, d_red);
        hipLaunchKernelGGL(k_level_sah, dim3(lchunks), dim3(256), 0, st, d_seg, d_perm, d_cen, d_tlo, d_thi, n, N, base,
                           d_red);
        hipLaunchKernelGGL(k_level_small, dim3(blocks(n_lev)), dim3(256), 0, st, N, base, n_lev, d_irank, d_perm, d_cen,
                           d_tlo, d_thi, n, d_red);
        hipLaunchKernelGGL(k_level_decide, dim3(blocks(n_lev)), dim3(256), 0, st, N, base, n_lev, d_irank, d_red,
                           next_base, d_err);
        hipLaunchKernelGGL(k_level_flags, dim3(blocks(n)), dim3(256), 0, st, d_seg, d_perm, d_cen, n, N, base, d_flags);
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, d_flags, d_lb, d_bsum, n);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, st, d_bsum, nb);
        hipLaunchKernelGGL(k_scan_add, dim3(blocks(n)), dim3(256), 0, st, d_lb, d_bsum, n);
        hipLaunchKernelGGL(k_level_ptr, dim3(blocks(n)), dim3(256), 0, st, d_seg, d_flags, d_lb, n, N, base, d_ptr);
        int rounds = 1;
        while ((1 << rounds) < maxc) ++rounds;
        for (int k = 0; k < rounds; ++k) {
            hipLaunchKernelGGL(k_level_jump, dim3(blocks(n)), dim3(256), 0, st, d_seg, d_ptr, d_ptr2, n);
            std::swap(d_ptr, d_ptr2);
        }
        hipLaunchKernelGGL(k_level_scatter, dim3(blocks(n)), dim3(256), 0, st, d_seg, d_flags, d_lb, d_ptr, d_perm,
                           d_perm2, d_seg2, n, N, base, next_base, d_err);
        std::swap(d_perm, d_perm2);
        std::swap(d_seg, d_seg2);
        level_off.push_back(next_base + 2 * n_int);
        if ((size_t)level_off.back() > cap) return crtx_set_error(CRT_ERR_HIP, "BVH build: node table overflow");
    }
    BTRY(hipGetLastError());
    const int total = level_off.back();
    const int n_levels = (int)level_off.size() - 1;
    for (int L = n_levels - 1; L >= 0; --L) {
        const int b = level_off[L], e = level_off[L + 1];
        hipLaunchKernelGGL(k_icount, dim3(blocks(e - b)), dim3(256), 0, st, N, b, e);
        hipLaunchKernelGGL(k_refit, dim3(blocks(e - b)), dim3(256), 0, st, N, b, e);
    }
    for (int L = 0; L < n_levels; ++L) {
        const int b = level_off[L], e = level_off[L + 1];
        hipLaunchKernelGGL(k_rank, dim3(blocks(e - b)), dim3(256), 0, st, N, b, e, d_err);
    }
    hipLaunchKernelGGL(k_emit, dim3(blocks(total)), dim3(256), 0, st, N, total, index_count, d_out);
    hipLaunchKernelGGL(k_permute, dim3(blocks(n)), dim3(256), 0, st, d_perm, d_idx, d_fm, d_idx_out, d_fm_out, n);
    BTRY(hipGetLastError());
    BTRY(hipEventRecord(e1, st));
    uint32_t b6[6];
    BTRY(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
    BTRY(hipMemcpyAsync(b6, d_box6, sizeof b6, hipMemcpyDeviceToHost, st));
    BTRY(hipStreamSynchronize(st));
    if (err & ERR_INDEX) return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "vertex index out of range");
    if (err & ERR_DEGENERATE)
        return crtx_set_error(CRT_ERR_UNSUPPORTED, "degenerate split (empty side): the reference's node cap applies; "
                                                   "use the host builder");
    if (err & ERR_STACK) return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "mesh BVH build stack overflow (reference stack is 64)");
    if (err & ERR_JUMP) return crtx_set_error(CRT_ERR_HIP, "BVH build: partition pointer jumping did not converge");
    BTRY(hipMemcpy(nodes, d_out, (size_t)total * sizeof(NodeOut), hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(indices, d_idx_out, 12 * (size_t)n, hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(face_materials, d_fm_out, 4 * (size_t)n, hipMemcpyDeviceToHost));
    for (int k = 0; k < 6; ++k) {
        const uint32_t o = b6[k];
        mesh_box[k] = vertex_count ? __builtin_bit_cast(float, (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o)
                                   : (k < 3 ? INFINITY : -INFINITY);
    }
    *node_count = total;
    if (build_ms) BTRY(hipEventElapsedTime(build_ms, e0, e1));
    return CRT_OK;
}

// ======================================================================================================
// The CRT_BVH_REBUILT binned-SAH build (crt_sah.h's Builder) on the GPU, level by level.
//
// Same rules as the host builder: node box = padded (pad_box) bounds of its items; CRT_SAH_BINS bins per axis over
// the centroid extent; SAH sweep with traversal cost C_trav and unit primitive cost; leaf when the node
// may be a leaf (no spheres, count <= leaf_size) and splitting does not pay; count 1 is a leaf; no usable
// split (all centroids equal) splits in half.  Bin counts and boxes are order-independent, so the splits
// equal the host's; the partition here is stable (the host's std::partition is not), so only the order
// of items inside a node can differ — any order is a valid tree for the rank rule.
// ======================================================================================================
#include "crt_sah.h"
#include "crt/ParallelFor.h"

namespace {

#ifndef CRT_SAH_BINS   // set by crt_sah.h (128)
#define CRT_SAH_BINS 128
#endif
constexpr int SAH_BINS = CRT_SAH_BINS;
constexpr int SAH_RED = 13 + 3 * SAH_BINS * 7;   // box lo3 hi3, centroid lo3 hi3, spheres; bins: count lo3 hi3

struct SahLevel {
    int* start;     // per tmp node
    int* count;
    int* left;      // tmp id of the left child, -1 = leaf
    float* lo;      // padded box, 3 per node
    float* hi;
    int* axis;      // split axis, -1 = split in half
    int* split;     // first bin of the right side
    int* nless;
    float* clo;     // centroid lower bound (3 per node)
    float* scale;   // bins / extent per axis, 0 = axis not binned
    int* internal;  // level-local: 1 when the node splits
};

__device__ __forceinline__ void pad_box_dev(float lo[3], float hi[3]) {   // crt_sah::pad_box
    float m = 1.0f;
    for (int a = 0; a < 3; ++a) m = fmaxf(m, fmaxf(fabsf(lo[a]), fabsf(hi[a])));
    const float pad = 1e-5f * m;
    for (int a = 0; a < 3; ++a) { lo[a] -= pad; hi[a] += pad; }
}
__device__ __forceinline__ float half_area_dev(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

__global__ void k_sah_reset(uint32_t* __restrict__ red, int n_lev) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)n_lev * SAH_RED) return;
    const int w = (int)(i % SAH_RED);
    uint32_t v;
    if (w < 12) v = (w % 6) < 3 ? ord(INFINITY) : ord(-INFINITY);     // lo3 hi3, clo3 chi3
    else if (w == 12) v = 0u;
    else {
        const int k = (w - 13) % 7;
        v = k == 0 ? 0u : k < 4 ? ord(INFINITY) : ord(-INFINITY);
    }
    red[i] = v;
}

// Positions per workgroup of k_sah_bounds / k_sah_bins.  A node's items occupy one contiguous range of positions, so a
// workgroup whose first and last positions belong to the same node holds that node only (the top levels: few nodes of
// many items).  Such a workgroup reduces in registers and LDS and adds its result to the node's with one global atomic
// per word; before round 5 every wave (bounds) or every item (bins) did, and the top levels' bins took 1M items x 21
// atomics on one node's 2,688 words (config E's SAH build: 65 ms of its 100 ms of kernels, profiles/r05l).  Min, max and
// add are order-independent, so the tree is the same.
constexpr int SAH_CHUNK = 4096;

// node bounds: item boxes, centroid bounds, sphere count
__global__ __launch_bounds__(256) void k_sah_bounds(const int* __restrict__ seg, const uint32_t* __restrict__ perm,
                                                    const float* __restrict__ ilo, const float* __restrict__ ihi,
                                                    const float* __restrict__ ic, const int* __restrict__ isph, int n,
                                                    const int* __restrict__ big, uint32_t* __restrict__ red) {
    __shared__ uint32_t part[4][13];
    const int p0 = blockIdx.x * SAH_CHUNK, p1 = min(n, p0 + SAH_CHUNK);
    const int s_first = seg[p0];
    if (s_first >= 0 && seg[p1 - 1] == s_first) {   // uniform workgroup: one node
        const int rb = big[s_first];
        if (rb < 0) return;                          // a small node: k_sah_small
        uint32_t v[12];
        for (int k = 0; k < 12; ++k) v[k] = ((k % 6) < 3) ? 0xffffffffu : 0u;
        uint32_t nsp = 0;
        for (int p = p0 + (int)threadIdx.x; p < p1; p += 256) {
            const uint32_t t = perm[p];
            for (int a = 0; a < 3; ++a) {
                v[a] = min(v[a], ord(ilo[(size_t)a * n + t]));
                v[3 + a] = max(v[3 + a], ord(ihi[(size_t)a * n + t]));
                const uint32_t c = ord(ic[(size_t)a * n + t]);
                v[6 + a] = min(v[6 + a], c);
                v[9 + a] = max(v[9 + a], c);
            }
            nsp += isph[t] != 0;
        }
        const int w = threadIdx.x >> 6;
        for (int k = 0; k < 12; ++k) {
            const uint32_t r = ((k % 6) < 3) ? wave_min(v[k]) : wave_max(v[k]);
            if ((threadIdx.x & 63) == 0) part[w][k] = r;
        }
        uint32_t ns = nsp;
        for (int o = 32; o > 0; o >>= 1) ns += (uint32_t)__shfl_xor((int)ns, o, 64);
        if ((threadIdx.x & 63) == 0) part[w][12] = ns;
        __syncthreads();
        if (threadIdx.x < 13) {
            const int k = threadIdx.x;
            uint32_t r = part[0][k];
            for (int q = 1; q < 4; ++q)
                r = k == 12 ? r + part[q][k] : ((k % 6) < 3) ? min(r, part[q][k]) : max(r, part[q][k]);
            uint32_t* o = red + (size_t)rb * SAH_RED;
            if (k == 12) { if (r) atomicAdd(&o[12], r); }
            else if ((k % 6) < 3) atomicMin(&o[k], r);
            else atomicMax(&o[k], r);
        }
        return;
    }
    for (int q = p0; q < p1; q += 256) {   // several nodes: per wave (one node) or per item
        const int p = q + (int)threadIdx.x;
        LaneSeg L;                          // over big-node indices (small nodes' positions: -1)
        {
            const int s = p < p1 ? seg[p] : -1;
            L.s = s >= 0 ? big[s] : -1;
            const int hi = wave_max_i(L.s), lo = wave_min_i(L.s >= 0 ? L.s : 0x7fffffff);
            L.uniform = hi >= 0 && lo == hi;
            L.s0 = hi;
        }
        if (L.s0 < 0) continue;
        const bool act = L.s >= 0;
        const uint32_t t = act ? perm[p] : 0;
        uint32_t v[12];
        for (int a = 0; a < 3; ++a) {
            v[a] = act ? ord(ilo[(size_t)a * n + t]) : 0xffffffffu;
            v[3 + a] = act ? ord(ihi[(size_t)a * n + t]) : 0u;
            v[6 + a] = act ? ord(ic[(size_t)a * n + t]) : 0xffffffffu;
            v[9 + a] = act ? ord(ic[(size_t)a * n + t]) : 0u;
        }
        const uint32_t sp = act ? (uint32_t)isph[t] : 0u;
        if (L.uniform) {
            uint32_t r[12];
            for (int k = 0; k < 12; ++k) r[k] = ((k % 6) < 3) ? wave_min(v[k]) : wave_max(v[k]);
            const uint64_t nsp = __ballot(sp != 0);
            if ((threadIdx.x & 63) == 0) {
                uint32_t* o = red + (size_t)L.s0 * SAH_RED;
                for (int k = 0; k < 12; ++k) ((k % 6) < 3) ? atomicMin(&o[k], r[k]) : atomicMax(&o[k], r[k]);
                if (nsp) atomicAdd(&o[12], (uint32_t)__popcll(nsp));
            }
        } else if (act) {
            uint32_t* o = red + (size_t)L.s * SAH_RED;
            for (int k = 0; k < 12; ++k) ((k % 6) < 3) ? atomicMin(&o[k], v[k]) : atomicMax(&o[k], v[k]);
            if (sp) atomicAdd(&o[12], 1u);
        }
    }
}

// per node: padded box, bin parameters (crt_sah.h build_range)
__global__ void k_sah_prep(SahLevel N, int base, int n_lev, const int* __restrict__ big, const uint32_t* __restrict__ red) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lev || big[li] < 0) return;
    const int X = base + li;
    const uint32_t* r = red + (size_t)big[li] * SAH_RED;
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) { lo[a] = unord(r[a]); hi[a] = unord(r[3 + a]); }
    pad_box_dev(lo, hi);
    for (int a = 0; a < 3; ++a) {
        N.lo[3 * (size_t)X + a] = lo[a];
        N.hi[3 * (size_t)X + a] = hi[a];
        const float clo = unord(r[6 + a]), chi = unord(r[9 + a]);
        const float ext = chi - clo;
        N.clo[3 * (size_t)X + a] = clo;
        N.scale[3 * (size_t)X + a] = (ext > 0.f && N.count[X] > 1) ? (float)SAH_BINS / ext : 0.f;
    }
}

__device__ __forceinline__ int sah_bin(float c, float clo, float scale) {
    return min(SAH_BINS - 1, (int)((c - clo) * scale));
}

__global__ __launch_bounds__(256) void k_sah_bins(const int* __restrict__ seg, const uint32_t* __restrict__ perm,
                                                  const float* __restrict__ ilo, const float* __restrict__ ihi,
                                                  const float* __restrict__ ic, int n, SahLevel N, int base,
                                                  const int* __restrict__ big, uint32_t* __restrict__ red) {
    constexpr int W = 3 * SAH_BINS * 7;
    __shared__ uint32_t lb[W];   // the workgroup's bins (uniform workgroups): count, lo[3], hi[3] per axis and bin
    const int p0 = blockIdx.x * SAH_CHUNK, p1 = min(n, p0 + SAH_CHUNK);
    const int s_first = seg[p0];
    if (s_first >= 0 && seg[p1 - 1] == s_first) {   // uniform workgroup: one node
        const int rb = big[s_first];
        if (rb < 0) return;                          // a small node: k_sah_small
        const int X = base + s_first;
        float sc[3], clo[3];
        for (int a = 0; a < 3; ++a) { sc[a] = N.scale[3 * (size_t)X + a]; clo[a] = N.clo[3 * (size_t)X + a]; }
        for (int i = threadIdx.x; i < W; i += 256) {
            const int k = i % 7;
            lb[i] = k == 0 ? 0u : k < 4 ? 0xffffffffu : 0u;
        }
        __syncthreads();
        for (int p = p0 + (int)threadIdx.x; p < p1; p += 256) {
            const uint32_t t = perm[p];
            uint32_t lo[3], hi[3];
            for (int k = 0; k < 3; ++k) { lo[k] = ord(ilo[(size_t)k * n + t]); hi[k] = ord(ihi[(size_t)k * n + t]); }
            for (int a = 0; a < 3; ++a) {
                if (sc[a] == 0.f) continue;
                uint32_t* o = lb + (a * SAH_BINS + sah_bin(ic[(size_t)a * n + t], clo[a], sc[a])) * 7;
                atomicAdd(&o[0], 1u);
                for (int k = 0; k < 3; ++k) { atomicMin(&o[1 + k], lo[k]); atomicMax(&o[4 + k], hi[k]); }
            }
        }
        __syncthreads();
        uint32_t* out = red + (size_t)rb * SAH_RED + 13;
        for (int b = threadIdx.x; b < 3 * SAH_BINS; b += 256) {
            const uint32_t* o = lb + b * 7;
            if (o[0] == 0u) continue;   // an empty bin leaves the node's bin as it is (count 0, empty box)
            atomicAdd(&out[b * 7], o[0]);
            for (int k = 0; k < 3; ++k) { atomicMin(&out[b * 7 + 1 + k], o[1 + k]); atomicMax(&out[b * 7 + 4 + k], o[4 + k]); }
        }
        return;
    }
    for (int p = p0 + (int)threadIdx.x; p < p1; p += 256) {   // several nodes: per item
        const int s = seg[p];
        if (s < 0 || big[s] < 0) continue;
        const int X = base + s;
        const uint32_t t = perm[p];
        uint32_t lo[3], hi[3];
        for (int k = 0; k < 3; ++k) { lo[k] = ord(ilo[(size_t)k * n + t]); hi[k] = ord(ihi[(size_t)k * n + t]); }
        for (int a = 0; a < 3; ++a) {
            const float sc = N.scale[3 * (size_t)X + a];
            if (sc == 0.f) continue;
            const int b = sah_bin(ic[(size_t)a * n + t], N.clo[3 * (size_t)X + a], sc);
            uint32_t* o = red + (size_t)big[s] * SAH_RED + 13 + (a * SAH_BINS + b) * 7;
            atomicAdd(&o[0], 1u);
            for (int k = 0; k < 3; ++k) { atomicMin(&o[1 + k], lo[k]); atomicMax(&o[4 + k], hi[k]); }
        }
    }
}

// SAH sweep and leaf test (crt_sah.h build_range, same float expressions)
__global__ void k_sah_decide(SahLevel N, int base, int n_lev, const int* __restrict__ big, const uint32_t* __restrict__ red,
                             int leaf_size, float trav_cost) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lev || big[li] < 0) return;
    const int X = base + li;
    const uint32_t* r = red + (size_t)big[li] * SAH_RED;
    const int count = N.count[X];
    N.internal[li] = 0;
    N.left[X] = -1;
    if (count <= 1) return;
    const bool leaf_ok = r[12] == 0 && count <= leaf_size;
    float best_cost = INFINITY;
    int best_axis = -1, best_split = 0;
    for (int a = 0; a < 3; ++a) {
        if (N.scale[3 * (size_t)X + a] == 0.f) continue;
        const uint32_t* bins = r + 13 + a * SAH_BINS * 7;
        float right_area[SAH_BINS];
        int right_cnt[SAH_BINS];
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int rc = 0;
        for (int b = SAH_BINS - 1; b > 0; --b) {
            const uint32_t* o = bins + b * 7;
            rc += (int)o[0];
            for (int q = 0; q < 3; ++q) { rlo[q] = fminf(rlo[q], unord(o[1 + q])); rhi[q] = fmaxf(rhi[q], unord(o[4 + q])); }
            right_cnt[b] = rc;
            right_area[b] = rc ? half_area_dev(rlo, rhi) : 0.f;
        }
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lc = 0;
        for (int b = 0; b < SAH_BINS - 1; ++b) {
            const uint32_t* o = bins + b * 7;
            lc += (int)o[0];
            for (int q = 0; q < 3; ++q) { llo[q] = fminf(llo[q], unord(o[1 + q])); lhi[q] = fmaxf(lhi[q], unord(o[4 + q])); }
            if (lc == 0 || right_cnt[b + 1] == 0) continue;
            const float cost = half_area_dev(llo, lhi) * lc + right_area[b + 1] * right_cnt[b + 1];
            if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = b + 1; }
        }
    }
    const float node_area = fmaxf(half_area_dev(&N.lo[3 * (size_t)X], &N.hi[3 * (size_t)X]), 1e-30f);
    if (leaf_ok && (best_axis < 0 || trav_cost + best_cost / node_area >= (float)count)) return;
    N.axis[X] = best_axis;
    N.split[X] = best_split;
    int l = count / 2;                            // no usable split: halves (every centroid is the same)
    if (best_axis >= 0) {
        l = 0;
        const uint32_t* bins = r + 13 + best_axis * SAH_BINS * 7;
        for (int b = 0; b < best_split; ++b) l += (int)bins[b * 7];
    }
    N.nless[X] = l;
    N.internal[li] = 1;
}

// Small nodes (at most SAH_SMALL items: the deep levels, where almost every node is one) are binned and decided by one
// thread each, from their items, without the reduction area: k_sah_bounds / k_sah_bins / k_sah_decide then run over
// the big nodes only, and the area holds big nodes (n / (SAH_SMALL + 1) at most) instead of every node of the level
// (n_lev x 10.7 KB: 2.7 GB at config E's deepest levels).  The decision is the binned one, candidate for candidate:
//   * bounds and centroid bounds: the same ord() minima and maxima;
//   * a split between bins b and b + 1 has the same cost for every b of a run of empty bins, so the strictly-smaller
//     sweep of k_sah_decide picks the first b of each run, the last non-empty bin on the left: this sweep visits the
//     non-empty bins only (the items sorted by bin), in the same order, with the same left / right boxes (the same fminf
//     / fmaxf sequence, empty bins being no-ops) and the same cost expression.
constexpr int SAH_SMALL = 16;

__global__ void k_sah_small(SahLevel N, int base, int n_lev, const int* __restrict__ big, const uint32_t* __restrict__ perm,
                            const float* __restrict__ ilo, const float* __restrict__ ihi, const float* __restrict__ ic,
                            const int* __restrict__ isph, int n, int leaf_size, float trav_cost) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lev || big[li] >= 0) return;
    const int X = base + li, count = N.count[X], start = N.start[X];
    N.internal[li] = 0;
    N.left[X] = -1;
    uint32_t t[SAH_SMALL];
    uint32_t blo[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, bhi[3] = {0u, 0u, 0u};
    uint32_t cmin[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, cmax[3] = {0u, 0u, 0u};
    int nsp = 0;
    for (int k = 0; k < count; ++k) {   // k_sah_bounds
        t[k] = perm[start + k];
        for (int a = 0; a < 3; ++a) {
            blo[a] = min(blo[a], ord(ilo[(size_t)a * n + t[k]]));
            bhi[a] = max(bhi[a], ord(ihi[(size_t)a * n + t[k]]));
            const uint32_t c = ord(ic[(size_t)a * n + t[k]]);
            cmin[a] = min(cmin[a], c);
            cmax[a] = max(cmax[a], c);
        }
        nsp += isph[t[k]] != 0;
    }
    float lo[3], hi[3], clo[3], sc[3];   // k_sah_prep
    for (int a = 0; a < 3; ++a) { lo[a] = unord(blo[a]); hi[a] = unord(bhi[a]); }
    pad_box_dev(lo, hi);
    for (int a = 0; a < 3; ++a) {
        N.lo[3 * (size_t)X + a] = lo[a];
        N.hi[3 * (size_t)X + a] = hi[a];
        clo[a] = unord(cmin[a]);
        const float ext = unord(cmax[a]) - clo[a];
        N.clo[3 * (size_t)X + a] = clo[a];
        sc[a] = (ext > 0.f && count > 1) ? (float)SAH_BINS / ext : 0.f;
        N.scale[3 * (size_t)X + a] = sc[a];
    }
    if (count <= 1) return;             // k_sah_decide
    const bool leaf_ok = nsp == 0 && count <= leaf_size;
    float best_cost = INFINITY;
    int best_axis = -1, best_split = 0;
    for (int a = 0; a < 3; ++a) {
        if (sc[a] == 0.f) continue;
        int bin[SAH_SMALL], ord_k[SAH_SMALL];
        for (int k = 0; k < count; ++k) {   // items by bin (insertion sort; equal bins keep item order)
            bin[k] = sah_bin(ic[(size_t)a * n + t[k]], clo[a], sc[a]);
            int j = k;
            while (j > 0 && bin[ord_k[j - 1]] > bin[k]) { ord_k[j] = ord_k[j - 1]; --j; }
            ord_k[j] = k;
        }
        // groups of equal bins: count, box (ord min / max of the items, as the bins hold them)
        int gb[SAH_SMALL], gc[SAH_SMALL], G = 0;
        uint32_t glo[SAH_SMALL][3], ghi[SAH_SMALL][3];
        for (int q = 0; q < count; ++q) {
            const int k = ord_k[q];
            if (G == 0 || gb[G - 1] != bin[k]) {
                gb[G] = bin[k];
                gc[G] = 0;
                for (int d = 0; d < 3; ++d) { glo[G][d] = 0xffffffffu; ghi[G][d] = 0u; }
                ++G;
            }
            ++gc[G - 1];
            for (int d = 0; d < 3; ++d) {
                glo[G - 1][d] = min(glo[G - 1][d], ord(ilo[(size_t)d * n + t[k]]));
                ghi[G - 1][d] = max(ghi[G - 1][d], ord(ihi[(size_t)d * n + t[k]]));
            }
        }
        float right_area[SAH_SMALL];
        int right_cnt[SAH_SMALL];
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int rc = 0;
        for (int g = G - 1; g > 0; --g) {   // the bins above the first non-empty one, from the top
            rc += gc[g];
            for (int d = 0; d < 3; ++d) { rlo[d] = fminf(rlo[d], unord(glo[g][d])); rhi[d] = fmaxf(rhi[d], unord(ghi[g][d])); }
            right_cnt[g] = rc;
            right_area[g] = half_area_dev(rlo, rhi);
        }
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lc = 0;
        for (int g = 0; g + 1 < G; ++g) {
            lc += gc[g];
            for (int d = 0; d < 3; ++d) { llo[d] = fminf(llo[d], unord(glo[g][d])); lhi[d] = fmaxf(lhi[d], unord(ghi[g][d])); }
            const float cost = half_area_dev(llo, lhi) * lc + right_area[g + 1] * right_cnt[g + 1];
            if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = gb[g] + 1; }
        }
    }
    const float node_area = fmaxf(half_area_dev(lo, hi), 1e-30f);
    if (leaf_ok && (best_axis < 0 || trav_cost + best_cost / node_area >= (float)count)) return;
    N.axis[X] = best_axis;
    N.split[X] = best_split;
    int l = count / 2;                            // no usable split: halves (every centroid is the same)
    if (best_axis >= 0) {
        l = 0;
        for (int k = 0; k < count; ++k) l += sah_bin(ic[(size_t)best_axis * n + t[k]], clo[best_axis], sc[best_axis]) < best_split;
    }
    N.nless[X] = l;
    N.internal[li] = 1;
}

// big[li] = the rank of level node li among the level's nodes of more than SAH_SMALL items, -1 for the others
// (single workgroup); total[0] = how many
__global__ __launch_bounds__(1024) void k_big_scan(SahLevel N, int base, int n_lev, int* __restrict__ big,
                                                   int* __restrict__ total) {
    __shared__ int part[1024];
    const int tid = threadIdx.x, per = (n_lev + 1023) / 1024;
    const int b = min(n_lev, tid * per), e = min(n_lev, b + per);
    int c = 0;
    for (int i = b; i < e; ++i) c += N.count[base + i] > SAH_SMALL;
    part[tid] = c;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int add = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    int r = part[tid] - c;
    for (int i = b; i < e; ++i) big[i] = N.count[base + i] > SAH_SMALL ? r++ : -1;
    if (tid == 1023) total[0] = part[1023];
}

// ranks of the level's splitting nodes (single workgroup); stats[0] = how many
__global__ __launch_bounds__(1024) void k_sah_scan(SahLevel N, int n_lev, int* __restrict__ irank, int* __restrict__ stats) {
    __shared__ int part[1024];
    const int tid = threadIdx.x, per = (n_lev + 1023) / 1024;
    const int b = min(n_lev, tid * per), e = min(n_lev, b + per);
    int c = 0;
    for (int i = b; i < e; ++i) c += N.internal[i];
    part[tid] = c;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int add = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    int r = part[tid] - c;
    for (int i = b; i < e; ++i) irank[i] = N.internal[i] ? r++ : -1;
    if (tid == 1023) stats[0] = part[1023];
}

__global__ void k_sah_children(SahLevel N, int base, int n_lev, const int* __restrict__ irank, int next_base) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lev || irank[li] < 0) return;
    const int X = base + li, cl = next_base + 2 * irank[li], l = N.nless[X];
    N.left[X] = cl;
    N.start[cl] = N.start[X];
    N.count[cl] = l;
    N.start[cl + 1] = N.start[X] + l;
    N.count[cl + 1] = N.count[X] - l;
    N.left[cl] = N.left[cl + 1] = -1;
}

__global__ void k_sah_flags(const int* __restrict__ seg, const uint32_t* __restrict__ perm, const float* __restrict__ ic,
                            int n, SahLevel N, int base, uint32_t* __restrict__ flags) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    uint32_t f = 0;
    if (s >= 0 && N.left[base + s] >= 0) {
        const int X = base + s, a = N.axis[X];
        if (a >= 0) f = sah_bin(ic[(size_t)a * n + perm[p]], N.clo[3 * (size_t)X + a], N.scale[3 * (size_t)X + a]) < N.split[X];
        else f = (p - N.start[X]) < N.nless[X];
    }
    flags[p] = f;
}

// stable two-sided partition; every position of a splitting node moves to its child's range
__global__ void k_sah_scatter(const int* __restrict__ seg, const uint32_t* __restrict__ flags,
                              const uint32_t* __restrict__ lb, const uint32_t* __restrict__ perm,
                              uint32_t* __restrict__ perm2, int* __restrict__ seg2, int n, SahLevel N, int base,
                              int next_base) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    if (s < 0 || N.left[base + s] < 0) { perm2[p] = perm[p]; seg2[p] = -1; return; }
    const int X = base + s, st = N.start[X], l = N.nless[X];
    const int less = (int)(lb[p] - lb[st]);
    const int dst = flags[p] ? st + less : st + l + ((p - st) - less);
    perm2[dst] = perm[p];
    const int c = N.left[X] + (dst - st < l ? 0 : 1);
    seg2[dst] = c - next_base;
}

}  // namespace

// Host entry used by crt_scene_create_ex / crt_scene_export (gpu_build): the tree crt_sah::Builder would build,
// as Builder::nodes() (root 0) and the item order (indices into `items`).
int crtx_build_sah_gpu(int device, const std::vector<crt_sah::Item>& items, int leaf_size, float trav_cost,
                       std::vector<crt_sah::Node>* nodes_out, std::vector<int>* order_out, int* max_depth) {
    const int n = (int)items.size();
    if (n <= 0) return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "SAH build: no items");
    int ndev = 0;
    BTRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return crtx_set_error(CRT_ERR_INVALID_ARGUMENT, "device ordinal out of range");
    BTRY(hipSetDevice(device));
    DeviceArena A;
    hipStream_t st = nullptr;
    std::vector<float> h(9 * (size_t)n);
    std::vector<int> hs((size_t)n);
    CRT::parallel_ranges((size_t)n, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) {
            for (int a = 0; a < 3; ++a) {
                h[(size_t)a * n + i] = items[i].lo[a];
                h[3 * (size_t)n + (size_t)a * n + i] = items[i].hi[a];
                h[6 * (size_t)n + (size_t)a * n + i] = items[i].c[a];
            }
            hs[i] = items[i].sphere ? 1 : 0;
        }
    });
    float* d_item = nullptr;
    int* d_sph = nullptr;
    BTRY(A.alloc(&d_item, 9 * (size_t)n));
    BTRY(A.alloc(&d_sph, n));
    BTRY(hipMemcpyAsync(d_item, h.data(), h.size() * 4, hipMemcpyHostToDevice, st));
    BTRY(hipMemcpyAsync(d_sph, hs.data(), hs.size() * 4, hipMemcpyHostToDevice, st));
    const float *d_lo = d_item, *d_hi = d_item + 3 * (size_t)n, *d_c = d_item + 6 * (size_t)n;
    const size_t cap = 2 * (size_t)n + 2;
    const size_t lev_cap = (size_t)n + 2;
    const int nb = (n + SCAN_ITEMS - 1) / SCAN_ITEMS;
    uint32_t *d_perm, *d_perm2, *d_flags, *d_lb, *d_bsum, *d_red;
    int *d_seg, *d_seg2, *d_irank, *d_stats;
    BTRY(A.alloc(&d_perm, n));
    BTRY(A.alloc(&d_perm2, n));
    BTRY(A.alloc(&d_flags, n));
    BTRY(A.alloc(&d_lb, n));
    BTRY(A.alloc(&d_bsum, nb));
    BTRY(A.alloc(&d_seg, n));
    BTRY(A.alloc(&d_seg2, n));
    BTRY(A.alloc(&d_irank, lev_cap));
    BTRY(A.alloc(&d_stats, 2));
    int* d_big;
    BTRY(A.alloc(&d_big, lev_cap));
    SahLevel N;
    BTRY(A.alloc(&N.start, cap));
    BTRY(A.alloc(&N.count, cap));
    BTRY(A.alloc(&N.left, cap));
    BTRY(A.alloc(&N.lo, 3 * cap));
    BTRY(A.alloc(&N.hi, 3 * cap));
    BTRY(A.alloc(&N.axis, cap));
    BTRY(A.alloc(&N.split, cap));
    BTRY(A.alloc(&N.nless, cap));
    BTRY(A.alloc(&N.clo, 3 * cap));
    BTRY(A.alloc(&N.scale, 3 * cap));
    BTRY(A.alloc(&N.internal, lev_cap));
    size_t red_cap = 0;
    d_red = nullptr;
    hipLaunchKernelGGL(k_iota, dim3(blocks(n)), dim3(256), 0, st, d_perm, d_seg, n);
    {
        const int zero = 0;
        BTRY(hipMemcpyAsync(N.start, &zero, 4, hipMemcpyHostToDevice, st));
        BTRY(hipMemcpyAsync(N.count, &n, 4, hipMemcpyHostToDevice, st));
        BTRY(hipMemsetAsync(N.left, 0xff, 4, st));
    }
    std::vector<int> level_off = {0, 1};
    for (;;) {
        const int base = level_off[level_off.size() - 2], n_lev = level_off.back() - base;
        hipLaunchKernelGGL(k_big_scan, dim3(1), dim3(1024), 0, st, N, base, n_lev, d_big, d_stats + 1);
        int n_big = 0;
        BTRY(hipMemcpyAsync(&n_big, d_stats + 1, 4, hipMemcpyDeviceToHost, st));
        BTRY(hipStreamSynchronize(st));
        if (n_big > 0) {
            if ((size_t)n_big * SAH_RED > red_cap) {   // grow the reduction area (big nodes only)
                red_cap = std::max((size_t)n_big * SAH_RED, 2 * red_cap);
                BTRY(A.alloc(&d_red, red_cap));
            }
            hipLaunchKernelGGL(k_sah_reset, dim3(blocks((size_t)n_big * SAH_RED)), dim3(256), 0, st, d_red, n_big);
            const int chunks = (n + SAH_CHUNK - 1) / SAH_CHUNK;
            hipLaunchKernelGGL(k_sah_bounds, dim3(chunks), dim3(256), 0, st, d_seg, d_perm, d_lo, d_hi, d_c, d_sph, n, d_big,
                               d_red);
            hipLaunchKernelGGL(k_sah_prep, dim3(blocks(n_lev)), dim3(256), 0, st, N, base, n_lev, d_big, d_red);
            hipLaunchKernelGGL(k_sah_bins, dim3(chunks), dim3(256), 0, st, d_seg, d_perm, d_lo, d_hi, d_c, n, N, base, d_big,
                               d_red);
            hipLaunchKernelGGL(k_sah_decide, dim3(blocks(n_lev)), dim3(256), 0, st, N, base, n_lev, d_big, d_red, leaf_size,
                               trav_cost);
        }
        if (n_big < n_lev)
            hipLaunchKernelGGL(k_sah_small, dim3(blocks(n_lev)), dim3(256), 0, st, N, base, n_lev, d_big, d_perm, d_lo, d_hi,
                               d_c, d_sph, n, leaf_size, trav_cost);
        hipLaunchKernelGGL(k_sah_scan, dim3(1), dim3(1024), 0, st, N, n_lev, d_irank, d_stats);
        int n_int = 0;
        BTRY(hipMemcpyAsync(&n_int, d_stats, 4, hipMemcpyDeviceToHost, st));
        BTRY(hipStreamSynchronize(st));
        if (n_int == 0) break;
        const int next_base = level_off.back();
        if ((size_t)next_base + 2 * (size_t)n_int > cap) return crtx_set_error(CRT_ERR_HIP, "SAH build: node table overflow");
        hipLaunchKernelGGL(k_sah_children, dim3(blocks(n_lev)), dim3(256), 0, st, N, base, n_lev, d_irank, next_base);
        hipLaunchKernelGGL(k_sah_flags, dim3(blocks(n)), dim3(256), 0, st, d_seg, d_perm, d_c, n, N, base, d_flags);
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, d_flags, d_lb, d_bsum, n);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, st, d_bsum, nb);
        hipLaunchKernelGGL(k_scan_add, dim3(blocks(n)), dim3(256), 0, st, d_lb, d_bsum, n);
        hipLaunchKernelGGL(k_sah_scatter, dim3(blocks(n)), dim3(256), 0, st, d_seg, d_flags, d_lb, d_perm, d_perm2, d_seg2,
                           n, N, base, next_base);
        std::swap(d_perm, d_perm2);
        std::swap(d_seg, d_seg2);
        level_off.push_back(next_base + 2 * n_int);
    }
    BTRY(hipGetLastError());
    const int total = level_off.back();
    std::vector<int> hstart(total), hcount(total), hleft(total);
    std::vector<float> hlo(3 * (size_t)total), hhi(3 * (size_t)total);
    std::vector<uint32_t> hperm(n);
    BTRY(hipMemcpy(hstart.data(), N.start, (size_t)total * 4, hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(hcount.data(), N.count, (size_t)total * 4, hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(hleft.data(), N.left, (size_t)total * 4, hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(hlo.data(), N.lo, (size_t)total * 12, hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(hhi.data(), N.hi, (size_t)total * 12, hipMemcpyDeviceToHost));
    BTRY(hipMemcpy(hperm.data(), d_perm, (size_t)n * 4, hipMemcpyDeviceToHost));
    nodes_out->assign((size_t)total, crt_sah::Node{});
    CRT::parallel_ranges((size_t)total, [&](size_t b, size_t e) {
        for (size_t t = b; t < e; ++t) {
            crt_sah::Node& o = (*nodes_out)[t];
            for (int a = 0; a < 3; ++a) { o.lo[a] = hlo[3 * t + a]; o.hi[a] = hhi[3 * t + a]; }
            o.child[0] = hleft[t];
            o.child[1] = hleft[t] < 0 ? -1 : hleft[t] + 1;
            o.first = hstart[t];
            o.count = hleft[t] < 0 ? hcount[t] : 0;
        }
    });
    order_out->assign(hperm.begin(), hperm.end());
    if (max_depth) *max_depth = (int)level_off.size() - 2;
    return CRT_OK;
}
