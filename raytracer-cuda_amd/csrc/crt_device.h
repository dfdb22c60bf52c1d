// crt_device.h — device-side building blocks of the gfx950 render kernel.
//
// Every function restates one reference function with the SAME floating-point
// operation order (no contraction: the library is built with -ffp-contract=off,
// IEEE f32/f64 division and sqrt), so the HIP path is bit-identical to the
// reference's arithmetic.  Reference paths are relative to CudaRayTracer/src/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace crt {

// ---------------------------------------------------------------- layout
// Flattened scene in HBM (built by crt_hip.hip from the host-built reference BVHs):
//
// nodes: 2 x float4 (32 B) per node, DFS preorder over the scene BVH with every
// mesh BVH spliced in after its scene leaf ("threaded" BVH: left child = next
// node, `skip` = first node after the subtree).  The left-first stack DFS of
// BVHNode::hit (BVHNode.cuh:115-156) and Mesh::hit (Mesh.cuh:55-110) visits
// exactly this order, so the traversal needs no stack at all.
//   A = (min.x, min.y, min.z, max.x)   B = (max.y, max.z, a, b)
//   internal mesh node : a = skip, b = NODE_MESH_INNER  (box tested against [0.001, closest])
//   scene node / scene mesh leaf : a = skip, b = NODE_SCENE_INNER (box tested against [0.001, inf),
//                                   the unshrunk ray_t of BVHNode::hit, BVHNode.cuh:129)
//   mesh leaf          : a = triangle count, b = first triangle prim (>= 0)
//   sphere leaf        : a = 0, b = SPHERE_BIT | sphere prim          (scene level: [0.001, inf))
//   every leaf continues at node + 1.
// prims: 3 x float4 (48 B) per primitive.
//   triangle: (v0.xyz, e1.x) (e1.y, e1.z, e2.xy) (e2.z, material, rank, 0)   e1 = v1-v0, e2 = v2-v0
//             (bit-identical to Mesh.cuh:277-278, which subtracts in f32 too)
//   sphere  : (center.xyz, radius) (radius^2, material, rank, 0) (0,0,0,0)
//   rank = position of the primitive in the reference's DFS visiting order (ties go to the higher rank);
//   rank_code[rank] = prim index (| SPHERE_BIT for spheres) maps a hit back to its record.
// CRT_BVH_REBUILT scenes hold 1 or 6 threaded layouts of the same tree back to back (n_nodes each; skip
// links relative to the layout); internal nodes are NODE_MESH_INNER, leaves as above.
// materials: 3 x float4 (48 B): (type, albedo.xyz) (emission.xyz, roughness) (ior, 0, 0, 0)
// shading records: 3 x float4 (48 B) per RANK, everything shade() needs for a hit in one independent pair
// of loads (instead of rank_code -> prim -> material, three dependent loads):
//   (a.xyz, kind) (payload) (1/radius, 0, 0, 0)
//   triangle: a = unit(cross(e1, e2)), the outward normal computed on the host with the device's f32
//             operation order (Mesh.cuh:303-304; bit-identical); sphere: a = center, kind | SHADE_SPHERE,
//             outward = (1/radius) * (hp - center) at the hit (Sphere.cuh:44), 1/radius in the third float4
//   kind & 15 = SHADE_LAMBERT / _METAL / _DIELECTRIC / _LIGHT / _NOEMIT (unknown type: emit 0) /
//               _INVALID (material index out of range: the same-ray bounce of CUDAKernels.h:127)
//   payload: lambertian (albedo.xyz, 0)  metal (albedo.xyz, min(roughness, 1))  light (emission.xyz, 0)
//            dielectric (ior, 1/ior, r0(1/ior), r0(ior)) with Schlick's r0(ri) = ((1 - ri) / (1 + ri))^2
constexpr uint32_t SHADE_LAMBERT = 0, SHADE_METAL = 1, SHADE_DIELECTRIC = 2, SHADE_LIGHT = 3, SHADE_NOEMIT = 4,
                   SHADE_INVALID = 5, SHADE_SPHERE = 16;
constexpr int NODE_MESH_INNER = -1;
constexpr int NODE_SCENE_INNER = -3;
constexpr int SPHERE_BIT = 1 << 30;

// Correctly rounded 1/x for the Möller–Trumbore determinant: v_rcp_f32 + one FMA Newton step.
// Exhaustively verified on gfx950 against IEEE division for EVERY float with
// 1e-8 <= |x| < RCP_FAST_MAX (crt_selftest_rcp, tests/test_gpu_parity.py); outside that range
// the exact division sequence is used, so the result always equals 1.f / x bit for bit.
constexpr float RCP_FAST_MAX = 8.507059e37f;   // 2^126: reciprocal stays a normal float
__device__ __forceinline__ float rcp_newton(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float recip_exact(float x) {
    return fabsf(x) < RCP_FAST_MAX ? rcp_newton(x) : 1.0f / x;
}
// 1.f / x for ANY x (the fast path only inside the exhaustively verified range).
constexpr float RCP_FAST_MIN = 1e-8f;
__device__ __forceinline__ float recip_exact_any(float x) {
    const float a = fabsf(x);
    return (a >= RCP_FAST_MIN && a < RCP_FAST_MAX) ? rcp_newton(x) : 1.0f / x;
}

// 1.f / x, bit for bit, by rcp_newton when every active lane's |x| lies in the exhaustively verified range (a
// wave-uniform branch, so a wave never runs both sequences), else by IEEE division.
__device__ __forceinline__ float recip_exact_wave(float x) {
    const float a = fabsf(x);
    if (__builtin_amdgcn_ballot_w64(!(a >= RCP_FAST_MIN && a < RCP_FAST_MAX)) == 0) return rcp_newton(x);
    return 1.0f / x;
}

// a / b from r = RN(1 / b): q0 = RN(a * r), the residual a - q0 * b (exact in one FMA), one correction step (Markstein's
// division iteration).  For next_ray's image coordinates (x + U) / width and / height only, and only for a frame size
// whose every reachable numerator was checked against the IEEE division on the device (crt_renderer_create,
// crt_uv_div_check_kernel); other sizes divide.
__device__ __forceinline__ float uv_div(float a, float b, float r) {
    const float q0 = a * r;
    return __builtin_fmaf(__builtin_fmaf(-q0, b, a), r, q0);
}

// sqrtf(x) bit for bit: r = v_rsq_f32(x), s0 = x * r, one correction step s0 + (x - s0 * s0) * (r / 2) (the residual
// exact in one FMA).  Exhaustively verified on gfx950 against the correctly rounded sqrtf for EVERY float in
// [2^-100, FLT_MAX] (tools/probes/sqrt_probe.hip, profiles/r02an; crt_selftest_sqrt, tests/test_gpu_parity.py).
// 5 VALU instead of the ~16 of the compiler's correctly rounded sequence (raw v_sqrt_f32 is off by one ulp for ~16 %
// of inputs, profiles/r01k).
constexpr float SQRT_FAST_MIN = 0x1p-100f;
__device__ __forceinline__ float sqrt_rsq(float x) {
    const float r = __builtin_amdgcn_rsqf(x);
    const float s0 = x * r;
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, x), 0.5f * r, s0);
}
// sqrtf(x) for ANY x: sqrt_rsq when every active lane's x lies in the verified range (a wave-uniform branch), else the
// IEEE sequence (0, denormals, x < 2^-100, inf, NaN, negative).
__device__ __forceinline__ float sqrt_exact_wave(float x) {
    if (__builtin_amdgcn_ballot_w64(!(x >= SQRT_FAST_MIN && x <= 3.40282347e38f)) == 0) return sqrt_rsq(x);
    __asm__ volatile("");   // keeps the branch: no if-conversion that would run both sequences
    return sqrtf(x);
}

struct V3 { float x, y, z; };

__device__ __forceinline__ V3 v3(float a, float b, float c) { return V3{a, b, c}; }
__device__ __forceinline__ V3 operator+(V3 u, V3 v) { return v3(u.x + v.x, u.y + v.y, u.z + v.z); }   // Vec3.cuh:173
__device__ __forceinline__ V3 operator-(V3 u, V3 v) { return v3(u.x - v.x, u.y - v.y, u.z - v.z); }   // :177
__device__ __forceinline__ V3 operator*(V3 u, V3 v) { return v3(u.x * v.x, u.y * v.y, u.z * v.z); }   // :181
__device__ __forceinline__ V3 operator*(float t, V3 v) { return v3(t * v.x, t * v.y, t * v.z); }      // :185
__device__ __forceinline__ V3 operator-(V3 v) { return v3(-v.x, -v.y, -v.z); }                       // :21
__device__ __forceinline__ float dot(V3 u, V3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }       // :216
__device__ __forceinline__ V3 cross(V3 u, V3 v) {                                                     // :220
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
__device__ __forceinline__ float len2(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }            // :95
// Vec3::unit: (1 / length) * v, the reciprocal and the square root exact (recip_exact_wave, -0.5 %, profiles/r02s;
// sqrt_exact_wave, profiles/r02an)
__device__ __forceinline__ V3 unit(V3 v) { return recip_exact_wave(sqrt_exact_wave(len2(v))) * v; }   // :201,:213
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return v - (2.0f * dot(v, n)) * n; }              // :225
__device__ __forceinline__ V3 refract(V3 uv, V3 n, float eta) {                                        // :229
    float cos_theta = fminf(dot(-uv, n), 1.0f);
    V3 perp = eta * (uv + cos_theta * n);
    V3 par = (-sqrt_exact_wave(fabsf(1.0f - len2(perp)))) * n;
    return perp + par;
}

// ------------------------------------------------------------------ XORWOW
// cuRAND XORWOW (CUDA 12.5 curand_kernel.h: curand, _curand_uniform) — see DESIGN.md.
struct Rng { uint32_t v0, v1, v2, v3, v4, d; };

__device__ __forceinline__ uint32_t next_u32(Rng& s) {
    uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1; s.v1 = s.v2; s.v2 = s.v3; s.v3 = s.v4;
    // (v4 ^ (v4 << 4)) ^ (t ^ (t << 1)): three of the four terms in one v_bitop3_b32 (0x96 = a ^ b ^ c)
    s.v4 = __builtin_amdgcn_bitop3_b32(s.v4, s.v4 << 4, t, 0x96) ^ (t << 1);
    s.d += 362437u;
    return s.v4 + s.d;
}
// curand_uniform: (float)x * 2^-32 + 2^-33 (CURAND_2POW32_INV and half of it).  Both constants are VOP2 literals, so
// no register holds them (an fma form, one rounding of the same exact product, needs both in VGPRs on gfx950 and
// measured +1.3 % through register pressure, profiles/r02t).
__device__ __forceinline__ float uniform(Rng& s) { return __builtin_fmaf((float)next_u32(s), 0x1p-32f, 0x1p-33f); }
// Utility.cuh:18-21: min + (max - min) * U, here min=-1, max=1: -1 + 2 * fl(X * 2^-32 + 2^-33).  (float)x has at most 24
// significant bits, so X * 2^-32 is exact and doubling commutes with the rounding: 2 * U = fl(X * 2^-31 + 2^-32), one
// multiply fewer than the literal restatement, the same bits.
__device__ __forceinline__ float rand_pm1(Rng& s) { return __builtin_fmaf(uniform(s), 2.0f, -1.0f); }

__device__ __forceinline__ V3 rand_unit_vector(Rng& s) {   // Utility.cuh:45-53, :73-76
    V3 p;
    for (;;) {
        float a = rand_pm1(s);
        float b = rand_pm1(s);
        float c = rand_pm1(s);
        p = v3(a, b, c);
        if (len2(p) >= 1) continue;
        break;
    }
    return unit(p);
}

// Material.cuh:132-137 with pow(float,int) restated as exponentiation by squaring.  r0 = ((1 - ref_idx) /
// (1 + ref_idx))^2 depends on the material and the face only: the shading record carries it (schlick_r0 in
// crt_hip.hip's shading_records, IEEE f32 on the host, the same bits), so a hit pays no division for it.
__device__ __forceinline__ float schlick_r0(float cosine, float r0) {
    float a = 1 - cosine;
    float r = 1.0f * a;          // e = 5: bit0
    a = a * a;                   // e = 2
    a = a * a;                   // e = 1
    r = r * a;
    return r0 + (1 - r0) * r;
}

__device__ __forceinline__ V3 sky(V3 d) {   // CRTUtility.cuh:34-38
    V3 ud = unit(d);
    float t = 0.5f * (ud.y + 1.0f);
    return (1.0f - t) * v3(1.0f, 1.0f, 1.0f) + t * v3(0.5f, 0.7f, 1.0f);
}

__device__ __forceinline__ unsigned char to_u8(float c) {   // CRTUtility.cuh:14-32
    double x = c;
    float g = (float)(x > 0 ? sqrt(x) : 0);
    if (g < 0.000f) g = 0.000f;
    else if (g > 0.999f) g = 0.999f;
    return (unsigned char)(256 * g);
}

}  // namespace crt
