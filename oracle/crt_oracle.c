/*
 * crt_oracle.c — CPU ORACLE for the crt-mi355x render path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline.  The product path (raytracer-cuda_amd/) never links or calls it.
 *
 * What it is: a literal, single-precision-faithful restatement of the reference
 * render path of Mordentary/RayTracer-Cuda (paths relative to
 * /root/reference/CudaRayTracer/src/), in the reference's own structure:
 * AoS BVH nodes in builder index order, explicit traversal stacks, per-visit
 * slab reciprocals, per-hit HitInfo.  Every function cites the lines it follows.
 * Compiled with -ffp-contract=off and without fast-math: no FMA contraction,
 * IEEE division and sqrt, double precision exactly where the reference uses it.
 *
 * PARITY STATUS:
 *   * The reference itself is UNBUILDABLE in this image: its render path needs
 *     cuda_runtime.h, curand_kernel.h and SFML headers, none of which exist here,
 *     and stand-ins are not allowed.  The reference has no tests, fixtures or
 *     golden vectors.  Whole-image parity against the reference binary is
 *     therefore "parity unpinned"; the oracle is pinned piecewise:
 *       - XORWOW subsequence jump A^(2^67 * 4^k): checked bit-for-bit against
 *         rocRAND's published table (rocrand_xorwow_precomputed.h,
 *         h_xorwow_sequence_jump_matrices) — same recurrence as cuRAND's.
 *       - cuRAND seeding constants / uniform mapping: restated from cuRAND
 *         (CUDA Toolkit 12.5, curand_kernel.h: _curand_init_scratch, curand,
 *         _curand_uniform); unverifiable offline.
 *       - pow(float,int) in Dielectric::schlicksReflectance (Material.cuh:136):
 *         CUDA's pow(float,int) overload; restated as exponentiation by squaring.
 *       - Argument evaluation order of Vec3(randomFloat(),randomFloat(),...)
 *         (Utility.cuh:40-42, :58) taken left-to-right.
 *       - nvcc's default -fmad=true contraction is NOT modelled (it is not
 *         reproducible across compilers); the oracle is the no-contraction path.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------ Vec3 */
/* Core/Vec3.cuh:8-234 */
typedef struct { float e[3]; } V3;
static inline V3 v3(float a, float b, float c) { V3 r; r.e[0] = a; r.e[1] = b; r.e[2] = c; return r; }
static inline V3 vadd(V3 u, V3 v) { return v3(u.e[0] + v.e[0], u.e[1] + v.e[1], u.e[2] + v.e[2]); }   /* :173 */
static inline V3 vsub(V3 u, V3 v) { return v3(u.e[0] - v.e[0], u.e[1] - v.e[1], u.e[2] - v.e[2]); }   /* :177 */
static inline V3 vmul(V3 u, V3 v) { return v3(u.e[0] * v.e[0], u.e[1] * v.e[1], u.e[2] * v.e[2]); }   /* :181 */
static inline V3 smul(float t, V3 v) { return v3(t * v.e[0], t * v.e[1], t * v.e[2]); }               /* :185 */
static inline V3 muls(V3 v, float t) { return v3(v.e[0] * t, v.e[1] * t, v.e[2] * t); }               /* :197 */
static inline V3 vdiv(V3 v, float t) { return smul(1 / t, v); }                                       /* :201 */
static inline V3 vneg(V3 v) { return v3(-v.e[0], -v.e[1], -v.e[2]); }                                  /* :21 */
static inline float len2(V3 v) { return v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]; }       /* :95 */
static inline float vlen(V3 v) { return sqrtf(len2(v)); }                                             /* :91 */
static inline V3 unitv(V3 v) { return vdiv(v, vlen(v)); }                                            /* :213 */
static inline float dot3(V3 u, V3 v) { return u.e[0] * v.e[0] + u.e[1] * v.e[1] + u.e[2] * v.e[2]; } /* :216 */
static inline V3 cross3(V3 u, V3 v) {                                                                 /* :220 */
    return v3(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
static inline int near_zero(V3 v) {                                                                   /* :99 */
    const float s = 1e-8f;
    return fabsf(v.e[0]) < s && fabsf(v.e[1]) < s && fabsf(v.e[2]) < s;
}
static inline V3 reflect3(V3 v, V3 n) { return vsub(v, smul(2 * dot3(v, n), n)); }                    /* :225 */
static inline V3 refract3(V3 uv, V3 n, float eta) {                                                   /* :229 */
    float cos_theta = fminf(dot3(vneg(uv), n), 1.0f);
    V3 perp = smul(eta, vadd(uv, smul(cos_theta, n)));
    V3 par = smul(-sqrtf(fabsf(1.0f - len2(perp))), n);
    return vadd(perp, par);
}

/* -------------------------------------------------------------- Interval */
/* Core/Interval.cuh:6-49 */
typedef struct { float min, max; } Iv;
static inline Iv iv(float a, float b) { Iv r; r.min = a; r.max = b; return r; }
static inline float iv_size(Iv a) { return a.max - a.min; }
static inline Iv iv_expand(Iv a, float delta) { float p = delta / 2.f; return iv(a.min - p, a.max + p); }

/* ------------------------------------------------------------------ AABB */
/* Core/AABB.cuh:9-189 */
typedef struct { Iv x, y, z; } Box;
static void box_pad(Box* b) {                                                        /* :181-186 */
    const float delta = 0.000001f;
    if (iv_size(b->x) < delta) b->x = iv_expand(b->x, delta);
    if (iv_size(b->y) < delta) b->y = iv_expand(b->y, delta);
    if (iv_size(b->z) < delta) b->z = iv_expand(b->z, delta);
}
static Box box_from_iv(Iv x, Iv y, Iv z) { Box b; b.x = x; b.y = y; b.z = z; box_pad(&b); return b; } /* :15-19 */
static Box box_empty(void) { return box_from_iv(iv(INFINITY, -INFINITY), iv(INFINITY, -INFINITY), iv(INFINITY, -INFINITY)); } /* :188 */
static Box box_default(void) { Box b; b.x = b.y = b.z = iv(INFINITY, -INFINITY); return b; }        /* :13 */
static Box box_from_points(V3 a, V3 b) {                                             /* :28-35 */
    Box r;
    r.x = iv(fminf(a.e[0], b.e[0]), fmaxf(a.e[0], b.e[0]));
    r.y = iv(fminf(a.e[1], b.e[1]), fmaxf(a.e[1], b.e[1]));
    r.z = iv(fminf(a.e[2], b.e[2]), fmaxf(a.e[2], b.e[2]));
    box_pad(&r);
    return r;
}
static void box_expand_pt(Box* b, V3 p) {                                             /* :51-59 (no pad) */
    b->x.min = fminf(b->x.min, p.e[0]); b->x.max = fmaxf(b->x.max, p.e[0]);
    b->y.min = fminf(b->y.min, p.e[1]); b->y.max = fmaxf(b->y.max, p.e[1]);
    b->z.min = fminf(b->z.min, p.e[2]); b->z.max = fmaxf(b->z.max, p.e[2]);
}
static void box_expand_box(Box* b, const Box* o) {                                    /* :83-89 (pads) */
    b->x = iv(fminf(b->x.min, o->x.min), fmaxf(b->x.max, o->x.max));
    b->y = iv(fminf(b->y.min, o->y.min), fmaxf(b->y.max, o->y.max));
    b->z = iv(fminf(b->z.min, o->z.min), fmaxf(b->z.max, o->z.max));
    box_pad(b);
}
static Box box_combine(const Box* a, const Box* b) {                                  /* :91-98 */
    return box_from_iv(iv(fminf(a->x.min, b->x.min), fmaxf(a->x.max, b->x.max)),
                       iv(fminf(a->y.min, b->y.min), fmaxf(a->y.max, b->y.max)),
                       iv(fminf(a->z.min, b->z.min), fmaxf(a->z.max, b->z.max)));
}
static float box_area(const Box* b) {                                                 /* :74-81 */
    float ex = iv_size(b->x), ey = iv_size(b->y), ez = iv_size(b->z);
    return 2.0f * (ex * ey + ey * ez + ez * ex);
}
typedef struct { V3 o, d; } Ray;
static inline V3 ray_at(const Ray* r, float t) { return vadd(r->o, smul(t, r->d)); }  /* Ray.cuh:18-21 */

static int box_hit(const Box* b, const Ray* r, Iv rt) {                              /* AABB.cuh:123-146 */
    V3 invD = v3(1.0f / r->d.e[0], 1.0f / r->d.e[1], 1.0f / r->d.e[2]);
    V3 t0s = vmul(vsub(v3(b->x.min, b->y.min, b->z.min), r->o), invD);
    V3 t1s = vmul(vsub(v3(b->x.max, b->y.max, b->z.max), r->o), invD);
    float tmin = fmaxf(fmaxf(fminf(t0s.e[0], t1s.e[0]), fminf(t0s.e[1], t1s.e[1])), fminf(t0s.e[2], t1s.e[2]));
    float tmax = fminf(fminf(fmaxf(t0s.e[0], t1s.e[0]), fmaxf(t0s.e[1], t1s.e[1])), fmaxf(t0s.e[2], t1s.e[2]));
    tmin = fmaxf(tmin, rt.min);
    tmax = fminf(tmax, rt.max);
    if (tmax <= tmin) return 0;
    return 1;
}

/* --------------------------------------------------------------- HitInfo */
typedef struct { V3 p, n; uint32_t mat; float t; int front; } Hit;   /* HitInfo.cuh:6-17 */
static inline void set_face_normal(Hit* h, const Ray* r, V3 outward) {
    h->front = dot3(r->d, outward) < 0;
    h->n = h->front ? outward : vneg(outward);
}

/* ---------------------------------------------------------------- XORWOW */
/* cuRAND XORWOW (CUDA 12.5 curand_kernel.h), see header comment.  The linear
 * map A on v[5] is captured as 160 columns of 5 words (rocRAND's layout:
 * m[(word*32+bit)*5 + k]).  seq[k] = A^(2^67 * 4^k). */
typedef struct { uint32_t v[5]; uint32_t d; } Rng;
static uint32_t g_seq[32][800];
static int g_seq_ready = 0;
static pthread_mutex_t g_seq_mu = PTHREAD_MUTEX_INITIALIZER;

static void xw_step_lin(uint32_t v[5]) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}
static void mat_vec(const uint32_t* m, uint32_t v[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 32; j++)
            if (v[i] & (1u << j))
                for (int k = 0; k < 5; k++) r[k] ^= m[(i * 32 + j) * 5 + k];
    memcpy(v, r, sizeof r);
}
static void mat_mul(const uint32_t* b, const uint32_t* a, uint32_t* c) { /* c = b∘a */
    for (int col = 0; col < 160; col++) {
        uint32_t v[5];
        memcpy(v, a + col * 5, sizeof v);
        mat_vec(b, v);
        memcpy(c + col * 5, v, sizeof v);
    }
}
static void build_seq_tables(void) {
    pthread_mutex_lock(&g_seq_mu);
    if (!g_seq_ready) {
        static uint32_t m[800], t[800];
        for (int col = 0; col < 160; col++) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[col / 32] = 1u << (col % 32);
            xw_step_lin(v);
            memcpy(m + col * 5, v, sizeof v);
        }
        for (int s = 0; s < 67; s++) { mat_mul(m, m, t); memcpy(m, t, sizeof m); }
        memcpy(g_seq[0], m, sizeof m);
        for (int k = 1; k < 32; k++) {
            mat_mul(g_seq[k - 1], g_seq[k - 1], t);
            mat_mul(t, t, g_seq[k]);
        }
        g_seq_ready = 1;
    }
    pthread_mutex_unlock(&g_seq_mu);
}
static void rng_init(Rng* s, unsigned long long seed, unsigned long long subseq) {
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    s->d = 6615241u + t1 + t0;
    s->v[0] = 123456789u + t0;
    s->v[1] = 362436069u ^ t0;
    s->v[2] = 521288629u + t1;
    s->v[3] = 88675123u ^ t1;
    s->v[4] = 5783321u + t0;
    for (int k = 0; subseq; k++, subseq >>= 2)
        for (unsigned q = 0; q < (unsigned)(subseq & 3u); q++) mat_vec(g_seq[k], s->v);
}
static inline uint32_t rng_next(Rng* s) {
    uint32_t t = s->v[0] ^ (s->v[0] >> 2);
    s->v[0] = s->v[1]; s->v[1] = s->v[2]; s->v[2] = s->v[3]; s->v[3] = s->v[4];
    s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
    s->d += 362437u;
    return s->v[4] + s->d;
}
static inline float curand_uniform(Rng* s) {
    const float inv = 2.3283064e-10f;
    return (float)rng_next(s) * inv + (inv / 2.0f);
}

/* --------------------------------------------------------------- Utility */
/* Core/Utility.cuh */
static inline float rand_range(float mn, float mx, Rng* s) { return mn + (mx - mn) * curand_uniform(s); } /* :168-171 */
static V3 rand_vec(float mn, float mx, Rng* s) {                                       /* :188-193 */
    float a = rand_range(mn, mx, s);
    float b = rand_range(mn, mx, s);
    float c = rand_range(mn, mx, s);
    return v3(a, b, c);
}
static V3 rand_in_unit_sphere(Rng* s) {                                                /* :195-203 */
    for (;;) {
        V3 p = rand_vec(-1, 1, s);
        if (len2(p) >= 1) continue;
        return p;
    }
}
static V3 rand_in_unit_disk(Rng* s) {                                                  /* :205-212 */
    for (;;) {
        float a = rand_range(-1, 1, s);
        float b = rand_range(-1, 1, s);
        V3 p = v3(a, b, 0);
        if (len2(p) >= 1) continue;
        return p;
    }
}
static V3 rand_unit_vector(Rng* s) { return unitv(rand_in_unit_sphere(s)); }           /* :223-226 */

/* ------------------------------------------------------------- Materials */
/* Core/Material.cuh */
enum { MT_LAMBERTIAN = 0, MT_METAL = 1, MT_DIELECTRIC = 2, MT_LIGHT = 3 };
typedef struct { int type; V3 albedo, emission; float roughness, ior; } Mat;

static float pow5i(float a) {       /* pow(float,int) with b = 5: exponentiation by squaring */
    unsigned e = 5; float r = 1.0f;
    for (;;) {
        if (e & 1u) r = r * a;
        e >>= 1;
        if (!e) return r;
        a = a * a;
    }
}
static float schlick(float cosine, float ref_idx) {                                     /* :132-137 */
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * pow5i(1 - cosine);
}
/* returns 1 if scattered, 0 if the path returns emit() */
static int mat_scatter(const Mat* m, const Ray* in, const Hit* h, V3* att, Ray* out, Rng* s) {
    switch (m->type) {
    case MT_LAMBERTIAN: {                                                                /* :66-77 */
        V3 sd = vadd(h->n, rand_unit_vector(s));
        if (near_zero(sd)) sd = h->n;
        out->o = h->p; out->d = sd; *att = m->albedo;
        return 1;
    }
    case MT_METAL: {                                                                     /* :89-96 */
        V3 refl = reflect3(in->d, h->n);
        refl = vadd(unitv(refl), smul(m->roughness, rand_unit_vector(s)));
        out->o = h->p; out->d = refl; *att = m->albedo;
        return dot3(out->d, h->n) > 0;
    }
    case MT_DIELECTRIC: {                                                                /* :109-128 */
        *att = v3(1.0f, 1.0f, 1.0f);
        float ri = h->front ? (1.0f / m->ior) : m->ior;
        V3 ud = unitv(in->d);
        double cos_theta = fminf(dot3(vneg(ud), h->n), 1.0f);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        int cannot_refract = (double)ri * sin_theta > 1.0;
        V3 dir;
        if (cannot_refract || schlick((float)cos_theta, ri) > curand_uniform(s))
            dir = reflect3(ud, h->n);
        else
            dir = refract3(ud, h->n, ri);
        out->o = h->p; out->d = dir;
        return 1;
    }
    default:                                                                             /* :51, :139-146 */
        return 0;
    }
}
static V3 mat_emit(const Mat* m) { return m->type == MT_LIGHT ? m->emission : v3(0, 0, 0); } /* :53-55, :144 */

/* ------------------------------------------------------------ BVH nodes */
/* Core/BVHNode.cuh:9-166 (the subset used by Mesh and the scene) */
typedef struct { Box box; int left, right, obj_index, obj_count, is_leaf; } Node;

/* ------------------------------------------------------------------ Mesh */
/* Core/Mesh.cuh:14-309 */
typedef struct {
    const float* verts;     /* positions, 3 floats per vertex slot (m_Vertices + vertexOffset) */
    uint32_t* idx;          /* m_Indices + indexOffset (permuted in place by the builder) */
    int32_t* fmat;          /* m_FaceMaterialIds + faceMatOffset (permuted) */
    uint32_t n_verts, n_idx, matid_off;
    Box box;
    Node* bvh;
    int n_nodes;
} Mesh;

static inline V3 mesh_pos(const Mesh* m, uint32_t i) { return v3(m->verts[3 * i], m->verts[3 * i + 1], m->verts[3 * i + 2]); }
static V3 tri_centroid(const Mesh* m, int i) {                                             /* :251-256 */
    V3 p0 = mesh_pos(m, m->idx[i]), p1 = mesh_pos(m, m->idx[i + 1]), p2 = mesh_pos(m, m->idx[i + 2]);
    return muls(vadd(vadd(p0, p1), p2), 1.f / 3.f);
}
static void expand_tri(const Mesh* m, Box* b, int i) {                                       /* :242-249 */
    box_expand_pt(b, mesh_pos(m, m->idx[i]));
    box_expand_pt(b, mesh_pos(m, m->idx[i + 1]));
    box_expand_pt(b, mesh_pos(m, m->idx[i + 2]));
}
static Box tris_aabb(const Mesh* m, int start, int count) {                                  /* :258-264 */
    Box b = box_empty();
    for (int i = start; i < start + count; i += 3) expand_tri(m, &b, i);
    return b;
}
static float eval_sah(const Mesh* m, int axis, float pos, int start, int end) {              /* :222-240 */
    Box lb = box_empty(), rb = box_empty();
    int lc = 0, rc = 0;
    for (int i = start; i < end; i += 3) {
        V3 c = tri_centroid(m, i);
        if (c.e[axis] < pos) { lc++; expand_tri(m, &lb, i); }
        else { rc++; expand_tri(m, &rb, i); }
    }
    float cost = (float)lc * box_area(&lb) + (float)rc * box_area(&rb);
    return cost < 1e-8f ? 1e-8f : cost;
}
#define MAX_STACK_SIZE 64
static int mesh_build(Mesh* m) {                                                             /* :18-53, :121-219 */
    if (m->n_verts > 0) {
        m->box = box_empty();
        for (uint32_t i = 0; i < m->n_verts; ++i) box_expand_pt(&m->box, mesh_pos(m, i));
    } else {
        m->box = box_default();
    }
    int ntri = (int)(m->n_idx / 3);
    int max_nodes = 2 * ntri - 1;
    if (max_nodes < 1) max_nodes = 1;
    m->bvh = (Node*)calloc((size_t)max_nodes, sizeof(Node));
    if (!m->bvh) return -1;
    struct { int start, end, node; } st[MAX_STACK_SIZE];
    int top = 0, next = 0;
    Node* root = &m->bvh[next++];
    root->box = m->box; root->obj_index = 0; root->obj_count = (int)m->n_idx; root->is_leaf = 0;
    st[top].start = 0; st[top].end = (int)m->n_idx; st[top].node = 0; top++;
    while (top > 0) {
        --top;
        int start = st[top].start, end = st[top].end, ni = st[top].node;
        Node* node = &m->bvh[ni];
        int span = end - start;
        if (span <= 30 || (next + 1) >= max_nodes) {
            node->is_leaf = 1; node->obj_index = start; node->obj_count = span;
            node->box = tris_aabb(m, start, span);
            continue;
        }
        int best_axis = 0; float best_pos = 0.f, best_cost = 1e30f;
        for (int axis = 0; axis < 3; axis++) {
            float mn = 1e30f, mx = -1e30f;
            for (int i = start; i < end; i += 3) {
                V3 c = tri_centroid(m, i);
                if (c.e[axis] < mn) mn = c.e[axis];
                if (c.e[axis] > mx) mx = c.e[axis];
            }
            float mid = 0.5f * (mn + mx);
            float cost = eval_sah(m, axis, mid, start, end);
            if (cost < best_cost) { best_cost = cost; best_axis = axis; best_pos = mid; }
        }
        int mid = start;
        for (int i = start; i < end; i += 3) {
            V3 c = tri_centroid(m, i);
            if (c.e[best_axis] < best_pos) {
                uint32_t a0 = m->idx[mid], a1 = m->idx[mid + 1], a2 = m->idx[mid + 2];  /* Core.cuh:25-39 */
                m->idx[mid] = m->idx[i]; m->idx[mid + 1] = m->idx[i + 1]; m->idx[mid + 2] = m->idx[i + 2];
                m->idx[i] = a0; m->idx[i + 1] = a1; m->idx[i + 2] = a2;
                int fl = mid / 3, fr = i / 3;
                int32_t tmp = m->fmat[fl]; m->fmat[fl] = m->fmat[fr]; m->fmat[fr] = tmp;
                mid += 3;
            }
        }
        node->left = next++;
        node->right = next++;
        node->is_leaf = 0;
        if (top + 2 > MAX_STACK_SIZE) return -2;   /* the reference overflows its stack here */
        st[top].start = mid; st[top].end = end; st[top].node = node->right; top++;
        st[top].start = start; st[top].end = mid; st[top].node = node->left; top++;
    }
    for (int i = next - 1; i >= 0; i--) {
        Node* nd = &m->bvh[i];
        if (!nd->is_leaf) {
            Box bl = m->bvh[nd->left].box, br = m->bvh[nd->right].box;
            nd->box = box_combine(&bl, &br);
        }
    }
    m->n_nodes = next;
    return 0;
}

typedef struct { unsigned long long rays, nodes, tris, spheres; } Counters;

static int tri_hit(const Mesh* m, const Ray* r, V3 v0, V3 v1, V3 v2, Iv rt, Hit* rec, int base) { /* :266-308 */
    const float EPSILON = 1e-8f;
    V3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    V3 h = cross3(r->d, e2);
    float a = dot3(e1, h);
    if (fabsf(a) < EPSILON) return 0;
    float f = 1.f / a;
    V3 s = vsub(r->o, v0);
    float u = f * dot3(s, h);
    if (u < 0.f || u > 1.f) return 0;
    V3 q = cross3(s, e1);
    float v = f * dot3(r->d, q);
    if (v < 0.f || (u + v) > 1.f) return 0;
    float t = f * dot3(e2, q);
    if (t < rt.min || t > rt.max) return 0;
    rec->t = t;
    rec->p = ray_at(r, t);
    rec->mat = (uint32_t)(m->fmat[base / 3] + (int32_t)m->matid_off);
    V3 n = unitv(cross3(e1, e2));
    set_face_normal(rec, r, n);
    return 1;
}
static int mesh_hit(const Mesh* m, const Ray* r, Iv rt, Hit* rec, Counters* cn) {           /* :55-110 */
    int any = 0;
    float closest = rt.max;
    uint32_t stack[MAX_STACK_SIZE];
    int sp = 0, ni = 0;
    for (;;) {
        const Node* node = &m->bvh[ni];
        Hit tmp;
        cn->nodes++;
        if (box_hit(&node->box, r, iv(rt.min, closest))) {
            if (!node->is_leaf) {
                stack[sp++] = (uint32_t)node->right;
                ni = node->left;
                continue;
            }
            for (int i = node->obj_index; i < node->obj_index + node->obj_count; i += 3) {
                V3 v0 = mesh_pos(m, m->idx[i]), v1 = mesh_pos(m, m->idx[i + 1]), v2 = mesh_pos(m, m->idx[i + 2]);
                cn->tris++;
                if (tri_hit(m, r, v0, v1, v2, iv(rt.min, closest), &tmp, i)) {
                    any = 1; closest = tmp.t; rt.max = closest; *rec = tmp;
                }
            }
        }
        if (sp == 0) break;
        ni = (int)stack[--sp];
    }
    return any;
}

/* ---------------------------------------------------------------- Sphere */
/* Core/Sphere.cuh:6-53 */
typedef struct { V3 c; float r, r2; uint32_t mat; Box box; } Sphere;
static Sphere make_sphere(V3 c, float rad, int mat) {                                        /* :20-25 */
    Sphere s; s.c = c; s.r = rad; s.r2 = rad * rad; s.mat = (uint32_t)mat;
    V3 rv = v3(rad, rad, rad);
    s.box = box_from_points(vsub(c, rv), vadd(c, rv));
    return s;
}
static int sphere_hit(const Sphere* sp, const Ray* r, Iv rt, Hit* rec) {                     /* :27-47 */
    V3 oc = vsub(r->o, sp->c);
    float a = dot3(r->d, r->d);
    float hb = dot3(oc, r->d);
    float c = dot3(oc, oc) - sp->r2;
    float disc = hb * hb - a * c;
    if (disc < 0) return 0;
    float sq = sqrtf(disc);
    float root = (-hb - sq) / a;
    if (root < rt.min || root > rt.max) {
        root = (-hb + sq) / a;
        if (root < rt.min || root > rt.max) return 0;
    }
    rec->t = root;
    rec->p = ray_at(r, rec->t);
    rec->mat = sp->mat;
    V3 on = vdiv(vsub(rec->p, sp->c), sp->r);
    set_face_normal(rec, r, on);
    return 1;
}

/* ----------------------------------------------------------------- Scene */
typedef struct { int is_mesh; int index; } Obj;
typedef struct {
    int n_meshes;
    Mesh* meshes;
    float* verts;          /* owned copies */
    uint32_t* idx;
    int32_t* fmat;
    int n_spheres;
    Sphere spheres[2];
    int n_obj;
    Obj objs[500];
    int n_mat;
    Mat mats[500];
    Node* snodes;
    int n_snodes;
} Scene;

static Box obj_box(const Scene* sc, int i) {
    const Obj* o = &sc->objs[i];
    return o->is_mesh ? sc->meshes[o->index].box : sc->spheres[o->index].box;
}
static int obj_hit(const Scene* sc, int i, const Ray* r, Iv rt, Hit* rec, Counters* cn) {
    const Obj* o = &sc->objs[i];
    if (o->is_mesh) return mesh_hit(&sc->meshes[o->index], r, rt, rec, cn);
    cn->spheres++;
    return sphere_hit(&sc->spheres[o->index], r, rt, rec);
}
static void build_scene_bvh(Scene* sc) {                                                   /* BVHNode.cuh:21-84 */
    int n = sc->n_obj;
    sc->snodes = (Node*)calloc((size_t)(2 * n - 1), sizeof(Node));
    struct { int start, end, node; } st[MAX_STACK_SIZE];
    int top = 0, next = 0;
    st[top].start = 0; st[top].end = n; st[top].node = 0; top++;
    while (top > 0) {
        --top;
        int start = st[top].start, end = st[top].end, ni = st[top].node;
        Node* node = &sc->snodes[ni];
        memset(node, 0, sizeof *node);
        int span = end - start;
        node->box = box_empty();
        for (int i = start; i < end; i++) { Box b = obj_box(sc, i); box_expand_box(&node->box, &b); }
        if (span == 1) {
            node->obj_index = start; node->obj_count = 1; node->is_leaf = 1;
        } else {
            int mid = start + span / 2;
            int l = ++next, rr = ++next;
            node->left = l; node->right = rr; node->is_leaf = 0;
            st[top].start = mid; st[top].end = end; st[top].node = rr; top++;
            st[top].start = start; st[top].end = mid; st[top].node = l; top++;
        }
    }
    sc->n_snodes = next + 1;
}
static int scene_hit(const Scene* sc, const Ray* r, Iv rt, Hit* rec, Counters* cn) {        /* BVHNode.cuh:115-156 */
    int any = 0;
    float closest = rt.max;
    uint32_t stack[MAX_STACK_SIZE / 2];
    int sp = 0, ni = 0;
    for (;;) {
        const Node* node = &sc->snodes[ni];
        cn->nodes++;
        if (box_hit(&node->box, r, rt)) {
            if (node->is_leaf) {
                Hit tmp;
                if (obj_hit(sc, node->obj_index, r, iv(rt.min, closest), &tmp, cn)) {
                    any = 1; closest = tmp.t; *rec = tmp;
                }
                if (sp == 0) break;
                ni = (int)stack[--sp];
            } else {
                stack[sp++] = (uint32_t)node->right;
                ni = node->left;
            }
        } else {
            if (sp == 0) break;
            ni = (int)stack[--sp];
        }
    }
    return any;
}

/* ---------------------------------------------------------------- Camera */
/* Core/Camera.cuh:18-44, :159-182 */
typedef struct {
    V3 pos, front, up, right, world_up;
    float yaw, pitch, aspect, vfov, aperture, focus;
    V3 llc, horiz, vert;
    float lens_r;
    int spp; float scale;
} Cam;
static void cam_update(Cam* c) {
    const float PI = 3.1415926535897932385f;
    V3 front;
    front.e[0] = -cosf(c->yaw * PI / 180.0f) * cosf(c->pitch * PI / 180.0f);
    front.e[1] = -sinf(c->pitch * PI / 180.0f);
    front.e[2] = -sinf(c->yaw * PI / 180.0f) * cosf(c->pitch * PI / 180.0f);
    c->front = unitv(front);
    c->right = unitv(cross3(c->front, c->world_up));
    c->up = unitv(cross3(c->right, c->front));
    float theta = c->vfov * PI / 180.0f;
    float h = tanf(theta / 2.0f);
    float vh = 2.0f * h;
    float vw = c->aspect * vh;
    c->horiz = smul(c->focus * vw, c->right);
    c->vert = smul(c->focus * vh, c->up);
    c->llc = vsub(vsub(vsub(c->pos, vdiv(c->horiz, 2.0f)), vdiv(c->vert, 2.0f)), smul(c->focus, c->front));
    c->lens_r = c->aperture / 2.0f;
}
static Ray cam_get_ray(const Cam* c, int px, int py, int w, int h, Rng* s) {
    V3 rd = smul(c->lens_r, rand_in_unit_disk(s));
    V3 off = vadd(muls(c->right, rd.e[0]), muls(c->up, rd.e[1]));
    float u = ((float)px + curand_uniform(s)) / (float)w;
    float v = ((float)py + curand_uniform(s)) / (float)h;
    Ray r;
    r.o = vadd(c->pos, off);
    r.d = vsub(vsub(vadd(vadd(c->llc, smul(u, c->horiz)), smul(v, c->vert)), c->pos), off);
    return r;
}

/* ------------------------------------------------------------- rayColor */
static V3 sky(const Ray* r) {                                                              /* CRTUtility.cuh:34-38 */
    V3 ud = unitv(r->d);
    float t = 0.5f * (ud.e[1] + 1.0f);
    return vadd(smul(1.0f - t, v3(1.0f, 1.0f, 1.0f)), smul(t, v3(0.5f, 0.7f, 1.0f)));
}
static V3 ray_color(const Scene* sc, Ray cur, int max_bounces, Rng* s, Counters* cn) {    /* CUDAKernels.h:102-145 */
    V3 acc = v3(1.0f, 1.0f, 1.0f);
    V3 fin = v3(0.0f, 0.0f, 0.0f);
    const int MIN_BOUNCES = 3;
    const float MAX_PROB = 0.95f;
    for (int b = 0; b < max_bounces; b++) {
        Hit rec;
        if (b >= MIN_BOUNCES) {
            float p = fmaxf(acc.e[0], fmaxf(acc.e[1], acc.e[2]));
            p = fminf(p, MAX_PROB);
            if (curand_uniform(s) > p) break;
            acc = smul(1 / p, acc);   /* operator/= : *this *= 1 / t */
        }
        cn->rays++;
        if (scene_hit(sc, &cur, iv(0.001f, INFINITY), &rec, cn)) {
            Ray sc_ray; V3 att;
            if (rec.mat < (uint32_t)sc->n_mat) {
                const Mat* m = &sc->mats[rec.mat];
                if (mat_scatter(m, &cur, &rec, &att, &sc_ray, s)) {
                    acc = vmul(acc, att);
                    cur = sc_ray;
                } else {
                    return mat_emit(m);
                }
            }
        } else {
            fin = vmul(acc, sky(&cur));
            break;
        }
    }
    return fin;
}

/* ------------------------------------------------------------ writeColor */
static inline float lin_to_gamma(float c) { double x = c; return (float)(x > 0 ? sqrt(x) : 0); } /* CRTUtility.cuh:14-19 */
static inline unsigned char to_u8(float x) {                                                     /* :21-32 */
    if (x < 0.000f) x = 0.000f;
    else if (x > 0.999f) x = 0.999f;
    return (unsigned char)(256 * x);
}

/* =================================================================== API */
EXPORT int oracle_abi_version(void) { return 1; }

EXPORT void oracle_seq_matrix(int k, uint32_t* out800) { build_seq_tables(); memcpy(out800, g_seq[k], sizeof g_seq[k]); }

EXPORT void oracle_rng_init(unsigned long long seed, unsigned long long subseq, uint32_t* state6) {
    build_seq_tables();
    Rng s; rng_init(&s, seed, subseq);
    memcpy(state6, s.v, 20); state6[5] = s.d;
}
EXPORT void oracle_rng_draw(uint32_t* state6, int n, uint32_t* out_u32, float* out_f) {
    Rng s; memcpy(s.v, state6, 20); s.d = state6[5];
    for (int i = 0; i < n; i++) {
        Rng c = s;
        if (out_f) out_f[i] = curand_uniform(&c);
        uint32_t x = rng_next(&s);
        if (out_u32) out_u32[i] = x;
    }
    memcpy(state6, s.v, 20); state6[5] = s.d;
}

/* mesh_info: per mesh 6 u32: vertexOffset, vertexCount, indexOffset, indexCount, faceMatOffset, matIDOffset
 * (SceneManager.h:125-195).  matdata: per material 9 floats: type, albedo3, emission3, roughness, ior
 * (Material.cuh:16-47).  Returns 0 on success. */
EXPORT int oracle_scene_create(int n_meshes, const float* positions, unsigned long long n_vert_total,
                               const uint32_t* indices, unsigned long long n_idx_total,
                               const int32_t* facemat, unsigned long long n_face_total,
                               const uint32_t* mesh_info, int n_mat, const float* matdata, void** out) {
    build_seq_tables();
    Scene* sc = (Scene*)calloc(1, sizeof(Scene));
    if (!sc) return -1;
    sc->n_meshes = n_meshes;
    sc->meshes = (Mesh*)calloc((size_t)(n_meshes > 0 ? n_meshes : 1), sizeof(Mesh));
    sc->verts = (float*)malloc(sizeof(float) * 3 * (n_vert_total ? n_vert_total : 1));
    sc->idx = (uint32_t*)malloc(sizeof(uint32_t) * (n_idx_total ? n_idx_total : 1));
    sc->fmat = (int32_t*)malloc(sizeof(int32_t) * (n_face_total ? n_face_total : 1));
    memcpy(sc->verts, positions, sizeof(float) * 3 * n_vert_total);
    memcpy(sc->idx, indices, sizeof(uint32_t) * n_idx_total);
    memcpy(sc->fmat, facemat, sizeof(int32_t) * n_face_total);
    /* createRandomWorld (CUDAKernels.h:56-84) */
    for (int i = 0; i < n_mat && sc->n_mat < 500; i++) {            /* createMaterialsKernel :28-54 */
        const float* d = matdata + 9 * i;
        Mat m; memset(&m, 0, sizeof m);
        m.type = (int)d[0];
        m.albedo = v3(d[1], d[2], d[3]);
        m.emission = v3(d[4], d[5], d[6]);
        m.roughness = d[7] < 1.f ? d[7] : 1.f;                        /* Metal ctor, Material.cuh:86 */
        m.ior = d[8];
        sc->mats[sc->n_mat++] = m;
    }
    for (int i = 0; i < n_meshes; i++) {
        const uint32_t* mi = mesh_info + 6 * i;
        Mesh* m = &sc->meshes[i];
        m->verts = sc->verts + 3 * (size_t)mi[0];
        m->n_verts = mi[1];
        m->idx = sc->idx + mi[2];
        m->n_idx = mi[3];
        m->fmat = sc->fmat + mi[4];
        m->matid_off = mi[5];
        int rc = mesh_build(m);
        if (rc) return rc;
        sc->objs[sc->n_obj].is_mesh = 1; sc->objs[sc->n_obj].index = i; sc->n_obj++;
    }
    Mat g; memset(&g, 0, sizeof g); g.type = MT_LAMBERTIAN; g.albedo = v3(0.5f, 0.5f, 0.5f);
    int gi = sc->n_mat; sc->mats[sc->n_mat++] = g;
    sc->spheres[0] = make_sphere(v3(0, -1000, 0), 999, gi);
    sc->objs[sc->n_obj].is_mesh = 0; sc->objs[sc->n_obj].index = 0; sc->n_obj++;
    Mat mt; memset(&mt, 0, sizeof mt); mt.type = MT_METAL; mt.albedo = v3((float)0.7, (float)0.6, (float)0.5); mt.roughness = 0.0f;
    int mti = sc->n_mat; sc->mats[sc->n_mat++] = mt;
    sc->spheres[1] = make_sphere(v3((float)0.2, (float)0.2, 0), 0.05f, mti);
    sc->objs[sc->n_obj].is_mesh = 0; sc->objs[sc->n_obj].index = 1; sc->n_obj++;
    sc->n_spheres = 2;
    build_scene_bvh(sc);
    *out = sc;
    return 0;
}
EXPORT void oracle_scene_destroy(void* p) {
    Scene* sc = (Scene*)p;
    if (!sc) return;
    for (int i = 0; i < sc->n_meshes; i++) free(sc->meshes[i].bvh);
    free(sc->meshes); free(sc->verts); free(sc->idx); free(sc->fmat); free(sc->snodes); free(sc);
}
/* Node dump: per node 6 floats box + 5 ints (left,right,obj_index,obj_count,is_leaf). which=-1: scene BVH. */
EXPORT int oracle_scene_nodes(void* p, int which, float* boxes, int32_t* ints) {
    Scene* sc = (Scene*)p;
    const Node* nodes = which < 0 ? sc->snodes : sc->meshes[which].bvh;
    int n = which < 0 ? sc->n_snodes : sc->meshes[which].n_nodes;
    if (boxes && ints)
        for (int i = 0; i < n; i++) {
            const Box* b = &nodes[i].box;
            float* o = boxes + 6 * i;
            o[0] = b->x.min; o[1] = b->y.min; o[2] = b->z.min; o[3] = b->x.max; o[4] = b->y.max; o[5] = b->z.max;
            int32_t* q = ints + 5 * i;
            q[0] = nodes[i].left; q[1] = nodes[i].right; q[2] = nodes[i].obj_index; q[3] = nodes[i].obj_count; q[4] = nodes[i].is_leaf;
        }
    return n;
}
EXPORT void oracle_scene_mesh_arrays(void* p, int which, uint32_t* idx_out, int32_t* fmat_out, float* box6) {
    Scene* sc = (Scene*)p;
    const Mesh* m = &sc->meshes[which];
    if (idx_out) memcpy(idx_out, m->idx, sizeof(uint32_t) * m->n_idx);
    if (fmat_out) memcpy(fmat_out, m->fmat, sizeof(int32_t) * (m->n_idx / 3));
    if (box6) { box6[0] = m->box.x.min; box6[1] = m->box.y.min; box6[2] = m->box.z.min; box6[3] = m->box.x.max; box6[4] = m->box.y.max; box6[5] = m->box.z.max; }
}

/* Camera ctor + updateCameraVectors (host trig).  out: 19 floats
 * origin3, llc3, horizontal3, vertical3, right3, up3, lens_radius. */
EXPORT void oracle_camera(float aspect, float vfov, const float* pos3, const float* up3, float aperture,
                          float focus, float yaw, float pitch, float* out19) {
    Cam c; memset(&c, 0, sizeof c);
    c.aspect = aspect; c.vfov = vfov; c.pos = v3(pos3[0], pos3[1], pos3[2]);
    c.aperture = aperture; c.focus = focus; c.world_up = v3(up3[0], up3[1], up3[2]);
    c.yaw = yaw; c.pitch = pitch;
    cam_update(&c);
    const V3* vs[6] = {&c.pos, &c.llc, &c.horiz, &c.vert, &c.right, &c.up};
    for (int i = 0; i < 6; i++) memcpy(out19 + 3 * i, vs[i]->e, 12);
    out19[18] = c.lens_r;
}

typedef struct {
    const Scene* sc; Cam cam; int w, h, spp, bounces; unsigned long long seed, subseq_base;
    int x0, y0, x1, y1;
    uint32_t* rng;   /* optional per-pixel XORWOW state (w*h*6: v[5], d), continued and stored back */
    float* sum; unsigned char* rgba; float scale;
    int next_row; pthread_mutex_t mu; Counters total;
} Job;

static void* worker(void* arg) {
    Job* j = (Job*)arg;
    Counters cn; memset(&cn, 0, sizeof cn);
    int rw = j->x1 - j->x0;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int y = j->next_row++;
        pthread_mutex_unlock(&j->mu);
        if (y >= j->y1) break;
        for (int x = j->x0; x < j->x1; x++) {                         /* CUDAKernels.h:147-166 */
            int pixel = y * j->w + x;
            Rng s;
            if (j->rng) memcpy(&s, j->rng + 6 * (size_t)pixel, sizeof s);   /* state persists (CUDAKernels.h:151,165) */
            else rng_init(&s, j->seed, j->subseq_base + (unsigned long long)pixel);
            V3 pc = v3(0, 0, 0);
            for (int smp = 0; smp < j->spp; smp++) {
                Ray r = cam_get_ray(&j->cam, x, y, j->w, j->h, &s);
                pc = vadd(pc, ray_color(j->sc, r, j->bounces, &s, &cn));
            }
            if (j->rng) memcpy(j->rng + 6 * (size_t)pixel, &s, sizeof s);
            size_t o = (size_t)(y - j->y0) * rw + (x - j->x0);
            if (j->sum) { j->sum[3 * o] = pc.e[0]; j->sum[3 * o + 1] = pc.e[1]; j->sum[3 * o + 2] = pc.e[2]; }
            if (j->rgba) {
                V3 c = smul(j->scale, pc);
                j->rgba[4 * o] = to_u8(lin_to_gamma(c.e[0]));
                j->rgba[4 * o + 1] = to_u8(lin_to_gamma(c.e[1]));
                j->rgba[4 * o + 2] = to_u8(lin_to_gamma(c.e[2]));
                j->rgba[4 * o + 3] = 255;
            }
        }
    }
    pthread_mutex_lock(&j->mu);
    j->total.rays += cn.rays; j->total.nodes += cn.nodes; j->total.tris += cn.tris; j->total.spheres += cn.spheres;
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

/* Render the sub-rectangle [x0,x1)x[y0,y1) of a w x h frame, spp samples per pixel,
 * RNG subsequence = subseq_base + y*w + x (CUDAKernels.h:18-26).  cam19 as from
 * oracle_camera.  sum_out: (y1-y0)*(x1-x0)*3 linear sums (pixel_color before
 * m_PixelSampleScale); rgba_out: writeColor(scale * sum) with scale = 1.f/spp_total.
 * counters_out (4 u64): rays, box tests, triangle tests, sphere tests. */
static int render_job(void* scene, const float* cam19, int w, int h, int spp, int spp_total, int max_bounces,
                      unsigned long long seed, unsigned long long subseq_base, uint32_t* rng, int x0, int y0, int x1,
                      int y1, int nthreads, float* sum_out, unsigned char* rgba_out, unsigned long long* counters_out) {
    build_seq_tables();
    Job j; memset(&j, 0, sizeof j);
    j.sc = (const Scene*)scene;
    memcpy(j.cam.pos.e, cam19, 12); memcpy(j.cam.llc.e, cam19 + 3, 12); memcpy(j.cam.horiz.e, cam19 + 6, 12);
    memcpy(j.cam.vert.e, cam19 + 9, 12); memcpy(j.cam.right.e, cam19 + 12, 12); memcpy(j.cam.up.e, cam19 + 15, 12);
    j.cam.lens_r = cam19[18];
    j.w = w; j.h = h; j.spp = spp; j.bounces = max_bounces; j.seed = seed; j.subseq_base = subseq_base; j.rng = rng;
    j.x0 = x0; j.y0 = y0; j.x1 = x1; j.y1 = y1; j.sum = sum_out; j.rgba = rgba_out;
    j.scale = 1.f / (float)spp_total;                                   /* Camera.cuh:23,71 */
    j.next_row = y0;
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j.mu);
    if (counters_out) {
        counters_out[0] = j.total.rays; counters_out[1] = j.total.nodes;
        counters_out[2] = j.total.tris; counters_out[3] = j.total.spheres;
    }
    return 0;
}

EXPORT int oracle_render(void* scene, const float* cam19, int w, int h, int spp, int spp_total, int max_bounces,
                         unsigned long long seed, unsigned long long subseq_base, int x0, int y0, int x1, int y1,
                         int nthreads, float* sum_out, unsigned char* rgba_out, unsigned long long* counters_out) {
    return render_job(scene, cam19, w, h, spp, spp_total, max_bounces, seed, subseq_base, NULL, x0, y0, x1, y1,
                      nthreads, sum_out, rgba_out, counters_out);
}

/* One frame of the reference's render loop over persistent RNG state: rng (w*h*6 words: v[5], d per
 * pixel, from oracle_rng_init or a previous frame) is continued and stored back, like the curandState
 * array across CUDARenderer::render calls (CUDAKernels.h:151, :165).  Full frame. */
EXPORT int oracle_render_rng(void* scene, const float* cam19, int w, int h, int spp, int spp_total, int max_bounces,
                             uint32_t* rng, int nthreads, float* sum_out, unsigned char* rgba_out,
                             unsigned long long* counters_out) {
    return render_job(scene, cam19, w, h, spp, spp_total, max_bounces, 0, 0, rng, 0, 0, w, h, nthreads, sum_out,
                      rgba_out, counters_out);
}

/* ---- Camera::updateCamera (Camera.cuh:46-157): the per-frame camera controller ----
 * Input = what the reference polls from SFML: mouse position, right button, keys held
 * (bits W=1 A=2 S=4 D=8 Space=16 LControl=32 F=64) and PageUp/PageDown presses (focus_steps,
 * WindowManager.h:64-67).  updateRotation's function-local statics are fields here. */
typedef struct {
    Cam c;
    int spp; float scale;
    int moves, rotates, hq;
    int rot_init, first_mouse;
    float last_x, last_y, smooth_x, smooth_y;
} CamCtl;

EXPORT void* oracle_camctl_new(float aspect, float vfov, const float* pos3, const float* up3, float aperture,
                               float focus) {
    CamCtl* k = (CamCtl*)calloc(1, sizeof(CamCtl));
    k->c.aspect = aspect; k->c.vfov = vfov; k->c.pos = v3(pos3[0], pos3[1], pos3[2]);
    k->c.aperture = aperture; k->c.focus = focus; k->c.world_up = v3(up3[0], up3[1], up3[2]);
    k->c.yaw = -90.0f; k->c.pitch = 0.0f;                                 /* Camera.cuh:18-30 */
    cam_update(&k->c);
    k->spp = 1; k->scale = 1.0f / 1;
    k->first_mouse = 1;
    return k;
}

EXPORT void oracle_camctl_free(void* p) { free(p); }

EXPORT void oracle_camctl_update(void* p, float dt, int ww, int wh, float mx, float my, int rmb, unsigned keys,
                                 int focus_steps) {
    CamCtl* k = (CamCtl*)p;
    Cam* c = &k->c;
    for (int i = 0; i < focus_steps; i++) { c->focus = fmaxf(0.1f, c->focus + 0.1f); cam_update(c); }   /* :79-83 */
    for (int i = 0; i > focus_steps; i--) { c->focus = fmaxf(0.1f, c->focus + -0.1f); cam_update(c); }
    /* updateRotation (:88-130) */
    if (!k->rot_init) {
        k->last_x = ww / 2.0f; k->last_y = wh / 2.0f; k->smooth_x = k->last_x; k->smooth_y = k->last_y;
        k->rot_init = 1;
    }
    const float sf = 0.5f, sens = 0.2f;
    if (rmb) {
        if (k->first_mouse) {
            k->last_x = mx; k->last_y = my; k->smooth_x = mx; k->smooth_y = my; k->first_mouse = 0;
        } else {
            k->rotates = 1;
            k->smooth_x = k->smooth_x * (1 - sf) + mx * sf;
            k->smooth_y = k->smooth_y * (1 - sf) + my * sf;
            float xo = k->smooth_x - k->last_x, yo = k->smooth_y - k->last_y;
            k->last_x = k->smooth_x; k->last_y = k->smooth_y;
            xo *= -sens; yo *= -sens;
            c->yaw += xo; c->pitch += yo;
            c->pitch = fmaxf(-89.0f, fminf(89.0f, c->pitch));
        }
    } else {
        k->first_mouse = 1; k->rotates = 0;
    }
    /* updatePosition (:131-157), movement speed 1 */
    float vel = 1.0f * dt;
    V3 prev = c->pos;
    if (keys & 1u) c->pos = vsub(c->pos, muls(c->front, vel));
    if (keys & 4u) c->pos = vadd(c->pos, muls(c->front, vel));
    if (keys & 2u) c->pos = vsub(c->pos, muls(c->right, vel));
    if (keys & 8u) c->pos = vadd(c->pos, muls(c->right, vel));
    if (keys & 16u) c->pos = vadd(c->pos, muls(c->world_up, vel));
    if (keys & 32u) c->pos = vsub(c->pos, muls(c->world_up, vel));
    k->moves = !(c->pos.e[0] == prev.e[0] && c->pos.e[1] == prev.e[1] && c->pos.e[2] == prev.e[2]);
    cam_update(c);
    /* :52-71 */
    if (keys & 64u) k->hq = !k->hq;
    if (k->rotates || k->moves) { k->spp = 1; k->hq = 0; }
    else if (k->hq) k->spp = 2000;
    else k->spp = 1;
    k->scale = 1.f / k->spp;
}

/* cam19 as oracle_camera; state8 = yaw, pitch, moving, rotating, high_quality, focus, spp, pixel_sample_scale */
EXPORT void oracle_camctl_get(const void* p, float* cam19, float* state8) {
    const CamCtl* k = (const CamCtl*)p;
    const Cam* c = &k->c;
    const V3* vs[6] = {&c->pos, &c->llc, &c->horiz, &c->vert, &c->right, &c->up};
    for (int i = 0; i < 6; i++) memcpy(cam19 + 3 * i, vs[i]->e, 12);
    cam19[18] = c->lens_r;
    state8[0] = c->yaw; state8[1] = c->pitch; state8[2] = (float)k->moves; state8[3] = (float)k->rotates;
    state8[4] = (float)k->hq; state8[5] = c->focus; state8[6] = (float)k->spp; state8[7] = k->scale;
}

/* ---- Known-answer entry points for the primitive functions (golden fixtures) ----
 * Each restates the reference function exactly as the render path uses it. */

/* rayTriangleIntersect (Mesh.cuh:266-308) on n records of 17 floats: o3 d3 v0 3 v1 3 v2 3 tmin tmax.
 * out: t, or -1 when rejected. */
EXPORT void oracle_kat_triangle(const float* in, int n, float* out) {
    static const Mesh none;
    for (int i = 0; i < n; i++) {
        const float* q = in + 17 * i;
        Ray r; r.o = v3(q[0], q[1], q[2]); r.d = v3(q[3], q[4], q[5]);
        Hit h;
        Mesh m = none;
        int32_t fm = 0;
        m.fmat = &fm;
        out[i] = tri_hit(&m, &r, v3(q[6], q[7], q[8]), v3(q[9], q[10], q[11]), v3(q[12], q[13], q[14]),
                         iv(q[15], q[16]), &h, 0) ? h.t : -1.f;
    }
}

/* AABB::hit (AABB.cuh:123-146) on n records of 14 floats: o3 d3 lo3 hi3 tmin tmax (the box as stored, no
 * padding applied here).  out: 1 hit / 0 miss. */
EXPORT void oracle_kat_box(const float* in, int n, int* out) {
    for (int i = 0; i < n; i++) {
        const float* q = in + 14 * i;
        Ray r; r.o = v3(q[0], q[1], q[2]); r.d = v3(q[3], q[4], q[5]);
        Box b; b.x = iv(q[6], q[9]); b.y = iv(q[7], q[10]); b.z = iv(q[8], q[11]);
        out[i] = box_hit(&b, &r, iv(q[12], q[13]));
    }
}

/* Sphere::hit (Sphere.cuh:27-47) on n records of 12 floats: o3 d3 center3 radius tmin tmax.  out: t or -1. */
EXPORT void oracle_kat_sphere(const float* in, int n, float* out) {
    for (int i = 0; i < n; i++) {
        const float* q = in + 12 * i;
        Ray r; r.o = v3(q[0], q[1], q[2]); r.d = v3(q[3], q[4], q[5]);
        Sphere s = make_sphere(v3(q[6], q[7], q[8]), q[9], 0);
        Hit h;
        out[i] = sphere_hit(&s, &r, iv(q[10], q[11]), &h) ? h.t : -1.f;
    }
}

/* Camera::getRay (Camera.cuh:32-44) for n pixels (xy[2i], xy[2i+1]) of a w x h image; rng: 6 words per
 * pixel, continued in place.  out: o3 d3 per pixel. */
EXPORT void oracle_kat_get_ray(const float* cam19, int w, int h, const int* xy, uint32_t* rng, int n, float* out) {
    Cam c; memset(&c, 0, sizeof c);
    memcpy(c.pos.e, cam19, 12); memcpy(c.llc.e, cam19 + 3, 12); memcpy(c.horiz.e, cam19 + 6, 12);
    memcpy(c.vert.e, cam19 + 9, 12); memcpy(c.right.e, cam19 + 12, 12); memcpy(c.up.e, cam19 + 15, 12);
    c.lens_r = cam19[18];
    for (int i = 0; i < n; i++) {
        Rng s; memcpy(&s, rng + 6 * i, sizeof s);
        Ray r = cam_get_ray(&c, xy[2 * i], xy[2 * i + 1], w, h, &s);
        memcpy(rng + 6 * i, &s, sizeof s);
        memcpy(out + 6 * i, r.o.e, 12);
        memcpy(out + 6 * i + 3, r.d.e, 12);
    }
}
