// wide_visits — node visits, box tests and triangle tests per ray of a W-wide collapse of the rebuilt tree, W = 4..8,
// traced on the CPU over one set of synthetic paths ("What the census says about a wider node").
//
//   tools/wide_visits.py builds and runs it: g++ -O2 -std=c++17 -I raytracer-cuda_amd/csrc tools/wide_visits.cpp
//
// The binary SAH tree is crt_sah::Builder's with the shipped options (leaf size 4, traversal cost 2); the W-wide nodes
// are the SAH-optimal cuts of it (crt_sah::Collapse, generalised here to W slots; W = 4 is the shipped tree).  The
// traversal is node_step4's (crt_hip.hip) for any W: the slots of a node are its internal children, then its leaf
// children; a step tests every slot's box against [0.001, closest], tests the primitives from the first to the last
// hit leaf child against the closest hit at the step's start, moves to the nearest hit internal child and stacks the
// others; a pop visits the next stacked child without re-testing its box.  The paths are not the renderer's (every
// surface scatters diffusely, no materials), so only the ratios between widths carry over: one path set, the same
// closest hits for every W (the hit does not depend on the tree), the same rays.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "crt_sah.h"

namespace {

struct V { float x, y, z; };
V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V operator*(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V unit(V a) { return a * (1.0f / std::sqrt(dot(a, a))); }

struct Rng {   // splitmix64: the synthetic paths only
    uint64_t s;
    float u() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return (float)((z ^ (z >> 31)) >> 40) * 0x1p-24f;
    }
};

// crt_sah::Collapse with W slots instead of 4
template <int W>
class CollapseW {
public:
    CollapseW(const std::vector<crt_sah::Node>& bn, double c_node) : bn_(bn), cover_(bn.size()), split_(bn.size()) {
        for (int n = (int)bn.size() - 1; n >= 0; --n) {
            const crt_sah::Node& N = bn[n];
            const double a = (double)crt_sah::half_area(N.lo, N.hi);
            auto& c = cover_[n];
            auto& s = split_[n];
            if (N.child[0] < 0) {
                for (int k = 1; k <= W; ++k) { c[k] = a * N.count; s[k] = 0; }
                continue;
            }
            const int l = N.child[0], r = N.child[1];
            double open[W + 1];
            int open_split[W + 1];
            for (int k = 2; k <= W; ++k) {
                open[k] = INFINITY;
                open_split[k] = 1;
                for (int i = 1; i < k; ++i) {
                    const double v = cover_[l][i] + cover_[r][k - i];
                    if (v < open[k]) { open[k] = v; open_split[k] = i; }
                }
            }
            c[1] = a * c_node + open[W];
            s[1] = 0;
            for (int k = 2; k <= W; ++k) {
                if (open[k] < c[k - 1]) { c[k] = open[k]; s[k] = open_split[k]; }
                else { c[k] = c[k - 1]; s[k] = -1; }
            }
        }
    }
    // slots of the node made from binary node n: internal first, then leaves
    std::vector<int> open(int n) const {
        std::vector<int> c;
        if (bn_[n].child[0] < 0) {
            c.push_back(n);
        } else {
            const int l = bn_[n].child[0], r = bn_[n].child[1];
            double best = INFINITY;
            int bi = 1;
            for (int i = 1; i < W; ++i) {
                const double v = cover_[l][i] + cover_[r][W - i];
                if (v < best) { best = v; bi = i; }
            }
            gather(l, bi, c);
            gather(r, W - bi, c);
        }
        std::vector<int> out;
        for (int m : c) if (bn_[m].child[0] >= 0) out.push_back(m);
        for (int m : c) if (bn_[m].child[0] < 0) out.push_back(m);
        return out;
    }
    int n_internal(const std::vector<int>& slots) const {
        int k = 0;
        for (int m : slots) k += bn_[m].child[0] >= 0;
        return k;
    }

private:
    const std::vector<crt_sah::Node>& bn_;
    std::vector<std::array<double, W + 1>> cover_;
    std::vector<std::array<int, W + 1>> split_;
    void gather(int m, int k, std::vector<int>& c) const {
        while (k > 1 && split_[m][k] < 0) --k;
        if (k == 1 || split_[m][k] == 0) { c.push_back(m); return; }
        const int i = split_[m][k];
        gather(bn_[m].child[0], i, c);
        gather(bn_[m].child[1], k - i, c);
    }
};

struct WideNode {
    std::vector<std::array<float, 6>> box;   // per slot lo xyz, hi xyz
    std::vector<int> child;                  // internal slot: wide node index
    int n_int = 0;
    std::vector<int> leaf_first, leaf_count; // leaf slot: primitive range (in the builder's item order)
};

struct Tri { V v0, e1, e2; };

struct Stats { double steps = 0, boxes = 0, tris = 0, leaf_steps = 0, rays = 0, pushes = 0; };

template <int W>
std::vector<WideNode> collapse(const std::vector<crt_sah::Node>& bn, double c_node) {
    const CollapseW<W> col(bn, c_node);
    std::vector<WideNode> out;
    std::vector<int> queue{0};
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const std::vector<int> slots = col.open(queue[qi]);
        WideNode w;
        w.n_int = col.n_internal(slots);
        for (size_t s = 0; s < slots.size(); ++s) {
            const crt_sah::Node& N = bn[slots[s]];
            w.box.push_back({N.lo[0], N.lo[1], N.lo[2], N.hi[0], N.hi[1], N.hi[2]});
            if ((int)s < w.n_int) {
                w.child.push_back((int)queue.size());
                queue.push_back(slots[s]);
            } else {
                w.leaf_first.push_back(N.first);
                w.leaf_count.push_back(N.count);
            }
        }
        out.push_back(std::move(w));
    }
    return out;
}

bool tri_hit(const Tri& T, V o, V d, float tmax, float& t) {   // Möller-Trumbore, the reference's rejections
    const V h = cross(d, T.e2);
    const float a = dot(T.e1, h);
    if (std::fabs(a) < 1e-8f) return false;
    const float f = 1.0f / a;
    const V s = o - T.v0;
    const float u = f * dot(s, h);
    if (u < 0.f || u > 1.f) return false;
    const V q = cross(s, T.e1);
    const float v = f * dot(d, q);
    if (v < 0.f || u + v > 1.f) return false;
    t = f * dot(T.e2, q);
    return t >= 0.001f && t <= tmax;
}

// closest hit through a W-wide tree, node_step4's visiting rule
int trace(const std::vector<WideNode>& nodes, const std::vector<Tri>& tris, V o, V d, float& closest, Stats& st) {
    const V inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    closest = INFINITY;
    int hit = -1, node = 0;
    std::vector<int> stack;
    while (node >= 0) {
        const WideNode& N = nodes[node];
        st.steps += 1;
        st.boxes += (double)N.box.size();
        const float entry = closest;
        std::vector<std::pair<float, int>> hits;
        int first_leaf = -1, last_leaf = -1;
        for (size_t s = 0; s < N.box.size(); ++s) {
            const auto& b = N.box[s];
            const float tx0 = (b[0] - o.x) * inv.x, tx1 = (b[3] - o.x) * inv.x;
            const float ty0 = (b[1] - o.y) * inv.y, ty1 = (b[4] - o.y) * inv.y;
            const float tz0 = (b[2] - o.z) * inv.z, tz1 = (b[5] - o.z) * inv.z;
            const float t0 = std::max(std::max(std::min(tx0, tx1), std::min(ty0, ty1)), std::max(std::min(tz0, tz1), 0.001f));
            const float t1 = std::min(std::min(std::max(tx0, tx1), std::max(ty0, ty1)), std::min(std::max(tz0, tz1), entry));
            if (!(t0 < t1)) continue;
            if ((int)s < N.n_int) hits.push_back({t0, N.child[s]});
            else {
                if (first_leaf < 0) first_leaf = (int)s - N.n_int;
                last_leaf = (int)s - N.n_int;
            }
        }
        if (first_leaf >= 0) {
            st.leaf_steps += 1;
            for (int l = first_leaf; l <= last_leaf; ++l)
                for (int i = N.leaf_first[l]; i < N.leaf_first[l] + N.leaf_count[l]; ++i) {
                    st.tris += 1;
                    float t;
                    if (tri_hit(tris[i], o, d, entry, t) && t < closest) { closest = t; hit = i; }
                }
        }
        std::sort(hits.begin(), hits.end());
        if (!hits.empty()) {
            node = hits[0].second;
            for (size_t i = hits.size() - 1; i >= 1; --i) stack.push_back(hits[i].second);
            st.pushes += hits.size() > 1;
        } else if (!stack.empty()) {
            node = stack.back();
            stack.pop_back();
        } else {
            node = -1;
        }
    }
    st.rays += 1;
    return hit;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: wide_visits <input.bin> [paths] [bounces] [c_node8]\n"); return 2; }
    const long n_paths = argc > 2 ? std::atol(argv[2]) : 200000;
    const int bounces = argc > 3 ? std::atoi(argv[3]) : 6;
    const double c_node_wide = argc > 4 ? std::atof(argv[4]) : 1.0;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) { std::perror("open"); return 2; }
    int32_t hdr[3];   // n_tris, width, height
    float cam[19];
    if (std::fread(hdr, 4, 3, f) != 3 || std::fread(cam, 4, 19, f) != 19) return 2;
    std::vector<float> raw((size_t)hdr[0] * 9);
    if (std::fread(raw.data(), 4, raw.size(), f) != raw.size()) return 2;
    std::fclose(f);
    std::vector<crt_sah::Item> items;
    std::vector<Tri> src;
    for (int p = 0; p < hdr[0]; ++p) {
        const float* r = &raw[9 * (size_t)p];
        Tri T{{r[0], r[1], r[2]}, {r[3], r[4], r[5]}, {r[6], r[7], r[8]}};
        src.push_back(T);
        crt_sah::Item it;
        it.src = p;
        it.sphere = false;
        const V v1 = T.v0 + T.e1, v2 = T.v0 + T.e2;
        const float vx[3] = {T.v0.x, v1.x, v2.x}, vy[3] = {T.v0.y, v1.y, v2.y}, vz[3] = {T.v0.z, v1.z, v2.z};
        it.lo[0] = std::min({vx[0], vx[1], vx[2]}); it.hi[0] = std::max({vx[0], vx[1], vx[2]});
        it.lo[1] = std::min({vy[0], vy[1], vy[2]}); it.hi[1] = std::max({vy[0], vy[1], vy[2]});
        it.lo[2] = std::min({vz[0], vz[1], vz[2]}); it.hi[2] = std::max({vz[0], vz[1], vz[2]});
        for (int a = 0; a < 3; ++a) it.c[a] = 0.5f * it.lo[a] + 0.5f * it.hi[a];
        items.push_back(it);
    }
    crt_sah::Builder B(std::move(items), 4, 2.0f);
    B.build();
    std::vector<Tri> tris;   // in the builder's item order (leaf ranges index it)
    for (const auto& it : B.items()) tris.push_back(src[it.src]);
    std::vector<std::vector<WideNode>> trees;
    trees.push_back(collapse<4>(B.nodes(), 1.0));
    trees.push_back(collapse<6>(B.nodes(), c_node_wide));
    trees.push_back(collapse<8>(B.nodes(), c_node_wide));
    const int widths[3] = {4, 6, 8};
    std::vector<Stats> st(3);
    const V origin{cam[0], cam[1], cam[2]}, llc{cam[3], cam[4], cam[5]}, hor{cam[6], cam[7], cam[8]},
        ver{cam[9], cam[10], cam[11]};
    long mismatched = 0;
    for (long p = 0; p < n_paths; ++p) {
        Rng rng{0x5eed0000ull + (uint64_t)p * 0x9e3779b97f4a7c15ull};
        const float u = rng.u(), v = rng.u();
        V o = origin, d = (llc + hor * u + ver * v) - origin;
        for (int b = 0; b < bounces; ++b) {
            float t[3];
            int h[3];
            for (int k = 0; k < 3; ++k) h[k] = trace(trees[k], tris, o, d, t[k], st[k]);
            if (h[1] != h[0] || h[2] != h[0]) ++mismatched;
            if (h[0] < 0) break;
            const Tri& T = tris[h[0]];
            V n = unit(cross(T.e1, T.e2));
            if (dot(n, d) > 0) n = n * -1.0f;
            o = o + d * t[0];
            // cosine-weighted scatter: n + a unit vector
            V r;
            do { r = {2 * rng.u() - 1, 2 * rng.u() - 1, 2 * rng.u() - 1}; } while (dot(r, r) > 1.f || dot(r, r) < 1e-6f);
            d = n + unit(r);
            if (dot(d, d) < 1e-12f) d = n;
        }
    }
    std::printf("{\"triangles\": %d, \"paths\": %ld, \"bounces\": %d, \"c_node_wide\": %.3f, \"hit_mismatches\": %ld,"
                " \"widths\": [", hdr[0], n_paths, bounces, c_node_wide, mismatched);
    for (int k = 0; k < 3; ++k) {
        const Stats& s = st[k];
        std::printf("%s{\"width\": %d, \"nodes\": %zu, \"rays\": %.0f, \"steps_per_ray\": %.4f, \"boxes_per_ray\": %.4f,"
                    " \"tris_per_ray\": %.4f, \"leaf_steps_per_ray\": %.4f, \"pushes_per_ray\": %.4f}",
                    k ? ", " : "", widths[k], trees[k].size(), s.rays, s.steps / s.rays, s.boxes / s.rays,
                    s.tris / s.rays, s.leaf_steps / s.rays, s.pushes / s.rays);
    }
    std::printf("]}\n");
    return 0;
}
