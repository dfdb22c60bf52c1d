// crt_sah.h — host-side binned-SAH BVH for the CRT_BVH_REBUILT scene mode (see include/crt_hip.h).
//
// The reference's BVHs (BVHNode::buildBVHScene, Mesh::buildBVH) are median splits with leaves of up to
// ten triangles and unpadded leaf boxes; on the benchmark scenes every ray ends up testing ~26 triangles
// and ~18 boxes.  The rebuilt mode keeps the reference's hit rule (closest t in [0.001, closest], ties
// to the primitive with the higher reference DFS rank) but traverses a tree built for the hardware:
//   * binned SAH (32 bins, all three axes) over primitive boxes, leaves of <= leaf_size triangles;
//   * every box padded outward (pad_box), so rounding in the slab test cannot cull a genuine hit;
//   * emitted as threaded DFS arrays (same node format as the reference mode, crt_device.h), once per
//     ray-direction class (dominant axis x sign): children ordered near-first along that axis, so the
//     stackless left-first traversal meets the closest hits early and culls more (multiple-threaded BVH).
// Spheres are always singleton leaves (the kernel's sphere-leaf node).
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <vector>

namespace crt_sah {

struct Item {
    float lo[3], hi[3];
    float c[3];          // box centre (binning key)
    int src;             // caller's primitive id
    bool sphere;
};

struct Node {
    float lo[3], hi[3];
    int child[2];        // internal: children; leaf: -1
    int first, count;    // leaf: items[first, first + count)
};

inline float half_area(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

// Outward padding of a box: 1e-5 of the larger of the box's coordinate magnitude and 1.  That is
// ~170 float ulps of the coordinates — far above the few-ulp error of the slab distances — and
// negligible against any box size that matters for culling.
inline void pad_box(float lo[3], float hi[3]) {
    float m = 1.0f;
    for (int a = 0; a < 3; ++a) m = std::max(m, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
    const float pad = 1e-5f * m;
    for (int a = 0; a < 3; ++a) {
        lo[a] -= pad;
        hi[a] += pad;
    }
}

class Builder {
public:
    Builder(std::vector<Item>&& items, int leaf_size, float trav_cost)
        : items_(std::move(items)), leaf_size_(leaf_size), trav_cost_(trav_cost) {}

    // Builds the tree; returns false on an empty item list.
    bool build() {
        if (items_.empty()) return false;
        nodes_.reserve(2 * items_.size() / std::max(1, leaf_size_ / 2) + 8);
        build_range(0, (int)items_.size(), 0);
        return true;
    }
    const std::vector<Node>& nodes() const { return nodes_; }
    const std::vector<Item>& items() const { return items_; }
    int max_depth() const { return max_depth_; }

private:
#ifndef CRT_SAH_BINS
#define CRT_SAH_BINS 32
#endif
    static constexpr int kBins = CRT_SAH_BINS;
    std::vector<Item> items_;
    std::vector<Node> nodes_;
    int leaf_size_;
    float trav_cost_;
    int max_depth_ = 0;

    int make_leaf(int idx, int first, int count) {
        nodes_[idx].child[0] = nodes_[idx].child[1] = -1;
        nodes_[idx].first = first;
        nodes_[idx].count = count;
        return idx;
    }

    int build_range(int first, int count, int depth) {
        max_depth_ = std::max(max_depth_, depth);
        const int idx = (int)nodes_.size();
        nodes_.push_back(Node{});
        Node nd;
        float clo[3], chi[3];
        int n_sph = 0;
        for (int a = 0; a < 3; ++a) {
            nd.lo[a] = clo[a] = INFINITY;
            nd.hi[a] = chi[a] = -INFINITY;
        }
        for (int i = first; i < first + count; ++i) {
            const Item& it = items_[i];
            n_sph += it.sphere;
            for (int a = 0; a < 3; ++a) {
                nd.lo[a] = std::min(nd.lo[a], it.lo[a]);
                nd.hi[a] = std::max(nd.hi[a], it.hi[a]);
                clo[a] = std::min(clo[a], it.c[a]);
                chi[a] = std::max(chi[a], it.c[a]);
            }
        }
        pad_box(nd.lo, nd.hi);
        nd.child[0] = nd.child[1] = -1;
        nd.first = first;
        nd.count = count;
        nodes_[idx] = nd;
        const bool leaf_ok = n_sph == 0 && count <= leaf_size_;
        if (count == 1) return make_leaf(idx, first, count);

        // binned SAH over the three axes (traversal cost trav_cost_, intersection cost 1 per primitive)
        float best_cost = INFINITY;
        int best_axis = -1, best_split = 0;
        for (int a = 0; a < 3; ++a) {
            const float ext = chi[a] - clo[a];
            if (!(ext > 0.f)) continue;
            const float scale = kBins / ext;
            int bcnt[kBins] = {0};
            float blo[kBins][3], bhi[kBins][3];
            for (int b = 0; b < kBins; ++b)
                for (int q = 0; q < 3; ++q) { blo[b][q] = INFINITY; bhi[b][q] = -INFINITY; }
            for (int i = first; i < first + count; ++i) {
                const Item& it = items_[i];
                const int b = std::min(kBins - 1, (int)((it.c[a] - clo[a]) * scale));
                ++bcnt[b];
                for (int q = 0; q < 3; ++q) {
                    blo[b][q] = std::min(blo[b][q], it.lo[q]);
                    bhi[b][q] = std::max(bhi[b][q], it.hi[q]);
                }
            }
            float right_area[kBins];
            int right_cnt[kBins];
            float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int rc = 0;
            for (int b = kBins - 1; b > 0; --b) {
                rc += bcnt[b];
                for (int q = 0; q < 3; ++q) { rlo[q] = std::min(rlo[q], blo[b][q]); rhi[q] = std::max(rhi[q], bhi[b][q]); }
                right_cnt[b] = rc;
                right_area[b] = rc ? half_area(rlo, rhi) : 0.f;
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int b = 0; b < kBins - 1; ++b) {   // split between bin b and b + 1
                lc += bcnt[b];
                for (int q = 0; q < 3; ++q) { llo[q] = std::min(llo[q], blo[b][q]); lhi[q] = std::max(lhi[q], bhi[b][q]); }
                if (lc == 0 || right_cnt[b + 1] == 0) continue;
                const float cost = half_area(llo, lhi) * lc + right_area[b + 1] * right_cnt[b + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = b + 1; }
            }
        }
        // split cost C_trav + (A_L N_L + A_R N_R) / A against leaf cost N
        const float node_area = std::max(half_area(nd.lo, nd.hi), 1e-30f);
        if (leaf_ok && (best_axis < 0 || trav_cost_ + best_cost / node_area >= (float)count))
            return make_leaf(idx, first, count);

        int mid;
        if (best_axis >= 0) {
            const int a = best_axis;
            const float scale = kBins / (chi[a] - clo[a]);
            Item* p = std::partition(items_.data() + first, items_.data() + first + count, [&](const Item& it) {
                return std::min(kBins - 1, (int)((it.c[a] - clo[a]) * scale)) < best_split;
            });
            mid = (int)(p - items_.data());
        } else {
            mid = first;
        }
        if (mid == first || mid == first + count) {   // no usable split (coincident centres): median by index
            int a = 0;
            for (int q = 1; q < 3; ++q)
                if (nd.hi[q] - nd.lo[q] > nd.hi[a] - nd.lo[a]) a = q;
            mid = first + count / 2;
            std::nth_element(items_.begin() + first, items_.begin() + mid, items_.begin() + first + count,
                             [a](const Item& x, const Item& y) { return x.c[a] < y.c[a]; });
        }
        const int l = build_range(first, mid - first, depth + 1);
        const int r = build_range(mid, first + count - mid, depth + 1);
        nodes_[idx].child[0] = l;
        nodes_[idx].child[1] = r;
        nodes_[idx].count = 0;
        return idx;
    }
};

// ---------------------------------------------------------------- 4-wide collapse
// Each BVH4 node holds the boxes of up to four children, a cut of the binary tree below it (Collapse below).  Slot
// order: internal children first (stored at consecutive node indices first_child + slot), then leaf children (their
// primitives consecutive from leaf_first, in slot order), then empty slots.
struct Wide {
    int n_internal = 0, n_slots = 0;
    int bin[4];          // binary-tree node of each slot
};

// SAH-optimal collapse: the cut of the binary tree that forms each 4-wide node, chosen by dynamic programming over
// the binary tree (Ylitie, Karras, Laine, "Efficient Incoherent Ray Traversal on GPUs Through Compressed Wide BVHs",
// HPG 2017, without their leaf merging).  Round 2 replaced the greedy collapse (open the largest-area internal child
// until four slots are used) with it: config C -1.6 %, config E (1M triangles) -9.0 %, the same frames
// (profiles/r02ax).  Cost of a subtree used as one slot of its parent:
//   leaf:     A(n) * count(n)                          (one triangle test per primitive, in ray-probability units)
//   internal: A(n) * c_node + best 4-slot cover of n   (n becomes a 4-wide node: one step, four box tests)
// cover(n, k) = the cheapest way to cover the subtree of n with at most k slots: n itself as one slot, or (internal n)
// the covers of its two children with i and k - i slots.  The tree shape does not change which hit a ray reports
// (closest t, ties to the higher reference rank), only the work to find it.
class Collapse {
public:
    Collapse(const std::vector<Node>& bn, double c_node) : bn_(bn), cover_(bn.size()), split_(bn.size()) {
        for (int n = (int)bn.size() - 1; n >= 0; --n) {   // children have larger indices than their parent
            const Node& N = bn[n];
            const double a = (double)half_area(N.lo, N.hi);
            auto& c = cover_[n];
            auto& s = split_[n];
            if (N.child[0] < 0) {
                for (int k = 1; k <= 4; ++k) { c[k] = a * N.count; s[k] = 0; }
                continue;
            }
            const int l = N.child[0], r = N.child[1];
            double open[5];
            int open_split[5];
            for (int k = 2; k <= 4; ++k) {
                open[k] = INFINITY;
                open_split[k] = 1;
                for (int i = 1; i < k; ++i) {
                    const double v = cover_[l][i] + cover_[r][k - i];
                    if (v < open[k]) { open[k] = v; open_split[k] = i; }
                }
            }
            c[1] = a * c_node + open[4];
            s[1] = 0;
            for (int k = 2; k <= 4; ++k) {
                if (open[k] < c[k - 1]) { c[k] = open[k]; s[k] = open_split[k]; }
                else { c[k] = c[k - 1]; s[k] = -1; }   // -1: the cover with fewer slots
            }
        }
    }

    // The slots of the 4-wide node made from internal binary node n (a leaf root: one leaf slot).
    Wide open(int n) const {
        Wide w;
        int c[4], k = 0;
        if (bn_[n].child[0] < 0) {
            c[k++] = n;
        } else {
            // n's own node: its best 4-slot cover, which opens n (split_[n][1] == 0 means "n as one slot" for its
            // parent; as a node n always opens): the split of open[4] is recomputed from the children's covers
            const int l = bn_[n].child[0], r = bn_[n].child[1];
            double best = INFINITY;
            int bi = 1;
            for (int i = 1; i < 4; ++i) {
                const double v = cover_[l][i] + cover_[r][4 - i];
                if (v < best) { best = v; bi = i; }
            }
            gather(l, bi, c, k);
            gather(r, 4 - bi, c, k);
        }
        for (int i = 0; i < k; ++i)
            if (bn_[c[i]].child[0] >= 0) w.bin[w.n_internal++] = c[i];
        w.n_slots = w.n_internal;
        for (int i = 0; i < k; ++i)
            if (bn_[c[i]].child[0] < 0) w.bin[w.n_slots++] = c[i];
        return w;
    }

private:
    const std::vector<Node>& bn_;
    std::vector<std::array<double, 5>> cover_;
    std::vector<std::array<int, 5>> split_;

    void gather(int m, int k, int* c, int& n) const {
        while (k > 1 && split_[m][k] < 0) --k;
        if (k == 1 || split_[m][k] == 0) { c[n++] = m; return; }
        const int i = split_[m][k];
        gather(bn_[m].child[0], i, c, n);
        gather(bn_[m].child[1], k - i, c, n);
    }
};

}  // namespace crt_sah
