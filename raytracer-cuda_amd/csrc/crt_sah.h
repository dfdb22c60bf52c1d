// crt_sah.h — host-side binned-SAH BVH for the CRT_BVH_REBUILT scene mode (see include/crt_hip.h).
//
// The reference's BVHs (BVHNode::buildBVHScene, Mesh::buildBVH) are median splits with leaves of up to
// ten triangles and unpadded leaf boxes; on the benchmark scenes every ray ends up testing ~26 triangles
// and ~18 boxes.  The rebuilt mode keeps the reference's hit rule (closest t in [0.001, closest], ties
// to the primitive with the higher reference DFS rank) but traverses a tree built for the hardware:
//   * binned SAH (CRT_SAH_BINS = 128 bins, all three axes) over primitive boxes, leaves of <= leaf_size triangles;
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
    int tri = -1;        // SpatialBuilder: index of the triangle's vertices (-1: split by its box alone)
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
// 128 bins (round 3, profiles/r03o: config C -0.2 %, config E -1.8 % against 32, three interleaved rounds each;
// 64 bins made E 3.5 % slower, reproducibly).  A build-time knob shared with the GPU builder (crt_bvh_build.hip),
// whose trees are tested identical to this builder's.
#ifndef CRT_SAH_BINS
#define CRT_SAH_BINS 128
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

// ---------------------------------------------------------------- spatial splits (SBVH)
// Binned SAH with spatial splits (Stich, Friedrich, Dietrich, "Spatial Splits in Bounding Volume Hierarchies",
// HPG 2009).  A node may also be cut by an axis-aligned plane: a primitive straddling it is referenced from both
// sides, each reference boxed by the part of the triangle on its side (the box of the vertices on that side and the
// edge/plane crossings, intersected with the reference's own box).  Long thin and overlapping triangles then stop
// inflating every node above them.
//
// Why the rebuilt hit rule survives duplication: the kernel reports the minimum t, ties to the
// highest reference rank, over the primitives of the leaves the ray reaches.  Every reference of a triangle carries
// the same record (same vertices, same rank), so a triangle tested from two leaves offers the same (t, rank) key
// twice.  The references' boxes cover the triangle (every point of it lies on one side of each cut, inside that
// side's reference box), and every node box is padded (pad_box), so the leaf holding the part of the triangle where
// a ray hits it is entered exactly when the unsplit triangle's leaf would be.
//
// Spatial splits are tried only where the best object split's children overlap by more than alpha of the root's
// area (the paper's lambda test), and while the reference count stays below (1 + max_dup) x the primitive count.
// Straddling references are "unsplit" (kept whole on one side) when that is cheaper by the SAH.
struct TriVerts {
    double v[3][3];
};

class SpatialBuilder {
public:
    SpatialBuilder(std::vector<Item>&& items, std::vector<TriVerts>&& verts, int leaf_size, float trav_cost,
                   float alpha, float max_dup)
        : in_(std::move(items)), verts_(std::move(verts)), leaf_size_(leaf_size), trav_cost_(trav_cost),
          alpha_(alpha), max_dup_(max_dup) {}

    bool build() {
        if (in_.empty()) return false;
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (const Item& it : in_) grow(lo, hi, it.lo, it.hi);
        min_overlap_ = alpha_ * half_area(lo, hi);
        n_refs_ = in_.size();
        max_refs_ = (size_t)((double)in_.size() * (1.0 + (double)max_dup_));
        out_.reserve(in_.size() + in_.size() / 4);
        build_node(std::move(in_), 0);
        return true;
    }
    const std::vector<Node>& nodes() const { return nodes_; }
    const std::vector<Item>& items() const { return out_; }   // leaf references, in leaf order
    int max_depth() const { return max_depth_; }
    long spatial_splits() const { return n_spatial_; }

private:
    static constexpr int kBins = CRT_SAH_BINS;
    static constexpr int kMaxSpatialDepth = 48;
    std::vector<Item> in_, out_;
    std::vector<TriVerts> verts_;
    std::vector<Node> nodes_;
    int leaf_size_;
    float trav_cost_, alpha_, max_dup_;
    float min_overlap_ = 0.f;
    size_t n_refs_ = 0, max_refs_ = 0;
    int max_depth_ = 0;
    long n_spatial_ = 0;

    static void grow(float lo[3], float hi[3], const float blo[3], const float bhi[3]) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], blo[a]); hi[a] = std::max(hi[a], bhi[a]); }
    }
    static float area_or0(const float lo[3], const float hi[3]) { return lo[0] <= hi[0] ? half_area(lo, hi) : 0.f; }
    static void set_centre(Item& it) {
        for (int a = 0; a < 3; ++a) it.c[a] = 0.5f * it.lo[a] + 0.5f * it.hi[a];
    }
    // outward rounding of a double bound to float
    static float down(double x) { float f = (float)x; return (double)f > x ? std::nextafter(f, -INFINITY) : f; }
    static float up(double x) { float f = (float)x; return (double)f < x ? std::nextafter(f, INFINITY) : f; }

    // The reference r cut by the plane x_axis = pos: the boxes of its parts below and above the plane.  Returns
    // false for a side that holds nothing of the primitive (then the reference lies wholly on the other side).
    void split_ref(const Item& r, int axis, float pos, Item& L, Item& R, bool& has_l, bool& has_r) const {
        L = r;
        R = r;
        if (r.tri < 0) {   // box only (spheres): the box's halves
            L.hi[axis] = std::min(L.hi[axis], pos);
            R.lo[axis] = std::max(R.lo[axis], pos);
        } else {
            double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            double rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            auto add = [](double lo[3], double hi[3], const double p[3]) {
                for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
            };
            const TriVerts& T = verts_[r.tri];
            const double pp = (double)pos;
            for (int e = 0; e < 3; ++e) {
                const double* v0 = T.v[e];
                const double* v1 = T.v[(e + 1) % 3];
                const double a0 = v0[axis], a1 = v1[axis];
                if (a0 <= pp) add(llo, lhi, v0);
                if (a0 >= pp) add(rlo, rhi, v0);
                if ((a0 < pp && a1 > pp) || (a0 > pp && a1 < pp)) {   // the edge crosses the plane
                    const double t = (pp - a0) / (a1 - a0);
                    double x[3];
                    for (int a = 0; a < 3; ++a) x[a] = v0[a] + (v1[a] - v0[a]) * t;
                    x[axis] = pp;
                    add(llo, lhi, x);
                    add(rlo, rhi, x);
                }
            }
            for (int a = 0; a < 3; ++a) {
                L.lo[a] = std::max(L.lo[a], down(llo[a]));
                L.hi[a] = std::min(L.hi[a], up(lhi[a]));
                R.lo[a] = std::max(R.lo[a], down(rlo[a]));
                R.hi[a] = std::min(R.hi[a], up(rhi[a]));
            }
            L.hi[axis] = std::min(L.hi[axis], pos);
            R.lo[axis] = std::max(R.lo[axis], pos);
        }
        has_l = L.lo[0] <= L.hi[0] && L.lo[1] <= L.hi[1] && L.lo[2] <= L.hi[2];
        has_r = R.lo[0] <= R.hi[0] && R.lo[1] <= R.hi[1] && R.lo[2] <= R.hi[2];
        set_centre(L);
        set_centre(R);
    }

    int make_leaf(int idx, std::vector<Item>& refs) {
        nodes_[idx].child[0] = nodes_[idx].child[1] = -1;
        nodes_[idx].first = (int)out_.size();
        nodes_[idx].count = (int)refs.size();
        out_.insert(out_.end(), refs.begin(), refs.end());
        std::vector<Item>().swap(refs);
        return idx;
    }

    int build_node(std::vector<Item>&& refs_in, int depth) {
        std::vector<Item> refs(std::move(refs_in));
        max_depth_ = std::max(max_depth_, depth);
        const int idx = (int)nodes_.size();
        nodes_.push_back(Node{});
        const int count = (int)refs.size();
        Node nd;
        float ulo[3] = {INFINITY, INFINITY, INFINITY}, uhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int n_sph = 0;
        for (const Item& it : refs) {
            n_sph += it.sphere;
            grow(ulo, uhi, it.lo, it.hi);
            grow(clo, chi, it.c, it.c);
        }
        for (int a = 0; a < 3; ++a) { nd.lo[a] = ulo[a]; nd.hi[a] = uhi[a]; }
        pad_box(nd.lo, nd.hi);
        nd.child[0] = nd.child[1] = -1;
        nd.first = 0;
        nd.count = count;
        nodes_[idx] = nd;
        if (count == 1) return make_leaf(idx, refs);
        const bool leaf_ok = n_sph == 0 && count <= leaf_size_;

        // object split: binned SAH over the centroids (Builder::build_range)
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
            for (const Item& it : refs) {
                const int b = std::min(kBins - 1, (int)((it.c[a] - clo[a]) * scale));
                ++bcnt[b];
                grow(blo[b], bhi[b], it.lo, it.hi);
            }
            float right_area[kBins];
            int right_cnt[kBins];
            float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int rc = 0;
            for (int b = kBins - 1; b > 0; --b) {
                rc += bcnt[b];
                grow(rlo, rhi, blo[b], bhi[b]);
                right_cnt[b] = rc;
                right_area[b] = rc ? half_area(rlo, rhi) : 0.f;
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int b = 0; b < kBins - 1; ++b) {
                lc += bcnt[b];
                grow(llo, lhi, blo[b], bhi[b]);
                if (lc == 0 || right_cnt[b + 1] == 0) continue;
                const float cost = half_area(llo, lhi) * lc + right_area[b + 1] * right_cnt[b + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = b + 1; }
            }
        }
        auto obj_side = [&](const Item& it) {
            const float scale = kBins / (chi[best_axis] - clo[best_axis]);
            return std::min(kBins - 1, (int)((it.c[best_axis] - clo[best_axis]) * scale)) < best_split;
        };

        // spatial split: tried when the object split's children overlap
        int sp_axis = -1;
        float sp_pos = 0.f, sp_cost = INFINITY;
        if (best_axis >= 0 && depth < kMaxSpatialDepth && n_refs_ < max_refs_) {
            float olo[3] = {INFINITY, INFINITY, INFINITY}, ohi[3] = {-INFINITY, -INFINITY, -INFINITY};
            float plo[3] = {INFINITY, INFINITY, INFINITY}, phi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (const Item& it : refs) {
                if (obj_side(it)) grow(olo, ohi, it.lo, it.hi);
                else grow(plo, phi, it.lo, it.hi);
            }
            float ilo[3], ihi[3];
            for (int a = 0; a < 3; ++a) { ilo[a] = std::max(olo[a], plo[a]); ihi[a] = std::min(ohi[a], phi[a]); }
            const bool overlap = ilo[0] < ihi[0] && ilo[1] < ihi[1] && ilo[2] < ihi[2];
            if (overlap && half_area(ilo, ihi) > min_overlap_) spatial_sweep(refs, ulo, uhi, sp_axis, sp_pos, sp_cost);
        }
        const bool spatial = sp_axis >= 0 && sp_cost < best_cost;
        const float split_cost = spatial ? sp_cost : best_cost;
        const bool have_split = spatial || best_axis >= 0;
        const float node_area = std::max(half_area(nd.lo, nd.hi), 1e-30f);
        if (leaf_ok && (!have_split || trav_cost_ + split_cost / node_area >= (float)count)) return make_leaf(idx, refs);

        std::vector<Item> left, right;
        if (spatial) spatial_partition(refs, sp_axis, sp_pos, left, right);
        if (left.empty() || right.empty() || (int)left.size() >= count || (int)right.size() >= count) {
            left.clear();
            right.clear();
            if (best_axis >= 0)
                for (const Item& it : refs) (obj_side(it) ? left : right).push_back(it);
            if (left.empty() || right.empty()) {   // no usable split (coincident centres): median by index
                left.clear();
                right.clear();
                int a = 0;
                for (int q = 1; q < 3; ++q)
                    if (uhi[q] - ulo[q] > uhi[a] - ulo[a]) a = q;
                const int mid = count / 2;
                std::nth_element(refs.begin(), refs.begin() + mid, refs.end(),
                                 [a](const Item& x, const Item& y) { return x.c[a] < y.c[a]; });
                left.assign(refs.begin(), refs.begin() + mid);
                right.assign(refs.begin() + mid, refs.end());
            }
        } else {
            ++n_spatial_;
            n_refs_ += left.size() + right.size() - refs.size();
        }
        std::vector<Item>().swap(refs);
        const int l = build_node(std::move(left), depth + 1);
        const int r = build_node(std::move(right), depth + 1);
        nodes_[idx].child[0] = l;
        nodes_[idx].child[1] = r;
        nodes_[idx].count = 0;
        return idx;
    }

    // Chopped binning over the node's box on every axis: a reference adds its part inside each bin it overlaps to
    // that bin's box, and counts once at its first bin (entries) and once at its last (exits).
    void spatial_sweep(const std::vector<Item>& refs, const float ulo[3], const float uhi[3], int& best_axis,
                       float& best_pos, float& best_cost) const {
        for (int a = 0; a < 3; ++a) {
            const float ext = uhi[a] - ulo[a];
            if (!(ext > 0.f)) continue;
            const float step = ext / kBins;
            auto plane = [&](int b) { return ulo[a] + step * (float)b; };   // left plane of bin b
            auto bin_of = [&](float x) { return std::max(0, std::min(kBins - 1, (int)((x - ulo[a]) / step))); };
            int enter[kBins] = {0}, leave[kBins] = {0};
            float blo[kBins][3], bhi[kBins][3];
            for (int b = 0; b < kBins; ++b)
                for (int q = 0; q < 3; ++q) { blo[b][q] = INFINITY; bhi[b][q] = -INFINITY; }
            for (const Item& it : refs) {
                const int b0 = bin_of(it.lo[a]), b1 = bin_of(it.hi[a]);
                ++enter[b0];
                ++leave[b1];
                if (b0 == b1) { grow(blo[b0], bhi[b0], it.lo, it.hi); continue; }
                Item rest = it;
                for (int b = b0; b < b1; ++b) {
                    Item L, R;
                    bool hl, hr;
                    split_ref(rest, a, plane(b + 1), L, R, hl, hr);
                    if (hl) grow(blo[b], bhi[b], L.lo, L.hi);
                    if (!hr) { rest.lo[0] = INFINITY; break; }
                    rest = R;
                }
                if (rest.lo[0] <= rest.hi[0]) grow(blo[b1], bhi[b1], rest.lo, rest.hi);
            }
            float right_area[kBins];
            int right_cnt[kBins];
            float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int rc = 0;
            for (int b = kBins - 1; b > 0; --b) {
                rc += leave[b];
                grow(rlo, rhi, blo[b], bhi[b]);
                right_cnt[b] = rc;
                right_area[b] = area_or0(rlo, rhi);
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int b = 0; b < kBins - 1; ++b) {
                lc += enter[b];
                grow(llo, lhi, blo[b], bhi[b]);
                if (lc == 0 || right_cnt[b + 1] == 0) continue;
                const float cost = area_or0(llo, lhi) * lc + right_area[b + 1] * right_cnt[b + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_pos = plane(b + 1); }
            }
        }
    }

    // Partition at the plane; a straddling reference is split, or kept whole on the side where that costs less
    // (reference unsplitting).
    void spatial_partition(const std::vector<Item>& refs, int a, float pos, std::vector<Item>& left,
                           std::vector<Item>& right) const {
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        std::vector<const Item*> straddle;
        for (const Item& it : refs) {
            if (it.hi[a] <= pos) { left.push_back(it); grow(llo, lhi, it.lo, it.hi); }
            else if (it.lo[a] >= pos) { right.push_back(it); grow(rlo, rhi, it.lo, it.hi); }
            else straddle.push_back(&it);
        }
        for (const Item* p : straddle) {
            Item L, R;
            bool hl, hr;
            split_ref(*p, a, pos, L, R, hl, hr);
            const float nl = (float)left.size(), nr = (float)right.size();
            auto with = [](const float lo[3], const float hi[3], const Item& it, float olo[3], float ohi[3]) {
                for (int q = 0; q < 3; ++q) { olo[q] = std::min(lo[q], it.lo[q]); ohi[q] = std::max(hi[q], it.hi[q]); }
            };
            float alo[3], ahi[3], blo_[3], bhi_[3], clo_[3], chi_[3], dlo[3], dhi[3];
            with(llo, lhi, *p, alo, ahi);   // whole reference left
            with(rlo, rhi, *p, blo_, bhi_); // whole reference right
            with(llo, lhi, L, clo_, chi_);  // left part
            with(rlo, rhi, R, dlo, dhi);    // right part
            const float c_left = half_area(alo, ahi) * (nl + 1) + area_or0(rlo, rhi) * nr;
            const float c_right = area_or0(llo, lhi) * nl + half_area(blo_, bhi_) * (nr + 1);
            const float c_split = (hl && hr) ? half_area(clo_, chi_) * (nl + 1) + half_area(dlo, dhi) * (nr + 1)
                                             : INFINITY;
            if (!hr || (hl && c_left <= c_right && c_left <= c_split)) {
                left.push_back(*p);
                grow(llo, lhi, p->lo, p->hi);
            } else if (!hl || c_right <= c_split) {
                right.push_back(*p);
                grow(rlo, rhi, p->lo, p->hi);
            } else {
                left.push_back(L);
                right.push_back(R);
                grow(llo, lhi, L.lo, L.hi);
                grow(rlo, rhi, R.lo, R.hi);
            }
        }
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
