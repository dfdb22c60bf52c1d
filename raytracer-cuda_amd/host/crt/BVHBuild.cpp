// BVHBuild.cpp — see BVHBuild.h.  Single precision, no contraction (-ffp-contract=off).
#include "BVHBuild.h"

#include <cstring>

namespace CRT {

namespace {

struct MeshCtx {
    const float* v;
    uint32_t* idx;
    int32_t* fmat;
    inline Vec3 pos(uint32_t i) const { return Vec3(v[3 * (size_t)i], v[3 * (size_t)i + 1], v[3 * (size_t)i + 2]); }
    inline Vec3 centroid(int i) const {                                  // Mesh.cuh:251-256
        Vec3 p0 = pos(idx[i]), p1 = pos(idx[i + 1]), p2 = pos(idx[i + 2]);
        return (p0 + p1 + p2) * (1.f / 3.f);
    }
    inline void expandTri(AABB& b, int i) const {                       // :242-249
        b.expand(pos(idx[i]));
        b.expand(pos(idx[i + 1]));
        b.expand(pos(idx[i + 2]));
    }
    AABB trisAABB(int start, int count) const {                          // :258-264
        AABB b = AABB::empty();
        for (int i = start; i < start + count; i += 3) expandTri(b, i);
        return b;
    }
    float sah(int axis, float pos_, int start, int end) const {          // :222-240
        AABB lb = AABB::empty(), rb = AABB::empty();
        int lc = 0, rc = 0;
        for (int i = start; i < end; i += 3) {
            Vec3 c = centroid(i);
            if (c[axis] < pos_) { lc++; expandTri(lb, i); }
            else { rc++; expandTri(rb, i); }
        }
        float cost = lc * lb.area() + rc * rb.area();
        return cost < 1e-8f ? 1e-8f : cost;
    }
};

constexpr int MAX_STACK_SIZE = 64;   // BVHNode.cuh:7

}  // namespace

BuildStatus buildMeshBVH(const float* verts, uint32_t vertexCount, uint32_t* indices, int32_t* faceMat,
                         uint32_t indexCount, AABB* meshBox, std::vector<crt_bvh_node_desc>* out) {
    BuildStatus st;
    MeshCtx m{verts, indices, faceMat};
    // Mesh ctor (Mesh.cuh:39-51): unpadded expand over every vertex slot
    AABB box;
    if (vertexCount > 0) {
        box = AABB::empty();
        for (uint32_t i = 0; i < vertexCount; ++i) box.expand(m.pos(i));
    }
    *meshBox = box;
    out->clear();
    const int numTriangles = (int)(indexCount / 3);
    if (numTriangles <= 0) return st;   // the reference would `new BVHNode[-1]`; an empty mesh has no BVH here
    const int maxNodes = 2 * numTriangles - 1;
    std::vector<AABB> boxes;
    std::vector<crt_bvh_node_desc> nodes((size_t)maxNodes);
    std::memset(nodes.data(), 0, nodes.size() * sizeof(crt_bvh_node_desc));
    boxes.resize((size_t)maxNodes);
    struct Entry { int start, end, node; } stack[MAX_STACK_SIZE];
    int top = 0, next = 0;
    // root (Mesh.cuh:132-136)
    boxes[next] = box;
    nodes[next].obj_index = 0;
    nodes[next].obj_count = (int)indexCount;
    nodes[next].is_leaf = 0;
    next++;
    stack[top++] = {0, (int)indexCount, 0};
    while (top > 0) {
        Entry cur = stack[--top];
        const int start = cur.start, end = cur.end, ni = cur.node;
        crt_bvh_node_desc& node = nodes[ni];
        const int span = end - start;
        if (span <= 30 || (next + 1) >= maxNodes) {                    // :148-156
            node.is_leaf = 1;
            node.obj_index = start;
            node.obj_count = span;
            boxes[ni] = m.trisAABB(start, span);
            continue;
        }
        int bestAxis = 0;
        float bestPos = 0.f, bestCost = 1e30f;
        for (int axis = 0; axis < 3; axis++) {                          // :164-179
            float minPos = 1e30f, maxPos = -1e30f;
            for (int i = start; i < end; i += 3) {
                Vec3 c = m.centroid(i);
                if (c[axis] < minPos) minPos = c[axis];
                if (c[axis] > maxPos) maxPos = c[axis];
            }
            float midPos = 0.5f * (minPos + maxPos);
            float cost = m.sah(axis, midPos, start, end);
            if (cost < bestCost) { bestCost = cost; bestAxis = axis; bestPos = midPos; }
        }
        int mid = start;                                                // :182-198
        for (int i = start; i < end; i += 3) {
            Vec3 c = m.centroid(i);
            if (c[bestAxis] < bestPos) {
                uint32_t t0 = indices[mid], t1 = indices[mid + 1], t2 = indices[mid + 2];
                indices[mid] = indices[i]; indices[mid + 1] = indices[i + 1]; indices[mid + 2] = indices[i + 2];
                indices[i] = t0; indices[i + 1] = t1; indices[i + 2] = t2;
                const int fl = mid / 3, fr = i / 3;
                int32_t tmp = faceMat[fl]; faceMat[fl] = faceMat[fr]; faceMat[fr] = tmp;
                mid += 3;
            }
        }
        node.left = next++;
        node.right = next++;
        node.is_leaf = 0;
        if (top + 2 > MAX_STACK_SIZE) { st.ok = false; st.error = "mesh BVH build stack overflow (reference stack is 64)"; return st; }
        stack[top++] = {mid, end, node.right};
        stack[top++] = {start, mid, node.left};
    }
    for (int i = next - 1; i >= 0; i--) {                               // :211-218 bottom-up refit
        crt_bvh_node_desc& nd = nodes[i];
        if (!nd.is_leaf) boxes[i] = AABB::combine(boxes[nd.left], boxes[nd.right]);
    }
    nodes.resize((size_t)next);
    for (int i = 0; i < next; ++i) storeBox(boxes[i], &nodes[i]);
    out->swap(nodes);
    return st;
}

BuildStatus buildSceneBVH(const std::vector<AABB>& objBoxes, std::vector<crt_bvh_node_desc>* out) {
    BuildStatus st;
    const int n = (int)objBoxes.size();
    out->clear();
    if (n <= 0) { st.ok = false; st.error = "scene has no objects"; return st; }
    std::vector<crt_bvh_node_desc> nodes((size_t)(2 * n - 1));
    std::memset(nodes.data(), 0, nodes.size() * sizeof(crt_bvh_node_desc));
    struct Entry { int start, end, node; } stack[MAX_STACK_SIZE];
    int top = 0, next = 0;
    stack[top++] = {0, n, 0};
    while (top > 0) {
        Entry cur = stack[--top];
        crt_bvh_node_desc& node = nodes[cur.node];
        const int span = cur.end - cur.start;
        AABB box = AABB::empty();                                       // :235-237
        for (int i = cur.start; i < cur.end; i++) box.expand(objBoxes[i]);
        storeBox(box, &node);
        if (span == 1) {
            node.obj_index = cur.start;
            node.obj_count = 1;
            node.is_leaf = 1;
        } else {
            const int mid = cur.start + span / 2;                       // :258 (no sort)
            const int l = ++next, r = ++next;
            node.left = l;
            node.right = r;
            node.is_leaf = 0;
            if (top + 2 > MAX_STACK_SIZE) { st.ok = false; st.error = "scene BVH stack overflow"; return st; }
            stack[top++] = {mid, cur.end, r};
            stack[top++] = {cur.start, mid, l};
        }
    }
    nodes.resize((size_t)next + 1);
    out->swap(nodes);
    return st;
}

}  // namespace CRT
