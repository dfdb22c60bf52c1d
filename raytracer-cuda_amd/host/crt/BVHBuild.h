// BVHBuild.h — host restatements of the reference's two BVH builders, producing
// the exact trees the reference builds on the device with one thread:
//   * buildMeshBVH  = Mesh ctor box + Mesh::buildBVHMesh (Core/Mesh.cuh:39-53, :121-264)
//   * buildSceneBVH = BVHNode::buildBVHScene (Core/BVHNode.cuh:21-84)
// Nodes come out in the reference's allocation (index) order; the HIP layer
// re-threads them into DFS preorder for the stackless traversal.
#pragma once
#include <cstdint>
#include <vector>

#include "Vec3.h"
#include "crt_hip.h"

namespace CRT {

struct BuildStatus {
    bool ok = true;
    const char* error = "";
};

// verts: positions of the mesh's vertex slots (Mesh::m_Vertices), indices / faceMat are
// permuted in place (swap_triplet, Core.cuh:25-39).  meshBox receives Mesh::m_BoundingBox.
BuildStatus buildMeshBVH(const float* verts, uint32_t vertexCount, uint32_t* indices, int32_t* faceMat,
                         uint32_t indexCount, AABB* meshBox, std::vector<crt_bvh_node_desc>* nodes);

// objBoxes[i] = m_Objects[i]->boundingBox() in HittableList order.
BuildStatus buildSceneBVH(const std::vector<AABB>& objBoxes, std::vector<crt_bvh_node_desc>* nodes);

inline void storeBox(const AABB& b, crt_bvh_node_desc* n) {
    n->bmin[0] = b.x.min; n->bmin[1] = b.y.min; n->bmin[2] = b.z.min;
    n->bmax[0] = b.x.max; n->bmax[1] = b.y.max; n->bmax[2] = b.z.max;
}
inline AABB loadBox(const crt_bvh_node_desc& n) {
    AABB b;
    b.x = Interval(n.bmin[0], n.bmax[0]);
    b.y = Interval(n.bmin[1], n.bmax[1]);
    b.z = Interval(n.bmin[2], n.bmax[2]);
    return b;
}

}  // namespace CRT
