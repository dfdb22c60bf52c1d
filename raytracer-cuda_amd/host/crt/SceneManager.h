// SceneManager.h — host scene assembly with the reference's API and semantics
// (CudaRayTracer/src/SceneManager.h:19-329, CUDAKernels.h:28-100).
//
// What the reference does on the device with <<<1,1>>> kernels (initMesh,
// createRandomWorld, createBVH) runs here on the host, bit-identically, and the
// result is handed to the HIP layer as flat arrays (crt_scene_create).
//   initializeScene  = loadObject per file (:198-329) + initMeshes concat/offsets
//                      (:100-196) + Mesh ctor BVH builds + createRandomWorld
//                      material/object order (CUDAKernels.h:56-84) + buildBVHScene.
//   getBVHNodes()/getWorld() return the device scene handle (the reference returns
//                      the device BVHNode* / HittableList*; CUDARenderer::render takes both).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "BVHBuild.h"
#include "CUDAHelpers.h"
#include "Material.h"
#include "Vec3.h"
#include "crt_hip.h"

struct Vertex {          // Mesh.cuh:5-10 (only Position is read by the render path)
    CRT::Vec3 Position;
    CRT::Vec3 Normal;
    float UV[2] = {0.f, 0.f};
};

struct MeshData {        // SceneManager.h:13-17
    std::vector<Vertex> vertices;
    std::vector<uint32_t> indices;
    std::vector<int> faceMaterialIds;
};

class SceneManager {
public:
    SceneManager(int width, int height, int device = 0);
    ~SceneManager();
    SceneManager(const SceneManager&) = delete;
    SceneManager& operator=(const SceneManager&) = delete;

    // Reference default model list (SceneManager.h:101-103); override before initializeScene.
    void setModelFiles(const std::vector<std::string>& files) { m_ModelFiles = files; }
    // Acceleration structure of the device scene (default CRT_BVH_REFERENCE, bit-exact); applies at uploadScene.
    void setSceneOptions(const crt_scene_options& opts) { m_SceneOptions = opts; }
    const std::vector<std::string>& modelFiles() const { return m_ModelFiles; }
    // Where the mesh BVHs are built: -1 = the host restatement (default), k >= 0 = GPU k (crt_build_mesh_bvh, the
    // same trees; meshes whose tree the reference's node cap decides still build on the host).
    void setMeshBuildDevice(int device) { m_BuildDevice = device; }
    double deviceBuildMs() const { return m_DeviceBuildMs; }   // device time of the GPU mesh builds

    // SceneManager::initializeScene (SceneManager.h:77-98).  randState is accepted for API
    // compatibility and unused (the reference passes it through and never draws from it).
    void initializeScene(const CUDAHelpers::RenderConfig& renderConfig, void* randState = nullptr);
    // Host-only variant: load + build, no device upload (used by tests / the CPU tools).
    void buildHostScene();
    void uploadScene();

    crt_scene* getBVHNodes() const { return m_Scene; }
    crt_scene* getWorld() const { return m_Scene; }

    // ---- host-side results (inspection / tests) ----
    const std::vector<MeshData>& meshData() const { return m_MeshData; }
    const std::vector<CRT::MaterialData>& sceneMaterialsData() const { return m_SceneMaterialsData; }
    const std::vector<float>& positions() const { return m_Positions; }
    const std::vector<uint32_t>& indices() const { return m_Indices; }          // permuted by the mesh BVH builds
    const std::vector<int32_t>& faceMaterials() const { return m_FaceMats; }   // permuted
    const std::vector<crt_mesh_desc>& meshes() const { return m_Meshes; }
    const std::vector<std::vector<crt_bvh_node_desc>>& meshBVHs() const { return m_MeshBVH; }
    const std::vector<crt_bvh_node_desc>& sceneBVH() const { return m_SceneBVH; }
    const std::vector<crt_material_desc>& materials() const { return m_Materials; }
    const std::vector<crt_sphere_desc>& spheres() const { return m_Spheres; }
    const std::vector<crt_object_desc>& objects() const { return m_Objects; }
    crt_scene_desc sceneDesc() const;

private:
    void initMeshes();
    void loadObject(const std::string& filename, std::vector<MeshData>& meshDataList);
    void createWorld();
    bool buildMeshOnDevice(int i, const float* pos, uint32_t* idx, int32_t* fm);

    int m_Width, m_Height, m_Device;
    std::vector<std::string> m_ModelFiles{"assets/models/CornellBox-Original.obj", "assets/models/bunny.obj"};
    std::vector<MeshData> m_MeshData;
    std::vector<CRT::MaterialData> m_SceneMaterialsData;
    std::vector<uint32_t> m_VertexOffsets, m_IndexOffsets, m_VertexCounts, m_IndexCounts, m_FaceMatOffsets, m_FaceCounts;
    std::vector<uint32_t> m_MaterialIDOffsets;

    std::vector<float> m_Positions;
    std::vector<uint32_t> m_Indices;
    std::vector<int32_t> m_FaceMats;
    std::vector<crt_mesh_desc> m_Meshes;
    std::vector<std::vector<crt_bvh_node_desc>> m_MeshBVH;
    std::vector<CRT::AABB> m_MeshBoxes;
    std::vector<crt_material_desc> m_Materials;
    std::vector<crt_sphere_desc> m_Spheres;
    std::vector<crt_object_desc> m_Objects;
    std::vector<crt_bvh_node_desc> m_SceneBVH;
    crt_scene* m_Scene = nullptr;
    crt_scene_options m_SceneOptions{};
    int m_BuildDevice = -1;
    double m_DeviceBuildMs = 0.0;
};
