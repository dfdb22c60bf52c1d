// SceneManager.cpp — see SceneManager.h.  Line references: CudaRayTracer/src/SceneManager.h
// unless noted.
#include "SceneManager.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <set>
#include <stdexcept>

#include "ObjLoader.h"
#include "ParallelFor.h"

namespace {
// CRT_SETUP_TRACE=1: the host loader's stages on stderr (tools/setup_breakdown.py; crt_hip.hip times the rest)
struct LoadTrace {
    bool on = std::getenv("CRT_SETUP_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* stage) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[crt load]  %-27s %8.2f ms\n", stage, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};
}  // namespace

SceneManager::SceneManager(int width, int height, int device) : m_Width(width), m_Height(height), m_Device(device) {}

SceneManager::~SceneManager() {
    if (m_Scene) crt_scene_destroy(m_Scene);
}

void SceneManager::initializeScene(const CUDAHelpers::RenderConfig& renderConfig, void* randState) {
    (void)renderConfig;
    (void)randState;
    buildHostScene();
    uploadScene();
}

void SceneManager::buildHostScene() {
    m_DeviceBuildMs = 0.0;
    m_MeshData.clear();
    m_SceneMaterialsData.clear();
    initMeshes();
    createWorld();
}

void SceneManager::uploadScene() {
    if (m_Scene) {
        crt_scene_destroy(m_Scene);
        m_Scene = nullptr;
    }
    crt_scene_desc d = sceneDesc();
    CRT_CHECK(crt_scene_create_ex(&d, m_Device, &m_SceneOptions, &m_Scene));
}

// GPU-parallel build of mesh i (crt_build_mesh_bvh: the same tree as buildMeshBVH).  false = the mesh needs the
// sequential builder (the reference's node cap decides its tree); other failures throw.
bool SceneManager::buildMeshOnDevice(int i, const float* pos, uint32_t* idx, int32_t* fm) {
    const uint32_t nTri = m_IndexCounts[i] / 3;
    std::vector<crt_bvh_node_desc> nodes(nTri > 0 ? 2 * (size_t)nTri - 1 : 0);
    int32_t count = 0;
    float box[6];
    float ms = 0.f;
    const int rc = crt_build_mesh_bvh(m_BuildDevice, pos, m_VertexCounts[i], idx, fm, m_IndexCounts[i], nodes.data(),
                                      &count, box, &ms);
    if (rc == CRT_ERR_UNSUPPORTED) return false;
    CRT_CHECK(rc);
    nodes.resize((size_t)count);
    m_MeshBVH[i].swap(nodes);
    m_MeshBoxes[i].x = CRT::Interval(box[0], box[3]);
    m_MeshBoxes[i].y = CRT::Interval(box[1], box[4]);
    m_MeshBoxes[i].z = CRT::Interval(box[2], box[5]);
    m_DeviceBuildMs += ms;
    return true;
}

// :100-196
void SceneManager::initMeshes() {
    LoadTrace tr;
    std::vector<MeshData> allMeshData;
    for (const auto& file : m_ModelFiles) loadObject(file, allMeshData);
    tr.lap("OBJ files (all)");
    m_MeshData = std::move(allMeshData);
    const std::vector<MeshData>& meshes = m_MeshData;
    const int n = (int)meshes.size();
    m_VertexOffsets.assign(n, 0); m_IndexOffsets.assign(n, 0); m_VertexCounts.assign(n, 0);
    m_IndexCounts.assign(n, 0); m_FaceMatOffsets.assign(n, 0); m_FaceCounts.assign(n, 0);
    std::vector<uint32_t> uniquePerMesh;
    m_Positions.clear(); m_Indices.clear(); m_FaceMats.clear();
    size_t n_vert = 0, n_idx = 0, n_fm = 0;
    for (const MeshData& md : meshes) { n_vert += md.vertices.size(); n_idx += md.indices.size(); n_fm += md.faceMaterialIds.size(); }
    m_Positions.resize(3 * n_vert);
    m_Indices.reserve(n_idx);
    m_FaceMats.reserve(n_fm);
    for (int i = 0; i < n; i++) {
        const MeshData& md = meshes[i];
        m_VertexOffsets[i] = i == 0 ? 0u : m_VertexOffsets[i - 1] + (uint32_t)meshes[i - 1].vertices.size();
        m_IndexOffsets[i] = (uint32_t)m_Indices.size();
        m_FaceMatOffsets[i] = (uint32_t)m_FaceMats.size();
        float* pos = m_Positions.data() + 3 * (size_t)m_VertexOffsets[i];
        CRT::parallel_ranges(md.vertices.size(), [&](size_t b, size_t e) {
            for (size_t v = b; v < e; ++v)
                for (int c = 0; c < 3; ++c) pos[3 * v + c] = md.vertices[v].Position[c];
        });
        m_Indices.insert(m_Indices.end(), md.indices.begin(), md.indices.end());
        m_FaceMats.insert(m_FaceMats.end(), md.faceMaterialIds.begin(), md.faceMaterialIds.end());
        // :143-145 std::set of the face material ids: its size.  loadObject clamps every id into [0, materials), so
        // a flag per material counts the same distinct values (other ids, which it never produces, go to a set)
        std::vector<char> seen;
        std::set<int> other;
        uint32_t distinct = 0;
        for (int id : md.faceMaterialIds) {
            if (id < 0 || id >= (1 << 20)) {
                distinct += other.insert(id).second ? 1u : 0u;
                continue;
            }
            if ((size_t)id >= seen.size()) seen.resize((size_t)id + 1, 0);
            distinct += !seen[(size_t)id];
            seen[(size_t)id] = 1;
        }
        uniquePerMesh.push_back(distinct);
        m_VertexCounts[i] = (uint32_t)md.vertices.size();
        m_IndexCounts[i] = (uint32_t)md.indices.size();
        m_FaceCounts[i] = (uint32_t)md.faceMaterialIds.size();
    }
    tr.lap("mesh arrays");
    m_MaterialIDOffsets.assign(n, 0);
    m_Meshes.assign(n, crt_mesh_desc{});
    m_MeshBVH.assign(n, {});
    m_MeshBoxes.assign(n, CRT::AABB());
    for (int i = 0; i < n; i++) {
        m_MaterialIDOffsets[i] = i == 0 ? 0 : uniquePerMesh[i - 1];                     // :177 (previous mesh only)
        for (uint32_t k = 0; k < m_IndexCounts[i]; ++k)
            if (m_Indices[m_IndexOffsets[i] + k] >= m_VertexCounts[i])
                throw std::runtime_error("mesh index out of range of its vertex slots");
        // Mesh ctor + buildBVHMesh (CUDAKernels.h:92-100, Mesh.cuh:18-53)
        const float* pos = m_Positions.data() + 3 * (size_t)m_VertexOffsets[i];
        uint32_t* idx = m_Indices.data() + m_IndexOffsets[i];
        int32_t* fm = m_FaceMats.data() + m_FaceMatOffsets[i];
        if (m_BuildDevice >= 0 && buildMeshOnDevice(i, pos, idx, fm)) continue;
        CRT::BuildStatus st = CRT::buildMeshBVH(pos, m_VertexCounts[i], idx, fm, m_IndexCounts[i], &m_MeshBoxes[i],
                                                &m_MeshBVH[i]);
        if (!st.ok) throw std::runtime_error(st.error);
    }
    tr.lap("mesh BVHs");
    for (int i = 0; i < n; i++) {
        crt_mesh_desc& d = m_Meshes[i];
        d.vertex_offset = m_VertexOffsets[i];
        d.vertex_count = m_VertexCounts[i];
        d.index_offset = m_IndexOffsets[i];
        d.index_count = m_IndexCounts[i];
        d.face_offset = m_FaceMatOffsets[i];
        d.material_id_offset = m_MaterialIDOffsets[i];
        d.nodes = m_MeshBVH[i].data();
        d.node_count = (int32_t)m_MeshBVH[i].size();
        const CRT::AABB& b = m_MeshBoxes[i];
        d.aabb[0] = b.x.min; d.aabb[1] = b.y.min; d.aabb[2] = b.z.min;
        d.aabb[3] = b.x.max; d.aabb[4] = b.y.max; d.aabb[5] = b.z.max;
    }
}

// :198-329
void SceneManager::loadObject(const std::string& filename, std::vector<MeshData>& meshDataList) {
    size_t last = filename.find_last_of("/\\");
    std::string base_dir = last != std::string::npos ? filename.substr(0, last + 1) : "./";
    CRT::ObjData od;
    std::string err;
    LoadTrace tr;
    if (!CRT::LoadObj(&od, &err, filename.c_str(), base_dir.c_str())) {
        if (!err.empty()) std::cerr << "ObjLoader error:   " << err << std::endl;
        throw std::runtime_error("Failed to load object: " + filename);
    }
    tr.lap("  LoadObj");
    for (const auto& mat : od.materials) {                                           // :222-247
        CRT::MaterialType mt = CRT::MaterialType::Lambertian;
        if (mat.emission[0] > 0.f || mat.emission[1] > 0.f || mat.emission[2] > 0.f) mt = CRT::MaterialType::DiffuseLight;
        else if (mat.dissolve < 1.f) mt = CRT::MaterialType::Dielectric;
        else if (mat.specular[0] > 0.f) mt = CRT::MaterialType::Metal;
        float r = 0.f;
        if (mt == CRT::MaterialType::Metal) {
            if (mat.roughness > 0.f) r = mat.roughness;
            else r = sqrtf(2.f / (mat.shininess + 2.f));
        }
        float ior = (mt == CRT::MaterialType::Dielectric ? mat.ior : 1.f);
        m_SceneMaterialsData.emplace_back(mt, CRT::Vec3(mat.diffuse[0], mat.diffuse[1], mat.diffuse[2]), r, ior,
                                          CRT::Vec3(mat.emission[0], mat.emission[1], mat.emission[2]));
    }
    MeshData meshData;
    const size_t nTri = od.triMaterial.size();
    if (nTri > 0) meshData.vertices.resize(od.vertices.size());                         // :253 (3x too many slots)
    for (size_t k = 0; k < 3 * nTri; ++k) {
        const int32_t vi = od.triIndices[k];
        if (vi < 0 || 3 * (size_t)vi + 2 >= od.vertices.size())
            throw std::runtime_error("face vertex index out of range in " + filename);
    }
    meshData.faceMaterialIds.resize(nTri);
    meshData.indices.resize(3 * nTri);
    const int n_mats = static_cast<int>(m_SceneMaterialsData.size());
    CRT::parallel_ranges(nTri, [&](size_t b, size_t e) {
        for (size_t f = b; f < e; ++f) {
            int faceMatId = od.triMaterial[f];                                        // :259-265
            if (faceMatId < 0 || faceMatId >= n_mats) faceMatId = 0;
            meshData.faceMaterialIds[f] = faceMatId;
            for (int v = 0; v < 3; v++) meshData.indices[3 * f + v] = (uint32_t)od.triIndices[3 * f + v];
        }
    });
    // :300 vertices[vi] = the face's vertex, last write wins: every face writes vertex vi's own position, so the slot
    // of each referenced index gets od.vertices[vi] (the rest stay zero)
    std::vector<char> used(od.vertices.size() / 3, 0);
    for (size_t k = 0; k < 3 * nTri; ++k) used[(size_t)od.triIndices[k]] = 1;
    CRT::parallel_ranges(used.size(), [&](size_t b, size_t e) {
        for (size_t vi = b; vi < e; ++vi)
            if (used[vi]) meshData.vertices[vi].Position = CRT::Vec3(od.vertices[3 * vi], od.vertices[3 * vi + 1], od.vertices[3 * vi + 2]);
    });
    tr.lap("  mesh data");
    meshDataList.push_back(std::move(meshData));
    // :307-325 — normalise every mesh loaded so far.  The bounds fold over the meshes' vertices in order, per range
    // and then over the ranges in order: fmin / fmax return the same operand on ties either way, so the result is the
    // sequential fold's
    CRT::Vec3 minBounds(std::numeric_limits<float>::max());
    CRT::Vec3 maxBounds(std::numeric_limits<float>::lowest());
    for (auto& md : meshDataList) {
        std::vector<CRT::Vec3> lo(16, CRT::Vec3(std::numeric_limits<float>::max()));
        std::vector<CRT::Vec3> hi(16, CRT::Vec3(std::numeric_limits<float>::lowest()));
        const size_t R = CRT::parallel_ranges_indexed(md.vertices.size(), [&](size_t r, size_t b, size_t e) {
            CRT::Vec3 l = lo[r], h = hi[r];
            for (size_t v = b; v < e; ++v) {
                l = CRT::Vec3::min(l, md.vertices[v].Position);
                h = CRT::Vec3::max(h, md.vertices[v].Position);
            }
            lo[r] = l;
            hi[r] = h;
        });
        for (size_t r = 0; r < R; ++r) {
            minBounds = CRT::Vec3::min(minBounds, lo[r]);
            maxBounds = CRT::Vec3::max(maxBounds, hi[r]);
        }
    }
    CRT::Vec3 center = (minBounds + maxBounds) * 0.5f;
    float scale = 0.6f / (maxBounds - minBounds).maxComponent();
    for (auto& md : meshDataList)
        CRT::parallel_ranges(md.vertices.size(), [&](size_t b, size_t e) {
            for (size_t v = b; v < e; ++v) md.vertices[v].Position = (md.vertices[v].Position - center) * scale;
        });
}

// createRandomWorld (CUDAKernels.h:28-84) + createBVH (:86-90)
void SceneManager::createWorld() {
    const int MAX_OBJECTS = 500, MAX_MATERIALS = 500;   // HittableList.cuh:70-71
    m_Materials.clear(); m_Spheres.clear(); m_Objects.clear();
    auto addMaterial = [&](const crt_material_desc& m) -> int {
        if ((int)m_Materials.size() < MAX_MATERIALS) { m_Materials.push_back(m); return (int)m_Materials.size() - 1; }
        return -1;
    };
    for (const auto& md : m_SceneMaterialsData) {
        crt_material_desc m{};
        m.type = (int32_t)md.getType();
        CRT::Vec3 a = md.getAlbedo(), e = md.getEmission();
        for (int c = 0; c < 3; ++c) { m.albedo[c] = a[c]; m.emission[c] = e[c]; }
        m.roughness = md.getRoughness() < 1.f ? md.getRoughness() : 1.f;          // Metal ctor, Material.cuh:86
        m.ior = md.getIOR();
        addMaterial(m);
    }
    std::vector<CRT::AABB> boxes;
    auto addObject = [&](int kind, int index, const CRT::AABB& box) {
        if ((int)m_Objects.size() < MAX_OBJECTS) { m_Objects.push_back({kind, index}); boxes.push_back(box); }
    };
    for (int i = 0; i < (int)m_Meshes.size(); ++i) addObject(CRT_OBJECT_MESH, i, m_MeshBoxes[i]);
    auto addSphere = [&](CRT::Vec3 c, float r, int mat) {
        crt_sphere_desc s{{c[0], c[1], c[2]}, r, mat};
        m_Spheres.push_back(s);
        CRT::Vec3 rv(r, r, r);
        addObject(CRT_OBJECT_SPHERE, (int)m_Spheres.size() - 1, CRT::AABB(c - rv, c + rv));   // Sphere.cuh:20-25
    };
    crt_material_desc ground{};
    ground.type = CRT_LAMBERTIAN;
    ground.albedo[0] = ground.albedo[1] = ground.albedo[2] = 0.5f;
    ground.ior = 1.f;
    int gi = addMaterial(ground);
    addSphere(CRT::Vec3(0, -1000, 0), 999, gi);
    crt_material_desc metal{};
    metal.type = CRT_METAL;
    metal.albedo[0] = (float)0.7; metal.albedo[1] = (float)0.6; metal.albedo[2] = (float)0.5;
    metal.roughness = 0.0f;
    metal.ior = 1.f;
    int mi = addMaterial(metal);
    addSphere(CRT::Vec3((float)0.2, (float)0.2, 0), 0.05f, mi);
    CRT::BuildStatus st = CRT::buildSceneBVH(boxes, &m_SceneBVH);
    if (!st.ok) throw std::runtime_error(st.error);
}

crt_scene_desc SceneManager::sceneDesc() const {
    crt_scene_desc d{};
    d.positions = m_Positions.data();
    d.n_positions = m_Positions.size() / 3;
    d.indices = m_Indices.data();
    d.n_indices = m_Indices.size();
    d.face_materials = m_FaceMats.data();
    d.n_faces = m_FaceMats.size();
    d.meshes = m_Meshes.data();
    d.n_meshes = (int32_t)m_Meshes.size();
    d.spheres = m_Spheres.data();
    d.n_spheres = (int32_t)m_Spheres.size();
    d.objects = m_Objects.data();
    d.n_objects = (int32_t)m_Objects.size();
    d.scene_nodes = m_SceneBVH.data();
    d.n_scene_nodes = (int32_t)m_SceneBVH.size();
    d.materials = m_Materials.data();
    d.n_materials = (int32_t)m_Materials.size();
    return d;
}
