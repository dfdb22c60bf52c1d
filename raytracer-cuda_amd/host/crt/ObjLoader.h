// ObjLoader.h — OBJ/MTL parser with tinyobjloader v1.0.x semantics, the
// third-party loader the reference calls at SceneManager.h:215 (6-argument
// LoadObj ⇒ v1.0.x API; tinyobjloader is not vendored in the reference and not in
// this image, so its version is unpinned).  Restated behaviour:
//   * tryParseDouble float parsing (mantissa accumulated in double, then cast);
//   * `v` positions, `f` with v / v/t / v//n / v/t/n tokens, fixIndex (1-based,
//     negative = relative to the vertices seen so far);
//   * polygon -> triangle FAN (0,k-1,k) triangulation, faces with <3 vertices dropped;
//   * per-face material id = the `usemtl` active when the face was read (-1 if none);
//   * `mtllib` resolved against the caller's base_dir; LoadMtl defaults
//     (dissolve 1, ior 1, shininess 1, roughness 0), `Tr` => dissolve = 1 - Tr.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace CRT {

struct ObjMaterial {
    std::string name;
    float diffuse[3] = {0, 0, 0};
    float specular[3] = {0, 0, 0};
    float emission[3] = {0, 0, 0};
    float dissolve = 1.f;
    float ior = 1.f;
    float shininess = 1.f;
    float roughness = 0.f;
};

struct ObjData {
    std::vector<float> vertices;         // attrib.vertices (3 floats per `v`)
    std::vector<int32_t> triIndices;     // 3 vertex_index per triangle (after fan triangulation)
    std::vector<int32_t> triMaterial;    // shape.mesh.material_ids per triangle
    std::vector<ObjMaterial> materials;
};

// Returns false and fills `err` on failure (file missing, malformed index).
bool LoadObj(ObjData* out, std::string* err, const char* filename, const char* mtl_basedir);

// tinyobj tryParseDouble restatement (exposed for tests).
bool TryParseDouble(const char* s, const char* s_end, double* result);

}  // namespace CRT
