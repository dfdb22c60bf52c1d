/*
 * crt_host.h — C ABI of the host scene pipeline (libcrt_host.so): the reference's
 * SceneManager host path (OBJ/MTL load, normalisation, mesh concat, Mesh/Scene BVH
 * builds, createRandomWorld order) and Camera, implemented in C++
 * (raytracer-cuda_amd/host/crt/) and exposed as plain C for FFI callers (the
 * Python bench/tests bind it with ctypes).  The C++ API itself (SceneManager,
 * CRT::Camera, CUDARenderer/HIPRenderer) is the drop-in for reference host code.
 */
#ifndef CRT_HOST_H
#define CRT_HOST_H

#include <stdint.h>

#include "crt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct crth_scene crth_scene;

/* Load + build on the host (SceneManager::initializeScene minus the upload). */
int crth_scene_load(const char* const* obj_files, int n_files, crth_scene** out);
void crth_scene_destroy(crth_scene* s);
/* The flat description handed to crt_scene_create (pointers stay owned by `s`). */
int crth_scene_desc(const crth_scene* s, crt_scene_desc* out);
/* Upload to `device` (crt_scene_create on the desc). */
int crth_scene_upload(const crth_scene* s, int device, crt_scene** out);
/* crth_scene_upload with crt_scene_options (NULL = CRT_BVH_REFERENCE). */
int crth_scene_upload_ex(const crth_scene* s, int device, const crt_scene_options* opts, crt_scene** out);

/* Loader output before the BVH permutation, for parity tests against the oracle loader.
 * counts_out: n_meshes, n_slots, n_indices, n_faces, n_materials (5 x int64). */
int crth_scene_counts(const crth_scene* s, int64_t* counts_out);
/* positions (n_slots*3), indices (unpermuted), face mats (unpermuted), mesh_info (n_meshes*6:
 * vertexOffset, vertexCount, indexOffset, indexCount, faceMatOffset, matIDOffset),
 * file materials (n_materials*9: type, albedo3, emission3, roughness, ior). Any pointer may be NULL. */
int crth_scene_loader_arrays(const crth_scene* s, float* positions, uint32_t* indices, int32_t* facemat,
                             uint32_t* mesh_info, float* materials);

/* CRT::Camera(aspect, fov, pos, target(ignored), up, aperture, focus) + setYawPitch + spp. */
int crth_camera(float aspect, float vfov, const float* pos3, const float* up3, float aperture, float focus,
                float yaw, float pitch, int spp, crt_camera_desc* out);

/* ---- frame output (WindowManager::drawFrame, WindowManager.h:79-93, headless) ----
 * rgba: W*H*4 bytes as the renderer holds them (row 0 = bottom).  flip != 0 writes the top row first, as
 * the window shows it (flipVertically).  Files are 8-bit RGB. */
#define CRTH_IMAGE_PPM 0
#define CRTH_IMAGE_PNG 1
/* Encode into out[*size]; on entry *size is the capacity (out may be NULL to query), on return the
 * encoded length.  Returns CRT_ERR_INVALID_ARGUMENT (with *size set) when the capacity is too small. */
int crth_encode_image(int format, const uint8_t* rgba, int width, int height, int flip, uint8_t* out, uint64_t* size);
/* Write .png or .ppm by the path's extension. */
int crth_write_image(const char* path, const uint8_t* rgba, int width, int height, int flip);

const char* crth_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
