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
/* crth_scene_load with the mesh BVHs built on GPU `build_device` (crt_build_mesh_bvh: the same trees as the host
 * restatement; meshes the reference's node cap decides fall back to the host); build_device < 0 = host. */
int crth_scene_load_ex(const char* const* obj_files, int n_files, int build_device, crth_scene** out);
/* Device milliseconds of the GPU mesh BVH builds of the last load (0 for host builds). */
double crth_scene_build_ms(const crth_scene* s);
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

/* The host restatement of Mesh::buildBVHMesh + the Mesh ctor box (Mesh.cuh:39-47, :121-264), same contract as
 * crt_build_mesh_bvh (crt_hip.h) but sequential on the host, exactly the reference's loop.  No GPU needed. */
int crth_build_mesh_bvh(const float* positions, uint32_t vertex_count, uint32_t* indices, int32_t* face_materials,
                        uint32_t index_count, crt_bvh_node_desc* nodes, int32_t* node_count, float mesh_box[6]);

/* ---- interactive loop (Raytracer.h:52-102, Camera.cuh:46-157), headless ----
 * The reference polls SFML each frame; here the caller passes what it would have polled. */
#define CRTH_KEY_W        1u
#define CRTH_KEY_A        2u
#define CRTH_KEY_S        4u
#define CRTH_KEY_D        8u
#define CRTH_KEY_SPACE    16u
#define CRTH_KEY_LCONTROL 32u
#define CRTH_KEY_F        64u   /* held: toggles high-quality mode (2000 spp) every frame, like isKeyPressed(F) */
typedef struct crth_input {
    float mouse_x, mouse_y;   /* sf::Mouse::getPosition(window) */
    int32_t right_mouse;      /* isRightMousePressed (rotation while held) */
    uint32_t keys;            /* CRTH_KEY_* held this frame */
    int32_t focus_steps;      /* PageUp (+1) / PageDown (-1) presses this frame: adjustFocusDistance(+-0.1) */
} crth_input;

/* Host-only camera controller: CRT::Camera(aspect, vfov, pos, target(ignored), up, aperture, focus) driven by
 * Camera::updateCamera(dt, w, h, input).  No GPU needed. */
typedef struct crth_camera_ctl crth_camera_ctl;
int  crth_camera_create(float aspect, float vfov, const float* pos3, const float* up3, float aperture, float focus,
                        crth_camera_ctl** out);
int  crth_camera_update(crth_camera_ctl* c, float dt, int window_width, int window_height, const crth_input* in);
/* state: yaw, pitch, moving, rotating, high_quality, focus (6 floats; flags as 0/1) */
int  crth_camera_get(const crth_camera_ctl* c, crt_camera_desc* desc, float* state6);
void crth_camera_destroy(crth_camera_ctl* c);

typedef struct crth_frame_info {
    int64_t frame;            /* frames rendered so far, this one included */
    int32_t spp;              /* samples traced this frame */
    int32_t accumulated;      /* samples in the displayed image */
    int32_t moving, high_quality;
    float kernel_ms;          /* render kernel (HIP events) */
    double frame_ms;          /* updateAndRender wall clock, synchronous */
} crth_frame_info;

/* Raytracer(width, height, aspect, vfov, aperture) over a loaded scene: uploads it to `device` with `opts`
 * (NULL = CRT_BVH_REFERENCE) and seeds every pixel's RNG (curand_init(seed, pixel, 0)).  pos3 NULL = the
 * reference's (0,4,4); focus <= 0 = |pos|.  accumulate != 0: still 1-spp frames add up (see Raytracer.h). */
typedef struct crth_viewer crth_viewer;
int  crth_viewer_create(const char* const* obj_files, int n_files, int device, const crt_scene_options* opts,
                        int width, int height, float aspect, float vfov, float aperture, const float* pos3,
                        float focus, unsigned long long seed, int accumulate, crth_viewer** out);
/* One frame: Raytracer::updateAndRender(dt, input); info may be NULL. */
int  crth_viewer_frame(crth_viewer* v, float dt, const crth_input* in, crth_frame_info* info);
int  crth_viewer_camera(const crth_viewer* v, crt_camera_desc* out);
/* The viewer's renderer (read_rgba8 / read_linear / read_rng / device pointers via crt_hip.h). */
crt_renderer* crth_viewer_renderer(crth_viewer* v);
void crth_viewer_destroy(crth_viewer* v);

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
