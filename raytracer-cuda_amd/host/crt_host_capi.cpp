// crt_host_capi.cpp — C ABI over the host C++ scene pipeline (include/crt_host.h).
#include <cstring>
#include <memory>
#include <exception>
#include <string>

#include "crt/Camera.h"
#include "crt/ImageIO.h"
#include "crt/Raytracer.h"
#include "crt/SceneManager.h"
#include "crt_host.h"

struct crth_scene {
    SceneManager sm{1, 1};
    // unpermuted loader output (before the mesh BVH builds reorder indices / face materials)
    std::vector<uint32_t> idx0;
    std::vector<int32_t> fmat0;
};

struct crth_camera_ctl {
    CRT::Camera cam;
};

struct crth_viewer {
    std::unique_ptr<CRT::Raytracer> rt;
};

static thread_local std::string g_err;

static CRT::InputState to_input(const crth_input* in) {
    CRT::InputState s;
    if (!in) return s;
    s.mouseX = in->mouse_x;
    s.mouseY = in->mouse_y;
    s.rightMouse = in->right_mouse != 0;
    s.keyW = (in->keys & CRTH_KEY_W) != 0;
    s.keyA = (in->keys & CRTH_KEY_A) != 0;
    s.keyS = (in->keys & CRTH_KEY_S) != 0;
    s.keyD = (in->keys & CRTH_KEY_D) != 0;
    s.keySpace = (in->keys & CRTH_KEY_SPACE) != 0;
    s.keyLControl = (in->keys & CRTH_KEY_LCONTROL) != 0;
    s.keyF = (in->keys & CRTH_KEY_F) != 0;
    s.focusSteps = in->focus_steps;
    return s;
}

extern "C" {

const char* crth_last_error(void) { return g_err.c_str(); }

int crth_scene_load(const char* const* files, int n, crth_scene** out) { return crth_scene_load_ex(files, n, -1, out); }

double crth_scene_build_ms(const crth_scene* s) { return s ? s->sm.deviceBuildMs() : 0.0; }

int crth_scene_load_ex(const char* const* files, int n, int build_device, crth_scene** out) {
    if (!files || n < 0 || !out) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    *out = nullptr;
    try {
        crth_scene* s = new crth_scene;
        std::vector<std::string> v;
        for (int i = 0; i < n; ++i) v.emplace_back(files[i]);
        s->sm.setModelFiles(v);
        s->sm.setMeshBuildDevice(build_device);
        s->sm.buildHostScene();
        // rebuild the unpermuted arrays from MeshData (the loader output)
        for (const auto& md : s->sm.meshData()) {
            s->idx0.insert(s->idx0.end(), md.indices.begin(), md.indices.end());
            s->fmat0.insert(s->fmat0.end(), md.faceMaterialIds.begin(), md.faceMaterialIds.end());
        }
        *out = s;
        return CRT_OK;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CRT_ERR_INVALID_ARGUMENT;
    }
}

void crth_scene_destroy(crth_scene* s) { delete s; }

int crth_scene_desc(const crth_scene* s, crt_scene_desc* out) {
    if (!s || !out) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    *out = s->sm.sceneDesc();
    return CRT_OK;
}

int crth_scene_upload(const crth_scene* s, int device, crt_scene** out) {
    if (!s || !out) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    crt_scene_desc d = s->sm.sceneDesc();
    int rc = crt_scene_create(&d, device, out);
    if (rc) g_err = crt_last_error();
    return rc;
}

int crth_scene_upload_ex(const crth_scene* s, int device, const crt_scene_options* opts, crt_scene** out) {
    if (!s || !out) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    crt_scene_desc d = s->sm.sceneDesc();
    int rc = crt_scene_create_ex(&d, device, opts, out);
    if (rc) g_err = crt_last_error();
    return rc;
}

int crth_scene_counts(const crth_scene* s, int64_t* c) {
    if (!s || !c) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    c[0] = (int64_t)s->sm.meshes().size();
    c[1] = (int64_t)s->sm.positions().size() / 3;
    c[2] = (int64_t)s->sm.indices().size();
    c[3] = (int64_t)s->sm.faceMaterials().size();
    c[4] = (int64_t)s->sm.sceneMaterialsData().size();
    return CRT_OK;
}

int crth_scene_loader_arrays(const crth_scene* s, float* pos, uint32_t* idx, int32_t* fm, uint32_t* info, float* mats) {
    if (!s) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    const auto& P = s->sm.positions();
    // (an empty vector's data() may be null, and memcpy from null is undefined even for 0 bytes: UBSan, tools/run_asan.sh)
    if (pos && !P.empty()) std::memcpy(pos, P.data(), P.size() * sizeof(float));
    if (idx && !s->idx0.empty()) std::memcpy(idx, s->idx0.data(), s->idx0.size() * sizeof(uint32_t));
    if (fm && !s->fmat0.empty()) std::memcpy(fm, s->fmat0.data(), s->fmat0.size() * sizeof(int32_t));
    if (info) {
        const auto& M = s->sm.meshes();
        for (size_t i = 0; i < M.size(); ++i) {
            uint32_t* o = info + 6 * i;
            o[0] = M[i].vertex_offset; o[1] = M[i].vertex_count; o[2] = M[i].index_offset;
            o[3] = M[i].index_count; o[4] = M[i].face_offset; o[5] = M[i].material_id_offset;
        }
    }
    if (mats) {
        const auto& D = s->sm.sceneMaterialsData();
        for (size_t i = 0; i < D.size(); ++i) {
            float* o = mats + 9 * i;
            o[0] = (float)(int)D[i].getType();
            for (int c = 0; c < 3; ++c) { o[1 + c] = D[i].getAlbedo()[c]; o[4 + c] = D[i].getEmission()[c]; }
            o[7] = D[i].getRoughness();
            o[8] = D[i].getIOR();
        }
    }
    return CRT_OK;
}

int crth_camera(float aspect, float vfov, const float* pos3, const float* up3, float aperture, float focus,
                float yaw, float pitch, int spp, crt_camera_desc* out) {
    if (!pos3 || !up3 || !out || spp <= 0) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    CRT::Camera cam(aspect, vfov, CRT::Vec3(pos3[0], pos3[1], pos3[2]), CRT::Vec3(0, 0, 0),
                    CRT::Vec3(up3[0], up3[1], up3[2]), aperture, focus);
    if (yaw != -90.0f || pitch != 0.0f) cam.setYawPitch(yaw, pitch);
    cam.setSamplesPerPixel(spp);
    *out = cam.toDesc();
    return CRT_OK;
}

int crth_build_mesh_bvh(const float* positions, uint32_t vertex_count, uint32_t* indices, int32_t* face_materials,
                        uint32_t index_count, crt_bvh_node_desc* nodes, int32_t* node_count, float mesh_box[6]) {
    if (!node_count || !mesh_box || (vertex_count && !positions) || (index_count && (!indices || !face_materials))) {
        g_err = "bad argument";
        return CRT_ERR_INVALID_ARGUMENT;
    }
    std::vector<crt_bvh_node_desc> out;
    CRT::AABB box;
    const CRT::BuildStatus st =
        CRT::buildMeshBVH(positions, vertex_count, indices, face_materials, index_count, &box, &out);
    if (!st.ok) { g_err = st.error; return CRT_ERR_INVALID_ARGUMENT; }
    if (!out.empty()) {
        if (!nodes) { g_err = "null nodes"; return CRT_ERR_INVALID_ARGUMENT; }
        std::memcpy(nodes, out.data(), out.size() * sizeof(crt_bvh_node_desc));
    }
    *node_count = (int32_t)out.size();
    mesh_box[0] = box.x.min; mesh_box[1] = box.y.min; mesh_box[2] = box.z.min;
    mesh_box[3] = box.x.max; mesh_box[4] = box.y.max; mesh_box[5] = box.z.max;
    return CRT_OK;
}

int crth_camera_create(float aspect, float vfov, const float* pos3, const float* up3, float aperture, float focus,
                       crth_camera_ctl** out) {
    if (!pos3 || !up3 || !out) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    *out = new crth_camera_ctl{CRT::Camera(aspect, vfov, CRT::Vec3(pos3[0], pos3[1], pos3[2]), CRT::Vec3(0, 0, 0),
                                       CRT::Vec3(up3[0], up3[1], up3[2]), aperture, focus)};
    return CRT_OK;
}

int crth_camera_update(crth_camera_ctl* c, float dt, int w, int h, const crth_input* in) {
    if (!c || !in) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    const CRT::InputState s = to_input(in);
    for (int k = 0; k < s.focusSteps; ++k) c->cam.adjustFocusDistance(0.1f);   // WindowManager.h:64-67
    for (int k = 0; k > s.focusSteps; --k) c->cam.adjustFocusDistance(-0.1f);
    c->cam.updateCamera(dt, w, h, s);
    return CRT_OK;
}

int crth_camera_get(const crth_camera_ctl* c, crt_camera_desc* desc, float* st) {
    if (!c) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    if (desc) *desc = c->cam.toDesc();
    if (st) {
        st[0] = c->cam.yaw();
        st[1] = c->cam.pitch();
        st[2] = c->cam.isMoving() ? 1.f : 0.f;
        st[3] = c->cam.isRotating() ? 1.f : 0.f;
        st[4] = c->cam.isHighQuality() ? 1.f : 0.f;
        st[5] = c->cam.getFocusDistance();
    }
    return CRT_OK;
}

void crth_camera_destroy(crth_camera_ctl* c) { delete c; }

int crth_viewer_create(const char* const* files, int n_files, int device, const crt_scene_options* opts, int width,
                       int height, float aspect, float vfov, float aperture, const float* pos3, float focus,
                       unsigned long long seed, int accumulate, crth_viewer** out) {
    if (!out || (n_files > 0 && !files) || n_files < 0 || width <= 0 || height <= 0) {
        g_err = "bad argument";
        return CRT_ERR_INVALID_ARGUMENT;
    }
    *out = nullptr;
    try {
        CRT::RaytracerOptions o;
        for (int i = 0; i < n_files; ++i) o.modelFiles.emplace_back(files[i]);
        if (opts) o.scene = *opts;
        o.seed = seed;
        o.device = device;
        if (pos3) { o.hasPose = true; o.position = CRT::Vec3(pos3[0], pos3[1], pos3[2]); }
        o.focusDist = focus;
        o.accumulate = accumulate != 0;
        auto v = std::make_unique<crth_viewer>();
        v->rt = std::make_unique<CRT::Raytracer>(width, height, aspect, vfov, aperture, o);
        *out = v.release();
        return CRT_OK;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CRT_ERR_INVALID_ARGUMENT;
    }
}

int crth_viewer_frame(crth_viewer* v, float dt, const crth_input* in, crth_frame_info* info) {
    if (!v || !in) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    try {
        const CRT::FrameInfo fi = v->rt->updateAndRender(dt, to_input(in));
        if (info) {
            info->frame = fi.frame;
            info->spp = fi.spp;
            info->accumulated = fi.accumulated;
            info->moving = fi.moving;
            info->high_quality = fi.highQuality;
            info->kernel_ms = fi.kernelMs;
            info->frame_ms = fi.frameMs;
        }
        return CRT_OK;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CRT_ERR_HIP;
    }
}

int crth_viewer_camera(const crth_viewer* v, crt_camera_desc* out) {
    if (!v || !out) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    *out = v->rt->camera().toDesc();
    return CRT_OK;
}

crt_renderer* crth_viewer_renderer(crth_viewer* v) { return v ? v->rt->renderer().handle() : nullptr; }

void crth_viewer_destroy(crth_viewer* v) { delete v; }

int crth_encode_image(int format, const uint8_t* rgba, int w, int h, int flip, uint8_t* out, uint64_t* size) {
    if (!rgba || !size || w <= 0 || h <= 0 || (format != CRTH_IMAGE_PPM && format != CRTH_IMAGE_PNG)) {
        g_err = "bad argument";
        return CRT_ERR_INVALID_ARGUMENT;
    }
    try {
        const std::vector<uint8_t> bytes = format == CRTH_IMAGE_PNG ? CRT::encodePNG(rgba, w, h, flip != 0)
                                                                    : CRT::encodePPM(rgba, w, h, flip != 0);
        const uint64_t cap = *size;
        *size = bytes.size();
        if (!out) return CRT_OK;
        if (cap < bytes.size()) { g_err = "output buffer too small"; return CRT_ERR_INVALID_ARGUMENT; }
        std::memcpy(out, bytes.data(), bytes.size());
        return CRT_OK;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CRT_ERR_INVALID_ARGUMENT;
    }
}

int crth_write_image(const char* path, const uint8_t* rgba, int w, int h, int flip) {
    if (!path) { g_err = "bad argument"; return CRT_ERR_INVALID_ARGUMENT; }
    try {
        CRT::writeImage(path, rgba, w, h, flip != 0);
        return CRT_OK;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CRT_ERR_INVALID_ARGUMENT;
    }
}

}  // extern "C"
