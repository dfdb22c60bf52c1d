/*
 * crt_hip.h — C ABI of the MI355X (gfx950) render layer: libcrt_hip.so.
 *
 * This is the drop-in boundary for the reference's device path
 * (Mordentary/RayTracer-Cuda, paths relative to CudaRayTracer/src/):
 *
 *   reference                                            replaced by
 *   ---------------------------------------------------  ------------------------------------
 *   CUDARenderer::initialize  (CUDARenderer.cuh:39-49)   crt_renderer_create + crt_renderer_init_rand
 *     initRandState<<<>>>     (CUDAKernels.h:18-26)      crt_renderer_init_rand
 *   CUDARenderer::updateCamera (CUDARenderer.cuh:51-53)  crt_renderer_set_camera
 *     cudaMemcpyToSymbol(d_camera) (Camera.cuh:213)
 *   CUDARenderer::render      (CUDARenderer.cuh:55-60)   crt_renderer_render + crt_renderer_resolve
 *     render<<<>>> / rayColor (CUDAKernels.h:102-166)    (crt_renderer_render_frame does both)
 *   CUDARenderer::getImageData (CUDARenderer.cuh:16)     crt_renderer_rgba_device_ptr / _read_rgba8
 *   CUDARenderer::getRandState (CUDARenderer.cuh:17)     crt_renderer_rng_device_ptr
 *   SceneManager::initializeScene device half           crt_scene_create (flat arrays; the host
 *     createRandomWorld / initMesh / createBVH <<<1,1>>>   builds the BVHs with the reference's
 *     (CUDAKernels.h:28-100, SceneManager.h:77-98)         semantics, see crt_host.h)
 *   SceneManager::getBVHNodes / getWorld (SceneManager.h:25-26)  the crt_scene handle
 *   CUDA_CHECK -> throw (CUDAHelpers.h:19-26)            int status + crt_last_error()
 *
 * Plain C: pointers and sizes only.  All device memory is owned by the opaque
 * handles; the caller owns every host buffer.  Handles are not thread-safe; use
 * one renderer per device (one process per GPU for multi-GPU).
 */
#ifndef CRT_HIP_H
#define CRT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRT_ABI_VERSION 3

enum crt_status {
    CRT_OK = 0,
    CRT_ERR_INVALID_ARGUMENT = -1,
    CRT_ERR_HIP = -2,          /* a HIP runtime call failed; see crt_last_error() */
    CRT_ERR_OUT_OF_MEMORY = -3,
    CRT_ERR_NO_DEVICE = -4,
    CRT_ERR_UNSUPPORTED = -5
};

/* Material.cuh:8-14 MaterialType */
enum crt_material_type { CRT_LAMBERTIAN = 0, CRT_METAL = 1, CRT_DIELECTRIC = 2, CRT_DIFFUSE_LIGHT = 3 };

/* Material.cuh:16-47 MaterialData (roughness is clamped to <= 1 like the Metal ctor, Material.cuh:86). */
typedef struct crt_material_desc {
    int32_t type;
    float albedo[3];
    float emission[3];
    float roughness;
    float ior;
} crt_material_desc;

/* One reference BVHNode (BVHNode.cuh:158-165 fields): box + children / leaf range. */
typedef struct crt_bvh_node_desc {
    float bmin[3];
    float bmax[3];
    int32_t left, right;          /* internal nodes */
    int32_t obj_index, obj_count; /* leaves: mesh = index range [obj_index, obj_index+obj_count) step 3;
                                     scene = object index */
    int32_t is_leaf;
} crt_bvh_node_desc;

/* One Mesh (Mesh.cuh:18-53 ctor arguments + its built BVH). */
typedef struct crt_mesh_desc {
    uint32_t vertex_offset, vertex_count;
    uint32_t index_offset, index_count;
    uint32_t face_offset;          /* into face_materials */
    uint32_t material_id_offset;   /* Mesh::m_MatIDOffset */
    const crt_bvh_node_desc* nodes;/* Mesh::m_MeshBVH in builder index order (root = 0) */
    int32_t node_count;
    float aabb[6];                 /* Mesh::m_BoundingBox  min xyz, max xyz */
} crt_mesh_desc;

/* Sphere.cuh:20-25 */
typedef struct crt_sphere_desc {
    float center[3];
    float radius;
    int32_t material;
} crt_sphere_desc;

enum crt_object_kind { CRT_OBJECT_MESH = 0, CRT_OBJECT_SPHERE = 1 };
typedef struct crt_object_desc {   /* HittableList::m_Objects entry (HittableList.cuh:73) */
    int32_t kind;
    int32_t index;                 /* into meshes[] or spheres[] */
} crt_object_desc;

typedef struct crt_scene_desc {
    const float* positions;        /* vertex slots, xyz per slot (Vertex::Position, Mesh.cuh:5-10) */
    uint64_t n_positions;
    const uint32_t* indices;       /* per-mesh local vertex indices, AFTER the mesh BVH build permuted them */
    uint64_t n_indices;
    const int32_t* face_materials; /* per triangle, permuted with the indices */
    uint64_t n_faces;
    const crt_mesh_desc* meshes;
    int32_t n_meshes;
    const crt_sphere_desc* spheres;
    int32_t n_spheres;
    const crt_object_desc* objects;   /* HittableList order (CUDAKernels.h:64-73) */
    int32_t n_objects;
    const crt_bvh_node_desc* scene_nodes;  /* BVHNode::buildBVHScene output, root = 0 */
    int32_t n_scene_nodes;
    const crt_material_desc* materials;    /* HittableList::m_Materials order */
    int32_t n_materials;
} crt_scene_desc;

/* Camera POD as the kernel needs it (Camera.cuh:32-44 reads exactly these). */
typedef struct crt_camera_desc {
    float origin[3];       /* m_Position */
    float lower_left[3];   /* m_LowerLeftCorner */
    float horizontal[3];   /* m_Horizontal */
    float vertical[3];     /* m_Vertical */
    float right[3];        /* m_Right */
    float up[3];           /* m_Up */
    float lens_radius;     /* m_LensRadius */
    int32_t samples_per_pixel;   /* m_SamplesPerPixel */
    float pixel_sample_scale;    /* m_PixelSampleScale = 1.f / spp */
} crt_camera_desc;

typedef struct crt_scene_stats {
    int64_t device_nodes;      /* flattened (threaded, DFS-preorder) nodes incl. scene level */
    int64_t device_prims;      /* triangles + spheres */
    int64_t device_bytes;      /* node + prim + material bytes resident in HBM */
    int32_t max_depth;         /* deepest node (scene + mesh levels) */
    int32_t n_materials;
    int32_t bvh;               /* CRT_BVH_REFERENCE | CRT_BVH_REBUILT */
    int32_t layouts;           /* threaded node orders resident (device_nodes counts all of them) */
    int64_t excluded_prims;    /* REBUILT: triangles the reference can never hit (zero-thickness boxes) */
    int32_t width;             /* 2 (threaded binary nodes) or 4 (4-wide nodes) */
    int32_t stack_bound;       /* width 4: traversal-stack entries a ray can need */
    int64_t spatial_splits;    /* REBUILT with spatial_splits: nodes cut by a plane (SBVH) */
    int64_t references;        /* REBUILT: primitive references in the tree's leaves (> primitives with spatial splits) */
} crt_scene_stats;

typedef struct crt_work_counters {  /* filled by a CRT_RENDER_COUNT_WORK render */
    uint64_t rays;           /* closest-hit queries = calls of the scene-level hit (CUDAKernels.h:123) */
    uint64_t box_tests;      /* AABB::hit calls (scene + mesh levels) */
    uint64_t tri_tests;      /* rayTriangleIntersect calls */
    uint64_t sphere_tests;   /* Sphere::hit calls */
    uint64_t paths;          /* samples completed */
} crt_work_counters;

/* render flags */
#define CRT_RENDER_ACCUMULATE  1u   /* add into the existing linear sum instead of starting from 0 */
#define CRT_RENDER_COUNT_WORK  2u   /* counting kernel variant: fills crt_work_counters (slower) */

typedef struct crt_scene crt_scene;
typedef struct crt_renderer crt_renderer;

int crt_abi_version(void);
/* How this library was compiled: CRT_BUILD_CHECKED = the checked build (-DCRT_CHECKED, lib/checked/libcrt_hip.so):
 * the leaf rounds re-check every (owner, primitive) pair and report a bad one through crt_renderer_synchronize
 * instead of loading outside the primitive array.  Same frames, slower. */
#define CRT_BUILD_CHECKED 1
int crt_build_flags(void);
const char* crt_last_error(void);   /* thread-local message of the last failing call */
int crt_device_count(int* out);

/* Acceleration structure the device scene is traversed with.
 *   CRT_BVH_REFERENCE — the reference's own scene + mesh BVHs, flattened unchanged (default).  Bit-exact:
 *     same boxes, same visiting order, same culling, same work counters as BVHNode::hit / Mesh::hit.
 *   CRT_BVH_REBUILT   — a binned-SAH BVH over the same primitives with small padded leaves, collapsed to
 *     4-wide nodes (default; width 2 = threaded binary layouts).  Same hit rule as the
 *     reference: closest t in [0.001, closest], ties to the primitive the reference visits LAST
 *     (every primitive carries its reference DFS rank), primitives the reference can never reach
 *     (inside a zero-thickness box) excluded.  Results differ from the reference only where the
 *     reference's unpadded boxes round away a genuine hit; see DESIGN.md §4b for the measured rate. */
#define CRT_BVH_REFERENCE 0
#define CRT_BVH_REBUILT   1

typedef struct crt_scene_options {
    int32_t bvh;              /* CRT_BVH_REFERENCE | CRT_BVH_REBUILT */
    int32_t leaf_size;        /* REBUILT: max triangles per leaf, 1..16 (0 = default 4) */
    int32_t layouts;          /* REBUILT: 1 (single left-first order) or 6 (direction-ordered, default) */
    float traversal_cost;     /* REBUILT: SAH cost of one node step relative to one triangle test (0 = default 2) */
    int32_t width;            /* REBUILT: 4 (default) = 4-wide nodes, stack traversal (kernel variant 4); the
                                 tree holds at most 2^24 - 1 primitive references (24-bit record addressing in the
                                 leaf rounds; larger scenes fail with CRT_ERR_INVALID_ARGUMENT);
                                 2 = threaded binary layouts (variants 0-3) */
    int32_t gpu_build;        /* REBUILT: 1 = build the binned-SAH tree on the GPU (crt_scene_create_ex: the scene's
                                 device; crt_scene_export: device 0), 0 = on the host (default) */
    int32_t stack_cap;        /* REBUILT width 4: 0 = the traversal-stack bound computed from the tree (default); > 0
                                 overrides it.  Testing only: a value below the bound makes a render that needs more
                                 entries report CRT_ERR_HIP at synchronisation (the entries are dropped). */
    int32_t spatial_splits;   /* REBUILT: 1 = binned SAH with spatial splits (SBVH, Stich et al. 2009): a primitive
                                 straddling a split plane is referenced from both sides, each reference boxed by its
                                 part of the triangle.  Built on the host (gpu_build is ignored).  0 = object splits
                                 only (default). */
    float spatial_alpha;      /* spatial_splits: try a spatial split where the object split's children overlap by more
                                 than this fraction of the root's surface area (0 = default 1e-5) */
    float spatial_max_dup;    /* spatial_splits: stop splitting once references exceed (1 + this) x primitives
                                 (0 = default 1.0) */
} crt_scene_options;

/* ---- scene (SceneManager device half) ---- */
/* Host-only: build the device arrays crt_scene_create_ex would upload and copy them out (no GPU needed;
 * used by the CPU tests to validate the rebuilt BVH).  4-wide nodes are returned in their logical row order;
 * crt_scene_create_ex uploads them swizzled (row k of node n at 16-B slot k ^ (n & 7) of its 128-B record).
 * Call with null arrays to get the sizes:
 * info = {node float4s, prim float4s, ranks, nodes per layout, layouts, width, stack bound, excluded,
 *         first per-ray sphere prim, per-ray spheres}. */
int  crt_scene_export(const crt_scene_desc* desc, const crt_scene_options* opts, float* nodes, float* prims,
                      int32_t* rank_code, int64_t info[10]);
int  crt_scene_create(const crt_scene_desc* desc, int device, crt_scene** out);
/* crt_scene_create with options (NULL = defaults = CRT_BVH_REFERENCE). */
int  crt_scene_create_ex(const crt_scene_desc* desc, int device, const crt_scene_options* opts, crt_scene** out);
int  crt_scene_get_stats(const crt_scene* scene, crt_scene_stats* out);
void crt_scene_destroy(crt_scene* scene);

/* Diagnostic (no reference counterpart): renders spp samples per pixel following scene A (the
 * renderer's RNG state is consumed, its framebuffer is left untouched) and traces every ray through
 * scene B as well.  out = {rays, rays whose hit primitive differs, rays with the same primitive but a
 * different t, of the differing rays those B misses, those A misses}.  Both scenes must come from the
 * same crt_scene_desc.  Synchronous. */
int  crt_scene_compare(crt_renderer* r, const crt_scene* a, const crt_scene* b, int spp, int max_bounces,
                       uint64_t out[5]);
/* As crt_scene_compare, also copying up to max_dump differing rays to dump (10 floats each:
 * o.xyz, d.xyz, rank in a, rank in b (int bits), t in a, t in b). */
int  crt_scene_compare_dump(crt_renderer* r, const crt_scene* a, const crt_scene* b, int spp, int max_bounces,
                            uint64_t out[5], float* dump, int max_dump);

/* ---- renderer (CUDARenderer) ---- */
int  crt_renderer_create(int width, int height, int device, crt_renderer** out);
void crt_renderer_destroy(crt_renderer* r);
/* curand_init(seed, subsequence_base + y*width + x, 0) per pixel (CUDAKernels.h:18-26).
 * subsequence_base = shard * width * height for spp sharding. */
int  crt_renderer_init_rand(crt_renderer* r, unsigned long long seed, unsigned long long subsequence_base, void* stream);
/* CRT_ERR_INVALID_ARGUMENT for a non-finite origin or lens radius, or |origin| >= 2^59 / lens_radius >= 2^58 (the
 * rebuilt tree's slab test needs |o| * 2^64 finite; every real scene is many orders of magnitude inside it). */
int  crt_renderer_set_camera(crt_renderer* r, const crt_camera_desc* cam);
/* Render-kernel variant (identical results, different wave scheduling).  Scenes with threaded binary nodes
 * (CRT_BVH_REFERENCE, or REBUILT width 2): 0 = per-lane BVH traversal with per-lane leaf loops; 1 = per-lane
 * traversal with wave-cooperative leaf intersection; 2 = 1 + traversal-step scheduling with parked-lane regeneration
 * (lanes start their next ray without waiting for the wave's slowest trace); 3 = 2 + next-node prefetch overlapping
 * the leaf rounds; 10 = 3 with one wave per workgroup over 8x8 tiles in cost-probe order; anything else = automatic:
 * 10 when the render runs the cost probe (spp >= its minimum), else 3.  Scenes with 4-wide nodes (CRT_BVH_REBUILT,
 * width 4): 4 = the variant-3 scheduling over 4-wide nodes with a per-lane stack, 16x16-pixel workgroups; 7 = 4 with a
 * persistent grid whose lanes take pixels from a global queue (no lane waits for its wave's slowest pixel); 8 = 4 with
 * one wave per workgroup over 8x8 tiles in cost-probe order (crt_renderer_set_schedule); anything else = automatic: 8
 * when the render runs the cost probe, else 7.  Accepted values: -1 (automatic, the default), 0-4, 7, 8, 10. */
int  crt_renderer_set_kernel_variant(crt_renderer* r, int variant);
/* Work order of variants 7 and 8 (4-wide scenes).  Cost probe: before the render, variant 4 traces probe_spp samples
 * per pixel over the same RNG state without writing anything, and the per-pixel work estimates order the work
 * most-expensive-first (variant 7: pixels handed to lanes from a global queue; variant 8: 8x8 tiles, one wave per
 * workgroup).  Renders with fewer than min_spp samples per pixel skip the probe.  flags bits 16-19: variant 8's tile
 * key (0 = slowest pixel, 1 = slowest + mean pixel, 2 = 0 raised to 3/4 of the neighbours'; the renderer starts with
 * 2, the measured best); bits 20-23: variant 8's probe stride (1 = every pixel, 2 or 4 = every 2nd / 4th pixel in x and
 * y, 1/4 or 1/16 of the probe's work; 0 = automatic: 2 below 1000 spp, else 1); other bits are ignored.
 * Default -1 (automatic: 4 probe samples for renders of >= 1000 spp, else 2), 64, 2 << 16; probe_spp 0 disables the
 * probe.  Results never depend on the order. */
int  crt_renderer_set_schedule(crt_renderer* r, int probe_spp, int min_spp, int flags);
/* Variants 2-4, 7, 8: number of parked lanes (1..64) that triggers a shading/regeneration pass; default 24 for
 * variants 2/3 and 44 for the 4-wide variants (setting it sets both). */
int  crt_renderer_set_regen_threshold(crt_renderer* r, int lanes);
/* Variant 8 with the cost probe: the first `tiles` tiles of the cost order (the most expensive; -1 = automatic, 4 per
 * CU, the default) trigger their shading/regeneration passes at `lanes` parked lanes (default 16) instead of the
 * regeneration threshold.  A frame with few tiles per wave slot ends with its most expensive tile, whose pixels' sample
 * chains are sequential; waiting less for the wave's other lanes shortens that chain.  Results never depend on it. */
int  crt_renderer_set_critical_tiles(crt_renderer* r, int tiles, int lanes);
/* 4-wide variants (4, 7, 8): a new ray's first `levels` node steps -- the root's, then the one of the internal child it
 * continues to -- run in the regeneration pass from a copy of those nodes in LDS instead of in traversal steps that
 * load them through L1/L2 (-1 = the compiled default, 1; at most the compiled CRT_TOP_LEVELS).  The box tests, their
 * order and the stack entries are the traversal's own, so results never depend on it (a ray whose step hits a leaf
 * child takes that node through the regular step). */
int  crt_renderer_set_top_levels(crt_renderer* r, int levels);
/* Variant 8's leaf-pair carry, a round-4 experiment that was measured and removed (DESIGN.md §8,
 * profiles/r04c/leaf_carry.patch).  Kept for ABI stability: returns CRT_ERR_UNSUPPORTED. */
int  crt_renderer_set_leaf_carry(crt_renderer* r, int lanes, int max_pairs);
/* Variant 7 without the cost probe (the interactive loop's 1-spp frames): 1 = dispatch its 8x8 tiles most expensive
 * first by the rays per pixel the previous variant-7 render of this renderer counted (consecutive frames share the cost
 * map; the first frame, and any after this call, use row order); 0 = row order (default for the renderer; the
 * CRT::Raytracer loop turns it on).  Results never depend on it. */
int  crt_renderer_set_temporal_order(crt_renderer* r, int on);
/* Variant 7 (frames below 64 spp): once its pixel queue is empty, a wave only drains, and its last paths' passes run
 * at `lanes` parked lanes (1..64) instead of the regeneration threshold, so they wait less for each other; 0 = the
 * regeneration threshold (the default).  Results never depend on it. */
int  crt_renderer_set_drain_threshold(crt_renderer* r, int lanes);
/* Variants 4 and 8: once fewer than the regeneration threshold of a wave's lanes still have samples, a shading pass
 * runs when `sixty_fourths`/64 of those live lanes are parked (1..64; 64 = only when all of them are; default 48), so
 * the wave's last pixels wait less for each other's paths.  Results never depend on it. */
int  crt_renderer_set_wave_drain(crt_renderer* r, int sixty_fourths);
/* Variant 8 with the cost probe: 1 = the blocks that share an XCD (block index mod 8, MI355X's round-robin dispatch)
 * render one screen strip of equal probe cost, most expensive tile first, so each XCD's L2 holds its strip's geometry;
 * 0 = one global cost order (default).  Ignored with pixel sharding.  Results never depend on it. */
int  crt_renderer_set_xcd_regions(crt_renderer* r, int on);
/* Pixel sharding, the bit-exact multi-GPU mode: renders of this renderer draw only shard `shard` of
 * `shards` -- the 8x8 tiles whose row-order index t has t % shards == shard, dispatched most expensive first when the
 * cost probe runs (row order without it) -- with all samples, and leave every other pixel of the linear framebuffer
 * at 0.  Summing the shards' framebuffers (the same reduce as spp
 * sharding, every rank with subsequence base 0) gives the unsharded frame bit for bit.  4-wide rebuilt scenes only
 * (variant 8); no CRT_RENDER_ACCUMULATE.  (0, 1) = unsharded, the default. */
int  crt_renderer_set_pixel_shard(crt_renderer* r, int shard, int shards);
/* Variant 4: per-lane traversal-stack entries kept in LDS (1..16, default 16); deeper entries spill to a
 * per-pixel region in HBM.  Results do not depend on it (tests force the HBM path with 1). */
int  crt_renderer_set_stack_lds(crt_renderer* r, int entries);
/* Register-allocation occupancy target in waves per SIMD (1 = compiler default, 4-8; 0 = auto, the default: 7 for
 * variant 8 when the frame has at least 4 of its 8x8 tiles per wave slot; below that, 4 when the cost probe finds the
 * frame chain-bound (its largest tile work over the mean work per occupancy-6 wave slot above 1.6; the host then waits
 * for the probe and the tile sort before launching the main kernel) and 6 otherwise; 6 for the other 4-wide launches
 * and for variants 3 and 10, 5 for variants 0-2).  Variant 8 at 4 loads each lane's next node rows during the leaf
 * round (crt_render_kernel<false, 8, 4>).  The 4-wide kernels keep 16 traversal-stack entries per lane in LDS at 4-5
 * waves, 12 at 6 and 8 at 7+ (LDS is allocated in 1-KiB steps per workgroup). */
int  crt_renderer_set_occupancy_target(crt_renderer* r, int waves_per_simd);
/* Trace `spp` samples per pixel continuing each pixel's RNG stream; the per-pixel
 * linear sum (pixel_color, CUDAKernels.h:157-162) is kept in an fp32 W*H*3 buffer. */
int  crt_renderer_render(crt_renderer* r, const crt_scene* scene, int spp, int max_bounces, unsigned flags, void* stream);
/* RGBA8 = writeColor(scale * sum) (CRTUtility.cuh:14-32); row 0 is the bottom row. */
int  crt_renderer_resolve(crt_renderer* r, float scale, void* stream);
/* The reference's CUDARenderer::render: fresh sum, camera spp, 20 bounces, resolve, synchronize. */
int  crt_renderer_render_frame(crt_renderer* r, const crt_scene* scene, void* stream);
int  crt_renderer_synchronize(crt_renderer* r, void* stream);
int  crt_renderer_read_linear(crt_renderer* r, float* host_out);        /* W*H*3 floats */
int  crt_renderer_read_rgba8(crt_renderer* r, uint8_t* host_out);        /* W*H*4 bytes */
int  crt_renderer_read_rng(crt_renderer* r, uint32_t* host_out);         /* W*H*6 words: v[5], d */
int  crt_renderer_write_linear(crt_renderer* r, const float* host_in);  /* e.g. after a host-side reduce */
int  crt_renderer_get_counters(crt_renderer* r, crt_work_counters* out);/* of the last render call */
/* Scheduling diagnostics of the last CRT_RENDER_COUNT_WORK render (kernel variant 1), read by
 * crt_renderer_get_counters: [0] lane-slots of traversal steps (compare box_tests), [1] lane-slots
 * of cooperative leaf rounds (compare tri_tests), [2] wave-level trace calls. */
int  crt_renderer_get_schedule_stats(crt_renderer* r, unsigned long long* out3);
/* Section profile of the last counting render (variant 4), summed over waves, shader-clock cycles:
 * {shading/regeneration passes, traversal steps (box tests + stack), leaf rounds, passes, waves,
 *  shade() inside the passes, next_ray() inside the passes}. */
int  crt_renderer_get_section_profile(crt_renderer* r, unsigned long long* out7);
/* The same plus word 7: ray_spheres() inside the passes (part of word 5); copies min(n, 8) words. */
int  crt_renderer_get_section_profile_ex(crt_renderer* r, unsigned long long* out, int n);
float* crt_renderer_linear_device_ptr(crt_renderer* r);   /* for RCCL reduce of the framebuffer */
/* Bind the linear-sum framebuffer to caller-owned device memory of W*H*3 floats on the renderer's
 * device (e.g. a tensor the caller all-reduces with RCCL); NULL re-binds the internal buffer. */
int crt_renderer_attach_linear(crt_renderer* r, float* device_ptr);
uint8_t* crt_renderer_rgba_device_ptr(crt_renderer* r);
uint32_t* crt_renderer_rng_device_ptr(crt_renderer* r);
/* Milliseconds of the last render kernel launch(es), measured with HIP events on the launch stream. */
float crt_renderer_last_kernel_ms(crt_renderer* r);
/* The occupancy choice of the last variant-8 render: out[0] = rho, the probe's largest tile work over the mean work per
 * occupancy-6 wave slot (0 when the choice did not use the probe), out[1] = the occupancy launched (waves per SIMD; 0
 * for other variants), out[2] = the largest tile work and out[3] = the mean tile work (probe cost units).  An
 * extension of this port (the reference has one kernel shape), like crt_renderer_last_timings. */
int crt_renderer_last_schedule(crt_renderer* r, float out[4]);
/* HIP-event times of the last render, in ms: out[0] = the whole render (== crt_renderer_last_kernel_ms), out[1] = what
 * runs before the main render kernel (variant 8 / 7: the cost probe and the tile sort; 0 otherwise), out[2] = the main
 * render kernel alone. */
int crt_renderer_last_timings(crt_renderer* r, float out[3]);
/* The same three times for an earlier render: back = 0 is the last render, 1 the one before, up to
 * CRT_TIMING_RING - 1.  A caller that enqueues K frames without synchronising reads every frame's main-kernel time
 * afterwards (bench.py averages them for the roofline).  CRT_ERR_INVALID_ARGUMENT when fewer renders exist. */
#define CRT_TIMING_RING 32
int crt_renderer_timing_history(crt_renderer* r, int back, float out[3]);
/* Template instantiation of the last render-kernel launch as rocprofv3 names it, e.g.
 * "crt_render_kernel<false, 4, 6>" (empty before the first launch and for variant 5). */
const char* crt_renderer_last_kernel_name(const crt_renderer* r);

/* ---- GPU-parallel mesh BVH build (replaces Mesh::buildBVHMesh <<<1,1>>>, Mesh.cuh:121-264, and the Mesh ctor
 * box, Mesh.cuh:39-47; launched by initMesh, CUDAKernels.h:28-33) ----
 * Same node array (reference allocation order, crt_bvh_node_desc as the host builder emits it) and the same
 * in-place permutation of indices / face_materials (swap_triplet, Core.cuh:25-39) as the reference's single-thread
 * builder, computed level-parallel on `device` (see csrc/crt_bvh_build.hip).  positions: vertex_count slots (xyz);
 * indices: index_count local indices (multiple of 3), permuted in place; nodes: capacity 2*(index_count/3) - 1;
 * mesh_box: min xyz, max xyz.  build_ms (optional): device time from the first upload to the last kernel.
 * Returns CRT_ERR_UNSUPPORTED (nothing written) for meshes where the reference's node cap decides the tree (a split
 * with an empty side) or index_count % 3 != 0: the caller uses the sequential host builder then.  Box bounds may
 * differ from a sequential build in the sign of a zero only. */
int crt_build_mesh_bvh(int device, const float* positions, uint32_t vertex_count, uint32_t* indices,
                       int32_t* face_materials, uint32_t index_count, crt_bvh_node_desc* nodes, int32_t* node_count,
                       float mesh_box[6], float* build_ms);

/* ---- self-test of the arithmetic the kernel depends on (IEEE f32/f64 div/sqrt) ---- */
/* For n inputs a[i], b[i] (f32) computes on the device: a/b, sqrtf(|a|), 1/a, (double)sqrt((double)|a|)
 * into out[4*i..4*i+3] (the last one converted to float bits as a double->float cast). */
int crt_selftest_math(const float* a, const float* b, int n, float* out, double* out_f64);
/* Exhaustive reciprocal self-test: counts floats x with bit patterns in [lo_bits, hi_bits) (and -x) for which
 * the kernel's fast reciprocal (v_rcp_f32 + FMA Newton step) differs from IEEE 1.f/x; first_bad = lowest such. */
int crt_selftest_rcp(uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches, uint32_t* first_bad);
/* Exhaustive square-root self-test: counts floats x with bit patterns in [lo_bits, hi_bits) for which the kernels'
 * fast square root (v_rsq_f32 + one FMA correction step, crt_device.h::sqrt_rsq) differs from the correctly rounded
 * sqrtf; first_bad = lowest such. */
int crt_selftest_sqrt(uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches, uint32_t* first_bad);
/* Exhaustive check of next_ray's image-coordinate division for one frame dimension (width or height): counts the
 * floats a in [2^-33, dim] (every value x + U can take) for which uv_div(a, dim, RN(1/dim)) differs from IEEE a / dim.
 * crt_renderer_create runs the same check and uses uv_div only when both dimensions have none. */
int crt_selftest_uv_div(int dim, unsigned long long* mismatches);
/* Wave64 scan self-test: for n_waves x 64 ints, out[3*i..] = DPP inclusive sum, ds_bpermute inclusive sum,
 * DPP inclusive max (per wave of 64 consecutive entries). */
int crt_selftest_scan(const int* in, int n_waves, int* out);
/* Known-answer self-test of the render path's primitive functions on the device (tests/golden/primitives.json).
 * kind 0: Möller–Trumbore (Mesh.cuh:266-308), in 17 floats per record (o3 d3 v0 v1 v2 tmin tmax; tmin is 0.001 in
 *         the render path), out t or -1;
 * kind 1: AABB::hit (AABB.cuh:123-146) against [0.001, inf), in 14 floats (o3 d3 lo3 hi3 tmin tmax), out 1 / 0;
 * kind 2: Sphere::hit (Sphere.cuh:27-47), in 12 floats (o3 d3 center3 radius tmin tmax), out t or -1;
 * kind 3: Camera::getRay (Camera.cuh:32-44), in 2 ints per pixel (x, y) of a width x height image, rng 6 words per
 *         pixel (continued in place), out o3 d3;
 * kind 4: the per-ray spheres' skip test (a root provably beyond the trace's closest hit), in 12 floats (o3 d3
 *         center3 radius closest unused), out 1 = skipped / 0 = tested exactly. */
int crt_selftest_geometry(int kind, const float* in, int n, const crt_camera_desc* cam, int width, int height,
                          uint32_t* rng, float* out);
/* XORWOW device self-test: init(seed, subseq[i]) then n_draw uniforms per entry. */
int crt_selftest_rng(unsigned long long seed, const unsigned long long* subseq, int n, int n_draw,
                     uint32_t* state_out /* n*6 */, float* uniforms_out /* n*n_draw */);

#ifdef __cplusplus
}
#endif
#endif /* CRT_HIP_H */
