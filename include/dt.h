/*
 * dt.h — C-ABI boundary of the MI355X-native distraytracer render loop.
 *
 * The reference has no FFI: its render loop is the C++ function
 *     void renderImage(const string& filename, const int frame,
 *                      const function<void(float)> sceneBuilder)
 *         (/root/reference/render_final_project.cpp:965)
 * reading ~60 mutable globals (render_final_project.cpp:48-137, re-declared
 * extern in helpers.h:32-84 and scene.h:17-101), plus the sky-only
 *     void renderImageCloud(const string& filename, const float frame)
 *         (render_final_project.cpp:1224).
 * This header is the drop-in replacement for that boundary: plain C structs,
 * plain pointers, integer status codes, no exceptions and no exit() across it.
 *
 *   reference                                   this ABI
 *   ------------------------------------------  -----------------------------------
 *   globals render_final_project.cpp:48-137     dt_globals (1:1 field mapping)
 *   vector<shared_ptr<GeoPrimitive>> shapes     dt_scene_desc.shapes (dt_shape_desc)
 *   vector<shared_ptr<LightPrimitive>> lights   dt_scene_desc.lights (dt_light_desc)
 *   texture_frames / texture_dims (helpers.h)   dt_scene_desc.textures
 *   generateBVH (helpers.h:381) at renderImage  dt_scene_create (same topology)
 *   renderImage pixel loop (…cpp:1031-1218)     dt_render
 *   renderImageCloud (…cpp:1224-1279)           dt_render_sky
 *   printf+throw / exit         status codes + dt_stats counters
 *   scene.h builders (buildFinal, …)            dt_build_scene (host input generation)
 *
 * Output layout is the reference's ppmOut (render_final_project.cpp:986,1215-1217):
 * float[3*W*H], index 3*((H-1-y)*W + x) + c, value clamp(c)*255.0f.
 */
#ifndef DT_H
#define DT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: dt_tiles ownership by hashed tile groups (dtd::tile_of) with equal-size slabs,
 *    dt_scene_prepare / dt_scene_upload / dt_accel_info_build, RectPrismWithCylinder
 *    (DT_SHAPE_RECTPRISM_CYL with the dt_scene_desc.holes array) */
/* 3: dt_stats.donations / donate_overflow (DFS work sharing inside a wave, DT_DONATE) */
/* 4: dt_scene_set_kernel (the trace-kernel choice per scene, not through the environment) */
/* 5: dt_accel_info.features */
/* 6: dt_trace_build (the trace-kernel build a render launches, and the features it covers) */
/* 7: dt_render_repeat_async; dt_accel_info.sg_sub_blocks / sg_sub_nodes / sg_sub_hash */
/* 8: dt_render_repeat_async removed (a measurement stand-in with no product caller) */
#define DT_ABI_VERSION 8

/* ---- status codes ------------------------------------------------------- */
#define DT_OK              0
#define DT_E_INVALID      -1   /* bad argument / descriptor */
#define DT_E_NO_DEVICE    -2   /* no HIP device or HIP runtime error */
#define DT_E_OOM          -3
#define DT_E_UNSUPPORTED  -4   /* shape/light type the device path does not implement */
#define DT_E_IO           -5   /* builder data file missing */
#define DT_E_LIMIT        -6   /* recursion stack / scene size above compiled limit */

/* ---- shapes (geometry.h:28-256) ----------------------------------------- */
enum dt_shape_type {
  DT_SHAPE_SPHERE           = 1, /* Sphere            geometry.cpp:83-210   */
  DT_SHAPE_CYLINDER         = 2, /* Cylinder          geometry.cpp:212-432  */
  DT_SHAPE_TRIANGLE         = 3, /* Triangle          geometry.cpp:434-602  */
  DT_SHAPE_RECTANGLE        = 4, /* Rectangle         geometry.cpp:604-782  */
  DT_SHAPE_RECTPRISM_V2     = 5, /* RectPrismV2       geometry.cpp:784-948  */
  DT_SHAPE_CHECKERBOARD     = 6, /* Checkerboard      geometry.cpp:2248-2341 */
  DT_SHAPE_CHECKERBOARD_HOLE= 7, /* CheckerboardWithHole geometry.cpp:2344-2561 */
  DT_SHAPE_CHECKER_CYLINDER = 8, /* CheckerCylinder   geometry.cpp:2563-2630 */
  DT_SHAPE_RECTPRISM_CYL    = 9  /* RectPrismWithCylinder geometry.cpp:1467-1821 (axis-aligned
                                    box of the 8 vertices with cylinder holes; holes[] below) */
};

/* GeoPrimitive::model (render_final_project.cpp:894-948) */
enum dt_model {
  DT_MODEL_PHONG         = 0,  /* any other string, e.g. "lambert": Lambert + Phong(phong) */
  DT_MODEL_OREN_NAYAR    = 1,  /* "oren-nayar"    */
  DT_MODEL_COOK_TORRANCE = 2,  /* "cook-torrance" */
  DT_MODEL_RAW           = 3   /* "raw"           */
};

/* reflect_params.material; refl_materials = {glass, steel, aluminum, water,
 * linoleum} (render_final_project.cpp:64) */
enum dt_material {
  DT_MAT_NONE = 0, DT_MAT_GLASS = 1, DT_MAT_STEEL = 2, DT_MAT_ALUMINUM = 3,
  DT_MAT_WATER = 4, DT_MAT_LINOLEUM = 5, DT_MAT_OTHER = 6
};

/* GeoPrimitive::name values with behaviour attached to them */
enum dt_emit {
  DT_EMIT_NONE   = 0,
  DT_EMIT_SPHERE = 1,  /* name "spherelight"    (render_final_project.cpp:777) */
  DT_EMIT_RECT   = 2   /* name "rectanglelight" (render_final_project.cpp:783) */
};

/* flag bits */
#define DT_F_LIGHT       (1u << 0)  /* GeoPrimitive::light                 */
#define DT_F_MOTION      (1u << 1)  /* GeoPrimitive::motion                */
#define DT_F_TEXTURE     (1u << 2)  /* GeoPrimitive::texture               */
#define DT_F_GLOSSY      (1u << 3)  /* reflect_params.glossy               */
#define DT_F_NAMED_RECT  (1u << 4)  /* name == "rectangle" (motion-blur shift, cpp:1113) */
#define DT_F_MESH        (1u << 5)  /* Triangle::mesh                      */
#define DT_F_UV_VERTS    (1u << 6)  /* Triangle::uv_verts                  */

typedef struct dt_shape_desc {
  int32_t  type;        /* dt_shape_type */
  int32_t  model;       /* dt_model      */
  int32_t  material;    /* dt_material   */
  int32_t  emit;        /* dt_emit       */
  uint32_t flags;       /* DT_F_*        */
  int32_t  tex_frame;   /* index into dt_scene_desc.textures, -1 none */
  float    roughness;   /* reflect_params.roughness */
  float    radius;      /* Sphere / Cylinder radius */
  float    S;           /* checker square side      */
  float    borderwidth; /* checker border width     */
  float    length;      /* Rectangle::length = |B-A| (float member) */
  float    width;       /* Rectangle::width  = |D-A| (float member) */
  double   refr[2];     /* reflect_params.refr (VEC2) */
  double   color[3];    /* GeoPrimitive::color       */
  double   color1[3];   /* Checkerboard colors       */
  double   color2[3];
  double   bordercolor[3];
  double   center[3];   /* GeoPrimitive::center (BVH centroid, emissive falloff) */
  /* geometry, by type:
   *   SPHERE            v[0] = center
   *   CYLINDER / CHECKER_CYLINDER  v[0] = c1, v[1] = c2
   *   TRIANGLE          v[0..2] = A,B,C
   *   RECTANGLE / CHECKERBOARD     v[0..3] = A,B,C,D
   *   RECTPRISM_V2      v[0..7] = A..H
   *   CHECKERBOARD_HOLE v[0..3] = A,B,C,D ; v[4..7] = hole rectangle A,B,C,D
   *   RECTPRISM_CYL     v[0..7] = A..H ; holes: dt_scene_desc.holes[hole_first ..
   *                     hole_first + n_holes) (RectPrismWithCylinder::holes, geometry.h:196) */
  double   v[8][3];
  double   mesh_normal[3];
  double   uv[3][2];    /* Triangle uvA, uvB, uvC */
  int32_t  hole_first;  /* RECTPRISM_CYL: first entry in dt_scene_desc.holes */
  int32_t  n_holes;     /* RECTPRISM_CYL: number of holes (0 for every other type) */
} dt_shape_desc;

/* ---- lights (geometry.h:279-307, geometry.cpp:2745-2849) ---------------- */
enum dt_light_type {
  DT_LIGHT_POINT  = 1,  /* pointLight::sampleRay = center - p          */
  DT_LIGHT_SPHERE = 2,  /* sphereLight::sampleRay = sampled point (Q11) */
  DT_LIGHT_RECT   = 3   /* rectangleLight::sampleRay = A + x(B-A) + y(D-A) - p */
};

typedef struct dt_light_desc {
  int32_t type;          /* dt_light_type */
  int32_t shape_index;   /* shapes[] entry that IS this light object (skipped by its own
                            shadow test, cpp:812-818), or -1 */
  float   radius;        /* sphere light radius */
  float   _pad;
  double  center[3];     /* LightPrimitive::center */
  double  color[3];      /* LightPrimitive::color  */
  double  baxis[3];      /* sphereLight::baxis     */
  double  A[3], B[3], D[3]; /* rectangle light sampling frame */
} dt_light_desc;

/* texture_frames[i] / texture_dims[i] (helpers.h:92-113): 8-bit RGB as decoded by
 * stb_image; the renderer uses byte/255.0 as the reference does. */
typedef struct dt_texture_desc {
  int32_t        width;
  int32_t        height;
  int32_t        channels;   /* bytes per texel (>=3), first 3 used */
  int32_t        _pad;
  const uint8_t* pixels;     /* row-major, width*height*channels */
} dt_texture_desc;

typedef struct dt_scene_desc {
  int32_t                n_shapes;
  int32_t                n_lights;
  int32_t                n_textures;
  int32_t                _pad;
  const dt_shape_desc*   shapes;
  const dt_light_desc*   lights;
  const dt_texture_desc* textures;
  /* Cylinder holes of RECTPRISM_CYL shapes (type CYLINDER records: v[0] = c1, v[1] = c2, radius,
   * color; geometry.cpp:227-240). They are not shapes of the scene: only their prism tests them. */
  int32_t                n_holes;
  int32_t                _pad2;
  const dt_shape_desc*   holes;
} dt_scene_desc;

/* ---- globals (render_final_project.cpp:48-137) -------------------------- */
typedef struct dt_globals {
  int32_t xRes, yRes;                    /* 52-53 */
  double  eye[3], lookingAt[3], up[3];   /* 56-58 */
  float   aspect, near_plane, fov;       /* 59-61 (aspect frozen at 1920/1080, Q3) */
  float   aperture, focal_length;        /* 62-63 */
  int32_t use_model, nogloss;            /* 64-65 */
  float   refr_air, refr_glass;          /* 69-70 */
  int32_t max_depth;                     /* 71 */
  float   phong;                         /* 76 */
  double  default_col[3];                /* 77 */
  float   c_isect, c_trav;               /* 81-82 */
  int32_t antialias_samples, brdf_samples, blur_samples, frame_range; /* 85-88 */
  int32_t frame_prism, frame_cloud, frame_blur, frame_start;  /* 112-115 */
  int32_t frame_move1, frame_move2, frame_sculp, total;       /* 116-119 */
  float   far_dist, move_per_frame, tot_move, accel_t;        /* 120-123 */
  double  cap_center[3];                                       /* 124 */
  double  sundir[3];                     /* 127 */
  int32_t perlin_cloud;                  /* 128 */
  float   saturation, clouddist, cloudhoff; /* 129-131 */
  double  sun_outer[3], sun_inner[3], sun_core[3], bluesky[3], redsky[3]; /* 132-136 */
  int32_t reflect;                       /* 138 */
  uint32_t seed;                         /* counter-RNG seed (reference RNG is unseeded, F7) */
} dt_globals;

/* ---- tiles / multi-GPU partition ---------------------------------------- */
enum dt_out_layout {
  DT_OUT_IMAGE = 0,  /* full ppmOut layout float[3*xRes*yRes]; only owned pixels written */
  DT_OUT_SLAB  = 1   /* owned tiles packed in tile order: dt_slab_floats() floats */
};

typedef struct dt_tiles {
  int32_t x0, y0, x1, y1;    /* pixel window [x0,x1) x [y0,y1); x1<=0 means full width/height */
  int32_t tile_w, tile_h;    /* tile size (<=0: 32x32) */
  int32_t rank, world;       /* the window's tiles (row-major) fall into groups of `world`
                                consecutive tiles; each rank owns one tile of every group, the
                                ranks rotated by a hash of the group (dt_scene_dev.h tile_of) */
  int32_t layout;            /* dt_out_layout */
  int32_t _pad;
} dt_tiles;

/* ---- stats --------------------------------------------------------------- */
typedef struct dt_stats {
  uint64_t pixels;            /* pixels rendered                                 */
  uint64_t samples;           /* pixel-samples (W*H*spp) = metric numerator      */
  uint64_t rays;              /* rayColor invocations with depth>0 (incl. blur)  */
  uint64_t shadow_rays;       /* light samples tested for occlusion              */
  uint64_t sky_pixels;        /* pixels that needed cloudColor                   */
  uint64_t uv_out_of_range;   /* reference terminates here (cpp:870-877), we count */
  uint64_t glossy_exhausted;  /* >10 invalid glossy resamples (cpp:724-740)      */
  uint64_t spherelight_exhausted; /* geometry.cpp:2785-2789                      */
  uint64_t prism_norm_fallback;   /* RectPrismV2::getNorm off-surface (geometry.cpp:895);
                                     RectPrismWithCylinder::getNorm's throw (geometry.cpp:1819-1820) */
  uint64_t reflect_errors;    /* refl.n <= 0 (cpp:631-638)                       */
  uint64_t nan_pixels;
  uint64_t tex_fetches;       /* texel reads (algorithmic bytes) */
  uint64_t stack_overflows;   /* DFS entries dropped (device stack limit); 0 when validated */
  uint64_t box_tests;         /* lane-level BVH slab tests      (these three: diagnostic builds */
  uint64_t prim_tests;        /* lane-level primitive tests       with -DDT_WORK_COUNTERS only; */
  uint64_t wave_node_visits;  /* wave-level BVH node visits        0 otherwise)  */
  double   kernel_ms;         /* device time of the render kernels (hipEvents, same stream) */
  double   trace_kernel_ms;   /* device time of the dominant (trace) kernel alone */
  uint64_t donations;         /* pending DFS subtrees run by another lane of the wave (work sharing) */
  uint64_t donate_overflow;   /* work-sharing records dropped (per-wave pool full); 0 when validated */
} dt_stats;

/* ---- API ------------------------------------------------------------------ */
typedef struct dt_scene dt_scene;   /* opaque: device-resident scene + BVH */

int         dt_abi_version(void);
const char* dt_last_error(void);

/* fill with the reference's initial global values (render_final_project.cpp:48-137) */
void dt_globals_default(dt_globals* g);

/* Build the reference-topology BVH (helpers.h:381-472) on the host and upload the
 * scene to the current HIP device. */
int  dt_scene_create(const dt_scene_desc* desc, const dt_globals* g, dt_scene** out);
void dt_scene_destroy(dt_scene* s);
/* dt_scene_create in two halves. dt_scene_prepare does the host work (flatten, BVH, acceleration
 * structures, primary-ray lists) and touches no device memory, so it can run on a worker thread
 * while a render fills the GPU; dt_scene_upload allocates and uploads (a few ms). A render of a
 * scene that was prepared but not uploaded uploads it first. No reference counterpart: the
 * reference builds its BVH inside renderImage (render_final_project.cpp:965-1030). */
int  dt_scene_prepare(const dt_scene_desc* desc, const dt_globals* g, dt_scene** out);
int  dt_scene_upload(dt_scene* s);

/* Which trace kernel the renders of scene s launch. No reference counterpart (the reference has
 * one loop, render_final_project.cpp:1031-1218); every choice renders the same bits.
 *   DT_KERNEL_AUTO     the DT_DONATE environment variable decides (default: the product kernels)
 *   DT_KERNEL_PRODUCT  the product kernels (dt_trace_kernel / _w5 by spp)
 *   DT_KERNEL_DONATE   DFS work sharing inside the wave (dt_trace_kernel_dn) where it applies
 *                      (max_depth <= 11, brdf_samples <= 6, no RectPrismWithCylinder)
 * A caller choosing per frame (tools/animate.py) sets it on that frame's scene instead of writing
 * the process environment while another thread builds the next scene. Calls on one scene must not
 * overlap across host threads (this one included). */
#define DT_KERNEL_AUTO     0
#define DT_KERNEL_PRODUCT  1
#define DT_KERNEL_DONATE   2
int  dt_scene_set_kernel(dt_scene* s, int32_t kernel);

/* BVH export for parity tests: node i = {first child or -1, n_children, first shape,
 * n_shapes, leaf, lbound[3], ubound[3]} in the reference's push order. */
typedef struct dt_bvh_node {
  int32_t first_child, n_children, first_index, n_indices, leaf, depth;
  double  lbound[3], ubound[3];
} dt_bvh_node;
int  dt_scene_bvh(const dt_scene* s, dt_bvh_node* nodes, int32_t cap,
                  int32_t* indices, int32_t index_cap, int32_t* n_nodes, int32_t* n_indices);

/* generateBVH (helpers.h:381-472) alone, on the host, no device needed: same export format
 * as dt_scene_bvh. */
int  dt_bvh_build(const dt_scene_desc* desc, const dt_globals* g, dt_bvh_node* nodes, int32_t cap,
                  int32_t* indices, int32_t index_cap, int32_t* n_nodes, int32_t* n_indices);

/* The acceleration structures dt_scene_create would upload for (desc, g), built on the host
 * only (no device): counts and FNV-1a content hashes, for A/B checks of build options
 * (DT_SG_BLOCK, DT_SG_ORDER, ...). No reference counterpart: the reference walks its own BVH
 * (helpers.h:381-472, geometry.cpp:2657-2740) and has no shadow grid. */
typedef struct dt_accel_info {
  int32_t n_nodes, n_fnodes, n_bnodes, boxes_ordered;
  int32_t sg_lights, sg_dim[3];
  int64_t sg_cells, sg_tree_cells, sg_list_pool, sg_list_entries;
  uint64_t nodes_hash, fnodes_hash, bnodes_hash;
  uint64_t sg_hash;            /* cells + list pool in storage order */
  uint64_t sg_contents_hash;   /* each cell's list as a sorted set (order-free) */
  float bump_pad, sg_reach;
  int64_t sg_umbra_cells;      /* (light, cell) records whose every segment to the light is occluded */
  uint32_t features;           /* the scene's trace-kernel feature mask: bit t for shape type t,
                                  12 sphere lights/emitters, 13 Oren-Nayar, 14 glass, 15 rectangle
                                  lights/emitters (the build dt_render launches) */
  int32_t sg_sub_blocks;       /* shadow-grid block subtrees (DT_SG_SUBTREE=1) and their nodes */
  int64_t sg_sub_nodes;
  uint64_t sg_sub_hash;        /* FNV-1a over the block records and subtree nodes */
} dt_accel_info;
int dt_accel_info_build(const dt_scene_desc* desc, const dt_globals* g, dt_accel_info* info);

/* The trace-kernel build dt_render launches for (desc, g) at `frame` with the automatic kernel
 * choice (the DT_* environment switches apply as in dt_render), decided on the host only (no
 * device): its kernel name (NUL-terminated, truncated to name_cap), the scene's feature mask (as
 * dt_accel_info.features) and the mask the build was compiled for (dt_kernels.hip DT_FEATURES).
 * dt_render refuses (DT_E_INVALID) a scene with a feature outside its build's mask rather than
 * launching code that has that case compiled out. No reference counterpart: the reference has one
 * CPU render loop (render_final_project.cpp:965-1222). */
int dt_trace_build(const dt_scene_desc* desc, const dt_globals* g, int32_t frame, char* name, int32_t name_cap,
                   uint32_t* scene_features, uint32_t* build_features);

/* number of floats a DT_OUT_SLAB output needs for (g, tiles) */
int64_t dt_slab_floats(const dt_globals* g, const dt_tiles* tiles);
int64_t dt_slab_floats_max(const dt_globals* g, const dt_tiles* tiles); /* max over ranks */

/* renderImage's pixel loop (render_final_project.cpp:1031-1218) for `frame`.
 * out: host pointer (out_on_device=0) or device pointer (1). stream: hipStream_t or NULL.
 * Synchronous unless dt_render_async is used. */
int dt_render(const dt_scene* s, const dt_globals* g, int32_t frame, const dt_tiles* tiles,
              float* out, int32_t out_on_device, void* stream, dt_stats* stats);
/* enqueue only (device output, no host sync, stats device-side until dt_collect_stats).
 * A scene's launches must be ordered: keep one scene object per stream (two frames in flight take
 * two scene objects, as bench.py does). A scene keeps two launch records and two counter blocks
 * on the device and alternates between them; each launch clears the other block, and a record is
 * uploaded only when its bytes change, so repeated renders of a still frame enqueue nothing but
 * their kernels. dt_collect_stats reports the scene's last launch. */
int dt_render_async(const dt_scene* s, const dt_globals* g, int32_t frame, const dt_tiles* tiles,
                    float* out_device, void* stream);
int dt_collect_stats(const dt_scene* s, void* stream, dt_stats* stats);

/* diagnostic builds (-DDT_STAMPS): per-phase cycle sums of the last render; zeros otherwise */
int dt_debug_counters(const dt_scene* s, uint64_t* out, int32_t n);
/* diagnostic builds (-DDT_ITEM_TIMES=2) with DT_ITEM_COSTS=1 in the environment: the last launch's
 * per-item durations (100 MHz clock ticks) by queue code (chunk items: pixel item * chunks + chunk),
 * min(n, items) of them into out; returns the number of items (0: none recorded; < 0: an error code) */
int64_t dt_debug_item_costs(const dt_scene* s, uint32_t* out, int64_t n);
/* numerics check: the device kernels' normalisation of n VEC3s (Eigen normalized(), dt_math.h),
 * host arrays of 3n doubles; synchronous */
int dt_debug_normalize(const double* in, double* out, int64_t n);

/* Intersection micro-benchmark (2^24 primary rays of the C3 camera). rayColor's first
 * step (render_final_project.cpp:491-538: BVH gather + closest hit) for primary rays of the globals'
 * camera (getDOFSamples + getPerspEyeRay, 195-210 / 1044-1072), as dt_render takes it. Ray r:
 * q = r / 8 -> pixel q mod (xRes*yRes) in raster order, sample r mod 8 + 8 * (q div (xRes*yRes)).
 * hit_shape[i], hit_t[i] for ray first_ray + i: the closest shape (-1: none) and its t (FLT_MAX:
 * none); host (out_on_device=0) or device (1) arrays of n_rays. Synchronous; kernel_ms (optional):
 * the kernel's HIP-event time. Scenes with a RectPrismWithCylinder: DT_E_UNSUPPORTED. It shares the
 * scene's primary-ray lists, which depend on the camera and resolution only (not on a tile split):
 * called with the globals of the scene's renders it rebuilds nothing. Its launch record, counters
 * and events are its own, but like every call on one scene it must not overlap another call on
 * that scene from another host thread. */
int dt_intersect_primary(const dt_scene* s, const dt_globals* g, int32_t frame, int64_t first_ray,
                         int64_t n_rays, int32_t* hit_shape, float* hit_t, int32_t out_on_device,
                         void* stream, float* kernel_ms);

/* renderImageCloud (render_final_project.cpp:1224-1279). Sets eye/up/lookingAt as the
 * reference does (1227-1229) on a local copy; g is not modified. */
int dt_render_sky(const dt_globals* g, float frame, const dt_tiles* tiles, float* out,
                  int32_t out_on_device, void* stream, dt_stats* stats);

/* Scatter a gathered set of per-rank slabs (rank-major, each dt_slab_floats_max floats)
 * into the full ppmOut image (host or device, same side as inputs). */
int dt_unpack_slabs(const dt_globals* g, const dt_tiles* tiles, int32_t world,
                    const float* slabs, float* image, int32_t on_device, void* stream);

/* ---- host scene builders (scene.h) ---------------------------------------- */
/* name: "final" (buildFinal scene.h:605), "spheres" (buildSceneSpheres 4399),
 * "dof" (buildSceneDOF 4422), "hw4" (buildSceneHW4 4451), "prismcyl"
 * (BuildScenePrismCylinder 3227, the `./render prismcyl` mode, cpp:1711-1723).
 * Mutates g exactly as the reference builder mutates its globals (Q23, fresh-process
 * semantics: call dt_globals_default first for a fresh frame).
 * data_dir holds textures/<name>.rgb and bones_<motion>.bin. */
int  dt_build_scene(const char* name, float frame, dt_globals* g, const char* data_dir,
                    dt_scene_desc** out);
void dt_scene_desc_free(dt_scene_desc* d);

/* skeleton.cpp/motion.cpp/displaySkeleton.cpp forward kinematics: the 30 bone-cylinder
 * endpoints buildFinal places (scene.h:637-658) for each posture id in frames[]
 * (out: n_frames * n_bones * 6 doubles, left xyz + right xyz). out == NULL only reports
 * the bone and posture counts. Used by tools/gen_bones.py to make the data table. */
int dt_mocap_bone_table(const char* asf, const char* amc, const int32_t* frames, int32_t n_frames,
                        double* out, int32_t* n_bones, int32_t* n_postures);

/* test hook: the OBJ ingest of finalBuildModels (loadObj, objHelper.h:6-85) on one file. counts =
 * {vertices, texcoords, triangles}; with capacities >= those, v gets 3 floats per vertex, vt 2 per
 * texcoord and faces 6 int32 per triangle (3 vertex + 3 texcoord indices, 0-based, -1: none).
 * Null arrays only report the counts. */
int dt_debug_load_obj(const char* path, float* v, int64_t cap_v, float* vt, int64_t cap_vt, int32_t* faces,
                      int64_t cap_faces, int64_t counts[3]);

/* writePPM (helpers.h:174-195): float -> unsigned char truncation */
int dt_write_ppm(const char* filename, int32_t xRes, int32_t yRes, const float* values);
/* the same pixels as an 8-bit RGB PNG (the output surface beside PPM) */
int dt_write_png(const char* filename, int32_t xRes, int32_t yRes, const float* values);

#ifdef __cplusplus
}
#endif
#endif /* DT_H */
