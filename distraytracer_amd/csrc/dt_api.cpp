// dt_api.cpp — the C-ABI entry points (include/dt.h) over the HIP kernels.
// No exception and no exit() crosses the boundary: every entry point returns a status
// code and leaves a message for dt_last_error().
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "host_internal.h"

using namespace dth;

extern "C" size_t dt_launch_size(void);
extern "C" size_t dt_scene_struct_offset(void);
extern "C" size_t dt_scene_struct_size(void);
extern "C" size_t dt_params_struct_offset(void);
extern "C" hipError_t dt_launch_sky(const void* dev_launch, float* out, int64_t n_threads, hipStream_t stream);
extern "C" hipError_t dt_launch_sky_miss(const void* dev_launch, float* out, int64_t n_px, hipStream_t stream);
extern "C" hipError_t dt_launch_chunk_sum(const void* dev_launch, float* out, int64_t n_px, hipStream_t stream);
extern "C" hipError_t dt_launch_unpack(const void* dev_launch, int world, int64_t slab_floats, const float* slabs,
                                       float* image, hipStream_t stream);
extern "C" hipError_t dt_launch_normalize(const double* in, double* out, int64_t n, hipStream_t stream);
// the trace-kernel builds (dt_kernels.hip DT_TRACE_KERNEL, Makefile TRACE_BUILDS)
#define DT_TRACE_BUILD(k)                                                                              \
  extern "C" hipError_t k##_launch(const void* dev_launch, float* out, int grid, hipStream_t stream); \
  extern "C" const void* k##_ptr(void);                                                                \
  extern "C" int k##_traits(void);
DT_TRACE_BUILD(dt_trace_kernel)
DT_TRACE_BUILD(dt_trace_kernel_mesh)
DT_TRACE_BUILD(dt_trace_kernel_full)
DT_TRACE_BUILD(dt_trace_kernel_tunnel)
DT_TRACE_BUILD(dt_trace_kernel_blur)
DT_TRACE_BUILD(dt_trace_kernel_sky)
DT_TRACE_BUILD(dt_trace_kernel_w5)
DT_TRACE_BUILD(dt_trace_kernel_w5_mesh)
DT_TRACE_BUILD(dt_trace_kernel_w5_full)
DT_TRACE_BUILD(dt_trace_kernel_w5_tunnel)
DT_TRACE_BUILD(dt_trace_kernel_w5_blur)
DT_TRACE_BUILD(dt_trace_kernel_w5_sky)
DT_TRACE_BUILD(dt_trace_kernel_dn)
DT_TRACE_BUILD(dt_trace_kernel_rpc)
#undef DT_TRACE_BUILD
extern "C" hipError_t dt_launch_isect(const void* dev_launch, int64_t first, int64_t n, int32_t* hit_shape, float* hit_t,
                                      int grid, hipStream_t stream);
extern "C" const void* dt_isect_kernel_ptr(void);

namespace {

thread_local std::string g_err;

// must match the device-side DScene (dt_kernels.hip)
struct HScene {
  const void* nodes;
  const void* fnodes;
  const uint32_t* sg_cells;
  const int32_t* sg_list;
  const int32_t* leaf_idx;
  const void* hdr;
  const double* geom;
  const void* mat;
  const void* lights;
  const uint8_t* tex;
  const float* cloud_z;
  unsigned long long* stats;
  unsigned long long* queue;
  const void* bnodes;       // motion-blur bump tree (host_fasttree.cpp)
  const int32_t* bparent;   // parent of every reference-tree node
  const uint32_t* pl_cells; // primary-ray candidate lists (host_primlists.cpp)
  const uint32_t* pl_list;
  uint8_t* sky_miss;
  void* dn_pool;
  uint32_t* again_list;
  unsigned int* again_n;
  const void* sub_nodes;      // shadow-grid block subtrees
  const uint32_t* sub_blocks;
  unsigned long long* clear0;   // the other parity's counters, zeroed by the launch (dt_kernels.hip)
  unsigned long long* clear1;
  int32_t n_clear0, n_clear1;
  double* chunk_cols;           // chunk items: per-pixel sample colours (dt_kernels.hip)
  uint32_t* item_cost;          // diagnostic builds: per-item durations (dt_debug_item_costs)
  void* pad_;
};

// DT_N_STAMPS (dt_scene_dev.h): diagnostic counter slots of -DDT_STAMPS builds (dt_debug_counters):
// phases, then (waves, lanes, hits) per (light, shape) shadow test
enum { ST_RAYS = 0, ST_SHADOW = 1, ST_SKY = 2, ST_UV = 3, ST_GLOSSY = 4, ST_SPHL = 5, ST_PRISM = 6,
       ST_REFL = 7, ST_NAN = 8, ST_PIXELS = 9, ST_SAMPLES = 10, ST_STACK = 11, ST_TEX = 12, ST_BOX = 13, ST_PRIM = 14, ST_WNODES = 15,
       ST_DONATE = 16, ST_DN_OVF = 17, ST_N = 18 };
// one parity's counter block: the trace launch's (counters, queue word, stamps slots, segment
// counters), the sky-item launch's (counters, queue word, list count)
constexpr size_t STATS1 = ST_N + DT_STAT_SLOT_OFF + (DT_STAT_SLOTS - 1) * DT_STAT_SLOT_STRIDE, STATS2 = ST_N + 2;

int fail(int code, const std::string& msg)
{
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(DT_E_NO_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));  \
  } while (0)

// Scene uploads go through a non-blocking stream of the calling thread: a plain hipMemcpy runs on
// the legacy null stream and waits for every kernel in flight, so a scene built on a worker
// thread while the previous frame renders (tools/animate.py) would wait for that render.
static hipStream_t upload_stream()
{
  thread_local hipStream_t s = nullptr;
  thread_local int s_dev = -1;   // streams belong to a device: a thread that switches gets a new one
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (s && s_dev != dev) s = nullptr;   // the old device's stream stays valid for its device
  if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
  s_dev = dev;
  return s;
}

template <class T>
int upload(const std::vector<T>& v, void** dptr)
{
  size_t bytes = v.size() * sizeof(T);
  if (bytes == 0) bytes = 16;
  HIPCHK(hipMalloc(dptr, bytes));
  if (v.empty()) return DT_OK;
  hipStream_t us = upload_stream();
  if (!us) {
    HIPCHK(hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return DT_OK;
  }
  HIPCHK(hipMemcpyAsync(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, us));
  HIPCHK(hipStreamSynchronize(us));
  return DT_OK;
}

int max_resident_waves(const void* kernel_fn, int block)
{
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 1024;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_fn, block, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  return per_cu * prop.multiProcessorCount;
}

}  // namespace

namespace dth {
void set_error(const std::string& e) { g_err = e; }
}  // namespace dth

struct dt_scene {
  int device = 0;
  FlatScene flat;
  void* d_nodes = nullptr;
  void* d_fnodes = nullptr;
  int n_fnodes = 0;
  void* d_bnodes = nullptr;    // bump tree for motion-blur passes (0 nodes: they walk the reference tree)
  void* d_bparent = nullptr;
  int n_bnodes = 0;
  float bump_pad = 0;          // y padding of its leaves: the largest |shift| a blur pass can draw
  bool bump_up_only = false;   // bump tree / blur-padded lists built for shifts >= 0 only
  bool no_cull = false;        // a RectPrismWithCylinder: no t-culling, no grid, no primary lists
  unsigned features = ~0u;     // the scene's feature mask (dt_scene_dev.h): which builds can render it
  int kernel = DT_KERNEL_AUTO; // dt_scene_set_kernel
  ShadowGrid sg;
  void* d_sg_cells = nullptr;
  void* d_sg_list = nullptr;
  void* d_sub_nodes = nullptr;    // shadow-grid block subtrees (ShadowGrid::sub_*)
  void* d_sub_blocks = nullptr;
  int ftree_mode = 0;
  int boxes_ordered = 0;   // lb <= ub on every axis of every node (both trees), no NaN bound
  void* d_leaf = nullptr;
  void* d_hdr = nullptr;
  void* d_geom = nullptr;
  void* d_mat = nullptr;
  void* d_lights = nullptr;
  void* d_tex = nullptr;
  void* d_zs = nullptr;
  size_t zs_cap = 0;
  // ST_N counters + queue word (+ the stamps builds' slots), twice: launches alternate between the
  // two (parity), and each zeroes the other for the next one (HScene::clear0)
  unsigned long long* d_stats = nullptr;
  int n_launch = 0;     // trace launches enqueued (the parity of the next: n_launch & 1)
  int last_parity = 0;  // the parity of the last one (dt_collect_stats)
  // the launch record's device copy, one per parity, uploaded only when its bytes changed (a still
  // frame rendered again uploads nothing: no copy kernel between its launches)
  void* d_launch = nullptr;
  std::vector<uint8_t> rec_last[2], rec2_last[2];
  std::vector<float> zs_last;   // the z table in d_zs
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_copy = nullptr;   // staging buffers may be rewritten once this has fired
  uint8_t* h_launch = nullptr;    // pinned staging for the launch record
  float* h_zs = nullptr;          // pinned staging for the cloud z sequence
  bool copy_pending = false;
  bool timed = false;
  bool launched = false;   // a trace launch was enqueued (may still read device-side lists)
  bool uploaded = false;   // dt_scene_upload ran (dt_scene_prepare builds on the host only)
  bool pl_dirty = false;   // the host primary lists changed since their last upload
  Accel acc;               // host acceleration structures until the upload
  // primary-ray candidate lists, rebuilt when the camera / resolution changes (host_primlists.cpp)
  std::vector<dtd::DNodeDev> fnodes_host, bnodes_host;
  std::vector<std::vector<P3>> fhull, bhull;   // leaf hull points per fast / bump tree node (host_hull.cpp)
  bool pl_bump = false;                        // lists for the blur passes follow the pass-0 lists
  std::vector<double> pl_key;
  uint8_t* d_sky_miss = nullptr;   // 1-spp launches: missed-pixel flags (dt_sky_miss_kernel clears them)
  int64_t sky_miss_cap = 0;
  // sky items (dt_kernels.hip DT_SKY_AGAIN): the list a still build leaves to its *_sky build, that
  // launch's record (pinned staging h_launch2, guarded by ev_copy like h_launch) and its counters
  uint32_t* d_again = nullptr;
  int64_t again_cap = 0;
  void* d_launch2 = nullptr;
  uint8_t* h_launch2 = nullptr;
  unsigned long long* d_stats2 = nullptr;   // ST_N counters + queue word + list count, twice (parity)
  bool again_used = false;                  // the last render ran the second launch
  void* d_dn_pool = nullptr;       // dt_trace_kernel_dn: DT_DN_POOL_REC work-sharing records per wave
  int64_t dn_pool_waves = 0;
  double* d_chunk_cols = nullptr;   // chunk items: spp sample colours per pixel item
  int64_t chunk_cols_cap = 0;
  uint32_t* d_item_cost = nullptr;  // DT_ITEM_COSTS=1 (diagnostic builds): per-item durations
  int64_t item_cost_cap = 0, item_cost_n = 0;
  PrimLists pl;
  bool pl_ok = false;
  void* d_pl_cells = nullptr;
  void* d_pl_list = nullptr;
  dtd::DParams last;
};

extern "C" {

int dt_abi_version(void) { return DT_ABI_VERSION; }

int dt_scene_set_kernel(dt_scene* s, int32_t kernel)
{
  if (!s) return fail(DT_E_INVALID, "null scene");
  if (kernel != DT_KERNEL_AUTO && kernel != DT_KERNEL_PRODUCT && kernel != DT_KERNEL_DONATE)
    return fail(DT_E_INVALID, "dt_scene_set_kernel: unknown kernel choice");
  s->kernel = kernel;
  return DT_OK;
}
const char* dt_last_error(void) { return g_err.c_str(); }

void dt_globals_default(dt_globals* g)
{
  // render_final_project.cpp:48-138
  memset(g, 0, sizeof(*g));
  g->xRes = 1920;
  g->yRes = 1080;
  g->eye[0] = -6; g->eye[1] = 0.5; g->eye[2] = 1;
  g->lookingAt[0] = 0.5; g->lookingAt[1] = 0.5; g->lookingAt[2] = 1;
  g->up[0] = 0; g->up[1] = 1; g->up[2] = 0;
  g->aspect = (float)1920 / (float)1080;
  g->near_plane = 1;
  g->fov = 45.0f;
  g->aperture = 0.2f;
  g->focal_length = 10;
  g->use_model = 1;
  g->nogloss = 0;
  g->refr_air = 1;
  g->refr_glass = 1.5f;
  g->max_depth = 10;
  g->phong = 10;
  g->c_isect = 1;
  g->c_trav = 0.33f;
  g->antialias_samples = 10;
  g->brdf_samples = 2;
  g->blur_samples = 2;
  g->frame_range = 1;
  g->frame_prism = 960;
  g->frame_cloud = 1952;
  g->frame_blur = 1600;
  g->frame_start = 120;
  g->frame_move1 = 480;
  g->frame_move2 = 960;
  g->frame_sculp = 600;
  g->total = 2400;
  g->far_dist = 200;
  g->move_per_frame = (float)(0.1 / 8);
  g->tot_move = 0;
  g->accel_t = (float)(80 / pow(360, 3));
  g->sundir[0] = 0; g->sundir[1] = 0.1; g->sundir[2] = -1;
  g->perlin_cloud = 0;
  g->saturation = 0.2f;
  g->clouddist = 10;
  g->cloudhoff = 0.2f;
  g->sun_outer[0] = 0.9; g->sun_outer[1] = 0.3; g->sun_outer[2] = 0.9;
  g->sun_inner[0] = 1.0; g->sun_inner[1] = 0.7; g->sun_inner[2] = 0.7;
  g->sun_core[0] = 1; g->sun_core[1] = 1; g->sun_core[2] = 1;
  g->bluesky[0] = 0.3; g->bluesky[1] = 0.55; g->bluesky[2] = 0.8;
  g->redsky[0] = 0.8; g->redsky[1] = 0.8; g->redsky[2] = 0.6;
  g->reflect = 1;
  g->seed = 0;
}

static int prepare_render(const dt_scene* sc, const dt_globals* g, int32_t frame, const dt_tiles* tiles,
                          dtd::DParams& P, std::vector<float>& zs);
static int update_primary_lists(dt_scene* sc, dtd::DParams& P, bool upload_now);
static int upload_primary_lists(dt_scene* sc);

static int scene_upload(dt_scene* s);

// Host half of dt_scene_create: flatten, BVH, acceleration structures, hulls and the primary-ray
// lists for the globals' camera. No device work, so it can run on a worker thread beside a render
// that fills the GPU (the persistent trace kernel holds every CU, so even a copy's blit kernel
// would wait for it: tools/animate.py builds frame n+1 this way and uploads it between frames).
static unsigned scene_features(const dt_scene_desc& d);

int dt_scene_prepare(const dt_scene_desc* desc, const dt_globals* g, dt_scene** out)
{
  if (!desc || !g || !out) return fail(DT_E_INVALID, "null argument");
  *out = nullptr;
  dt_scene* s = new dt_scene();
  std::string err;
  // DT_TIMING=1: host stage times of the scene build on stderr
  const bool timing = getenv("DT_TIMING") != nullptr;
  auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double t_stage = now();
  auto stage = [&](const char* name) {
    if (!timing) return;
    const double t = now();
    fprintf(stderr, "dt_scene_create %-12s %8.2f ms\n", name, t - t_stage);
    t_stage = t;
  };
  int rc = flatten_scene(*desc, *g, s->flat, err);
  stage("flatten+bvh");
  if (rc) {
    delete s;
    return fail(rc, err);
  }
  s->features = scene_features(*desc);
  if (hipGetDevice(&s->device) != hipSuccess) {
    delete s;
    return fail(DT_E_NO_DEVICE, "no HIP device");
  }
  const FlatScene& f = s->flat;
  Accel& acc = s->acc;
  build_accel(f, *g, acc, stage);
  s->n_fnodes = acc.n_fnodes;
  s->n_bnodes = acc.n_bnodes;
  s->bump_pad = acc.bump_pad;
  s->bump_up_only = acc.bump_up_only;
  s->no_cull = acc.no_cull;
  s->ftree_mode = acc.ftree_mode;
  s->boxes_ordered = acc.boxes_ordered;
  s->sg = std::move(acc.sg);
  s->fnodes_host = acc.fnodes;
  s->bnodes_host = acc.bnodes;
  {   // leaf hulls for the primary lists' hull culling (host_primlists.cpp); the bump tree's with
      // the moving rectangles' shifted corners
    s->fhull.assign(s->fnodes_host.size(), {});
    s->bhull.assign(s->bnodes_host.size(), {});
    for (int i = 0; i < s->n_fnodes; ++i)
      if (s->fnodes_host[i].meta & dtd::DN_LEAF) leaf_hull_points(f, s->fnodes_host[i], -1, 0.0, s->fhull[i]);
    for (int i = 0; i < s->n_bnodes; ++i)
      if (s->bnodes_host[i].meta & dtd::DN_LEAF) leaf_hull_points(f, s->bnodes_host[i], -1, (double)s->bump_pad, s->bhull[i], acc.bump_up_only);
  }
  {   // the primary-ray lists for the globals' camera and resolution; a render with another
      // camera rebuilds them
    dtd::DParams P;
    std::vector<float> zs;
    dt_tiles whole;
    memset(&whole, 0, sizeof(whole));
    whole.world = 1;
    if (prepare_render(s, g, 0, &whole, P, zs) == DT_OK) (void)update_primary_lists(s, P, false);
    stage("primary lists");
  }
  *out = s;
  return DT_OK;
}

// every device buffer, event and pinned staging buffer of a scene, released and reset to null
// (dt_scene_destroy, and a failed upload so that a retry starts from nothing)
static void release_device(dt_scene* s)
{
  void** bufs[] = {&s->d_pl_cells, &s->d_pl_list, &s->d_nodes, &s->d_fnodes, &s->d_bnodes, &s->d_bparent,
                   &s->d_sg_cells, &s->d_sg_list, &s->d_sub_nodes, &s->d_sub_blocks, &s->d_leaf, &s->d_hdr, &s->d_geom, &s->d_mat, &s->d_lights,
                   &s->d_tex, &s->d_zs, (void**)&s->d_stats, &s->d_launch, (void**)&s->d_sky_miss, &s->d_dn_pool,
                   (void**)&s->d_again, &s->d_launch2, (void**)&s->d_stats2, (void**)&s->d_chunk_cols,
                   (void**)&s->d_item_cost};
  for (void** b : bufs) {
    if (*b) (void)hipFree(*b);
    *b = nullptr;
  }
  for (hipEvent_t* e : {&s->ev0, &s->ev1, &s->ev_copy}) {
    if (*e) (void)hipEventDestroy(*e);
    *e = nullptr;
  }
  if (s->h_launch) (void)hipHostFree(s->h_launch);
  if (s->h_launch2) (void)hipHostFree(s->h_launch2);
  if (s->h_zs) (void)hipHostFree(s->h_zs);
  s->h_launch = nullptr;
  s->h_launch2 = nullptr;
  s->again_cap = 0;
  s->again_used = false;
  s->h_zs = nullptr;
  s->zs_cap = 0;
  s->sky_miss_cap = 0;
  s->dn_pool_waves = 0;
  s->chunk_cols_cap = 0;
  s->item_cost_cap = s->item_cost_n = 0;
  s->copy_pending = s->timed = s->launched = false;
  s->pl_dirty = true;   // the primary lists go up again with the next upload
}

// Device half: allocations and uploads of everything dt_scene_prepare built (a few ms). On a
// failure everything allocated so far is released, so the next render's lazy upload retries cleanly.
static int scene_upload(dt_scene* s)
{
  if (s->uploaded) return DT_OK;
  const FlatScene& f = s->flat;
  const Accel& acc = s->acc;
  int rc;
  if ((rc = upload(s->sg.cells, &s->d_sg_cells)) || (rc = upload(s->sg.list, &s->d_sg_list)) ||
      (rc = upload(s->sg.sub_nodes, &s->d_sub_nodes)) || (rc = upload(s->sg.sub_blocks, &s->d_sub_blocks)) ||
      (rc = upload(acc.dnodes, &s->d_nodes)) || (rc = upload(acc.fnodes, &s->d_fnodes)) ||
      (rc = upload(acc.bnodes, &s->d_bnodes)) || (rc = upload(acc.bparent, &s->d_bparent)) || (rc = upload(acc.leaf, &s->d_leaf)) || (rc = upload(f.hdr, &s->d_hdr)) ||
      (rc = upload(f.geom, &s->d_geom)) || (rc = upload(f.mat, &s->d_mat)) || (rc = upload(f.lights, &s->d_lights)) ||
      (rc = upload(f.tex, &s->d_tex))) {
    release_device(s);
    return rc;
  }
  if (hipMalloc((void**)&s->d_stats, sizeof(unsigned long long) * 2 * STATS1) != hipSuccess ||
      hipMemset(s->d_stats, 0, sizeof(unsigned long long) * 2 * STATS1) != hipSuccess ||
      hipMalloc(&s->d_launch, 2 * dt_launch_size()) != hipSuccess || hipEventCreate(&s->ev0) != hipSuccess ||
      hipEventCreate(&s->ev1) != hipSuccess || hipEventCreateWithFlags(&s->ev_copy, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void**)&s->h_launch, dt_launch_size(), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&s->h_zs, 2048 * sizeof(float), hipHostMallocDefault) != hipSuccess) {
    release_device(s);
    return fail(DT_E_NO_DEVICE, "device allocation failed");
  }
  s->rec_last[0].clear();
  s->rec_last[1].clear();
  s->zs_last.clear();
  s->uploaded = true;
  return DT_OK;
}

int dt_scene_upload(dt_scene* s)
{
  if (!s) return fail(DT_E_INVALID, "null scene");
  if (int rc = scene_upload(s)) return rc;
  return upload_primary_lists(s);   // the primary lists dt_scene_prepare built
}

int dt_scene_create(const dt_scene_desc* desc, const dt_globals* g, dt_scene** out)
{
  int rc = dt_scene_prepare(desc, g, out);
  if (rc) return rc;
  if ((rc = dt_scene_upload(*out))) {
    dt_scene_destroy(*out);
    *out = nullptr;
    return rc;
  }
  return DT_OK;
}

void dt_scene_destroy(dt_scene* s)
{
  if (!s) return;
  release_device(s);
  delete s;
}

static int export_bvh(const FlatBVH& b, dt_bvh_node* nodes, int32_t cap, int32_t* indices, int32_t index_cap,
                      int32_t* n_nodes, int32_t* n_indices)
{
  for (size_t i = 0; i < b.nodes.size() && (int32_t)i < cap; ++i) {
    const dtd::DNode& n = b.nodes[i];
    dt_bvh_node& o = nodes[i];
    o.leaf = b.n_children[i] == 0 ? 1 : 0;
    o.n_children = b.n_children[i];
    o.first_child = b.n_children[i] ? (int32_t)i + 1 : -1;
    o.depth = b.depth[i];
    o.first_index = o.leaf ? n.first : -1;
    o.n_indices = o.leaf ? n.count : 0;
    for (int k = 0; k < 3; ++k) {
      o.lbound[k] = n.lb[k];
      o.ubound[k] = n.ub[k];
    }
  }
  for (size_t i = 0; i < b.leaf_idx.size() && (int32_t)i < index_cap; ++i) indices[i] = b.leaf_idx[i];
  if (n_nodes) *n_nodes = (int32_t)b.nodes.size();
  if (n_indices) *n_indices = (int32_t)b.leaf_idx.size();
  return DT_OK;
}

int dt_scene_bvh(const dt_scene* s, dt_bvh_node* nodes, int32_t cap, int32_t* indices, int32_t index_cap,
                 int32_t* n_nodes, int32_t* n_indices)
{
  if (!s) return fail(DT_E_INVALID, "null scene");
  return export_bvh(s->flat.bvh, nodes, cap, indices, index_cap, n_nodes, n_indices);
}

int dt_bvh_build(const dt_scene_desc* desc, const dt_globals* g, dt_bvh_node* nodes, int32_t cap, int32_t* indices,
                 int32_t index_cap, int32_t* n_nodes, int32_t* n_indices)
{
  if (!desc || !g) return fail(DT_E_INVALID, "null argument");
  if (desc->n_shapes < 0 || (desc->n_shapes > 0 && !desc->shapes)) return fail(DT_E_INVALID, "invalid descriptor");
  FlatBVH b;
  build_bvh(*desc, *g, b);
  return export_bvh(b, nodes, cap, indices, index_cap, n_nodes, n_indices);
}

// the scene's features (dt_scene_dev.h): which trace-kernel builds can render it (enqueue_render)
static unsigned scene_features(const dt_scene_desc& d)
{
  unsigned feat = 0;
  for (int i = 0; i < d.n_shapes; ++i) {
    const int t = d.shapes[i].type;
    feat |= (t >= 0 && t < DT_FEAT_SPHL) ? 1u << t : 1u << 31;
    if (d.shapes[i].model == DT_MODEL_OREN_NAYAR) feat |= 1u << DT_FEAT_ON;
    if (d.shapes[i].material == DT_MAT_GLASS) feat |= 1u << DT_FEAT_GLASS;
    if (d.shapes[i].emit == DT_EMIT_SPHERE) feat |= 1u << DT_FEAT_SPHL;
    if (d.shapes[i].emit == DT_EMIT_RECT) feat |= 1u << DT_FEAT_RECTL;
  }
  for (int i = 0; i < d.n_lights; ++i) {
    const int t = d.lights[i].type;
    if (t == DT_LIGHT_RECT) feat |= 1u << DT_FEAT_RECTL;
    else if (t != DT_LIGHT_POINT) feat |= 1u << DT_FEAT_SPHL;
  }
  return feat;
}

int dt_accel_info_build(const dt_scene_desc* desc, const dt_globals* g, dt_accel_info* info)
{
  if (!desc || !g || !info) return fail(DT_E_INVALID, "null argument");
  if (desc->n_shapes < 0 || (desc->n_shapes > 0 && !desc->shapes)) return fail(DT_E_INVALID, "invalid descriptor");
  // DT_TIMING=1: host stage times on stderr, as dt_scene_create
  const bool timing = getenv("DT_TIMING") != nullptr;
  auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double t_stage = now();
  auto stage = [&](const char* name) {
    if (!timing) return;
    const double t = now();
    fprintf(stderr, "dt_accel_info_build %-12s %8.2f ms\n", name, t - t_stage);
    t_stage = t;
  };
  FlatScene f;
  std::string err;
  int rc = flatten_scene(*desc, *g, f, err);
  if (rc) return fail(rc, err);
  stage("flatten+bvh");
  Accel a;
  build_accel(f, *g, a, stage);
  memset(info, 0, sizeof(*info));
  info->n_nodes = (int32_t)a.dnodes.size();
  info->n_fnodes = a.n_fnodes;
  info->n_bnodes = a.n_bnodes;
  info->boxes_ordered = a.boxes_ordered;
  info->features = scene_features(*desc);
  for (size_t b = 1; b < a.sg.sub_blocks.size(); b += 2) info->sg_sub_blocks += a.sg.sub_blocks[b] > 0;
  info->sg_sub_nodes = (int64_t)a.sg.sub_nodes.size();
  {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
    for (uint32_t x : a.sg.sub_blocks) mix(x);
    info->sg_sub_hash = (h ^ nodes_hash(a.sg.sub_nodes)) * 1099511628211ull;
  }
  info->sg_lights = a.sg.n_lights;
  for (int k = 0; k < 3; ++k) info->sg_dim[k] = a.sg.dim[k];
  info->sg_cells = (int64_t)(a.sg.cells.size() / 2);
  for (size_t c = 0; c + 1 < a.sg.cells.size(); c += 2) {
    if (a.sg.cells[c + 1] == DT_SG_WALK) info->sg_tree_cells++;
    else info->sg_list_entries += a.sg.cells[c + 1];
  }
  info->sg_list_pool = (int64_t)a.sg.list.size();
  info->nodes_hash = nodes_hash(a.dnodes);
  info->fnodes_hash = a.n_fnodes ? nodes_hash(a.fnodes) : 0;
  info->bnodes_hash = a.n_bnodes ? nodes_hash(a.bnodes) : 0;
  info->sg_hash = sg_hash(a.sg, false);
  info->sg_contents_hash = sg_hash(a.sg, true);
  info->bump_pad = a.bump_pad;
  info->sg_reach = a.sg.reach;
  info->sg_umbra_cells = a.sg.umbra_cells;
  return DT_OK;
}

int64_t dt_slab_floats(const dt_globals* g, const dt_tiles* tiles)
{
  dtd::DParams P;
  std::string err;
  if (!g || fill_sky_params(*g, 0.0f, tiles, P, err)) return -1;
  return P.n_owned_tiles * P.tw * P.th * 3;
}

int64_t dt_slab_floats_max(const dt_globals* g, const dt_tiles* tiles)
{
  if (!g || !tiles) return -1;
  dt_tiles t = *tiles;
  t.rank = 0;   // every rank has the same number of slots (dtd::tile_of)
  return dt_slab_floats(g, &t);
}

static int prepare_render(const dt_scene* sc, const dt_globals* g, int32_t frame, const dt_tiles* tiles,
                          dtd::DParams& P, std::vector<float>& zs)
{
  std::string err;
  int rc = fill_params(*g, frame, tiles, P, err);
  if (rc) return fail(rc, err);
  const int need = g->max_depth * (2 + (g->brdf_samples > 1 ? g->brdf_samples : 1));
  if (need > 48) return fail(DT_E_LIMIT, "max_depth*(2+brdf_samples) exceeds the device DFS stack (48)");
  zs = cloud_z_steps(*g);
  if (g->perlin_cloud && zs.size() > 2048) return fail(DT_E_LIMIT, "clouddist/0.05 exceeds 2048 march steps");
  P.n_nodes = (int32_t)sc->flat.bvh.nodes.size();
  P.n_fnodes = sc->n_fnodes;
  P.n_bnodes = sc->n_bnodes;
  P.bump_pad = sc->bump_pad;
  P.bump_up_only = sc->bump_up_only ? 1 : 0;
  P.no_cull = sc->no_cull ? 1 : 0;
  P.ftree_mode = sc->ftree_mode;
  P.boxes_ordered = sc->boxes_ordered;
  P.sg_n = sc->sg.n_lights;
  for (int a = 0; a < 3; ++a) {
    P.sg_dim[a] = sc->sg.dim[a];
    P.sg_lo[a] = sc->sg.lo[a];
    P.sg_inv[a] = sc->sg.inv_h[a];
  }
  for (int l = 0; l < DT_MAX_SGRID; ++l) {
    P.sg_base[l] = sc->sg.base[l];
    P.sg_base0[l] = sc->sg.base0[l];
  }
  P.sg_reach = sc->sg.reach;
  for (int l = 0; l < DT_MAX_SGRID; ++l) P.sgb_base[l] = sc->sg.sub_base[l];
  P.sgb_bx = sc->sg.sub_bx;
  P.sgb_by = sc->sg.sub_by;
  P.sgb_nbx = sc->sg.sub_nbx;
  P.sgb_nby = sc->sg.sub_nby;
  P.sgb_bz = sc->sg.sub_bz > 0 ? sc->sg.sub_bz : 1;
  // DT_SG_SUB_MULTI: a wave whose lanes lie in up to this many blocks walks their subtrees in turn
  // (default 1: only waves within one block); read per render
  const char* smu = getenv("DT_SG_SUB_MULTI");
  P.sgb_multi = smu && atoi(smu) > 0 ? atoi(smu) : 1;
  P.sg_ypad = (float)sc->sg.ypad;
  // start-side culling (host_shadowgrid.cpp) assumed every ray origin inside sg.org_lo..org_hi: a
  // camera whose eye region (eye +- the aperture) leaves it walks the trees instead of the lists
  if (sc->sg.org_check) {
    const double r = std::fabs((double)P.aperture);
    for (int a = 0; a < 3; ++a)
      if (!(P.eye[a] - r >= sc->sg.org_lo[a] && P.eye[a] + r <= sc->sg.org_hi[a])) P.sg_n = 0;
  }

  P.n_lights = (int32_t)sc->flat.lights.size();
  P.ls_first = 0;
  while (P.ls_first < P.n_lights && sc->flat.lights[P.ls_first].type != DT_LIGHT_RECT) ++P.ls_first;
  P.n_shapes = (int32_t)sc->flat.hdr.size();
  return DT_OK;
}

// Primary-ray candidate lists for P's camera (DT_PRIM_LISTS=0 disables them; DT_PL_BLOCK: pixels
// per block side, default 8). Rebuilt only when the camera or resolution changes; the device copy
// is replaced after the device has drained, since earlier launches may still read it.
static int update_primary_lists(dt_scene* sc, dtd::DParams& P, bool upload_now)
{
  P.pl_block = P.pl_nbx = P.pl_nby = P.pl_bump = 0;
  const char* e = getenv("DT_PRIM_LISTS");
  if ((e && e[0] == '0') || sc->n_fnodes <= 0 || !(sc->ftree_mode & 1) || sc->no_cull) return DT_OK;
  const char* b = getenv("DT_PL_BLOCK");
  const int B = b && atoi(b) > 0 ? atoi(b) : 8;
  // DT_PL_HULL=0: no hull culling; DT_PL_SUPER: blocks per super-block side (8); DT_PL_BUMP=0: the
  // blur passes walk the bump tree instead of taking lists
  const char* ph = getenv("DT_PL_HULL");
  const bool hull = !(ph && ph[0] == '0');
  const char* ps = getenv("DT_PL_SUPER");
  const int SB = ps && atoi(ps) > 0 ? atoi(ps) : 8;
  const char* pb = getenv("DT_PL_BUMP");
  const bool bump = !(pb && pb[0] == '0') && sc->n_bnodes > 0;
  std::vector<double> key = {(double)B, (double)P.xRes, (double)P.yRes, (double)P.l, (double)P.r, (double)P.t,
                             (double)P.b, (double)P.focal_length, (double)P.near_plane, (double)P.aperture,
                             (double)hull, (double)SB, (double)bump};
  for (int k = 0; k < 3; ++k) key.insert(key.end(), {P.eye[k], P.X[k], P.Y[k], P.Z[k]});
  if (key != sc->pl_key) {
    sc->pl_key = key;
    sc->pl_dirty = true;
    sc->pl_ok = build_primary_lists(sc->fnodes_host, sc->n_fnodes, P, B, sc->pl, hull ? &sc->fhull : nullptr, SB);
    sc->pl_bump = false;
    PrimLists pb_lists;
    if (sc->pl_ok && bump &&
        build_primary_lists(sc->bnodes_host, sc->n_bnodes, P, B, pb_lists, hull ? &sc->bhull : nullptr, SB)) {
      // the blur passes' lists follow: cells nblk.. 2 nblk - 1, entries after the pass-0 pool
      const uint32_t base = (uint32_t)(sc->pl.list.size() / 2);
      for (size_t c = 0; c < pb_lists.cells.size(); c += 2) {
        sc->pl.cells.push_back(pb_lists.cells[c] + base);
        sc->pl.cells.push_back(pb_lists.cells[c + 1]);
      }
      sc->pl.list.insert(sc->pl.list.end(), pb_lists.list.begin(), pb_lists.list.end());
      sc->pl_bump = true;
    }
  }
  if (upload_now)
    if (int rc = upload_primary_lists(sc)) return rc;
  if (sc->pl_ok) {
    P.pl_block = sc->pl.block;
    P.pl_nbx = sc->pl.nbx;
    P.pl_nby = sc->pl.nby;
    P.pl_bump = sc->pl_bump ? 1 : 0;
  }
  return DT_OK;
}

// device copy of the host primary lists, replaced once this scene's last trace launch has finished
// (it may still read the old one). Launches of one scene are stream-ordered (they share its launch
// record), so that is the event recorded after the last one; no device-wide barrier, which would
// also wait for unrelated work such as an RCCL gather in flight.
static int upload_primary_lists(dt_scene* sc)
{
  if (!sc->pl_dirty || !sc->uploaded) return DT_OK;
  if (sc->launched) HIPCHK(hipEventSynchronize(sc->ev1));
  if (sc->d_pl_cells) (void)hipFree(sc->d_pl_cells);
  if (sc->d_pl_list) (void)hipFree(sc->d_pl_list);
  sc->d_pl_cells = sc->d_pl_list = nullptr;
  sc->pl_dirty = false;
  if (sc->pl_ok) {
    int rc;
    if ((rc = upload(sc->pl.cells, &sc->d_pl_cells)) || (rc = upload(sc->pl.list, &sc->d_pl_list))) {
      sc->pl_ok = false;
      sc->pl_key.clear();
      return rc;
    }
  }
  return DT_OK;
}

// the device pointers of a scene's uploaded structures, as the kernels' DScene sees them
static void fill_hscene(const dt_scene* sc, HScene& hs)
{
  memset(&hs, 0, sizeof(hs));
  hs.nodes = sc->d_nodes;
  hs.fnodes = sc->d_fnodes;
  hs.bnodes = sc->d_bnodes;
  hs.bparent = (const int32_t*)sc->d_bparent;
  hs.sg_cells = (const uint32_t*)sc->d_sg_cells;
  hs.sg_list = (const int32_t*)sc->d_sg_list;
  hs.leaf_idx = (const int32_t*)sc->d_leaf;
  hs.hdr = sc->d_hdr;
  hs.geom = (const double*)sc->d_geom;
  hs.mat = sc->d_mat;
  hs.lights = sc->d_lights;
  hs.tex = (const uint8_t*)sc->d_tex;
  hs.pl_cells = (const uint32_t*)sc->d_pl_cells;
  hs.pl_list = (const uint32_t*)sc->d_pl_list;
  hs.sub_nodes = sc->d_sub_nodes;
  hs.sub_blocks = (const uint32_t*)sc->d_sub_blocks;
}

// The trace-kernel builds (dt_kernels.hip DT_TRACE_KERNEL, Makefile TRACE_BUILDS) and the choice
// of one per render.
struct Build {
  hipError_t (*launch)(const void*, float*, int, hipStream_t);
  const void* (*ptr)(void);
  int (*traits)(void);
  const char* name;
  int resident;
};
#define DT_B(k) {k##_launch, k##_ptr, k##_traits, #k, 0}
// per wave count (4, 5): room, mesh, full (still frames); tunnel, blur (motion-blur frames); sky
static Build g_builds[2][6] = {
    {DT_B(dt_trace_kernel), DT_B(dt_trace_kernel_mesh), DT_B(dt_trace_kernel_full),
     DT_B(dt_trace_kernel_tunnel), DT_B(dt_trace_kernel_blur), DT_B(dt_trace_kernel_sky)},
    {DT_B(dt_trace_kernel_w5), DT_B(dt_trace_kernel_w5_mesh), DT_B(dt_trace_kernel_w5_full),
     DT_B(dt_trace_kernel_w5_tunnel), DT_B(dt_trace_kernel_w5_blur), DT_B(dt_trace_kernel_w5_sky)}};
static Build g_dn_build = DT_B(dt_trace_kernel_dn), g_rpc_build = DT_B(dt_trace_kernel_rpc);
#undef DT_B

// the feature mask a build was compiled for (its traits' bits 8..23: dt_kernels.hip DT_FEATURES)
static unsigned build_features(const Build& b) { return ((unsigned)b.traits() >> 8) & 0xFFFFu; }
// the *_sky build of the same wave count as the product build b (it renders b's sky items)
static Build& sky_build_for(const Build& b)
{
  for (int v = 0; v < 6; ++v)
    if (&b == &g_builds[1][v]) return g_builds[1][5];
  return g_builds[0][5];
}

// The build a render of a scene with these features launches (kernel_choice: dt_scene_set_kernel).
static Build& choose_build(unsigned scene_features, bool no_cull, int kernel_choice, const dtd::DParams& P)
{
  // scenes with a RectPrismWithCylinder take the trace kernel compiled with its tests (dt_kernels.hip
  // DT_WITH_RPC), whose occupancy may differ. DFS work sharing inside the wave (dt_trace_kernel_dn)
  // when DT_DONATE=1; its pre-order paths hold 10 levels of 3 bits (max_depth <= 11, brdf_samples <= 6)
  // (dt_scene_set_kernel; DT_KERNEL_AUTO: the DT_DONATE environment variable)
  const char* dn_env = kernel_choice == DT_KERNEL_AUTO ? getenv("DT_DONATE") : nullptr;
  const bool want_dn = kernel_choice == DT_KERNEL_DONATE || (dn_env && dn_env[0] == '1');
  const bool donate = !no_cull && want_dn && P.max_depth <= 11 && P.brdf_samples <= 6;
  if (no_cull) return g_rpc_build;
  if (donate) return g_dn_build;
  // one pixel per wave (spp >= 64) takes the 5-waves-per-SIMD build (dt_kernels.hip DT_W5): C3 +1.8%,
  // C4 +4%; with several pixels per wave (C2, 16 spp) it loses 8% (profiles/r03ba_ab_w5.log).
  // DT_W5=0 never, DT_W5=1 at any spp with at most 8 pixels per wave (its per-pixel sums have 8 slots).
  const char* w5_env = getenv("DT_W5");
  const bool w5 = P.ppw <= 8 && (w5_env ? w5_env[0] == '1' : P.spp >= 64);
  // below frame_prism every motion-blur pass shifts by 0 (the reference's val, Q19), so those frames
  // take the product kernels built without the shift paths (dt_kernels.hip DT_NOSHIFT), room scenes
  // the builds without the shape types, lights and materials they lack (DT_FEATURES); later frames
  // the *_blur builds (DT_BLUR_KERNEL=1: those for every frame, the tests' check of the builds
  // against each other)
  const char* bk_env = getenv("DT_BLUR_KERNEL");
  const bool blur = P.frame >= P.frame_prism || (bk_env && bk_env[0] == '1');
  // DT_FULL_KERNEL=1: the builds with every feature for any scene (the tests' check of the
  // feature builds against them)
  const char* fk_env = getenv("DT_FULL_KERNEL");
  const unsigned feats = fk_env && fk_env[0] == '1' ? ~0u : scene_features;
  auto within = [&](unsigned mask) { return (feats & ~mask) == 0; };
  const int variant = blur ? (within(DT_TUNNEL_FEATURES) ? 3 : 4)
                           : within(DT_ROOM_FEATURES) ? 0 : within(DT_MESH_FEATURES) ? 1 : 2;
  return g_builds[w5 ? 1 : 0][variant];
}

int dt_trace_build(const dt_scene_desc* desc, const dt_globals* g, int32_t frame, char* name, int32_t name_cap,
                   uint32_t* scene_feats, uint32_t* build_feats)
{
  if (!desc || !g) return fail(DT_E_INVALID, "null argument");
  if (desc->n_shapes < 0 || (desc->n_shapes > 0 && !desc->shapes)) return fail(DT_E_INVALID, "invalid descriptor");
  dtd::DParams P;
  std::string err;
  int rc = fill_params(*g, frame, nullptr, P, err);
  if (rc) return fail(rc, err);
  bool no_cull = false;   // as build_accel: a RectPrismWithCylinder takes the rpc build
  for (int i = 0; i < desc->n_shapes; ++i) no_cull |= desc->shapes[i].type == DT_SHAPE_RECTPRISM_CYL;
  const unsigned f = scene_features(*desc);
  const Build& b = choose_build(f, no_cull, DT_KERNEL_AUTO, P);
  if (name && name_cap > 0) {
    strncpy(name, b.name, (size_t)name_cap - 1);
    name[name_cap - 1] = 0;
  }
  if (scene_feats) *scene_feats = f;
  if (build_feats) *build_feats = build_features(b);
  return DT_OK;
}

static int enqueue_render(dt_scene* sc, dtd::DParams P, const std::vector<float>& zs, float* out_dev,
                          hipStream_t st)
{
  if (int rc = scene_upload(sc)) return rc;
  if (int rc = update_primary_lists(sc, P, true)) return rc;
  // Fully asynchronous: the launch record and z table go through pinned staging that is
  // only rewritten after the previous call's copies have executed (ev_copy); the device
  // copies themselves are stream-ordered after any earlier kernel that reads them.
  if (sc->copy_pending) HIPCHK(hipEventSynchronize(sc->ev_copy));
  size_t nz = zs.size() < 2048 ? zs.size() : 2048;
  if (nz > sc->zs_cap) {
    if (sc->d_zs) HIPCHK(hipStreamSynchronize(st));
    if (sc->d_zs) (void)hipFree(sc->d_zs);
    sc->d_zs = nullptr;
    sc->zs_last.clear();
    sc->zs_cap = 2048;
    HIPCHK(hipMalloc(&sc->d_zs, sc->zs_cap * sizeof(float)));
  }
  if (nz) memcpy(sc->h_zs, zs.data(), nz * sizeof(float));
  HScene hs;
  fill_hscene(sc, hs);
  hs.cloud_z = (const float*)sc->d_zs;
  const int par = sc->n_launch & 1;
  hs.stats = sc->d_stats + par * STATS1;
  hs.queue = hs.stats + ST_N;
  hs.clear0 = sc->d_stats + (1 - par) * STATS1;
  hs.n_clear0 = (int32_t)STATS1;
  hs.clear1 = nullptr;
  hs.n_clear1 = 0;
  const int kernel_choice = sc->kernel;
  Build& kb = choose_build(sc->features, sc->no_cull, kernel_choice, P);
  const bool donate = &kb == &g_dn_build;
  Build& kb2 = sky_build_for(kb);
  // the build must handle every feature of the scene: its DT_FEATURES compile the others out to
  // __builtin_unreachable() (tests/test_host.py checks every builder scene; this guards the rest)
  if (sc->features & ~build_features(kb))
    return fail(DT_E_INVALID, "no trace-kernel build covers the scene's features");
  if (!kb.resident) kb.resident = max_resident_waves(kb.ptr(), 64);
  const int64_t waves = kb.resident;
  // Chunk items (spp > 64: C4's 256): every 64-sample chunk of a pixel is a queue item of its own, so
  // a pixel's chunks run on different waves and a long pixel no longer holds one wave for four
  // chunks in turn. The chunks store their sample colours; dt_chunk_sum_kernel adds each pixel's up
  // in sample order after the trace launch(es) (dt_kernels.hip). For a rank's share of a split frame
  // (world > 1): C4's world-8 shares 44.0 against 48.6 ms for the slowest (profiles/r06c_rb_*). A
  // whole frame keeps one item per pixel: there the stored colours and the sum kernel cost C4 1.5%
  // (1710 against 1736 Mpixel-samples/s with the chunks of a pixel dequeued together, r06b).
  // DT_CHUNK_ITEMS=0 / 1 / 2 (2: the queue chunk-major, the tests' check) overrides the default.
  const char* ci_env = getenv("DT_CHUNK_ITEMS");
  int chunk_items = ci_env ? atoi(ci_env) : (P.world > 1 ? 1 : 0);
  // (the build and, for a sky-item launch, its *_sky build must carry the code: trait bit 1)
  if (!(kb.traits() & 2) || !(kb2.traits() & 2) || P.chunks < 2 || P.chunks > 255 || chunk_items < 0 ||
      chunk_items > 2 || (double)P.n_items * P.chunks >= 4294967296.0)
    chunk_items = 0;
  P.chunk_items = chunk_items;
  if (chunk_items) {
    const int64_t n_cols = P.n_items * (int64_t)P.spp * 3;
    if (n_cols > sc->chunk_cols_cap) {
      HIPCHK(hipStreamSynchronize(st));
      if (sc->d_chunk_cols) (void)hipFree(sc->d_chunk_cols);
      sc->d_chunk_cols = nullptr;
      sc->chunk_cols_cap = 0;
      HIPCHK(hipMalloc((void**)&sc->d_chunk_cols, sizeof(double) * (size_t)n_cols));
      sc->chunk_cols_cap = n_cols;
    }
  }
  hs.chunk_cols = chunk_items ? sc->d_chunk_cols : nullptr;
  const int64_t n_queue = P.n_items * (chunk_items ? P.chunks : 1);
  // DT_ITEM_COSTS=1: every item's duration, for builds that record it (-DDT_ITEM_TIMES=2; others leave
  // the array as it is): dt_debug_item_costs
  hs.item_cost = nullptr;
  if (getenv("DT_ITEM_COSTS") && getenv("DT_ITEM_COSTS")[0] == '1' && n_queue > 0) {
    if (n_queue > sc->item_cost_cap) {
      HIPCHK(hipStreamSynchronize(st));
      if (sc->d_item_cost) (void)hipFree(sc->d_item_cost);
      sc->d_item_cost = nullptr;
      sc->item_cost_cap = 0;
      HIPCHK(hipMalloc((void**)&sc->d_item_cost, sizeof(uint32_t) * (size_t)n_queue));
      sc->item_cost_cap = n_queue;
    }
    HIPCHK(hipMemsetAsync(sc->d_item_cost, 0, sizeof(uint32_t) * (size_t)n_queue, st));
    hs.item_cost = sc->d_item_cost;
    sc->item_cost_n = n_queue;
  }
  int64_t grid = n_queue < waves ? n_queue : waves;
  if (grid < 1) grid = 1;
  hs.dn_pool = nullptr;
  if (donate) {
    if (grid > sc->dn_pool_waves) {
      if (sc->d_dn_pool) {
        HIPCHK(hipStreamSynchronize(st));
        (void)hipFree(sc->d_dn_pool);
        sc->d_dn_pool = nullptr;
        sc->dn_pool_waves = 0;
      }
      HIPCHK(hipMalloc(&sc->d_dn_pool, (size_t)grid * DT_DN_POOL_REC * 32));
      sc->dn_pool_waves = grid;
    }
    hs.dn_pool = sc->d_dn_pool;
  }
  // two items per queue atomic pays when every wave takes many items (C3: ~500, +2%; C3's 1/8
  // tile share: 63, its kernel -3.3%, profiles/r03x); with few (C2: ~30) the coarser tail costs
  // more (-11%). DT_BATCH_ITEMS: the items per wave from which DT_BATCH_SIZE (2) are dequeued at once
  dtd::DParams PL = P;
  const char* bi = getenv("DT_BATCH_ITEMS");
  const char* bs = getenv("DT_BATCH_SIZE");
  const int64_t batch_from = bi && atoi(bi) > 0 ? atoi(bi) : 32;
  // Items of several 64-sample chunks (spp > 64: C4's 256) take one per atomic: their dequeues are
  // rare already, and two consecutive pixels per wave cost C4 2.7% (profiles/r04zl_c4_batch.log)
  // Three per atomic once every wave takes 256 or more (a whole C3 frame: ~405 per wave, +0.6%,
  // profiles/r05q_ab_switches.txt); the 1/8 shares (~50 per wave) keep two, where three cost their
  // bound 2.5% in round 4 (r04zj_ab_batch_policies.log)
  PL.item_batch = n_queue >= batch_from * grid && (PL.chunks == 1 || (bs && atoi(bs) > 0))
                      ? (bs && atoi(bs) > 0 ? atoi(bs) : (n_queue >= 256 * grid ? 3 : 2)) : 1;
  // The queue in 8 contiguous segments, each with its own counter, wave b's home segment b % 8 (the
  // XCD workgroup b runs on), a drained segment sending its waves on to the next (dt_kernels.hip),
  // for a rank's share of a split frame of one-chunk items: C3's world-8 shares 4.46 against 4.54 ms
  // (bound 0.933 against 0.921, profiles/r05zg_rank_balance_segs_default.log), C2's 0.569 against
  // 0.591. A whole frame keeps one counter (C3 -1.4%, C4 -3.4%, C2 -0.5% with eight), and so do
  // pixels of several chunks in one item (C4's world-8 shares 49.4 against 47.1 ms with eight,
  // profiles/r05zi_*). Chunk items take eight: C4's slowest world-8 share 43.97 against 45.77 ms
  // (profiles/r06c_rb_m1s8.log, r06c_rb_m1.log). DT_QUEUE_SEGS=<n> (1..8) overrides.
  const char* qs = getenv("DT_QUEUE_SEGS");
  PL.queue_segs = qs ? std::max(1, std::min(atoi(qs), DT_QSEG_MAX))
                     : (PL.world > 1 && (PL.chunks == 1 || PL.chunk_items) ? DT_QSEG_MAX : 1);
  // deep-cascade waves raise their priority (dt_kernels.hip, DT_PRIO_STEPS) when the frame is split
  // over ranks, where one such wave bounds a rank's kernel, and after 2 DFS steps in whole frames of
  // several pixels per wave (spp < 64: C2, whose frame is bounded by a column of 30x-mean glossy items,
  // profiles/r06h_tail_c2.log): C2 +0.9%, C3 +0.1%, C4 -0.4% (so not there; profiles/r06o_ab.txt).
  // DT_PRIO_STEPS=<n> overrides (0: off)
  const char* ps = getenv("DT_PRIO_STEPS");
  PL.prio_steps = ps ? atoi(ps) : (PL.world > 1 ? 8 : PL.ppw > 1 ? 2 : 0);
  // 1 spp (C5's cloud frames, n >= 244: nearly every pixel is sky): the trace kernel only flags
  // the missed pixels and dt_sky_miss_kernel marches their sky one pixel per lane, instead of the
  // wave marching each of its 64 pixels cooperatively in turn. DT_SKY_DEFER=0 disables it.
  const bool defer_on = !(getenv("DT_SKY_DEFER") && getenv("DT_SKY_DEFER")[0] == '0');
  const int64_t n_px = PL.n_items * PL.ppw;
  PL.sky_defer = 0;
  hs.sky_miss = nullptr;
  if (defer_on && PL.spp == 1 && PL.perlin_cloud && n_px > 0) {
    if (n_px > sc->sky_miss_cap) {
      HIPCHK(hipStreamSynchronize(st));
      if (sc->d_sky_miss) (void)hipFree(sc->d_sky_miss);
      sc->d_sky_miss = nullptr;
      HIPCHK(hipMalloc((void**)&sc->d_sky_miss, n_px));
      HIPCHK(hipMemsetAsync(sc->d_sky_miss, 0, n_px, st));
      sc->sky_miss_cap = n_px;
    }
    PL.sky_defer = 1;
    hs.sky_miss = sc->d_sky_miss;
  }
  // DT_GENERAL_WALKS=1: every wave takes the exact reference-tree walks that axis-parallel rays
  // take (the tests' check of those rare, out-of-line paths against the product walks)
  const char* gw_env = getenv("DT_GENERAL_WALKS");
  if (gw_env && gw_env[0] == '1') PL.boxes_ordered = 0;
  // a still build without the sky march lists its items with a missed sample (multi-sample
  // renders of a scene with perlin_cloud; dt_kernels.hip DT_SKY_AGAIN) and the *_sky build of the
  // same wave count renders them in a second launch with counters of its own. The first launch
  // counts the listed items, the second takes their counts back but for their sky and NaN pixels;
  // dt_collect_stats adds the two up.
  const bool again = (kb.traits() & 1) && PL.perlin_cloud && !PL.sky_defer;
  PL.sky_again = again ? 1 : 0;
  hs.again_list = nullptr;
  hs.again_n = nullptr;
  if (again) {
    if (!sc->d_stats2 || !sc->d_launch2 || !sc->h_launch2) {
      // all three or none: allocated into temporaries, committed together, freed on a failure
      unsigned long long* st2 = nullptr;
      void* dl2 = nullptr;
      uint8_t* hl2 = nullptr;
      hipError_t e = hipMalloc((void**)&st2, sizeof(unsigned long long) * 2 * STATS2);
      if (e == hipSuccess) e = hipMemsetAsync(st2, 0, sizeof(unsigned long long) * 2 * STATS2, st);
      if (e == hipSuccess) e = hipMalloc(&dl2, 2 * dt_launch_size());
      if (e == hipSuccess) e = hipHostMalloc((void**)&hl2, dt_launch_size(), hipHostMallocDefault);
      if (e != hipSuccess) {
        if (st2) (void)hipFree(st2);
        if (dl2) (void)hipFree(dl2);
        if (hl2) (void)hipHostFree(hl2);
        return fail(DT_E_NO_DEVICE, std::string("sky-item launch buffers: ") + hipGetErrorString(e));
      }
      if (sc->d_stats2) (void)hipFree(sc->d_stats2);
      if (sc->d_launch2) (void)hipFree(sc->d_launch2);
      if (sc->h_launch2) (void)hipHostFree(sc->h_launch2);
      sc->d_stats2 = st2;
      sc->d_launch2 = dl2;
      sc->h_launch2 = hl2;
      sc->rec2_last[0].clear();
      sc->rec2_last[1].clear();
    }
    if (n_queue > sc->again_cap) {   // (a listed item: its queue code, dt_kernels.hip)
      HIPCHK(hipStreamSynchronize(st));
      if (sc->d_again) (void)hipFree(sc->d_again);
      sc->d_again = nullptr;
      HIPCHK(hipMalloc((void**)&sc->d_again, sizeof(uint32_t) * n_queue));
      sc->again_cap = n_queue;
    }
    hs.again_list = sc->d_again;
    hs.again_n = (unsigned int*)(sc->d_stats2 + par * STATS2 + ST_N + 1);
  }
  if (sc->d_stats2) {   // the sky-item counters of the next launch, whether or not it runs one
    hs.clear1 = sc->d_stats2 + (1 - par) * STATS2;
    hs.n_clear1 = (int32_t)STATS2;
  }
  PL.donate = donate ? 1 : 0;
  const char* dn_after = getenv("DT_DONATE_AFTER");
  PL.donate_after = dn_after ? atoi(dn_after) : 2;
  if (sizeof(HScene) != dt_scene_struct_size()) return fail(DT_E_INVALID, "HScene does not match the device DScene");
  memset(sc->h_launch, 0, dt_launch_size());
  memcpy(sc->h_launch + dt_scene_struct_offset(), &hs, sizeof(hs));   // after every hs field is set
  memcpy(sc->h_launch + dt_params_struct_offset(), &PL, sizeof(PL));
  // the z table too only when it changed (the same for every frame of a scene's sky)
  if (nz && (sc->zs_last.size() != nz || memcmp(sc->zs_last.data(), sc->h_zs, nz * sizeof(float)) != 0)) {
    HIPCHK(hipMemcpyAsync(sc->d_zs, sc->h_zs, nz * sizeof(float), hipMemcpyHostToDevice, st));
    sc->zs_last.assign(sc->h_zs, sc->h_zs + nz);
  }
  const size_t rec_size = dt_launch_size();
  uint8_t* const d_rec = (uint8_t*)sc->d_launch + par * rec_size;
  if (sc->rec_last[par].size() != rec_size || memcmp(sc->rec_last[par].data(), sc->h_launch, rec_size) != 0) {
    HIPCHK(hipMemcpyAsync(d_rec, sc->h_launch, rec_size, hipMemcpyHostToDevice, st));
    sc->rec_last[par].assign(sc->h_launch, sc->h_launch + rec_size);
  }
  uint8_t* const d_rec2 = sc->d_launch2 ? (uint8_t*)sc->d_launch2 + par * rec_size : nullptr;
  if (again) {   // the second launch: the listed items, counters of its own
    HScene hs2 = hs;
    hs2.stats = sc->d_stats2 + par * STATS2;
    hs2.queue = hs2.stats + ST_N;
    hs2.clear0 = nullptr;   // the first launch cleared them
    hs2.n_clear0 = 0;
    hs2.clear1 = nullptr;
    hs2.n_clear1 = 0;
    dtd::DParams PL2 = PL;
    PL2.sky_again = 2;
    PL2.item_batch = 1;
    PL2.queue_segs = 1;
    PL2.prio_steps = 0;
    memset(sc->h_launch2, 0, dt_launch_size());
    memcpy(sc->h_launch2 + dt_scene_struct_offset(), &hs2, sizeof(hs2));
    memcpy(sc->h_launch2 + dt_params_struct_offset(), &PL2, sizeof(PL2));
    if (sc->rec2_last[par].size() != rec_size || memcmp(sc->rec2_last[par].data(), sc->h_launch2, rec_size) != 0) {
      HIPCHK(hipMemcpyAsync(d_rec2, sc->h_launch2, rec_size, hipMemcpyHostToDevice, st));
      sc->rec2_last[par].assign(sc->h_launch2, sc->h_launch2 + rec_size);
    }
  }
  HIPCHK(hipEventRecord(sc->ev_copy, st));
  sc->copy_pending = true;
  HIPCHK(hipEventRecord(sc->ev0, st));
  HIPCHK(kb.launch(d_rec, out_dev, (int)grid, st));
  sc->last_parity = par;
  sc->n_launch++;
  if (again) {
    if (!kb2.resident) kb2.resident = max_resident_waves(kb2.ptr(), 64);
    // a few listed items in the scenes that use it (room frames: none to a handful): 512 waves
    // start and drain faster than a full persistent grid
    int64_t g2 = grid < kb2.resident ? grid : kb2.resident;
    g2 = g2 < 512 ? g2 : 512;
    HIPCHK(kb2.launch(d_rec2, out_dev, (int)g2, st));
  }
  sc->again_used = again;
  if (PL.sky_defer) HIPCHK(dt_launch_sky_miss(d_rec, out_dev, n_px, st));
  // chunk items: every pixel's sample colours added up in sample order, once both launches stored theirs
  if (PL.chunk_items) HIPCHK(dt_launch_chunk_sum(d_rec, out_dev, PL.n_items, st));
  HIPCHK(hipEventRecord(sc->ev1, st));
  sc->timed = true;
  sc->launched = true;
  sc->last = P;
  return DT_OK;
}

int dt_collect_stats(const dt_scene* sc_c, void* stream, dt_stats* stats)
{
  dt_scene* sc = const_cast<dt_scene*>(sc_c);
  if (!sc) return fail(DT_E_INVALID, "null scene");
  if (!sc->uploaded) return fail(DT_E_INVALID, "scene not uploaded (dt_scene_upload)");
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipStreamSynchronize(st));
  if (!stats) return DT_OK;
  unsigned long long h[ST_N];
  {   // the counters and their per-slot copies (dt_kernels.hip: wave b adds to copy b % DT_STAT_SLOTS)
    std::vector<unsigned long long> blk(STATS1);
    HIPCHK(hipMemcpy(blk.data(), sc->d_stats + sc->last_parity * STATS1, sizeof(unsigned long long) * STATS1,
                     hipMemcpyDeviceToHost));
    for (int k = 0; k < ST_N; ++k) {
      h[k] = blk[k];
      for (int s = 1; s < DT_STAT_SLOTS; ++s) h[k] += blk[ST_N + DT_STAT_SLOT_OFF + (s - 1) * DT_STAT_SLOT_STRIDE + k];
    }
  }
  if (sc->again_used) {   // the listed items' second launch (dt_kernels.hip DT_SKY_AGAIN)
    unsigned long long h2[ST_N];
    HIPCHK(hipMemcpy(h2, sc->d_stats2 + sc->last_parity * STATS2, sizeof(h2), hipMemcpyDeviceToHost));
    for (int k = 0; k < ST_N; ++k) h[k] += h2[k];
  }
  memset(stats, 0, sizeof(*stats));
  const dtd::DParams& P = sc->last;
  int64_t px = 0;
  {
    // pixels rendered = owned pixels inside the window
    int64_t tiles_y = (P.y1 - P.y0 + P.th - 1) / P.th;
    for (int64_t k = 0; k < P.n_owned_tiles; ++k) {
      int64_t t = dtd::tile_of(k, P.rank, P.world);
      if (t >= P.n_tiles) continue;
      int ty = (int)(t / P.tiles_x), tx = (int)(t % P.tiles_x);
      (void)tiles_y;
      int w = P.x1 - (P.x0 + tx * P.tw);
      int hh = P.y1 - (P.y0 + ty * P.th);
      w = w < P.tw ? w : P.tw;
      hh = hh < P.th ? hh : P.th;
      px += (int64_t)w * hh;
    }
  }
  stats->pixels = px;
  stats->samples = (uint64_t)px * P.spp;
  stats->rays = h[ST_RAYS];
  stats->shadow_rays = h[ST_SHADOW];
  stats->sky_pixels = h[ST_SKY];
  stats->uv_out_of_range = h[ST_UV];
  stats->glossy_exhausted = h[ST_GLOSSY];
  stats->spherelight_exhausted = h[ST_SPHL];
  stats->prism_norm_fallback = h[ST_PRISM];
  stats->reflect_errors = h[ST_REFL];
  stats->nan_pixels = h[ST_NAN];
  stats->tex_fetches = h[ST_TEX];
  stats->stack_overflows = h[ST_STACK];
  stats->box_tests = h[ST_BOX];
  stats->prim_tests = h[ST_PRIM];
  stats->wave_node_visits = h[ST_WNODES];
  stats->donations = h[ST_DONATE];
  stats->donate_overflow = h[ST_DN_OVF];
  if (sc->timed) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, sc->ev0, sc->ev1) == hipSuccess) {
      stats->kernel_ms = ms;
      stats->trace_kernel_ms = ms;
    }
  }
  return DT_OK;
}

int dt_render_async(const dt_scene* sc_c, const dt_globals* g, int32_t frame, const dt_tiles* tiles,
                    float* out_device, void* stream)
{
  dt_scene* sc = const_cast<dt_scene*>(sc_c);
  if (!sc || !g || !out_device) return fail(DT_E_INVALID, "null argument");
  dtd::DParams P;
  std::vector<float> zs;
  int rc = prepare_render(sc, g, frame, tiles, P, zs);
  if (rc) return rc;
  return enqueue_render(sc, P, zs, out_device, (hipStream_t)stream);
}

int dt_render(const dt_scene* sc_c, const dt_globals* g, int32_t frame, const dt_tiles* tiles, float* out,
              int32_t out_on_device, void* stream, dt_stats* stats)
{
  dt_scene* sc = const_cast<dt_scene*>(sc_c);
  if (!sc || !g || !out) return fail(DT_E_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  dtd::DParams P;
  std::vector<float> zs;
  int rc = prepare_render(sc, g, frame, tiles, P, zs);
  if (rc) return rc;
  float* dout = out;
  size_t n_out = P.layout == DT_OUT_SLAB ? (size_t)(P.n_owned_tiles * P.tw * P.th * 3)
                                         : (size_t)g->xRes * g->yRes * 3;
  if (!out_on_device) {
    HIPCHK(hipMalloc((void**)&dout, n_out * sizeof(float)));
    // a render that writes every float of the output (the whole image, one rank) needs no copy of
    // the caller's buffer; otherwise the pixels it does not own keep the caller's values
    const bool covers = P.layout == DT_OUT_IMAGE && P.world == 1 && P.x0 == 0 && P.y0 == 0 && P.x1 == g->xRes &&
                        P.y1 == g->yRes;
    if (!covers) HIPCHK(hipMemcpyAsync(dout, out, n_out * sizeof(float), hipMemcpyHostToDevice, st));
  }
  rc = enqueue_render(sc, P, zs, dout, st);
  if (rc == DT_OK && !out_on_device) {
    hipError_t e = hipMemcpyAsync(out, dout, n_out * sizeof(float), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) rc = fail(DT_E_NO_DEVICE, hipGetErrorString(e));
  }
  if (rc == DT_OK) rc = dt_collect_stats(sc, stream, stats);
  if (!out_on_device) (void)hipFree(dout);
  return rc;
}

// Intersection micro-benchmark: dt_isect_kernel over rays first_ray .. first_ray+n_rays-1
// of the globals' camera. Synchronous; its own launch record and counters, so it may run beside
// renders of the same scene on other streams.
int dt_intersect_primary(const dt_scene* sc_c, const dt_globals* g, int32_t frame, int64_t first_ray, int64_t n_rays,
                         int32_t* hit_shape, float* hit_t, int32_t out_on_device, void* stream, float* kernel_ms)
{
  dt_scene* sc = const_cast<dt_scene*>(sc_c);
  if (!sc || !g || !hit_shape || !hit_t) return fail(DT_E_INVALID, "null argument");
  if (first_ray < 0 || n_rays < 0) return fail(DT_E_INVALID, "negative ray range");
  if (sc->no_cull) return fail(DT_E_UNSUPPORTED, "dt_intersect_primary: scenes with a RectPrismWithCylinder");
  if (n_rays == 0) {
    if (kernel_ms) *kernel_ms = 0;
    return DT_OK;
  }
  hipStream_t st = (hipStream_t)stream;
  dtd::DParams P;
  std::vector<float> zs;
  dt_tiles whole;
  memset(&whole, 0, sizeof(whole));
  whole.world = 1;
  int rc = prepare_render(sc, g, frame, &whole, P, zs);
  if (rc) return rc;
  if ((rc = scene_upload(sc)) || (rc = update_primary_lists(sc, P, true))) return rc;
  struct Tmp {   // released on every return path, after the stream's work that may use them
    hipStream_t st = nullptr;
    void *launch = nullptr, *stats = nullptr, *shape = nullptr, *t = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    ~Tmp()
    {
      if (launch) (void)hipStreamSynchronize(st);
      for (void* b : {launch, stats, shape, t})
        if (b) (void)hipFree(b);
      if (e0) (void)hipEventDestroy(e0);
      if (e1) (void)hipEventDestroy(e1);
    }
  } tmp;
  tmp.st = st;
  const size_t n_stats = sizeof(unsigned long long) * (ST_N + 1);
  HIPCHK(hipMalloc(&tmp.launch, dt_launch_size()));
  HIPCHK(hipMalloc(&tmp.stats, n_stats));
  HIPCHK(hipMemsetAsync(tmp.stats, 0, n_stats, st));
  HScene hs;
  fill_hscene(sc, hs);
  hs.stats = (unsigned long long*)tmp.stats;
  hs.queue = hs.stats + ST_N;
  std::vector<uint8_t> L(dt_launch_size(), 0);
  memcpy(L.data() + dt_scene_struct_offset(), &hs, sizeof(hs));
  memcpy(L.data() + dt_params_struct_offset(), &P, sizeof(P));
  HIPCHK(hipMemcpyAsync(tmp.launch, L.data(), L.size(), hipMemcpyHostToDevice, st));
  int32_t* dshape = hit_shape;
  float* dt_ = hit_t;
  if (!out_on_device) {
    HIPCHK(hipMalloc(&tmp.shape, (size_t)n_rays * sizeof(int32_t)));
    HIPCHK(hipMalloc(&tmp.t, (size_t)n_rays * sizeof(float)));
    dshape = (int32_t*)tmp.shape;
    dt_ = (float*)tmp.t;
  }
  static int resident = 0;
  if (!resident) resident = max_resident_waves(dt_isect_kernel_ptr(), 64);
  const int64_t waves = (n_rays + 63) / 64;
  const int grid = (int)(waves < resident ? waves : resident);
  HIPCHK(hipEventCreate(&tmp.e0));
  HIPCHK(hipEventCreate(&tmp.e1));
  HIPCHK(hipEventRecord(tmp.e0, st));
  HIPCHK(dt_launch_isect(tmp.launch, first_ray, n_rays, dshape, dt_, grid > 0 ? grid : 1, st));
  HIPCHK(hipEventRecord(tmp.e1, st));
  if (!out_on_device) {
    HIPCHK(hipMemcpyAsync(hit_shape, dshape, (size_t)n_rays * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(hit_t, dt_, (size_t)n_rays * sizeof(float), hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  if (kernel_ms) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tmp.e0, tmp.e1));
    *kernel_ms = ms;
  }
  return DT_OK;
}

int dt_render_sky(const dt_globals* g, float frame, const dt_tiles* tiles, float* out, int32_t out_on_device,
                  void* stream, dt_stats* stats)
{
  if (!g || !out) return fail(DT_E_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  dtd::DParams P;
  std::string err;
  int rc = fill_sky_params(*g, frame, tiles, P, err);
  if (rc) return fail(rc, err);
  std::vector<float> zs = cloud_z_steps(*g);
  void *d_zs = nullptr, *d_launch = nullptr;
  float* dout = out;
  size_t n_out = P.layout == DT_OUT_SLAB ? (size_t)(P.n_owned_tiles * P.tw * P.th * 3) : (size_t)g->xRes * g->yRes * 3;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<uint8_t> L(dt_launch_size(), 0);
  HScene hs;
  memset(&hs, 0, sizeof(hs));
  HIPCHK(hipMalloc(&d_zs, (zs.size() + 1) * sizeof(float)));
  HIPCHK(hipMalloc(&d_launch, L.size()));
  HIPCHK(hipMemcpyAsync(d_zs, zs.data(), zs.size() * sizeof(float), hipMemcpyHostToDevice, st));
  hs.cloud_z = (const float*)d_zs;
  memcpy(L.data() + dt_scene_struct_offset(), &hs, sizeof(hs));
  memcpy(L.data() + dt_params_struct_offset(), &P, sizeof(P));
  HIPCHK(hipMemcpyAsync(d_launch, L.data(), L.size(), hipMemcpyHostToDevice, st));
  if (!out_on_device) {
    HIPCHK(hipMalloc((void**)&dout, n_out * sizeof(float)));
    HIPCHK(hipMemcpyAsync(dout, out, n_out * sizeof(float), hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipEventRecord(e0, st));
  HIPCHK(dt_launch_sky(d_launch, dout, P.n_owned_tiles * P.tw * P.th, st));
  HIPCHK(hipEventRecord(e1, st));
  if (!out_on_device) HIPCHK(hipMemcpyAsync(out, dout, n_out * sizeof(float), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    stats->kernel_ms = ms;
    stats->trace_kernel_ms = ms;
    int64_t w = P.x1 - P.x0, h = P.y1 - P.y0;
    stats->pixels = P.world == 1 ? (uint64_t)(w * h) : 0;
    stats->samples = stats->pixels;
    stats->sky_pixels = stats->pixels;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d_zs);
  (void)hipFree(d_launch);
  if (!out_on_device) (void)hipFree(dout);
  return DT_OK;
}

int dt_unpack_slabs(const dt_globals* g, const dt_tiles* tiles, int32_t world, const float* slabs, float* image,
                    int32_t on_device, void* stream)
{
  if (!g || !tiles || !slabs || !image || world < 1) return fail(DT_E_INVALID, "null argument");
  dt_tiles t = *tiles;
  t.rank = 0;
  t.world = world;
  dtd::DParams P;
  std::string err;
  int rc = fill_sky_params(*g, 0.0f, &t, P, err);
  if (rc) return fail(rc, err);
  int64_t slab_floats = P.n_owned_tiles * P.tw * P.th * 3;
  if (!on_device) {
    // host scatter
    int64_t ntiles = (int64_t)P.tiles_x * ((P.y1 - P.y0 + P.th - 1) / P.th);
    for (int r = 0; r < world; ++r) {
      int64_t owned = (ntiles + world - 1) / world;
      for (int64_t slot = 0; slot < owned; ++slot) {
        int64_t tid = dtd::tile_of(slot, r, world);
        if (tid >= ntiles) continue;
        int ty = (int)(tid / P.tiles_x), tx = (int)(tid % P.tiles_x);
        for (int py = 0; py < P.th; ++py)
          for (int px = 0; px < P.tw; ++px) {
            int x = P.x0 + tx * P.tw + px, y = P.y0 + ty * P.th + py;
            if (x >= P.x1 || y >= P.y1) continue;
            const float* s = slabs + r * slab_floats + ((slot * P.th + py) * P.tw + px) * 3;
            float* d = image + 3 * ((int64_t)(g->yRes - 1 - y) * g->xRes + x);
            d[0] = s[0];
            d[1] = s[1];
            d[2] = s[2];
          }
      }
    }
    return DT_OK;
  }
  hipStream_t st = (hipStream_t)stream;
  void* d_launch = nullptr;
  std::vector<uint8_t> L(dt_launch_size(), 0);
  memcpy(L.data() + dt_params_struct_offset(), &P, sizeof(P));
  HIPCHK(hipMalloc(&d_launch, L.size()));
  HIPCHK(hipMemcpyAsync(d_launch, L.data(), L.size(), hipMemcpyHostToDevice, st));
  HIPCHK(dt_launch_unpack(d_launch, world, slab_floats, slabs, image, st));
  HIPCHK(hipStreamSynchronize(st));
  (void)hipFree(d_launch);
  return DT_OK;
}

int dt_write_ppm(const char* filename, int32_t xRes, int32_t yRes, const float* values)
{
  // helpers.h:174-195: float -> unsigned char conversion (truncation)
  if (!filename || !values || xRes <= 0 || yRes <= 0) return fail(DT_E_INVALID, "bad arguments");
  size_t total = (size_t)xRes * yRes * 3;
  std::vector<unsigned char> px(total);
  for (size_t i = 0; i < total; ++i) px[i] = (unsigned char)values[i];
  FILE* fp = fopen(filename, "wb");
  if (!fp) return fail(DT_E_IO, std::string("could not open ") + filename);
  fprintf(fp, "P6\n%d %d\n255\n", xRes, yRes);
  fwrite(px.data(), 1, total, fp);
  fclose(fp);
  return DT_OK;
}

static void put_be32(std::vector<unsigned char>& v, uint32_t x)
{
  v.push_back((unsigned char)(x >> 24)); v.push_back((unsigned char)(x >> 16));
  v.push_back((unsigned char)(x >> 8)); v.push_back((unsigned char)x);
}

int dt_write_png(const char* filename, int32_t xRes, int32_t yRes, const float* values)
{
  // the same 8-bit pixels as dt_write_ppm (float -> unsigned char truncation), as an RGB PNG
  if (!filename || !values || xRes <= 0 || yRes <= 0) return fail(DT_E_INVALID, "bad arguments");
  const size_t row = (size_t)xRes * 3;
  std::vector<unsigned char> raw((row + 1) * (size_t)yRes);
  for (int y = 0; y < yRes; ++y) {
    raw[y * (row + 1)] = 0;   // filter type none
    for (size_t i = 0; i < row; ++i) raw[y * (row + 1) + 1 + i] = (unsigned char)values[(size_t)y * row + i];
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<unsigned char> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return fail(DT_E_IO, "zlib failed");
  z.resize(zlen);
  std::vector<unsigned char> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  auto chunk = [&](const char* type, const std::vector<unsigned char>& data) {
    put_be32(png, (uint32_t)data.size());
    const size_t at = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), data.begin(), data.end());
    put_be32(png, (uint32_t)crc32(0L, png.data() + at, (uInt)(png.size() - at)));
  };
  std::vector<unsigned char> ihdr;
  put_be32(ihdr, (uint32_t)xRes);
  put_be32(ihdr, (uint32_t)yRes);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit, RGB, deflate, no filter, no interlace
  chunk("IHDR", ihdr);
  chunk("IDAT", z);
  chunk("IEND", {});
  FILE* fp = fopen(filename, "wb");
  if (!fp) return fail(DT_E_IO, std::string("could not open ") + filename);
  fwrite(png.data(), 1, png.size(), fp);
  fclose(fp);
  return DT_OK;
}

}  // extern "C"

extern "C" int dt_debug_counters(const dt_scene* sc, uint64_t* out, int32_t n)
{
  if (!sc || !out || n < 0 || n > DT_N_STAMPS) return fail(DT_E_INVALID, "bad arguments");
  if (!sc->uploaded) return fail(DT_E_INVALID, "scene not uploaded (dt_scene_upload)");
  std::vector<unsigned long long> h(ST_N + 1 + DT_N_STAMPS);
  HIPCHK(hipMemcpy(h.data(), sc->d_stats + sc->last_parity * STATS1, sizeof(unsigned long long) * h.size(),
                   hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i) out[i] = h[ST_N + 1 + i];
  return DT_OK;
}

extern "C" int64_t dt_debug_item_costs(const dt_scene* sc, uint32_t* out, int64_t n)
{
  if (!sc || (n > 0 && !out) || n < 0) return (int64_t)fail(DT_E_INVALID, "bad arguments");
  if (!sc->d_item_cost || sc->item_cost_n == 0) return 0;
  const int64_t m = n < sc->item_cost_n ? n : sc->item_cost_n;
  if (m > 0) {
    if (hipDeviceSynchronize() != hipSuccess) return (int64_t)fail(DT_E_NO_DEVICE, "hipDeviceSynchronize");
    if (hipMemcpy(out, sc->d_item_cost, sizeof(uint32_t) * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess)
      return (int64_t)fail(DT_E_NO_DEVICE, "hipMemcpy");
  }
  return sc->item_cost_n;
}

extern "C" int dt_debug_normalize(const double* in, double* out, int64_t n)
{
  if (!in || !out || n < 0 || n > (int64_t)1 << 28) return fail(DT_E_INVALID, "bad arguments");
  if (n == 0) return DT_OK;
  int dev_count = 0;
  if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count < 1) return fail(DT_E_NO_DEVICE, "no HIP device");
  const size_t bytes = (size_t)n * 3 * sizeof(double);
  double *din = nullptr, *dout = nullptr;
  if (hipMalloc((void**)&din, bytes) != hipSuccess) return fail(DT_E_OOM, "hipMalloc");
  if (hipMalloc((void**)&dout, bytes) != hipSuccess) {
    (void)hipFree(din);
    return fail(DT_E_OOM, "hipMalloc");
  }
  hipError_t e = hipMemcpy(din, in, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = dt_launch_normalize(din, dout, n, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(din);
  (void)hipFree(dout);
  if (e != hipSuccess) return fail(DT_E_NO_DEVICE, std::string("HIP: ") + hipGetErrorString(e));
  return DT_OK;
}
