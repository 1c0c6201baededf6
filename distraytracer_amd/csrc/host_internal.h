// host_internal.h — host-side pieces of libdt (not part of the C ABI).
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <array>
#include <vector>

#include "../../include/dt.h"
#include "dt_math.h"
#include "dt_scene_dev.h"

namespace dth {

struct FlatBVH {
  std::vector<dtd::DNode> nodes;   // traversal order, skip links
  std::vector<int32_t> leaf_idx;
  std::vector<int32_t> depth;
  std::vector<int32_t> n_children;
};

void shape_bounds(const dt_shape_desc& sh, dtm::V3& lb, dtm::V3& ub);
void build_bvh(const dt_scene_desc& d, const dt_globals& g, FlatBVH& out);
// host_fasttree.cpp: same leaves, SAH inner nodes, 16-bit leaf ranks in meta (false: no fast tree)
// ypad > 0: the motion-blur bump tree (leaf y-bounds padded, leaf skip = reference node index)
// eye: children ordered nearer-to-eye first (null: SAH order); the gathered set never depends on it
// up_only: every blur shift is >= 0, so single-shape planar leaves are padded by what their shape
// can reach (host_fasttree.cpp) instead of +-ypad
bool build_fast_tree(const std::vector<dtd::DNodeDev>& ref, std::vector<dtd::DNodeDev>& out, double ypad = 0,
                     const double* eye = nullptr, bool up_only = false);
// the same SAH tree over a subset of the reference's leaves (node indices into ref), for the shadow
// grid's block subtrees: leaves are copies of the reference leaves (skip links local to `out`)
void build_fast_subtree(const std::vector<dtd::DNodeDev>& ref, const std::vector<int32_t>& leaf_nodes,
                        std::vector<dtd::DNodeDev>& out);
// parent of every node of a pre-order skip-link tree (-1 at the root)
std::vector<int32_t> tree_parents(const std::vector<dtd::DNodeDev>& ref);

// host_shadowgrid.cpp: per-light candidate-occluder lists per grid cell (false: no grid)
struct ShadowGrid {
  ShadowGrid() { for (int l = 0; l < DT_MAX_SGRID; ++l) sub_base[l] = -1; }
  int n_lights = 0;                  // lights 0..n_lights-1 (base[l] < 0: that light has none)
  int32_t base[DT_MAX_SGRID] = {};   // first cell record of light l in `cells`
  int32_t base0[DT_MAX_SGRID] = {};  // the same for pass-0 (unshifted) rays: `base`, or an unpadded
                                     // second grid appended to `cells` / `list` (host_accel.cpp)
  int dim[3] = {0, 0, 0};
  float lo[3] = {0, 0, 0}, inv_h[3] = {0, 0, 0};
  float reach = 0.5f;                // a cell's list covers points this many cells outside it
  std::vector<uint32_t> cells;       // (offset into list | DT_SG_UMBRA, count | DT_SG_WALK) per cell
  std::vector<int32_t> list;         // leaf node indices (reference tree)
  double ypad = 0;                   // lists also hold for blur passes with |shift| <= ypad
  // Block subtrees (DT_SG_SUBTREE): for each block of sub_bx x sub_by x sub_bz cells holding a cell that
  // walks the tree, an SAH tree over the leaves whose box meets the block's swept box to the light
  // (the block's list, uncapped). Pass-0 waves whose lanes all lie in one such block walk it instead
  // of the whole tree (C4's mesh cells).
  int sub_bx = 0, sub_by = 0, sub_bz = 1, sub_nbx = 0, sub_nby = 0, sub_nbz = 0;
  int32_t sub_base[DT_MAX_SGRID];        // light l's first block record in sub_blocks (-1: none)
  std::vector<uint32_t> sub_blocks;      // (first node, node count) per block; count 0: none
  std::vector<dtd::DNodeDev> sub_nodes;
  long plane_dropped = 0;            // (leaf, cell) pairs left out by plane culling (diagnostic)
  long start_dropped = 0;            // of those, by start-side culling (diagnostic)
  // start-side culling assumed every ray origin inside this box (the root box and the camera's
  // eye region at build time); a render whose camera leaves it must not use the lists
  // (dt_api.cpp prepare_render)
  bool org_check = false;
  double org_lo[3] = {0, 0, 0}, org_hi[3] = {0, 0, 0};
  long umbra_cells = 0;              // (light, cell) records flagged DT_SG_UMBRA (diagnostic)
};
struct FlatScene;

// host_hull.cpp: convex-hull separation (exact culling of shadow-grid and primary-ray lists)
using P3 = std::array<double, 3>;
inline double dot3(const P3& a, const P3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline P3 sub3(const P3& a, const P3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
inline P3 mad3(const P3& a, const P3& b, double s) { return {a[0] + s * b[0], a[1] + s * b[1], a[2] + s * b[2]}; }
// points whose hull holds every hit a planar shape's float tests can report (moving named
// rectangles: also shifted by +-ypad in y); false for spheres and cylinders
bool shape_hull_points(const dtd::DShapeHdr& h, const double* g, double ypad, std::vector<P3>& pts,
                       bool up_only = false);
// the hull points of a leaf's shapes but `skip_shape`; false (empty) when one has none
bool leaf_hull_points(const FlatScene& fs, const dtd::DNodeDev& leaf, int skip_shape, double ypad, std::vector<P3>& out,
                      bool up_only = false);
// min over A minus max over B of the projections on v, in units of |v|
double hull_gap(const P3* A, int na, const P3* B, int nb, const P3& v);
// are the hulls of A and B more than `margin` apart? (GJK direction, then the exact gap along it;
// `hint`: a direction tried first, returned as the one GJK ended with)
bool hulls_separated(const P3* A, int na, const P3* B, int nb, double margin, P3& hint);

// Blur passes: how far below / above its box a reference leaf's shapes can be hit at any shift
// the frame draws (|shift| <= ypad): +-ypad for spheres, cylinders and leaves of several shapes
// (the bumped box); with non-negative shifts (up_only) a single planar shape is hit on itself up to
// the rounding of its float tests, far inside the 1e-2 leaf padding: [0, ypad] for a moving
// "rectangle", nothing for any other.
inline void blur_leaf_pad(const dtd::DNodeDev& n, double ypad, bool up_only, double& below, double& above)
{
  below = above = ypad;
  if (!up_only || !(n.meta & dtd::DN_SINGLE)) return;
  const int type = (int)((n.meta >> 4) & 15u);
  const uint32_t flags = (n.meta >> 8) & 0xffu;
  if (type == DT_SHAPE_TRIANGLE || type == DT_SHAPE_RECTANGLE || type == DT_SHAPE_RECTPRISM_V2 ||
      type == DT_SHAPE_CHECKERBOARD || type == DT_SHAPE_CHECKERBOARD_HOLE) {
    below = 0;
    above = (flags & DT_F_NAMED_RECT) ? ypad : 0;
  }
}
// cam / cam_r: the camera's eye and aperture radius (start-side culling, host_shadowgrid.cpp header;
// null: off)
bool build_shadow_grid(const std::vector<dtd::DNodeDev>& nodes, const FlatScene& fs, ShadowGrid& g,
                       double target_cells = 32768, float reach = 0.5f, double ypad = 0, bool up_only = false,
                       const double* cam = nullptr, double cam_r = 0);

// device-layout scene produced from a descriptor (host_flatten.cpp)
struct FlatScene {
  FlatBVH bvh;
  std::vector<dtd::DShapeHdr> hdr;
  std::vector<double> geom;
  std::vector<dtd::DMat> mat;
  std::vector<dtd::DLight> lights;
  std::vector<uint8_t> tex;
};
int flatten_scene(const dt_scene_desc& d, const dt_globals& g, FlatScene& out, std::string& err);

// DT_SG_BLOCK: null -> 8x4 (default), "0" -> 1x1 (per-cell tests), "XxY" with X, Y >= 1; false
// (and the default) for anything else
bool sg_parse_block(const char* s, int& bx, int& by);

// host_accel.cpp: everything dt_scene_create uploads besides the flat scene, built without a device
struct Accel {
  std::vector<dtd::DNodeDev> dnodes;   // reference tree, device layout
  std::vector<dtd::DNodeDev> fnodes;   // alternative closest-hit tree (1 dummy node when n_fnodes == 0)
  std::vector<dtd::DNodeDev> bnodes;   // motion-blur bump tree (1 dummy node when n_bnodes == 0)
  std::vector<int32_t> bparent;        // parent of every reference node
  std::vector<int32_t> leaf;           // leaf_idx (never empty)
  int n_fnodes = 0, n_bnodes = 0;
  float bump_pad = 0;
  bool bump_up_only = false;           // every blur shift >= 0 (blur_leaf_pad)
  bool no_cull = false;                // a RectPrismWithCylinder: no t-culling, no shadow grid (DParams::no_cull)
  int ftree_mode = 0;
  int boxes_ordered = 0;
  ShadowGrid sg;
};
void build_accel(const FlatScene& f, const dt_globals& g, Accel& a,
                 const std::function<void(const char*)>& stage = [](const char*) {});
uint64_t sg_hash(const ShadowGrid& sg, bool contents_only);
uint64_t nodes_hash(const std::vector<dtd::DNodeDev>& v);

// host_primlists.cpp: per pixel-block candidate leaves (fast-tree node indices, sorted by the
// smallest ray parameter they can be reached at) for the primary rays' closest hit
struct PrimLists {
  int block = 0, nbx = 0, nby = 0;
  std::vector<uint32_t> cells;   // (first entry, count) per block
  std::vector<uint32_t> list;    // (fast-tree node, float bits of t_near) per entry
};
// hulls: per tree node, the leaf's shape hull points (host_hull.cpp; empty: never culled), or null;
// SB: blocks per super-block side
bool build_primary_lists(const std::vector<dtd::DNodeDev>& fnodes, int n_fnodes, const dtd::DParams& P, int B,
                         PrimLists& out, const std::vector<std::vector<P3>>* hulls = nullptr, int SB = 8);

// camera / params (host_flatten.cpp)
int fill_params(const dt_globals& g, int frame, const dt_tiles* tiles, dtd::DParams& P, std::string& err);
int fill_sky_params(const dt_globals& g, float frame, const dt_tiles* tiles, dtd::DParams& P, std::string& err);
std::vector<float> cloud_z_steps(const dt_globals& g);

void set_error(const std::string& e);

}  // namespace dth
