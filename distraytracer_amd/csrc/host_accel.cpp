// host_accel.cpp — every acceleration structure dt_scene_create uploads, built on the host with
// no device: the reference-topology tree in device layout, the alternative closest-hit tree, the
// motion-blur bump tree and the per-light shadow grid. dt_scene_create uploads the result;
// dt_accel_info (CPU tests, A/B of build options) reports counts and content hashes of it.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host_internal.h"

namespace dth {

bool sg_parse_block(const char* s, int& bx, int& by)
{
  bx = 8;
  by = 4;
  if (!s) return true;
  if (strcmp(s, "0") == 0) {   // per-cell tests only (1 x 1 blocks)
    bx = by = 1;
    return true;
  }
  int x = 0, y = 0;
  char tail = 0;
  if (sscanf(s, "%dx%d%c", &x, &y, &tail) == 2 && x >= 1 && y >= 1) {
    bx = x;
    by = y;
    return true;
  }
  return false;
}

void build_accel(const FlatScene& f, const dt_globals& g, Accel& a, const std::function<void(const char*)>& stage)
{
  a = Accel();
  a.leaf = f.bvh.leaf_idx;
  if (a.leaf.empty()) a.leaf.push_back(0);
  std::vector<dtd::DNodeDev>& dnodes = a.dnodes;
  dnodes.resize(f.bvh.nodes.size());
  for (size_t i = 0; i < dnodes.size(); ++i) {
    const dtd::DNode& n = f.bvh.nodes[i];
    dtd::DNodeDev& o = dnodes[i];
    for (int k = 0; k < 3; ++k) { o.lb[k] = n.lb[k]; o.ub[k] = n.ub[k]; }
    o.skip = n.skip;
    o.meta = n.leaf ? dtd::DN_LEAF : 0u;
    o.first = n.first;
    o.aux = n.count;
    if (n.leaf && n.count == 1) {
      const dtd::DShapeHdr& h = f.hdr[f.bvh.leaf_idx[n.first]];
      o.meta |= dtd::DN_SINGLE | ((uint32_t)h.type << 4) | ((h.flags & 0xffu) << 8);
      o.first = f.bvh.leaf_idx[n.first];
      o.aux = h.off;
    }
  }
  // Alternative traversal tree (host_fasttree.cpp): exact by construction. Every fast walk uses it
  // by default. DT_FAST_TREE: 1 (default) every fast walk, c closest-hit walks only, s shadow walks
  // only, 0 none. Round 1 kept shadow walks on the reference tree (C3 1666 vs 1624 then); since the
  // shadow grid answers nearly every C3 shadow ray, the tree walks left are C4's mesh cells, where
  // the fast tree is 14% faster end to end (1325 vs 1164 Mpixel-samples/s; C3, C2 and the tunnel
  // frames within 0.3%, profiles/r02aa_ab_fasttree.log).
  const char* ft = getenv("DT_FAST_TREE");
  a.ftree_mode = !ft ? 3 : ft[0] == '1' ? 3 : ft[0] == 'c' ? 1 : ft[0] == 's' ? 2 : 0;
  // DT_EYE_ORDER=0: children in SAH order instead of nearer-to-the-camera first
  const char* eo = getenv("DT_EYE_ORDER");
  const double* eye = (eo && eo[0] == '0') ? nullptr : g.eye;
  if (!a.ftree_mode || !build_fast_tree(dnodes, a.fnodes, 0, eye)) a.fnodes.clear();
  stage("fast tree");
  a.n_fnodes = (int)a.fnodes.size();
  a.boxes_ordered = 1;
  for (const auto* v : {&a.dnodes, &a.fnodes})
    for (const dtd::DNodeDev& n : *v)
      for (int k = 0; k < 3; ++k)
        if (!(n.lb[k] <= n.ub[k])) a.boxes_ordered = 0;
  if (a.fnodes.empty()) a.fnodes.push_back(dnodes.empty() ? dtd::DNodeDev() : dnodes[0]);
  // Motion-blur bump tree: leaves padded by the largest |val| of cpp:1108-1135 for these globals
  // (|move_per_frame| d + |accel_t| d^3 over d = frame_sample - frame in [0, frame_range], plus
  // margin for the float evaluation). The device checks every lane's shift against the pad and
  // walks the reference tree when one exceeds it. DT_BUMP_TREE=0 disables it.
  a.bparent = tree_parents(dnodes);
  // every blur shift is >= 0 when move_per_frame, accel_t and frame_range are (cpp:1101-1111):
  // planar leaves then need no padding below (blur_leaf_pad; DT_BUMP_UP=0: +-pad everywhere)
  const char* bu = getenv("DT_BUMP_UP");
  const bool up_only = !(bu && bu[0] == '0') && g.move_per_frame >= 0 && g.accel_t >= 0 && g.frame_range >= 0;
  a.bump_up_only = up_only;
  {
    const char* bt = getenv("DT_BUMP_TREE");
    const double d = fabs((double)g.frame_range) * (1.0 + 1e-3) + 1e-3;
    // DT_BUMP_PAD_SCALE (tests): shrink the pad so that some lanes exceed it and take the fallback
    const char* bps = getenv("DT_BUMP_PAD_SCALE");
    const double pad = (((double)fabsf(g.move_per_frame) * d + (double)fabsf(g.accel_t) * d * d * d) * 1.01 + 1e-6) *
                       (bps ? atof(bps) : 1.0);
    a.bump_pad = (float)pad;
    // every shift is >= 0 when move_per_frame, accel_t and frame_range are (cpp:1101-1111):
    // planar leaves then need no padding below (DT_BUMP_UP=0: the symmetric +-pad of round 1)

    if (!(bt && bt[0] == '0') && g.blur_samples > 0 && pad > 0 && pad < 1e3 && build_fast_tree(dnodes, a.bnodes, pad, eye, up_only))
      a.n_bnodes = (int)a.bnodes.size();
    else
      a.bnodes.clear();
  }
  if (a.bnodes.empty()) a.bnodes.push_back(dnodes.empty() ? dtd::DNodeDev() : dnodes[0]);
  if (a.bparent.empty()) a.bparent.push_back(-1);
  stage("bump tree");
  // RectPrismWithCylinder (geometry.cpp:1653-1790) reports a shadow hit wherever the ray's line
  // crosses its box ahead of the start, past the light included, and a hit on one of its holes can
  // lie outside its box: the exactness arguments of t-culling, of the shadow grid and of the
  // primary lists (an occluder lies on the segment, a hit inside its leaf box) do not hold for it.
  // A scene that holds one walks the trees without culling (DParams::no_cull).
  for (const dtd::DShapeHdr& h : f.hdr)
    if (h.type == DT_SHAPE_RECTPRISM_CYL) a.no_cull = true;
  // shadow grid (host_shadowgrid.cpp); DT_SHADOW_GRID=0: every shadow test walks a tree.
  // Reach 0.25 cells and lists of up to 96 leaves (round 1: 0.5, 48): C3 +0.6%, C2 +0.5%, C4 +0.2%,
  // C5 transition frame 1088 -9%, tunnel frames -2% (profiles/r02bj_ab_reach_cap.log)
  const char* sgv = getenv("DT_SHADOW_GRID");
  const char* sgc = getenv("DT_SG_CELLS");
  const char* sgr = getenv("DT_SG_REACH");
  // Start-side culling (host_shadowgrid.cpp header), DT_SG_START: 0 off, 2 always, default: a second
  // build with it when the first one's lists fit (at most 10% of the cells walk the tree). Where the
  // lists overflow (the C5 transition frames n = 120-139) the shorter lists gain nothing on the
  // device and the tests cost 30% more host time, in the frame that starts the animation.
  const char* sgs = getenv("DT_SG_START");
  const int start_mode = sgs ? atoi(sgs) : 1;
  const double ypad_main = a.n_bnodes > 0 ? (double)a.bump_pad : 0.0;
  if ((sgv && sgv[0] == '0') || a.no_cull ||
      !build_shadow_grid(dnodes, f, a.sg, sgc ? atof(sgc) : 32768.0, sgr ? (float)atof(sgr) : DT_SG_REACH_DEFAULT,
                         ypad_main, up_only, start_mode == 2 ? g.eye : nullptr, (double)g.aperture))
    a.sg = ShadowGrid();
  else if (start_mode == 1) {
    size_t walk = 0, cells = a.sg.cells.size() / 2;
    for (size_t c = 0; c < cells; ++c) walk += a.sg.cells[2 * c + 1] == DT_SG_WALK;
    ShadowGrid s2;
    if (walk <= cells / 10 &&
        build_shadow_grid(dnodes, f, s2, sgc ? atof(sgc) : 32768.0, sgr ? (float)atof(sgr) : DT_SG_REACH_DEFAULT,
                          ypad_main, up_only, g.eye, (double)g.aperture))
      a.sg = std::move(s2);
  }
  for (int l = 0; l < DT_MAX_SGRID; ++l) a.sg.base0[l] = a.sg.base[l];
  // Large blur shifts pad the lists until most cells overflow and walk the tree, pass-0 rays
  // included (C5 frames 1760-1920: 45-70% of the cells). Then an unpadded grid for the pass-0 rays
  // goes after it in the same pools (same cells, other lists; 0-5% of its cells walk).
  // DT_SG_PASS0: 0 never, 1 whenever the lists are padded, default when > 10% of cells walk.
  if (a.sg.ypad > 0 && !a.sg.cells.empty()) {
    size_t walk = 0, cells = a.sg.cells.size() / 2;
    for (size_t c = 0; c < cells; ++c) walk += a.sg.cells[2 * c + 1] == DT_SG_WALK;
    const char* p0 = getenv("DT_SG_PASS0");
    const bool want = p0 ? p0[0] == '1' : walk > cells / 10;
    ShadowGrid g0;
    if (want && build_shadow_grid(dnodes, f, g0, sgc ? atof(sgc) : 32768.0, sgr ? (float)atof(sgr) : DT_SG_REACH_DEFAULT, 0.0) &&
        g0.n_lights == a.sg.n_lights && g0.dim[0] == a.sg.dim[0] && g0.dim[1] == a.sg.dim[1] && g0.dim[2] == a.sg.dim[2]) {
      const uint32_t cell_off = (uint32_t)(a.sg.cells.size() / 2), list_off = (uint32_t)a.sg.list.size();
      for (size_t c = 0; c < g0.cells.size(); c += 2) {
        uint32_t o = g0.cells[c];
        if (g0.cells[c + 1] != DT_SG_WALK) o = (o & DT_SG_UMBRA) | ((o & ~DT_SG_UMBRA) + list_off);
        a.sg.cells.push_back(o);
        a.sg.cells.push_back(g0.cells[c + 1]);
      }
      a.sg.list.insert(a.sg.list.end(), g0.list.begin(), g0.list.end());
      for (int l = 0; l < DT_MAX_SGRID; ++l) a.sg.base0[l] = g0.base[l] >= 0 ? g0.base[l] + (int32_t)cell_off : -1;
      a.sg.umbra_cells += g0.umbra_cells;
    }
  }
  if (getenv("DT_SG_VERBOSE")) {
    size_t cells = a.sg.cells.size() / 2, tree = 0, sum = 0, mx = 0;
    for (size_t c = 0; c < cells; ++c) {
      const uint32_t n = a.sg.cells[2 * c + 1];
      if (n == DT_SG_WALK) { ++tree; continue; }
      sum += n;
      mx = std::max(mx, (size_t)n);
    }
    fprintf(stderr, "shadow grid: lights %d dim %dx%dx%d cells %zu (tree %zu) mean list %.2f max %zu list pool %zu "
            "plane-culled %ld (start-side %ld) umbra cells %ld ypad %g hash %016llx\n",
            a.sg.n_lights, a.sg.dim[0], a.sg.dim[1], a.sg.dim[2], cells, tree,
            cells > tree ? (double)sum / (cells - tree) : 0.0, mx, a.sg.list.size(), a.sg.plane_dropped, a.sg.start_dropped, a.sg.umbra_cells, a.sg.ypad,
            (unsigned long long)sg_hash(a.sg, false));
  }
  stage("shadow grid");
}

// FNV-1a over the cell records and lists in storage order, or (sorted) over each cell's list
// contents only: the second is independent of list order (DT_SG_ORDER) and of how identical lists
// are shared in the pool.
uint64_t sg_hash(const ShadowGrid& sg, bool contents_only)
{
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](uint32_t x) { h = (h ^ x) * 1099511628211ull; };
  if (!contents_only) {
    for (auto x : sg.cells) mix(x);
    for (auto x : sg.list) mix((uint32_t)x);
    return h;
  }
  std::vector<int32_t> tmp;
  for (size_t c = 0; c + 1 < sg.cells.size(); c += 2) {
    const uint32_t off = sg.cells[c] & ~DT_SG_UMBRA, n = sg.cells[c + 1];
    if (n == DT_SG_WALK) { mix(n); continue; }
    if (sg.cells[c] & DT_SG_UMBRA) mix(DT_SG_UMBRA);
    tmp.assign(sg.list.begin() + off, sg.list.begin() + off + n);
    std::sort(tmp.begin(), tmp.end());
    mix(n);
    for (auto x : tmp) mix((uint32_t)x);
  }
  return h;
}

uint64_t nodes_hash(const std::vector<dtd::DNodeDev>& v)
{
  uint64_t h = 1469598103934665603ull;
  for (const dtd::DNodeDev& n : v) {
    const unsigned char* p = (const unsigned char*)&n;
    for (size_t i = 0; i < sizeof(n); ++i) h = (h ^ p[i]) * 1099511628211ull;
  }
  return h;
}

}  // namespace dth
