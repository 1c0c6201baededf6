// host_fasttree.cpp — the traversal tree the device walks for ordinary waves.
//
// Why a second tree can stand in for the reference's (helpers.h:330-472): the reference gathers a
// leaf iff its own box and every ancestor box pass BoundingVolume::intersect
// (geometry.cpp:2657-2740). Every ancestor box contains its descendants' boxes (setBounds over all
// of the subtree's shapes, geometry.cpp:2642-2655), and for a finite ray the slab test is monotone
// in the bounds: a larger box gives entries <= and exits >= those of a box inside it, the rounding
// to float included. So a leaf whose own box passes always has passing ancestors, and the gathered
// set is exactly {leaves whose own box passes}, whatever hierarchy sits above the leaves. This
// tree keeps the reference's leaves (same boxes, same shape lists) under new inner nodes (binned
// SAH over the leaf boxes, each inner box the exact union of its leaves), so it gathers the same
// leaves with fewer visits. Order only matters for the closest-hit tie rule (strict <, first in
// the reference's gather order): every leaf carries its rank in that order and the device breaks
// equal-t ties by rank. Axis-parallel rays (isinf branch) are not monotone: those waves walk the
// reference tree.
//
// Motion-blur passes (bumpBVH, helpers.h:530-552) pad every LEAF box by the sample's shift in y
// and leave the inner boxes alone, so the gathered set there is {leaves whose bumped box passes
// and whose reference ancestors all pass}. The bump tree (ypad > 0) holds the same leaves with
// their y-bounds padded by the largest |shift| the frame can draw, under SAH inner nodes: every
// bumped leaf box and every shifted "rectangle" lies inside its padded leaf box, so a wave-uniform
// walk over it reaches every leaf the reference could gather. At such a leaf the device decides
// the reference's predicate exactly: the bumped box test, and the ancestors -- implied when the
// unbumped leaf box passes (containment + monotonicity, as above), tested one by one up the
// reference tree (tree_parents) otherwise. Leaves keep their reference index in `skip`.
#include <algorithm>
#include <cmath>
#include <vector>

#include "host_internal.h"

namespace dth {

namespace {

struct LeafRef {
  double lb[3], ub[3], c[3];
  int node;   // index of the leaf in the reference's flattened tree
  int rank;   // its position in the reference's gather order
};

double area(const double lb[3], const double ub[3])
{
  double d0 = ub[0] - lb[0], d1 = ub[1] - lb[1], d2 = ub[2] - lb[2];
  return 2 * (d0 * d1 + d1 * d2 + d2 * d0);
}

struct Builder {
  const std::vector<dtd::DNodeDev>& ref;   // reference tree, device format
  double ypad;                             // bump tree: leaf boxes padded by this in y
  const double* eye;                       // children nearer to it first (null: SAH order)
  std::vector<LeafRef> leaves;
  std::vector<dtd::DNodeDev> out;

  Builder(const std::vector<dtd::DNodeDev>& r, double yp, const double* e) : ref(r), ypad(yp), eye(e) {}

  // squared distance from the eye to the box of ids[lo, hi)
  double eye_dist2(const std::vector<int>& ids, int lo, int hi) const
  {
    double lb[3], ub[3], d2 = 0;
    box_of(ids, lo, hi, lb, ub);
    for (int a = 0; a < 3; ++a) {
      const double d = eye[a] < lb[a] ? lb[a] - eye[a] : eye[a] > ub[a] ? eye[a] - ub[a] : 0.0;
      d2 += d * d;
    }
    return d2;
  }

  void box_of(const std::vector<int>& ids, int lo, int hi, double lb[3], double ub[3]) const
  {
    for (int a = 0; a < 3; ++a) { lb[a] = INFINITY; ub[a] = -INFINITY; }
    for (int k = lo; k < hi; ++k)
      for (int a = 0; a < 3; ++a) {
        lb[a] = std::min(lb[a], leaves[ids[k]].lb[a]);
        ub[a] = std::max(ub[a], leaves[ids[k]].ub[a]);
      }
  }

  int build(std::vector<int>& ids, int lo, int hi)
  {
    const int me = (int)out.size();
    out.emplace_back();
    if (hi - lo == 1) {
      const LeafRef& L = leaves[ids[lo]];
      dtd::DNodeDev nd = ref[L.node];
      nd.meta = (nd.meta & 0xffffu) | ((uint32_t)L.rank << 16);
      nd.skip = me + 1;
      if (ypad > 0) {   // bump tree: padded box, skip = the leaf's index in the reference tree
        for (int a = 0; a < 3; ++a) { nd.lb[a] = L.lb[a]; nd.ub[a] = L.ub[a]; }
        nd.skip = L.node;
      }
      out[me] = nd;
      return me;
    }
    // SAH sweep on each axis over the leaf-box centroids
    int best_axis = 0, best_split = lo + (hi - lo) / 2;
    double best_cost = INFINITY;
    std::vector<double> right_area(hi - lo + 1);
    for (int axis = 0; axis < 3; ++axis) {
      std::sort(ids.begin() + lo, ids.begin() + hi, [&](int a, int b) {
        if (leaves[a].c[axis] != leaves[b].c[axis]) return leaves[a].c[axis] < leaves[b].c[axis];
        return leaves[a].rank < leaves[b].rank;
      });
      double rl[3] = {INFINITY, INFINITY, INFINITY}, ru[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int k = hi - 1; k > lo; --k) {
        for (int a = 0; a < 3; ++a) {
          rl[a] = std::min(rl[a], leaves[ids[k]].lb[a]);
          ru[a] = std::max(ru[a], leaves[ids[k]].ub[a]);
        }
        right_area[k - lo] = area(rl, ru);
      }
      double ll[3] = {INFINITY, INFINITY, INFINITY}, lu[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int k = lo; k < hi - 1; ++k) {
        for (int a = 0; a < 3; ++a) {
          ll[a] = std::min(ll[a], leaves[ids[k]].lb[a]);
          lu[a] = std::max(lu[a], leaves[ids[k]].ub[a]);
        }
        const double cost = area(ll, lu) * (k - lo + 1) + right_area[k + 1 - lo] * (hi - k - 1);
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = axis;
          best_split = k + 1;
        }
      }
    }
    std::sort(ids.begin() + lo, ids.begin() + hi, [&](int a, int b) {
      if (leaves[a].c[best_axis] != leaves[b].c[best_axis]) return leaves[a].c[best_axis] < leaves[b].c[best_axis];
      return leaves[a].rank < leaves[b].rank;
    });
    dtd::DNodeDev nd;
    box_of(ids, lo, hi, nd.lb, nd.ub);
    nd.meta = 0;
    nd.first = 0;
    nd.aux = 0;
    out[me] = nd;
    // the walk visits the first child first: with an eye, the nearer one (camera rays then find
    // their closest hit early and cull the boxes behind it). Order never changes the result.
    if (eye && eye_dist2(ids, best_split, hi) < eye_dist2(ids, lo, best_split)) {
      build(ids, best_split, hi);
      build(ids, lo, best_split);
    } else {
      build(ids, lo, best_split);
      build(ids, best_split, hi);
    }
    out[me].skip = (int)out.size();
    return me;
  }
};

}  // namespace

// ref: the reference tree in device format (pre-order, last child first, skip links).
// Returns false (and leaves `out` empty) when the tree cannot carry 16-bit leaf ranks.
bool build_fast_tree(const std::vector<dtd::DNodeDev>& ref, std::vector<dtd::DNodeDev>& out, double ypad,
                     const double* eye, bool up_only)
{
  out.clear();
  Builder b(ref, ypad, eye);
  for (size_t i = 0; i < ref.size(); ++i) {
    if (!(ref[i].meta & dtd::DN_LEAF)) continue;
    LeafRef L;
    for (int a = 0; a < 3; ++a) {
      L.lb[a] = ref[i].lb[a];
      L.ub[a] = ref[i].ub[a];
      L.c[a] = 0.5 * (L.lb[a] + L.ub[a]);
    }
    if (ypad > 0) {
      // The leaf box only filters the walk (the device decides the reference's gather exactly at
      // the leaf, bump_leaf_gathered) and bounds its culling, so it must hold every point the
      // leaf's shapes can be hit at. Spheres and cylinders, and leaves of several shapes: the
      // bumped box at the largest shift, +-ypad. With non-negative shifts (up_only) a planar
      // shape's hits lie on it up to the rounding of its float tests, far inside the 1e-2 leaf
      // padding (the argument of the shadow grid's hull culling): a moving "rectangle" within
      // [lb, ub + ypad], any other planar shape within [lb, ub].
      double lo_pad, hi_pad;
      blur_leaf_pad(ref[i], ypad, up_only, lo_pad, hi_pad);
      L.lb[1] = L.lb[1] - lo_pad;
      L.ub[1] = L.ub[1] + hi_pad;
      if (!(L.lb[1] <= L.ub[1])) return false;
    }
    L.node = (int)i;
    L.rank = (int)b.leaves.size();
    b.leaves.push_back(L);
  }
  if (b.leaves.empty() || b.leaves.size() > 0xffff) return false;
  std::vector<int> ids(b.leaves.size());
  for (size_t i = 0; i < ids.size(); ++i) ids[i] = (int)i;
  b.build(ids, 0, (int)ids.size());
  out.swap(b.out);
  return true;
}

void build_fast_subtree(const std::vector<dtd::DNodeDev>& ref, const std::vector<int32_t>& leaf_nodes,
                        std::vector<dtd::DNodeDev>& out)
{
  out.clear();
  Builder b(ref, 0.0, nullptr);
  for (int32_t i : leaf_nodes) {
    LeafRef L;
    for (int a = 0; a < 3; ++a) {
      L.lb[a] = ref[i].lb[a];
      L.ub[a] = ref[i].ub[a];
      L.c[a] = 0.5 * (L.lb[a] + L.ub[a]);
    }
    L.node = i;
    L.rank = (int)b.leaves.size();   // any-hit walks: the order of the leaves does not matter
    b.leaves.push_back(L);
  }
  if (b.leaves.empty()) return;
  std::vector<int> ids(b.leaves.size());
  for (size_t i = 0; i < ids.size(); ++i) ids[i] = (int)i;
  b.build(ids, 0, (int)ids.size());
  out.swap(b.out);
}

std::vector<int32_t> tree_parents(const std::vector<dtd::DNodeDev>& ref)
{
  // pre-order with skip = end of the subtree for inner nodes (a leaf's subtree ends at i + 1)
  std::vector<int32_t> parent(ref.size(), -1);
  std::vector<int> open;
  for (int i = 0; i < (int)ref.size(); ++i) {
    while (!open.empty() && ref[open.back()].skip <= i) open.pop_back();
    parent[i] = open.empty() ? -1 : open.back();
    if (!(ref[i].meta & dtd::DN_LEAF)) open.push_back(i);
  }
  return parent;
}

}  // namespace dth
