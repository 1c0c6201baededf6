// host_bvh.cpp — the reference's BVH builder (helpers.h:330-472, BoundingVolume ctor
// geometry.cpp:2632-2655), reproduced topology-for-topology, then flattened into the
// device's traversal order.
//
// Why the same topology: the reference gathers the shapes of every hit leaf in stack
// order and keeps the FIRST of equal-t hits (strict <, cpp:527), and the Checkerboard
// edge-on path reuses the previous shape's t (Q16) — both depend on the order shapes are
// tested, which is fixed by the tree. Flattening in the reference's pop order (pre-order,
// last child first) with skip links lets the kernel visit shapes in exactly that order
// without a stack.
#include "host_internal.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <memory>
#include <vector>

using namespace dtm;

namespace dth {

namespace {

struct BV {
  std::vector<std::unique_ptr<BV>> nodes;
  std::vector<int> indices;
  bool leaf = false;
  V3 lb, ub;
};

struct Builder {
  const dt_shape_desc* shapes;
  float c_isect, c_trav;

  double center(int i, int axis) const { return shapes[i].center[axis]; }

  // BoundingVolume(indices, shapes, leaf): FLT_MAX / FLT_MIN init (Q18), setBounds, ±1e-2
  std::unique_ptr<BV> make(const std::vector<int>& inds, bool is_leaf) const
  {
    auto b = std::make_unique<BV>();
    b->indices = inds;
    b->leaf = is_leaf;
    V3 lb = v3(FLT_MAX, FLT_MAX, FLT_MAX), ub = v3(FLT_MIN, FLT_MIN, FLT_MIN);
    for (int ind : inds) {
      V3 l, u;
      shape_bounds(shapes[ind], l, u);
      lb = cmin(lb, l);
      ub = cmax(ub, u);
    }
    b->lb = sub(lb, v3(1e-2, 1e-2, 1e-2));
    b->ub = add(ub, v3(1e-2, 1e-2, 1e-2));
    return b;
  }

  // helpers.h:330-361
  void bounds(const std::vector<int>& inds, double x[2], double y[2], double z[2]) const
  {
    x[0] = FLT_MAX; x[1] = FLT_MIN;
    y[0] = FLT_MAX; y[1] = FLT_MIN;
    z[0] = FLT_MAX; z[1] = FLT_MIN;
    for (int ind : inds) {
      if (center(ind, 0) < x[0]) x[0] = center(ind, 0);
      if (center(ind, 0) > x[1]) x[1] = center(ind, 0);
      if (center(ind, 1) < y[0]) y[0] = center(ind, 1);
      if (center(ind, 1) > y[1]) y[1] = center(ind, 1);
      if (center(ind, 2) < z[0]) z[0] = center(ind, 2);
      if (center(ind, 2) > z[1]) z[1] = center(ind, 2);
    }
  }

  // helpers.h:249-272 (Lomuto, float pivot)
  void order(std::vector<int>& inds, int axis, int low, int high) const
  {
    if (low < high) {
      float pivot = (float)center(inds[high], axis);
      int i = low;
      for (int j = low; j < high; j++) {
        if (center(inds[j], axis) < pivot) {
          std::swap(inds[j], inds[i]);
          i++;
        }
      }
      std::swap(inds[i], inds[high]);
      order(inds, axis, low, i - 1);
      order(inds, axis, i + 1, high);
    }
  }

  // centroid bounds of a run of shapes, grown one shape at a time exactly as getBounds scans
  // (helpers.h:330-361: FLT_MAX / FLT_MIN init, strict < and >), and getSAH's per-half cost
  // (helpers.h:364-378) of them
  struct Box6 {
    double x[2], y[2], z[2];
    static Box6 empty()
    {
      Box6 b;
      b.x[0] = FLT_MAX; b.x[1] = FLT_MIN;
      b.y[0] = FLT_MAX; b.y[1] = FLT_MIN;
      b.z[0] = FLT_MAX; b.z[1] = FLT_MIN;
      return b;
    }
    Box6 with(const Builder& B, int ind) const
    {
      Box6 b = *this;
      if (B.center(ind, 0) < b.x[0]) b.x[0] = B.center(ind, 0);
      if (B.center(ind, 0) > b.x[1]) b.x[1] = B.center(ind, 0);
      if (B.center(ind, 1) < b.y[0]) b.y[0] = B.center(ind, 1);
      if (B.center(ind, 1) > b.y[1]) b.y[1] = B.center(ind, 1);
      if (B.center(ind, 2) < b.z[0]) b.z[0] = B.center(ind, 2);
      if (B.center(ind, 2) > b.z[1]) b.z[1] = B.center(ind, 2);
      return b;
    }
    float cost(float base_area, size_t count) const
    {
      return (float)((((x[1] - x[0]) * (y[1] - y[0]) * 2 + (x[1] - x[0]) * (z[1] - z[0]) * 2) +
                      (y[1] - y[0]) * (z[1] - z[0]) * 2) /
                     base_area * (double)count);
    }
  };

  // helpers.h:381-472
  std::unique_ptr<BV> generate(std::vector<int> indices) const
  {
    if (indices.size() == 1) return make(indices, true);
    double x[2], y[2], z[2];
    bounds(indices, x, y, z);
    double extent[3] = {x[1] - x[0], y[1] - y[0], z[1] - z[0]};
    int axis = 0;
    if (extent[1] > extent[0]) axis = extent[2] > extent[1] ? 2 : 1;
    else if (extent[2] > extent[0]) axis = 2;
    if (extent[axis] < 1e-3) return make(indices, true);
    order(indices, axis, 0, (int)indices.size() - 1);
    auto tmp = make(indices, false);
    const size_t n = indices.size();
    if (n == 2) {
      tmp->nodes.push_back(generate(std::vector<int>(1, indices[0])));
      tmp->nodes.push_back(generate(std::vector<int>(1, indices[1])));
      return tmp;
    }
    if (n == 3) {
      tmp->nodes.push_back(generate(std::vector<int>(1, indices[0])));
      tmp->nodes.push_back(generate(std::vector<int>(indices.begin() + 1, indices.end())));
      return tmp;
    }
    if (n == 4) {
      tmp->nodes.push_back(generate(std::vector<int>(indices.begin(), indices.begin() + 2)));
      tmp->nodes.push_back(generate(std::vector<int>(indices.begin() + 2, indices.end())));
      return tmp;
    }
    float base_area = (float)((extent[0] * extent[1] * 2 + extent[1] * extent[2] * 2) + extent[0] * extent[2] * 2);
    float sah_cost = FLT_MAX;
    size_t slice = 1;
    // The reference evaluates getSAH(v1, v2) for every split i, re-scanning both halves (O(n^2) per
    // node: 62 ms of C4's host build). The centroid bounds of a half are mins and maxes, exact and
    // independent of scan order, so prefix and suffix bounds give every split the same doubles, the
    // same cost expression and the same float -- the same slice, in O(n).
    std::vector<Box6> pre(n + 1), suf(n + 1);
    pre[0] = Box6::empty();
    for (size_t i = 0; i < n; ++i) pre[i + 1] = pre[i].with(*this, indices[i]);
    suf[n] = Box6::empty();
    for (size_t i = n; i-- > 0;) suf[i] = suf[i + 1].with(*this, indices[i]);
    for (size_t i = 1; i < n - 1; i++) {
      float c = c_trav + c_isect * (pre[i].cost(base_area, i) + suf[i].cost(base_area, n - i));
      if (c < sah_cost) {
        sah_cost = c;
        slice = i;
      }
    }
    if (c_isect * (float)n <= sah_cost) return make(indices, true);
    tmp->nodes.push_back(generate(std::vector<int>(indices.begin(), indices.begin() + slice)));
    tmp->nodes.push_back(generate(std::vector<int>(indices.begin() + slice, indices.end())));
    return tmp;
  }
};

// pre-order, last child first (the reference's stack pop order, cpp:496-510)
void flatten(const BV* b, int depth, FlatBVH& out)
{
  int me = (int)out.nodes.size();
  out.nodes.emplace_back();
  out.depth.push_back(depth);
  dtd::DNode& nd = out.nodes[me];
  nd.lb[0] = b->lb.x; nd.lb[1] = b->lb.y; nd.lb[2] = b->lb.z;
  nd.ub[0] = b->ub.x; nd.ub[1] = b->ub.y; nd.ub[2] = b->ub.z;
  // the reference treats a node as a leaf only if it has indices (cpp:502)
  nd.leaf = (b->leaf && !b->indices.empty()) ? 1 : 0;
  nd.first = (int)out.leaf_idx.size();
  nd.count = nd.leaf ? (int)b->indices.size() : 0;
  if (nd.leaf) out.leaf_idx.insert(out.leaf_idx.end(), b->indices.begin(), b->indices.end());
  out.n_children.push_back(b->leaf ? 0 : (int)b->nodes.size());
  if (!b->leaf)
    for (int c = (int)b->nodes.size() - 1; c >= 0; --c) flatten(b->nodes[c].get(), depth + 1, out);
  out.nodes[me].skip = (int)out.nodes.size();
}

}  // namespace

void shape_bounds(const dt_shape_desc& sh, V3& lb, V3& ub)
{
  switch (sh.type) {
    case DT_SHAPE_SPHERE: {  // geometry.cpp:206-210
      V3 c = v3a(sh.v[0]);
      lb = v3(c.x - sh.radius, c.y - sh.radius, c.z - sh.radius);
      ub = v3(c.x + sh.radius, c.y + sh.radius, c.z + sh.radius);
      return;
    }
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER: {  // geometry.cpp:427-431
      V3 c1 = v3a(sh.v[0]), c2 = v3a(sh.v[1]);
      double r = sh.radius;
      lb = cmin(v3(c1.x - r, c1.y - r, c1.z - r), v3(c2.x - r, c2.y - r, c2.z - r));
      ub = cmax(v3(c1.x + r, c1.y + r, c1.z + r), v3(c2.x + r, c2.y + r, c2.z + r));
      return;
    }
    default: {  // Triangle 596-602, Rectangle 761-770, RectPrismV2 922-941
      // RectPrismV2 / RectPrismWithCylinder (RectPrism::getBounds, geometry.cpp:922-941, 1382-1401): 8 vertices
      int n = sh.type == DT_SHAPE_TRIANGLE ? 3 : ((sh.type == DT_SHAPE_RECTPRISM_V2 || sh.type == DT_SHAPE_RECTPRISM_CYL) ? 8 : 4);
      V3 mn = cmin(v3a(sh.v[0]), v3a(sh.v[1])), mx = cmax(v3a(sh.v[0]), v3a(sh.v[1]));
      for (int k = 2; k < n; ++k) {
        mn = cmin(mn, v3a(sh.v[k]));
        mx = cmax(mx, v3a(sh.v[k]));
      }
      lb = mn;
      ub = mx;
      return;
    }
  }
}

void build_bvh(const dt_scene_desc& d, const dt_globals& g, FlatBVH& out)
{
  out = FlatBVH();
  if (d.n_shapes < 1) return;
  Builder b{d.shapes, g.c_isect, g.c_trav};
  std::vector<int> range(d.n_shapes);
  for (int i = 0; i < d.n_shapes; ++i) range[i] = i;
  auto root = b.generate(range);
  flatten(root.get(), 0, out);
}

}  // namespace dth
