// host_hull.cpp — convex-hull separation tests for the host's exact culling (shadow-grid lists,
// umbra cells, primary-ray lists): the points whose hull holds every surface point a shape's float
// intersection tests can report, and a GJK distance test whose answer is checked exactly.
#include <algorithm>
#include <array>
#include <cmath>
#include <vector>

#include "host_internal.h"

namespace dth {

// Points whose convex hull holds everything intersectShadow can report a hit on: parallelogram
// corners of rectangle / checkerboard / prism-face tests, triangle vertices. A moving named
// rectangle (blur passes, |shift| <= ypad in y) adds its shifted corners. false: no planar hull
// (spheres, cylinders).
bool shape_hull_points(const dtd::DShapeHdr& h, const double* g, double ypad, std::vector<std::array<double, 3>>& pts,
                       bool up_only)
{
  auto para = [&](const double* R, double yp) {
    for (int k = 0; k < 4; ++k) {
      std::array<double, 3> p;
      for (int a = 0; a < 3; ++a)
        p[a] = R[dtd::R_A + a] + ((k & 1) ? R[dtd::R_V1N + a] * R[dtd::R_LEN1] : 0.0) +
               ((k & 2) ? R[dtd::R_V2N + a] * R[dtd::R_LEN2] : 0.0);
      if (yp > 0) {
        pts.push_back({p[0], p[1] - yp, p[2]});
        pts.push_back({p[0], p[1] + yp, p[2]});
      } else {
        pts.push_back(p);
      }
    }
  };
  switch (h.type) {
    case DT_SHAPE_RECTANGLE:
      if (h.flags & DT_F_NAMED_RECT) {   // shifted copies: rect_hit_raw on A, B, D (parallelogram A, B, D, B + D - A)
        const double* A = g + dtd::RC_A;
        const double* B = g + dtd::RC_B;
        const double* D = g + dtd::RC_D;
        const double q[4][3] = {{A[0], A[1], A[2]}, {B[0], B[1], B[2]}, {D[0], D[1], D[2]},
                                {B[0] + D[0] - A[0], B[1] + D[1] - A[1], B[2] + D[2] - A[2]}};
        for (const auto& p : q) {   // non-negative shifts (up_only): [p, p + ypad]
          pts.push_back({p[0], p[1] - (up_only ? 0.0 : ypad), p[2]});
          pts.push_back({p[0], p[1] + ypad, p[2]});
        }
      }
      para(g + dtd::RC_R, 0.0);
      return true;
    case DT_SHAPE_CHECKERBOARD:
    case DT_SHAPE_CHECKERBOARD_HOLE:
      para(g + dtd::CK_R, 0.0);
      return true;
    case DT_SHAPE_TRIANGLE: {
      const double* A = g + dtd::TR_A;
      const double* r1 = g + dtd::TR_R1;
      const double* r2 = g + dtd::TR_R2;
      pts.push_back({A[0], A[1], A[2]});
      pts.push_back({A[0] + r1[0], A[1] + r1[1], A[2] + r1[2]});
      pts.push_back({A[0] + r2[0], A[1] + r2[1], A[2] + r2[2]});
      return true;
    }
    case DT_SHAPE_RECTPRISM_V2:
      for (int f = 0; f < 6; ++f) para(g + dtd::PR_F + f * dtd::R_SIZE, 0.0);
      return true;
  }
  return false;
}

namespace {

// closest point to the origin on triangle (a, b, c) (Ericson, Real-Time Collision Detection 5.1.5);
// W is reduced to the feature (vertex, edge or face) holding it
P3 closest_tri(P3* W, int& n)
{
  const P3 a = W[0], b = W[1], c = W[2];
  const P3 ab = sub3(b, a), ac = sub3(c, a);
  const P3 ap = {-a[0], -a[1], -a[2]};
  const double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { n = 1; return a; }
  const P3 bp = {-b[0], -b[1], -b[2]};
  const double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { W[0] = b; n = 1; return b; }
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) { n = 2; W[1] = b; return mad3(a, ab, d1 / (d1 - d3)); }
  const P3 cp = {-c[0], -c[1], -c[2]};
  const double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { W[0] = c; n = 1; return c; }
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) { n = 2; W[1] = c; return mad3(a, ac, d2 / (d2 - d6)); }
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    n = 2; W[0] = b; W[1] = c;
    return mad3(b, sub3(c, b), (d4 - d3) / ((d4 - d3) + (d5 - d6)));
  }
  const double den = 1.0 / (va + vb + vc);
  return mad3(mad3(a, ab, vb * den), ac, vc * den);
}

// closest point to the origin on the simplex W (1-4 points), reducing W; false: the origin lies
// inside the tetrahedron
bool closest_simplex(P3* W, int& n, P3& v)
{
  if (n == 1) { v = W[0]; return true; }
  if (n == 2) {
    const P3 ab = sub3(W[1], W[0]);
    const double l2 = dot3(ab, ab);
    const double t = l2 > 0 ? -dot3(W[0], ab) / l2 : 0.0;
    if (t <= 0) { n = 1; v = W[0]; }
    else if (t >= 1) { W[0] = W[1]; n = 1; v = W[0]; }
    else v = mad3(W[0], ab, t);
    return true;
  }
  if (n == 3) { v = closest_tri(W, n); return true; }
  // tetrahedron: the faces whose plane separates the origin from the opposite vertex
  static const int F[4][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {1, 3, 2, 0}};
  double best = INFINITY;
  P3 bv{};
  P3 bw[3];
  int bn = 0;
  bool outside_any = false;
  for (const auto& f : F) {
    const P3 a = W[f[0]], b = W[f[1]], c = W[f[2]], d = W[f[3]];
    const P3 ab = sub3(b, a), ac = sub3(c, a);
    const P3 nrm = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2], ab[0] * ac[1] - ab[1] * ac[0]};
    const double so = -dot3(nrm, a), sd = dot3(nrm, sub3(d, a));
    if (!(so * sd < 0)) continue;   // origin on the same side as d (or degenerate)
    outside_any = true;
    P3 w[3] = {a, b, c};
    int m = 3;
    const P3 p = closest_tri(w, m);
    const double d2 = dot3(p, p);
    if (d2 < best) {
      best = d2; bv = p; bn = m;
      for (int k = 0; k < m; ++k) bw[k] = w[k];
    }
  }
  if (!outside_any) return false;
  n = bn;
  for (int k = 0; k < n; ++k) W[k] = bw[k];
  v = bv;
  return true;
}

}  // namespace

// gap between the projections of the hulls of A and B on direction v (min over A minus max over B),
// in units of |v|
double hull_gap(const P3* A, int na, const P3* B, int nb, const P3& v)
{
  const double vn = std::sqrt(dot3(v, v));
  if (!(vn > 0) || !std::isfinite(vn)) return -INFINITY;
  double amin = INFINITY, bmax = -INFINITY;
  for (int k = 0; k < na; ++k) amin = std::min(amin, dot3(A[k], v));
  for (int k = 0; k < nb; ++k) bmax = std::max(bmax, dot3(B[k], v));
  return (amin - bmax) / vn;
}

// Are the convex hulls of A and B at least `margin` apart? GJK on A - B proposes the direction,
// then the gap between the projections of A and B on it is checked exactly. `hint`: a direction
// tried first (the last one of a neighbouring test); it returns the direction GJK ended with.
bool hulls_separated(const P3* A, int na, const P3* B, int nb, double margin, P3& hint)
{
  if (hull_gap(A, na, B, nb, hint) > margin) return true;
  auto support = [&](const P3& d) {   // support point of A - B in direction d
    int ia = 0, ib = 0;
    double sa = -INFINITY, sb = INFINITY;
    for (int k = 0; k < na; ++k) { const double s = dot3(A[k], d); if (s > sa) { sa = s; ia = k; } }
    for (int k = 0; k < nb; ++k) { const double s = dot3(B[k], d); if (s < sb) { sb = s; ib = k; } }
    return sub3(A[ia], B[ib]);
  };
  P3 v = sub3(A[0], B[0]);
  P3 W[4];
  int n = 0;
  for (int it = 0; it < 48; ++it) {
    const double vv = dot3(v, v);
    if (!(vv > margin * margin)) break;   // the hulls are closer than the margin
    const P3 w = support({-v[0], -v[1], -v[2]});
    if (dot3(v, w) > margin * std::sqrt(vv)) break;   // v already separates with the margin
    if (vv - dot3(v, w) <= 1e-12 * vv) break;         // converged
    W[n++] = w;
    if (!closest_simplex(W, n, v)) break;             // the hulls overlap
  }
  hint = v;
  return hull_gap(A, na, B, nb, v) > margin;   // the exact check along v
}

bool leaf_hull_points(const FlatScene& fs, const dtd::DNodeDev& leaf, int skip_shape, double ypad, std::vector<P3>& out,
                      bool up_only)
{
  out.clear();
  const int nq = (leaf.meta & dtd::DN_SINGLE) ? 1 : (int)leaf.aux;
  for (int q = 0; q < nq; ++q) {
    const int sid = (leaf.meta & dtd::DN_SINGLE) ? (int)leaf.first : fs.bvh.leaf_idx[leaf.first + q];
    if (sid == skip_shape) continue;
    if (sid < 0 || sid >= (int)fs.hdr.size() ||
        !shape_hull_points(fs.hdr[sid], fs.geom.data() + fs.hdr[sid].off, ypad, out, up_only)) {
      out.clear();
      return false;
    }
  }
  return !out.empty();
}

}  // namespace dth
