// host_shadowgrid.cpp — per-light candidate-occluder lists over a uniform grid of shading-point
// cells, for the shadow test (render_final_project.cpp:806-855).
//
// The reference decides a shadow ray by gathering every leaf whose box the ray passes and
// testing each leaf's shapes with intersectShadow. Only a shape hit at distance t < t_max along
// the segment from isectP + 1e-3·sn counts, and every shape lies inside its leaf box with 1e-2 to
// spare (BoundingVolume pads its bounds, geometry.cpp:2632-2655). For a point or rectangle light
// the segment ends on the light, so a segment starting in cell C lies in the swept box between C
// (widened by the reach below) and the light's box. A leaf whose box misses it cannot occlude any
// segment from C, whatever the
// rounding of the reference's tests (1e-6 relative, far inside the margins below). Each list holds
// the leaves whose box meets the hull. The device tests exactly those leaves (box test, then the
// shapes), which answers as the full gather does. Sphere lights are excluded: their sampleRay
// returns the sampled point itself (Q11), so the "segment" does not end on the light.
//
// Plane culling: a leaf whose box meets the swept box is still left out when every one of its
// shapes is separated from the segments by a plane: all of the widened cell box and the light box
// lie strictly on one side of a rectangle's, checkerboard's or triangle's plane, or on the
// outside of one face plane of a (convex) RectPrismV2. Such a segment cannot cross the plane (a
// prism: cannot reach any face, all of which lie on the inner side), so intersectShadow finds
// nothing in (eps, t_max). The margin (1e-3 plus 1e-6 of the scene's coordinate scale) is orders
// above the rounding of the device's plane parameter (f32 dn, ~1e-7 relative). This drops walls,
// floors and tunnel panels, which the boxes of interior cells meet but no segment crosses.
//
// Hull culling: plane culling only tries the shapes' own planes. A planar shape (rectangle,
// checkerboard, triangle, or a prism's faces) can also be left out when the convex hull of its
// corners keeps a distance above the margin from the convex hull H of the widened cell box and the
// light (its point, or its parallelogram's corners), since every segment of the cell lies in H.
// A reported hit of the reference's float tests lies on the segment (t rounded to f32: ~1e-7 of
// t_max) and inside the shape up to the f32 rounding of its checks, far inside the margin. GJK
// proposes the direction; the separation is then checked exactly along it (the gap between the
// two hulls' projections), so a poorly converged GJK can only keep a leaf, never drop one.
// Spheres and cylinders (round 6) are hull-culled by their axis segment (a point for a sphere):
// the reference's f32 quadratic reports a hit only at a point of the ray within r + delta of the
// axis and inside the axial range (the range check runs on that point), where the discriminant's
// roundings (coefficients rounded once, ~4u B^2) admit a false hit out to
// r + 2u |start - axis|^2 / r and move a true one along the ray by ~sqrt(4u) t, i.e. off the
// surface by ~u t^2 / 2r; delta = 1e-3 + 1e-6 (1 + L^2 / r), L bounding |point - axis end| over
// the hull, covers both with a factor of 8. The segment's points lie in the hull, so a hull that
// keeps r + delta + the usual margin from the axis segment sees no hit (DT_SG_QUAD=0: off).
//
// Umbra cells: a cell all of whose segments to the light cross the inside of one fixed planar
// face (a rectangle that is not a moving "rectangle", a checkerboard without hole, a prism face)
// flagged DT_SG_UMBRA, its list reduced to the face's leaf: a coherent wave in it answers
// "occluded" without testing anything (scattered waves test the one leaf). The proof,
// on the widened cell box P (8 corners) and the light's points Q (1 or 4): every corner of P lies
// on one side of the face's plane and every point of Q on the other, each at least mu' away, and
// the crossing point of every segment (corner of P, point of Q) lies inside the face's checks
// (0 <= v1.(X-A) <= len1, likewise v2) with mu to spare. The segments between the two convex sets
// fill conv(P u Q), whose section by the plane is the hull of those crossing points, so every
// segment crosses the face with margin mu: the reference's rect test reports t in (eps, t_max)
// there whatever its f32 rounding. mu' (>= 2e-3 times the longest segment) also keeps the crossing
// far enough from the start for the reference's leaf-box test from isectP + 1e-3 sray to pass,
// so the reference's gather holds the face's leaf: its shadow test answers "occluded" as well.
//
// Start-side culling: a cell next to a wall contains points of the wall
// itself, so the wall's plane meets the cell box and plane culling keeps it, though no shadow
// segment from a point on the wall (or in front of it) to a light in front of it can cross it. The
// reference's test (rect_plane_hit, geometry.cpp:640-741) starts at o = p + 1e-3 sn and reports a
// hit only at t_final = (float)(((A - o).n) / (float)(sn.n)) in (eps, t_max). Write d(x) = s (n.x - c)
// for the plane (unit n), s the side of the light box, D = min d over the light box (> 0). Then
// d(o) = (1 - l) d(p) + l d(q) with l = 1e-3 / |q - p| <= 1e-3 / Lmax, so d(o) >= min(d(p), 0) +
// 1e-3 D / Lmax; the segment's end q + 1e-3 sn has d >= D - 1e-3; d is linear along the ray, so
// when both ends are positive the ray never reaches the plane in [0, t_max]: the numerator's sign
// (double, exact far below the margins) makes t_final negative when the ray moves away from the
// plane, and beyond t_max by the relative gap d(end) / d(o) >= (D - 1e-3) / maxdist when it moves
// toward it (the float roundings of t_final and t_max are ~1e-7 relative). What remains is a lower
// bound of d(p) over the shading points p that use the cell's list: the points of the widened
// cell box that some closest-hit test reported. Such a p = start + t_f ray has an exact
// counterpart X* = start + t* ray on (or, for a near miss of the float tests, within rho of) the
// shape's box, with |t_f - t*| <= eta |t*|. Class 0, eta 1.25e-7: the plane test of a rectangle
// or checkerboard whose box is flat in one axis. Its normal is that axis exactly (two exact zeros
// in the cross product of two edges, normalised to +-1), so num = (A - start).n is one rounded
// difference and dn = (float)(ray.n) one rounding of an exact product: t_f = t* (1 + e1)(1 + e3) /
// (1 + e2), |e2|, |e3| <= 2^-24, |e1| ~ 2^-53, so |t_f / t* - 1| <= 1.1921e-7; X* lies on the
// box's plane exactly and a near miss of the float checks leaves the box only within the plane
// (rho is not added along the flat axis). Class 2, eta 1e-6: every other planar test (tilted
// planes and prism faces: a float ratio of a double numerator, ~1.2e-7; triangles: a double
// product with a float 1/det, ~2e-7). Class 1, eta 2e-3: the float quadratics of spheres
// and cylinders, whose coefficients A, B, C are each rounded once (u = 2^-24) and whose
// discriminant is formed in double: |d disc| <= 2u B^2 + 2u |4AC| + u |disc| ~ 4u B^2 at tangency,
// so the root moves by sqrt(4u) |B| / 2A ~ 4.9e-4 t (a near miss of the true surface lands at the
// ray's closest approach by the same bound); 2e-3 leaves a factor 4. So |d(p) - d(X*)| <=
// eta |d(X*) - d(start)|, which is at most eta times the span of d over the box of X* and the box
// of ray origins. That box (round 6, second version) holds the camera's eye region and, around
// each shape whose material spawns secondary rays (refl_materials, cpp:574-576), where those rays
// start: the hit point, within eta |X* - start| of the shape's box, plus 1e-3 times the unit
// in / refl_ray or a glossy sample_refl (<= 3080 long). It is computed twice, bounding
// |X* - start| first by the root box's diagonal and then by the first box's; before, it was the
// root box, which C3's window-frame prisms stretch to y = +-1000. p lies within eta times the
// diagonal of the origin box and the shape's box of X*, and within 1e-3 of the start o from which
// the device picks the cell (pad: the sum, + 1e-3). Per cell and class the host keeps the
// bounding box of {shape box + rho} ^ {cell box + pad} over the shapes that meet it (and per
// aligned 8x4x1 block, the union, for the tests on blocks of cells); d's minimum over those
// boxes, less eta times the span, is the bound. A wall is then left out of a cell's list for a
// light when that bound, plus 1e-3 D / Lmax, stays above 1e-7 (1 + scale), D - 1e-3 above 1e-5
// maxdist (|d| over the root box and the eye region), and the cell box keeps 2e-3 from the light
// box. The origin box is recorded: a render whose camera's eye region leaves it walks the trees
// (dt_api.cpp prepare_render). host_accel.cpp builds the lists with it only where they fit
// (DT_SG_START). Only rectangles and checkerboards are tried as the culled shape.
// A tilted rectangle or checkerboard (class 3; C3's ceiling sinks by 0.025 across the room) has a
// box that leaves its plane, so the box bound fails in the cells that hold it. Its own points are
// bounded by its own plane test instead: with num = (A - start).n and dn = (float)(ray.n),
// d(p) = d(start) + dn t_f = d(start) (r - e) + e_num (1 - r)(1 + e), |e| <= 2.0001 * 2^-24, where
// r = e_dn / (dn + e_dn) carries the f64 dot product's error e_dn <= 2^-53 sqrt(3) |ray| and
// |d(start) r| ~ t_f |e_dn| <= 2^-53 sqrt(3) |p - start|: so |d(p)| <= 1.25e-7 |d(start)| +
// 1e-12 (1 + scale) whatever the angle. Per cell and aligned block the host keeps which class-3
// shape is there (none, one, several); where it is the culled shape alone, its points take that
// bound and the box bound serves the other classes. Cylinders' boxes are the axis segment's
// widened by r sqrt(1 - a_k^2) per axis plus eta_1 times the origin box's diagonal (X* lies that
// close to the slab between the caps that p passed), not the caps' centres +- r on every axis.
// Blur shifts that are all >= 0 (up_only) move a "rectangle"'s plane toward the light box on side
// s by at most max(0, s n_y) ypad, not |n_y| ypad.
// With ypad > 0 (blur passes) every "rectangle" moves by up to ypad in y: its box grows by ypad in
// y, and as the culled shape its plane moves by |n_y| ypad (nothing for a wall with a horizontal
// normal), which D and the bound lose. C3: the ceiling, back and side walls leave the lists of the
// boundary cells for the four ceiling lights (263802 -> 195500 list entries; 225677 with the root
// box as the origin box).
//
// Motion blur: with ypad > 0 the lists also serve the blur passes (bumped leaf boxes, "rectangle"
// shapes shifted by |val| <= ypad in y): leaf boxes are padded by ypad in y, and a moving
// rectangle's plane must clear the hull by ypad more.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <thread>
#include <vector>

#include "host_internal.h"

namespace dth {

namespace {

// does the segment p -> q meet the box [lo, hi]? (list ordering only: not a correctness test)
bool segment_meets_box(const double p[3], const double q[3], const double lo[3], const double hi[3])
{
  double t0 = 0.0, t1 = 1.0;
  for (int a = 0; a < 3; ++a) {
    const double d = q[a] - p[a];
    if (std::fabs(d) < 1e-300) {
      if (p[a] < lo[a] || p[a] > hi[a]) return false;
      continue;
    }
    double ta = (lo[a] - p[a]) / d, tb = (hi[a] - p[a]) / d;
    if (ta > tb) std::swap(ta, tb);
    t0 = std::max(t0, ta);
    t1 = std::min(t1, tb);
    if (t0 > t1) return false;
  }
  return true;
}

// cells i in [0, n) whose interval [lo + i h - m, lo + (i+1) h + m], joined with the light
// interval [llo, lhi], meets the leaf interval [a, b]
void cell_range(double lo, double h, int n, double m, double llo, double lhi, double a, double b, int& i0,
                int& i1)
{
  // hull interval: [min(cell_lo, llo), max(cell_hi, lhi)]; meets [a, b] iff
  // min(cell_lo, llo) <= b and max(cell_hi, lhi) >= a
  i0 = 0;
  i1 = n - 1;
  if (llo > b) {   // need cell_lo = lo + i h - m <= b
    const double lim = std::floor((b + m - lo) / h);
    i1 = std::min(i1, (int)std::max(-1.0, std::min((double)n, lim)));
  }
  if (lhi < a) {   // need cell_hi = lo + (i+1) h + m >= a
    const double lim = std::ceil((a - m - lo) / h - 1);
    i0 = std::max(i0, (int)std::min((double)n, std::max(-1.0, lim)));
  }
}

// Does some segment from box C to box L meet box B? Every such segment lies in the swept box
// {(1-t) C + t L : t in [0,1]} (per axis an interval whose ends move linearly in t), which is
// tighter than the box hull of C and L for oblique cells. Per axis the overlap condition is two
// linear inequalities in t; the test passes iff their solution sets meet in [0, 1].
bool swept_meets(const double clo[3], const double chi[3], const double llo[3], const double lhi[3],
                 const double* blo, const double* bhi)
{
  double t0 = 0, t1 = 1;
  const double slack = 1e-9;
  for (int a = 0; a < 3; ++a) {
    // lower end clo + t (llo - clo) <= bhi
    const double d0 = llo[a] - clo[a], r0 = bhi[a] - clo[a];
    if (d0 > 0) t1 = std::min(t1, r0 / d0 + slack);
    else if (d0 < 0) t0 = std::max(t0, r0 / d0 - slack);
    else if (r0 < 0) return false;
    // upper end chi + t (lhi - chi) >= blo
    const double d1 = lhi[a] - chi[a], r1 = blo[a] - chi[a];
    if (d1 < 0) t1 = std::min(t1, r1 / d1 + slack);
    else if (d1 > 0) t0 = std::max(t0, r1 / d1 - slack);
    else if (r1 > 0) return false;
    if (t0 > t1) return false;
  }
  return true;
}

// signed distances to the plane (p0, n) of the points of the boxes [alo, ahi] and [blo, bhi]:
// [mn, mx] (false when n is degenerate)
bool plane_range(const double* p0, const double* n, const double alo[3], const double ahi[3], const double blo[3],
                 const double bhi[3], double& mn, double& mx)
{
  const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  if (!(nn > 0) || !std::isfinite(nn)) return false;
  const double c = n[0] * p0[0] + n[1] * p0[1] + n[2] * p0[2];
  mn = INFINITY;
  mx = -INFINITY;
  for (int k = 0; k < 2; ++k) {
    const double* lo = k ? blo : alo;
    const double* hi = k ? bhi : ahi;
    double smin = -c, smax = -c;
    for (int a = 0; a < 3; ++a) {
      smin += n[a] * (n[a] > 0 ? lo[a] : hi[a]);
      smax += n[a] * (n[a] > 0 ? hi[a] : lo[a]);
    }
    mn = std::min(mn, smin / nn);
    mx = std::max(mx, smax / nn);
  }
  return std::isfinite(mn) && std::isfinite(mx);
}

// no segment between the two boxes can make this shape's intersectShadow true (see the header)
bool shape_separated(const dtd::DShapeHdr& h, const double* g, const double clo[3], const double chi[3],
                     const double llo[3], const double lhi[3], double margin, double ypad)
{
  double mn, mx;
  double m = margin + ((h.flags & DT_F_NAMED_RECT) ? ypad : 0.0);
  switch (h.type) {
    case DT_SHAPE_RECTANGLE: {
      const double* R = g + dtd::RC_R;
      if (h.flags & DT_F_NAMED_RECT) {
        // a shift by s in y moves the plane by s * |n_y| / |n| along its normal (tunnel panels
        // with near-horizontal normals barely move), so that is all the margin it needs
        const double* n = R + dtd::R_N;
        const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (nn > 0) m = margin + ypad * std::fabs(n[1]) / nn * (1 + 1e-9) + 1e-9 * ypad;
      }
      return plane_range(R + dtd::R_A, R + dtd::R_N, clo, chi, llo, lhi, mn, mx) && (mn > m || mx < -m);
    }
    case DT_SHAPE_CHECKERBOARD:
    case DT_SHAPE_CHECKERBOARD_HOLE: {
      const double* R = g + dtd::CK_R;
      return plane_range(R + dtd::R_A, R + dtd::R_N, clo, chi, llo, lhi, mn, mx) && (mn > m || mx < -m);
    }
    case DT_SHAPE_TRIANGLE: {
      const double* r1 = g + dtd::TR_R1;
      const double* r2 = g + dtd::TR_R2;
      const double n[3] = {r1[1] * r2[2] - r1[2] * r2[1], r1[2] * r2[0] - r1[0] * r2[2], r1[0] * r2[1] - r1[1] * r2[0]};
      return plane_range(g + dtd::TR_A, n, clo, chi, llo, lhi, mn, mx) && (mn > m || mx < -m);
    }
    case DT_SHAPE_RECTPRISM_V2: {
      // centroid: mean of the six face centres; a face plane with the hull strictly outside it
      double cen[3] = {0, 0, 0};
      for (int f = 0; f < 6; ++f) {
        const double* R = g + dtd::PR_F + f * dtd::R_SIZE;
        for (int a = 0; a < 3; ++a)
          cen[a] += (R[dtd::R_A + a] + 0.5 * (R[dtd::R_V1N + a] * R[dtd::R_LEN1] + R[dtd::R_V2N + a] * R[dtd::R_LEN2])) / 6;
      }
      for (int f = 0; f < 6; ++f) {
        const double* R = g + dtd::PR_F + f * dtd::R_SIZE;
        const double* A = R + dtd::R_A;
        const double* n = R + dtd::R_N;
        const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (!(nn > 0)) continue;
        const double side = ((cen[0] - A[0]) * n[0] + (cen[1] - A[1]) * n[1] + (cen[2] - A[2]) * n[2]) / nn;
        if (!(std::fabs(side) > 1e-6)) continue;   // flat prism: no inner side
        if (!plane_range(A, n, clo, chi, llo, lhi, mn, mx)) continue;
        if ((side > 0 && mx < -m) || (side < 0 && mn > m)) return true;
      }
      return false;
    }
  }
  return false;
}

}  // namespace

bool build_shadow_grid(const std::vector<dtd::DNodeDev>& nodes, const FlatScene& fs, ShadowGrid& g,
                       double target_cells, float reach, double ypad, bool up_only, const double* cam, double cam_r)
{
  const double t_entry = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  const std::vector<dtd::DLight>& lights = fs.lights;
  g = ShadowGrid();
  for (int l = 0; l < DT_MAX_SGRID; ++l) g.sub_base[l] = -1;
  g.reach = reach;
  g.ypad = ypad;
  if (nodes.empty() || !(nodes[0].lb[0] <= nodes[0].ub[0])) return false;
  std::vector<int> leaves;
  for (size_t i = 0; i < nodes.size(); ++i)
    if (nodes[i].meta & dtd::DN_LEAF) leaves.push_back((int)i);
  // large leaf counts (meshes): the per-leaf cell ranges would cost seconds of host time per
  // scene and the lists would overflow anyway; such scenes walk the tree
  // (DT_SG_MAX_LEAVES overrides the cap, for measurements)
  const char* ml = getenv("DT_SG_MAX_LEAVES");
  if (leaves.empty() || leaves.size() > (ml ? (size_t)atol(ml) : (size_t)4096)) return false;
  // Grid box: where the shading points are. A few giant shapes (C3's window-frame prisms span
  // y in [-996, 1004]) would stretch a box around everything into useless slabs. Per axis the
  // box is the hull of
  //  * the union of the 90% shortest leaf intervals, widened by half its size (where most
  //    shapes are), and
  //  * the union of all leaf intervals but the few giant ones: the fewest longest leaves
  //    (at most max(4, 10%)) whose removal shrinks the union at least 4x (the room; with
  //    thousands of small mesh triangles the first term alone would shrink onto the meshes),
  // within the root box. Points outside the grid walk the tree.
  double lo[3], ext[3], vol = 1;
  for (int a = 0; a < 3; ++a) {
    std::vector<std::pair<double, int>> byext;
    for (int l : leaves) byext.push_back({nodes[l].ub[a] - nodes[l].lb[a], l});
    std::sort(byext.begin(), byext.end());
    const size_t n = byext.size();
    // plo/phi[k]: union of the k shortest leaf intervals
    std::vector<double> plo(n + 1, INFINITY), phi(n + 1, -INFINITY);
    for (size_t k = 0; k < n; ++k) {
      plo[k + 1] = std::min(plo[k], nodes[byext[k].second].lb[a]);
      phi[k + 1] = std::max(phi[k], nodes[byext[k].second].ub[a]);
    }
    const size_t k90 = std::max((size_t)1, std::min(n, (size_t)(0.9 * (double)n) + 1));
    double c0 = plo[k90], c1 = phi[k90];
    const double w = c1 - c0;
    c0 -= 0.5 * w;
    c1 += 0.5 * w;
    size_t keep = n;
    const size_t max_drop = std::max((size_t)4, n / 10);
    for (size_t k = n - 1; k >= 1 && n - k <= max_drop; --k)
      if (phi[n] - plo[n] > 4.0 * (phi[k] - plo[k])) { keep = k; break; }
    c0 = std::max(std::min(c0, plo[keep]), nodes[0].lb[a]);
    c1 = std::min(std::max(c1, phi[keep]), nodes[0].ub[a]);
    if (!(c1 > c0)) return false;
    lo[a] = c0;
    ext[a] = std::max(c1 - c0, 1e-3);
    vol *= ext[a];
  }
  if (!std::isfinite(vol) || vol <= 0) return false;
  const double h = std::cbrt(vol / target_cells);
  double hh[3];
  for (int a = 0; a < 3; ++a) {
    g.dim[a] = std::max(1, std::min(256, (int)std::ceil(ext[a] / h)));
    hh[a] = ext[a] / g.dim[a];
    g.lo[a] = (float)lo[a];
    g.inv_h[a] = (float)(1.0 / hh[a]);
  }
  const int ncell = g.dim[0] * g.dim[1] * g.dim[2];
  // margins: a cell's list serves every shading point within `reach` cells of it (the
  // device checks that reach per lane), plus slack for the f32 cell coordinates (m1); the
  // segment ends 1e-3 past the light sample (m2)
  double scale = 0;
  for (int a = 0; a < 3; ++a) scale = std::max({scale, std::fabs(lo[a]), std::fabs(lo[a] + ext[a])});
  const double m1 = (reach + 0.05) * std::max({hh[0], hh[1], hh[2]}) + 1e-4 * (1 + scale);
  const double m2 = 2e-3 + 1e-4 * (1 + scale);
  const double mplane = 1e-3 + 1e-6 * (1 + scale);
  // leaf boxes, padded in y by where the blur passes can hit their shapes (blur_leaf_pad)
  std::vector<std::array<double, 6>> lbox(nodes.size());
  for (int leaf : leaves) {
    double below = 0, above = 0;
    if (ypad > 0) blur_leaf_pad(nodes[leaf], ypad, up_only, below, above);
    for (int a = 0; a < 3; ++a) {
      lbox[leaf][a] = nodes[leaf].lb[a] - (a == 1 ? below : 0.0);
      lbox[leaf][3 + a] = nodes[leaf].ub[a] + (a == 1 ? above : 0.0);
    }
  }
  // shapes of each leaf (shape ids)
  auto leaf_shapes = [&](int leaf, std::vector<int>& out) {
    out.clear();
    const dtd::DNodeDev& nd = nodes[leaf];
    if (nd.meta & dtd::DN_SINGLE) out.push_back(nd.first);
    else
      for (int64_t q = 0; q < (int64_t)nd.aux; ++q) out.push_back(fs.bvh.leaf_idx[nd.first + q]);
  };
  long dropped = 0;
  std::atomic<long> start_dropped(0);
  const bool timing = getenv("DT_TIMING") != nullptr;
  // start-side culling (header): on when the caller passes the camera (host_accel.cpp decides)
  const bool start_on = cam != nullptr;
  const size_t nshape = fs.hdr.size();
  const int ncell_all = g.dim[0] * g.dim[1] * g.dim[2];
  // |t_f - t*| <= eta |t*| per class of closest-hit test (header): 0 axis-aligned plane tests, 1 the
  // f32 quadratics, 2 other planar tests (prism faces, triangles), 3 tilted rectangles and
  // checkerboards (the culled shape's own points are bounded apart: occ3)
  constexpr int NK = 4;
  const double eta_k[NK] = {1.25e-7, 2e-3, 1e-6, 1e-6};
  // per cell (occ3) and per aligned block (bocc3): the class-3 shape there, -1 none, -2 several
  std::vector<int32_t> occ3, bocc3;
  std::vector<double> occ;                 // per cell and class: box (lo[3], hi[3]) of possible shading points
  std::vector<int8_t> s_plane;             // shapes tried as the culled one: 1 axis-aligned, 2 tilted (record in sp)
  // per shape tried as the culled one (start-side culling): plane, bounds and, per light, the side
  // and distance of the light box; one record per shape, so that a test touches few cache lines
  struct SPlane {
    double n[3], c, maxd, move;
    double dblo, dbhi;         // n.x - c over the box of ray origins
    double mvs[2];             // move toward the light box on side -1 / +1 (one-sided blur shifts)
    double sD[DT_MAX_SGRID];   // side * D per light (0: the light box is not on one side with margin)
    double box[6];             // tilted planes: the shape's own box (prefilter)
  };
  std::vector<SPlane> sp;
  const int OB = 8, OB2 = 4;               // occ per aligned block of cells (bocc)
  int ob_nx = 0, ob_ny = 0;
  std::vector<double> bocc;
  if (start_on) {
    double olo[3], ohi[3];
    for (int a = 0; a < 3; ++a) {
      olo[a] = std::min((double)nodes[0].lb[a], cam[a] - cam_r);
      ohi[a] = std::max((double)nodes[0].ub[a], cam[a] + cam_r);
    }
    double diag = 0;
    for (int a = 0; a < 3; ++a) diag += (ohi[a] - olo[a]) * (ohi[a] - olo[a]);
    diag = std::sqrt(diag) * 1.02;
    occ.assign((size_t)ncell_all * 6 * NK, 0.0);
    for (size_t c = 0; c < (size_t)ncell_all * NK; ++c)
      for (int a = 0; a < 3; ++a) { occ[c * 6 + a] = INFINITY; occ[c * 6 + 3 + a] = -INFINITY; }
    ob_nx = (g.dim[0] + OB - 1) / OB;
    ob_ny = (g.dim[1] + OB2 - 1) / OB2;
    bocc.assign((size_t)ob_nx * ob_ny * g.dim[2] * 6 * NK, 0.0);
    for (size_t c = 0; c < bocc.size() / 6; ++c)
      for (int a = 0; a < 3; ++a) { bocc[c * 6 + a] = INFINITY; bocc[c * 6 + 3 + a] = -INFINITY; }
    // each shape's box (+ rho) and class, then the cells' boxes, on threads by z-slabs of cells
    struct SBox { double lo[3], hi[3], pad; int k, sid; bool refl, glossy; };
    std::vector<SBox> sbox;
    bool bounded = true;
    std::vector<P3> pts;
    for (size_t sid = 0; sid < nshape && bounded; ++sid) {
      const dtd::DShapeHdr& hd = fs.hdr[sid];
      const double* gp = fs.geom.data() + hd.off;
      SBox b;
      double* blo = b.lo;
      double* bhi = b.hi;
      int k = 1;
      const int mt = fs.mat[sid].material;
      b.refl = mt == DT_MAT_GLASS || mt == DT_MAT_STEEL || mt == DT_MAT_ALUMINUM || mt == DT_MAT_WATER ||
               mt == DT_MAT_LINOLEUM;
      b.glossy = (fs.mat[sid].flags & DT_F_GLOSSY) != 0;
      pts.clear();
      if (hd.type == DT_SHAPE_SPHERE) {
        const double r = std::sqrt(gp[dtd::SP_R2]);
        for (int a = 0; a < 3; ++a) { blo[a] = gp[dtd::SP_C + a] - r; bhi[a] = gp[dtd::SP_C + a] + r; }
      } else if (hd.type == DT_SHAPE_CYLINDER || hd.type == DT_SHAPE_CHECKER_CYLINDER) {
        const double r = std::sqrt(gp[dtd::CY_R2]);
        for (int a = 0; a < 3; ++a) {
          blo[a] = std::min(gp[dtd::CY_C1 + a], gp[dtd::CY_C2 + a]) - r;
          bhi[a] = std::max(gp[dtd::CY_C1 + a], gp[dtd::CY_C2 + a]) + r;
        }
      } else if (shape_hull_points(hd, gp, 0.0, pts) && !pts.empty()) {
        k = 2;
        for (int a = 0; a < 3; ++a) { blo[a] = INFINITY; bhi[a] = -INFINITY; }
        for (const P3& q : pts)
          for (int a = 0; a < 3; ++a) { blo[a] = std::min(blo[a], q[a]); bhi[a] = std::max(bhi[a], q[a]); }
      } else {   // a shape type without bounds here: nothing is start-culled
        bounded = false;
        break;
      }
      if (ypad > 0 && hd.type == DT_SHAPE_RECTANGLE && (hd.flags & DT_F_NAMED_RECT)) {   // moves in the blur passes
        blo[1] -= ypad;
        bhi[1] += ypad;
      }
      double sd = 0;
      for (int a = 0; a < 3; ++a) sd += (bhi[a] - blo[a]) * (bhi[a] - blo[a]);
      const double rho = 1e-6 * (1 + std::sqrt(sd));
      // class 0: a rectangle or checkerboard whose box is flat in one axis has the exact axis
      // normal (the cross product of two edges in that plane has two exact zeros), so X* lies on
      // the box's plane; a near miss of the float checks only leaves the box within the plane
      int flat = -1;
      if (k == 2 && (hd.type == DT_SHAPE_RECTANGLE || hd.type == DT_SHAPE_CHECKERBOARD ||
                     hd.type == DT_SHAPE_CHECKERBOARD_HOLE)) {
        int nflat = 0;
        for (int a = 0; a < 3; ++a)
          if (bhi[a] == blo[a]) { flat = a; ++nflat; }
        if (nflat == 1) k = 0;
        else { flat = -1; k = 3; }
      }
      for (int a = 0; a < 3; ++a)
        if (a != flat) { blo[a] -= rho; bhi[a] += rho; }
      b.pad = 0;
      b.k = k;
      b.sid = (int)sid;
      sbox.push_back(b);
    }
    if (!bounded) occ.clear();
    // The box of every ray origin (header): the camera's eye region and, around each shape whose
    // material spawns secondary rays (refl_materials, cpp:574-576), where such a ray can start:
    // isectP within eta |X* - start| of the shape's box, plus eps (1e-3) times the direction: the
    // unit in / refl_ray (cpp:618, 765) or a glossy sample_refl (cpp:760), whose length stays below
    // 1.5 |gloss_ray| + 7.2 <= 3080 (multiplier <= 2^11, the rectangle's length |lv| <= |gloss_ray|
    // when lv falls back to the unnormalised cross product, the first rectangle's squeeze). Pass 1
    // bounds |X* - start| by the root box's diagonal, pass 2 by the diagonal of pass 1's box and the
    // shape's (starts lie in pass 1's box): each pass's box holds every origin by induction along the
    // rays' parent chains.
    auto box_diag = [](const double* alo, const double* ahi, const double* blo_, const double* bhi_) {
      double s2 = 0;
      for (int a = 0; a < 3; ++a) {
        const double e = std::max(ahi[a], bhi_[a]) - std::min(alo[a], blo_[a]);
        s2 += e * e;
      }
      return std::sqrt(s2) * (1 + 1e-9);
    };
    double blo1[3], bhi1[3];
    for (int a = 0; a < 3; ++a) { blo1[a] = olo[a]; bhi1[a] = ohi[a]; }
    if (!occ.empty()) {
      for (int pass = 0; pass < 2; ++pass) {
        double nlo[3], nhi[3];
        for (int a = 0; a < 3; ++a) { nlo[a] = cam[a] - cam_r; nhi[a] = cam[a] + cam_r; }
        for (const SBox& b : sbox) {
          if (!b.refl) continue;
          const double dist = pass == 0 ? diag + 1e-3 * 3080 * 2 : box_diag(blo1, bhi1, b.lo, b.hi);
          const double pad = eta_k[b.k] * dist + 1e-3 * (b.glossy ? 3080.0 : 1.01) + 1e-9;
          for (int a = 0; a < 3; ++a) {
            nlo[a] = std::min(nlo[a], b.lo[a] - pad);
            nhi[a] = std::max(nhi[a], b.hi[a] + pad);
          }
        }
        // pass 1's box as it is (its pads may leave the root box); pass 2: both boxes hold every
        // origin, so their intersection does
        for (int a = 0; a < 3; ++a) {
          blo1[a] = pass == 0 ? nlo[a] : std::max(nlo[a], blo1[a]);
          bhi1[a] = pass == 0 ? nhi[a] : std::min(nhi[a], bhi1[a]);
        }
      }
      // Cylinders: the box above holds the caps' centres +- r on every axis. X* lies on the
      // infinite cylinder (or at the ray's closest approach, a near miss) within eta_1 |X* - start|
      // of the slab between the caps, which p passed (cyl_in_caps), so on axis k it lies within
      // r sqrt(1 - a_k^2) plus that of the caps' centres: C3's ceiling column no longer stretches
      // 3 units above the ceiling
      for (SBox& b : sbox) {
        const dtd::DShapeHdr& hd = fs.hdr[b.sid];
        if (hd.type != DT_SHAPE_CYLINDER && hd.type != DT_SHAPE_CHECKER_CYLINDER) continue;
        const double* gp = fs.geom.data() + hd.off;
        const double r = std::sqrt(gp[dtd::CY_R2]);
        const double w = eta_k[1] * box_diag(blo1, bhi1, b.lo, b.hi) + 1e-6 * (1 + r);
        for (int a = 0; a < 3; ++a) {
          const double ax = gp[dtd::CY_AX + a];
          const double e = r * std::sqrt(std::max(0.0, 1 - ax * ax)) * (1 + 1e-9) + w;
          b.lo[a] = std::max(b.lo[a], std::min(gp[dtd::CY_C1 + a], gp[dtd::CY_C2 + a]) - e);
          b.hi[a] = std::min(b.hi[a], std::max(gp[dtd::CY_C1 + a], gp[dtd::CY_C2 + a]) + e);
        }
      }
      // + 2e-3: the device picks the cell from o = p + 1e-3 sn, not from p
      for (SBox& b : sbox) b.pad = eta_k[b.k] * box_diag(blo1, bhi1, b.lo, b.hi) + 2e-3;
    }
    g.org_check = true;
    for (int a = 0; a < 3; ++a) { g.org_lo[a] = blo1[a]; g.org_hi[a] = bhi1[a]; }
    if (timing)
      fprintf(stderr, "dt: start-side origin box [%g %g %g] - [%g %g %g] (root and eye: [%g %g %g] - [%g %g %g])\n",
              blo1[0], blo1[1], blo1[2], bhi1[0], bhi1[1], bhi1[2], olo[0], olo[1], olo[2], ohi[0], ohi[1], ohi[2]);
    auto occ_slab = [&](int z_lo, int z_hi) {
      for (const SBox& b : sbox) {
        int i0[3], i1[3];
        bool any = true;
        for (int a = 0; a < 3; ++a) {
          // cells whose widened box [lo + i h - m1, lo + (i + 1) h + m1] meets [blo - pad, bhi + pad]
          i0[a] = std::max(0, (int)std::ceil((b.lo[a] - b.pad - m1 - lo[a]) / hh[a] - 1) - 1);
          i1[a] = std::min(g.dim[a] - 1, (int)std::floor((b.hi[a] + b.pad + m1 - lo[a]) / hh[a]) + 1);
          if (i0[a] > i1[a]) any = false;
        }
        i0[2] = std::max(i0[2], z_lo);
        i1[2] = std::min(i1[2], z_hi - 1);
        if (!any || i0[2] > i1[2]) continue;
        for (int z = i0[2]; z <= i1[2]; ++z)
          for (int y = i0[1]; y <= i1[1]; ++y)
            for (int x = i0[0]; x <= i1[0]; ++x) {
              const int ci[3] = {x, y, z};
              double clo[3], chi[3];
              bool meet = true;
              for (int a = 0; a < 3; ++a) {
                clo[a] = std::max(b.lo[a], lo[a] + ci[a] * hh[a] - m1 - b.pad);
                chi[a] = std::min(b.hi[a], lo[a] + (ci[a] + 1) * hh[a] + m1 + b.pad);
                if (clo[a] > chi[a]) meet = false;
              }
              if (!meet) continue;
              const size_t ci_ = ((size_t)z * g.dim[1] + y) * g.dim[0] + x;
              double* o = occ.data() + ci_ * 6 * NK + b.k * 6;
              for (int a = 0; a < 3; ++a) { o[a] = std::min(o[a], clo[a]); o[3 + a] = std::max(o[3 + a], chi[a]); }
              if (b.k == 3) occ3[ci_] = occ3[ci_] == -1 || occ3[ci_] == b.sid ? b.sid : -2;
            }
      }
    };
    if (!occ.empty()) {
      occ3.assign((size_t)ncell_all, -1);
      bocc3.assign((size_t)ob_nx * ob_ny * g.dim[2], -1);
      const int nt = std::max(1, std::min({(int)std::thread::hardware_concurrency(), 16, g.dim[2]}));
      std::vector<std::thread> th;
      for (int t = 1; t < nt; ++t) th.emplace_back(occ_slab, g.dim[2] * t / nt, g.dim[2] * (t + 1) / nt);
      occ_slab(0, g.dim[2] / nt);
      for (auto& t : th) t.join();
      // the same per aligned block of OB x OB2 x 1 cells (range queries: the blocks covering them)
      for (int z = 0; z < g.dim[2]; ++z)
        for (int y = 0; y < g.dim[1]; ++y)
          for (int x = 0; x < g.dim[0]; ++x) {
            const double* o = occ.data() + (((size_t)z * g.dim[1] + y) * g.dim[0] + x) * 6 * NK;
            double* q = bocc.data() + (((size_t)z * ob_ny + y / OB2) * ob_nx + x / OB) * 6 * NK;
            for (int k = 0; k < NK; ++k)
              for (int a = 0; a < 3; ++a) {
                q[k * 6 + a] = std::min(q[k * 6 + a], o[k * 6 + a]);
                q[k * 6 + 3 + a] = std::max(q[k * 6 + 3 + a], o[k * 6 + 3 + a]);
              }
            const int32_t c3 = occ3[((size_t)z * g.dim[1] + y) * g.dim[0] + x];
            int32_t& q3 = bocc3[((size_t)z * ob_ny + y / OB2) * ob_nx + x / OB];
            if (c3 != -1) q3 = q3 == -1 || q3 == c3 ? c3 : -2;
          }
    }
    if (!occ.empty()) {
      s_plane.assign(nshape, 0);
      sp.assign(nshape, SPlane());
      for (size_t sid = 0; sid < nshape; ++sid) {
        const dtd::DShapeHdr& hd = fs.hdr[sid];
        const double* R = nullptr;
        if (hd.type == DT_SHAPE_RECTANGLE) R = fs.geom.data() + hd.off + dtd::RC_R;
        else if (hd.type == DT_SHAPE_CHECKERBOARD || hd.type == DT_SHAPE_CHECKERBOARD_HOLE) R = fs.geom.data() + hd.off + dtd::CK_R;
        if (!R) continue;
        const double* n = R + dtd::R_N;
        const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (!(nn > 0) || !std::isfinite(nn)) continue;
        SPlane& P = sp[sid];
        for (int a = 0; a < 3; ++a) P.n[a] = n[a] / nn;
        P.c = P.n[0] * R[dtd::R_A] + P.n[1] * R[dtd::R_A + 1] + P.n[2] * R[dtd::R_A + 2];
        double md = 0;
        for (int q = 0; q < 8; ++q) {
          double d = -P.c;
          for (int a = 0; a < 3; ++a) d += P.n[a] * (((q >> a) & 1) ? ohi[a] : olo[a]);
          md = std::max(md, std::fabs(d));
        }
        // a "rectangle" shifted by |v| <= ypad in y (blur passes) moves its plane by |n_y| |v|
        P.move = (ypad > 0 && hd.type == DT_SHAPE_RECTANGLE && (hd.flags & DT_F_NAMED_RECT))
                     ? std::fabs(P.n[1]) * ypad * (1 + 1e-9) + 1e-12 : 0.0;
        P.maxd = 1.02 * md + 1e-3 + P.move;
        // with every shift >= 0 (up_only) the plane only moves by n_y v, v in [0, ypad]: toward
        // the light box on side s (d = s (n.x - c)) by at most max(0, s n_y) ypad
        for (int sd = 0; sd < 2; ++sd)
          P.mvs[sd] = P.move == 0.0 || !up_only ? P.move
                                                : std::max(0.0, (sd ? 1.0 : -1.0) * P.n[1]) * ypad * (1 + 1e-9) + 1e-12;
        P.dblo = INFINITY;
        P.dbhi = -INFINITY;
        for (int q = 0; q < 8; ++q) {
          double d = -P.c;
          for (int a = 0; a < 3; ++a) d += P.n[a] * (((q >> a) & 1) ? g.org_hi[a] : g.org_lo[a]);
          P.dblo = std::min(P.dblo, d);
          P.dbhi = std::max(P.dbhi, d);
        }
        s_plane[sid] = 1;
        int zeros = 0;
        for (int a = 0; a < 3; ++a) zeros += P.n[a] == 0.0;
        if (zeros < 2) {   // a tilted plane: its own box is not flat (prefilter below)
          s_plane[sid] = 2;
          for (int a = 0; a < 3; ++a) { P.box[a] = sbox[sid].lo[a]; P.box[3 + a] = sbox[sid].hi[a]; }
        }
      }
    }
  }
  // per (shape, light): the light box's side of the shape's plane (+-1, 0: both) and D, its
  // distance from the plane less the plane's blur movement (filled once the light boxes are known)
  // can no shadow segment from the shading points of cells [c0, c1] (widened box [clo, chi]) to
  // light l's box [llo, lhi] make shape sid's test true? (start-side culling, header)
  auto start_separated = [&](int sid, size_t l, const double* clo, const double* chi, const int* c0, const int* c1,
                             const double* llo, const double* lhi) {
    if (occ.empty() || !s_plane[sid]) return false;
    const SPlane& P = sp[sid];
    const double sD = P.sD[l];
    if (sD == 0) return false;
    const double s = sD > 0 ? 1.0 : -1.0, D = std::fabs(sD);
    const bool one = c0[0] == c1[0] && c0[1] == c1[1] && c0[2] == c1[2];
    // the class-3 shape of the cells (-1 none, -2 several): when it is the culled shape itself, its
    // points are bounded by its own plane test (below), not by their box
    int32_t id3 = -1;
    if (one) {
      id3 = occ3[((size_t)c0[2] * g.dim[1] + c0[1]) * g.dim[0] + c0[0]];
    } else {
      for (int z = c0[2]; z <= c1[2]; ++z)
        for (int by = c0[1] / OB2; by <= c1[1] / OB2; ++by)
          for (int bx = c0[0] / OB; bx <= c1[0] / OB; ++bx) {
            const int32_t q3 = bocc3[((size_t)z * ob_ny + by) * ob_nx + bx];
            if (q3 != -1) id3 = id3 == -1 || id3 == q3 ? q3 : -2;
          }
    }
    // a tilted plane whose own box meets the cells along with other tilted planes: the box's
    // corners leave the plane by far more than the margin, so the bound fails (a host-time
    // prefilter; it only keeps leaves)
    if (s_plane[sid] == 2 && id3 != sid) {
      const double* b = P.box;
      if (b[0] <= chi[0] && b[3] >= clo[0] && b[1] <= chi[1] && b[4] >= clo[1] && b[2] <= chi[2] && b[5] >= clo[2])
        return false;
    }
    const double* n = P.n;
    const double c = P.c, mv = P.mvs[sD > 0 ? 1 : 0];
    double lmax2 = 0, lmin2 = 0;
    for (int a = 0; a < 3; ++a) {
      const double far = std::max(std::fabs(chi[a] - llo[a]), std::fabs(lhi[a] - clo[a]));
      const double gap = std::max({0.0, llo[a] - chi[a], clo[a] - lhi[a]});
      lmax2 += far * far;
      lmin2 += gap * gap;
    }
    if (!(lmin2 > 4e-6)) return false;
    // the cells' boxes of possible shading points: the cell's own, or the aligned blocks covering
    // the range (a superset: the bound can only be lower)
    double mn = INFINITY;
    for (int k = 0; k < NK; ++k) {
      if (k == 3 && id3 == sid) {
        // the culled shape's own points (header): its plane test puts p within
        // 1.25e-7 |d(start)| + O(2^-53 size) of its own plane. A moving rectangle is tested in the
        // pass's shifted scene, the shading points' and the culled plane alike: the bound holds for
        // the shifted plane, whose distances from the origins grow by at most mv (D already less mv)
        const double dmax = std::max(std::fabs(P.dblo), std::fabs(P.dbhi)) + P.move;
        mn = std::min(mn, -1.25e-7 * dmax * (1 + 1e-6) - 1e-12 * (1 + scale));
        continue;
      }
      double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      auto take = [&](const double* o) {
        for (int a = 0; a < 3; ++a) { blo[a] = std::min(blo[a], o[a]); bhi[a] = std::max(bhi[a], o[3 + a]); }
      };
      if (one) {
        take(occ.data() + (((size_t)c0[2] * g.dim[1] + c0[1]) * g.dim[0] + c0[0]) * 6 * NK + k * 6);
      } else {
        for (int z = c0[2]; z <= c1[2]; ++z)
          for (int by = c0[1] / OB2; by <= c1[1] / OB2; ++by)
            for (int bx = c0[0] / OB; bx <= c1[0] / OB; ++bx)
              take(bocc.data() + (((size_t)z * ob_ny + by) * ob_nx + bx) * 6 * NK + k * 6);
      }
      if (!(blo[0] <= bhi[0] && blo[1] <= bhi[1] && blo[2] <= bhi[2])) continue;   // no such shape here
      double d = -s * c, ulo = -c, uhi = -c;
      for (int a = 0; a < 3; ++a) {
        d += std::min(s * n[a] * blo[a], s * n[a] * bhi[a]);
        ulo += std::min(n[a] * blo[a], n[a] * bhi[a]);
        uhi += std::max(n[a] * blo[a], n[a] * bhi[a]);
      }
      // |d(p) - d(X*)| <= eta |d(X*) - d(start)|: X* in these boxes, the start in the origin box
      const double span = std::max(uhi, P.dbhi) - std::min(ulo, P.dblo);
      mn = std::min(mn, d - mv - eta_k[k] * span * (1 + 1e-6) - 1e-12 * (1 + scale));
    }
    const double d_o = std::min(mn, 0.0) + 1e-3 * D / std::sqrt(lmax2);
    return d_o > 1e-7 * (1 + scale);
  };
  // DT_SG_ORDER=1: lists ordered likely-occluder first. Opt-in: +0.6% on C3, +1.4 ms host build
  // 
  const char* so = getenv("DT_SG_ORDER");
  const bool order_lists = so && atoi(so) != 0;
  // DT_SG_HULL: hull culling (header) 0 off, 1 on blocks of cells (default), 2 on blocks and
  // single cells (C5 tunnel frames: -46% kernel time with 1, 1% more with 2, for 3x the host time)
  const char* sh = getenv("DT_SG_HULL");
  const int hull_cull = sh ? atoi(sh) : 1;
  // DT_SG_QUAD=0: spheres and cylinders keep their leaves out of hull culling (before round 6)
  const char* sq = getenv("DT_SG_QUAD");
  const bool quad_hull = !(sq && sq[0] == '0');
  // DT_SG_MAX_LIST: cells with longer lists walk the tree instead (default DT_SGRID_MAX_LIST)
  const char* mls = getenv("DT_SG_MAX_LIST");
  const int max_list = mls && atoi(mls) > 0 ? atoi(mls) : DT_SGRID_MAX_LIST;
  int blk_x = 8, blk_y = 4;
  if (!sg_parse_block(getenv("DT_SG_BLOCK"), blk_x, blk_y))
    fprintf(stderr, "dt: DT_SG_BLOCK='%s' not understood (use 0 or XxY with X, Y >= 1): default 8x4\n",
            getenv("DT_SG_BLOCK"));
  auto now_ms = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const int hw_threads = (int)std::max(1u, std::thread::hardware_concurrency());

  // umbra cells (header), DT_SG_UMBRA: 0 off, 1 whole blocks of cells (default), 2 also single
  // cells of the other blocks (C3: 2.7% more umbra cells for 4x the host time)
  const char* su = getenv("DT_SG_UMBRA");
  const bool umbra_on = !(su && su[0] == '0');
  const bool umbra_cells_too = su && su[0] == '2';
  const double mu = m2 + mplane;
  struct Face { P3 A, n, v1, v2; double c, len1, len2; };
  std::vector<Face> faces_all;
  std::vector<int> face_shape;
  {
    const double hmax = std::max({hh[0], hh[1], hh[2]});
    auto add_face = [&](const double* R, int sid) {
      Face f;
      for (int a = 0; a < 3; ++a) {
        f.A[a] = R[dtd::R_A + a];
        f.n[a] = R[dtd::R_N + a];
        f.v1[a] = R[dtd::R_V1N + a];
        f.v2[a] = R[dtd::R_V2N + a];
      }
      const double nn = std::sqrt(dot3(f.n, f.n));
      if (!(nn > 0) || !std::isfinite(nn)) return;
      for (int a = 0; a < 3; ++a) f.n[a] /= nn;
      f.c = dot3(f.n, f.A);
      f.len1 = R[dtd::R_LEN1];
      f.len2 = R[dtd::R_LEN2];
      // faces smaller than a few cells hardly ever cover a whole cell's view of the light
      if (!(f.len1 > 2 * hmax + 2 * mu && f.len2 > 2 * hmax + 2 * mu)) return;
      faces_all.push_back(f);
      face_shape.push_back(sid);
    };
    for (size_t sid = 0; sid < fs.hdr.size(); ++sid) {
      const dtd::DShapeHdr& hd = fs.hdr[sid];
      const double* gp = fs.geom.data() + hd.off;
      if (hd.type == DT_SHAPE_RECTANGLE && !(hd.flags & DT_F_NAMED_RECT)) add_face(gp + dtd::RC_R, (int)sid);
      else if (hd.type == DT_SHAPE_CHECKERBOARD) add_face(gp + dtd::CK_R, (int)sid);
      else if (hd.type == DT_SHAPE_RECTPRISM_V2)
        for (int f = 0; f < 6; ++f) add_face(gp + dtd::PR_F + f * dtd::R_SIZE, (int)sid);
    }
  }
  std::vector<int32_t> shape_leaf(fs.hdr.size(), -1);   // reference-tree leaf of each shape
  {
    std::vector<int> shp;
    for (int leaf : leaves) {
      leaf_shapes(leaf, shp);
      for (int sid : shp)
        if (sid >= 0 && sid < (int)shape_leaf.size()) shape_leaf[sid] = leaf;
    }
    std::vector<Face> kept;
    std::vector<int> kept_shape;
    for (size_t k = 0; k < faces_all.size(); ++k)
      if (shape_leaf[face_shape[k]] >= 0) {
        kept.push_back(faces_all[k]);
        kept_shape.push_back(face_shape[k]);
      }
    faces_all.swap(kept);
    face_shape.swap(kept_shape);
  }
  // Is every segment from the box [clo, chi] to the light points Q through face f (header)?
  // 1: yes; 0: no; -1: no, and neither for any box inside this one (every crossing point breaks
  // the same check, and a sub-box's crossing points lie in the hull of these)
  auto box_umbra = [&](const Face& f, const double* clo, const double* chi, const std::vector<P3>& Q, double mud) {
    P3 pc[8];
    double dp[8], dq[4];
    for (int k = 0; k < 8; ++k) {
      pc[k] = {(k & 1) ? chi[0] : clo[0], (k & 2) ? chi[1] : clo[1], (k & 4) ? chi[2] : clo[2]};
      dp[k] = dot3(f.n, pc[k]) - f.c;
    }
    const double sgn = dp[0] > 0 ? 1.0 : -1.0;
    for (int k = 0; k < 8; ++k)
      if (!(sgn * dp[k] > mud)) return 0;
    for (size_t j = 0; j < Q.size(); ++j) {
      dq[j] = dot3(f.n, Q[j]) - f.c;
      if (!(sgn * dq[j] < -mud)) return 0;
    }
    bool all_in = true;
    int broken = 15;   // checks that every crossing point breaks so far (bits: c1 low/high, c2 low/high)
    for (int k = 0; k < 8; ++k)
      for (size_t j = 0; j < Q.size(); ++j) {
        const double s = dp[k] / (dp[k] - dq[j]);
        const P3 X = mad3(pc[k], sub3(Q[j], pc[k]), s);
        const P3 XA = sub3(X, f.A);
        const double c1 = dot3(f.v1, XA), c2 = dot3(f.v2, XA);
        const int bad = (c1 < mu ? 1 : 0) | (c1 > f.len1 - mu ? 2 : 0) | (c2 < mu ? 4 : 0) | (c2 > f.len2 - mu ? 8 : 0);
        all_in = all_in && !bad;
        broken &= bad;
      }
    return all_in ? 1 : broken ? -1 : 0;
  };
  // Per light: the (leaf, cell) tests on bands of cell rows and the umbra marking on rows of
  // blocks, then the lists packed into the pools. The tests and the umbra rows of every light run
  // as one set of work items on one thread pool (threads pull items in light order); each item
  // writes only its own rows of its light's arrays, every cell sees the leaves (faces) in the same
  // order, so the lists and umbra cells are those of a one-thread build. The packing (identical
  // lists stored once, across lights too) then runs light by light, as before.
  struct LightSetup {
    bool on = false;
    double llo[3], lhi[3];
    double lpts[5][3];
    int n_lpts = 1;
    std::vector<P3> lhull;   // hull culling and umbra cells (header): a point light; a rectangle's corners
    double mud = 0;          // umbra margin
    std::vector<int> fl;     // faces with the light strictly on one side
  };
  const size_t nl = std::min(lights.size(), (size_t)DT_MAX_SGRID);
  std::vector<LightSetup> ls(nl);
  for (size_t l = 0; l < nl; ++l) {
    const dtd::DLight& L = lights[l];
    g.base[l] = -1;
    if (L.type != DT_LIGHT_POINT && L.type != DT_LIGHT_RECT) continue;
    LightSetup& S = ls[l];
    S.on = true;
    for (int a = 0; a < 3; ++a) {
      if (L.type == DT_LIGHT_POINT) {
        S.llo[a] = S.lhi[a] = L.center[a];
      } else {   // parallelogram A, B, B + D - A, D (rect_sample stays inside it)
        const double c = L.B[a] + L.D[a] - L.A[a];
        S.llo[a] = std::min({L.A[a], L.B[a], L.D[a], c});
        S.lhi[a] = std::max({L.A[a], L.B[a], L.D[a], c});
      }
      S.llo[a] -= m2;
      S.lhi[a] += m2;
    }
    // light sample points for the list ordering: a point light, or a rectangle's centre and corners
    for (int a = 0; a < 3; ++a) {
      if (L.type == DT_LIGHT_POINT) {
        S.lpts[0][a] = L.center[a];
      } else {
        S.lpts[0][a] = 0.5 * (L.B[a] + L.D[a]);
        S.lpts[1][a] = L.A[a];
        S.lpts[2][a] = L.B[a];
        S.lpts[3][a] = L.D[a];
        S.lpts[4][a] = L.B[a] + L.D[a] - L.A[a];
      }
    }
    if (L.type != DT_LIGHT_POINT) S.n_lpts = 5;
    if (L.type == DT_LIGHT_POINT) S.lhull.push_back({L.center[0], L.center[1], L.center[2]});
    else
      for (int k = 1; k < 5; ++k) S.lhull.push_back({S.lpts[k][0], S.lpts[k][1], S.lpts[k][2]});
    if (!umbra_on) continue;
    // longest segment: from the grid box's far corner to the light (mu' keeps the leaf-box test)
    double lmax = 0;
    for (int k = 0; k < 8; ++k) {
      const P3 p = {lo[0] + ((k & 1) ? ext[0] : 0), lo[1] + ((k & 2) ? ext[1] : 0), lo[2] + ((k & 4) ? ext[2] : 0)};
      for (const P3& q : S.lhull) lmax = std::max(lmax, std::sqrt(dot3(sub3(p, q), sub3(p, q))));
    }
    S.mud = std::max(mu, 2e-3 * (lmax + 1));
    for (size_t fi = 0; fi < faces_all.size(); ++fi) {
      if (face_shape[fi] == L.shape_index) continue;   // skipped by the test (cpp:832)
      const Face& f = faces_all[fi];
      double qmn = INFINITY, qmx = -INFINITY;
      for (const P3& q : S.lhull) {
        const double d = dot3(f.n, q) - f.c;
        qmn = std::min(qmn, d);
        qmx = std::max(qmx, d);
      }
      if (qmn > S.mud || qmx < -S.mud) S.fl.push_back((int)fi);
    }
  }
  if (!occ.empty()) {   // start-side culling: each plane's side of each light box
    for (size_t sid = 0; sid < nshape; ++sid) {
      if (!s_plane[sid]) continue;
      SPlane& P = sp[sid];
      for (size_t l = 0; l < nl; ++l) {
        P.sD[l] = 0;
        if (!ls[l].on) continue;
        double dlo = INFINITY, dhi = -INFINITY;
        for (int q = 0; q < 8; ++q) {
          double d = -P.c;
          for (int a = 0; a < 3; ++a) d += P.n[a] * (((q >> a) & 1) ? ls[l].lhi[a] : ls[l].llo[a]);
          dlo = std::min(dlo, d);
          dhi = std::max(dhi, d);
        }
        const int side = dlo > 0 ? 1 : dhi < 0 ? -1 : 0;
        const double D = (side > 0 ? dlo : -dhi) - (side > 0 ? P.mvs[1] : P.mvs[0]);
        // the far end's margin (header): D - 1e-3 above 1e-5 maxdist
        if (side != 0 && D - 1e-3 > 1e-5 * P.maxd) P.sD[l] = side * D;
      }
    }
  }
  // umbra cells of light l, rows of blocks (BX x BY x 1 cells) t, t + nt, ...: every cell tries
  // the faces in the same order, so the result does not depend on the partition
  const int UBX = std::max(1, blk_x), UBY = std::max(1, blk_y);
  const int unby = (g.dim[1] + UBY - 1) / UBY, unrows = unby * g.dim[2];
  auto umbra_rows = [&](size_t l, std::vector<int32_t>& um, int t, int nt) {
    const LightSetup& S = ls[l];
    for (int row = t; row < unrows; row += nt) {
      const int z = row / unby, yb = (row % unby) * UBY, ye = std::min(yb + UBY, g.dim[1]) - 1;
      for (int xb = 0; xb < g.dim[0]; xb += UBX) {
        const int xe = std::min(xb + UBX, g.dim[0]) - 1;
        double clo[3], chi[3];
        const int c0[3] = {xb, yb, z}, c1[3] = {xe, ye, z};
        for (int a = 0; a < 3; ++a) {
          clo[a] = lo[a] + c0[a] * hh[a] - m1;
          chi[a] = lo[a] + (c1[a] + 1) * hh[a] + m1;
        }
        for (int fi : S.fl) {
          const Face& f = faces_all[fi];
          const int32_t leaf = shape_leaf[face_shape[fi]];
          const int r = box_umbra(f, clo, chi, S.lhull, S.mud);
          if (r < 0) continue;
          if (r == 0 && !umbra_cells_too) continue;
          if (r > 0) {
            for (int y = yb; y <= ye; ++y)
              for (int x = xb; x <= xe; ++x) {
                int32_t& u = um[((size_t)z * g.dim[1] + y) * g.dim[0] + x];
                if (u < 0) u = leaf;
              }
            break;   // the whole block is settled
          }
          for (int y = yb; y <= ye; ++y)
            for (int x = xb; x <= xe; ++x) {
              int32_t& u = um[((size_t)z * g.dim[1] + y) * g.dim[0] + x];
              if (u >= 0) continue;
              const int cc[3] = {x, y, z};
              double qlo[3], qhi[3];
              for (int a = 0; a < 3; ++a) {
                qlo[a] = lo[a] + cc[a] * hh[a] - m1;
                qhi[a] = lo[a] + (cc[a] + 1) * hh[a] + m1;
              }
              if (box_umbra(f, qlo, qhi, S.lhull, S.mud) > 0) u = leaf;
            }
        }
      }
    }
  };
  // The (leaf, cell) tests of light l on the cell rows [row_lo, row_hi). Every band visits the
  // leaves in the same order, so each cell's list comes out in leaf order, as from one thread.
  const int rows = g.dim[1] * g.dim[2];
  // a band's lists, CSR: cells [cell_lo, cell_hi), cell c's leaves ent[off[c - cell_lo], off[c - cell_lo + 1])
  struct Band {
    int cell_lo = 0, cell_hi = 0;
    std::vector<int32_t> off, ent;
  };
  auto test_rows = [&](size_t l, Band& band, int row_lo, int row_hi, long& dropped_n) {
    std::vector<std::pair<int32_t, int32_t>> pr;   // (cell, leaf), each cell's leaves in leaf order
    // leaves listed so far per cell of the band: a cell past max_list walks the tree whatever else
    // is listed (the packing below), so its remaining (leaf, cell) tests are skipped. Umbra cells
    // are decided by umbra_rows alone. (Lists are not reordered then: order_lists needs them whole.)
    const size_t band_lo = (size_t)row_lo * g.dim[0];
    std::vector<int32_t> listed(order_lists ? 0 : (size_t)(row_hi - row_lo) * g.dim[0], 0);
    const dtd::DLight& L = lights[l];
    const LightSetup& S = ls[l];
    const double* llo = S.llo;
    const double* lhi = S.lhi;
    const std::vector<P3>& lhull = S.lhull;
    std::vector<int> shp;
    std::vector<P3> shull, hA(8 + lhull.size());
    struct Quad { P3 a, b; double r; };
    std::vector<Quad> squad;
    for (size_t k = 0; k < lhull.size(); ++k) hA[8 + k] = lhull[k];
    for (int leaf : leaves) {
      const dtd::DNodeDev& nd = nodes[leaf];
      // the light's own shape is skipped by the shadow test (cpp:832): a leaf holding only it
      // never occludes this light
      if ((nd.meta & dtd::DN_SINGLE) && (int32_t)nd.first == L.shape_index) continue;
      const double* blo = lbox[leaf].data();
      const double* bhi = lbox[leaf].data() + 3;
      int r0[3], r1[3];
      for (int a = 0; a < 3; ++a) cell_range(lo[a], hh[a], g.dim[a], m1, llo[a], lhi[a], blo[a], bhi[a], r0[a], r1[a]);
      if (r0[0] > r1[0]) continue;
      bool have_shapes = false;
      // Cells go in blocks of BX x BY x 1. A cell's box lies inside its block's box, so when the
      // block's swept box misses the leaf box, or all the leaf's shapes are separated from the
      // block, the same holds for every cell in it. The lists come out as from per-cell tests
      // (the margins m1 and mplane lie far above the rounding of the box corners).
      const int BX = blk_x, BY = blk_y;
      bool have_hull = false;   // shull: the leaf's planar hull points; squad: its spheres and cylinders
      bool hull_ok = false;     // every shape of the leaf is planar, a sphere or a cylinder
      P3 qhint = {0, 0, 0};
      P3 hint = {0, 0, 0};      // last GJK direction for this leaf (neighbouring cells separate alike)
      long start_n = 0;   // shapes of this test left out by start-side culling alone
      auto separated = [&](const double* clo, const double* chi, int hmode, const int* c0, const int* c1) {
        bool sep = !shp.empty();
        start_n = 0;
        for (int sid : shp)
          if (sid != L.shape_index &&
              !shape_separated(fs.hdr[sid], fs.geom.data() + fs.hdr[sid].off, clo, chi, llo, lhi, mplane, ypad)) {
            if (start_separated(sid, l, clo, chi, c0, c1, llo, lhi)) { ++start_n; continue; }
            sep = false;
            break;
          }
        if (sep || hull_cull < hmode) return sep;
        start_n = 0;
        if (!have_hull) {
          have_hull = true;
          hull_ok = true;
          shull.clear();
          squad.clear();
          for (int sid : shp) {
            if (sid == L.shape_index) continue;
            const dtd::DShapeHdr& hd = fs.hdr[sid];
            const double* gp = fs.geom.data() + hd.off;
            if (shape_hull_points(hd, gp, ypad, shull, up_only)) continue;
            // spheres and cylinders: their axis (a point for a sphere) and radius (header, "Hull
            // culling"); they do not move in the blur passes
            Quad q;
            if (hd.type == DT_SHAPE_SPHERE && quad_hull) {
              q.a = {gp[dtd::SP_C], gp[dtd::SP_C + 1], gp[dtd::SP_C + 2]};
              q.b = q.a;
              q.r = std::sqrt(gp[dtd::SP_R2]);
            } else if (!quad_hull) {
              hull_ok = false;
              break;
            } else if (hd.type == DT_SHAPE_CYLINDER || hd.type == DT_SHAPE_CHECKER_CYLINDER) {
              q.a = {gp[dtd::CY_C1], gp[dtd::CY_C1 + 1], gp[dtd::CY_C1 + 2]};
              q.b = {gp[dtd::CY_C2], gp[dtd::CY_C2 + 1], gp[dtd::CY_C2 + 2]};
              q.r = std::sqrt(gp[dtd::CY_R2]);
            } else {
              hull_ok = false;
              break;
            }
            if (!(q.r > 0) || !std::isfinite(q.r)) { hull_ok = false; break; }
            squad.push_back(q);
          }
        }
        if (!hull_ok || (shull.empty() && squad.empty())) return false;
        for (int k = 0; k < 8; ++k) hA[k] = {(k & 1) ? chi[0] : clo[0], (k & 2) ? chi[1] : clo[1], (k & 4) ? chi[2] : clo[2]};
        if (!shull.empty() && !hulls_separated(hA.data(), (int)hA.size(), shull.data(), (int)shull.size(), m2 + mplane, hint))
          return false;
        for (const Quad& q : squad) {
          double L = 0;
          for (const P3& h : hA) L = std::max(L, std::sqrt(dot3(sub3(h, q.a), sub3(h, q.a))));
          L += std::sqrt(dot3(sub3(q.b, q.a), sub3(q.b, q.a)));
          const P3 seg[2] = {q.a, q.b};
          const double m = q.r + 1e-3 + 1e-6 * (1 + L * L / q.r) + m2 + mplane;
          if (!hulls_separated(hA.data(), (int)hA.size(), seg, 2, m, qhint)) return false;
        }
        return true;
      };
      auto cell_box = [&](int x0, int y0, int z0, int x1, int y1, int z1, double* clo, double* chi) {
        const int c0[3] = {x0, y0, z0}, c1[3] = {x1, y1, z1};
        for (int a = 0; a < 3; ++a) {
          clo[a] = lo[a] + c0[a] * hh[a] - m1;
          chi[a] = lo[a] + (c1[a] + 1) * hh[a] + m1;
        }
      };
      for (int z = r0[2]; z <= r1[2]; ++z)
        for (int yb = r0[1]; yb <= r1[1]; yb += BY) {
          const int ye = std::min(yb + BY - 1, r1[1]);
          if (z * g.dim[1] + ye < row_lo || z * g.dim[1] + yb >= row_hi) continue;
          if (!have_shapes) { leaf_shapes(leaf, shp); have_shapes = true; }
          for (int xb = r0[0]; xb <= r1[0]; xb += BX) {
            const int xe = std::min(xb + BX - 1, r1[0]);
            double clo[3], chi[3];
            cell_box(xb, yb, z, xe, ye, z, clo, chi);
            if (!swept_meets(clo, chi, llo, lhi, blo, bhi)) continue;
            const int b0[3] = {xb, yb, z}, b1[3] = {xe, ye, z};
            const bool block_sep = separated(clo, chi, 1, b0, b1);
            const bool block_start = block_sep && start_n > 0;
            for (int y = yb; y <= ye; ++y) {
              const int row = z * g.dim[1] + y;
              if (row < row_lo || row >= row_hi) continue;
              for (int x = xb; x <= xe; ++x) {
                const size_t cell = (size_t)row * g.dim[0] + x;
                if (!listed.empty() && listed[cell - band_lo] > max_list) continue;
                cell_box(x, y, z, x, y, z, clo, chi);
                if (!swept_meets(clo, chi, llo, lhi, blo, bhi)) continue;
                const int q0[3] = {x, y, z};
                if (block_sep || separated(clo, chi, 2, q0, q0)) {
                  ++dropped_n;
                  if (block_start || start_n > 0) start_dropped.fetch_add(1, std::memory_order_relaxed);
                  continue;
                }
                pr.push_back({(int32_t)cell, leaf});
                if (!listed.empty()) ++listed[cell - band_lo];
              }
            }
          }
        }
    }
    // stable counting sort by cell: each cell's leaves keep their (leaf) order
    band.cell_lo = (int)((size_t)row_lo * g.dim[0]);
    band.cell_hi = (int)((size_t)row_hi * g.dim[0]);
    band.off.assign((size_t)(band.cell_hi - band.cell_lo) + 1, 0);
    for (const auto& e : pr) ++band.off[(size_t)(e.first - band.cell_lo) + 1];
    for (size_t k = 1; k < band.off.size(); ++k) band.off[k] += band.off[k - 1];
    band.ent.resize(pr.size());
    {
      std::vector<int32_t> pos(band.off.begin(), band.off.end() - 1);
      for (const auto& e : pr) band.ent[(size_t)pos[(size_t)(e.first - band.cell_lo)]++] = e.second;
    }
    // Likely occluders first. The test is any-hit, so the order never changes an answer, but a
    // lane stops testing at its first occluder and a wave leaves the list once all its lanes
    // are occluded. Score: how many segments from the cell centre to the light's sample points
    // (centre and corners) cross the leaf box; ties keep leaf order.
    if (!order_lists) return;
    std::vector<std::pair<int, int32_t>> keyed;
    for (int row = row_lo; row < row_hi; ++row) {
      const int y = row % g.dim[1], z = row / g.dim[1];
      for (int x = 0; x < g.dim[0]; ++x) {
        const size_t ci_ = (size_t)row * g.dim[0] + x - (size_t)band.cell_lo;
        int32_t* v = band.ent.data() + band.off[ci_];
        const int n = band.off[ci_ + 1] - band.off[ci_];
        if (n < 2 || n > max_list) continue;
        const int ci[3] = {x, y, z};
        double p[3];
        for (int a = 0; a < 3; ++a) p[a] = lo[a] + (ci[a] + 0.5) * hh[a];
        keyed.clear();
        for (int k2 = 0; k2 < n; ++k2) {
          const int32_t leaf = v[k2];
          int sc = 0;
          for (int k = 0; k < S.n_lpts; ++k) sc += segment_meets_box(p, S.lpts[k], lbox[leaf].data(), lbox[leaf].data() + 3);
          keyed.push_back({-sc, leaf});
        }
        std::stable_sort(keyed.begin(), keyed.end(),
                         [](const std::pair<int, int32_t>& a, const std::pair<int, int32_t>& b) { return a.first < b.first; });
        for (int k = 0; k < n; ++k) v[k] = keyed[(size_t)k].second;
      }
    }
  };
  std::vector<std::vector<Band>> bands_l(nl);
  std::vector<std::vector<int32_t>> umbra_l(nl);   // per cell: the occluding face's leaf, or -1
  struct Item { int l, kind, t, nt; };             // kind 0: test rows, 1: umbra rows
  std::vector<Item> items;
  const int nthr = std::max(1, std::min({hw_threads, rows, 16}));
  const int nt_u = std::max(1, std::min({hw_threads, unrows, 16}));
  for (size_t l = 0; l < nl; ++l) {
    if (!ls[l].on) continue;
    bands_l[l].resize((size_t)nthr);
    umbra_l[l].assign(ncell, -1);
    for (int t = 0; t < nthr; ++t) items.push_back({(int)l, 0, t, nthr});
    if (umbra_on)
      for (int t = 0; t < nt_u; ++t) items.push_back({(int)l, 1, t, nt_u});
  }
  std::vector<long> dropped_item(items.size(), 0);
  const double t_setup = now_ms();
  if (timing) fprintf(stderr, "  shadow grid setup: %.2f ms (%zu leaves, %d cells)\n", t_setup - t_entry, leaves.size(), ncell);
  {
    std::atomic<size_t> next(0);
    auto runner = [&]() {
      for (size_t k; (k = next.fetch_add(1)) < items.size();) {
        const Item& it = items[k];
        if (it.kind == 0)
          test_rows((size_t)it.l, bands_l[it.l][(size_t)it.t], (int)((long)rows * it.t / it.nt),
                    (int)((long)rows * (it.t + 1) / it.nt), dropped_item[k]);
        else
          umbra_rows((size_t)it.l, umbra_l[it.l], it.t, it.nt);
      }
    };
    const int np = std::max(1, std::min(hw_threads, 16));
    std::vector<std::thread> pool;
    for (int t = 1; t < np; ++t) pool.emplace_back(runner);
    runner();
    for (auto& th : pool) th.join();
  }
  for (long d : dropped_item) dropped += d;
  const double t_tests = now_ms();
  // identical lists are stored once, in first-occurrence order over lights then cells (the pools
  // do not depend on the thread count): hash -> (offset, length), contents compared on a match.
  // An umbra cell's list is its face's leaf alone.
  // open addressing: slot = (hash, offset, length); a length of 0xffffffff marks an empty slot
  struct Seen { uint64_t h; uint32_t off, len; };
  std::vector<Seen> seen((size_t)1 << 16, Seen{0, 0, 0xffffffffu});
  size_t n_seen = 0;
  auto seen_insert = [&](std::vector<Seen>& tab, const Seen& e) {
    size_t k = (size_t)(e.h ^ (e.h >> 29)) & (tab.size() - 1);
    while (tab[k].len != 0xffffffffu) k = (k + 1) & (tab.size() - 1);
    tab[k] = e;
  };
  g.cells.reserve(g.cells.size() + 2 * (size_t)ncell * nl);
  for (size_t l = 0; l < nl; ++l) {
    if (!ls[l].on) continue;
    const std::vector<int32_t>& umbra = umbra_l[l];
    g.base[l] = (int32_t)g.cells.size() / 2;
    size_t b = 0;
    std::vector<char> in_union;
    size_t nu = 0, tree_cells = 0;
    const bool verbose = getenv("DT_SG_VERBOSE") != nullptr;
    if (verbose) in_union.assign(nodes.size(), 0);
    for (int c = 0; c < ncell; ++c) {
      while (c >= bands_l[l][b].cell_hi) ++b;
      const Band& band = bands_l[l][b];
      const size_t ci = (size_t)(c - band.cell_lo);
      const int32_t* v = band.ent.data() + band.off[ci];
      int n = band.off[ci + 1] - band.off[ci];
      if (umbra[c] >= 0) {
        v = &umbra[c];
        n = 1;
        ++g.umbra_cells;
      }
      if (verbose) {
        if (n > max_list) ++tree_cells;
        for (int k = 0; k < n; ++k) if (!in_union[v[k]]) { in_union[v[k]] = 1; ++nu; }
      }
      if (n > max_list) {   // the tree walk is cheaper for long lists
        g.cells.push_back(0);
        g.cells.push_back(DT_SG_WALK);
        continue;
      }
      uint64_t h = 1469598103934665603ull ^ (uint64_t)n;
      for (int k = 0; k < n; ++k) h = (h ^ (uint32_t)v[k]) * 1099511628211ull;
      uint32_t off = 0;
      bool found = false;
      for (size_t k = (size_t)(h ^ (h >> 29)) & (seen.size() - 1); seen[k].len != 0xffffffffu; k = (k + 1) & (seen.size() - 1))
        if (seen[k].h == h && seen[k].len == (uint32_t)n && std::equal(v, v + n, g.list.begin() + seen[k].off)) {
          off = seen[k].off;
          found = true;
          break;
        }
      if (!found) {
        off = (uint32_t)g.list.size();
        g.list.insert(g.list.end(), v, v + n);
        if (2 * (n_seen + 1) > seen.size()) {   // keep the load under 1/2
          std::vector<Seen> bigger(seen.size() * 2, Seen{0, 0, 0xffffffffu});
          for (const Seen& e : seen)
            if (e.len != 0xffffffffu) seen_insert(bigger, e);
          seen.swap(bigger);
        }
        seen_insert(seen, Seen{h, off, (uint32_t)n});
        ++n_seen;
      }
      g.cells.push_back(off | (umbra[c] >= 0 ? DT_SG_UMBRA : 0u));
      g.cells.push_back((uint32_t)n);
    }
    g.n_lights = (int)l + 1;
    if (verbose)
      fprintf(stderr, "  shadow grid light %zu: union of cell lists %zu of %zu leaves, %zu tree cells\n", l, nu,
              leaves.size(), tree_cells);
  }
  if (timing)
    fprintf(stderr, "  shadow grid: tests and umbra of %zu lights %.2f ms (%d threads), lists %.2f ms\n", nl,
            t_tests - t_setup, std::max(1, std::min(hw_threads, 16)), now_ms() - t_tests);
  // Block subtrees (ShadowGrid::sub_*; DT_SG_SUBTREE=1; for pass-0 rays, whose leaf boxes are the
  // reference's: lists selected with blur-padded boxes only hold more leaves than they need). A cell
  // whose list exceeds the cap walks the whole tree; for the blocks of BX x BY x 1 cells that hold
  // such a cell, the leaves whose box meets the block's swept box to the light (every segment from
  // any cell of the block, reach margin m1 included, lies in it) and whose shapes are not all
  // plane-separated from it, under SAH inner nodes. The device walks it for pass-0 waves whose
  // active lanes all lie in the block: every leaf that can hold an occluder of their segments is
  // in it, the walk's box tests and shape tests are the full tree's, and any-hit order is free.
  const char* sst = getenv("DT_SG_SUBTREE");
  if (sst && sst[0] == '1') {
    const double t_sub = now_ms();
    // DT_SG_SUB_BLOCK: the subtree blocks' size in cells (XxY, default the grid tests' 8x4): smaller
    // blocks hold shorter lists, larger ones serve more scattered waves
    // (blocks of XxYxZ cells: a scattered wave's lanes on a mesh spread over z as much as over x, y)
    int SBX = std::max(1, blk_x), SBY = std::max(1, blk_y), SBZ = 1;
    if (const char* sb = getenv("DT_SG_SUB_BLOCK")) {
      int x = 0, y = 0, z = 1;
      const int n = sscanf(sb, "%dx%dx%d", &x, &y, &z);
      if (n >= 2 && x >= 1 && y >= 1 && z >= 1) {
        SBX = x;
        SBY = y;
        SBZ = n == 3 ? z : 1;
      } else {
        fprintf(stderr, "dt: DT_SG_SUB_BLOCK='%s' not understood (use XxY or XxYxZ): %dx%dx1\n", sb, SBX, SBY);
      }
    }
    g.sub_bx = SBX;
    g.sub_by = SBY;
    g.sub_bz = SBZ;
    g.sub_nbx = (g.dim[0] + SBX - 1) / SBX;
    g.sub_nby = (g.dim[1] + SBY - 1) / SBY;
    g.sub_nbz = (g.dim[2] + SBZ - 1) / SBZ;
    const size_t nblk = (size_t)g.sub_nbx * g.sub_nby * g.sub_nbz;
    struct SubItem { int l; size_t blk; };
    std::vector<SubItem> sitems;
    for (size_t l = 0; l < (size_t)DT_MAX_SGRID; ++l) g.sub_base[l] = -1;
    for (size_t l = 0; l < nl; ++l) {
      if (!ls[l].on || g.base[l] < 0) continue;
      std::vector<char> mark(nblk, 0);
      bool any = false;
      for (int c = 0; c < ncell; ++c)
        if (g.cells[2 * ((size_t)g.base[l] + c) + 1] == DT_SG_WALK) {
          const int x = c % g.dim[0], y = (c / g.dim[0]) % g.dim[1], z = c / (g.dim[0] * g.dim[1]);
          mark[((size_t)(z / SBZ) * g.sub_nby + y / SBY) * g.sub_nbx + x / SBX] = 1;
          any = true;
        }
      if (!any) continue;
      g.sub_base[l] = (int32_t)(g.sub_blocks.size() / 2);
      g.sub_blocks.resize(g.sub_blocks.size() + 2 * nblk, 0u);
      for (size_t k = 0; k < nblk; ++k)
        if (mark[k]) sitems.push_back({(int)l, k});
    }
    std::vector<std::vector<dtd::DNodeDev>> sub(sitems.size());
    std::atomic<size_t> next(0);
    auto runner = [&]() {
      std::vector<int> shp;
      std::vector<int32_t> list;
      for (size_t k; (k = next.fetch_add(1)) < sitems.size();) {
        const size_t l = (size_t)sitems[k].l, blk = sitems[k].blk;
        const LightSetup& S = ls[l];
        const dtd::DLight& L = lights[l];
        const int bz = (int)(blk / ((size_t)g.sub_nbx * g.sub_nby));
        const int by = (int)((blk / g.sub_nbx) % g.sub_nby), bx = (int)(blk % g.sub_nbx);
        const int c0[3] = {bx * SBX, by * SBY, bz * SBZ};
        const int c1[3] = {std::min((bx + 1) * SBX, g.dim[0]) - 1, std::min((by + 1) * SBY, g.dim[1]) - 1,
                           std::min((bz + 1) * SBZ, g.dim[2]) - 1};
        double clo[3], chi[3];
        for (int a = 0; a < 3; ++a) {
          clo[a] = lo[a] + c0[a] * hh[a] - m1;
          chi[a] = lo[a] + (c1[a] + 1) * hh[a] + m1;
        }
        list.clear();
        for (int leaf : leaves) {
          const dtd::DNodeDev& nd = nodes[leaf];
          if ((nd.meta & dtd::DN_SINGLE) && (int32_t)nd.first == L.shape_index) continue;   // cpp:832
          if (!swept_meets(clo, chi, S.llo, S.lhi, lbox[leaf].data(), lbox[leaf].data() + 3)) continue;
          leaf_shapes(leaf, shp);
          bool sep = !shp.empty();
          for (int sid : shp)
            if (sid != L.shape_index &&
                !shape_separated(fs.hdr[sid], fs.geom.data() + fs.hdr[sid].off, clo, chi, S.llo, S.lhi, mplane, ypad)) {
              sep = false;
              break;
            }
          if (!sep) list.push_back(leaf);
        }
        build_fast_subtree(nodes, list, sub[k]);
      }
    };
    {
      const int np = std::max(1, std::min(hw_threads, 16));
      std::vector<std::thread> pool;
      for (int t = 1; t < np; ++t) pool.emplace_back(runner);
      runner();
      for (auto& th : pool) th.join();
    }
    for (size_t k = 0; k < sitems.size(); ++k) {
      const size_t rec = (size_t)g.sub_base[sitems[k].l] + sitems[k].blk;
      g.sub_blocks[2 * rec] = (uint32_t)g.sub_nodes.size();
      g.sub_blocks[2 * rec + 1] = (uint32_t)sub[k].size();
      g.sub_nodes.insert(g.sub_nodes.end(), sub[k].begin(), sub[k].end());
    }
    if (timing)
      fprintf(stderr, "  shadow grid: %zu block subtrees, %zu nodes, %.2f ms\n", sitems.size(), g.sub_nodes.size(),
              now_ms() - t_sub);
  }
  g.plane_dropped = dropped;
  g.start_dropped = start_dropped.load();
  if (timing) fprintf(stderr, "  shadow grid lights: %.2f ms\n", now_ms() - t_setup);
  return g.n_lights > 0;
}

}  // namespace dth
