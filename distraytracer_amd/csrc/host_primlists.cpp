// host_primlists.cpp — per pixel-block candidate leaves for the primary (camera) rays' closest hit.
//
// Every primary ray of pixel (x, y) starts at an eye sample E = eye + ex X + ey Y with
// |ex|, |ey| <= aperture/2 (getDOFSamples, render_final_project.cpp:195-210) and goes through the
// pixel's focal point F = eye + focal_length (a X + b Y - near Z) (cpp:1067-1072, helpers.h:320-324).
// In camera coordinates (u, v along X, Y; depth w along -Z, from the eye) the ray point at parameter
// t >= 0 is (ex (1-t) + t f a, ey (1-t) + t f b, t f near), so over a block of pixels, at parameter t,
// the rays cover u in [t f a0 - rho |1-t|, t f a1 + rho |1-t|] (likewise v) at depth t f near.
// A leaf whose camera-space box misses that set for every t can hold no hit of any primary ray of
// the block. The fast tree (host_fasttree.cpp) is walked with that test; each block keeps the
// leaves that pass, sorted by the smallest ray parameter their box can be reached at.
//
// Why the device may test only these leaves: a shape hit at t > eps lies inside its leaf's box
// (the reference pads leaf bounds by 1e-2, geometry.cpp:2632-2655), so the reference's gather
// always contains the leaf of the closest hit; closest-hit ties go to the lower reference rank, as
// on the fast tree. The margins below (1e-6 relative) lie far above the rounding of the double camera
// arithmetic; the float pixel coordinates are recomputed exactly as the device computes them.
//
// Super-blocks and hull culling: the tree is walked once per super-block (SB x SB blocks) and each
// block filters the super-block's leaves with its own frustum, which yields the same lists as a walk
// per block (the block's frustum lies inside the super-block's, and the walk order is kept). With
// `hulls`, a super-block also drops the leaves whose shapes' hull (host_hull.cpp) stays more than a
// margin away from the hull of its rays: the eye-sample square's corners and the points the rays
// reach at the depth of the scene's far end (every ray point up to there is a convex combination of
// the two). No primary ray of the super-block can then report a hit on those shapes, so the closest
// hit never comes from them. The margin (1e-3 plus 1e-5 of the scene scale) covers the f32 ray
// parameters of the shape tests (~1e-7 of the distance) and the camera rounding.
//
// Motion-blur passes use lists built over the bump tree (padded leaf boxes; leaf hulls with the
// moving rectangles' shifted corners), tested with the exact bumped gather on the device.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "host_internal.h"

namespace dth {

namespace {

// t-interval [lo, hi] intersected with {t : c0 + c1 t <= 0}
inline void constrain(double c0, double c1, double& lo, double& hi)
{
  if (c1 > 0) hi = std::min(hi, -c0 / c1);
  else if (c1 < 0) lo = std::max(lo, -c0 / c1);
  else if (c0 > 0) hi = -INFINITY;
}

struct Frustum {
  double fa0, fa1, fb0, fb1;   // f*a and f*b ranges of the block's focal points
  double rho;                  // eye-sample offset bound per axis
  double fn;                   // depth per unit of t (f * near)
};

// does some primary ray of the block meet the camera-space box [u0,u1]x[v0,v1]x[w0,w1]?
// tnear: the smallest t at which it can
bool frustum_meets(const Frustum& F, const double b[6], double& tnear)
{
  const double u0 = b[0], u1 = b[1], v0 = b[2], v1 = b[3], w0 = b[4], w1 = b[5];
  bool any = false;
  tnear = INFINITY;
  for (int piece = 0; piece < 2; ++piece) {
    double lo = piece == 0 ? 0.0 : 1.0, hi = piece == 0 ? 1.0 : INFINITY;
    // depth: w0 <= t fn <= w1
    constrain(w0, -F.fn, lo, hi);
    constrain(-w1, F.fn, lo, hi);
    const double r = F.rho;
    if (piece == 0) {   // |1-t| = 1-t
      constrain(-r - u1, F.fa0 + r, lo, hi);   // lower u edge <= u1
      constrain(u0 - r, r - F.fa1, lo, hi);    // upper u edge >= u0
      constrain(-r - v1, F.fb0 + r, lo, hi);
      constrain(v0 - r, r - F.fb1, lo, hi);
    } else {            // |1-t| = t-1
      constrain(r - u1, F.fa0 - r, lo, hi);
      constrain(u0 + r, -(F.fa1 + r), lo, hi);
      constrain(r - v1, F.fb0 - r, lo, hi);
      constrain(v0 + r, -(F.fb1 + r), lo, hi);
    }
    if (lo <= hi) {
      any = true;
      tnear = std::min(tnear, lo);
    }
  }
  return any;
}

}  // namespace

bool build_primary_lists(const std::vector<dtd::DNodeDev>& fnodes, int n_fnodes, const dtd::DParams& P, int B,
                         PrimLists& out, const std::vector<std::vector<P3>>* hulls, int SB)
{
  out = PrimLists();
  if (n_fnodes <= 0 || B < 1 || P.xRes < 1 || P.yRes < 1) return false;
  if (!(P.focal_length > 0) || !(P.near_plane > 0) || !(P.aperture >= 0)) return false;
  if (SB < 1) SB = 1;
  const double X[3] = {P.X[0], P.X[1], P.X[2]}, Y[3] = {P.Y[0], P.Y[1], P.Y[2]}, Z[3] = {P.Z[0], P.Z[1], P.Z[2]};
  const double* eye = P.eye;
  double scale = 1;
  for (int k = 0; k < 3; ++k) scale = std::max(scale, std::fabs(eye[k]));
  for (int k = 0; k < 3; ++k)
    scale = std::max({scale, std::fabs(fnodes[0].lb[k]), std::fabs(fnodes[0].ub[k])});
  if (!std::isfinite(scale)) return false;
  const double m = 1e-6 * (1 + scale);
  // camera-space boxes of every node (the AABB of its 8 corners), widened by m
  std::vector<std::array<double, 6>> cb(n_fnodes);
  double wmax = 0;   // camera depth of the scene's far end (root box)
  for (int i = 0; i < n_fnodes; ++i) {
    const dtd::DNodeDev& nd = fnodes[i];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int c = 0; c < 8; ++c) {
      const double p[3] = {(c & 1 ? nd.ub[0] : nd.lb[0]) - eye[0], (c & 2 ? nd.ub[1] : nd.lb[1]) - eye[1],
                           (c & 4 ? nd.ub[2] : nd.lb[2]) - eye[2]};
      const double q[3] = {p[0] * X[0] + p[1] * X[1] + p[2] * X[2], p[0] * Y[0] + p[1] * Y[1] + p[2] * Y[2],
                           -(p[0] * Z[0] + p[1] * Z[1] + p[2] * Z[2])};
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(lo[k], q[k]);
        hi[k] = std::max(hi[k], q[k]);
      }
    }
    for (int k = 0; k < 3; ++k) {
      if (!std::isfinite(lo[k]) || !std::isfinite(hi[k])) return false;
      cb[i][2 * k] = lo[k] - m;
      cb[i][2 * k + 1] = hi[k] + m;
    }
    if (i == 0) wmax = hi[2];
  }
  out.block = B;
  out.nbx = (P.xRes + B - 1) / B;
  out.nby = (P.yRes + B - 1) / B;
  const int nblk = out.nbx * out.nby;
  std::vector<std::vector<std::pair<float, int32_t>>> lists(nblk);
  const double f = P.focal_length;
  // the device's float pixel coordinates (camera_ray): a = l + (r - l) * x / xRes
  auto acoord = [&](int x) { return P.l + (P.r - P.l) * (float)x / (float)P.xRes; };
  auto bcoord = [&](int y) { return P.b + (P.t - P.b) * (float)y / (float)P.yRes; };
  const double rho = (double)P.aperture * 0.5 * (1 + 1e-6) + 1e-7;
  // the frustum of the pixels [x0, x1] x [y0, y1] (and their a, b ranges)
  auto frustum = [&](int x0, int x1, int y0, int y1, double ab[4]) {
    const double a0 = std::min(acoord(x0), acoord(x1)), a1 = std::max(acoord(x0), acoord(x1));
    const double b0 = std::min(bcoord(y0), bcoord(y1)), b1 = std::max(bcoord(y0), bcoord(y1));
    ab[0] = a0; ab[1] = a1; ab[2] = b0; ab[3] = b1;
    Frustum F;
    const double ma = 1e-6 * (1 + std::fabs(f) * std::max(std::fabs(a0), std::fabs(a1))) + m;
    const double mb = 1e-6 * (1 + std::fabs(f) * std::max(std::fabs(b0), std::fabs(b1))) + m;
    F.fa0 = f * a0 - ma;
    F.fa1 = f * a1 + ma;
    F.fb0 = f * b0 - mb;
    F.fb1 = f * b1 + mb;
    F.rho = rho;
    F.fn = f * (double)P.near_plane * (1 - 1e-9);
    return F;
  };
  // hull culling (header): the rays' points up to parameter T, where they pass the far end
  const double T = std::max(1.0, (wmax + 1.0) / (f * (double)P.near_plane));
  const double mhull = 1e-3 + 1e-5 * (1 + scale);
  const int nsbx = (out.nbx + SB - 1) / SB, nsby = (out.nby + SB - 1) / SB;
  const int nthr = std::max(1, std::min({(int)std::thread::hardware_concurrency(), nsby, 16}));
  auto work = [&](int t) {
    std::vector<int32_t> cand;
    std::vector<P3> A(20);
    P3 hint = {0, 0, 0};
    for (int sby = nsby * t / nthr; sby < nsby * (t + 1) / nthr; ++sby)
      for (int sbx = 0; sbx < nsbx; ++sbx) {
        const int bx0 = sbx * SB, bx1 = std::min(out.nbx, bx0 + SB) - 1;
        const int by0 = sby * SB, by1 = std::min(out.nby, by0 + SB) - 1;
        double ab[4];
        const Frustum FS = frustum(bx0 * B, std::min(P.xRes, (bx1 + 1) * B) - 1, by0 * B,
                                   std::min(P.yRes, (by1 + 1) * B) - 1, ab);
        cand.clear();
        int i = 0;
        while (i < n_fnodes) {
          double tn;
          const bool hit = frustum_meets(FS, cb[i].data(), tn);
          if (fnodes[i].meta & dtd::DN_LEAF) {
            if (hit) cand.push_back(i);
            ++i;
          } else {
            i = hit ? i + 1 : fnodes[i].skip;
          }
        }
        if (hulls) {
          for (int k = 0; k < 4; ++k) {   // eye-sample corners, then the far points
            const double ex = (k & 1) ? rho : -rho, ey = (k & 2) ? rho : -rho;
            for (int a = 0; a < 3; ++a) A[k][a] = eye[a] + ex * X[a] + ey * Y[a];
          }
          for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 4; ++j) {
              const double a = ab[j & 1], b = ab[2 + (j >> 1)];
              P3& q = A[4 + 4 * k + j];
              for (int c = 0; c < 3; ++c) {
                const double F = eye[c] + f * (a * X[c] + b * Y[c] - (double)P.near_plane * Z[c]);
                q[c] = A[k][c] + T * (F - A[k][c]);
              }
            }
          size_t w = 0;
          for (int32_t leaf : cand) {
            const std::vector<P3>& hl = (*hulls)[leaf];
            if (!hl.empty() && hulls_separated(A.data(), 20, hl.data(), (int)hl.size(), mhull, hint)) continue;
            cand[w++] = leaf;
          }
          cand.resize(w);
        }
        for (int by = by0; by <= by1; ++by)
          for (int bx = bx0; bx <= bx1; ++bx) {
            const Frustum F = frustum(bx * B, std::min(P.xRes, bx * B + B) - 1, by * B, std::min(P.yRes, by * B + B) - 1, ab);
            std::vector<std::pair<float, int32_t>>& L = lists[(size_t)by * out.nbx + bx];
            for (int32_t leaf : cand) {
              double tn;
              // conservative float t: rounded down, less a relative margin
              if (frustum_meets(F, cb[leaf].data(), tn)) L.push_back({(float)(tn * (1 - 1e-6)) - 1e-6f, leaf});
            }
            std::stable_sort(L.begin(), L.end(), [](const std::pair<float, int32_t>& p, const std::pair<float, int32_t>& q) {
              return p.first < q.first;
            });
          }
      }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nthr; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  out.cells.resize(2 * (size_t)nblk);
  for (int c = 0; c < nblk; ++c) {
    const auto& L = lists[c];
    out.cells[2 * c] = (uint32_t)(out.list.size() / 2);
    out.cells[2 * c + 1] = (uint32_t)L.size();
    for (const auto& e : L) {
      uint32_t tb;
      memcpy(&tb, &e.first, 4);
      out.list.push_back((uint32_t)e.second);
      out.list.push_back(tb);
    }
  }
  if (out.list.empty()) out.list.assign(2, 0u);
  return true;
}

}  // namespace dth
