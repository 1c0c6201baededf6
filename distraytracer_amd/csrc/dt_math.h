// dt_math.h — double-precision 3-vectors with the reference's Eigen semantics, usable from
// host precomputation (g++ -ffp-contract=off) and device code (hipcc -ffp-contract=off).
// The reference's VEC3 is Eigen::Matrix<double,3,1> (SETTINGS.h:13,20); the operation
// orders below are those of Eigen 3.3/3.4's default x86-64 SSE2 build:
//   dot = (a0*b0 + a1*b1) + a2*b2 ; normalized = a / sqrt(dot(a,a)) if > 0 ;
//   isApprox(0) <=> dot(a,a) <= 1e-24*min(dot(a,a),0) ; cross as in Eigen's cross_impl.
// Identical IEEE operation sequences on host and device give identical bits (division and
// sqrt are correctly rounded on both; no FMA contraction anywhere).
#pragma once

#if defined(__HIPCC__)
#define DT_HD __host__ __device__ __forceinline__
#else
#define DT_HD inline
#endif

#include <math.h>
#include <float.h>
#include <stdint.h>

namespace dtm {

struct V3 {
  double x, y, z;
};

DT_HD V3 v3(double x, double y, double z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
DT_HD V3 v3a(const double* a) { return v3(a[0], a[1], a[2]); }
DT_HD V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
DT_HD V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
DT_HD V3 mul(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
DT_HD V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
DT_HD V3 divs(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
DT_HD double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
DT_HD V3 cross(V3 a, V3 b)
{
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
DT_HD double norm(V3 a) { return sqrt(dot(a, a)); }
DT_HD V3 normalized(V3 a)
{
  double n = dot(a, a);
  if (n > 0) return divs(a, sqrt(n));
  return a;
}
DT_HD double dmin(double a, double b) { return (b < a) ? b : a; }   // std::min
DT_HD double dmax(double a, double b) { return (a < b) ? b : a; }   // std::max
DT_HD float fminr(float a, float b) { return (b < a) ? b : a; }
DT_HD float fmaxr(float a, float b) { return (a < b) ? b : a; }
DT_HD bool is_approx_zero(V3 a)
{
  double s = dot(a, a);
  return s <= 1e-24 * dmin(s, 0.0);
}
DT_HD V3 cmin(V3 a, V3 b) { return v3(dmin(a.x, b.x), dmin(a.y, b.y), dmin(a.z, b.z)); }
DT_HD V3 cmax(V3 a, V3 b) { return v3(dmax(a.x, b.x), dmax(a.y, b.y), dmax(a.z, b.z)); }
DT_HD V3 cwise(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
// helpers.h:231-236 — clamp takes and returns float
DT_HD float clampf01(float v)
{
  if (v < 0.0) return 0.0f;
  else if (v > 1.0) return 1.0f;
  return v;
}

}  // namespace dtm
