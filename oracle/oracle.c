/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h). Parity checker and CPU baseline.
 *
 * Plain-C restatement of the reference's per-pixel render loop, written to follow the
 * reference statement by statement, including its float/double mix and its
 * quirks. Every function cites the reference file:line it follows.
 * Built with gcc -O2 -ffp-contract=off (no FMA contraction, like the reference's plain
 * x86-64 SSE2 build, Makefile:3).
 *
 * Eigen semantics used (Eigen 3.3/3.4, default x86-64 SSE2 build; Eigen is not vendored,
 * version unpinned):
 *   dot(a,b)      = (a0*b0 + a1*b1) + a2*b2
 *   norm(a)       = sqrt(dot(a,a))
 *   normalized(a) = dot(a,a) > 0 ? a / sqrt(dot(a,a)) : a       (component division)
 *   a.isApprox(0) = dot(a,a) <= 1e-24 * min(dot(a,a), 0)
 *   cross(a,b)    = (a1*b2 - a2*b1, a2*b0 - a0*b2, a0*b1 - a1*b0)
 *   4x4 products  = sequential sum over k = 0..3
 *   scalar*vector with a float scalar promotes the scalar to double.
 * C++ <cmath> overloads: cos/sin/tan/acos/sqrt/abs of a float are the float functions;
 * pow(float,int) and pow(float,double) are double pow.
 */
#include "oracle.h"
#include "../include/dt_work.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* float libm calls evaluated correctly rounded, f32(f64 function) — the definition the
 * device uses too (dt_kernels.hip cr_cosf...). */
static inline float cr_cosf(float x) { return (float)cos((double)x); }
static inline float cr_sinf(float x) { return (float)sin((double)x); }
static inline float cr_tanf(float x) { return (float)tan((double)x); }
static inline float cr_acosf(float x) { return (float)acos((double)x); }

/* ======================================================================= */
/* vector helpers (Eigen semantics, header comment)                         */
/* ======================================================================= */
typedef struct { double x, y, z; } V3;

static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 v3a(const double* a) { return v3(a[0], a[1], a[2]); }
static inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 mul(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 divs(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline V3 cross(V3 a, V3 b)
{
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double norm(V3 a) { return sqrt(dot(a, a)); }
static inline V3 normalized(V3 a)
{
  double n = dot(a, a);
  if (n > 0) return divs(a, sqrt(n));
  return a;
}
static inline double dmin(double a, double b) { return (b < a) ? b : a; }  /* std::min */
static inline double dmax(double a, double b) { return (a < b) ? b : a; }  /* std::max */
static inline float fminr(float a, float b) { return (b < a) ? b : a; }
static inline float fmaxr(float a, float b) { return (a < b) ? b : a; }
static inline int is_approx_zero(V3 a)
{
  double s = dot(a, a);
  return s <= 1e-24 * dmin(s, 0.0);
}
static inline V3 cmin(V3 a, V3 b) { return v3(dmin(a.x, b.x), dmin(a.y, b.y), dmin(a.z, b.z)); }
static inline V3 cmax(V3 a, V3 b) { return v3(dmax(a.x, b.x), dmax(a.y, b.y), dmax(a.z, b.z)); }
static inline double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* helpers.h:231-236 */
static inline float clampf01(float value)
{
  if (value < 0.0) return 0.0f;
  else if (value > 1.0) return 1.0f;
  return value;
}

/* ======================================================================= */
/* noise.h:25-136 (value noise)                                             */
/* ======================================================================= */
static const int PRIMES[10][3] = {
  {995615039, 600173719, 701464987}, {831731269, 162318869, 136250887},
  {174329291, 946737083, 245679977}, {362489573, 795918041, 350777237},
  {457025711, 880830799, 909678923}, {787070341, 177340217, 593320781},
  {405493717, 291031019, 391950901}, {458904767, 676625681, 424452397},
  {531736441, 939683957, 810651871}, {997169939, 842027887, 423882827}};

/* noise.h:25-29 */
static double cos_interpolate(double a, double b, double x)
{
  double angle = x * M_PI;
  double f = (1 - cos(angle)) * 0.5;
  return a * (1 - f) + b * f;
}

/* noise.h:31-39. int32 arithmetic wraps (two's complement), emulated in uint32. */
double or_noise3d(int i, int x, int y, int z)
{
  int n = (int)((double)(x + y * 57) + (double)z * pow(57, 2));
  uint32_t un = (uint32_t)n;
  un = (un << 13) ^ un;
  uint32_t a = (uint32_t)PRIMES[i][0], b = (uint32_t)PRIMES[i][1], c = (uint32_t)PRIMES[i][2];
  uint32_t t = (un * (un * un * a + b) + c) & 0x7fffffffu;
  return 1.0 - (double)(int)t / 1073741823;
}

/* noise.h:51-70 */
double or_smoothed3d(int i, int x, int y, int z)
{
  double alpha = 9.0 / 18;
  double beta = 2.0 / (8 * 18);
  double gamma = 4.0 / (6 * 18);
  double delta = 3.0 / (12 * 18);
#define N(dx, dy, dz) or_noise3d(i, x + (dx), y + (dy), z + (dz))
  double corners = N(-1, -1, -1) + N(1, -1, -1) + N(-1, 1, -1) + N(1, 1, -1) +
                   N(-1, -1, 1) + N(1, -1, 1) + N(-1, 1, 1) + N(1, 1, 1);
  double sides = N(-1, 0, 0) + N(1, 0, 0) + N(0, 1, 0) + N(0, -1, 0) + N(0, 0, -1) + N(0, 0, 1);
  double dgsides = N(-1, 0, -1) + N(1, 0, -1) + N(0, 1, -1) + N(0, -1, -1) + N(-1, 0, 1) +
                   N(1, 0, 1) + N(0, 1, 1) + N(-1, -1, 0) + N(0, -1, 1) + N(1, -1, 0) +
                   N(-1, 1, 0) + N(1, 1, 0);
  double center = N(0, 0, 0);
#undef N
  return alpha * center + beta * corners + gamma * sides + delta * dgsides;
}

/* noise.h:81-107 */
double or_interpolated_noise3d(int i, double x, double y, double z)
{
  int integer_X = (int)x;
  double fractional_X = x - integer_X;
  int integer_Y = (int)y;
  double fractional_Y = y - integer_Y;
  int integer_Z = (int)z;
  double fractional_Z = z - integer_Z;

  double v1 = or_smoothed3d(i, integer_X, integer_Y, integer_Z);
  double v2 = or_smoothed3d(i, integer_X + 1, integer_Y, integer_Z);
  double v3_ = or_smoothed3d(i, integer_X, integer_Y + 1, integer_Z);
  double v4 = or_smoothed3d(i, integer_X + 1, integer_Y + 1, integer_Z);
  double v5 = or_smoothed3d(i, integer_X, integer_Y, integer_Z + 1);
  double v6 = or_smoothed3d(i, integer_X + 1, integer_Y, integer_Z + 1);
  double v7 = or_smoothed3d(i, integer_X, integer_Y + 1, integer_Z + 1);
  double v8 = or_smoothed3d(i, integer_X + 1, integer_Y + 1, integer_Z + 1);

  double w1 = cos_interpolate(v5, v6, fractional_X);
  double w2 = cos_interpolate(v7, v8, fractional_X);
  double w3 = cos_interpolate(v1, v2, fractional_X);
  double w4 = cos_interpolate(v3_, v4, fractional_X);

  double i1 = cos_interpolate(w3, w4, fractional_Y);
  double i2 = cos_interpolate(w1, w2, fractional_Y);
  return cos_interpolate(i1, i2, fractional_Z);
}

/* noise.h:124-136 with numOctaves=4, persistence=0.5, primeIndex=0 */
double or_value_noise3d(double x, double y, double z)
{
  const int numOctaves = 4;
  const double persistence = 0.5;
  double total = 0;
  double frequency = pow(2, numOctaves);
  double amplitude = pow(persistence, numOctaves);
  for (int i = 0; i < numOctaves; ++i) {
    frequency /= 2;
    amplitude /= persistence;
    total += or_interpolated_noise3d((0 + i) % 10, x * frequency, y * frequency, z * frequency) *
             amplitude;
  }
  return total;
}

/* ======================================================================= */
/* sky: render_final_project.cpp:146-192                                    */
/* ======================================================================= */
void or_sky_color(const dt_globals* g, const double ray_[3], double out[3])
{
  V3 ray = v3a(ray_);
  V3 color = v3(0, 0, 0);
  V3 rnorm = normalized(ray);
  V3 sun = normalized(v3a(g->sundir));
  float sundot = clampf01((float)dot(rnorm, sun));
  V3 so = v3a(g->sun_outer), si = v3a(g->sun_inner), sc = v3a(g->sun_core);
  double p1 = pow(sundot, 1.0), p2 = pow(sundot, 2.0), p256 = pow(sundot, 256.0);
  V3 term = add(add(mul(p1, mul(0.05, so)), mul(p2, mul(0.1, si))), mul(p256, mul(0.9, sc)));
  color = add(color, term);
  double p8 = pow(sundot, 8);
  V3 bs = v3a(g->bluesky), rs = v3a(g->redsky);
  V3 sky = add(mul(1 - 1.5 * p8, bs), mul(p8, mul(1.5, rs)));
  color = add(color, mul(1.0 - 0.8 * rnorm.y, sky));
  out[0] = color.x; out[1] = color.y; out[2] = color.z;
}

void or_cloud_color(const dt_globals* g, const double ray_[3], const double origin_[3],
                    float frame, double out[3])
{
  V3 ray = v3a(ray_), origin = v3a(origin_);
  double skyc[3];
  or_sky_color(g, ray_, skyc);
  V3 skycolor = v3a(skyc);
  V3 color = skycolor;
  for (float z = g->clouddist; z > 0; z -= 0.05) {   /* float loop variable, Q15 */
    V3 p = add(origin, mul(z, ray));
    float noise = 0.7 * or_value_noise3d(p.x, p.y, p.z + frame);
    float clouddistance = p.y + noise + g->cloudhoff;
    if (clouddistance < 0) {
      float density = clampf01(fabsf(clouddistance));
      V3 skycol_rev = v3(skycolor.z, skycolor.y, skycolor.x);
      V3 cloudcolor = sub(v3(1, 1, 1), mul(density, skycol_rev));
      color = add(mul(1 - density * 0.4, color), mul(density * 0.4, cloudcolor));
    }
  }
  /* contrast: clamp() takes and returns float (helpers.h:231) */
  color = v3(clampf01((float)color.x), clampf01((float)color.y), clampf01((float)color.z));
  color = sub(mul(3, v3(pow(color.x, 2), pow(color.y, 2), pow(color.z, 2))),
              mul(2, v3(pow(color.x, 3), pow(color.y, 3), pow(color.z, 3))));
  /* saturation; Eigen sum() of 3 = (c0 + c1) + c2 */
  double s = (color.x + color.y) + color.z;
  V3 grey = v3(0.33 * s, 0.33 * s, 0.33 * s);
  color = sub(mul(1 + g->saturation, color), mul(g->saturation, grey));
  out[0] = color.x; out[1] = color.y; out[2] = color.z;
}

/* ======================================================================= */
/* counter RNG — Philox4x32-10. Replaces the unseedable      */
/* random_device/mt19937 draws of the reference (F7).                         */
/* ======================================================================= */
void or_philox4x32(const uint32_t ctr_[4], const uint32_t key_[2], uint32_t out[4])
{
  uint32_t c0 = ctr_[0], c1 = ctr_[1], c2 = ctr_[2], c3 = ctr_[3];
  uint32_t k0 = key_[0], k1 = key_[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* 53-bit uniform in [0,1) from two words (genrand_res53 construction) */
double or_u01(uint32_t w0, uint32_t w1)
{
  return ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) * (1.0 / 9007199254740992.0);
}

/* one word as a double in [0,1): the area-light (float)uniform draws */
double or_u32_01(uint32_t w) { return (double)w * (1.0 / 4294967296.0); }

static inline uint32_t fmix32(uint32_t h)
{
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
static inline uint32_t root_key(int pass) { return fmix32(0x12345678u + (uint32_t)pass); }
static inline uint32_t child_key(uint32_t parent, int slot)
{
  return fmix32(parent * 0x9E3779B1u + (uint32_t)slot + 1u);
}

enum { P_DOF = 1, P_LIGHT = 2, P_SPHL = 3, P_GLOSSY = 4, P_BLUR = 5 };

typedef struct { uint32_t key[2]; uint32_t pixel; uint32_t sample; } Rng;

static void rng2(const Rng* r, uint32_t node, uint32_t purpose, uint32_t sub, double* u0,
                 double* u1)
{
  uint32_t ctr[4] = {r->pixel, r->sample, node, (purpose << 24) | sub};
  uint32_t o[4];
  or_philox4x32(ctr, r->key, o);
  *u0 = or_u01(o[0], o[1]);
  *u1 = or_u01(o[2], o[3]);
}

/* glossy sample i, attempt a: attempts 2k and 2k+1 share the draw with sub-index (i << 8) | k,
   words 0-1 / 2-3, one word per (float)uniform */
static void glossy_xy(const Rng* r, uint32_t node, int i, int attempt, double* u0, double* u1)
{
  uint32_t ctr[4] = {r->pixel, r->sample, node,
                     ((uint32_t)P_GLOSSY << 24) | ((uint32_t)i << 8) | ((uint32_t)attempt >> 1)};
  uint32_t o[4];
  or_philox4x32(ctr, r->key, o);
  const int k = (attempt & 1) * 2;
  *u0 = or_u32_01(o[k]);
  *u1 = or_u32_01(o[k + 1]);
}

/* ======================================================================= */
/* scene access                                                             */
/* ======================================================================= */
typedef struct {
  int leaf, nchild, child[2], first, count;
  V3 lb, ub;
} BNode;

typedef struct {
  const dt_scene_desc* d;
  const dt_globals* g;
  BNode* nodes;
  int n_nodes, cap_nodes;
  int* idx;
  int n_idx, cap_idx;
  int root;
} Scene;

typedef struct {
  const Scene* s;
  Rng rng;
  float shift;     /* motion-blur y shift of "rectangle" shapes + leaf bump (cpp:1106-1160) */
  dt_stats* st;
  uint64_t* wk;    /* include/dt_work.h event counts of the reference's loop (or_render_work), or NULL */
} Ctx;

#define WK(c, k) do { if ((c)->wk) (c)->wk[(k)]++; } while (0)

static inline const dt_shape_desc* SH(const Scene* s, int i) { return &s->d->shapes[i]; }

/* vertex k of shape, with the motion-blur shift applied to shapes named "rectangle"
 * (shape->A[1] += val ..., cpp:1113-1119; only A..D exist on a Rectangle) */
static inline V3 VX(const Ctx* c, const dt_shape_desc* sh, int k)
{
  V3 p = v3a(sh->v[k]);
  if ((sh->flags & DT_F_NAMED_RECT) && c->shift != 0.0f && k < 4) p.y = p.y + c->shift;
  return p;
}

/* ======================================================================= */
/* geometry.cpp primitives                                                  */
/* ======================================================================= */

/* geometry.cpp:106-140 */
static int sphere_intersect(V3 center, float radius, V3 ray, V3 start, float* t, int* inside)
{
  V3 sc = sub(start, center);
  float A = (float)dot(ray, ray);
  float B = (float)(2 * dot(ray, sc));
  float C = (float)(dot(sc, sc) - pow(radius, 2));
  float discriminant = (float)(pow(B, 2) - 4 * A * C);
  if (discriminant < 0) return 0;
  float t0 = (-B + sqrtf(discriminant)) / (2 * A);
  float t1 = (-B - sqrtf(discriminant)) / (2 * A);
  if (t0 <= 0.001 && t1 <= 0.001) { *inside = 0; return 0; }
  else if (t0 <= 0.001 || t1 <= 0.001) { *t = fmaxr(t0, t1); *inside = 1; return 1; }
  *t = fminr(t0, t1);
  *inside = 0;
  return 1;
}

/* geometry.cpp:173-197 */
static int sphere_shadow(V3 center, float radius, V3 ray, V3 start, float t_max)
{
  float eps = 1e-3f;
  V3 sc = sub(start, center);
  float A = (float)dot(ray, ray);
  float B = (float)(2 * dot(ray, sc));
  float C = (float)(dot(sc, sc) - pow(radius, 2));
  float discriminant = (float)(pow(B, 2) - 4 * A * C);
  if (discriminant < 0) return 0;
  float t0 = (-B + sqrtf(discriminant)) / (2 * A);
  float t1 = (-B - sqrtf(discriminant)) / (2 * A);
  if ((t0 <= eps || t0 >= t_max) && (t1 <= eps || t1 >= t_max)) return 0;
  return 1;
}

/* geometry.cpp:199-204 */
static V3 sphere_norm(V3 center, V3 point)
{
  V3 n = sub(point, center);
  return divs(n, norm(n));
}

/* geometry.cpp:212-240 constructor: axis = (v2 - v1).normalized() */
static V3 cyl_axis(const dt_shape_desc* sh) { return normalized(sub(v3a(sh->v[1]), v3a(sh->v[0]))); }

/* geometry.cpp:242-295 (body only; caps are never tested) */
static int cyl_intersect(const dt_shape_desc* sh, V3 ray, V3 start, float* t, int* inside)
{
  float eps = 1e-3f;
  V3 c1 = v3a(sh->v[0]), c2 = v3a(sh->v[1]), axis = cyl_axis(sh);
  V3 ray_a_proj = sub(ray, mul(dot(ray, axis), axis));
  V3 sc1 = sub(start, c1);
  V3 constant = sub(sc1, mul(dot(sc1, axis), axis));
  float A = (float)dot(ray_a_proj, ray_a_proj);
  float B = (float)(2 * dot(ray_a_proj, constant));
  float C = (float)(dot(constant, constant) - pow(sh->radius, 2));
  float discriminant = (float)(pow(B, 2) - 4 * A * C);
  float t1_body = FLT_MIN, t2_body = FLT_MIN;
  if (discriminant >= 0) {
    t1_body = (-B + sqrtf(discriminant)) / (2 * A);
    t2_body = (-B - sqrtf(discriminant)) / (2 * A);
    if (t1_body <= eps && t2_body <= eps) { *inside = 0; return 0; }
    else if (t1_body <= eps || t2_body <= eps) {
      V3 p = add(start, mul(t1_body, ray));
      if (dot(axis, sub(p, c1)) > 0 && dot(axis, sub(p, c2)) < 0) { *t = t1_body; *inside = 1; return 1; }
      return 0;
    } else {
      V3 p = add(start, mul(t2_body, ray));
      if (dot(axis, sub(p, c1)) > 0 && dot(axis, sub(p, c2)) < 0) { *t = t2_body; *inside = 0; return 1; }
      return 0;
    }
  }
  return 0;
}

/* geometry.cpp:368-417 */
static int cyl_shadow(const dt_shape_desc* sh, V3 ray, V3 start, float t_max)
{
  float eps = 1e-3f;
  V3 c1 = v3a(sh->v[0]), c2 = v3a(sh->v[1]), axis = cyl_axis(sh);
  V3 ray_a_proj = sub(ray, mul(dot(ray, axis), axis));
  V3 sc1 = sub(start, c1);
  V3 constant = sub(sc1, mul(dot(sc1, axis), axis));
  float A = (float)dot(ray_a_proj, ray_a_proj);
  float B = (float)(2 * dot(ray_a_proj, constant));
  float C = (float)(dot(constant, constant) - pow(sh->radius, 2));
  float discriminant = (float)(pow(B, 2) - 4 * A * C);
  if (discriminant >= 0) {
    float t1_body = (-B + sqrtf(discriminant)) / (2 * A);
    float t2_body = (-B - sqrtf(discriminant)) / (2 * A);
    if ((t1_body <= eps || t1_body >= t_max) && (t2_body <= eps || t2_body >= t_max)) return 0;
    else if (t1_body <= eps || t2_body <= eps) {
      V3 p = add(start, mul(t1_body, ray));
      return dot(axis, sub(p, c1)) > 0 && dot(axis, sub(p, c2)) < 0 && t1_body < t_max;
    } else {
      V3 p = add(start, mul(t2_body, ray));
      return dot(axis, sub(p, c1)) > 0 && dot(axis, sub(p, c2)) < 0 && t2_body < t_max;
    }
  }
  return 0;
}

/* geometry.cpp:419-425 */
static V3 cyl_norm(const dt_shape_desc* sh, V3 point)
{
  V3 axis = cyl_axis(sh);
  V3 pc = sub(point, v3a(sh->v[0]));
  return normalized(sub(pc, mul(dot(pc, axis), axis)));
}

/* geometry.cpp:488-553 (Moller-Trumbore) */
static int tri_intersect(const dt_shape_desc* sh, V3 ray, V3 start, float* t, int* inside)
{
  *inside = 0;
  V3 A = v3a(sh->v[0]), B = v3a(sh->v[1]), C = v3a(sh->v[2]);
  V3 r1 = sub(B, A), r2 = sub(C, A);
  V3 h = cross(ray, r2);
  float det = (float)dot(r1, h);
  float invdet = (float)(1.0 / det);
  if (det >= -0.0001 && det <= 0.0001) return 0;
  V3 A0 = sub(start, A);
  float u = (float)(invdet * dot(A0, h));
  if (u < 0 || u > 1) return 0;
  V3 DA0 = cross(A0, r1);
  float v = (float)(dot(ray, DA0) * invdet);
  if (v < 0 || u + v > 1) return 0;
  float t_final = (float)(dot(r2, DA0) * invdet);
  if (t_final > 0.0001) {
    if (sh->flags & DT_F_MESH) {
      if (dot(ray, v3a(sh->mesh_normal)) > 0) *inside = 1;
    }
    *t = t_final;
    return 1;
  }
  return 0;
}

/* geometry.cpp:555-586 */
static int tri_shadow(const dt_shape_desc* sh, V3 ray, V3 start, float t_max)
{
  V3 A = v3a(sh->v[0]), B = v3a(sh->v[1]), C = v3a(sh->v[2]);
  V3 r1 = sub(B, A), r2 = sub(C, A);
  V3 h = cross(ray, r2);
  float det = (float)dot(r1, h);
  float invdet = (float)(1.0 / det);
  if (det >= -0.0001 && det <= 0.0001) return 0;
  V3 A0 = sub(start, A);
  float u = (float)(invdet * dot(A0, h));
  if (u < 0 || u > 1) return 0;
  V3 DA0 = cross(A0, r1);
  float v = (float)(dot(ray, DA0) * invdet);
  if (v < 0 || u + v > 1) return 0;
  float t_final = (float)(dot(r2, DA0) * invdet);
  return t_final > 0.001 && t_final < t_max;
}

/* geometry.cpp:588-594 / 743-749: (B-A) x (C-A), normalized */
static V3 tri_norm(V3 A, V3 B, V3 C) { return normalized(cross(sub(B, A), sub(C, A))); }

/* geometry.cpp:465-479 */
static V3 barycentric3d(V3 p, V3 A, V3 B, V3 C)
{
  V3 n = cross(sub(B, A), sub(C, A));
  V3 n_a = cross(sub(C, B), sub(p, B));
  V3 n_b = cross(sub(A, C), sub(p, C));
  float n_sqnorm = (float)dot(n, n);
  float alpha = (float)(dot(n, n_a) / n_sqnorm);
  float beta = (float)(dot(n, n_b) / n_sqnorm);
  float gamma = 1 - alpha - beta;
  return v3(alpha, beta, gamma);
}

/* geometry.cpp:640-694 (rect_eps 1e-4) and the Checkerboard variants' plane/bounds part
 * (geometry.cpp:2292-2312, 2389-2410; eps 1e-3). Returns 1 if inside the quad. */
static int rect_plane_hit(V3 A, V3 B, V3 C, V3 D, V3 ray, V3 start, float eps, float* t_out,
                          float* check1_out, float* check2_out)
{
  V3 nrm = normalized(tri_norm(A, B, C));   /* getNorm(start).normalized() */
  float dn = (float)dot(ray, nrm);
  if (dn == 0) return 0;
  float t_final = (float)(dot(sub(A, start), nrm) / dn);
  if (t_final <= eps) return 0;
  V3 point = add(start, mul(t_final, ray));
  V3 V_hit = sub(point, A);
  V3 V1 = sub(B, A), V2 = sub(D, A);
  float check1 = (float)dot(normalized(V1), V_hit);
  float check2 = (float)dot(normalized(V2), V_hit);
  if (0 <= check1 && check1 <= norm(V1) && 0 <= check2 && check2 <= norm(V2)) {
    *t_out = t_final;
    if (check1_out) *check1_out = check1;
    if (check2_out) *check2_out = check2;
    return 1;
  }
  return 0;
}

/* geometry.cpp:640-694 */
static int rect_intersect(V3 A, V3 B, V3 C, V3 D, V3 ray, V3 start, float* t, int* inside)
{
  *inside = 0;
  float tt;
  if (rect_plane_hit(A, B, C, D, ray, start, 1e-4f, &tt, NULL, NULL)) { *t = tt; return 1; }
  return 0;
}

/* geometry.cpp:696-741 */
static int rect_shadow(V3 A, V3 B, V3 C, V3 D, V3 ray, V3 start, float t_max, float eps)
{
  float tt;
  if (rect_plane_hit(A, B, C, D, ray, start, eps, &tt, NULL, NULL)) return tt < t_max;
  return 0;
}

/* geometry.cpp:751-759 */
static void rect_uv(V3 A, V3 C, V3 D, V3 p, float* u, float* v)
{
  V3 ad = sub(D, A), dc = sub(C, D);
  *u = (float)(norm(cross(sub(p, A), ad)) / (norm(ad) * norm(dc)));
  *v = (float)(norm(cross(sub(p, D), dc)) / (norm(dc) * norm(ad)));
}

/* geometry.cpp:772-782, with the counter RNG draws x = u0, y = u1 */
static V3 rect_sample(V3 A, V3 B, V3 D, double u0, double u1)
{
  float x = (float)u0, y = (float)u1;
  return add(add(A, mul(x, sub(B, A))), mul(y, sub(D, A)));
}

/* RectPrismV2 faces (geometry.cpp:798-803) */
static const int PRISM_FACES[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4},
                                      {3, 0, 4, 7}, {1, 2, 6, 5}, {2, 3, 7, 6}};

/* geometry.cpp:44-72 */
static int segment_intersect(V3 A, V3 B, V3 ray, V3 origin)
{
  V3 P1 = A, P2 = B, P3 = add(ray, origin), P4 = origin;
  V3 d13 = sub(P1, P3), d43 = sub(P4, P3), d21 = sub(P2, P1);
  float u1 = (float)((dot(d13, d43) * dot(d43, d21) - dot(d13, d21) * dot(d43, d43)) /
                     (pow(norm(d21), 2) * pow(norm(d43), 2) - pow(dot(d43, d21), 2)));
  float u2 = (float)((dot(d13, d43) + u1 * dot(d43, d21)) / pow(norm(d43), 2));
  if (u1 < 0 || u1 > 1) return 0;
  if (u2 < 0) return 0;
  V3 p1 = add(A, mul(u1, sub(B, A)));
  V3 p2 = add(origin, mul(u2, ray));
  return norm(sub(p2, p1)) < 1e-4;
}

/* Checkerboard colour selection (geometry.cpp:2315-2337) */
static V3 checker_color(const dt_shape_desc* sh, float check1, float check2)
{
  int i = (int)(check1 / sh->S), j = (int)(check2 / sh->S);
  V3 color = v3a(sh->color);
  if (i % 2 == 0) {
    if (j % 2 == 0) color = v3a(sh->color1);
    if (j % 2 == 1) color = v3a(sh->color2);
  }
  if (i % 2 == 1) {
    if (j % 2 == 0) color = v3a(sh->color2);
    if (j % 2 == 1) color = v3a(sh->color1);
  }
  return color;
}

/* ---- RectPrismWithCylinder (geometry.cpp:1467-1821) -------------------------------------- */
/* RectPrism::getBounds (1382-1401), used by the constructor for the box the tests slab */
static void rpc_bounds(const dt_shape_desc* sh, V3* lb, V3* ub)
{
  V3 mn = cmin(v3a(sh->v[0]), v3a(sh->v[1])), mx = cmax(v3a(sh->v[0]), v3a(sh->v[1]));
  for (int k = 2; k < 8; ++k) { mn = cmin(mn, v3a(sh->v[k])); mx = cmax(mx, v3a(sh->v[k])); }
  *lb = mn;
  *ub = mx;
}

/* Cylinder::intersectCap (297-324): both cap planes, no radius test */
static int cyl_intersect_cap(const dt_shape_desc* cyl, V3 ray, V3 start, float* t, int* inside)
{
  float eps = 1e-3f;
  *inside = 0;
  V3 c1 = v3a(cyl->v[0]), c2 = v3a(cyl->v[1]), axis = cyl_axis(cyl);
  float rdota = (float)dot(ray, axis);
  if (rdota == 0) return 0;
  float t1 = (float)((dot(c1, axis) - dot(start, axis)) / rdota);
  float t2 = (float)((dot(c2, axis) - dot(start, axis)) / rdota);
  if (t1 < eps && t2 < eps) return 0;
  else if (t1 < eps || t2 < eps) { *inside = 1; *t = fmaxr(t1, t2); return 1; }
  *t = fminr(t1, t2);
  return 1;
}

/* the per-axis part of the box slab test (1515-1533 and the y/z copies): 0 = miss */
static int rpc_axis(double r, double s, double l, double u, double inv, int open_interval, float* mn, float* mx)
{
  float eps = 1e-4f;
  if (fabs(r) < eps) {
    int in = open_interval ? (s > l && s < u) : (s >= l && s <= u);
    if (!in) return 0;
    *mn = FLT_MIN;
    *mx = FLT_MAX;
  } else if (r < 0) {
    *mn = (float)((u - s) * inv);
    *mx = (float)((l - s) * inv);
  } else {
    *mn = (float)((l - s) * inv);
    *mx = (float)((u - s) * inv);
  }
  return 1;
}

/* the box's slab sequence (1511-1588 / 1657-1734); 0 = miss */
static int rpc_box(const dt_shape_desc* sh, V3 ray, V3 start, int open_interval, float* tmin_o, float* tmax_o)
{
  V3 lb, ub;
  rpc_bounds(sh, &lb, &ub);
  V3 inv_ray = v3(1.0 / ray.x, 1.0 / ray.y, 1.0 / ray.z);   /* ray.cwiseInverse() */
  float tmin, tmax, tymin, tymax, tzmin, tzmax;
  if (!rpc_axis(ray.x, start.x, lb.x, ub.x, inv_ray.x, open_interval, &tmin, &tmax)) return 0;
  if (!rpc_axis(ray.y, start.y, lb.y, ub.y, inv_ray.y, open_interval, &tymin, &tymax)) return 0;
  if (tmin > tymax || tymin > tmax) return 0;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  if (!rpc_axis(ray.z, start.z, lb.z, ub.z, inv_ray.z, open_interval, &tzmin, &tzmax)) return 0;
  if (tmin > tzmax || tzmin > tmax) return 0;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  *tmin_o = tmin;
  *tmax_o = tmax;
  return 1;
}

/* RectPrismWithCylinder::intersect (1507-1651). The reference's `hit` and `cap_hit` are
 * uninitialised: taken as false. Where it stores the hit hole's colour into the shape (sticky for
 * every later ray, render-order dependent) the hit record carries it instead: *hole = the hole
 * whose body was hit, -1. */
static int rpc_intersect(const Scene* s, const dt_shape_desc* sh, V3 ray, V3 start, float* t, int* inside,
                         int* hole)
{
  float eps = 1e-4f;
  float tmin, tmax;
  *inside = 0;
  if (!rpc_box(sh, ray, start, 0, &tmin, &tmax)) return 0;
  if (tmax <= eps) return 0;
  if (tmin < eps && tmax > eps) { *t = tmax; *inside = 1; }
  *t = tmin;
  float tcyl = FLT_MAX;
  int inside_cyl = 0, hit = 0, cap_hit = 0, hit_cyl = -1;
  for (int i = 0; i < sh->n_holes; i++) {
    const dt_shape_desc* cyl = &s->d->holes[sh->hole_first + i];
    float t_tmp = 0;
    int inside_tmp = 0;
    int hit_tmp = cyl_intersect(cyl, ray, start, &t_tmp, &inside_tmp);
    if (hit_tmp) {
      hit = 1;
      if (t_tmp <= tcyl) { hit_cyl = i; inside_cyl = inside_tmp; tcyl = t_tmp; }
    }
    hit_tmp = cyl_intersect_cap(cyl, ray, start, &t_tmp, &inside_tmp);
    if (hit_tmp) {
      hit = 1;
      if (t_tmp <= tcyl) { hit_cyl = i; cap_hit = 1; inside_cyl = inside_tmp; tcyl = t_tmp; }
    }
  }
  if (hit) {
    if (tcyl <= *t) {
      if (cap_hit) return 0;
      *inside = inside_cyl;
      *t = tcyl;
      *hole = hit_cyl;
    }
  }
  return 1;
}

/* RectPrismWithCylinder::intersectShadow (1653-1790) */
static int rpc_shadow(const Scene* s, const dt_shape_desc* sh, V3 ray, V3 start, float t_max)
{
  float eps = 1e-4f;
  float tmin, tmax, t;
  if (!rpc_box(sh, ray, start, 1, &tmin, &tmax)) return 0;
  if (tmax <= eps) return 0;
  if (tmin < eps && tmax > eps) {
    if (tmax >= t_max) return 0;
    t = tmax;
  }
  t = tmin;
  float tcyl = FLT_MAX;
  int hit = 0, cap_hit = 0;
  for (int i = 0; i < sh->n_holes; i++) {
    const dt_shape_desc* cyl = &s->d->holes[sh->hole_first + i];
    float t_tmp = FLT_MIN;
    int inside_tmp = 0;
    int hit_tmp = cyl_intersect(cyl, ray, start, &t_tmp, &inside_tmp);
    if (hit_tmp && t_tmp > eps && t_tmp < t_max) {
      hit = 1;
      if (t_tmp <= tcyl) tcyl = t_tmp;
    }
    hit_tmp = cyl_intersect_cap(cyl, ray, start, &t_tmp, &inside_tmp);
    if (hit_tmp && t_tmp > eps && t_tmp < t_max) {
      hit = 1;
      if (t_tmp <= tcyl) { cap_hit = 1; tcyl = t_tmp; }
    }
  }
  if (hit) {
    if (tcyl <= t && tcyl > eps && tcyl < t_max) {
      if (cap_hit) return 0;
    }
  }
  return 1;
}

/* RectPrismWithCylinder::getNorm (1792-1821). lastHit is -1 whenever the shape is the closest hit
 * (intersect resets it before `return true`). Past the three face tests the reference throws: counted
 * as prism_norm_fallback; the hit hole's normal, else the front normal. */
static V3 rpc_norm(const Ctx* c, const dt_shape_desc* sh, V3 point, int hole)
{
  float eps = 1e-3f;
  V3 A = v3a(sh->v[0]), B = v3a(sh->v[1]), D = v3a(sh->v[3]), E = v3a(sh->v[4]);
  V3 F = v3a(sh->v[5]), H = v3a(sh->v[7]);
  V3 normbot = neg(normalized(cross(sub(F, E), sub(H, E))));
  V3 normright = normalized(cross(sub(E, A), sub(D, A)));
  V3 normfront = normalized(cross(sub(B, A), sub(E, A)));
  if (dot(sub(point, A), normbot) <= eps) return normbot;
  if (dot(sub(point, A), normright) <= eps) return normright;
  if (dot(sub(point, A), normfront) <= eps) return normfront;
  if (c->st) c->st->prism_norm_fallback++;
  if (hole >= 0) return cyl_norm(&c->s->d->holes[sh->hole_first + hole], point);
  return normfront;
}

/* RectPrism::getUV (1442-1461), inherited by RectPrismWithCylinder */
static int rpc_uv(const dt_shape_desc* sh, V3 p, double* uo, double* vo)
{
  V3 A = v3a(sh->v[0]), C = v3a(sh->v[2]), D = v3a(sh->v[3]);
  V3 ad = sub(D, A), dc = sub(C, D);
  if (fabs(dot(cross(ad, dc), p)) <= 1e-5) {
    float u = (float)(norm(cross(sub(p, A), ad)) / (norm(ad) * norm(dc)));
    float v = (float)(norm(cross(sub(p, D), dc)) / (norm(dc) * norm(ad)));
    *uo = u; *vo = v;
    return 1;
  }
  *uo = -1; *vo = -1;
  return 0;
}

/* GeoPrimitive::intersect dispatch. t is only written when the shape writes it (the
 * Checkerboard edge-on path returns true without setting t, Q16). hit_color receives the
 * colour the reference's intersect() would have stored into shape->color. */
static int shape_intersect(const Ctx* c, int si, V3 ray, V3 start, float* t, int* inside,
                           V3* hit_color, int* hole)
{
  const dt_shape_desc* sh = SH(c->s, si);
  *hit_color = v3a(sh->color);
  *hole = -1;
  if (sh->type > 0 && sh->type < 10) WK(c, DT_WK_HIT_SHAPE + sh->type);
  switch (sh->type) {
    case DT_SHAPE_RECTPRISM_CYL: {
      int r = rpc_intersect(c->s, sh, ray, start, t, inside, hole);
      if (r && *hole >= 0) *hit_color = v3a(c->s->d->holes[sh->hole_first + *hole].color);
      return r;
    }
    case DT_SHAPE_SPHERE:
      return sphere_intersect(v3a(sh->v[0]), sh->radius, ray, start, t, inside);
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER:
      return cyl_intersect(sh, ray, start, t, inside);
    case DT_SHAPE_TRIANGLE:
      return tri_intersect(sh, ray, start, t, inside);
    case DT_SHAPE_RECTANGLE:
      return rect_intersect(VX(c, sh, 0), VX(c, sh, 1), VX(c, sh, 2), VX(c, sh, 3), ray, start, t,
                            inside);
    case DT_SHAPE_RECTPRISM_V2: { /* geometry.cpp:815-838 */
      float tmin = FLT_MAX, t_tmp;
      int inside_tmp;
      for (int f = 0; f < 6; ++f) {
        const int* q = PRISM_FACES[f];
        if (rect_intersect(v3a(sh->v[q[0]]), v3a(sh->v[q[1]]), v3a(sh->v[q[2]]),
                           v3a(sh->v[q[3]]), ray, start, &t_tmp, &inside_tmp)) {
          if (t_tmp < tmin) { tmin = t_tmp; *inside = inside_tmp; }
        }
      }
      if (tmin < FLT_MAX) { *t = tmin; return 1; }
      return 0;
    }
    case DT_SHAPE_CHECKERBOARD:
    case DT_SHAPE_CHECKERBOARD_HOLE: { /* geometry.cpp:2269-2341, 2366-2444 */
      V3 A = v3a(sh->v[0]), B = v3a(sh->v[1]), C = v3a(sh->v[2]), D = v3a(sh->v[3]);
      *inside = 0;
      if (dot(tri_norm(A, B, C), ray) == 0) {
        if (segment_intersect(A, B, ray, start)) return 1;
        if (segment_intersect(A, D, ray, start)) return 1;
        if (segment_intersect(B, C, ray, start)) return 1;
        if (segment_intersect(C, D, ray, start)) return 1;
        return 0;
      }
      float tt, ch1, ch2;
      if (!rect_plane_hit(A, B, C, D, ray, start, 1e-3f, &tt, &ch1, &ch2)) return 0;
      if (sh->type == DT_SHAPE_CHECKERBOARD_HOLE) {
        float t_tmp;
        int ins;
        if (rect_intersect(v3a(sh->v[4]), v3a(sh->v[5]), v3a(sh->v[6]), v3a(sh->v[7]), ray, start,
                           &t_tmp, &ins)) {
          *inside = ins;
          return 0;
        }
      }
      *t = tt;
      *hit_color = checker_color(sh, ch1, ch2);
      return 1;
    }
  }
  return 0;
}

/* GeoPrimitive::intersectShadow dispatch */
static int shape_shadow(const Ctx* c, int si, V3 ray, V3 start, float t_max)
{
  const dt_shape_desc* sh = SH(c->s, si);
  if (sh->type > 0 && sh->type < 10) WK(c, DT_WK_SHADOW_SHAPE + sh->type);
  switch (sh->type) {
    case DT_SHAPE_RECTPRISM_CYL:
      return rpc_shadow(c->s, sh, ray, start, t_max);
    case DT_SHAPE_SPHERE:
      return sphere_shadow(v3a(sh->v[0]), sh->radius, ray, start, t_max);
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER:
      return cyl_shadow(sh, ray, start, t_max);
    case DT_SHAPE_TRIANGLE:
      return tri_shadow(sh, ray, start, t_max);
    case DT_SHAPE_RECTANGLE:
    case DT_SHAPE_CHECKERBOARD:  /* Checkerboard inherits Rectangle::intersectShadow */
      return rect_shadow(VX(c, sh, 0), VX(c, sh, 1), VX(c, sh, 2), VX(c, sh, 3), ray, start, t_max,
                         1e-4f);
    case DT_SHAPE_RECTPRISM_V2: /* geometry.cpp:840-861 */
      for (int f = 0; f < 6; ++f) {
        const int* q = PRISM_FACES[f];
        if (rect_shadow(v3a(sh->v[q[0]]), v3a(sh->v[q[1]]), v3a(sh->v[q[2]]), v3a(sh->v[q[3]]), ray,
                        start, t_max, 1e-4f))
          return 1;
      }
      return 0;
    case DT_SHAPE_CHECKERBOARD_HOLE: /* geometry.cpp:2446-2498 */
      if (rect_shadow(v3a(sh->v[0]), v3a(sh->v[1]), v3a(sh->v[2]), v3a(sh->v[3]), ray, start, t_max,
                      1e-3f)) {
        if (rect_shadow(v3a(sh->v[4]), v3a(sh->v[5]), v3a(sh->v[6]), v3a(sh->v[7]), ray, start,
                        t_max, 1e-4f))
          return 0;
        return 1;
      }
      return 0;
  }
  return 0;
}

/* GeoPrimitive::getNorm dispatch */
static V3 shape_norm(const Ctx* c, int si, V3 p, int hole)
{
  const dt_shape_desc* sh = SH(c->s, si);
  switch (sh->type) {
    case DT_SHAPE_RECTPRISM_CYL: return rpc_norm(c, sh, p, hole);
    case DT_SHAPE_SPHERE: return sphere_norm(v3a(sh->v[0]), p);
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER: return cyl_norm(sh, p);
    case DT_SHAPE_TRIANGLE: return tri_norm(v3a(sh->v[0]), v3a(sh->v[1]), v3a(sh->v[2]));
    case DT_SHAPE_RECTANGLE:
    case DT_SHAPE_CHECKERBOARD:
    case DT_SHAPE_CHECKERBOARD_HOLE:
      return tri_norm(VX(c, sh, 0), VX(c, sh, 1), VX(c, sh, 2));
    case DT_SHAPE_RECTPRISM_V2: { /* geometry.cpp:863-920 */
      float eps = 1e-3f;
      V3 A = v3a(sh->v[0]), B = v3a(sh->v[1]), D = v3a(sh->v[3]), E = v3a(sh->v[4]);
      V3 F = v3a(sh->v[5]), G = v3a(sh->v[6]), H = v3a(sh->v[7]);
      V3 normbot = neg(normalized(cross(sub(F, E), sub(H, E))));
      V3 normright = normalized(cross(sub(E, A), sub(D, A)));
      V3 normfront = normalized(cross(sub(B, A), sub(E, A)));
      float pa_bot = (float)fabs(dot(normalized(sub(p, A)), normbot));
      float pg_bot = (float)fabs(dot(normalized(sub(p, G)), normbot));
      if (pa_bot <= eps || pg_bot <= eps) return normbot;
      float pa_right = (float)fabs(dot(normalized(sub(p, A)), normright));
      float pg_right = (float)fabs(dot(normalized(sub(p, G)), normright));
      if (pa_right <= eps || pg_right <= eps) return normright;
      float pa_front = (float)fabs(dot(normalized(sub(p, A)), normfront));
      float pg_front = (float)fabs(dot(normalized(sub(p, G)), normfront));
      if (pa_front <= eps || pg_front <= eps) return normfront;
      if (c->st) c->st->prism_norm_fallback++;
      float vals[6] = {pa_bot, pg_bot, pa_right, pg_right, pa_front, pg_front};
      float min_side = vals[0];
      for (int i = 1; i < 6; ++i) if (vals[i] < min_side) min_side = vals[i];
      if (pa_bot == min_side || pg_bot == min_side) return normbot;
      if (pa_right == min_side || pg_right == min_side) return normright;
      return normfront;
    }
  }
  return v3(0, 0, 0);
}

/* geometry.cpp:17-24 */
static V3 fix_norm(V3 ray, V3 nrm)
{
  if (dot(mul(1e4, ray), nrm) >= 0) return mul(-1, nrm);
  return nrm;
}

/* geometry.cpp:27-41 buildCOB + CheckerCylinder ctor (2563-2586): objM = cob * origin */
static void checker_cyl_objM(const dt_shape_desc* sh, double M[4][4])
{
  V3 c1 = v3a(sh->v[0]);
  V3 w = normalized(cyl_axis(sh));
  V3 u = normalized(cross(v3(1, 0, 0), w));
  if (is_approx_zero(u)) u = normalized(cross(v3(0, 1, 0), w));
  V3 v = normalized(cross(w, u));
  double cob[4][4] = {{u.x, u.y, u.z, 0}, {v.x, v.y, v.z, 0}, {w.x, w.y, w.z, 0}, {0, 0, 0, 1}};
  double org[4][4] = {{1, 0, 0, -c1.x}, {0, 1, 0, -c1.y}, {0, 0, 1, -c1.z}, {0, 0, 0, 1}};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = cob[i][0] * org[0][j];
      for (int k = 1; k < 4; ++k) s = s + cob[i][k] * org[k][j];
      M[i][j] = s;
    }
}

/* GeoPrimitive::getUV dispatch: returns type (valid) 0/1/2, writes u,v */
static int shape_uv(const Ctx* c, int si, V3 p, double* uo, double* vo)
{
  const dt_shape_desc* sh = SH(c->s, si);
  switch (sh->type) {
    case DT_SHAPE_RECTPRISM_CYL: return rpc_uv(sh, p, uo, vo);
    case DT_SHAPE_RECTANGLE: {
      float u, v;
      rect_uv(VX(c, sh, 0), VX(c, sh, 2), VX(c, sh, 3), p, &u, &v);
      *uo = u; *vo = v;
      return 1;
    }
    case DT_SHAPE_RECTPRISM_V2: { /* faces[0] = (a,b,c,d) */
      float u, v;
      rect_uv(v3a(sh->v[0]), v3a(sh->v[2]), v3a(sh->v[3]), p, &u, &v);
      *uo = u; *vo = v;
      return 1;
    }
    case DT_SHAPE_TRIANGLE: { /* geometry.cpp:447-463 */
      V3 b = barycentric3d(p, v3a(sh->v[0]), v3a(sh->v[1]), v3a(sh->v[2]));
      if (b.x < 0 || b.x > 1 || b.y < 0 || b.y > 1 || b.z < 0 || b.z > 1) {
        *uo = -1; *vo = -1;
        return 0;
      }
      *uo = (b.x * sh->uv[0][0] + b.y * sh->uv[1][0]) + b.z * sh->uv[2][0];
      *vo = (b.x * sh->uv[0][1] + b.y * sh->uv[1][1]) + b.z * sh->uv[2][1];
      return 1;
    }
    case DT_SHAPE_CHECKERBOARD_HOLE: { /* geometry.cpp:2500-2561 */
      V3 A = v3a(sh->v[0]), B = v3a(sh->v[1]), C = v3a(sh->v[2]), D = v3a(sh->v[3]);
      V3 V_hit = sub(p, A), V1 = sub(B, A), V2 = sub(D, A);
      float check1 = (float)dot(normalized(V1), V_hit);
      float check2 = (float)dot(normalized(V2), V_hit);
      if (0 <= check1 && check1 <= norm(V1) && 0 <= check2 && check2 <= norm(V2)) {
        /* diagonal probe ray, Q17 */
        if (rect_shadow(v3a(sh->v[4]), v3a(sh->v[5]), v3a(sh->v[6]), v3a(sh->v[7]), v3(1, 1, 1),
                        sub(p, v3(1, 1, 1)), FLT_MAX, 1e-4f)) {
          *uo = -1; *vo = -1;
          return 0;
        }
        V3 ad = sub(D, A), dc = sub(C, D);
        float u = (float)(norm(cross(sub(p, A), ad)) / (norm(ad) * norm(dc)));
        float v = (float)(norm(cross(sub(p, D), dc)) / (norm(dc) * norm(ad)));
        float miniu_dist = sh->S / sh->length;
        float miniv_dist = sh->S / sh->width;
        float miniu = u / miniu_dist - (int)(u / miniu_dist);
        float miniv = v / miniv_dist - (int)(v / miniv_dist);
        if (miniu < 0) miniu = 0;
        if (miniv < 0) miniv = 0;
        *uo = miniu; *vo = miniv;
        float bw = sh->borderwidth / (2 * sh->S);
        if ((miniu <= bw || miniu >= 1 - bw) || (miniv <= bw || miniv >= 1 - bw)) return 2;
        return 1;
      }
      *uo = -1; *vo = -1;
      return 0;
    }
    case DT_SHAPE_CHECKER_CYLINDER: { /* geometry.cpp:2588-2630 */
      double M[4][4];
      checker_cyl_objM(sh, M);
      double ph[4] = {p.x, p.y, p.z, 1};
      double po[3];
      for (int i = 0; i < 3; ++i) {
        double s = M[i][0] * ph[0];
        for (int k = 1; k < 4; ++k) s = s + M[i][k] * ph[k];
        po[i] = s;
      }
      V3 axis = cyl_axis(sh);
      float u = 0;
      if (p.x != 0) u = (float)((atan2(po[1], po[0]) + M_PI) / (2 * M_PI));
      float v = (float)(po[2] / norm(axis));
      float miniu_dist = (float)(sh->S / (2 * M_PI * sh->radius));
      float miniv_dist = (float)(sh->S / norm(axis));
      float miniu = u / miniu_dist - (int)(u / miniu_dist);
      float miniv = v / miniv_dist - (int)(v / miniv_dist);
      if (miniu > 1 || miniu < 0 || miniv > 1 || miniv < 0) {
        if (c->st) c->st->uv_out_of_range++;   /* reference terminates (2610-2614) */
      }
      *uo = miniu; *vo = miniv;
      float bw = sh->borderwidth / (2 * sh->S);
      if ((miniu <= bw || miniu >= 1 - bw) || (miniv <= bw || miniv >= 1 - bw)) return 2;
      return 1;
    }
  }
  /* GeoPrimitive::getUV default body is empty (geometry.h:35): treat as type 0 */
  *uo = -1; *vo = -1;
  return 0;
}

/* GeoPrimitive::getBounds dispatch (for the BVH) */
static void shape_bounds(const dt_shape_desc* sh, V3* lb, V3* ub)
{
  switch (sh->type) {
    case DT_SHAPE_SPHERE: { /* geometry.cpp:206-210 */
      V3 c = v3a(sh->v[0]);
      *lb = v3(c.x - sh->radius, c.y - sh->radius, c.z - sh->radius);
      *ub = v3(c.x + sh->radius, c.y + sh->radius, c.z + sh->radius);
      return;
    }
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER: { /* geometry.cpp:427-431 */
      V3 c1 = v3a(sh->v[0]), c2 = v3a(sh->v[1]);
      double r = sh->radius;
      *lb = cmin(v3(c1.x - r, c1.y - r, c1.z - r), v3(c2.x - r, c2.y - r, c2.z - r));
      *ub = cmax(v3(c1.x + r, c1.y + r, c1.z + r), v3(c2.x + r, c2.y + r, c2.z + r));
      return;
    }
    case DT_SHAPE_RECTPRISM_CYL: /* RectPrism::getBounds (1382-1401) */
      rpc_bounds(sh, lb, ub);
      return;
    default: {
      int n = sh->type == DT_SHAPE_TRIANGLE ? 3 : (sh->type == DT_SHAPE_RECTPRISM_V2 ? 8 : 4);
      V3 mn = cmin(v3a(sh->v[0]), v3a(sh->v[1]));
      V3 mx = cmax(v3a(sh->v[0]), v3a(sh->v[1]));
      for (int k = 2; k < n; ++k) { mn = cmin(mn, v3a(sh->v[k])); mx = cmax(mx, v3a(sh->v[k])); }
      *lb = mn; *ub = mx;
      return;
    }
  }
}

/* ======================================================================= */
/* BVH build: helpers.h:330-472, BoundingVolume geometry.cpp:2632-2655      */
/* ======================================================================= */
static int bvh_push_node(Scene* s, int leaf, const int* inds, int n)
{
  if (s->n_nodes == s->cap_nodes) {
    s->cap_nodes = s->cap_nodes ? 2 * s->cap_nodes : 64;
    s->nodes = (BNode*)realloc(s->nodes, sizeof(BNode) * s->cap_nodes);
  }
  BNode* b = &s->nodes[s->n_nodes];
  b->leaf = leaf;
  b->nchild = 0;
  b->first = -1;
  b->count = 0;
  /* BoundingVolume ctor: lbound=FLT_MAX, ubound=FLT_MIN (Q18), setBounds over all inds */
  V3 lb = v3(FLT_MAX, FLT_MAX, FLT_MAX), ub = v3(FLT_MIN, FLT_MIN, FLT_MIN);
  for (int i = 0; i < n; ++i) {
    V3 l, u;
    shape_bounds(&s->d->shapes[inds[i]], &l, &u);
    lb = cmin(lb, l);
    ub = cmax(ub, u);
  }
  b->lb = sub(lb, v3(1e-2, 1e-2, 1e-2));
  b->ub = add(ub, v3(1e-2, 1e-2, 1e-2));
  if (leaf) {
    if (s->n_idx + n > s->cap_idx) {
      while (s->n_idx + n > s->cap_idx) s->cap_idx = s->cap_idx ? 2 * s->cap_idx : 256;
      s->idx = (int*)realloc(s->idx, sizeof(int) * s->cap_idx);
    }
    b->first = s->n_idx;
    b->count = n;
    memcpy(s->idx + s->n_idx, inds, sizeof(int) * n);
    s->n_idx += n;
  }
  return s->n_nodes++;
}

static double shape_center(const Scene* s, int i, int axis) { return s->d->shapes[i].center[axis]; }

/* helpers.h:330-361: VEC2(FLT_MAX, FLT_MIN) initialisation (Q18) */
static void centroid_bounds(const Scene* s, const int* inds, int n, double b[3][2])
{
  for (int a = 0; a < 3; ++a) { b[a][0] = FLT_MAX; b[a][1] = FLT_MIN; }
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) {
      double c = shape_center(s, inds[i], a);
      if (c < b[a][0]) b[a][0] = c;
      if (c > b[a][1]) b[a][1] = c;
    }
}

/* helpers.h:249-272: Lomuto quicksort with a float pivot */
static void order_index(const Scene* s, int* inds, int axis, int low, int high)
{
  if (low < high) {
    float pivot = (float)shape_center(s, inds[high], axis);
    int i = low;
    for (int j = low; j < high; j++) {
      if (shape_center(s, inds[j], axis) < pivot) {
        int tmp = inds[j]; inds[j] = inds[i]; inds[i] = tmp;
        i++;
      }
    }
    int tmp = inds[i]; inds[i] = inds[high]; inds[high] = tmp;
    order_index(s, inds, axis, low, i - 1);
    order_index(s, inds, axis, i + 1, high);
  }
}

/* helpers.h:364-378 */
static float get_sah(const Scene* s, const int* v1, int n1, const int* v2, int n2, float base_area)
{
  double b[3][2];
  centroid_bounds(s, v1, n1, b);
  float v1_cost = (float)((((b[0][1] - b[0][0]) * (b[1][1] - b[1][0]) * 2 +
                            (b[0][1] - b[0][0]) * (b[2][1] - b[2][0]) * 2) +
                           (b[1][1] - b[1][0]) * (b[2][1] - b[2][0]) * 2) /
                          base_area * (double)n1);
  centroid_bounds(s, v2, n2, b);
  float v2_cost = (float)((((b[0][1] - b[0][0]) * (b[1][1] - b[1][0]) * 2 +
                            (b[0][1] - b[0][0]) * (b[2][1] - b[2][0]) * 2) +
                           (b[1][1] - b[1][0]) * (b[2][1] - b[2][0]) * 2) /
                          base_area * (double)n2);
  float cost = s->g->c_trav + s->g->c_isect * (v1_cost + v2_cost);
  return cost;
}

/* helpers.h:381-472 */
static int generate_bvh(Scene* s, int* inds, int n)
{
  if (n == 1) return bvh_push_node(s, 1, inds, n);
  double b[3][2];
  centroid_bounds(s, inds, n, b);
  double extent[3] = {b[0][1] - b[0][0], b[1][1] - b[1][0], b[2][1] - b[2][0]};
  int axis = 0;
  if (extent[1] > extent[0]) {
    if (extent[2] > extent[1]) axis = 2;
    else axis = 1;
  } else if (extent[2] > extent[0]) {
    axis = 2;
  }
  if (extent[axis] < 1e-3) return bvh_push_node(s, 1, inds, n);
  order_index(s, inds, axis, 0, n - 1);
  int node = bvh_push_node(s, 0, inds, n);
  int c0 = -1, c1 = -1;
  if (n == 2) {
    c0 = generate_bvh(s, inds, 1);
    c1 = generate_bvh(s, inds + 1, 1);
  } else if (n == 3) {
    c0 = generate_bvh(s, inds, 1);
    c1 = generate_bvh(s, inds + 1, 2);
  } else if (n == 4) {
    c0 = generate_bvh(s, inds, 2);
    c1 = generate_bvh(s, inds + 2, 2);
  } else {
    float base_area = (float)((extent[0] * extent[1] * 2 + extent[1] * extent[2] * 2) +
                              extent[0] * extent[2] * 2);
    float sah_cost = FLT_MAX;
    int slice = 1;
    for (int i = 1; i < n - 1; i++) {
      float tmp_cost = get_sah(s, inds, i, inds + i, n - i, base_area);
      if (tmp_cost < sah_cost) { sah_cost = tmp_cost; slice = i; }
    }
    if (s->g->c_isect * (float)n <= sah_cost) {
      /* the interior node already pushed becomes the leaf (reference returns a new leaf
         over the same indices: identical bounds) */
      BNode* b2 = &s->nodes[node];
      (void)b2;
      s->n_nodes--;  /* drop interior node; re-push as leaf */
      return bvh_push_node(s, 1, inds, n);
    }
    /* children get copies of the index sub-ranges: sorting inside them must not disturb
       the parent's order (vector<int> by value in the reference) */
    int* left = (int*)malloc(sizeof(int) * slice);
    int* right = (int*)malloc(sizeof(int) * (n - slice));
    memcpy(left, inds, sizeof(int) * slice);
    memcpy(right, inds + slice, sizeof(int) * (n - slice));
    c0 = generate_bvh(s, left, slice);
    c1 = generate_bvh(s, right, n - slice);
    free(left);
    free(right);
  }
  s->nodes[node].nchild = 2;
  s->nodes[node].child[0] = c0;
  s->nodes[node].child[1] = c1;
  return node;
}

static void scene_init(Scene* s, const dt_scene_desc* d, const dt_globals* g)
{
  memset(s, 0, sizeof(*s));
  s->d = d;
  s->g = g;
  int n = d->n_shapes;
  int* range = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
  for (int i = 0; i < n; ++i) range[i] = i;
  s->root = n > 0 ? generate_bvh(s, range, n) : -1;
  free(range);
}

static void scene_free(Scene* s)
{
  free(s->nodes);
  free(s->idx);
}

/* canonical export: pre-order in the reference's stack-pop order (last child first) */
static void export_rec(const Scene* s, int node, int depth, dt_bvh_node* out, int cap, int* n,
                       int* inds, int icap, int* ni)
{
  const BNode* b = &s->nodes[node];
  int me = *n;
  if (me < cap) {
    dt_bvh_node* o = &out[me];
    o->leaf = b->leaf;
    o->n_children = b->nchild;
    o->first_child = b->nchild ? me + 1 : -1;
    o->depth = depth;
    o->first_index = b->leaf ? *ni : -1;
    o->n_indices = b->leaf ? b->count : 0;
    o->lbound[0] = b->lb.x; o->lbound[1] = b->lb.y; o->lbound[2] = b->lb.z;
    o->ubound[0] = b->ub.x; o->ubound[1] = b->ub.y; o->ubound[2] = b->ub.z;
  }
  (*n)++;
  if (b->leaf) {
    for (int i = 0; i < b->count; ++i) {
      if (*ni < icap) inds[*ni] = s->idx[b->first + i];
      (*ni)++;
    }
  }
  for (int c = b->nchild - 1; c >= 0; --c)
    export_rec(s, b->child[c], depth + 1, out, cap, n, inds, icap, ni);
}

int or_bvh(const dt_scene_desc* d, const dt_globals* g, dt_bvh_node* nodes, int cap, int* indices,
           int index_cap, int* n_nodes, int* n_indices)
{
  Scene s;
  scene_init(&s, d, g);
  int n = 0, ni = 0;
  if (s.root >= 0) export_rec(&s, s.root, 0, nodes, cap, &n, indices, index_cap, &ni);
  *n_nodes = n;
  *n_indices = ni;
  scene_free(&s);
  return 0;
}

/* geometry.cpp:2657-2740 */
static int box_intersect(const BNode* b, float bump, V3 ray, V3 inv_ray, V3 start)
{
  double lb[3] = {b->lb.x, b->lb.y, b->lb.z}, ub[3] = {b->ub.x, b->ub.y, b->ub.z};
  if (b->leaf && bump != 0.0f) { lb[1] -= bump; ub[1] += bump; }  /* bumpBVH, helpers.h:530-552 */
  double r[3] = {ray.x, ray.y, ray.z}, ir[3] = {inv_ray.x, inv_ray.y, inv_ray.z};
  double st[3] = {start.x, start.y, start.z};
  float tmin, tmax;
  if (isinf(ir[0])) {
    if (!(st[0] >= lb[0] && st[0] <= ub[0])) return 0;
    tmin = FLT_MIN; tmax = FLT_MAX;
  } else if (r[0] < 0) {
    tmin = (float)((ub[0] - st[0]) * ir[0]);
    tmax = (float)((lb[0] - st[0]) * ir[0]);
  } else {
    tmin = (float)((lb[0] - st[0]) * ir[0]);
    tmax = (float)((ub[0] - st[0]) * ir[0]);
  }
  float tymin, tymax;
  if (isinf(ir[1])) {
    if (!(st[1] >= lb[1] && st[1] <= ub[1])) return 0;
    tymin = FLT_MIN; tymax = FLT_MAX;
  } else if (r[1] < 0) {
    tymin = (float)((ub[1] - st[1]) * ir[1]);
    tymax = (float)((lb[1] - st[1]) * ir[1]);
  } else {
    tymin = (float)((lb[1] - st[1]) * ir[1]);
    tymax = (float)((ub[1] - st[1]) * ir[1]);
  }
  if (tmin > tymax || tymin > tmax) return 0;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  float tzmin, tzmax;
  if (isinf(ir[2])) {
    if (!(st[2] >= lb[2] && st[2] <= ub[2])) return 0;
    tzmin = FLT_MIN; tzmax = FLT_MAX;
  } else if (r[2] < 0) {
    tzmin = (float)((ub[2] - st[2]) * ir[2]);
    tzmax = (float)((lb[2] - st[2]) * ir[2]);
  } else {
    tzmin = (float)((lb[2] - st[2]) * ir[2]);
    tzmax = (float)((ub[2] - st[2]) * ir[2]);
  }
  if (tmin > tzmax || tzmin > tmax) return 0;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  return tmax > 0;
}

/* BVH gather (cpp:491-512 / 806-829): all indices of hit leaves, stack order */
static int bvh_gather(const Ctx* c, V3 ray, V3 start, int* out)
{
  const Scene* s = c->s;
  if (s->root < 0) return 0;
  int stack[256];
  int sp = 0, n = 0;
  stack[sp++] = s->root;
  V3 inv_ray = v3(1.0 / ray.x, 1.0 / ray.y, 1.0 / ray.z);
  while (sp > 0) {
    const BNode* b = &s->nodes[stack[--sp]];
    WK(c, DT_WK_BOX);
    if (box_intersect(b, c->shift, ray, inv_ray, start)) {
      if (b->leaf && b->count > 0) {
        for (int i = 0; i < b->count; ++i) out[n++] = s->idx[b->first + i];
      } else if (b->nchild > 0) {
        for (int k = 0; k < b->nchild; ++k) stack[sp++] = b->child[k];
      }
    }
  }
  return n;
}

/* ======================================================================= */
/* lights: geometry.cpp:2745-2849                                           */
/* ======================================================================= */
static V3 light_sample(const Ctx* c, int li, V3 point, uint32_t node)
{
  const dt_light_desc* L = &c->s->d->lights[li];
  if (L->type == DT_LIGHT_POINT) return sub(v3a(L->center), point);
  if (L->type == DT_LIGHT_RECT) {
    /* area lights 2k and 2k+1 share the draw with sub-index k: words 0-1 / 2-3, one word per
       (float)uniform */
    uint32_t ctr[4] = {c->rng.pixel, c->rng.sample, node, ((uint32_t)P_LIGHT << 24) | ((uint32_t)li >> 1)};
    uint32_t o[4];
    or_philox4x32(ctr, c->rng.key, o);
    const int k = (li & 1) * 2;
    return sub(rect_sample(v3a(L->A), v3a(L->B), v3a(L->D), or_u32_01(o[k]), or_u32_01(o[k + 1])), point);
  }
  /* sphereLight::sampleRay returns the sampled point itself (Q11) */
  V3 C = v3a(L->center);
  double radius = L->radius;
  int attempt = 0;
  double u0, u1;
  rng2(&c->rng, node, P_SPHL, ((uint32_t)li << 8) | (uint32_t)attempt, &u0, &u1);
  double theta = 2 * M_PI * u0;
  double phi = acos(1 - 2 * u1);
  V3 dir = v3(sin(phi) * cos(theta), sin(phi) * sin(theta), cos(phi));
  V3 tmp = add(mul(radius, dir), C);
  V3 baxis = v3a(L->baxis);
  int use_b = !is_approx_zero(baxis);
  int sample_limit = 20;
  while (dot(sub(tmp, C), sub(point, C)) < 0 || (use_b && dot(sub(tmp, C), baxis) < 0)) {
    if (sample_limit < 0) {
      if (c->st) c->st->spherelight_exhausted++;
      break;
    }
    V3 rev_tmp = add(mul(-radius, dir), C);
    if (dot(sub(rev_tmp, C), sub(point, C)) >= 0 && (!use_b || dot(sub(rev_tmp, C), baxis) >= 0)) {
      tmp = rev_tmp;
      break;
    }
    attempt++;
    rng2(&c->rng, node, P_SPHL, ((uint32_t)li << 8) | (uint32_t)attempt, &u0, &u1);
    theta = 2 * M_PI * u0;
    phi = acos(1 - 2 * u1);
    dir = v3(sin(phi) * cos(theta), sin(phi) * sin(theta), cos(phi));
    tmp = add(mul(radius, dir), C);
    sample_limit--;
  }
  return tmp;
}

/* ======================================================================= */
/* rayColor: render_final_project.cpp:487-961                              */
/* ======================================================================= */
static int is_refl_material(int m)
{
  return m == DT_MAT_GLASS || m == DT_MAT_STEEL || m == DT_MAT_ALUMINUM || m == DT_MAT_WATER ||
         m == DT_MAT_LINOLEUM;
}

/* helpers.h:284-293 */
static int refraction_ray(V3* out, V3 in, V3 normal, float sin_theta, float cos_theta, float refr_1,
                          float refr_2)
{
  float int_refl_check =
      (float)(1 - pow(refr_1 / refr_2, 2) * (1 - pow(dot(in, normal), 2)));
  if (int_refl_check < 0) return 0;
  float a = refr_1 / refr_2 * sin_theta;
  float b = 1 / sin_theta;
  float sq = sqrtf(int_refl_check);
  V3 inner = add(in, mul(cos_theta, normal));
  *out = sub(mul(a, mul(b, inner)), mul(sq, normal));
  return 1;
}

/* helpers.h:297-303 */
static void fresnel(float cos_theta, float cos_phi, float refr_1, float refr_2, float* k_refl,
                    float* k_refr)
{
  float rho_par = (refr_2 * cos_theta - refr_1 * cos_phi) / (refr_2 * cos_theta + refr_1 * cos_phi);
  float rho_perp = (refr_1 * cos_theta - refr_2 * cos_phi) / (refr_1 * cos_theta + refr_2 * cos_phi);
  *k_refl = (float)(0.5 * (pow(rho_par, 2) + pow(rho_perp, 2)));
  *k_refr = 1 - *k_refl;
}

/* helpers.h:313-317 (Q10: sum, not product) */
static float schlick_complex(float cos_theta, const double refr[2])
{
  float R0 = (float)((pow(refr[0] - 1, 2) + pow(refr[1], 2)) / (pow(refr[0] + 1, 2) + pow(refr[1], 2)));
  return (float)((R0 + (1 - R0)) + pow(1 - cos_theta, 5));
}

/* glossy sample rectangle construction, cpp:648-669 / 742-755 */
static void glossy_rect(V3 refl_ray, V3 isectP, float multiplier_or_two, V3* A, V3* B, V3* C, V3* D,
                        V3* width_vector, V3* length_vector)
{
  const float length = 1, width = 0.5;
  V3 gloss_ray = mul(multiplier_or_two, refl_ray);
  V3 lv = normalized(cross(gloss_ray, v3(1, 0, 0)));
  if (is_approx_zero(lv)) lv = cross(gloss_ray, v3(0, 0, 1));
  V3 cc = add(gloss_ray, isectP);
  V3 p1 = add(mul(length / 2, lv), cc);
  V3 wv = normalized(cross(neg(gloss_ray), lv));
  *A = add(divs(mul(width, wv), 2), p1);
  *B = sub(*A, mul(length, lv));
  *C = sub(*B, mul(width, wv));
  *D = sub(*A, mul(width, wv));
  *width_vector = wv;
  *length_vector = lv;
}

static void ray_color(const Ctx* c, V3 ray, V3 eye, int depth, V3* color, int* hit, int* in_motion,
                      float k, uint32_t node)
{
  if (depth == 0) return;
  const Scene* s = c->s;
  const dt_globals* g = s->g;
  if (c->st) c->st->rays++;

  /* TRAVERSE TREE (491-512) */
  int* shape_inds = (int*)malloc(sizeof(int) * (s->d->n_shapes > 0 ? s->d->n_shapes : 1));
  int n_inds = bvh_gather(c, ray, eye, shape_inds);

  /* closest hit (514-538) */
  float t_dist = FLT_MAX, t_min = FLT_MAX;
  int any_intersect = 0, inside = 0, hit_i = -1;
  V3 hit_shape_color = v3(0, 0, 0);
  int hit_hole = -1;
  *in_motion = 0;
  for (int q = 0; q < n_inds; ++q) {
    int ins = 0, hole = -1;
    V3 hc;
    int r = shape_intersect(c, shape_inds[q], ray, eye, &t_dist, &ins, &hc, &hole);
    if (r) {
      any_intersect = 1;
      *hit = 1;
      if (t_dist < t_min) {
        hit_i = shape_inds[q];
        inside = ins;  /* Q5: the reference reads an uninitialised variable here */
        t_min = t_dist;
        hit_shape_color = hc;
        hit_hole = hole;
      }
    }
  }
  if (!any_intersect || hit_i < 0) { free(shape_inds); return; }
  const dt_shape_desc* hs = SH(s, hit_i);
  WK(c, DT_WK_HIT);

  V3 isectP = add(eye, mul(t_min, ray));
  V3 normal = shape_norm(c, hit_i, isectP, hit_hole);
  V3 in = normalized(ray);
  V3 shape_color = hit_shape_color;
  int model = hs->model;
  float roughness = hs->roughness;
  int material = hs->material;
  int hit_light = (hs->flags & DT_F_LIGHT) != 0;
  *in_motion = (hs->flags & DT_F_MOTION) != 0;
  normal = fix_norm(in, normal);

  /* Material reflection (571-769) */
  if (g->reflect && is_refl_material(material)) {
    float eps = 1e-3f;
    int glossy = (hs->flags & DT_F_GLOSSY) != 0;
    float k_refl = 1, k_refr = 1;
    if (material == DT_MAT_GLASS) {
      WK(c, DT_WK_REFRACT);
      float cos_theta = (float)dot(normal, neg(in));
      float sin_theta = (float)sqrt(1 - pow(cos_theta, 2));
      V3 out;
      int refr;
      if (inside) refr = refraction_ray(&out, in, normal, sin_theta, cos_theta, g->refr_glass, g->refr_air);
      else refr = refraction_ray(&out, in, normal, sin_theta, cos_theta, g->refr_air, g->refr_glass);
      if (refr) {
        V3 adj_org = add(isectP, mul(eps, in));
        float cos_phi = (float)sqrt(1 - pow(g->refr_glass / g->refr_air, 2) * (1 - pow(dot(in, normal), 2)));
        fresnel(cos_theta, cos_phi, g->refr_air, g->refr_glass, &k_refl, &k_refr);
        ray_color(c, out, adj_org, depth - 1, color, hit, in_motion, k_refr * k, child_key(node, 0));
      }
    }
    V3 refl_ray = sub(in, mul(2 * dot(normal, in), normal));
    if (dot(refl_ray, normal) <= 0) {
      if (c->st) c->st->reflect_errors++;   /* reference: printf + throw (631-638) */
    } else if (dot(refl_ray, normal) > eps) {
      if (glossy && !g->nogloss) {
        V3 A, B, C, D, wv, lv;
        WK(c, DT_WK_GLOSSY_RECT);
        glossy_rect(refl_ray, isectP, 2.0f, &A, &B, &C, &D, &wv, &lv);
        V3 width_adj = wv;
        if (dot(wv, normal) <= 0) width_adj = neg(width_adj);
        V3 length_adj = lv;
        if (dot(lv, normal) <= 0) length_adj = neg(length_adj);
        while (dot(sub(A, isectP), normal) <= 0) A = add(add(A, mul(0.1, width_adj)), mul(0.1, length_adj));
        while (dot(sub(B, isectP), normal) <= 0) B = add(add(B, mul(0.1, width_adj)), mul(0.1, length_adj));
        while (dot(sub(C, isectP), normal) <= 0) C = add(add(C, mul(0.1, width_adj)), mul(0.1, length_adj));
        while (dot(sub(D, isectP), normal) <= 0) D = add(add(D, mul(0.1, width_adj)), mul(0.1, length_adj));
        for (int i = 0; i < g->brdf_samples; i++) {
          int hit_tmp = 0;
          int attempt = 0;
          double u0, u1;
          WK(c, DT_WK_GLOSSY);
          glossy_xy(&c->rng, node, i, attempt, &u0, &u1);
          V3 sample_refl = sub(rect_sample(A, B, D, u0, u1), isectP);
          int sample_limit = 10;
          int exhausted = 0;
          while (dot(sample_refl, normal) <= 0) {
            if (sample_limit < 0) { exhausted = 1; break; }
            float multiplier = (float)pow(2, 11 - sample_limit);
            WK(c, DT_WK_GLOSSY);
            WK(c, DT_WK_GLOSSY_RECT);
            glossy_rect(refl_ray, isectP, multiplier, &A, &B, &C, &D, &wv, &lv);
            attempt++;
            glossy_xy(&c->rng, node, i, attempt, &u0, &u1);
            sample_refl = sub(rect_sample(A, B, D, u0, u1), isectP);
            sample_limit--;
          }
          if (exhausted) {   /* reference throws (724-740) */
            if (c->st) c->st->glossy_exhausted++;
            continue;
          }
          ray_color(c, sample_refl, add(isectP, mul(eps, sample_refl)), depth - 1, color, &hit_tmp,
                    in_motion, k_refl * k / g->brdf_samples, child_key(node, 2 + i));
        }
      } else {
        WK(c, DT_WK_MIRROR);
        ray_color(c, refl_ray, add(isectP, mul(eps, refl_ray)), depth - 1, color, hit, in_motion,
                  k_refl * k, child_key(node, 1));
      }
    }
  }

  /* SHADING (771-960) */
  if (hit_light) {
    WK(c, DT_WK_EMIT);
    if (hs->emit == DT_EMIT_SPHERE) {
      float hitdot = (float)dot(in, normalized(sub(v3a(hs->center), isectP)));
      double f = (0.1 * pow(hitdot, 1) + 0.05 * pow(hitdot, 5)) + 0.9;
      *color = add(*color, mul(f, mul(k, shape_color)));
    }
    if (hs->emit == DT_EMIT_RECT) {
      V3 A = v3a(hs->v[0]), B = v3a(hs->v[1]), C = v3a(hs->v[2]), D = v3a(hs->v[3]);
      float dist = (float)((((norm(sub(isectP, A)) + norm(sub(isectP, B))) + norm(sub(isectP, C))) +
                            norm(sub(isectP, D))) /
                           (8 * norm(sub(v3a(hs->center), A))));
      double f = (0.1 * pow(dist, 1) + 0.05 * pow(dist, 5)) + 0.9;
      *color = add(*color, mul(f, mul(k, shape_color)));
    }
  } else {
    V3 e = normalized(sub(eye, isectP));
    int hits = 0;
    V3 tmp_color = v3(0, 0, 0);
    for (int li = 0; li < s->d->n_lights; ++li) {
      const dt_light_desc* L = &s->d->lights[li];
      WK(c, DT_WK_LIGHT);
      V3 sray = light_sample(c, li, isectP, node);
      float t_max = (float)norm(sray);
      int shadow = 1;
      if (c->st) c->st->shadow_rays++;
      int n_sh = bvh_gather(c, sray, add(isectP, mul(1e-3, sray)), shape_inds);
      V3 sn = normalized(sray);
      for (int q = 0; q < n_sh; ++q) {
        if (shape_inds[q] == L->shape_index) continue;   /* same object as the light */
        if (shape_shadow(c, shape_inds[q], sn, add(isectP, mul(1e-3, sn)), t_max)) {
          shadow = 0;
          break;
        }
      }
      if (shadow == 0) continue;
      V3 r = normalized(add(mul(-1, sray), mul(2 * dot(normal, sray), normal)));
      V3 ray_col;
      V3 lc = v3a(L->color);
      if (hs->flags & DT_F_TEXTURE) {
        double u, v;
        WK(c, DT_WK_TEX);
        int type = shape_uv(c, hit_i, isectP, &u, &v);
        if (type == 0) { free(shape_inds); return; }   /* Q8 */
        if (u < 0 || v < 0 || u > 1 || v > 1) {
          if (c->st) c->st->uv_out_of_range++;       /* reference terminates (870-877) */
        }
        if (type == 2) {
          shape_color = v3a(hs->bordercolor);
        } else if (type == 1) {
          const dt_texture_desc* T = &s->d->textures[hs->tex_frame];
          double dims0 = T->width, dims1 = T->height;
          int x_tex = (int)((float)((int)dims0 - 1) * (float)u);
          int y_tex = (int)((float)((int)dims1 - 1) * (float)v);
          int uv_ind = (int)(y_tex * dims0 + x_tex);
          if (uv_ind < 0) uv_ind = 0;
          if (uv_ind >= T->width * T->height) uv_ind = T->width * T->height - 1;
          const uint8_t* px = T->pixels + (size_t)uv_ind * T->channels;
          shape_color = v3(px[0] / 255.0, px[1] / 255.0, px[2] / 255.0);
        }
      }
      if (model >= 0 && model < 4) WK(c, DT_WK_BRDF + model);
      if (model == DT_MODEL_OREN_NAYAR) {  /* 894-913 */
        float A = (float)(1.0 - (0.5 * pow(roughness, 2)) / (pow(roughness, 2) + 0.33));
        float B = (float)((0.45 * pow(roughness, 2)) / (pow(roughness, 2) + 0.09));
        float vn = (float)dot(e, normal);
        float ln = (float)dot(sn, normal);
        float irradiance = fmaxr(0.0f, ln);
        float vn_theta = cr_acosf(vn);
        float ln_theta = cr_acosf(ln);
        float angleDiff = (float)dmax(0.0, dot(normalized(sub(e, mul(vn, normal))),
                                               normalized(sub(sray, mul(ln, normal)))));
        float alpha = fmaxr(vn_theta, ln_theta);
        float beta = fminr(vn_theta, ln_theta);
        float f = A + B * angleDiff * cr_sinf(alpha) * cr_tanf(beta);
        V3 sc_lc = v3(shape_color.x * lc.x, shape_color.y * lc.y, shape_color.z * lc.z);
        ray_col = mul(f, mul(irradiance, sc_lc));
      } else if (model == DT_MODEL_COOK_TORRANCE) {  /* 914-938 */
        V3 H = normalized(add(e, sray));
        float hn = (float)dmax(0.0, dot(normal, H));
        float vh = (float)dot(e, H);
        float vn = (float)dot(e, normal);
        float ln = (float)dot(sn, normal);
        float alpha = cr_acosf(hn);
        float D = (float)(1 / (pow(roughness, 2) * pow(cr_cosf(alpha), 4)) *
                          exp(-pow(cr_tanf(alpha) / roughness, 2)));
        float G1 = (float)(2.0 * hn * vn / vh);
        float G2 = (float)(2.0 * hn * ln / vh);
        float G = 1.0f;                       /* std::min({1, G1, G2}) */
        if (G1 < G) G = G1;
        if (G2 < G) G = G2;
        float F = schlick_complex(vn, hs->refr);
        float fdg = F * D * G;
        double den = (double)(ln * vn) * M_PI;
        V3 shader_rgb = add(mul(fmaxr(0.0f, ln), mul(0.4, lc)), divs(mul(fdg, mul(0.8, lc)), den));
        ray_col = v3(shape_color.x * shader_rgb.x, shape_color.y * shader_rgb.y,
                     shape_color.z * shader_rgb.z);
      } else if (model == DT_MODEL_RAW) {
        ray_col = shape_color;
      } else {  /* 943-948 */
        double m1 = dmax(0.0, dot(normal, sn));
        double p = pow(dmax(0.0, dot(r, e)), g->phong);
        V3 shader_rgb = add(mul(m1, lc), mul(p, lc));
        ray_col = v3(shape_color.x * shader_rgb.x, shape_color.y * shader_rgb.y,
                     shape_color.z * shader_rgb.z);
      }
      if (!is_approx_zero(ray_col)) {
        hits++;
        tmp_color = add(tmp_color, mul(k, ray_col));
      }
    }
    if (hits > 0) *color = add(*color, divs(tmp_color, hits));
  }
  free(shape_inds);
}

/* ======================================================================= */
/* renderImage / renderImageCloud pixel loops                               */
/* ======================================================================= */
typedef struct {
  V3 X, Y, Z, eye;
  float l, r, t, b;
  double mcam[4][4];
} Cam;

static void mat4_mul(const double A[4][4], const double B[4][4], double R[4][4])
{
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = A[i][0] * B[0][j];
      for (int k = 1; k < 4; ++k) s = s + A[i][k] * B[k][j];
      R[i][j] = s;
    }
}

static V3 mat4_point(const double M[4][4], V3 p)
{
  double ph[4] = {p.x, p.y, p.z, 1};
  double o[3];
  for (int i = 0; i < 3; ++i) {
    double s = M[i][0] * ph[0];
    for (int k = 1; k < 4; ++k) s = s + M[i][k] * ph[k];
    o[i] = s;
  }
  return v3(o[0], o[1], o[2]);
}

/* near plane (cpp:1024-1027) */
static void near_plane(const dt_globals* g, Cam* cam)
{
  cam->t = (float)(tan(g->fov * M_PI / 360.0) * fabsf(g->near_plane));
  cam->b = -cam->t;
  cam->r = g->aspect * cam->t;
  cam->l = -cam->r;
}

/* helpers.h:320-324 */
static V3 persp_eye_ray(const dt_globals* g, const Cam* cam, int i, int j)
{
  float a = cam->l + (cam->r - cam->l) * (float)i / (float)g->xRes;
  float b = cam->b + (cam->t - cam->b) * (float)j / (float)g->yRes;
  return sub(add(mul(a, cam->X), mul(b, cam->Y)), mul(g->near_plane, cam->Z));
}

/* pixel (x,y) of window/tile set -> output offset; returns -1 if not owned */
static long long out_offset(const dt_globals* g, const dt_tiles* T, int x, int y)
{
  int x0 = T->x0, y0 = T->y0;
  int x1 = T->x1 > 0 ? T->x1 : g->xRes, y1 = T->y1 > 0 ? T->y1 : g->yRes;
  if (x < x0 || x >= x1 || y < y0 || y >= y1) return -1;
  int tw = T->tile_w > 0 ? T->tile_w : 32, th = T->tile_h > 0 ? T->tile_h : 32;
  int world = T->world > 0 ? T->world : 1;
  int tiles_x = (x1 - x0 + tw - 1) / tw;
  int tx = (x - x0) / tw, ty = (y - y0) / th;
  long long tid = (long long)ty * tiles_x + tx;
  /* multi-GPU tile ownership (dt_scene_dev.h tile_of): group tid / world, ranks rotated by a hash */
  long long slot = tid / world;
  unsigned h = (unsigned)slot * 2654435761u;
  h ^= h >> 15;
  h *= 0x2c1b3c6du;
  h ^= h >> 12;
  if ((long long)(((unsigned)(tid % world) + (unsigned)world - h % (unsigned)world) % (unsigned)world) != T->rank) return -1;
  if (T->layout == DT_OUT_SLAB) {
    int px = (x - x0) % tw, py = (y - y0) % th;
    return ((slot * th + py) * tw + px) * 3;
  }
  return 3LL * ((long long)(g->yRes - 1 - y) * g->xRes + x);
}

int or_render_sky(const dt_globals* g0, float frame, const dt_tiles* tiles, float* out, int nthreads)
{
  dt_globals g = *g0;
  /* cpp:1227-1229 */
  g.eye[0] = 0.5; g.eye[1] = 1.5; g.eye[2] = 1;
  g.up[0] = 0; g.up[1] = 0; g.up[2] = 1;
  g.lookingAt[0] = 0.5; g.lookingAt[1] = -1; g.lookingAt[2] = 1;
  Cam cam;
  cam.eye = v3a(g.eye);
  cam.Z = neg(normalized(sub(v3a(g.lookingAt), cam.eye)));
  cam.X = normalized(cross(v3a(g.up), cam.Z));
  if (is_approx_zero(cam.X)) return DT_E_INVALID;
  cam.Y = normalized(cross(cam.Z, cam.X));
  near_plane(&g, &cam);
  /* cob rows X, Y, -Z (cpp:1262-1263) */
  double cob[4][4] = {{cam.X.x, cam.X.y, cam.X.z, 0},
                      {cam.Y.x, cam.Y.y, cam.Y.z, 0},
                      {-cam.Z.x, -cam.Z.y, -cam.Z.z, 0},
                      {0, 0, 0, 1}};
  double org[4][4] = {{1, 0, 0, -cam.eye.x}, {0, 1, 0, -cam.eye.y}, {0, 0, 1, -cam.eye.z}, {0, 0, 0, 1}};
  mat4_mul(cob, org, cam.mcam);
  int x0 = tiles->x0, y0 = tiles->y0;
  int x1 = tiles->x1 > 0 ? tiles->x1 : g.xRes, y1 = tiles->y1 > 0 ? tiles->y1 : g.yRes;
  long long npx = (long long)(x1 - x0) * (y1 - y0);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (long long q = 0; q < npx; ++q) {
    int x = x0 + (int)(q % (x1 - x0)), y = y0 + (int)(q / (x1 - x0));
    long long off = out_offset(&g, tiles, x, y);
    if (off < 0) continue;
    V3 rayDir = persp_eye_ray(&g, &cam, x, y);
    V3 point = mat4_point(cam.mcam, add(rayDir, cam.eye));
    double pr[3] = {point.x, point.y, point.z}, o[3] = {0, 0, 0}, col[3];
    or_cloud_color(&g, pr, o, frame, col);
    out[off + 0] = clampf01((float)col[0]) * 255.0f;
    out[off + 1] = clampf01((float)col[1]) * 255.0f;
    out[off + 2] = clampf01((float)col[2]) * 255.0f;
  }
  return DT_OK;
}

typedef struct {
  Scene scene;
  Cam cam;
  double new_mcam[4][4];
  int frame;
  int sampled_n;
} RenderCtx;

static int render_setup(RenderCtx* R, const dt_scene_desc* d, const dt_globals* g, int frame)
{
  scene_init(&R->scene, d, g);
  R->frame = frame;
  Cam* cam = &R->cam;
  cam->eye = v3a(g->eye);
  /* cpp:989-998 */
  cam->Z = neg(normalized(sub(v3a(g->lookingAt), cam->eye)));
  cam->X = normalized(cross(v3a(g->up), cam->Z));
  if (is_approx_zero(cam->X)) return DT_E_INVALID;
  cam->Y = normalized(cross(cam->Z, cam->X));
  /* cpp:1004-1021 */
  V3 newX = v3(0, 0, 0), newY = v3(0, 0, 0);
  if (frame >= g->frame_cloud) {
    V3 new_up = v3(-1, 0, 0);
    newX = normalized(cross(new_up, cam->Z));
    newY = normalized(cross(cam->Z, newX));
  }
  double cob[4][4] = {{cam->X.x, cam->X.y, cam->X.z, 0},
                      {cam->Y.x, cam->Y.y, cam->Y.z, 0},
                      {cam->Z.x, cam->Z.y, cam->Z.z, 0},
                      {0, 0, 0, 1}};
  double org[4][4] = {{1, 0, 0, -cam->eye.x}, {0, 1, 0, -cam->eye.y}, {0, 0, 1, -cam->eye.z}, {0, 0, 0, 1}};
  mat4_mul(cob, org, cam->mcam);
  double ncob[4][4] = {{newX.x, newX.y, newX.z, 0},
                       {newY.x, newY.y, newY.z, 0},
                       {cam->Z.x, cam->Z.y, cam->Z.z, 0},
                       {0, 0, 0, 1}};
  mat4_mul(ncob, org, R->new_mcam);
  near_plane(g, cam);
  int n = (int)sqrt(g->antialias_samples);
  R->sampled_n = (int)pow(n, 2);
  return DT_OK;
}

/* one sample of renderImage's inner loop (cpp:1062-1211) */
static void render_sample(const RenderCtx* R, const dt_globals* g, int x, int y, int i, V3* out,
                          int* out_hit, dt_stats* st, uint64_t* wk)
{
  const Cam* cam = &R->cam;
  Ctx c;
  c.s = &R->scene;
  c.st = st;
  c.wk = wk;
  WK(&c, DT_WK_CAMERA);
  c.shift = 0.0f;
  c.rng.key[0] = g->seed;
  c.rng.key[1] = (uint32_t)R->frame;
  c.rng.pixel = (uint32_t)(y * g->xRes + x);
  c.rng.sample = (uint32_t)i;
  /* getDOFSamples (cpp:195-210) */
  V3 eye_sample = cam->eye;
  if (g->aperture > 0) {
    double u0, u1;
    rng2(&c.rng, 0, P_DOF, 0, &u0, &u1);
    float r = (float)(g->aperture / 2 * u0);
    float theta = (float)(2 * M_PI * u1);
    eye_sample = add(add(cam->eye, mul(r * cr_cosf(theta), cam->X)), mul(r * cr_sinf(theta), cam->Y));
  }
  V3 rayDir = persp_eye_ray(g, cam, x, y);
  V3 focalPoint = add(cam->eye, mul(g->focal_length, rayDir));
  V3 tmp_color = v3(0, 0, 0);
  int hit = 0, motion = 0;
  ray_color(&c, sub(focalPoint, eye_sample), eye_sample, g->max_depth, &tmp_color, &hit, &motion, 1.0f,
            root_key(0));
  if (!hit) {
    if (g->perlin_cloud) {
      V3 point = mat4_point(R->frame >= g->frame_cloud ? R->new_mcam : cam->mcam, focalPoint);
      double pr[3] = {point.x, point.y, point.z}, o[3] = {0, 0, 0}, col[3];
      or_cloud_color(g, pr, o, (float)R->frame, col);
      tmp_color = v3a(col);
      if (st) st->sky_pixels++;
      WK(&c, DT_WK_SKY);
    } else {
      tmp_color = v3a(g->default_col);
    }
  }
  if (motion) { /* cpp:1095-1210 */
    for (int m = 0; m < g->blur_samples; m++) {
      double u0, u1;
      rng2(&c.rng, 0, P_BLUR, (uint32_t)m, &u0, &u1);
      float frame_sample = (float)((float)R->frame + u0 * g->frame_range);
      float val = 0.0f;  /* reference leaves val uninitialised below frame_prism (Q19) */
      if (R->frame >= g->frame_prism) {
        if (R->frame >= g->frame_blur)
          val = (float)(g->move_per_frame * (frame_sample - R->frame) +
                        g->accel_t * pow((frame_sample - R->frame), 3));
        else
          val = g->move_per_frame * (frame_sample - R->frame);
      }
      Ctx cm = c;
      cm.shift = val;
      WK(&c, DT_WK_CAMERA);
      V3 motion_color = v3(0, 0, 0);
      ray_color(&cm, sub(focalPoint, eye_sample), eye_sample, g->max_depth, &motion_color, &hit, &motion,
                1.0f, root_key(m + 1));
      if (!hit) {
        if (g->perlin_cloud) {
          V3 point = mat4_point(R->frame >= g->frame_cloud ? R->new_mcam : cam->mcam, focalPoint);
          double pr[3] = {point.x, point.y, point.z}, o[3] = {0, 0, 0}, col[3];
          or_cloud_color(g, pr, o, (float)R->frame, col);
          motion_color = v3a(col);
          WK(&c, DT_WK_SKY);
        } else {
          motion_color = v3a(g->default_col);
        }
      }
      tmp_color = add(tmp_color, motion_color);
    }
    tmp_color = divs(tmp_color, g->blur_samples + 1);
  }
  *out = tmp_color;
  if (out_hit) *out_hit = hit;
}

int or_sample_color(const dt_scene_desc* d, const dt_globals* g, int frame, int x, int y, int sample,
                    double out_color[3], int* out_hit)
{
  RenderCtx R;
  int rc = render_setup(&R, d, g, frame);
  if (rc == DT_OK) {
    V3 col;
    render_sample(&R, g, x, y, sample, &col, out_hit, NULL, NULL);
    out_color[0] = col.x; out_color[1] = col.y; out_color[2] = col.z;
  }
  scene_free(&R.scene);
  return rc;
}

/* The intersection micro-benchmark's reference (include/dt.h dt_intersect_primary): for primary rays
 * first .. first+n-1 (ray r: q = r / 8, pixel q mod W*H, sample r mod 8 + 8 (q div W*H)), the
 * camera ray of render_sample (getDOFSamples + getPerspEyeRay, cpp:195-210, 1062-1072) and
 * rayColor's gather + closest hit (cpp:491-538, ray_color above): the closest shape (-1: none)
 * and its t (FLT_MAX: none). */
int or_primary_hit(const dt_scene_desc* d, const dt_globals* g, int frame, long long first, long long n,
                   int* shape, float* t, int nthreads)
{
  RenderCtx R;
  int rc = render_setup(&R, d, g, frame);
  if (rc != DT_OK) { scene_free(&R.scene); return rc; }
  const long long npx = (long long)g->xRes * g->yRes;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    int* inds = (int*)malloc(sizeof(int) * (d->n_shapes > 0 ? d->n_shapes : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
    for (long long i = 0; i < n; ++i) {
      const long long r = first + i, q = r / 8, p = q % npx;
      const int x = (int)(p % g->xRes), y = (int)(p / g->xRes);
      const Cam* cam = &R.cam;
      Ctx c;
      c.s = &R.scene;
      c.st = NULL;
      c.wk = NULL;
      c.shift = 0.0f;
      c.rng.key[0] = g->seed;
      c.rng.key[1] = (uint32_t)frame;
      c.rng.pixel = (uint32_t)(y * g->xRes + x);
      c.rng.sample = (uint32_t)(r % 8 + 8 * (q / npx));
      V3 eye_sample = cam->eye;
      if (g->aperture > 0) {
        double u0, u1;
        rng2(&c.rng, 0, P_DOF, 0, &u0, &u1);
        float rr = (float)(g->aperture / 2 * u0);
        float theta = (float)(2 * M_PI * u1);
        eye_sample = add(add(cam->eye, mul(rr * cr_cosf(theta), cam->X)), mul(rr * cr_sinf(theta), cam->Y));
      }
      V3 focalPoint = add(cam->eye, mul(g->focal_length, persp_eye_ray(g, cam, x, y)));
      V3 ray = sub(focalPoint, eye_sample);
      int n_inds = bvh_gather(&c, ray, eye_sample, inds);
      float t_dist = FLT_MAX, t_min = FLT_MAX;
      int any = 0, hit_i = -1;
      for (int k = 0; k < n_inds; ++k) {
        int ins = 0, hole = -1;
        V3 hc;
        if (shape_intersect(&c, inds[k], ray, eye_sample, &t_dist, &ins, &hc, &hole)) {
          any = 1;
          if (t_dist < t_min) {
            hit_i = inds[k];
            t_min = t_dist;
          }
        }
      }
      const int hit = any && hit_i >= 0;
      shape[i] = hit ? hit_i : -1;
      t[i] = hit ? t_min : FLT_MAX;
    }
    free(inds);
  }
  scene_free(&R.scene);
  return DT_OK;
}

int or_render_work(const dt_scene_desc* d, const dt_globals* g, int frame, const dt_tiles* tiles, float* out,
                   int nthreads, dt_stats* stats, uint64_t* work);

int or_render(const dt_scene_desc* d, const dt_globals* g, int frame, const dt_tiles* tiles, float* out,
              int nthreads, dt_stats* stats)
{
  return or_render_work(d, g, frame, tiles, out, nthreads, stats, NULL);
}

/* or_render, also counting the include/dt_work.h events of the reference's loop into work[DT_WK_N] */
int or_render_work(const dt_scene_desc* d, const dt_globals* g, int frame, const dt_tiles* tiles, float* out,
                   int nthreads, dt_stats* stats, uint64_t* work)
{
  RenderCtx R;
  int rc = render_setup(&R, d, g, frame);
  if (rc != DT_OK) { scene_free(&R.scene); return rc; }
  int x0 = tiles->x0, y0 = tiles->y0;
  int x1 = tiles->x1 > 0 ? tiles->x1 : g->xRes, y1 = tiles->y1 > 0 ? tiles->y1 : g->yRes;
  long long npx = (long long)(x1 - x0) * (y1 - y0);
  dt_stats total;
  memset(&total, 0, sizeof(total));
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    dt_stats local;
    memset(&local, 0, sizeof(local));
    uint64_t wk[DT_WK_N];
    memset(wk, 0, sizeof(wk));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (long long q = 0; q < npx; ++q) {
      int x = x0 + (int)(q % (x1 - x0)), y = y0 + (int)(q / (x1 - x0));
      long long off = out_offset(g, tiles, x, y);
      if (off < 0) continue;
      V3 color = v3(0, 0, 0);
      for (int i = 0; i < R.sampled_n; i++) {
        V3 tc;
        render_sample(&R, g, x, y, i, &tc, NULL, &local, work ? wk : NULL);
        color = add(color, tc);
      }
      color = divs(color, R.sampled_n);
      local.pixels++;
      local.samples += R.sampled_n;
      out[off + 0] = clampf01((float)color.x) * 255.0f;
      out[off + 1] = clampf01((float)color.y) * 255.0f;
      out[off + 2] = clampf01((float)color.z) * 255.0f;
      if (isnan(out[off]) || isnan(out[off + 1]) || isnan(out[off + 2])) local.nan_pixels++;
    }
#ifdef _OPENMP
#pragma omp critical
#endif
    {
      total.pixels += local.pixels; total.samples += local.samples; total.rays += local.rays;
      total.shadow_rays += local.shadow_rays; total.sky_pixels += local.sky_pixels;
      total.uv_out_of_range += local.uv_out_of_range; total.glossy_exhausted += local.glossy_exhausted;
      total.spherelight_exhausted += local.spherelight_exhausted;
      total.prism_norm_fallback += local.prism_norm_fallback;
      total.reflect_errors += local.reflect_errors; total.nan_pixels += local.nan_pixels;
      if (work)
        for (int k = 0; k < DT_WK_N; ++k) work[k] += wk[k];
    }
  }
  if (stats) *stats = total;
  scene_free(&R.scene);
  return DT_OK;
}
