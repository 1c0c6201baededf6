// dt_kernels.hip — gfx950 (CDNA4) kernels for the distraytracer per-pixel render loop.
//
// Reference hot path: renderImage pixel/sample loop (render_final_project.cpp:1031-1218),
// rayColor (487-961), cloudColor/skyColor (146-192), noise.h, geometry.cpp primitives.
// Design:
//   * one wave64 = the samples of one pixel (spp >= 64: 64 samples per chunk) or of
//     64/spp pixels: the 64 lanes shoot nearly identical primary rays (same pixel, DoF
//     jitter only), so BVH traversal, shape dispatch and shading stay wave-coherent;
//   * BVH traversal is stackless and WAVE-UNIFORM over the reference's static pre-order:
//     node/shape data are read with uniform indices (scalar loads), each lane keeps one
//     int "resume" index, a __ballot decides descend/skip. Per-lane visit order equals the
//     reference's gather order, so closest-hit ties resolve identically;
//   * rayColor's recursion tree runs as a per-lane DFS on a private stack in pre-order,
//     with a FINISH entry per node so each node's own light is added after its children,
//     exactly as the reference's `color +=` order;
//   * a persistent grid dequeues pixel groups from an atomic counter;
//   * sky (cloudColor, 200-step value-noise march) is per-pixel deterministic (Q4): it is
//     computed once per pixel by all 64 lanes cooperatively, only for pixels with misses.
// Numerics: FP64 wherever the reference uses VEC3/double, FP32 where it declares float,
// compiled with -ffp-contract=off (no FMA contraction), correctly rounded div/sqrt.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dt.h"
#include "../../include/dt_work.h"
#include "dt_math.h"
#include "dt_scene_dev.h"

using namespace dtm;
using namespace dtd;

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

// diagnostic build (-DDT_STAMPS): per-phase cycle sums and wave-level event counts
#ifdef DT_STAMPS
#define DT_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define DT_ACC(k, a, b) cnt.ph[k] += (b) - (a)
#define DT_PH_N 72   // stamp slots (dt_api.cpp DT_N_STAMPS, tools/stamps.py)
#define DT_CNT(k) cnt.ph[k] += 1   // wave-uniform event count (7 DFS steps, 8 prim tests, 9 lights)
#else
#define DT_CNT(k)
#define DT_T(v)
#define DT_ACC(k, a, b)
#endif

// Work counters (include/dt_work.h: the §8(d) event counts the VALU roofline prices): compiled in
// only with -DDT_WORK_COUNTERS (the diagnostic library libdt_work.so; in the traversal loops they
// cost several %). DT_WK(k, cond) adds the number of executing lanes with `cond` to event k: one
// lane (the lowest such) adds the ballot's popcount to the wave's LDS counter, so the call sites may
// sit in divergent code. Flushed to the stats block (dt_debug_counters) at kernel exit.
#ifdef DT_WORK_COUNTERS
#define DT_WORK(...) __VA_ARGS__
#define DT_WK(k, cond)                                                                   \
  do {                                                                                   \
    const unsigned long long m_ = __ballot(cond);                                        \
    if (m_ && (int)(threadIdx.x & 63) == (int)__builtin_ctzll(m_)) cnt.wk[(k)] += (unsigned)__popcll(m_); \
  } while (0)
#else
#define DT_WORK(...)
#define DT_WK(k, cond) do { } while (0)
#endif

// DT_WITH_RPC=1 (the second compilation of this file, build/dt_kernels_rpc.o): the trace kernel
// dt_trace_kernel_rpc for scenes holding a RectPrismWithCylinder, with that shape's tests and no
// t-culling (DParams::no_cull). Its code stays out of the hot dt_trace_kernel, whose register
// allocation it would disturb (VGPR spills 196 -> 258 when compiled in).
#ifndef DT_WITH_RPC
#define DT_WITH_RPC 0
#endif
// DT_DONATE=1 (a third compilation, build/dt_kernels_dn.o): dt_trace_kernel_dn, whose idle lanes take
// whole pending subtrees from lanes with deep DFS trees (see "DFS work sharing" below)
#ifndef DT_DONATE
#define DT_DONATE 0
#endif
// DT_ISECT=1 (a fourth compilation, build/dt_kernels_isect.o): only dt_isect_kernel, the intersection
// micro-benchmark, so that its call sites of the shared device functions stay out of the trace kernel's
// object
#ifndef DT_ISECT
#define DT_ISECT 0
#endif
// DT_W5=1 (build/dt_kernels_w5.o): the trace kernel at 5 waves per SIMD (96 VGPRs, under 8 KiB of
// LDS per wave: DT_PSUM_LDS=2), launched for one-pixel-per-wave work (spp >= 64; never
// with more than 8 pixels per wave, the slots DT_PSUM_LDS=2 keeps)
#ifndef DT_W5
#define DT_W5 0
#endif
// DT_NOSHIFT=1 (build/dt_kernels.o, build/dt_kernels_w5.o): the product kernels for frames without
// motion-blur shifts (frame < frame_prism, where the reference's blur value is 0, Q19: C1-C4 and
// C5's room frames). shift is the constant 0, so the bump walks, bump lists and shifted shape tests
// compile away. DT_NOSHIFT=0 (build/dt_kernels_blur.o, build/dt_kernels_w5_blur.o): the same kernels
// with every shift path, named *_blur, for frames >= frame_prism (dt_api.cpp picks per launch).
#ifndef DT_NOSHIFT
#define DT_NOSHIFT 0
#endif
// DT_SKY_AGAIN: the still builds carry no cooperative sky march (its noise code took ~95 of the
// 5-wave build's 133 spilled VGPRs). A multi-sample item with a missed sample is listed instead of
// stored, and a second launch of the *_sky build of the same wave count (DT_SKY_BUILD: still frames,
// every feature, the march; its queue runs over the list, DT_AGAIN_QUEUE) renders the listed items
// again from the same counter-RNG draws (dt_api.cpp enqueue_render; P.sky_again). Room scenes never
// miss. Diagnostic builds (work counters, stamps) keep the march so their counts stay one launch's.
#ifndef DT_SKY_BUILD
#define DT_SKY_BUILD 0
#endif
#if DT_NOSHIFT && !DT_SKY_BUILD && !defined(DT_WORK_COUNTERS) && !defined(DT_STAMPS)
#define DT_SKY_AGAIN 1
#else
#define DT_SKY_AGAIN 0
#endif
#define DT_AGAIN_QUEUE DT_SKY_BUILD
// DT_CHUNK_ITEMS=1 (every build): the build can run chunk items (P.chunk_items, spp > 64: a pixel's
// 64-sample chunks on different waves); dt_api.cpp reads the trait bit. A/B switch: the 5-wave room
// build without the code ran C3 1.3% slower (register allocation: 3872 against 3920 Mpixel-samples/s,
// profiles/r06d_*), so it stays in.
#ifndef DT_CHUNK_ITEMS
#define DT_CHUNK_ITEMS 1
#endif
// DT_FEATURES: the scene features a build handles (dt_scene_dev.h: bit t for shape type t,
// DT_FEAT_SPHL sphere lights and emitters, DT_FEAT_RECTL rectangle lights and emitters, DT_FEAT_ON
// Oren-Nayar, DT_FEAT_GLASS refraction). A build without some of them has those cases compiled out;
// dt_api.cpp launches it only for scenes whose feature mask it covers.
#ifndef DT_FEATURES
#define DT_FEATURES 0xFFFFu
#endif
#define DT_HAS(bit) (((DT_FEATURES) >> (bit)) & 1u)
#define DT_NEED(bit) do { if (!DT_HAS(bit)) __builtin_unreachable(); } while (0)
// DT_KNAME: the kernel's name, per build (Makefile TRACE_BUILDS: work sharing, RectPrismWithCylinder,
// and the product kernels at 4 and 5 waves per SIMD for still frames of room scenes (C2, C3, C5's
// room frames), of room scenes with meshes (*_mesh: C4), of any scene (*_full), for frames with
// motion-blur shifts in tunnel scenes (*_tunnel) and in any scene (*_blur), and the *_sky builds
// that render the items the still builds list)
#ifdef DT_KNAME
#define DT_TRACE_KERNEL DT_KNAME
#elif DT_WITH_RPC
#define DT_TRACE_KERNEL dt_trace_kernel_rpc
#elif DT_DONATE
#define DT_TRACE_KERNEL dt_trace_kernel_dn
#elif DT_W5
#define DT_TRACE_KERNEL dt_trace_kernel_w5
#else
#define DT_TRACE_KERNEL dt_trace_kernel
#endif
// DT_HELPERS=1 (the 4-wave room build): also the small kernels and the launch-record helpers
#ifndef DT_HELPERS
#define DT_HELPERS 0
#endif

#define DT_STACK_MAX 48
#define DT_MAX_CLOUD_STEPS 2048
#define DT_CLOUD_CHUNK 256
#define DT_WAVE 64
// Measured-and-dropped variants are not kept here (DESIGN.md §8 lists them with their A/B logs;
// git history holds their code). The switches left select the four instantiations (Makefile).
#define DT_PRIO_LEVEL 3    // issue priority of long DFS items (P.prio_steps, dt_api.cpp)
#ifndef DT_PSUM_LDS
#define DT_PSUM_LDS 1   // per-pixel sums in LDS: 1 for up to 64 pixels per wave, 2 for up to 8 (DT_W5)
#endif

enum { ST_RAYS = 0, ST_SHADOW = 1, ST_SKY = 2, ST_UV = 3, ST_GLOSSY = 4, ST_SPHL = 5, ST_PRISM = 6,
       ST_REFL = 7, ST_NAN = 8, ST_PIXELS = 9, ST_SAMPLES = 10, ST_STACK = 11, ST_TEX = 12, ST_BOX = 13, ST_PRIM = 14, ST_WNODES = 15,
       ST_DONATE = 16, ST_DN_OVF = 17, ST_N = 18 };

__constant__ uint32_t c_primes[10][3] = {
    {995615039u, 600173719u, 701464987u}, {831731269u, 162318869u, 136250887u},
    {174329291u, 946737083u, 245679977u}, {362489573u, 795918041u, 350777237u},
    {457025711u, 880830799u, 909678923u}, {787070341u, 177340217u, 593320781u},
    {405493717u, 291031019u, 391950901u}, {458904767u, 676625681u, 424452397u},
    {531736441u, 939683957u, 810651871u}, {997169939u, 842027887u, 423882827u}};

// Read-only scene arrays are accessed through the constant address space: with a wave-uniform
// index (BVH walk, leaf shapes, lights) the compiler emits scalar s_load's into SGPRs
// (scalar cache), with a per-lane index (hit-shape shading) ordinary vector loads.
#if defined(__HIP_DEVICE_COMPILE__)
#define DT_CAS __attribute__((address_space(4)))
#else
#define DT_CAS
#endif
template <class T>
__device__ __forceinline__ const DT_CAS T* cas(const T* p)
{
  return (const DT_CAS T*)p;
}
typedef const DT_CAS double* GP;

struct DScene {
  const DNodeDev* nodes;    // the reference's tree (general walks)
  const DNodeDev* fnodes;   // same leaves, SAH inner nodes (host_fasttree.cpp; fast walks)
  const uint32_t* sg_cells; // shadow grid (host_shadowgrid.cpp): (offset, count) per light x cell
  const int32_t* sg_list;   // candidate occluder leaves (indices into nodes)
  const int32_t* leaf_idx;
  const DShapeHdr* hdr;
  const double* geom;
  const DMat* mat;
  const DLight* lights;
  const uint8_t* tex;
  const float* cloud_z;   // float z sequence of cloudColor's loop (cpp:172)
  unsigned long long* stats;
  unsigned long long* queue;
  const DNodeDev* bnodes;   // bump tree for motion-blur passes (host_fasttree.cpp; leaf skip = reference index)
  const int32_t* bparent;   // parent of every reference node (-1: root)
  const uint32_t* pl_cells; // primary-ray candidate lists (host_primlists.cpp): (first, count) per pixel block
  const uint32_t* pl_list;  // (fast-tree node, float bits of t_near) per entry
  uint8_t* sky_miss;        // P.sky_defer: per queue position, 1 when the pixel's sample missed
  void* dn_pool;            // P.donate: DT_DN_POOL_REC records of 32 B per resident wave (DFS work sharing)
  uint32_t* again_list;     // P.sky_again: the items a launch without the sky left to a launch with it
  unsigned int* again_n;    // ... and their count
  const DNodeDev* sub_nodes;   // shadow-grid block subtrees (host_shadowgrid.cpp; P.sgb_*)
  const uint32_t* sub_blocks;  // (first node, node count) per (light, block); count 0: none
  // counters of the scene's next launch (the other parity, dt_api.cpp), zeroed by workgroup 0: none of
  // this launch's waves touches them, so no per-launch memset (a blit kernel) has to run between frames
  unsigned long long* clear0;
  unsigned long long* clear1;
  int32_t n_clear0, n_clear1;
  // P.chunk_items (spp > 64): per pixel item, its spp sample colours (3 doubles each, sample order),
  // stored by the chunk items that traced them and added up by dt_chunk_sum_kernel
  double* chunk_cols;
  // diagnostic builds (-DDT_ITEM_TIMES=2, DT_ITEM_COSTS=1): per queue code, the item's duration on the
  // 100 MHz clock (dt_debug_item_costs, tools/chunk_costs.py); null otherwise
  uint32_t* item_cost;
  void* pad_;   // (keeps sizeof(DScene) a multiple of 16: DLaunch::P at the offset it had)
};

// pow(x, n) for the integer exponents the reference writes as pow(x, 2.0) etc. pow(x, 1) is x
// and pow(x, 2) is the correctly rounded x*x (glibc's pow is correctly rounded for these,
// OCML's pow_f64 is not, and its inlined body was the largest source of register spills);
// higher powers by repeated multiplication (<= 8 roundings, ~1e-14 relative, far inside the
// 1e-4 parity bound).
__device__ __forceinline__ double pw1(double x) { return x; }
__device__ __forceinline__ double pw2(double x) { return x * x; }
__device__ __forceinline__ double pw3(double x) { return (x * x) * x; }
__device__ __forceinline__ double pw4(double x) { double x2 = x * x; return x2 * x2; }
__device__ __forceinline__ double pw5(double x) { double x2 = x * x; return (x2 * x2) * x; }
__device__ __forceinline__ double pw8(double x) { double x2 = x * x, x4 = x2 * x2; return x4 * x4; }
__device__ __forceinline__ double pw256(double x)
{
#pragma unroll
  for (int i = 0; i < 8; ++i) x = x * x;
  return x;
}
// pow(x, y) for a runtime exponent (the Phong exponent): small non-negative integers by
// binary powering, anything else through pow.
__device__ __forceinline__ double pw_rt(double x, double y)
{
  if (y >= 0 && y <= 64 && y == (double)(int)y) {
    int n = (int)y;
    double r = 1.0, b = x;
    while (n) {
      if (n & 1) r = r * b;
      n >>= 1;
      if (n) b = b * b;
    }
    return r;
  }
  return pow(x, y);
}

// The reference's float libm calls (cosf/sinf/tanf/acosf through <cmath>'s float overloads)
// are evaluated correctly rounded, as f32(f64 function): the reference's float libm is
// platform dependent (glibc's cosf is not correctly rounded either) and its float quadratic
// solves amplify a 1-ulp difference in a DoF offset into ~30 ulp of a hit distance. The oracle
// uses the same definition (oracle.c cr_cosf...), so both sides agree bit for bit.
// sin/cos of a float argument: Cody-Waite reduction by pi/2 in f64 (exact for |x| < 1e5: k*PIO2_1
// is exact with a 33-bit PIO2_1) and Taylor polynomials to r^17/r^16 on |r| <= pi/4 (truncation
// < 1e-19). The f64 result is within ~1e-16 of sin/cos, so rounding it to f32 gives the same
// float as f32(glibc sin/cos) (checked on 5e7 arguments in [0, 2pi): no mismatch).
__device__ __forceinline__ void cr_sincos_d(float xf, double& s_out, double& c_out)
{
  if (!(fabsf(xf) < 1e5f)) {   // large or non-finite: the library path
    s_out = sin((double)xf);
    c_out = cos((double)xf);
    return;
  }
  const double PIO2_1 = 1.57079632673412561417e+00, PIO2_1T = 6.07710050650619224932e-11;
  const double x = xf;
  const double k = rint(x * 0.63661977236758134308);
  const double r = (x - k * PIO2_1) - k * PIO2_1T;
  const double r2 = r * r;
  const double sp = r + r * r2 * (-1.0 / 6 + r2 * (1.0 / 120 + r2 * (-1.0 / 5040 + r2 * (1.0 / 362880 +
                    r2 * (-1.0 / 39916800 + r2 * (1.0 / 6227020800.0 + r2 * (-1.0 / 1307674368000.0 +
                    r2 * (1.0 / 355687428096000.0))))))));
  const double cp = 1 + r2 * (-0.5 + r2 * (1.0 / 24 + r2 * (-1.0 / 720 + r2 * (1.0 / 40320 + r2 * (-1.0 / 3628800 +
                    r2 * (1.0 / 479001600 + r2 * (-1.0 / 87178291200.0 + r2 * (1.0 / 20922789888000.0))))))));
  const int q = ((int)k) & 3;
  s_out = q == 0 ? sp : q == 1 ? cp : q == 2 ? -sp : -cp;
  c_out = q == 0 ? cp : q == 1 ? -sp : q == 2 ? -cp : sp;
}
__device__ __forceinline__ float cr_cosf(float x) { double s, c; cr_sincos_d(x, s, c); return (float)c; }
__device__ __forceinline__ float cr_sinf(float x) { double s, c; cr_sincos_d(x, s, c); return (float)s; }
// tan as sin/cos of the same reduction (one correctly rounded f64 division: within ~3e-16)
__device__ __forceinline__ float cr_tanf(float x) { double s, c; cr_sincos_d(x, s, c); return (float)(s / c); }
__device__ __forceinline__ float cr_acosf(float x) { return (float)acos((double)x); }

// =====================================================================================
// value noise (noise.h:25-136) and sky (render_final_project.cpp:146-192)
// =====================================================================================
__device__ __forceinline__ double noise3d(int i, int x, int y, int z)
{
  // (int)(x + y*57 + z*pow(57,2)) is an exact integer for in-range lattice coordinates
  int n = x + y * 57 + z * 3249;
  uint32_t un = (uint32_t)n;
  un = (un << 13) ^ un;
  uint32_t t = (un * (un * un * c_primes[i][0] + c_primes[i][1]) + c_primes[i][2]) & 0x7fffffffu;
  // (double)t / 1073741823 without the division: q0 = t * RN(1/c) corrected by one fma residual
  // step is the correctly rounded quotient for every t in [0, 2^31) (checked exhaustively,
  // tools/noise_div_check.c, tests/test_noise_division.py)
  const double c = 1073741823.0, r = 1.0 / 1073741823.0;
  const double td = (double)(int)t;
  const double q0 = td * r;
  return 1.0 - fma(fma(-c, q0, td), r, q0);
}

// noise.h:51-70, summation order preserved term by term
__device__ __forceinline__ double smoothed3d(int i, int x, int y, int z)
{
#define N(dx, dy, dz) noise3d(i, x + (dx), y + (dy), z + (dz))
  double corners = N(-1, -1, -1) + N(1, -1, -1) + N(-1, 1, -1) + N(1, 1, -1) + N(-1, -1, 1) +
                   N(1, -1, 1) + N(-1, 1, 1) + N(1, 1, 1);
  double sides = N(-1, 0, 0) + N(1, 0, 0) + N(0, 1, 0) + N(0, -1, 0) + N(0, 0, -1) + N(0, 0, 1);
  double dgsides = N(-1, 0, -1) + N(1, 0, -1) + N(0, 1, -1) + N(0, -1, -1) + N(-1, 0, 1) +
                   N(1, 0, 1) + N(0, 1, 1) + N(-1, -1, 0) + N(0, -1, 1) + N(1, -1, 0) +
                   N(-1, 1, 0) + N(1, 1, 0);
  double center = N(0, 0, 0);
#undef N
  const double alpha = 9.0 / 18, beta = 2.0 / (8 * 18), gamma = 4.0 / (6 * 18),
               delta = 3.0 / (12 * 18);
  return alpha * center + beta * corners + gamma * sides + delta * dgsides;
}

__device__ __forceinline__ double cos_f(double x) { return (1 - cos(x * M_PI)) * 0.5; }
__device__ __forceinline__ double lerp_f(double a, double b, double f) { return a * (1 - f) + b * f; }

// noise.h:81-107; cos(angle) of the same fractional part is evaluated once (same bits)
__device__ double interpolated_noise3d(int i, double x, double y, double z)
{
  int ix = (int)x, iy = (int)y, iz = (int)z;
  double fx = x - ix, fy = y - iy, fz = z - iz;
  double v1 = smoothed3d(i, ix, iy, iz);
  double v2 = smoothed3d(i, ix + 1, iy, iz);
  double v3_ = smoothed3d(i, ix, iy + 1, iz);
  double v4 = smoothed3d(i, ix + 1, iy + 1, iz);
  double v5 = smoothed3d(i, ix, iy, iz + 1);
  double v6 = smoothed3d(i, ix + 1, iy, iz + 1);
  double v7 = smoothed3d(i, ix, iy + 1, iz + 1);
  double v8 = smoothed3d(i, ix + 1, iy + 1, iz + 1);
  double cx = cos_f(fx), cy = cos_f(fy), cz = cos_f(fz);
  double w1 = lerp_f(v5, v6, cx), w2 = lerp_f(v7, v8, cx);
  double w3 = lerp_f(v1, v2, cx), w4 = lerp_f(v3_, v4, cx);
  double i1 = lerp_f(w3, w4, cy), i2 = lerp_f(w1, w2, cy);
  return lerp_f(i1, i2, cz);
}

// noise.h:124-136 (4 octaves; frequency 8,4,2,1 and amplitude .125,.25,.5,1 are exact)
__device__ double value_noise3d(double x, double y, double z)
{
  double total = 0;
  double frequency = 16.0, amplitude = 0.0625;
  for (int i = 0; i < 4; ++i) {
    frequency /= 2;
    amplitude /= 0.5;
    total += interpolated_noise3d(i, x * frequency, y * frequency, z * frequency) * amplitude;
  }
  return total;
}

// render_final_project.cpp:146-162
__device__ V3 sky_color(const DParams& P, V3 ray)
{
  V3 color = v3(0, 0, 0);
  V3 rnorm = normalized(ray);
  V3 sun = v3a(P.sun);
  float sundot = clampf01((float)dot(rnorm, sun));
  double sd = sundot;
  double p1 = pw1(sd), p2 = pw2(sd), p256 = pw256(sd);
  V3 term = add(add(mul(p1, mul(0.05, v3a(P.sun_outer))), mul(p2, mul(0.1, v3a(P.sun_inner)))),
                mul(p256, mul(0.9, v3a(P.sun_core))));
  color = add(color, term);
  double p8 = pw8(sd);
  V3 sky = add(mul(1 - 1.5 * p8, v3a(P.bluesky)), mul(p8, mul(1.5, v3a(P.redsky))));
  color = add(color, mul(1.0 - 0.8 * rnorm.y, sky));
  return color;
}

// one march step of cloudColor (cpp:172-185): density, or -1 when the step adds nothing
__device__ __forceinline__ float cloud_step(const DParams& P, float z, V3 ray)
{
  V3 p = add(v3(0, 0, 0), mul(z, ray));
  float noise = (float)(0.7 * value_noise3d(p.x, p.y, p.z + P.frame_f));
  float cd = (float)((p.y + noise) + P.cloudhoff);
  if (cd < 0) return clampf01(fabsf(cd));
  return -1.0f;
}

__device__ __forceinline__ double cloud_apply(double c, double skyrev, float density)
{
  double cloudcolor = 1 - density * skyrev;
  return (1 - density * 0.4) * c + density * 0.4 * cloudcolor;
}

// cpp:187-191 contrast + saturation
__device__ V3 cloud_finish(const DParams& P, V3 color)
{
  color = v3(clampf01((float)color.x), clampf01((float)color.y), clampf01((float)color.z));
  color = sub(mul(3, v3(pw2(color.x), pw2(color.y), pw2(color.z))),
              mul(2, v3(pw3(color.x), pw3(color.y), pw3(color.z))));
  double s = (color.x + color.y) + color.z;
  V3 grey = v3(0.33 * s, 0.33 * s, 0.33 * s);
  return sub(mul(1 + P.saturation, color), mul(P.saturation, grey));
}

// The cloud band of one march step (cpp:175-179), decided without the noise where its bound
// settles it. |ValueNoise_3D| <= 1.875 (4 octaves of amplitudes 1/8..1; each Smoothed3D is a
// convex combination of Noise3D values in [-1.0000000019, 1], each cosInterpolate a convex
// combination), so |noise| = |float(0.7 * vn)| <= 1.3125002. With yh = p.y + cloudhoff:
//   yh >= 1.3126:  clouddistance >= 9.9e-5 > 0, the step adds nothing;
//   yh <= -2.3126: clouddistance <= -1.00009, so density = clamp(|cd|) = 1 exactly.
// The margins dwarf the roundings of the two double additions and the float conversion
// (about |p.y| * 2^-52, below 1e-9 for any |p.y| < 1e6; a NaN yh fails both tests and marches).
// Only steps in between evaluate the noise.
#define DT_CLOUD_ABOVE 1.3126
#define DT_CLOUD_BELOW (-2.3126)

// DT_SKY_CALL=1: the two cloudColor entry points below emitted as real calls instead of inlined
// (csrc/Makefile: the tunnel and blur builds, whose cooperative march would otherwise shape the
// trace kernel's register allocation: VGPR spills 158 -> 71 in the 5-wave blur build). The called
// march used to return wrong colours: the cause was -mllvm -disable-machine-cse, no longer among
// the code-generation flags (tools/call_repro, tests/test_codegen.py).
#ifndef DT_SKY_CALL
#define DT_SKY_CALL 0
#endif
#if DT_SKY_CALL
#define DT_SKY_FN __noinline__
#else
#define DT_SKY_FN __forceinline__
#endif

// full cloudColor on one lane
__device__ DT_SKY_FN V3 cloud_color_lane(const DParams& P, const float* __restrict__ zs, V3 ray)
{
  V3 sky = sky_color(P, ray);
  V3 color = sky;
  for (int s = 0; s < P.n_cloud_steps; ++s) {
    const float z = zs[s];
    const double yh = (double)z * ray.y + (double)P.cloudhoff;
    if (yh >= DT_CLOUD_ABOVE) continue;
    float d = yh <= DT_CLOUD_BELOW ? 1.0f : cloud_step(P, z, ray);
    if (d >= 0.0f) {
      color.x = cloud_apply(color.x, sky.z, d);
      color.y = cloud_apply(color.y, sky.y, d);
      color.z = cloud_apply(color.z, sky.x, d);
    }
  }
  return cloud_finish(P, color);
}

// cloudColor for one (wave-uniform) ray computed by all 64 lanes: the march steps are
// spread over lanes (the noise is 99% of the work), the per-channel recurrence then runs
// on lanes 0..2 in step order, so every addition happens in the reference's order.
__device__ DT_SKY_FN V3 cloud_color_coop(const DParams& P, const float* __restrict__ zs, V3 ray,
                               float* __restrict__ dens, double* __restrict__ chan)
{
  // the march in chunks of DT_CLOUD_CHUNK steps: densities in parallel over the lanes, then
  // the per-channel recurrence on lanes 0-2 in step order (same arithmetic as one pass)
  const int lane = (int)(threadIdx.x & 63);
  V3 sky = sky_color(P, ray);
  double c = lane == 0 ? sky.x : (lane == 1 ? sky.y : sky.z);
  const double rev = lane == 0 ? sky.z : (lane == 1 ? sky.y : sky.x);
  for (int s0 = 0; s0 < P.n_cloud_steps; s0 += DT_CLOUD_CHUNK) {
    const int n = P.n_cloud_steps - s0 < DT_CLOUD_CHUNK ? P.n_cloud_steps - s0 : DT_CLOUD_CHUNK;
    for (int s = lane; s < n; s += DT_WAVE) dens[s] = cloud_step(P, zs[s0 + s], ray);
    __syncthreads();
    if (lane < 3) {
      for (int s = 0; s < n; ++s) {
        float d = dens[s];
        if (d >= 0.0f) c = cloud_apply(c, rev, d);
      }
    }
    __syncthreads();
  }
  if (lane < 3) chan[lane] = c;
  __syncthreads();
  V3 col = v3(chan[0], chan[1], chan[2]);
  __syncthreads();
  return cloud_finish(P, col);
}

// Philox products as one 32x32->64 multiply each (v_mad_u64_u32) instead of mul_hi + mul_lo: C3
// +0.9%, C2 +0.3%, but C4 -0.6% (the mesh builds keep mul_hi/mul_lo: csrc/Makefile MESH), the same
// words (profiles/r05y_ab_philox_mad64.txt; round 3, less VALU-bound, measured it neutral)
#ifndef DT_PHILOX_MAD64
#define DT_PHILOX_MAD64 1
#endif
// =====================================================================================
// counter RNG: Philox4x32-10 (oracle/oracle.c or_philox4x32)
// =====================================================================================
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                       uint32_t k1, uint32_t o[4])
{
#pragma unroll
  for (int r = 0; r < 10; ++r) {
#if DT_PHILOX_MAD64
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#else
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
#endif
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3;
}
__device__ __forceinline__ double u01(uint32_t w0, uint32_t w1)
{
  return ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ uint32_t fmix32(uint32_t h)
{
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t root_key(int pass) { return fmix32(0x12345678u + (uint32_t)pass); }
__device__ __forceinline__ uint32_t child_key(uint32_t parent, int slot)
{
  return fmix32(parent * 0x9E3779B1u + (uint32_t)slot + 1u);
}
enum { P_DOF = 1, P_LIGHT = 2, P_SPHL = 3, P_GLOSSY = 4, P_BLUR = 5 };

struct Rng {
  uint32_t k0, k1, pixel, sample;
  __device__ void draw_words(uint32_t node, uint32_t purpose, uint32_t sub, uint32_t o[4]) const
  {
    // opaque key: the 10-round key schedule is recomputed per draw (20 SALU adds) instead of
    // being hoisted into 20 SGPRs that stay live across the whole kernel and spill
    uint32_t a = __builtin_amdgcn_readfirstlane(k0), b = __builtin_amdgcn_readfirstlane(k1);   // uniform key
    asm volatile("" : "+s"(a), "+s"(b));
    philox(pixel, sample, node, (purpose << 24) | sub, a, b, o);
  }
  __device__ void draw(uint32_t node, uint32_t purpose, uint32_t sub, double& u0, double& u1) const
  {
    uint32_t o[4];
    draw_words(node, purpose, sub, o);
    u0 = u01(o[0], o[1]);
    u1 = u01(o[2], o[3]);
  }
};

// one 32-bit word as the float the reference gets from (float)uniform(generator)
__device__ __forceinline__ float f01(uint32_t w) { return (float)((double)w * (1.0 / 4294967296.0)); }

// =====================================================================================
// primitives (geometry.cpp), geometry from the precomputed pool
// =====================================================================================
__device__ __forceinline__ V3 v3a(GP a) { return v3(a[0], a[1], a[2]); }
__device__ __forceinline__ V3 G3(GP g, int o) { return v3(g[o], g[o + 1], g[o + 2]); }

// Rectangle plane + quad bounds test (geometry.cpp:640-741 / 2292-2312): R record
// tlim: the caller discards t >= tlim (shadow tests: t_max), so such planes may be rejected early
// A: the corner, R_A of the record unless a motion-blur pass moved it (shifted_exact)
__device__ __forceinline__ bool rect_hit_RA(GP R, V3 A, V3 ray, V3 start, float eps,
                                            float& t_out, float& ch1, float& ch2, float tlim = INFINITY)
{
  V3 n = G3(R, R_N);
  float dn = (float)dot(ray, n);
  if (dn == 0) return false;
  const double num = dot(sub(A, start), n);
  // t = num/dn <= 0 < eps whenever the signs differ or num is 0: reject before the f64
  // division (identical outcome; a NaN num still reaches the division and fails below)
  if ((num > 0) != (dn > 0) && !(num != num)) return false;
  // |num| >= |dn| tlim (1 + 2^-20) puts num/dn, and its f32 rounding, at or past tlim;
  // |num| <= |dn| eps (1 - 2^-20) puts it at or below eps: both decided without the division
  {
    const double an = fabs(num), ad = fabs((double)dn);
    if (an >= ad * (double)tlim * (1.0 + 0x1p-20)) return false;
    if (an <= ad * (double)eps * (1.0 - 0x1p-20)) return false;
  }
  float t_final = (float)(num / dn);
  if (t_final <= eps) return false;
  V3 point = add(start, mul(t_final, ray));
  V3 V_hit = sub(point, A);
  float check1 = (float)dot(G3(R, R_V1N), V_hit);
  float check2 = (float)dot(G3(R, R_V2N), V_hit);
  if (0 <= check1 && check1 <= R[R_LEN1] && 0 <= check2 && check2 <= R[R_LEN2]) {
    t_out = t_final;
    ch1 = check1;
    ch2 = check2;
    return true;
  }
  return false;
}
__device__ __forceinline__ bool rect_hit_R(GP R, V3 ray, V3 start, float eps,
                                           float& t_out, float& ch1, float& ch2, float tlim = INFINITY)
{
  return rect_hit_RA(R, G3(R, R_A), ray, start, eps, t_out, ch1, ch2, tlim);
}

// same, R computed from (shifted) raw vertices — motion-blur retraces of "rectangle" shapes
__device__ bool rect_hit_raw(V3 A, V3 B, V3 C, V3 D, V3 ray, V3 start, float eps, float& t_out)
{
  V3 n = normalized(normalized(cross(sub(B, A), sub(C, A))));
  float dn = (float)dot(ray, n);
  if (dn == 0) return false;
  float t_final = (float)(dot(sub(A, start), n) / dn);
  if (t_final <= eps) return false;
  V3 point = add(start, mul(t_final, ray));
  V3 V_hit = sub(point, A);
  V3 V1 = sub(B, A), V2 = sub(D, A);
  float check1 = (float)dot(normalized(V1), V_hit);
  float check2 = (float)dot(normalized(V2), V_hit);
  if (0 <= check1 && check1 <= norm(V1) && 0 <= check2 && check2 <= norm(V2)) {
    t_out = t_final;
    return true;
  }
  return false;
}

__device__ __forceinline__ void shifted_rect(GP g, float shift, V3& A, V3& B,
                                             V3& C, V3& D)
{
  A = G3(g, RC_A); B = G3(g, RC_B); C = G3(g, RC_C); D = G3(g, RC_D);
  A.y = A.y + shift; B.y = B.y + shift; C.y = C.y + shift; D.y = D.y + shift;
}

// A "rectangle" shifted by a motion-blur pass (cpp:1113; vertices' y + shift): when the shifted y
// differences equal the unshifted ones, (P.y + s) - (A.y + s) == P.y - A.y for P = B, C, D, every
// edge vector of the shifted rectangle is bit for bit the unshifted one, so the normal, edge
// directions and lengths the reference recomputes per call (Rectangle::intersect, geometry.cpp:
// 640-741) are the record's (the same IEEE expressions of the same operands); only the corner A
// moves. Exact in the tunnel scenes for every shift tested (the y + s sums need no rounding); a
// lane for which it fails takes rect_hit_raw.
__device__ __forceinline__ bool shifted_exact(GP g, float shift, V3& As)
{
  const double ay = g[RC_A + 1], ays = ay + shift;
  As = v3(g[RC_A], ays, g[RC_A + 2]);
  return ((g[RC_B + 1] + shift) - ays == g[RC_B + 1] - ay) & ((g[RC_C + 1] + shift) - ays == g[RC_C + 1] - ay) &
         ((g[RC_D + 1] + shift) - ays == g[RC_D + 1] - ay);
}

// quadratic of Sphere/Cylinder (geometry.cpp:108-124 / 246-256)
__device__ __forceinline__ bool quad_roots(float A, float B, float C, float& t0, float& t1)
{
  float disc = (float)(pw2((double)B) - (double)(4 * A * C));
  if (disc < 0) return false;
  float sq = sqrtf(disc);
  t0 = (-B + sq) / (2 * A);
  t1 = (-B - sq) / (2 * A);
  return true;
}

__device__ __forceinline__ bool sphere_hit(GP g, V3 ray, V3 start, float& t,
                                           int& inside)
{
  V3 sc = sub(start, G3(g, SP_C));
  float A = (float)dot(ray, ray);
  float B = (float)(2 * dot(ray, sc));
  float C = (float)(dot(sc, sc) - g[SP_R2]);
  float t0, t1;
  if (!quad_roots(A, B, C, t0, t1)) return false;
  if (t0 <= 0.001 && t1 <= 0.001) { inside = 0; return false; }
  if (t0 <= 0.001 || t1 <= 0.001) { t = fmaxr(t0, t1); inside = 1; return true; }
  t = fminr(t0, t1);
  inside = 0;
  return true;
}

__device__ __forceinline__ bool sphere_shadow(GP g, V3 ray, V3 start, float t_max)
{
  const float eps = 1e-3f;
  V3 sc = sub(start, G3(g, SP_C));
  float A = (float)dot(ray, ray);
  float B = (float)(2 * dot(ray, sc));
  float C = (float)(dot(sc, sc) - g[SP_R2]);
  float t0, t1;
  if (!quad_roots(A, B, C, t0, t1)) return false;
  return !((t0 <= eps || t0 >= t_max) && (t1 <= eps || t1 >= t_max));
}

__device__ __forceinline__ void cyl_coef(GP g, V3 ray, V3 start, float& A,
                                         float& B, float& C)
{
  V3 axis = G3(g, CY_AX);
  V3 rap = sub(ray, mul(dot(ray, axis), axis));
  V3 sc1 = sub(start, G3(g, CY_C1));
  V3 cst = sub(sc1, mul(dot(sc1, axis), axis));
  A = (float)dot(rap, rap);
  B = (float)(2 * dot(rap, cst));
  C = (float)(dot(cst, cst) - g[CY_R2]);
}

__device__ __forceinline__ bool cyl_in_caps(GP g, V3 p)
{
  V3 axis = G3(g, CY_AX);
  return dot(axis, sub(p, G3(g, CY_C1))) > 0 && dot(axis, sub(p, G3(g, CY_C2))) < 0;
}

__device__ bool cyl_hit(GP g, V3 ray, V3 start, float& t, int& inside)
{
  const float eps = 1e-3f;
  float A, B, C, t1, t2;
  cyl_coef(g, ray, start, A, B, C);
  if (!quad_roots(A, B, C, t1, t2)) return false;
  if (t1 <= eps && t2 <= eps) { inside = 0; return false; }
  if (t1 <= eps || t2 <= eps) {
    if (cyl_in_caps(g, add(start, mul(t1, ray)))) { t = t1; inside = 1; return true; }
    return false;
  }
  if (cyl_in_caps(g, add(start, mul(t2, ray)))) { t = t2; inside = 0; return true; }
  return false;
}

__device__ bool cyl_shadow(GP g, V3 ray, V3 start, float t_max)
{
  const float eps = 1e-3f;
  float A, B, C, t1, t2;
  cyl_coef(g, ray, start, A, B, C);
  if (!quad_roots(A, B, C, t1, t2)) return false;
  if ((t1 <= eps || t1 >= t_max) && (t2 <= eps || t2 >= t_max)) return false;
  if (t1 <= eps || t2 <= eps) return cyl_in_caps(g, add(start, mul(t1, ray))) && t1 < t_max;
  return cyl_in_caps(g, add(start, mul(t2, ray))) && t2 < t_max;
}

#if DT_WITH_RPC
// Cylinder::intersectCap (geometry.cpp:297-324): the two cap PLANES (no radius test), c1.axis and
// c2.axis precomputed (RH_C1A / RH_C2A)
__device__ __forceinline__ bool cyl_cap(GP h, V3 ray, V3 start, float& t, int& inside)
{
  const float eps = 1e-3f;
  inside = 0;
  const V3 axis = G3(h, RH_AX);
  const float rdota = (float)dot(ray, axis);
  if (rdota == 0) return false;
  const double sa = dot(start, axis);
  const float t1 = (float)((h[RH_C1A] - sa) / rdota);
  const float t2 = (float)((h[RH_C2A] - sa) / rdota);
  if (t1 < eps && t2 < eps) return false;
  if (t1 < eps || t2 < eps) {
    inside = 1;
    t = fmaxr(t1, t2);
    return true;
  }
  t = fminr(t1, t2);
  return true;
}

// RectPrismWithCylinder's slab test of its own bounds (geometry.cpp:1509-1592 / 1655-1734):
// near-parallel axes (|ray| < 1e-4) take FLT_MIN/FLT_MAX when the start lies inside the slab
// (closed interval for intersect, open for intersectShadow); false: missed
template <bool SHADOW>
__device__ __forceinline__ bool rpc_slab(GP g, V3 ray, V3 start, float& tmin_o, float& tmax_o)
{
  const float eps = 1e-4f;
  const V3 inv = v3(1.0 / ray.x, 1.0 / ray.y, 1.0 / ray.z);
  const V3 lb = G3(g, RP_LB), ub = G3(g, RP_UB);
  float mn[3], mx[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double r = a == 0 ? ray.x : a == 1 ? ray.y : ray.z;
    const double s = a == 0 ? start.x : a == 1 ? start.y : start.z;
    const double l = a == 0 ? lb.x : a == 1 ? lb.y : lb.z, u = a == 0 ? ub.x : a == 1 ? ub.y : ub.z;
    const double iv = a == 0 ? inv.x : a == 1 ? inv.y : inv.z;
    if (fabs(r) < (double)eps) {
      if (SHADOW ? !(s > l && s < u) : !(s >= l && s <= u)) return false;
      mn[a] = FLT_MIN;
      mx[a] = FLT_MAX;
    } else if (r < 0) {
      mn[a] = (float)((u - s) * iv);
      mx[a] = (float)((l - s) * iv);
    } else {
      mn[a] = (float)((l - s) * iv);
      mx[a] = (float)((u - s) * iv);
    }
  }
  float tmin = mn[0], tmax = mx[0];
  if (tmin > mx[1] || mn[1] > tmax) return false;
  if (mn[1] > tmin) tmin = mn[1];
  if (mx[1] < tmax) tmax = mx[1];
  if (tmin > mx[2] || mn[2] > tmax) return false;
  if (mn[2] > tmin) tmin = mn[2];
  if (mx[2] < tmax) tmax = mx[2];
  tmin_o = tmin;
  tmax_o = tmax;
  return true;
}

// RectPrismWithCylinder::intersect (geometry.cpp:1507-1651). t is the box's entry tmin (also when
// the start lies inside, where the reference sets inside and then overwrites t = tmax with tmin).
// The holes: the nearest body or cap-plane crossing; a cap crossing at or before the box entry
// lets the ray through (false), a body hit there replaces t. The reference's uninitialised `hit` /
// `cap_hit` are taken as false. It stores the hit hole's colour into the shape (sticky across later
// rays, so the image depended on the render order); here it is the hit record's colour instead
// (hcol: the hole colour's geom offset, -1: the prism colour).
__device__ __forceinline__ bool rpc_hit(GP g, V3 ray, V3 start, float& t, int& inside, int& hcol)
{
  const float eps = 1e-4f;
  float tmin, tmax;
  inside = 0;
  if (!rpc_slab<false>(g, ray, start, tmin, tmax)) return false;
  if (tmax <= eps) return false;
  if (tmin < eps && tmax > eps) inside = 1;
  float tb = tmin;
  float tcyl = FLT_MAX;
  bool hit = false, cap_hit = false;
  int ins_cyl = 0, hc = -1;
  const int nh = (int)g[RP_NH];
  for (int i = 0; i < nh; ++i) {
    const int o = RP_H + i * RH_SIZE;
    float tt;
    int it = 0;
    if (cyl_hit(g + o, ray, start, tt, it)) {
      hit = true;
      if (tt <= tcyl) { hc = o + RH_COL; ins_cyl = it; tcyl = tt; }
    }
    if (cyl_cap(g + o, ray, start, tt, it)) {
      hit = true;
      if (tt <= tcyl) { hc = o + RH_COL; cap_hit = true; ins_cyl = it; tcyl = tt; }
    }
  }
  if (hit && tcyl <= tb) {
    if (cap_hit) return false;
    inside = ins_cyl;
    tb = tcyl;
    hcol = hc;
  }
  t = tb;
  return true;
}

// RectPrismWithCylinder::intersectShadow (geometry.cpp:1653-1790): the box test ignores t_max
// unless the start lies inside it (a box past the light occludes); a hole's cap crossing inside
// (eps, t_max) at or before the box entry lets the ray through
__device__ __forceinline__ bool rpc_shadow(GP g, V3 ray, V3 start, float t_max)
{
  const float eps = 1e-4f;
  float tmin, tmax;
  if (!rpc_slab<true>(g, ray, start, tmin, tmax)) return false;
  if (tmax <= eps) return false;
  if (tmin < eps && tmax > eps && tmax >= t_max) return false;
  const float tb = tmin;
  float tcyl = FLT_MAX;
  bool hit = false, cap_hit = false;
  const int nh = (int)g[RP_NH];
  for (int i = 0; i < nh; ++i) {
    const int o = RP_H + i * RH_SIZE;
    float tt = FLT_MIN;
    int it = 0;
    if (cyl_hit(g + o, ray, start, tt, it) && tt > eps && tt < t_max) {
      hit = true;
      if (tt <= tcyl) tcyl = tt;
    }
    if (cyl_cap(g + o, ray, start, tt, it) && tt > eps && tt < t_max) {
      hit = true;
      if (tt <= tcyl) { cap_hit = true; tcyl = tt; }
    }
  }
  if (hit && tcyl <= tb && tcyl > eps && tcyl < t_max && cap_hit) return false;
  return true;
}

#endif  // DT_WITH_RPC

// Moller-Trumbore (geometry.cpp:488-586); returns 0 miss, else writes t_final
__device__ __forceinline__ bool tri_core(GP g, V3 ray, V3 start, float& t_final)
{
  V3 r1 = G3(g, TR_R1), r2 = G3(g, TR_R2);
  V3 h = cross(ray, r2);
  float det = (float)dot(r1, h);
  float invdet = (float)(1.0 / det);
  if (det >= -0.0001 && det <= 0.0001) return false;
  V3 A0 = sub(start, G3(g, TR_A));
  float u = (float)(invdet * dot(A0, h));
  if (u < 0 || u > 1) return false;
  V3 DA0 = cross(A0, r1);
  float v = (float)(dot(ray, DA0) * invdet);
  if (v < 0 || u + v > 1) return false;
  t_final = (float)(dot(r2, DA0) * invdet);
  return true;
}

// segmentIntersect (geometry.cpp:44-72) for Checkerboard's edge-on case
__device__ bool segment_hit(V3 A, V3 B, V3 ray, V3 origin)
{
  V3 P3 = add(ray, origin), P4 = origin;
  V3 d13 = sub(A, P3), d43 = sub(P4, P3), d21 = sub(B, A);
  float u1 = (float)((dot(d13, d43) * dot(d43, d21) - dot(d13, d21) * dot(d43, d43)) /
                     (pw2(norm(d21)) * pw2(norm(d43)) - pw2(dot(d43, d21))));
  float u2 = (float)((dot(d13, d43) + u1 * dot(d43, d21)) / pw2(norm(d43)));
  if (u1 < 0 || u1 > 1) return false;
  if (u2 < 0) return false;
  V3 p1 = add(A, mul(u1, sub(B, A)));
  V3 p2 = add(origin, mul(u2, ray));
  return norm(sub(p2, p1)) < 1e-4;
}

// GeoPrimitive::intersect. t only written when the reference writes it (Q16).
__device__ bool shape_hit(const DScene& S, int sid, int type, uint32_t flags, GP g,
                          V3 ray, V3 start, float shift, float& t, int& inside, int& ccol, int& edge)
{
  ccol = -1;
  switch (type) {
    case DT_SHAPE_SPHERE:
      DT_NEED(DT_SHAPE_SPHERE);
      return sphere_hit(g, ray, start, t, inside);
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER:
      return cyl_hit(g, ray, start, t, inside);
    case DT_SHAPE_TRIANGLE: {
      DT_NEED(DT_SHAPE_TRIANGLE);
      inside = 0;
      float tf;
      if (!tri_core(g, ray, start, tf)) return false;
      if (tf > 0.0001) {
        if ((flags & DT_F_MESH) && dot(ray, G3(g, TR_MN)) > 0) inside = 1;
        t = tf;
        return true;
      }
      return false;
    }
    case DT_SHAPE_RECTANGLE: {
      inside = 0;
      float tt, c1, c2;
      if ((flags & DT_F_NAMED_RECT) && shift != 0.0f) {
        V3 As;
        if (shifted_exact(g, shift, As)) {
          if (rect_hit_RA(g + RC_R, As, ray, start, 1e-4f, tt, c1, c2)) { t = tt; return true; }
          return false;
        }
        V3 A, B, C, D;
        shifted_rect(g, shift, A, B, C, D);
        if (rect_hit_raw(A, B, C, D, ray, start, 1e-4f, tt)) { t = tt; return true; }
        return false;
      }
      if (rect_hit_R(g + RC_R, ray, start, 1e-4f, tt, c1, c2)) { t = tt; return true; }
      return false;
    }
    case DT_SHAPE_RECTPRISM_V2: {
      float tmin = FLT_MAX, tt, c1, c2;
#pragma unroll 1
      for (int f = 0; f < 6; ++f) {
        if (rect_hit_R(g + PR_F + f * R_SIZE, ray, start, 1e-4f, tt, c1, c2)) {
          if (tt < tmin) { tmin = tt; inside = 0; }
        }
      }
      if (tmin < FLT_MAX) { t = tmin; return true; }
      return false;
    }
#if DT_WITH_RPC
    case DT_SHAPE_RECTPRISM_CYL:
      return rpc_hit(g, ray, start, t, inside, ccol);
#endif
    case DT_SHAPE_CHECKERBOARD:
      DT_NEED(DT_SHAPE_CHECKERBOARD);
      [[fallthrough]];
    case DT_SHAPE_CHECKERBOARD_HOLE: {
      inside = 0;
      if (dot(G3(g, CK_GN), ray) == 0) {
        V3 A = G3(g, CK_A), B = G3(g, CK_B), C = G3(g, CK_C), D = G3(g, CK_D);
        // edge-on: returns true without t; colour keeps its construction value
        if (segment_hit(A, B, ray, start) || segment_hit(A, D, ray, start) ||
            segment_hit(B, C, ray, start) || segment_hit(C, D, ray, start)) {
          ccol = CK_COL;

          edge = 1;   // t is the stale value of the previous test: order dependent
          return true;
        }
        return false;
      }
      float tt, ch1, ch2;
      if (!rect_hit_R(g + CK_R, ray, start, 1e-3f, tt, ch1, ch2)) return false;
      if (type == DT_SHAPE_CHECKERBOARD_HOLE) {
        float th, a, b;
        if (rect_hit_R(g + CK_HOLE, ray, start, 1e-4f, th, a, b)) return false;
      }
      t = tt;
      float Sq = (float)g[CK_S];
      int i = (int)(ch1 / Sq), j = (int)(ch2 / Sq);
      // the checker colour the reference stores in the shape (geometry.cpp:2314-2337), as the
      // geom offset of that colour: the walk carries one int instead of three doubles
      int col = CK_COL;
      if (i % 2 == 0) {
        if (j % 2 == 0) col = CK_COL1;
        if (j % 2 == 1) col = CK_COL2;
      }
      if (i % 2 == 1) {
        if (j % 2 == 0) col = CK_COL2;
        if (j % 2 == 1) col = CK_COL1;
      }
      ccol = col;
      return true;
    }
  }
  return false;
}

// GeoPrimitive::intersectShadow
__device__ bool shape_shadow(int type, uint32_t flags, GP g, V3 ray, V3 start,
                             float t_max, float shift)
{
  float tt, a, b;
  switch (type) {
    case DT_SHAPE_SPHERE:
      DT_NEED(DT_SHAPE_SPHERE);
      return sphere_shadow(g, ray, start, t_max);
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER:
      return cyl_shadow(g, ray, start, t_max);
    case DT_SHAPE_TRIANGLE: {
      DT_NEED(DT_SHAPE_TRIANGLE);
      float tf;
      if (!tri_core(g, ray, start, tf)) return false;
      return tf > 0.001 && tf < t_max;
    }
    case DT_SHAPE_RECTANGLE:
      if ((flags & DT_F_NAMED_RECT) && shift != 0.0f) {
        V3 As;
        if (shifted_exact(g, shift, As)) return rect_hit_RA(g + RC_R, As, ray, start, 1e-4f, tt, a, b, t_max) && tt < t_max;
        V3 A, B, C, D;
        shifted_rect(g, shift, A, B, C, D);
        return rect_hit_raw(A, B, C, D, ray, start, 1e-4f, tt) && tt < t_max;
      }
      return rect_hit_R(g + RC_R, ray, start, 1e-4f, tt, a, b, t_max) && tt < t_max;
    case DT_SHAPE_CHECKERBOARD:
      DT_NEED(DT_SHAPE_CHECKERBOARD);
      return rect_hit_R(g + CK_R, ray, start, 1e-4f, tt, a, b, t_max) && tt < t_max;
    case DT_SHAPE_RECTPRISM_V2:
#pragma unroll 1
      for (int f = 0; f < 6; ++f)
        if (rect_hit_R(g + PR_F + f * R_SIZE, ray, start, 1e-4f, tt, a, b, t_max) && tt < t_max) return true;
      return false;
#if DT_WITH_RPC
    case DT_SHAPE_RECTPRISM_CYL:
      return rpc_shadow(g, ray, start, t_max);
#endif
    case DT_SHAPE_CHECKERBOARD_HOLE:
      if (rect_hit_R(g + CK_R, ray, start, 1e-3f, tt, a, b, t_max) && tt < t_max) {
        if (rect_hit_R(g + CK_HOLE, ray, start, 1e-4f, tt, a, b, t_max) && tt < t_max) return false;
        return true;
      }
      return false;
  }
  return false;
}

// GeoPrimitive::getNorm (per-lane shape index); ccol: the hit record's colour offset (a
// RectPrismWithCylinder hole: its record is at ccol - RH_COL)
__device__ __forceinline__ V3 shape_norm(int type, uint32_t flags, GP g, V3 p, float shift,
                         unsigned int* st_prism, int ccol)
{
  switch (type) {
#if DT_WITH_RPC
    case DT_SHAPE_RECTPRISM_CYL: {
      // RectPrismWithCylinder::getNorm (geometry.cpp:1792-1821): lastHit is always -1 here (intersect
      // resets it before every `return true`), so the face tests below decide, signed and unnormalised
      const float eps = 1e-3f;
      const V3 pa = sub(p, G3(g, RP_A));
      if (dot(pa, G3(g, RP_NBOT)) <= eps) return G3(g, RP_NBOT);
      if (dot(pa, G3(g, RP_NRIGHT)) <= eps) return G3(g, RP_NRIGHT);
      if (dot(pa, G3(g, RP_NFRONT)) <= eps) return G3(g, RP_NFRONT);
      // the reference throws ("point is not on prism", 1819-1820): counted; the hit hole's normal
      // (Cylinder::getNorm, 419-425), else the front normal
      atomicAdd(st_prism, 1u);
      if (ccol >= 0) {
        const int h = ccol - RH_COL;
        const V3 axis = G3(g, h + RH_AX), pc = sub(p, G3(g, h + RH_C1));
        return normalized(sub(pc, mul(dot(pc, axis), axis)));
      }
      return G3(g, RP_NFRONT);
    }
#endif
    case DT_SHAPE_SPHERE: {
      DT_NEED(DT_SHAPE_SPHERE);
      V3 n = sub(p, G3(g, SP_C));
      return divs(n, norm(n));
    }
    case DT_SHAPE_CYLINDER:
    case DT_SHAPE_CHECKER_CYLINDER: {
      V3 axis = G3(g, CY_AX);
      V3 pc = sub(p, G3(g, CY_C1));
      return normalized(sub(pc, mul(dot(pc, axis), axis)));
    }
    case DT_SHAPE_TRIANGLE:
      DT_NEED(DT_SHAPE_TRIANGLE);
      return normalized(cross(G3(g, TR_R1), G3(g, TR_R2)));
    case DT_SHAPE_RECTANGLE: {
      V3 A, B, C, D;
      if ((flags & DT_F_NAMED_RECT) && shift != 0.0f) shifted_rect(g, shift, A, B, C, D);
      else { A = G3(g, RC_A); B = G3(g, RC_B); C = G3(g, RC_C); }
      return normalized(cross(sub(B, A), sub(C, A)));
    }
    case DT_SHAPE_CHECKERBOARD:
    case DT_SHAPE_CHECKERBOARD_HOLE:
      return G3(g, CK_GN);
    case DT_SHAPE_RECTPRISM_V2: {
      const float eps = 1e-3f;
      V3 A = G3(g, PR_A), G = G3(g, PR_G);
      V3 nb = G3(g, PR_NBOT), nr = G3(g, PR_NRIGHT), nf = G3(g, PR_NFRONT);
      V3 pa = normalized(sub(p, A)), pg = normalized(sub(p, G));
      float pa_bot = (float)fabs(dot(pa, nb)), pg_bot = (float)fabs(dot(pg, nb));
      if (pa_bot <= eps || pg_bot <= eps) return nb;
      float pa_right = (float)fabs(dot(pa, nr)), pg_right = (float)fabs(dot(pg, nr));
      if (pa_right <= eps || pg_right <= eps) return nr;
      float pa_front = (float)fabs(dot(pa, nf)), pg_front = (float)fabs(dot(pg, nf));
      if (pa_front <= eps || pg_front <= eps) return nf;
      atomicAdd(st_prism, 1u);
      float m = pa_bot;
      if (pg_bot < m) m = pg_bot;
      if (pa_right < m) m = pa_right;
      if (pg_right < m) m = pg_right;
      if (pa_front < m) m = pa_front;
      if (pg_front < m) m = pg_front;
      if (pa_bot == m || pg_bot == m) return nb;
      if (pa_right == m || pg_right == m) return nr;
      return nf;
    }
  }
  return v3(0, 0, 0);
}

// GeoPrimitive::getUV (type 0/1/2)
__device__ __forceinline__ int shape_uv(int type, uint32_t flags, GP g, V3 p, float shift,
                        double& uo, double& vo)
{
  switch (type) {
    case DT_SHAPE_RECTANGLE: {
      V3 A, B, C, D;
      if ((flags & DT_F_NAMED_RECT) && shift != 0.0f) shifted_rect(g, shift, A, B, C, D);
      else { A = G3(g, RC_A); C = G3(g, RC_C); D = G3(g, RC_D); }
      V3 ad = sub(D, A), dc = sub(C, D);
      double nadc = ((flags & DT_F_NAMED_RECT) && shift != 0.0f) ? norm(ad) * norm(dc) : g[RC_NADC];
      uo = (float)(norm(cross(sub(p, A), ad)) / nadc);
      vo = (float)(norm(cross(sub(p, D), dc)) / nadc);
      return 1;
    }
#if DT_WITH_RPC
    case DT_SHAPE_RECTPRISM_CYL: {
      // RectPrism::getUV (geometry.cpp:1442-1461): valid only where |(ad x dc).p| <= 1e-5
      if (fabs(dot(G3(g, RP_ADC), p)) <= 1e-5) {
        uo = (float)(norm(cross(sub(p, G3(g, RP_A)), G3(g, RP_AD))) / g[RP_NADC]);
        vo = (float)(norm(cross(sub(p, G3(g, RP_D)), G3(g, RP_DC))) / g[RP_NADC]);
        return 1;
      }
      uo = -1; vo = -1;
      return 0;
    }
#endif
    case DT_SHAPE_RECTPRISM_V2: {
      V3 A = G3(g, PR_F + R_A), ad = G3(g, PR_AD), dc = G3(g, PR_DC), D = G3(g, PR_D);
      uo = (float)(norm(cross(sub(p, A), ad)) / g[PR_NADC]);
      vo = (float)(norm(cross(sub(p, D), dc)) / g[PR_NADC]);
      return 1;
    }
    case DT_SHAPE_TRIANGLE: {
      DT_NEED(DT_SHAPE_TRIANGLE);
      V3 A = G3(g, TR_A), B = G3(g, TR_B), C = G3(g, TR_C);
      V3 n = cross(sub(B, A), sub(C, A));
      V3 n_a = cross(sub(C, B), sub(p, B));
      V3 n_b = cross(sub(A, C), sub(p, C));
      float nsq = (float)dot(n, n);
      float al = (float)(dot(n, n_a) / nsq), be = (float)(dot(n, n_b) / nsq);
      float ga = 1 - al - be;
      if (al < 0 || al > 1 || be < 0 || be > 1 || ga < 0 || ga > 1) { uo = -1; vo = -1; return 0; }
      uo = ((double)al * g[TR_UV + 0] + (double)be * g[TR_UV + 2]) + (double)ga * g[TR_UV + 4];
      vo = ((double)al * g[TR_UV + 1] + (double)be * g[TR_UV + 3]) + (double)ga * g[TR_UV + 5];
      return 1;
    }
    case DT_SHAPE_CHECKERBOARD_HOLE: {
      V3 A = G3(g, CK_A), D = G3(g, CK_D);
      V3 V_hit = sub(p, A);
      float check1 = (float)dot(G3(g, CK_R + R_V1N), V_hit);
      float check2 = (float)dot(G3(g, CK_R + R_V2N), V_hit);
      if (0 <= check1 && check1 <= g[CK_R + R_LEN1] && 0 <= check2 && check2 <= g[CK_R + R_LEN2]) {
        float tt, a, b;
        if (rect_hit_R(g + CK_HOLE, v3(1, 1, 1), sub(p, v3(1, 1, 1)), 1e-4f, tt, a, b) && tt < FLT_MAX) {
          uo = -1; vo = -1;
          return 0;
        }
        V3 ad = G3(g, CK_AD), dc = G3(g, CK_DC);
        float u = (float)(norm(cross(sub(p, A), ad)) / g[CK_NADC]);
        float v = (float)(norm(cross(sub(p, D), dc)) / g[CK_NADC]);
        float mud = (float)g[CK_MUD], mvd = (float)g[CK_MVD], bw = (float)g[CK_BW];
        float miniu = u / mud - (int)(u / mud);
        float miniv = v / mvd - (int)(v / mvd);
        if (miniu < 0) miniu = 0;
        if (miniv < 0) miniv = 0;
        uo = miniu; vo = miniv;
        if ((miniu <= bw || miniu >= 1 - bw) || (miniv <= bw || miniv >= 1 - bw)) return 2;
        return 1;
      }
      uo = -1; vo = -1;
      return 0;
    }
    case DT_SHAPE_CHECKER_CYLINDER: {
      double ph[4] = {p.x, p.y, p.z, 1};
      double po[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        double s = g[CY_M + i * 4 + 0] * ph[0];
        s = s + g[CY_M + i * 4 + 1] * ph[1];
        s = s + g[CY_M + i * 4 + 2] * ph[2];
        s = s + g[CY_M + i * 4 + 3] * ph[3];
        po[i] = s;
      }
      float u = 0;
      if (p.x != 0) u = (float)((atan2(po[1], po[0]) + M_PI) / (2 * M_PI));
      float v = (float)(po[2] / g[CY_NAX]);
      float mud = (float)g[CY_MUD], mvd = (float)g[CY_MVD], bw = (float)g[CY_BW];
      float miniu = u / mud - (int)(u / mud);
      float miniv = v / mvd - (int)(v / mvd);
      uo = miniu; vo = miniv;
      if ((miniu <= bw || miniu >= 1 - bw) || (miniv <= bw || miniv >= 1 - bw)) return 2;
      return 1;
    }
  }
  uo = -1; vo = -1;
  return 0;
}

// =====================================================================================
// BVH: wave-uniform stackless traversal (geometry.cpp:2657-2740 box test)
// =====================================================================================
// Per-ray constants of the slab test, computed once per traversal.
struct RayBox {
  V3 inv;                      // ray.cwiseInverse()
  bool nx, ny, nz;             // ray[a] < 0
  bool ix, iy, iz;             // isinf(inv[a])
};

__device__ __forceinline__ RayBox make_raybox(V3 ray)
{
  RayBox r;
  r.inv = v3(1.0 / ray.x, 1.0 / ray.y, 1.0 / ray.z);
  r.nx = ray.x < 0; r.ny = ray.y < 0; r.nz = ray.z < 0;
  r.ix = isinf(r.inv.x); r.iy = isinf(r.inv.y); r.iz = isinf(r.inv.z);
  return r;
}

// BoundingVolume::intersect (geometry.cpp:2657-2740), branch-free: every early `return false`
// of the reference becomes a cleared `ok`, every conditional assignment a select, so a wave
// evaluates one straight-line sequence per node with no exec-mask traffic. lb1/ub1: the
// y-bounds after the motion-blur leaf bump (helpers.h:530-552).
__device__ __forceinline__ bool box_hit(const DNodeDev& b, double lb1, double ub1, const RayBox& r, V3 st)
{
  bool ok;
  float tmin, tmax, tymin, tymax, tzmin, tzmax;
  {
    double lo = r.nx ? b.ub[0] : b.lb[0], hi = r.nx ? b.lb[0] : b.ub[0];
    float a = (float)((lo - st.x) * r.inv.x), c = (float)((hi - st.x) * r.inv.x);
    bool in = (st.x >= b.lb[0]) & (st.x <= b.ub[0]);
    tmin = r.ix ? FLT_MIN : a;
    tmax = r.ix ? FLT_MAX : c;
    ok = r.ix ? in : true;
  }
  {
    double lo = r.ny ? ub1 : lb1, hi = r.ny ? lb1 : ub1;
    float a = (float)((lo - st.y) * r.inv.y), c = (float)((hi - st.y) * r.inv.y);
    bool in = (st.y >= lb1) & (st.y <= ub1);
    tymin = r.iy ? FLT_MIN : a;
    tymax = r.iy ? FLT_MAX : c;
    ok = ok & (r.iy ? in : true);
  }
  ok = ok & !((tmin > tymax) | (tymin > tmax));
  tmin = (tymin > tmin) ? tymin : tmin;
  tmax = (tymax < tmax) ? tymax : tmax;
  {
    double lo = r.nz ? b.ub[2] : b.lb[2], hi = r.nz ? b.lb[2] : b.ub[2];
    float a = (float)((lo - st.z) * r.inv.z), c = (float)((hi - st.z) * r.inv.z);
    bool in = (st.z >= b.lb[2]) & (st.z <= b.ub[2]);
    tzmin = r.iz ? FLT_MIN : a;
    tzmax = r.iz ? FLT_MAX : c;
    ok = ok & (r.iz ? in : true);
  }
  ok = ok & !((tmin > tzmax) | (tzmin > tmax));
  tmax = (tzmax < tmax) ? tzmax : tmax;
  return ok & (tmax > 0);
}

// The same test for waves where no lane's ray has a zero component (no isinf(inv) axis, the
// common case): both slab ends are computed from the unswapped bounds and selected in f32,
// which yields the identical floats ((lo - st) * inv is evaluated for the same lo either way).
// `tcull` additionally rejects boxes whose entry parameter lies beyond any hit that could
// still change the result (closest hit: past the best t; shadow: past the light). A shape lies
// inside its leaf box (bounds of its own vertices/extent, +-1e-2 leaf padding), so a culled box
// holds no hit the reference would have used: the result is unchanged, only the gather is
// smaller. Callers pass FLT_MAX to disable it.
__device__ __forceinline__ bool box_hit_exact_finite(const DNodeDev& b, const RayBox& r, V3 st, float tcull)
{
  const float ax = (float)((b.lb[0] - st.x) * r.inv.x), cx = (float)((b.ub[0] - st.x) * r.inv.x);
  const float ay = (float)((b.lb[1] - st.y) * r.inv.y), cy = (float)((b.ub[1] - st.y) * r.inv.y);
  const float az = (float)((b.lb[2] - st.z) * r.inv.z), cz = (float)((b.ub[2] - st.z) * r.inv.z);
  // The reference's slab sequence accepts iff every entry value <= every exit value
  // (tx_min <= ty_max, ty_min <= tx_max, max(..) <= tz_max, tz_min <= min(..)) and the
  // final exit > 0: i.e. max3(entries) <= min3(exits) && min3(exits) > 0. No NaN can occur
  // here (finite inverse), and +-0 compare equal, so the min/max form decides identically.
  // The entry of an axis is min(a, c) and its exit max(a, c): with lb <= ub (checked on the
  // host for every node, P.boxes_ordered, else every wave takes the general test) rounding is
  // monotone, so a <= c for inv > 0 and c <= a for inv < 0 -- the sign select of the
  // reference, without per-ray sign masks held in SGPRs across the walk.
  const float tmin = fmaxf(fmaxf(fminf(ax, cx), fminf(ay, cy)), fminf(az, cz));
  const float tmax = fminf(fminf(fmaxf(ax, cx), fmaxf(ay, cy)), fmaxf(az, cz));
  return (tmin <= tmax) & (tmax > 0) & (tmin <= tcull);
}

// The slab decision for waves where no lane's ray has a zero component (no isinf(inv) axis,
// the common case). `tcull` additionally rejects boxes whose entry parameter lies beyond any
// hit that could still change the result (closest hit: past the best t; shadow: past the
// light). A shape lies inside its leaf box (bounds of its own vertices/extent, +-1e-2 leaf
// padding), so a culled box holds no hit the reference would have used: the result is
// unchanged, only the gather is smaller. Callers pass FLT_MAX to disable it.
// (Measured slower and dropped: an f32 pre-test with an exact fallback, 1515 vs 1606 Msps on C3;
// wave-uniform slab-end selection for sign-coherent waves, 1482 vs 1630; again in round 4 with the
// selection on the scalar unit: VALU +1.9%, SALU +10%, C3 -2.4%, C4 -7%, profiles/r04b_ab.log.)
__device__ __forceinline__ bool box_hit_finite(const DNodeDev& b, const RayBox& r, V3 st, float tcull)
{
  return box_hit_exact_finite(b, r, st, tcull);
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Lane sets of the walks are wave-uniform lane masks (SGPR pairs): a per-lane bool carried through
// a walk was kept as a 0/1 value in a VGPR and turned back into a mask at every use (up to six VALU
// instructions per list entry). inv(m): this lane's bit of a uniform mask m, with no VALU
// (llvm.amdgcn.inverse.ballot: an exec-mask operation).
__device__ __forceinline__ bool inv(unsigned long long m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v)
{
  unsigned long long x = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}


// wave-uniform traversal state shared by closest_hit / occluded
struct Walk {
  RayBox rb;
  bool inf_wave;   // some lane has an axis-parallel ray: exact isinf path
  bool bump_wave;  // some lane shifts leaves (motion-blur pass)
};

// inf_wave also takes NaN rays/origins: the reference's slab sequence treats a NaN axis
// asymmetrically (x fails, y/z are skipped), which only the exact general test reproduces.
__device__ __forceinline__ Walk make_walk(const DParams& P, bool active, V3 ray, V3 st, float shift)
{
  Walk w;
  w.rb = make_raybox(ray);
  const bool odd = w.rb.ix | w.rb.iy | w.rb.iz | isnan(ray.x) | isnan(ray.y) | isnan(ray.z) | isnan(st.x) |
                   isnan(st.y) | isnan(st.z);
  w.inf_wave = __ballot(active && odd) != 0 || !P.boxes_ordered;
  w.bump_wave = !DT_NOSHIFT && __ballot(active && shift != 0.0f) != 0;
  return w;
}

// GENERAL: the exact slab test for any wave (axis-parallel rays, motion-blur leaf bump);
// otherwise the finite-ray test with no bump code at all (the hot instantiation).
template <bool GENERAL>
__device__ __forceinline__ bool node_hit(const Walk& w, const DNodeDev& nd, float shift, V3 st, float tcull)
{
  if (!GENERAL) return box_hit_finite(nd, w.rb, st, tcull);
  double lb1 = nd.lb[1], ub1 = nd.ub[1];
  if ((nd.meta & DN_LEAF) && shift != 0.0f) {   // bumpBVH (helpers.h:530-552): leaves only
    lb1 = lb1 - shift;
    ub1 = ub1 + shift;
  }
  return box_hit(nd, lb1, ub1, w.rb, st);
}

// The finite-ray decision of box_hit_exact_finite as the wave's lane mask: the three compares write
// their masks straight into SGPRs (llvm.amdgcn.fcmp: ordered <=, >, <=, false for NaN as the C
// compares), so no per-lane bool is materialised and turned back into a mask. Lanes outside exec
// get no bit, as with a ballot; the callers run at wave-uniform control flow.
// The six slab values are compared as the reference's floats, but rounded only after the min/max:
// f64 -> f32 rounding is monotone, so min/max of the rounded values are the rounded min/max (no NaN
// on this path). Two conversions instead of six (DT_BOX_F64MINMAX=0: the six-conversion form).
#ifndef DT_BOX_F64MINMAX
#define DT_BOX_F64MINMAX 1
#endif
__device__ __forceinline__ unsigned long long box_mask_finite(const DNodeDev& b, const RayBox& r, V3 st, float tcull)
{
#if DT_BOX_F64MINMAX
  const double ax = (b.lb[0] - st.x) * r.inv.x, cx = (b.ub[0] - st.x) * r.inv.x;
  const double ay = (b.lb[1] - st.y) * r.inv.y, cy = (b.ub[1] - st.y) * r.inv.y;
  const double az = (b.lb[2] - st.z) * r.inv.z, cz = (b.ub[2] - st.z) * r.inv.z;
  const float tmin = (float)__builtin_fmax(__builtin_fmax(__builtin_fmin(ax, cx), __builtin_fmin(ay, cy)), __builtin_fmin(az, cz));
  const float tmax = (float)__builtin_fmin(__builtin_fmin(__builtin_fmax(ax, cx), __builtin_fmax(ay, cy)), __builtin_fmax(az, cz));
#else
  const float ax = (float)((b.lb[0] - st.x) * r.inv.x), cx = (float)((b.ub[0] - st.x) * r.inv.x);
  const float ay = (float)((b.lb[1] - st.y) * r.inv.y), cy = (float)((b.ub[1] - st.y) * r.inv.y);
  const float az = (float)((b.lb[2] - st.z) * r.inv.z), cz = (float)((b.ub[2] - st.z) * r.inv.z);
  const float tmin = fmaxf(fmaxf(fminf(ax, cx), fminf(ay, cy)), fminf(az, cz));
  const float tmax = fminf(fminf(fmaxf(ax, cx), fmaxf(ay, cy)), fmaxf(az, cz));
#endif
  return __builtin_amdgcn_fcmpf(tmin, tmax, 5 /*OLE*/) & __builtin_amdgcn_fcmpf(tmax, 0.0f, 2 /*OGT*/) &
         __builtin_amdgcn_fcmpf(tmin, tcull, 5 /*OLE*/);
}

// node_hit as a lane mask: GENERAL waves test lane by lane (act: the lane's own walk state), the
// finite-ray test runs for the lanes of actm
template <bool GENERAL>
__device__ __forceinline__ unsigned long long node_mask(const Walk& w, const DNodeDev& nd, float shift, V3 st,
                                                        float tcull, unsigned long long actm, bool act)
{
  if (GENERAL) return __ballot(act & node_hit<true>(w, nd, shift, st, tcull));
  return actm & box_mask_finite(nd, w.rb, st, tcull);
}

// q-th shape of a leaf: (id, type, flags, geom offset), all wave-uniform
__device__ __forceinline__ void leaf_shape(const DScene& S, const DNodeDev& nd, int q, int& sid, int& type,
                                           uint32_t& flags, int& off)
{
  if (nd.meta & DN_SINGLE) {
    sid = nd.first;
    type = (int)((nd.meta >> 4) & 15u);
    flags = (nd.meta >> 8) & 0xffu;
    off = nd.aux;
  } else {
    sid = uni(cas(S.leaf_idx)[nd.first + q]);
    const DShapeHdr hd = cas(S.hdr)[sid];
    type = hd.type;
    flags = hd.flags;
    off = hd.off;
  }
}

struct Counters;
struct HitRec {
  float t_min;
  int shape;
  int rank;       // leaf rank of the hit in the reference's gather order (fast-tree ties)
  int edge;       // a checkerboard edge-on hit (Q16) was taken
  int inside;
  int ccol;       // checker colour of the hit (geom offset), -1: the material colour
};

// Motion-blur passes on the bump tree: whether the reference gathers the leaf `r` (its index in
// the reference tree) for this lane: the bumped leaf box passes (node_hit<true>) and so do all its
// reference ancestors -- implied when the unbumped leaf box passes (the ancestors contain it and
// the finite-ray slab test is monotone), otherwise tested up the parent chain (host_fasttree.cpp).
__device__ __forceinline__ bool bump_leaf_gathered(const DScene& S, const Walk& w, int r, float shift, V3 st)
{
  const DNodeDev rn = cas(S.nodes)[r];
  const bool bumped = box_hit(rn, rn.lb[1] - shift, rn.ub[1] + shift, w.rb, st);
  const bool unb = box_hit(rn, rn.lb[1], rn.ub[1], w.rb, st);
  bool ok = bumped & unb;
  const bool need = bumped & !unb;
  if (__ballot(need)) {
    bool anc = true;
    for (int a = uni(cas(S.bparent)[r]); a >= 0; a = uni(cas(S.bparent)[a])) {
      const DNodeDev an = cas(S.nodes)[a];
      anc = anc & box_hit(an, an.lb[1], an.ub[1], w.rb, st);
    }
    ok = ok | (need & anc);
  }
  return ok;
}

// Closest hit with shapes first (closest_hit_walk, closest_hit_plist: blur passes) needs shape tests
// that read no earlier test's state: not with checkerboards (the edge-on case reuses the previous t,
// Q16), so only in the builds without them (the tunnel builds: C5's frames with motion blur)
#ifndef DT_SHAPE_FIRST
#define DT_SHAPE_FIRST 1
#endif
static_assert(DT_SHAPE_CHECKERBOARD == 6 && DT_SHAPE_CHECKERBOARD_HOLE == 7 && DT_SHAPE_CHECKER_CYLINDER == 8,
              "DT_HAS(6/7/8) below");
// scattered shadow waves: lanes whose own cell is an umbra cell answer "occluded" without joining
// the union of the lanes' lists (the coherent path already answered a whole wave so)
#ifndef DT_UMBRA_EARLY
#define DT_UMBRA_EARLY 1   // umbra cells of point lights decided before the light sample (light loop)
#endif
#ifndef DT_UMBRA_LANES
#define DT_UMBRA_LANES 1
#endif
#ifndef DT_SF_CLOSEST
#define DT_SF_CLOSEST (DT_SHAPE_FIRST && !DT_HAS(6) && !DT_HAS(7) && !DT_HAS(8))
#endif

// every active lane's motion-blur shift lies within the bump tree's padding, and is >= 0 when the
// tree (and the blur-padded grid lists) were padded for non-negative shifts only (host_accel.cpp):
// the render's globals may draw shifts the build's did not
__device__ __forceinline__ bool bump_tree_ok(const DParams& P, bool active, float shift)
{
  return P.n_bnodes > 0 && !__ballot(active && !(fabsf(shift) <= P.bump_pad && (shift >= 0.0f || !P.bump_up_only)));
}

// closest hit over the lanes with `active` (cpp:491-538)
// MODE 0: finite rays, no bump (fast tree, culled); 1: the reference tree, exact for any wave;
// 2: finite rays of a motion-blur pass on the bump tree (culled, exact gather at the leaves)
template <int MODE, class CNT>
__device__ __forceinline__ bool closest_hit_walk(const DScene& S, const DParams& P, const Walk& w, bool active, V3 ray,
                                                 V3 org, float shift, HitRec& h, CNT& cnt)
{
  constexpr bool GENERAL = MODE == 1, BUMP = MODE == 2;
  // fast walks use the alternative tree when one was built (DT_FAST_TREE), else the reference's
  const bool ftree = BUMP || (!GENERAL && P.n_fnodes > 0 && (P.ftree_mode & 1));
  const DNodeDev* const NODES = BUMP ? S.bnodes : ftree ? S.fnodes : S.nodes;
  int resume = active ? 0 : 0x7fffffff;
  const unsigned long long am = __ballot(active);
  float t_dist = FLT_MAX;
  float tcull = FLT_MAX;   // culling bound from the best hit so far (updated with it)
  bool any = false;
  h.t_min = FLT_MAX;
  h.shape = -1;
  h.rank = 0x7fffffff;
  h.edge = 0;
  h.inside = 0;
  h.ccol = -1;
  int i = 0;
  const int n_nodes = BUMP ? P.n_bnodes : ftree ? P.n_fnodes : P.n_nodes;
  while (i < n_nodes) {
    const DNodeDev nd = cas(NODES)[i];
    // fast walks need no per-lane resume point: every box contains its subtree's boxes and the
    // finite-ray slab test (with the shrinking tcull) is monotone in the box, so a lane that
    // failed an ancestor fails here too (host_fasttree.cpp)
    const bool act = GENERAL ? resume <= i : inv(am);
    tcull = (h.t_min == FLT_MAX || (DT_WITH_RPC && P.no_cull)) ? FLT_MAX : h.t_min * 1.0001f + 1e-4f;
    unsigned long long hbm = node_mask<GENERAL>(w, nd, shift, org, tcull, am, act);
    const bool hb = inv(hbm);
    DT_WORK(cnt.wnodes++);
    DT_WK(DT_WK_BOX, act);
    DT_CNT(26);
    if (nd.meta & DN_LEAF) {
      DT_WK(DT_WK_BOX, BUMP && hb);   // the exact bumped gather: the reference leaf's own box test
      if (BUMP && DT_SF_CLOSEST) {
        // shapes first into a tentative record, the exact gather only for the lanes with a hit
        // (shadow_leaf_bump): the same result in either order, as no shape test here reads an
        // earlier test's state (no checkerboards in these builds: DT_SF_CLOSEST)
        if (hbm) {
          HitRec th = h;
          bool tany = false, chg = false;
          const int nq = (nd.meta & DN_SINGLE) ? 1 : nd.aux;
          for (int q = 0; q < nq; ++q) {
            int sid, type, off;
            uint32_t flags;
            leaf_shape(S, nd, q, sid, type, flags, off);
            DT_CNT(8);
            DT_CNT(10 + (type & 7));
            if (inv(hbm)) {
              DT_WK(DT_WK_HIT_SHAPE + type, true);
              int ins = 0, cc = -1;
              if (shape_hit(S, sid, type, flags, cas(S.geom) + off, ray, org, shift, t_dist, ins, cc, th.edge)) {
                tany = true;
                const int rank = ftree ? (int)(nd.meta >> 16) : 0;
                if (t_dist < th.t_min || (ftree && t_dist == th.t_min && rank < th.rank)) {
                  th.rank = rank;
                  th.shape = sid;
                  th.inside = ins;
                  th.t_min = t_dist;
                  th.ccol = cc;
                  chg = true;
                }
              }
            }
          }
          if (__ballot(tany)) {
            const bool g = bump_leaf_gathered(S, w, nd.skip, shift, org);
            if (tany && g) {
              any = true;
              if (chg) h = th;
            }
          }
        }
        hbm = 0;
      }
      if (BUMP && !DT_SF_CLOSEST && hbm) hbm = __ballot(hb & bump_leaf_gathered(S, w, nd.skip, shift, org));
      if (hbm) {
        DT_T(q0);
        const int nq = (nd.meta & DN_SINGLE) ? 1 : nd.aux;
        for (int q = 0; q < nq; ++q) {
          int sid, type, off;
          uint32_t flags;
          leaf_shape(S, nd, q, sid, type, flags, off);
          DT_CNT(8);
          DT_CNT(10 + (type & 7));   // closest-hit prim tests by type (8 -> 10)
          if (inv(hbm)) {
            DT_WK(DT_WK_HIT_SHAPE + type, true);
            int ins = 0, cc = -1;
            if (shape_hit(S, sid, type, flags, cas(S.geom) + off, ray, org, shift, t_dist, ins, cc, h.edge)) {
              any = true;
              // strict < in the reference's gather order; the fast tree visits leaves in another
              // order, so equal distances go to the lower reference rank
              const int rank = ftree ? (int)(nd.meta >> 16) : 0;
              if (t_dist < h.t_min || (ftree && t_dist == h.t_min && rank < h.rank)) {
                h.rank = rank;
                h.shape = sid;
                h.inside = ins;
                h.t_min = t_dist;
                h.ccol = cc;
              }
            }
          }
        }
        DT_T(q1);
        DT_ACC(33, q0, q1);
      }
      if (GENERAL && act) resume = nd.skip;
      i = i + 1;
    } else {
      if (GENERAL && act && !hb) resume = nd.skip;
      i = hbm ? i + 1 : nd.skip;
    }
  }
  return any;
}

// Closest hit of primary rays over their pixel block's candidate leaves (host_primlists.cpp), in
// order of the smallest ray parameter each leaf's box can be reached at: once every lane's best hit
// lies before the next entry, no later leaf can change a result. Same box filter, shape tests and
// tie rule (reference rank) as the fast-tree walk.
// BUMP: a motion-blur pass over the bump tree's lists: padded leaf boxes, then the exact bumped
// gather (bump_leaf_gathered) and the shifted shapes, as in the bump-tree walk.
template <bool BUMP, class CNT>
__device__ __forceinline__ bool closest_hit_plist(const DScene& S, const DParams& P, const Walk& w, bool active, V3 ray,
                                                  V3 org, float shift, HitRec& h, uint32_t off, uint32_t n, CNT& cnt)
{
  float t_dist = FLT_MAX;
  bool any = false;
  const unsigned long long am = __ballot(active);
  h.t_min = FLT_MAX;
  h.shape = -1;
  h.rank = 0x7fffffff;
  h.edge = 0;
  h.inside = 0;
  h.ccol = -1;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t node = __builtin_amdgcn_readfirstlane(cas(S.pl_list)[2 * (size_t)(off + k)]);
    const float tn = __uint_as_float(__builtin_amdgcn_readfirstlane(cas(S.pl_list)[2 * (size_t)(off + k) + 1]));
    if (!__ballot(active && !(h.t_min < tn))) break;
    const DNodeDev nd = cas(BUMP ? S.bnodes : S.fnodes)[node];
    const float tcull = h.t_min == FLT_MAX ? FLT_MAX : h.t_min * 1.0001f + 1e-4f;
    unsigned long long hbm = am & box_mask_finite(nd, w.rb, org, tcull);
    DT_WK(DT_WK_BOX, active);
    DT_WK(DT_WK_BOX, BUMP && inv(hbm));
    DT_WORK(cnt.wnodes++);
    DT_CNT(26);
    if (BUMP && DT_SF_CLOSEST) {   // shapes first, then the exact gather (closest_hit_walk)
      if (hbm) {
        HitRec th = h;
        bool tany = false, chg = false;
        const int nq = (nd.meta & DN_SINGLE) ? 1 : nd.aux;
        const int rank = (int)(nd.meta >> 16);
        for (int q = 0; q < nq; ++q) {
          int sid, type, off2;
          uint32_t flags;
          leaf_shape(S, nd, q, sid, type, flags, off2);
          DT_CNT(8);
          DT_CNT(10 + (type & 7));
          if (inv(hbm)) {
            DT_WK(DT_WK_HIT_SHAPE + type, true);
            int ins = 0, cc = -1;
            if (shape_hit(S, sid, type, flags, cas(S.geom) + off2, ray, org, shift, t_dist, ins, cc, th.edge)) {
              tany = true;
              if (t_dist < th.t_min || (t_dist == th.t_min && rank < th.rank)) {
                th.rank = rank;
                th.shape = sid;
                th.inside = ins;
                th.t_min = t_dist;
                th.ccol = cc;
                chg = true;
              }
            }
          }
        }
        if (__ballot(tany)) {
          const bool g = bump_leaf_gathered(S, w, nd.skip, shift, org);
          if (tany && g) {
            any = true;
            if (chg) h = th;
          }
        }
      }
      hbm = 0;
    }
    if (BUMP && !DT_SF_CLOSEST && hbm) hbm = __ballot(inv(hbm) & bump_leaf_gathered(S, w, nd.skip, shift, org));
    if (hbm) {
      const int nq = (nd.meta & DN_SINGLE) ? 1 : nd.aux;
      const int rank = (int)(nd.meta >> 16);
      for (int q = 0; q < nq; ++q) {
        int sid, type, off2;
        uint32_t flags;
        leaf_shape(S, nd, q, sid, type, flags, off2);
        DT_CNT(8);
        DT_CNT(10 + (type & 7));
        if (inv(hbm)) {
          DT_WK(DT_WK_HIT_SHAPE + type, true);
          int ins = 0, cc = -1;
          if (shape_hit(S, sid, type, flags, cas(S.geom) + off2, ray, org, BUMP ? shift : 0.0f, t_dist, ins, cc, h.edge)) {
            any = true;
            if (t_dist < h.t_min || (t_dist == h.t_min && rank < h.rank)) {
              h.rank = rank;
              h.shape = sid;
              h.inside = ins;
              h.t_min = t_dist;
              h.ccol = cc;
            }
          }
        }
      }
    }
  }
  return any;
}

// The exact walks on the reference tree for waves with an axis-parallel or NaN ray (MODE 1) are
// rare in the still builds (never taken for motion blur there): called out of line (DT_GENERAL_OOL),
// so their code does not shape the register allocation of the hot walks. Records go by value both ways, so no
// address of the caller's hit record or counters escapes into memory.
// Out of line in the 4-wave still builds only: C2 +5%, but the 5-wave build (96 VGPRs) loses 7.5% on
// C3 to the call's register save/restore (profiles/r04r_ab_general_ool.log)
#ifndef DT_GENERAL_OOL
#define DT_GENERAL_OOL (DT_NOSHIFT && !DT_W5)
#endif
template <class CNT>
struct GeneralHit {
  HitRec h;
  CNT cnt;
  bool any;
};
template <class CNT>
__device__ __noinline__ GeneralHit<CNT> closest_hit_general(const DScene* S, const DParams* P, Walk w, bool active,
                                                            V3 ray, V3 org, HitRec h, CNT cnt)
{
  GeneralHit<CNT> o;
  o.any = closest_hit_walk<1>(*S, *P, w, active, ray, org, 0.0f, h, cnt);
  o.h = h;
  o.cnt = cnt;
  return o;
}
template <class CNT>
struct GeneralOcc {
  CNT cnt;
  bool occl;
};
template <class CNT>
__device__ __noinline__ GeneralOcc<CNT> occluded_general(const DScene* S, const DParams* P, Walk w, bool active,
                                                         V3 bstart, V3 sn, V3 sstart, float t_max, int skip_shape,
                                                         CNT cnt);
template <class CNT>
__device__ __forceinline__ bool closest_hit_exact(const DScene& S, const DParams& P, const Walk& w, bool active, V3 ray,
                                                  V3 org, float shift, HitRec& h, CNT& cnt)
{
#if DT_GENERAL_OOL
  const GeneralHit<CNT> o = closest_hit_general(&S, &P, w, active, ray, org, h, cnt);
  h = o.h;
  cnt = o.cnt;
  return o.any;
#else
  return closest_hit_walk<1>(S, P, w, active, ray, org, shift, h, cnt);
#endif
}

template <class CNT>
__device__ __forceinline__ bool closest_hit(const DScene& S, const DParams& P, bool active, V3 ray, V3 org, float shift,
                                            HitRec& h, CNT& cnt, int pblock = -1)
{
  const Walk w = make_walk(P, active, ray, org, shift);
  if (w.inf_wave || (w.bump_wave && !bump_tree_ok(P, active, shift))) {
    return closest_hit_exact(S, P, w, active, ray, org, shift, h, cnt);
  }
  bool any;
  if (pblock >= 0 && (!w.bump_wave || P.pl_bump)) {
    // blur passes take the bump tree's lists, stored after the pass-0 lists
    const int cell = w.bump_wave ? pblock + P.pl_nbx * P.pl_nby : pblock;
    const uint32_t off = cas(S.pl_cells)[2 * cell], n = cas(S.pl_cells)[2 * cell + 1];
    any = w.bump_wave ? closest_hit_plist<true>(S, P, w, active, ray, org, shift, h, off, n, cnt)
                      : closest_hit_plist<false>(S, P, w, active, ray, org, 0.0f, h, off, n, cnt);
  } else {
    any = w.bump_wave ? closest_hit_walk<2>(S, P, w, active, ray, org, shift, h, cnt)
                      : closest_hit_walk<0>(S, P, w, active, ray, org, shift, h, cnt);
  }
  // an edge-on checkerboard hit keeps the previous test's t (Q16): only the reference order
  // reproduces it, so with the alternative trees such waves (never seen in practice) repeat the
  // walk on the reference tree
  if ((w.bump_wave || (P.n_fnodes > 0 && (P.ftree_mode & 1))) && __ballot(h.edge)) {
    return closest_hit_exact(S, P, w, active, ray, org, shift, h, cnt);
  }
  return any;
}

// intersectShadow over a gathered leaf's shapes (cpp:832-852) for the lanes of hbm that are not
// occluded yet; om collects the occluded lanes
template <class CNT>
__device__ __forceinline__ void shadow_leaf(const DScene& S, const DNodeDev& nd, unsigned long long hbm,
                                            unsigned long long& om, V3 sn, V3 sstart, float t_max, int skip_shape,
                                            float shift, CNT& cnt)
{
  DT_T(q0);
  const int nq = (nd.meta & DN_SINGLE) ? 1 : nd.aux;
  for (int q = 0; q < nq; ++q) {
    int sid, type, off;
    uint32_t flags;
    leaf_shape(S, nd, q, sid, type, flags, off);
    DT_CNT(8);
    DT_CNT(18 + (type & 7));   // shadow prim tests by type (8 -> 18)
#ifdef DT_STAMPS
    cnt.ph[42 + cnt.cur_path] += 1;   // wave-level shadow prim tests by path
#endif
    const unsigned long long tm = sid != skip_shape ? hbm & ~om : 0ull;   // lanes that test this shape
    bool o = false;
    if (inv(tm)) {
      DT_WK(DT_WK_SHADOW_SHAPE + type, true);
      o = shape_shadow(type, flags, cas(S.geom) + off, sn, sstart, t_max, shift);
    }
    const unsigned long long om_new = __ballot(o);
#ifdef DT_STAMPS
    cnt.ph[47 + (type & 7)] += __popcll(tm);
    cnt.ph[55 + (type & 7)] += __popcll(om_new);
    {   // per (light, shape): waves, lanes, hits (added by lane 0)
      if ((threadIdx.x & 63) == 0 && sid < 254 && cnt.cur_li < 8) {
        unsigned long long* h = S.stats + ST_N + 1 + DT_PH_N + 3 * (cnt.cur_li * 256 + sid);
        atomicAdd(h, 1ull);
        atomicAdd(h + 1, (unsigned long long)__popcll(tm));
        atomicAdd(h + 2, (unsigned long long)__popcll(om_new));
      }
    }
#endif
    om |= om_new;
  }
  DT_T(q1);
  DT_ACC(32, q0, q1);
}

#ifndef DT_SHAPE_FIRST
#define DT_SHAPE_FIRST 1
#endif
// Shapes first (DT_SHAPE_FIRST, motion-blur passes): a leaf occludes a lane iff the reference gathers
// it (bump_leaf_gathered) and the lane's segment hits one of its shapes. Both tests are exact, so
// they may run in either order: the shapes first for the lanes whose bumped leaf box passes (the
// gather's own first test), and the rest of the gather (the unbumped box, the parent chain) only for
// the lanes with a hit. With large shifts the padded boxes pass for most segments and the shapes
// miss (C5 frame 1920: no shadow hit in ~2900 lane tests per item), while the gather walks the
// reference ancestors for every lane whose unbumped box fails.
template <class CNT>
__device__ __forceinline__ void shadow_leaf_bump(const DScene& S, const DNodeDev& nd, int r, const Walk& w,
                                                 unsigned long long cand, unsigned long long& om, V3 bstart, V3 sn,
                                                 V3 sstart, float t_max, int skip_shape, float shift, CNT& cnt)
{
  unsigned long long hit = 0;
  shadow_leaf(S, nd, cand, hit, sn, sstart, t_max, skip_shape, shift, cnt);
  if (hit) {
    const bool g = bump_leaf_gathered(S, w, r, shift, bstart);
    om |= __ballot(inv(hit) && g);
  }
}
__device__ __forceinline__ bool bump_box(const DScene& S, const Walk& w, int r, float shift, V3 st)
{
  const DNodeDev rn = cas(S.nodes)[r];
  return box_hit(rn, rn.lb[1] - shift, rn.ub[1] + shift, w.rb, st);
}

// an occluder at distance t' < t_max along sn from sstart sits at sray-parameter
// u < 1 + 1e-3/|sray| from bstart; margins cover the f32 rounding
__device__ __forceinline__ float shadow_tcull(float t_max)
{
  return t_max > 1e-3f ? (1.0f + 1e-3f / t_max) * 1.0001f + 1e-4f : FLT_MAX;
}

// any-hit shadow test (cpp:806-855): box test with sray from isectP+sray*1e-3, shape test
// with normalized sray from isectP+sn*1e-3, skipping the light's own shape.
// MODE 3: a shadow-grid block subtree (sub, n_sub: host_shadowgrid.cpp), finite rays, no bump
template <int MODE, class CNT>
__device__ __forceinline__ bool occluded_walk(const DScene& S, const DParams& P, const Walk& w, bool active, V3 bstart,
                                              V3 sn, V3 sstart, float t_max, int skip_shape, float shift, CNT& cnt,
                                              const DNodeDev* sub = nullptr, int n_sub = 0)
{
  constexpr bool GENERAL = MODE == 1, BUMP = MODE == 2, SUB = MODE == 3;   // as closest_hit_walk
  // fast walks use the alternative tree when one was built (DT_FAST_TREE), else the reference's
  const bool ftree = !BUMP && !GENERAL && !SUB && P.n_fnodes > 0 && (P.ftree_mode & 2);
  const DNodeDev* const NODES = SUB ? sub : BUMP ? S.bnodes : ftree ? S.fnodes : S.nodes;   // any-hit: order free
  int resume = active ? 0 : 0x7fffffff;
  const unsigned long long am = __ballot(active);
  unsigned long long om = 0;   // occluded lanes
  const float tcull = (DT_WITH_RPC && P.no_cull) ? FLT_MAX : shadow_tcull(t_max);
  int i = 0;
#ifdef DT_STAMPS
  unsigned long long nv = 0;
#endif
  const int n_nodes = SUB ? n_sub : BUMP ? P.n_bnodes : ftree ? P.n_fnodes : P.n_nodes;
  while (i < n_nodes) {
    const DNodeDev nd = cas(NODES)[i];
    const bool act = GENERAL ? resume <= i : inv(am & ~om);   // see closest_hit_walk
    unsigned long long hbm = node_mask<GENERAL>(w, nd, shift, bstart, tcull, am & ~om, act);
    const bool hb = inv(hbm);
    DT_WORK(cnt.wnodes++);
    DT_WK(DT_WK_BOX, act);
    DT_CNT(27);
#ifdef DT_STAMPS
    ++nv;
#endif
    if (nd.meta & DN_LEAF) {
      DT_WK(DT_WK_BOX, BUMP && hb);
      if (BUMP && DT_SHAPE_FIRST) {
        if (hbm) shadow_leaf_bump(S, nd, nd.skip, w, hbm, om, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
      } else {
        if (BUMP && hbm) hbm = __ballot(hb & bump_leaf_gathered(S, w, nd.skip, shift, bstart));
        if (hbm) shadow_leaf(S, nd, hbm, om, sn, sstart, t_max, skip_shape, shift, cnt);
      }
      if (GENERAL) {
        if (act) resume = inv(om) ? 0x7fffffff : nd.skip;
        if (!__ballot(resume != 0x7fffffff)) break;
      } else if (!(am & ~om)) {
        break;
      }
      i = i + 1;
    } else {
      if (GENERAL && act && !hb) resume = nd.skip;
      i = hbm ? i + 1 : nd.skip;
    }
  }
#ifdef DT_STAMPS
  {   // walks whose active lanes all ended occluded (28 visits, 29 walks) / none occluded (30, 31)
    if (am && om == am) { cnt.ph[28] += nv; cnt.ph[29] += 1; }
    if (am && om == 0) { cnt.ph[30] += nv; cnt.ph[31] += 1; }
  }
#endif
  return inv(om);
}

// The shadow test over a cell's candidate list (host_shadowgrid.cpp): the same box test and
// shape tests as the walk, on the only leaves that can hold an occluder for this cell and light.
// BUMP: a motion-blur pass (lists built with sg_ypad >= bump_pad): the exact bumped gather test
template <bool BUMP, class CNT, bool SF = false>
__device__ bool occluded_list(const DScene& S, const Walk& w, bool active, V3 bstart, V3 sn, V3 sstart, float t_max,
                              int skip_shape, float shift, uint32_t off, uint32_t n, CNT& cnt)
{
  const unsigned long long am = __ballot(active);
  unsigned long long om = 0;
  const float tcull = shadow_tcull(t_max);
  for (uint32_t k = 0; k < n; ++k) {
    const int r = uni(cas(S.sg_list)[off + k]);
    const DNodeDev nd = cas(S.nodes)[r];
    const bool live = inv(am & ~om);
    DT_WK(DT_WK_BOX, live);
    DT_WK(DT_WK_BOX, BUMP && live);
    DT_CNT(34);
    if (BUMP && SF) {
      const unsigned long long cand = __ballot(live && bump_box(S, w, r, shift, bstart));
      if (cand) shadow_leaf_bump(S, nd, r, w, cand, om, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
    } else {
      const unsigned long long hbm = BUMP ? __ballot(live & bump_leaf_gathered(S, w, r, shift, bstart))
                                          : (am & ~om) & box_mask_finite(nd, w.rb, bstart, tcull);
      if (hbm) shadow_leaf(S, nd, hbm, om, sn, sstart, t_max, skip_shape, shift, cnt);
    }
    if (!(am & ~om)) break;
  }
  return inv(om);
}

// wave minimum of a per-lane int, returned wave-uniform: DPP within rows of 16 (quad perms, half
// mirror, mirror: no LDS round trips), then the four row minima through readlane on the scalar unit.
// Every lane must be enabled in exec (the callers run at wave-uniform control flow).
__device__ __forceinline__ int wave_min_u(int v)
{
  // bound_ctrl set: every source lane of these row permutations is valid, so it changes nothing, but
  // it lets the compiler fold each move into the min (v_min_i32_dpp: 4 VALU instead of 12; VALU
  // -0.9%, C3 +0.2%, C4 +0.8%, profiles/r04b_ab.log)
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));   // row_half_mirror
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));   // row_mirror
  const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return min(min(a, b), min(c, d));
}

// Scattered waves (lanes in different grid cells): each lane's own cell list holds every leaf that
// can occlude it, so the wave tests the union of its lanes' lists -- merged in leaf order (the
// lists are sorted by leaf index, built in leaf order), each leaf once, with the same exact box
// test and shape tests as the walk. A lane testing a leaf outside its own list is harmless: the
// box and shape tests are the reference's own, the list only bounds where an occluder can be.
template <bool BUMP, class CNT, bool SF = false>
__device__ bool occluded_union(const DScene& S, const Walk& w, bool active, V3 bstart, V3 sn, V3 sstart, float t_max,
                               int skip_shape, float shift, uint32_t off, uint32_t n, CNT& cnt)
{
  const unsigned long long am = __ballot(active);
  unsigned long long om = 0;
  const float tcull = shadow_tcull(t_max);
  uint32_t k = 0;
  // head: the lane's next leaf; nxt: the one after it, loaded an iteration ahead
  int head = (active && n > 0) ? S.sg_list[off] : INT_MAX;
  int nxt = (active && n > 1) ? S.sg_list[off + 1] : INT_MAX;
  while (true) {
    const int m = wave_min_u(inv(om) ? INT_MAX : head);
    if (m == INT_MAX) break;
    const DNodeDev nd = cas(S.nodes)[m];
    const bool live = inv(am & ~om);
    // only the lanes whose own list holds leaf m test it: m cannot occlude the others (their lists
    // hold every leaf that can), and a wave whose listing lanes all miss m's box skips its shapes
    const bool has = head == m;
    DT_WK(DT_WK_BOX, live);
    DT_WK(DT_WK_BOX, BUMP && live);
    DT_CNT(34);
    if (BUMP && SF) {
      const unsigned long long cand = __ballot(live && has && bump_box(S, w, m, shift, bstart));
      if (cand) shadow_leaf_bump(S, nd, m, w, cand, om, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
    } else {
      const unsigned long long hbm = BUMP ? __ballot(live & has & bump_leaf_gathered(S, w, m, shift, bstart))
                                          : (am & ~om) & __ballot(has) & box_mask_finite(nd, w.rb, bstart, tcull);
      if (hbm) shadow_leaf(S, nd, hbm, om, sn, sstart, t_max, skip_shape, shift, cnt);
    }
    if (has) {
      ++k;
      head = nxt;
      nxt = k + 1 < n ? S.sg_list[off + k + 1] : INT_MAX;
    }
  }
  return inv(om);
}

// shading point in grid-cell coordinates
__device__ __forceinline__ void sg_coords(const DParams& P, V3 p, float& x, float& y, float& z)
{
  x = ((float)p.x - P.sg_lo[0]) * P.sg_inv[0];
  y = ((float)p.y - P.sg_lo[1]) * P.sg_inv[1];
  z = ((float)p.z - P.sg_lo[2]) * P.sg_inv[2];
}

template <class CNT>
__device__ __noinline__ GeneralOcc<CNT> occluded_general(const DScene* S, const DParams* P, Walk w, bool active,
                                                         V3 bstart, V3 sn, V3 sstart, float t_max, int skip_shape,
                                                         CNT cnt)
{
  GeneralOcc<CNT> o;
  o.occl = occluded_walk<1>(*S, *P, w, active, bstart, sn, sstart, t_max, skip_shape, 0.0f, cnt);
  o.cnt = cnt;
  return o;
}

template <class CNT>
__device__ __forceinline__ bool occluded_impl(const DScene& S, const DParams& P, bool active, V3 sray, V3 bstart, V3 sn,
                                              V3 sstart, float t_max, int skip_shape, int li, float shift, CNT& cnt)
{
  const Walk w = make_walk(P, active, sray, bstart, shift);
#ifdef DT_STAMPS
  cnt.cur_path = 2;
#endif
  if (w.inf_wave || (w.bump_wave && !bump_tree_ok(P, active, shift))) {
#if DT_GENERAL_OOL
    const GeneralOcc<CNT> o = occluded_general(&S, &P, w, active, bstart, sn, sstart, t_max, skip_shape, cnt);
    cnt = o.cnt;
    return o.occl;
#else
    return occluded_walk<1>(S, P, w, active, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
#endif
  }
  // blur passes use the grid when its lists were built for their shifts (sg_ypad)
  // (umbra cells are only proven for shifts >= 0: with symmetric padding blur waves walk the tree)
  const bool bump_list = w.bump_wave && P.sg_ypad >= P.bump_pad && P.bump_up_only;
  if (w.bump_wave && !bump_list) return occluded_walk<2>(S, P, w, active, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
  // Shadow grid: the first active lane's cell serves every lane within sg_reach cells of it.
  // Waves whose lanes all lie within that reach (coherent primary bounces) test the cell's
  // candidate list. Scattered waves (mostly glossy bounces) test the union of their lanes' own
  // cell lists, merged in leaf order (C3: 4.8 leaves per union against ~24 node visits per tree
  // walk); a wave with a lane outside the grid or in a cell whose list is too long walks the tree.
  // Measured slower for scattered waves: per-lane list walks with a per-lane shape switch (C3 1725
  // vs 1932, C4 843 vs 936 Mpixel-samples/s), the lists of two cells in turn; round 4, per-lane
  // stackless tree walks (skip links, vector node loads) for the waves that fall back to the tree:
  // C3 -18% (register allocation), C4 +0.3%, the C5 transition share +16% (profiles/r04f_ab_lane_walks.log);
  // the same for scattered closest-hit walks: C3 -8.7%, C4 +3.6%, and +9% on the C5 transition share
  // in the work-sharing kernel (r04g_ab_uniform_pixel.log). The wave-uniform walk on the scalar unit wins.
  // blur passes use the padded lists, pass-0 rays the unpadded ones when a second grid was built
  const int sg_b = w.bump_wave ? P.sg_base[li] : P.sg_base0[li];
  if (li < P.sg_n && sg_b >= 0) {
    const unsigned long long am = __ballot(active);
    if (!am) return false;
    float x, y, z;
    sg_coords(P, sstart, x, y, z);
    const int first = (int)__builtin_ctzll(am);
    const float x0 = floorf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), first)));
    const float y0 = floorf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(y), first)));
    const float z0 = floorf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), first)));
    const bool inside = x0 >= 0.0f && y0 >= 0.0f && z0 >= 0.0f && x0 < (float)P.sg_dim[0] &&
                        y0 < (float)P.sg_dim[1] && z0 < (float)P.sg_dim[2];
    const float r = P.sg_reach;
    const bool near = (x >= x0 - r) & (x <= x0 + 1.0f + r) & (y >= y0 - r) & (y <= y0 + 1.0f + r) &
                      (z >= z0 - r) & (z <= z0 + 1.0f + r);
    DT_CNT(inside ? 36 : 38);   // (stamps: 38 is 0 in every config measured; also counts scattered waves below)
    if (inside && !__ballot(active & !near)) {
      const int c0 = ((int)z0 * P.sg_dim[1] + (int)y0) * P.sg_dim[0] + (int)x0;
      const DT_CAS uint32_t* e = cas(S.sg_cells) + 2 * (size_t)(sg_b + c0);
      const uint32_t off = e[0], n = e[1];
      if (off & DT_SG_UMBRA) return true;   // every segment of the cell crosses one face (host_shadowgrid.cpp)
      if (n != DT_SG_WALK) {
        DT_CNT(35);
#ifdef DT_STAMPS
        cnt.cur_path = 0;
#endif
        if (bump_list)
          return occluded_list<true, CNT, DT_SHAPE_FIRST>(S, w, active, bstart, sn, sstart, t_max, skip_shape, shift, off, n, cnt);
        return occluded_list<false>(S, w, active, bstart, sn, sstart, t_max, skip_shape, 0.0f, off, n, cnt);
      }
      DT_CNT(37);
    }
    {   // scattered waves: the union of the lanes' own cell lists, when every lane has one
      const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
      bool lin = fx >= 0.0f && fy >= 0.0f && fz >= 0.0f && fx < (float)P.sg_dim[0] && fy < (float)P.sg_dim[1] &&
                 fz < (float)P.sg_dim[2];
      uint32_t loff = 0, ln = 0;
      bool umb = false;   // the lane's own cell is an umbra cell: every segment from it crosses one face
      if (active && lin) {
        const int cl = ((int)fz * P.sg_dim[1] + (int)fy) * P.sg_dim[0] + (int)fx;
        const uint2 e = ((const uint2*)S.sg_cells)[(size_t)sg_b + cl];
        loff = e.x;
        ln = e.y;
        lin = ln != DT_SG_WALK;
        umb = DT_UMBRA_LANES && lin && (loff & DT_SG_UMBRA) != 0u;
      }
      DT_CNT(40);
      if (!lin) ln = 0;
      loff &= ~DT_SG_UMBRA;   // an umbra cell's list holds its occluding face's leaf
      // (a wave with some lanes outside the lists walks the tree for all of them: splitting it,
      // the union for the others, measured C3 +0.9% and C4 -3.2%, profiles/r03t)
      const unsigned long long out_lanes = __ballot(active && !lin);
#ifdef DT_STAMPS
      if (out_lanes && __ballot(active && !(fx >= 0.0f && fy >= 0.0f && fz >= 0.0f && fx < (float)P.sg_dim[0] &&
                                            fy < (float)P.sg_dim[1] && fz < (float)P.sg_dim[2])))
        cnt.ph[38] += 1;   // a scattered wave with a lane outside the grid
#endif
      if (!out_lanes) {
        DT_CNT(41);
#ifdef DT_STAMPS
        cnt.cur_path = 1;
#endif
        // lanes in umbra cells are occluded as they are; the rest take the union of their lists
        const bool rest = active && !umb;
        if (DT_UMBRA_LANES && !__ballot(rest)) return true;
        if (bump_list)
          return occluded_union<true, CNT, DT_SHAPE_FIRST>(S, w, rest, bstart, sn, sstart, t_max, skip_shape, shift, loff, ln, cnt) || umb;
        return occluded_union<false>(S, w, rest, bstart, sn, sstart, t_max, skip_shape, 0.0f, loff, ln, cnt) || umb;
      }
// (bit 3: DT_SHAPE_TRIANGLE is an enum constant, which #if would read as 0; rounds 4-5 had that, so
// this block was compiled out of the mesh builds)
static_assert(DT_SHAPE_TRIANGLE == 3, "DT_HAS(3) below");
#if DT_HAS(3)
      // Some lanes' cells walk the tree (lists over the cap: C4's mesh cells; with scattered glossy
      // bounces one such lane used to send all 64 down the whole tree). With block subtrees
      // (host_shadowgrid.cpp, DT_SG_SUBTREE; pass-0 waves, every lane inside the grid) the wave is
      // split: the lanes of list cells take the union of their lists as above, and the lanes of
      // tree-walk cells, when they lie in at most P.sgb_multi blocks (DT_SG_SUB_MULTI), walk their
      // blocks' subtrees, one block after another with its own lanes. A block's subtree holds every
      // leaf that can occlude a segment from any of its cells. Otherwise the whole tree as before.
      DT_CNT(64);   // scattered waves with lanes in tree-walk cells (stamps 64-68: the subtree gates)
      if (!w.bump_wave && P.sgb_base[li] >= 0) {
        DT_CNT(65);
        const bool gin = fx >= 0.0f && fy >= 0.0f && fz >= 0.0f && fx < (float)P.sg_dim[0] &&
                         fy < (float)P.sg_dim[1] && fz < (float)P.sg_dim[2];
        const int blk = gin ? (((int)fz / P.sgb_bz) * P.sgb_nby + (int)fy / P.sgb_by) * P.sgb_nbx + (int)fx / P.sgb_bx : -1;
        const uint2* const recs = (const uint2*)S.sub_blocks + P.sgb_base[li];
        const bool wl = active && !lin;   // lanes in tree-walk cells (or outside the grid: blk < 0)
        unsigned long long rem = __ballot(wl);
        int nb = 0;
        while (rem && nb < P.sgb_multi) {
          const int b0 = __builtin_amdgcn_readlane(blk, (int)__builtin_ctzll(rem));
          if (b0 < 0 || recs[b0].y == 0) {
            DT_CNT(b0 < 0 ? 66 : 67);
            break;
          }
          rem &= ~__ballot(wl && blk == b0);
          ++nb;
        }
        if (rem && nb >= P.sgb_multi) DT_CNT(68);   // lanes in more blocks than sgb_multi
        if (!rem) {
          bool occl = false;
          const bool ll = active && lin;
          if (__ballot(ll)) {
            DT_CNT(41);
#ifdef DT_STAMPS
            cnt.cur_path = 1;
#endif
            occl = occluded_union<false>(S, w, ll, bstart, sn, sstart, t_max, skip_shape, 0.0f, loff, ln, cnt) && ll;
          }
          unsigned long long todo = __ballot(wl);
          while (todo) {
            const int b0 = __builtin_amdgcn_readlane(blk, (int)__builtin_ctzll(todo));
            const uint2 e = recs[b0];
            const bool mine = inv(todo) && blk == b0;
            todo &= ~__ballot(mine);
            DT_CNT(63);
#ifdef DT_STAMPS
            cnt.cur_path = 3;
#endif
            const bool o = occluded_walk<3>(S, P, w, mine, bstart, sn, sstart, t_max, skip_shape, 0.0f, cnt,
                                            S.sub_nodes + uni((int)e.x), uni((int)e.y));
            occl = occl || (mine && o);
          }
          return occl;
        }
      }
#endif
    }
  }
#ifdef DT_STAMPS
  cnt.cur_path = 2;
#endif
  if (w.bump_wave) return occluded_walk<2>(S, P, w, active, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
  return occluded_walk<0>(S, P, w, active, bstart, sn, sstart, t_max, skip_shape, shift, cnt);
}

// the shadow test (occluded_impl); stamps builds: its cycles by path (69 cell list, 70 union of the
// lanes' lists, 71 tree walks and the rest)
template <class CNT>
__device__ __forceinline__ bool occluded(const DScene& S, const DParams& P, bool active, V3 sray, V3 bstart, V3 sn,
                                         V3 sstart, float t_max, int skip_shape, int li, float shift, CNT& cnt)
{
#ifdef DT_STAMPS
  DT_T(oa);
  const bool o = occluded_impl(S, P, active, sray, bstart, sn, sstart, t_max, skip_shape, li, shift, cnt);
  DT_T(ob);
  cnt.ph[69 + (cnt.cur_path == 0 ? 0 : cnt.cur_path == 1 ? 1 : 2)] += ob - oa;
  return o;
#else
  return occluded_impl(S, P, active, sray, bstart, sn, sstart, t_max, skip_shape, li, shift, cnt);
#endif
}

// =====================================================================================
// rayColor as a per-lane DFS (render_final_project.cpp:487-961)
// =====================================================================================
struct Entry {
  V3 a;        // NODE: ray     FINISH: colour to add
  V3 b;        // NODE: origin
  float k;
  int depth;   // >0 NODE ; -1 FINISH
  uint32_t key;
  int _pad;
};

struct PassOut {
  V3 color;
  bool hit;
  bool in_motion;
};

// per-lane event counters, kept in registers for the whole persistent loop and reduced
// across the wave once at kernel exit (same-address atomics per lane serialise at L2)
// wave-level event counters of dt_stats (rays, shadow rays, texel fetches) in the wave's LDS: one
// lane adds the ballot's popcount. Per-lane counters in VGPRs were live across every walk and
// spilled/reloaded around them (a scratch store per light iteration).
// The abort conditions the reference reports (stack overflows, reflection errors, glossy and
// sphere-light resample exhaustion, UV out of range, prism-normal fallbacks) count per lane into the
// same LDS words (LDS atomics), so that an item's counts can be taken back (DT_SKY_AGAIN items).
enum { WC_RAYS = 0, WC_SHADOW = 1, WC_TEX = 2, WC_STACK = 3, WC_REFL = 4, WC_GLOSSY = 5, WC_UV = 6, WC_PRISM = 7,
       WC_SPHL = 8, WC_N = 9 };
#define DT_WCNT(k, cond)                                                                 \
  do {                                                                                   \
    const unsigned long long m_ = __ballot(cond);                                        \
    if (m_ && (int)(threadIdx.x & 63) == (int)__builtin_ctzll(m_)) cnt.wc[(k)] += (unsigned)__popcll(m_); \
  } while (0)

struct Counters {
  unsigned int* wc;                  // WC_N wave counters (LDS), flushed at exit
  uint32_t box, prim;
  uint32_t wnodes;                   // wave-level
#ifdef DT_WORK_COUNTERS
  unsigned int* wk;                  // the wave's DT_WK_N event counters (LDS)
#endif
#ifdef DT_STAMPS
  unsigned long long ph[DT_PH_N];   // diagnostic build only: cycles per phase, event counts (wave-uniform)
  int cur_li;                  // light of the current shadow test (per-shape histogram)
  int cur_path;                // shadow path of the current test: 0 cell list, 1 union, 2 tree walk
#endif
};

struct Ctx {
  const DScene* S;
  const DParams* P;
  Rng rng;
};

__device__ __forceinline__ bool is_refl_material(int m)
{
  return m == DT_MAT_GLASS || m == DT_MAT_STEEL || m == DT_MAT_ALUMINUM || m == DT_MAT_WATER ||
         m == DT_MAT_LINOLEUM;
}

// glossy sample rectangle (cpp:648-669 / 742-755)
__device__ __forceinline__ void glossy_rect(V3 refl_ray, V3 isectP, float mult, V3& A, V3& B, V3& C, V3& D, V3& wv, V3& lv)
{
  const float length = 1, width = 0.5;
  V3 gloss_ray = mul(mult, refl_ray);
  lv = normalized(cross(gloss_ray, v3(1, 0, 0)));
  if (is_approx_zero(lv)) lv = cross(gloss_ray, v3(0, 0, 1));
  V3 cc = add(gloss_ray, isectP);
  V3 p1 = add(mul(length / 2, lv), cc);
  wv = normalized(cross(neg(gloss_ray), lv));
  A = add(divs(mul(width, wv), 2), p1);
  B = sub(A, mul(length, lv));
  C = sub(B, mul(width, wv));
  D = sub(A, mul(width, wv));
}

__device__ __forceinline__ V3 rect_sample_f(V3 A, V3 B, V3 D, float x, float y)
{
  return add(add(A, mul(x, sub(B, A))), mul(y, sub(D, A)));
}
__device__ __forceinline__ V3 rect_sample(V3 A, V3 B, V3 D, double u0, double u1)
{
  return rect_sample_f(A, B, D, (float)u0, (float)u1);
}

// sphereLight::sampleRay (geometry.cpp:2770-2826, Q11: returns the sampled point) -- rejection
// sampling with acos/sin/cos (no C2-C5 scene has a sphere light). Everything stays inlined: a real
// call anywhere in the trace kernel costs ~25% (calling-convention register saves/spills)
__device__ __forceinline__ V3 sphere_light_sample(const Ctx& c, const DT_CAS DLight& L, int li, V3 point,
                                                            uint32_t node, unsigned int* st_sphl)
{
  V3 C = v3a(L.center), baxis = v3a(L.baxis);
  int attempt = 0;
  double u0, u1;
  c.rng.draw(node, P_SPHL, ((uint32_t)li << 8) | (uint32_t)attempt, u0, u1);
  double theta = 2 * M_PI * u0, phi = acos(1 - 2 * u1);
  V3 dir = v3(sin(phi) * cos(theta), sin(phi) * sin(theta), cos(phi));
  V3 tmp = add(mul(L.radius, dir), C);
  int sample_limit = 20;
  while (dot(sub(tmp, C), sub(point, C)) < 0 || (L.use_baxis && dot(sub(tmp, C), baxis) < 0)) {
    if (sample_limit < 0) { if (st_sphl) atomicAdd(st_sphl, 1u); break; }
    V3 rev = add(mul(-L.radius, dir), C);
    if (dot(sub(rev, C), sub(point, C)) >= 0 && (!L.use_baxis || dot(sub(rev, C), baxis) >= 0)) {
      tmp = rev;
      break;
    }
    attempt++;
    c.rng.draw(node, P_SPHL, ((uint32_t)li << 8) | (uint32_t)attempt, u0, u1);
    theta = 2 * M_PI * u0;
    phi = acos(1 - 2 * u1);
    dir = v3(sin(phi) * cos(theta), sin(phi) * sin(theta), cos(phi));
    tmp = add(mul(L.radius, dir), C);
    sample_limit--;
  }
  return tmp;
}

// light sampleRay (geometry.cpp:2751-2849)
// Area lights 2k and 2k+1 share one draw (sub-index k): words 0-1 are light 2k's (x, y), words
// 2-3 light 2k+1's. `pair` keeps words 2-3 of an even light's draw, with
// pair[2] = the odd light they belong to, so the odd light does not draw again.
__device__ __forceinline__ V3 light_sample(const Ctx& c, const DT_CAS DLight& L, int li, V3 point, uint32_t node,
                                           unsigned int* st_sphl, uint32_t* pair = nullptr)
{
  if (L.type == DT_LIGHT_POINT) return sub(v3a(L.center), point);
  if (L.type == DT_LIGHT_RECT) {
    DT_NEED(DT_FEAT_RECTL);
    const bool odd = (li & 1) != 0;
    uint32_t w0, w1;
    if (odd && pair && pair[2] == (uint32_t)li) {
      w0 = pair[0];
      w1 = pair[1];
    } else {
      uint32_t o[4];
      c.rng.draw_words(node, P_LIGHT, (uint32_t)li >> 1, o);
      w0 = odd ? o[2] : o[0];
      w1 = odd ? o[3] : o[1];
      if (pair && !odd) { pair[0] = o[2]; pair[1] = o[3]; pair[2] = (uint32_t)li + 1u; }
    }
    return sub(rect_sample_f(v3a(L.A), v3a(L.B), v3a(L.D), f01(w0), f01(w1)), point);
  }
  DT_NEED(DT_FEAT_SPHL);
  return sphere_light_sample(c, L, li, point, node, st_sphl);
}

// helpers.h:313-317 (Q10)
// R0 = (float)(((r0-1)^2 + r1^2) / ((r0+1)^2 + r1^2)) is per material (DMat::ct_r0, host)
__device__ __forceinline__ float schlick_complex(float cos_theta, float R0)
{
  return (float)((R0 + (1 - R0)) + pw5((double)(1 - cos_theta)));
}

// the light's BRDF at a hit (cpp:894-948): Oren-Nayar, Cook-Torrance, raw or Phong
__device__ __forceinline__ V3 brdf(const DParams& P, const DMat& M, const DT_CAS DLight& L, V3 normal, V3 e_dir,
                                   V3 sray, V3 sn, V3 shape_color)
{
  V3 lc = v3a(L.color);
  V3 ray_col;
  const float roughness = M.roughness;
  if (M.model == DT_MODEL_OREN_NAYAR) {
    DT_NEED(DT_FEAT_ON);
    const float A = M.on_a, B = M.on_b;   // per material (host, cpp:896-897)
    float vn = (float)dot(e_dir, normal);
    float ln = (float)dot(sn, normal);
    float irradiance = fmaxr(0.0f, ln);
    float vn_theta = cr_acosf(vn), ln_theta = cr_acosf(ln);
    float angleDiff = (float)dmax(0.0, dot(normalized(sub(e_dir, mul(vn, normal))),
                                           normalized(sub(sray, mul(ln, normal)))));
    float alpha = fmaxr(vn_theta, ln_theta), beta = fminr(vn_theta, ln_theta);
    float f = A + B * angleDiff * cr_sinf(alpha) * cr_tanf(beta);
    ray_col = mul(f, mul(irradiance, cwise(shape_color, lc)));
  }
  else if (M.model == DT_MODEL_COOK_TORRANCE) {
    V3 H = normalized(add(e_dir, sray));
    float hn = (float)dmax(0.0, dot(normal, H));
    float vh = (float)dot(e_dir, H);
    float vn = (float)dot(e_dir, normal);
    float ln = (float)dot(sn, normal);
    float alpha = cr_acosf(hn);
    double sa, ca;
    cr_sincos_d(alpha, sa, ca);   // cosf(alpha), tanf(alpha) from one reduction
    const float cos_a = (float)ca, tan_a = (float)(sa / ca);
    float D = (float)(1 / (pw2((double)roughness) * pw4((double)cos_a)) *
                      exp(-pw2((double)(tan_a / roughness))));
    float G1 = (float)(2.0 * hn * vn / vh);
    float G2 = (float)(2.0 * hn * ln / vh);
    float G = 1.0f;
    if (G1 < G) G = G1;
    if (G2 < G) G = G2;
    float F = schlick_complex(vn, M.ct_r0);
    float fdg = F * D * G;
    double den = (double)(ln * vn) * M_PI;
    V3 shader_rgb = add(mul(fmaxr(0.0f, ln), mul(0.4, lc)), divs(mul(fdg, mul(0.8, lc)), den));
    ray_col = cwise(shape_color, shader_rgb);
  } else if (M.model == DT_MODEL_RAW) {
    ray_col = shape_color;
  } else {
    V3 r = normalized(add(mul(-1, sray), mul(2 * dot(normal, sray), normal)));
    double m1 = dmax(0.0, dot(normal, sn));
    double pp = pw_rt(dmax(0.0, dot(r, e_dir)), (double)P.phong);
    V3 shader_rgb = add(mul(m1, lc), mul(pp, lc));
    ray_col = cwise(shape_color, shader_rgb);
  }
  return ray_col;
}

// =====================================================================================
// DFS work sharing (DT_DONATE, dt_trace_kernel_dn)
// =====================================================================================
// A deep glossy cascade keeps one lane of its wave busy for ~100 DFS steps while the other 63 are
// done (at 8 ranks one such wave bounds a rank's kernel). Here a lane whose own sample
// is finished takes a whole pending subtree (a NODE entry) from a lane that has more than one, and
// runs it as a DFS of its own. The reference adds every node's own light to one accumulator in DFS
// post-order; a subtree's additions are a contiguous run of that sequence, so the thief records its
// colours in order in a list (records in global memory) and the owner, reaching the REPLAY marker
// left in place of the entry, adds them one by one: the same additions in the same order, bit for
// bit. A thief's own donations become SUBLIST records of its list, replayed in place. in_motion
// (the last rayColor's, Q6) is kept as the value of the node with the largest pre-order path
// (_pad: 3 bits per level, the call slot + 1), so it does not depend on who ran which node.
#if DT_DONATE
#define DN_BLK 16              // records per block; the last slot of a block links to the next
#define DN_NBLK (DT_DN_POOL_REC / DN_BLK)
#define DN_LIMIT (DN_NBLK / 2) // no new donation once this many blocks are in use
enum { DN_COLOR = 1, DN_LINK = 2, DN_SUB = 3, DN_END = 4 };
struct DnRec {
  double x, y, z;
  uint32_t tag;
  uint32_t aux;                // LINK: next record; SUB: the sublist's first block; END: max pre-order path
};
struct DnCtx {
  DnRec* pool;                 // this wave's records
  unsigned* next;              // LDS: blocks handed out
  unsigned* done;              // LDS: bit per block: the list starting there is complete
  int* pair;                   // LDS: donor lane per pairing rank
};
// append a record to the list being filled at pos (chaining a new block when this one is full)
__device__ __forceinline__ void dn_put(const DnCtx& dn, int& pos, double x, double y, double z, uint32_t tag,
                                       uint32_t aux, unsigned long long* ovf)
{
  if ((pos & (DN_BLK - 1)) == DN_BLK - 1) {
    const unsigned nb = atomicAdd(dn.next, 1u);
    if (nb >= DN_NBLK) {
      // pool full: the list ends here (an END record in the link slot, so its replay terminates);
      // counted in dt_stats.donate_overflow, which the tests require to be zero
      atomicAdd(ovf, 1ull);
      DnRec& l = dn.pool[pos];
      l.x = 0.0;
      l.tag = DN_END;
      l.aux = 0u;
      return;
    }
    DnRec& l = dn.pool[pos];
    l.tag = DN_LINK;
    l.aux = nb * DN_BLK;
    pos = (int)(nb * DN_BLK);
  }
  DnRec& r = dn.pool[pos];
  r.x = x; r.y = y; r.z = z;
  r.tag = tag;
  r.aux = aux;
  ++pos;
}
#define DT_ROOT_PAD 0
#else
#define DT_ROOT_PAD 1
#endif

// One full rayColor tree for the lanes with `active`. Appends to out.color in the
// reference's accumulation order.
__device__ __forceinline__ void run_pass(const Ctx& c_in, bool active, V3 ray0, V3 org0, uint32_t rootkey, float shift_in,
                         PassOut& out, Entry* stack, Counters& cnt, double (*nrec)[DT_WAVE],
                         double (*ocol)[DT_WAVE], double (*tcol)[DT_WAVE]
#if DT_DONATE
                         , const DnCtx& dn
#endif
                         )
{
#if DT_DONATE
  // the sample whose node the lane works on: its own, or (a thief) the donor's
  Ctx c = c_in;
  float shift = shift_in;
  int out_pos = -1;            // -1: own sample (colours into ocol); else the next record of the list being filled
  int out_blk = 0;             // first block of that list (its done bit)
  int npend = 0;               // NODE entries (depth > 0) on the lane's stack
  int mk_o = -1, mk_t = -1;    // largest pre-order path seen: own sample / current list
  bool mo_o = false, mo_t = false;   // its in_motion
  int dn_steps = 0;
  const int lane_ = threadIdx.x & (DT_WAVE - 1);
  if (lane_ == 0) *dn.next = 0;
  for (int q = lane_; q < DN_NBLK / 32; q += DT_WAVE) dn.done[q] = 0u;
  __syncthreads();
  auto emit = [&](const V3& a) {   // a node's own light, in the reference's accumulation order
    if (out_pos < 0) {
      ocol[0][lane_] = ocol[0][lane_] + a.x;
      ocol[1][lane_] = ocol[1][lane_] + a.y;
      ocol[2][lane_] = ocol[2][lane_] + a.z;
    } else {
      dn_put(dn, out_pos, a.x, a.y, a.z, DN_COLOR, 0u, c.S->stats + ST_DN_OVF);
    }
  };
#else
  const Ctx& c = c_in;
  const float shift = DT_NOSHIFT ? 0.0f : shift_in;
#endif
  const DScene& S = *c.S;
  const DParams& P = *c.P;
  int sp = 0;
  int prio_steps = 0;
  if (active && P.max_depth > 0) {
    Entry e;
    e.a = ray0; e.b = org0; e.k = 1.0f; e.depth = P.max_depth; e.key = rootkey; e._pad = DT_ROOT_PAD;  // root
    stack[sp++] = e;
#if DT_DONATE
    npend = 1;
#endif
  }
  while (true) {
    DT_T(t0);
#if DT_DONATE
    // ---- work sharing: a free lane (own sample finished, no list open) takes the bottom-most
    // pending NODE of a lane that has two or more (the one processed last: the most overlap) ----
    // only once the pass has run P.donate_after steps: the common item (1.5 steps) never pays for it
    if (P.donate && ++dn_steps > P.donate_after) {
      const bool free_l = sp == 0 && out_pos < 0;
      const bool donor = npend >= 2 && *dn.next < DN_LIMIT;
      const unsigned long long fm = __ballot(free_l), dm = __ballot(donor);
      if (fm && dm) {
        const int np = min(__popcll(fm), __popcll(dm));
        const int rf = __popcll(fm & ((1ull << lane_) - 1)), rd = __popcll(dm & ((1ull << lane_) - 1));
        const bool give = donor && rd < np, take = free_l && rf < np;
        if (give) dn.pair[rd] = lane_;
        __syncthreads();
        const int src = take ? dn.pair[rf] : lane_;
        __syncthreads();
        Entry de;
        de.a = v3(0, 0, 0); de.b = v3(0, 0, 0); de.k = 0; de.depth = 0; de.key = 0; de._pad = 0;
        uint32_t blk = 0;
        if (give) {
          int b = 0;
          while (stack[b].depth <= 0) ++b;   // npend >= 2: a NODE entry exists below the top
          de = stack[b];
          blk = atomicAdd(dn.next, 1u);
          stack[b].depth = -2;               // REPLAY the list that starts at block blk
          stack[b].key = blk;
          --npend;
          atomicAdd(S.stats + ST_DONATE, 1ull);
        }
        // move the entry and the donor's sample identity (RNG pixel/sample, blur shift) to the thief
        const int* ew = (const int*)&de;
        int tw[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) tw[q] = __shfl(ew[q], src, DT_WAVE);
        const uint32_t tblk = (uint32_t)__shfl((int)blk, src, DT_WAVE);
        const uint32_t tpix = (uint32_t)__shfl((int)c.rng.pixel, src, DT_WAVE);
        const uint32_t tsmp = (uint32_t)__shfl((int)c.rng.sample, src, DT_WAVE);
        const float tsh = __int_as_float(__shfl(__float_as_int(shift), src, DT_WAVE));
        if (take) {
          Entry te;
          int* tv = (int*)&te;
#pragma unroll
          for (int q = 0; q < 16; ++q) tv[q] = tw[q];
          stack[0] = te;
          sp = 1;
          npend = 1;
          out_blk = (int)tblk;
          out_pos = (int)(tblk * DN_BLK);
          c.rng.pixel = tpix;
          c.rng.sample = tsmp;
          shift = tsh;
          mk_t = -1;
          mo_t = false;
        }
      }
    }
#endif
    // pop FINISH entries (own-light contributions), then the next NODE
    bool have = false;
#if DT_DONATE
    bool waiting = false;   // a donated subtree's list is not complete yet
#endif
    int pidx = 0;   // the popped NODE entry's slot
#if DT_DONATE
    while (sp > 0) {
      const int d = stack[--sp].depth;
      if (d == -1) {
        emit(stack[sp].a);
      } else if (d > 0) {
        pidx = sp;
        have = true;
        --npend;
        break;
      } else if (d <= -2) {   // a donated subtree: REPLAY its list (-2), or CONTINUE replaying it (-3)
        const uint32_t blk = stack[sp].key;
        if (out_pos >= 0) {    // filling a list ourselves: splice the sublist in, replayed in place later
          dn_put(dn, out_pos, 0.0, 0.0, 0.0, DN_SUB, blk, S.stats + ST_DN_OVF);
          continue;
        }
        if (!(dn.done[blk >> 5] & (1u << (blk & 31)))) {   // its thief is still at it: wait
          ++sp;
          waiting = true;
          break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the records were written by another lane
        int pos = d == -2 ? (int)(blk * DN_BLK) : (int)__float_as_uint(stack[sp].k);
        while (true) {
          const DnRec r = dn.pool[pos];
          if (r.tag == DN_COLOR) {
            ocol[0][lane_] = ocol[0][lane_] + r.x;
            ocol[1][lane_] = ocol[1][lane_] + r.y;
            ocol[2][lane_] = ocol[2][lane_] + r.z;
            ++pos;
          } else if (r.tag == DN_LINK) {
            pos = (int)r.aux;
          } else if (r.tag == DN_SUB) {
            // the rest of this list after the sublist: CONTINUE here, the sublist's REPLAY above it
            stack[sp].depth = -3;
            stack[sp].k = __uint_as_float((uint32_t)(pos + 1));
            ++sp;
            if (sp < DT_STACK_MAX) {
              stack[sp].depth = -2;
              stack[sp].key = r.aux;
              ++sp;
            } else {
              atomicAdd(cnt.wc + WC_STACK, 1u);
            }
            break;
          } else {   // DN_END: the list's (largest pre-order path, in_motion)
            if ((int)r.aux >= mk_o) { mk_o = (int)r.aux; mo_o = r.x != 0.0; }
            break;
          }
        }
      }
      // d == 0: an exhausted glossy sample's no-op entry
    }
    if (out_pos >= 0 && sp == 0 && !have) {
      // a thief's subtree is done: close its list, then it is free again (its own identity back)
      dn_put(dn, out_pos, mo_t ? 1.0 : 0.0, 0.0, 0.0, DN_END, (uint32_t)mk_t, S.stats + ST_DN_OVF);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      atomicOr(&dn.done[(uint32_t)out_blk >> 5], 1u << ((uint32_t)out_blk & 31));
      out_pos = -1;
      c.rng = c_in.rng;
      shift = shift_in;
    }
    if (!__ballot(have || waiting)) break;
#else
    while (sp > 0) {
      // read the depth word first: a FINISH entry only carries its colour
      const int d = stack[--sp].depth;
      if (d < 0) {
        const V3 a = stack[sp].a;
        const int l = threadIdx.x & (DT_WAVE - 1);   // out.color += own light (in LDS)
        ocol[0][l] = ocol[0][l] + a.x;
        ocol[1][l] = ocol[1][l] + a.y;
        ocol[2][l] = ocol[2][l] + a.z;
      } else if (d > 0) {
        pidx = sp;
        have = true;
        break;
      }
    }
    if (!__ballot(have)) break;
#endif
    DT_CNT(7);
    // A deep glossy cascade (fan-out 2 per bounce, ~100 DFS steps for one lane against ~1.5 on
    // average; C3 has a column of such pixels) keeps its wave busy up to ~80x the mean item (7.6 ms
    // of wave time, tools/item_times.py): with the frame split over ranks that one wave bounds a
    // rank's kernel. Such a wave raises its issue priority once its tree grows long (reset at the
    // end of the item). C3 at 8 ranks: slowest rank 7.45 -> 6.95 ms; at 1 rank it costs 0.5%, so
    // the host enables it for tile splits only (P.prio_steps).
    if (++prio_steps == P.prio_steps) __builtin_amdgcn_s_setprio(DT_PRIO_LEVEL);
    // The popped NODE entry stays in its stack slot until this step's FINISH record overwrites it
    // at the very end (the FINISH slot is that same slot), so its fields are read from there where
    // they are used, behind compiler barriers, instead of being held in registers across the walks:
    // the allocator spilled them to scratch right after the pop, a store of data already there.
    // (re-reading node key and k inside the light loops as well measured C3 -2.7%, profiles/r03f)
#define DT_EF(f) (stack[pidx].f)
    V3 ray = DT_EF(a), eye = DT_EF(b);
    const bool is_root = have && DT_EF(_pad) == DT_ROOT_PAD;
#if DT_DONATE
    // in_motion of the node with the largest pre-order path so far (own sample / current list)
    if (have) {
      const int path = DT_EF(_pad);
      if (out_pos < 0) { if (path >= mk_o) { mk_o = path; mo_o = false; } }
      else if (path >= mk_t) { mk_t = path; mo_t = false; }
    }
#else
    if (have) out.in_motion = false;   // cpp:519
#endif
    DT_WCNT(WC_RAYS, have);

    DT_T(t1);
    DT_ACC(0, t0, t1);
    HitRec h;
#ifdef DT_STAMPS
    const unsigned long long v_before = cnt.ph[26];
#endif
    // primary rays: the pixel block's candidate list, when the wave's pixels share one block
    // (host_primlists.cpp; blur passes take the bump tree's lists when they were built)
    int pblock = -1;
    if (P.pl_block > 0 && __ballot(is_root) && (P.pl_bump || !__ballot(have && shift != 0.0f)) && P.n_fnodes > 0 &&
        (P.ftree_mode & 1)) {
      const int px = (int)(c.rng.pixel % (uint32_t)P.xRes), py = (int)(c.rng.pixel / (uint32_t)P.xRes);
      const int blk = (py / P.pl_block) * P.pl_nbx + px / P.pl_block;
      const int b0 = uni(blk);
      if (!__ballot(have && blk != b0)) pblock = b0;
    }
    bool any = closest_hit(S, P, have, ray, eye, shift, h, cnt, pblock);
    asm volatile("" ::: "memory");   // the entry's fields: fresh loads, not values kept across the walk
    ray = DT_EF(a);
    eye = DT_EF(b);
    const int depth = DT_EF(depth);
    const float k = DT_EF(k);
    const uint32_t node = DT_EF(key);
#ifdef DT_STAMPS
    if (__ballot(is_root)) { cnt.ph[46] += cnt.ph[26] - v_before; cnt.ph[39] += 1; }
#endif
    DT_T(t2);
    DT_ACC(1, t1, t2);
    any = any && have && h.shape >= 0;
    if (have && is_root && any) out.hit = true;

    // ---- per-lane hit processing: normal, reflection children (cpp:546-769) ----------
    V3 isectP = v3(0, 0, 0), normal = v3(0, 0, 0), in = v3(0, 0, 0), shape_color = v3(0, 0, 0);
    int sid = any ? h.shape : 0;
    DShapeHdr hd;
    hd.type = 0; hd.off = 0; hd.flags = 0;
    int fin_slot = -1;
    bool shade = false;     // needs the light loop
    V3 own = v3(0, 0, 0);
    if (any) {
      DT_WK(DT_WK_HIT, true);
      hd = S.hdr[sid];
      GP g = cas(S.geom) + hd.off;
      const DMat& M = S.mat[sid];
      isectP = add(eye, mul(h.t_min, ray));
      normal = shape_norm(hd.type, hd.flags, g, isectP, shift, cnt.wc + WC_PRISM, h.ccol);
      in = normalized(ray);
      shape_color = h.ccol >= 0 ? G3(g, h.ccol) : v3a(M.color);
#if DT_DONATE
      {
        const bool mv = (M.flags & DT_F_MOTION) != 0;
        const int path = DT_EF(_pad);
        if (out_pos < 0) { if (path == mk_o) mo_o = mv; }
        else if (path == mk_t) mo_t = mv;
      }
#else
      out.in_motion = (M.flags & DT_F_MOTION) != 0;
#endif
      if (dot(mul(1e4, in), normal) >= 0) normal = mul(-1, normal);   // fixNorm

      // reserve the FINISH slot below the children
      if (sp < DT_STACK_MAX) { fin_slot = sp++; }
      else atomicAdd(cnt.wc + WC_STACK, 1u);

      if (P.reflect && is_refl_material(M.material)) {
        const float eps = 1e-3f;
        const bool glossy = (M.flags & DT_F_GLOSSY) != 0;
        float k_refl = 1, k_refr = 1;
        // Children are written straight into their stack slots in reverse call order, so the
        // reference's call order comes out of the LIFO: [base, base+nref) reflection children
        // (glossy sample nref-1 .. 0, or the mirror ray), base+nref the refraction child
        // (glass, called first in cpp:592-626). A glossy sample that exhausts its resamples
        // leaves a depth-0 entry, which pops as a no-op (a depth-0 rayColor returns at once).
        // At depth 1 the children would return immediately: none are generated.
        if (depth - 1 > 0) {
#if DT_DONATE
          // pre-order path of a child: the parent's, plus its call slot + 1 at the child's level (3 bits
          // per level from bit 27 down; host: max_depth <= 11, brdf_samples <= 6)
          const int cpath_base = DT_EF(_pad);
          const int cpath_shift = 30 - 3 * (P.max_depth - depth + 1);
#define DT_CPATH(d) (cpath_base | ((d) << cpath_shift))
#define DT_NPEND(cond) (npend += (cond) ? 1 : 0)
#else
#define DT_CPATH(d) 0
#define DT_NPEND(cond) ((void)0)
#endif
          V3 refl_ray = sub(in, mul(2 * dot(normal, in), normal));
          const double rn = dot(refl_ray, normal);
          int nref = 0;
          if (rn <= 0) atomicAdd(cnt.wc + WC_REFL, 1u);
          else if (rn > eps) nref = (glossy && !P.nogloss) ? P.brdf_samples : 1;
          const bool glass = DT_HAS(DT_FEAT_GLASS) && M.material == DT_MAT_GLASS;
          const int base = sp;
          if (base + nref + (glass ? 1 : 0) > DT_STACK_MAX) {
            atomicAdd(cnt.wc + WC_STACK, 1u);
            nref = 0;
          } else {
            sp = base + nref;
            if (glass) {
              DT_WK(DT_WK_REFRACT, true);
              float cos_theta = (float)dot(normal, neg(in));
              float sin_theta = (float)sqrt(1 - pw2((double)cos_theta));
              float r1 = h.inside ? P.refr_glass : P.refr_air, r2 = h.inside ? P.refr_air : P.refr_glass;
              float chk = (float)(1 - pw2((double)(r1 / r2)) * (1 - pw2(dot(in, normal))));
              if (chk >= 0) {
                float a = r1 / r2 * sin_theta;
                float b = 1 / sin_theta;
                float sq = sqrtf(chk);
                V3 outr = sub(mul(a, mul(b, add(in, mul(cos_theta, normal)))), mul(sq, normal));
                V3 adj_org = add(isectP, mul(eps, in));
                float cos_phi = (float)sqrt(1 - pw2((double)(P.refr_glass / P.refr_air)) *
                                                    (1 - pw2(dot(in, normal))));
                float rp = (P.refr_glass * cos_theta - P.refr_air * cos_phi) /
                           (P.refr_glass * cos_theta + P.refr_air * cos_phi);
                float rs = (P.refr_air * cos_theta - P.refr_glass * cos_phi) /
                           (P.refr_air * cos_theta + P.refr_glass * cos_phi);
                k_refl = (float)(0.5 * (pw2((double)rp) + pw2((double)rs)));
                k_refr = 1 - k_refl;
                Entry ch; ch.a = outr; ch.b = adj_org; ch.k = k_refr * k; ch.depth = depth - 1;
                ch.key = child_key(node, 0); ch._pad = DT_CPATH(1);
                stack[sp++] = ch;
                DT_NPEND(1);
              }
            }
            if (nref > 0 && glossy && !P.nogloss) {
              DT_WK(DT_WK_GLOSSY_RECT, true);
              V3 A, B, C, D, wv, lv;
              glossy_rect(refl_ray, isectP, 2.0f, A, B, C, D, wv, lv);
              V3 wa = wv, la = lv;
              if (dot(wv, normal) <= 0) wa = neg(wa);
              if (dot(lv, normal) <= 0) la = neg(la);
              // squeeze (cpp:680-695); bounded so a degenerate normal cannot hang the GPU
              for (int it = 0; it < 100000 && dot(sub(A, isectP), normal) <= 0; ++it) A = add(add(A, mul(0.1, wa)), mul(0.1, la));
              for (int it = 0; it < 100000 && dot(sub(B, isectP), normal) <= 0; ++it) B = add(add(B, mul(0.1, wa)), mul(0.1, la));
              for (int it = 0; it < 100000 && dot(sub(C, isectP), normal) <= 0; ++it) C = add(add(C, mul(0.1, wa)), mul(0.1, la));
              for (int it = 0; it < 100000 && dot(sub(D, isectP), normal) <= 0; ++it) D = add(add(D, mul(0.1, wa)), mul(0.1, la));
              const float kg = k_refl * k / P.brdf_samples;
              // attempts 2a and 2a+1 of glossy sample i share one draw (sub-index (i << 8) | a):
              // words 0-1 / 2-3 are their (x, y); gw keeps the odd attempt's words
              uint32_t gw[2] = {0u, 0u};
              for (int i = 0; i < nref; i++) {
                DT_WK(DT_WK_GLOSSY, true);
                int attempt = 0;
                uint32_t o[4];
                c.rng.draw_words(node, P_GLOSSY, (uint32_t)i << 8, o);
                gw[0] = o[2]; gw[1] = o[3];
                V3 sample_refl = sub(rect_sample_f(A, B, D, f01(o[0]), f01(o[1])), isectP);
                int sample_limit = 10;
                bool exhausted = false;
                while (dot(sample_refl, normal) <= 0) {
                  if (sample_limit < 0) { exhausted = true; break; }
                  DT_WK(DT_WK_GLOSSY, true);
                  DT_WK(DT_WK_GLOSSY_RECT, true);
                  float multiplier = (float)ldexp(1.0, 11 - sample_limit);   // pow(2, 11 - limit), exact
                  glossy_rect(refl_ray, isectP, multiplier, A, B, C, D, wv, lv);
                  attempt++;
                  float gx, gy;
                  if (attempt & 1) {
                    gx = f01(gw[0]); gy = f01(gw[1]);
                  } else {
                    c.rng.draw_words(node, P_GLOSSY, ((uint32_t)i << 8) | ((uint32_t)attempt >> 1), o);
                    gx = f01(o[0]); gy = f01(o[1]);
                    gw[0] = o[2]; gw[1] = o[3];
                  }
                  sample_refl = sub(rect_sample_f(A, B, D, gx, gy), isectP);
                  sample_limit--;
                }
                if (exhausted) atomicAdd(cnt.wc + WC_GLOSSY, 1u);
                Entry ch; ch.a = sample_refl; ch.b = add(isectP, mul(eps, sample_refl));
                ch.k = kg; ch.depth = exhausted ? 0 : depth - 1; ch.key = child_key(node, 2 + i);
                ch._pad = DT_CPATH(2 + i);
                stack[base + nref - 1 - i] = ch;
                DT_NPEND(!exhausted);
              }
            } else if (nref > 0) {
              DT_WK(DT_WK_MIRROR, true);
              Entry ch; ch.a = refl_ray; ch.b = add(isectP, mul(eps, refl_ray)); ch.k = k_refl * k;
              ch.depth = depth - 1; ch.key = child_key(node, 1); ch._pad = DT_CPATH(2);
              stack[base] = ch;
              DT_NPEND(1);
            }
          }
        }
      }

      // emissive (cpp:775-789)
      if (M.flags & DT_F_LIGHT) {
        DT_WK(DT_WK_EMIT, true);
        if (DT_HAS(DT_FEAT_SPHL) && M.emit == DT_EMIT_SPHERE) {
          float hitdot = (float)dot(in, normalized(sub(v3a(M.center), isectP)));
          double f = (0.1 * pw1((double)hitdot) + 0.05 * pw5((double)hitdot)) + 0.9;
          own = mul(f, mul(k, shape_color));
        }
        if (DT_HAS(DT_FEAT_RECTL) && M.emit == DT_EMIT_RECT) {
          V3 A = G3(g, RC_A), B = G3(g, RC_B), C = G3(g, RC_C), D = G3(g, RC_D);
          float dist = (float)((((norm(sub(isectP, A)) + norm(sub(isectP, B))) + norm(sub(isectP, C))) +
                                norm(sub(isectP, D))) /
                               (8 * norm(sub(v3a(M.center), A))));
          double f = (0.1 * pw1((double)dist) + 0.05 * pw5((double)dist)) + 0.9;
          own = mul(f, mul(k, shape_color));
        }
      } else {
        shade = true;
      }
    }

    DT_T(t3);
    DT_ACC(2, t2, t3);
    // ---- direct lighting (cpp:800-959) ------------------------------------------------
    // One packet shadow walk per light; the shading inputs (normal, eye, colour) are parked in
    // LDS across the walks so they run with a small live register set (the loop below).
    if (__ballot(shade)) {
      // getUV/texel depend only on the hit point: once per node (the reference repeats them
      // per unoccluded light with the same result). UV type 0 makes the node's own light 0
      // whichever lights are visible (Q8 abort, or no hits), so such lanes walk nothing.
      int uvt = 1;
      double tu = 0, tv = 0;
      const bool textured = shade && (S.mat[sid].flags & DT_F_TEXTURE);
      if (textured) uvt = shape_uv(hd.type, hd.flags, cas(S.geom) + hd.off, isectP, shift, tu, tv);
      const bool walk = shade && uvt != 0;
      const int ln_ = threadIdx.x & (DT_WAVE - 1);
      // One pass over the lights: each light's BRDF right after its shadow walk, for the lanes the
      // light reaches, in light order as the reference's loop (cpp:800-959). The walk's sray and sn
      // serve the BRDF, so the sample is neither kept for nor regenerated in a second pass. Parked
      // in LDS across the walks: the normal, the eye direction (normalised once per node) and the
      // base colour; the colour sum of the lit lights in tcol. (Round 3 walked every light first and
      // then evaluated the BRDFs in a second pass, regenerating each sample: C3 -4.8%, C2 -4.6%,
      // 62 more spilled VGPRs in the 5-wave kernel, profiles/r04e_ab_onepass_all.log.)
      if (walk) {
        V3 base = shape_color;
        if (textured) {
          const DMat& M = S.mat[sid];
          if (uvt == 2) {
            base = v3a(M.bordercolor);
          } else if (uvt == 1 && M.tex >= 0) {
            double dims0 = M.tex_w;
            int x_tex = (int)((float)(M.tex_w - 1) * (float)tu);
            int y_tex = (int)((float)(M.tex_h - 1) * (float)tv);
            int uv_ind = (int)(y_tex * dims0 + x_tex);
            if (uv_ind < 0) uv_ind = 0;
            if (uv_ind >= M.tex_w * M.tex_h) uv_ind = M.tex_w * M.tex_h - 1;
            const uint8_t* px = S.tex + M.tex_off + (int64_t)uv_ind * M.tex_ch;
            base = v3(px[0] / 255.0, px[1] / 255.0, px[2] / 255.0);
          }
        }
        const V3 e_dir = normalized(sub(eye, isectP));
        nrec[0][ln_] = normal.x; nrec[1][ln_] = normal.y; nrec[2][ln_] = normal.z;
        nrec[3][ln_] = e_dir.x; nrec[4][ln_] = e_dir.y; nrec[5][ln_] = e_dir.z;
        nrec[6][ln_] = base.x; nrec[7][ln_] = base.y; nrec[8][ln_] = base.z;
        tcol[0][ln_] = 0; tcol[1][ln_] = 0; tcol[2][ln_] = 0;
      }
      const bool uv_oob = textured && (tu < 0 || tv < 0 || tu > 1 || tv > 1);
      asm volatile("" ::: "memory");
      int hits = 0;
      DT_WORK(bool tex_counted = false);
      uint32_t pair[3] = {0u, 0u, 0xffffffffu};   // area-light draw shared with the next light
      for (int li = 0; li < P.n_lights; ++li) {
        const DT_CAS DLight& L = cas(S.lights)[li];
        DT_CNT(9);
        V3 sray = v3(1, 0, 0);
        float t_max = 0;
        V3 sn = v3(1, 0, 0);
        // A point light (no draw) whose umbra holds the shading point's own grid cell: the shadow
        // ray starts at o = p + 1e-3 sn, inside the cell's box widened by m1 >= 0.05 cells, over
        // which the umbra is proven (host_shadowgrid.cpp), so it is occluded before the sample,
        // the ray setup and the walk. Unshifted lanes only (pass-0 geometry). C3's window light.
        bool umb0 = false;
        if (DT_UMBRA_EARLY && L.type == DT_LIGHT_POINT && li < P.sg_n && P.sg_base0[li] >= 0 && walk &&
            shift == 0.0f) {
          float x, y, z;
          sg_coords(P, isectP, x, y, z);
          const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
          if (fx >= 0.0f && fy >= 0.0f && fz >= 0.0f && fx < (float)P.sg_dim[0] && fy < (float)P.sg_dim[1] &&
              fz < (float)P.sg_dim[2]) {
            const int cl = ((int)fz * P.sg_dim[1] + (int)fy) * P.sg_dim[0] + (int)fx;
            umb0 = (((const uint2*)S.sg_cells)[(size_t)P.sg_base0[li] + cl].x & DT_SG_UMBRA) != 0u;
          }
        }
        const bool ws = walk && !umb0;
        if (ws) {
          DT_WK(DT_WK_LIGHT, true);
          sray = light_sample(c, L, li, isectP, node, cnt.wc + WC_SPHL, pair);
          t_max = (float)norm(sray);
          sn = normalized(sray);
        }
        DT_WCNT(WC_SHADOW, walk);
        DT_T(t4);
#ifdef DT_STAMPS
        cnt.cur_li = li;
#endif
        bool occl = umb0;
        if (!DT_UMBRA_EARLY || __ballot(ws))
          occl = occluded(S, P, ws, sray, add(isectP, mul(1e-3, sray)), sn, add(isectP, mul(1e-3, sn)), t_max,
                          L.shape_index, li, shift, cnt) ||
                 umb0;
        DT_T(t5);
        DT_ACC(3, t4, t5);
#ifdef DT_STAMPS
        {   // per light: (waves, active lanes, occluded lanes), (cycles)
          const unsigned long long bw = __ballot(walk), bo = __ballot(walk && occl);
          if ((threadIdx.x & 63) == 0 && li < 8) {
            unsigned long long* h = S.stats + ST_N + 1 + DT_PH_N + 3 * (li * 256 + 255);
            atomicAdd(h, 1ull);
            atomicAdd(h + 1, (unsigned long long)__popcll(bw));
            atomicAdd(h + 2, (unsigned long long)__popcll(bo));
            atomicAdd(h - 3, (unsigned long long)(t5 - t4));
          }
        }
#endif
        asm volatile("" ::: "memory");
        if (walk && !occl) {
          const DMat& M = S.mat[sid];
#ifdef DT_WORK_COUNTERS
          for (int m = 0; m < 4; ++m) DT_WK(DT_WK_BRDF + m, M.model == m);
#endif
          const V3 normal = v3(nrec[0][ln_], nrec[1][ln_], nrec[2][ln_]);
          const V3 e_dir = v3(nrec[3][ln_], nrec[4][ln_], nrec[5][ln_]);
          const V3 shape_color = v3(nrec[6][ln_], nrec[7][ln_], nrec[8][ln_]);
          if (textured) {
            DT_WK(DT_WK_TEX, !tex_counted);   // getUV + texel once per node, as the two-pass count
            DT_WORK(tex_counted = true);
            if (uv_oob) atomicAdd(cnt.wc + WC_UV, 1u);   // the reference terminates here (Q9)
            DT_WCNT(WC_TEX, uvt == 1 && M.tex >= 0);
          }
          const V3 ray_col = brdf(P, M, cas(S.lights)[li], normal, e_dir, sray, sn, shape_color);
          if (!is_approx_zero(ray_col)) {
            hits++;
            tcol[0][ln_] = tcol[0][ln_] + k * ray_col.x;
            tcol[1][ln_] = tcol[1][ln_] + k * ray_col.y;
            tcol[2][ln_] = tcol[2][ln_] + k * ray_col.z;
          }
        }
      }
      if (hits > 0) own = divs(v3(tcol[0][ln_], tcol[1][ln_], tcol[2][ln_]), hits);
    }
    DT_T(t6);
    DT_ACC(4, t3, t6);
    if (fin_slot >= 0) {
      if (sp == fin_slot + 1) {
        // no children were pushed: the FINISH entry would be the very next pop, so the own light
        // goes into the accumulator now, in the same order, without a stack round trip
        sp = fin_slot;
#if DT_DONATE
        emit(own);
#else
        const int l = threadIdx.x & (DT_WAVE - 1);
        ocol[0][l] = ocol[0][l] + own.x;
        ocol[1][l] = ocol[1][l] + own.y;
        ocol[2][l] = ocol[2][l] + own.z;
#endif
      } else {   // a FINISH entry: colour and depth only
        stack[fin_slot].a = own;
        stack[fin_slot].depth = -1;
      }
    }
  }
#if DT_DONATE
  out.in_motion = mo_o;
#endif
}


// =====================================================================================
// render kernel: persistent waves over pixel groups
// =====================================================================================
__device__ __forceinline__ void pixel_of(const DParams& P, int64_t q, int& x, int& y, int64_t& slab_off,
                                         bool& valid)
{
  const int64_t tile_px = (int64_t)P.tw * P.th;
  const int64_t slot = q / tile_px;
  const int local = (int)(q - slot * tile_px);
  int py = local / P.tw, px = local - py * P.tw;
  int64_t t = tile_of(slot, P.rank, P.world);
  int ty = (int)(t / P.tiles_x), tx = (int)(t - (int64_t)ty * P.tiles_x);
  x = P.x0 + tx * P.tw + px;
  y = P.y0 + ty * P.th + py;
  valid = slot < P.n_owned_tiles && t < P.n_tiles && x < P.x1 && y < P.y1;
  slab_off = q * 3;
}

__device__ __forceinline__ void store_pixel(const DParams& P, float* out, int x, int y, int64_t slab_off, V3 color)
{
  int64_t off = P.layout == DT_OUT_SLAB ? slab_off : 3 * ((int64_t)(P.yRes - 1 - y) * P.xRes + x);
  out[off + 0] = clampf01((float)color.x) * 255.0f;
  out[off + 1] = clampf01((float)color.y) * 255.0f;
  out[off + 2] = clampf01((float)color.z) * 255.0f;
}

// getPerspEyeRay + DoF jitter (render_final_project.cpp:195-210, 1044-1072; helpers.h:320-324):
// the sample's eye point and the unnormalised ray through the pixel's focal point
__device__ __forceinline__ void camera_ray(const Ctx& c, const DParams& P, int px_x, int px_y, V3& eye_sample,
                                           V3& ray0)
{
  const V3 eye = v3a(P.eye), X = v3a(P.X), Y = v3a(P.Y), Z = v3a(P.Z);
  eye_sample = eye;
  if (P.aperture > 0) {
    double u0, u1;
    c.rng.draw(0, P_DOF, 0, u0, u1);
    float r = (float)(P.aperture / 2 * u0);
    float theta = (float)(2 * M_PI * u1);
    double st, ct;
    cr_sincos_d(theta, st, ct);
    eye_sample = add(add(eye, mul(r * (float)ct, X)), mul(r * (float)st, Y));
  }
  float a = P.l + (P.r - P.l) * (float)px_x / (float)P.xRes;
  float b = P.b + (P.t - P.b) * (float)px_y / (float)P.yRes;
  V3 rayDir = sub(add(mul(a, X), mul(b, Y)), mul(P.near_plane, Z));
  V3 focalPoint = add(eye, mul(P.focal_length, rayDir));
  ray0 = sub(focalPoint, eye_sample);
}

struct DLaunch {
  DScene S;
  DParams P;
};

#ifndef DT_TRACE_MIN_WAVES
#define DT_TRACE_MIN_WAVES 1
#endif
#ifndef DT_REPRO
#define DT_REPRO 0
#endif
#if DT_REPRO
// DT_REPRO=1 (tools/call_repro: never part of libdt.so): the sky of dt_sky_miss_kernel (cpp:1074-1092,
// cloudColor of mcam * focalPoint per pixel) through cloud_color_lane inlined and through the same
// function behind a real call, on the same pixels, for the called-function defect
__device__ __noinline__ V3 cloud_color_lane_call(const DParams& P, const float* __restrict__ zs, V3 ray)
{
  return cloud_color_lane(P, zs, ray);
}
template <bool CALL>
__device__ __forceinline__ void repro_sky(const DParams* __restrict__ Pp, const float* __restrict__ zs, int x0, int y0,
                                          int w, int n, double* __restrict__ out)
{
  const DParams& P = *Pp;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) {
    const int x = x0 + q % w, y = y0 + q / w;
    const V3 eye = v3a(P.eye), X = v3a(P.X), Y = v3a(P.Y), Z = v3a(P.Z);
    float aa = P.l + (P.r - P.l) * (float)x / (float)P.xRes;
    float bb = P.b + (P.t - P.b) * (float)y / (float)P.yRes;
    V3 rd = sub(add(mul(aa, X), mul(bb, Y)), mul(P.near_plane, Z));
    V3 fp = add(eye, mul(P.focal_length, rd));
    V3 pt;
    pt.x = ((P.sky_m[0][0] * fp.x + P.sky_m[0][1] * fp.y) + P.sky_m[0][2] * fp.z) + P.sky_m[0][3] * 1.0;
    pt.y = ((P.sky_m[1][0] * fp.x + P.sky_m[1][1] * fp.y) + P.sky_m[1][2] * fp.z) + P.sky_m[1][3] * 1.0;
    pt.z = ((P.sky_m[2][0] * fp.x + P.sky_m[2][1] * fp.y) + P.sky_m[2][2] * fp.z) + P.sky_m[2][3] * 1.0;
    const V3 c = CALL ? cloud_color_lane_call(P, zs, pt) : cloud_color_lane(P, zs, pt);
    out[3 * q] = c.x;
    out[3 * q + 1] = c.y;
    out[3 * q + 2] = c.z;
  }
}
extern "C" __global__ void __launch_bounds__(256) dt_repro_inline(const DParams* Pp, const float* zs, int x0, int y0,
                                                                  int w, int n, double* out)
{
  repro_sky<false>(Pp, zs, x0, y0, w, n, out);
}
extern "C" __global__ void __launch_bounds__(256) dt_repro_call(const DParams* Pp, const float* zs, int x0, int y0,
                                                                int w, int n, double* out)
{
  repro_sky<true>(Pp, zs, x0, y0, w, n, out);
}
extern "C" hipError_t dt_repro_launch(int call, const void* Pp, const float* zs, int x0, int y0, int w, int n,
                                      double* out)
{
  if (call)
    hipLaunchKernelGGL(dt_repro_call, dim3((n + 255) / 256), dim3(256), 0, 0, (const DParams*)Pp, zs, x0, y0, w, n, out);
  else
    hipLaunchKernelGGL(dt_repro_inline, dim3((n + 255) / 256), dim3(256), 0, 0, (const DParams*)Pp, zs, x0, y0, w, n, out);
  return hipGetLastError();
}
#else   // !DT_REPRO
#if DT_ISECT
// Intersection micro-benchmark (2^24 primary rays of the C3 camera): rayColor's first
// step for the camera's primary rays (getDOFSamples + getPerspEyeRay, cpp:195-210 / 1044-1072; the
// BVH gather and closest hit, cpp:491-538), taken exactly as the trace kernel takes it for a root
// ray -- the pixel block's primary list when the wave's rays share a block, else the fast tree --
// one ray per lane. Ray r (pixel-major, DT_ISECT_RPP rays per pixel): q = r / RPP, pixel q mod W*H
// (raster order), sample r mod RPP + RPP * (q div W*H). Out: the hit shape (-1: none) and its t
// (FLT_MAX: none), as oracle/oracle.c or_primary_hit.
#define DT_ISECT_RPP 8
extern "C" __global__ void __launch_bounds__(64)
dt_isect_kernel(const DLaunch* __restrict__ Lp, int64_t first, int64_t n, int32_t* __restrict__ hit_shape,
                float* __restrict__ hit_t)
{
  const DScene& S = Lp->S;
  const DParams& P = Lp->P;
  const int lane = threadIdx.x;
  __shared__ unsigned int wc_lds[WC_N];
  if (lane < WC_N) wc_lds[lane] = 0;
  __syncthreads();
  Counters cnt;
  cnt.wc = wc_lds;
  cnt.box = 0; cnt.prim = 0; cnt.wnodes = 0;
  Ctx c;
  c.S = &S;
  c.P = &P;
  c.rng.k0 = P.seed;
  c.rng.k1 = (uint32_t)P.frame;
  const int64_t npx = (int64_t)P.xRes * P.yRes;
  const bool lists = P.pl_block > 0 && P.n_fnodes > 0 && (P.ftree_mode & 1);
  for (int64_t base = (int64_t)blockIdx.x * DT_WAVE; base < n; base += (int64_t)gridDim.x * DT_WAVE) {
    const int64_t i = base + lane;
    const bool act = i < n;
    const int64_t r = first + i;
    const int64_t q = r / DT_ISECT_RPP;
    const int64_t p = q % npx;
    const int x = (int)(p % P.xRes), y = (int)(p / P.xRes);
    c.rng.pixel = (uint32_t)(y * P.xRes + x);
    c.rng.sample = (uint32_t)(r % DT_ISECT_RPP + DT_ISECT_RPP * (q / npx));
    V3 eye_sample = v3a(P.eye), ray0 = v3(0, 0, 0);
    if (act) camera_ray(c, P, x, y, eye_sample, ray0);
    int pblock = -1;
    if (lists) {
      const int blk = (y / P.pl_block) * P.pl_nbx + x / P.pl_block;
      const int b0 = uni(blk);
      if (!__ballot(act && blk != b0)) pblock = b0;
    }
    HitRec h;
    const bool any = closest_hit(S, P, act, ray0, eye_sample, 0.0f, h, cnt, pblock);
    if (act) {
      const bool hit = any && h.shape >= 0;
      hit_shape[i] = hit ? h.shape : -1;
      hit_t[i] = hit ? h.t_min : FLT_MAX;
    }
  }
  if (lane == 0) atomicAdd(S.stats + ST_WNODES, (unsigned long long)cnt.wnodes);
}
extern "C" hipError_t dt_launch_isect(const void* dev_launch, int64_t first, int64_t n, int32_t* hit_shape, float* hit_t,
                                      int grid, hipStream_t stream)
{
  hipLaunchKernelGGL(dt_isect_kernel, dim3(grid), dim3(64), 0, stream, (const DLaunch*)dev_launch, first, n, hit_shape,
                     hit_t);
  return hipGetLastError();
}
extern "C" const void* dt_isect_kernel_ptr(void) { return (const void*)dt_isect_kernel; }
#else
// The launch record: a device copy per counter parity (dt_api.cpp), uploaded only when it changed
extern "C" __global__ void __launch_bounds__(64, DT_TRACE_MIN_WAVES)
DT_TRACE_KERNEL(const DLaunch* __restrict__ Lp, float* __restrict__ out)
{
  const DScene& S = Lp->S;
  const DParams& P = Lp->P;
  if (blockIdx.x == 0) {
    for (int i = (int)threadIdx.x; i < S.n_clear0; i += DT_WAVE) S.clear0[i] = 0ull;
    for (int i = (int)threadIdx.x; i < S.n_clear1; i += DT_WAVE) S.clear1[i] = 0ull;
  }
  // LDS (one wave per block). nrec holds a lane's shading record across the shadow walks
  // (inside run_pass only); red (per-chunk sample colours) and dens (cloud march chunk) are
  // used after the passes, so they share its space. ocol: the DFS colour accumulator,
  // psum: the per-pixel sums, parked here instead of in registers across the DFS.
  __shared__ double nrec[9][DT_WAVE];
  double* const red = &nrec[0][0];                        // DT_WAVE * 3 doubles
  float* const dens = (float*)(&nrec[0][0] + DT_WAVE * 3);  // DT_CLOUD_CHUNK floats
  __shared__ double ocol[3][DT_WAVE];
  // DT_PSUM_LDS=2: slots for up to 8 pixels per wave only (spp >= 8; 192 B instead of 1536 B)
  __shared__ double psum[3][DT_PSUM_LDS == 2 ? 8 : DT_WAVE];
  __shared__ double chan[4];
  __shared__ double tcol[3][DT_WAVE];   // the lit lights' colour sum of the node being shaded
  __shared__ unsigned long long item_s;
  Entry stack[DT_STACK_MAX];
  const int lane = threadIdx.x;
#ifdef DT_WORK_COUNTERS
  __shared__ unsigned int wk_lds[DT_WK_N];
  if (lane < DT_WK_N) wk_lds[lane] = 0;
  __syncthreads();
#endif
  Ctx c;
  c.S = &S;
  c.P = &P;
  c.rng.k0 = P.seed;
  c.rng.k1 = (uint32_t)P.frame;
  unsigned long long sky_px = 0;
  Counters cnt;
  __shared__ unsigned int wc_lds[WC_N];
#if DT_AGAIN_QUEUE
  __shared__ unsigned int wc_snap[WC_N];
#endif
  if (lane < WC_N) wc_lds[lane] = 0;
  __syncthreads();
  cnt.wc = wc_lds;
  cnt.box = 0; cnt.prim = 0; cnt.wnodes = 0;
#ifdef DT_WORK_COUNTERS
  cnt.wk = wk_lds;
#endif
#ifdef DT_STAMPS
  for (int k = 0; k < DT_PH_N; ++k) cnt.ph[k] = 0;
  cnt.cur_li = 0;
  cnt.cur_path = 0;
#endif

#if DT_DONATE
  __shared__ unsigned dn_next;
  __shared__ unsigned dn_done[DN_NBLK / 32];
  __shared__ int dn_pair[DT_WAVE];
  DnCtx dn;
  dn.pool = (DnRec*)S.dn_pool + (size_t)blockIdx.x * DT_DN_POOL_REC;
  dn.next = &dn_next;
  dn.done = dn_done;
  dn.pair = dn_pair;
#endif

  // items are dequeued P.item_batch at a time (one same-address atomic per batch). The first batch
  // of every wave is its own by block index: 5120 waves starting at once would otherwise queue
  // behind one another on the one atomic word; the shared counter hands out the items after them.
  const int batch = P.item_batch > 1 ? P.item_batch : 1;
  // P.sky_again == 2: the queue runs over the items a launch without the sky listed
  const int64_t n_queue = DT_AGAIN_QUEUE && P.sky_again == 2 ? (int64_t)*S.again_n
                                                             : P.n_items * (DT_CHUNK_ITEMS && P.chunk_items ? P.chunks : 1);
  // P.queue_segs > 1: the queue in that many contiguous segments with a counter each; wave b starts
  // in segment b % segs (workgroups go round-robin to the XCDs) and takes its first batch there by
  // block index, then from the segment's counter; a drained segment sends the wave to the next one,
  // and the wave ends once it has found every segment drained in turn (counters only grow)
  const int segs = (DT_AGAIN_QUEUE && P.sky_again == 2) || P.queue_segs < 2 ? 1 : P.queue_segs;
  const int64_t seg_len = (n_queue + segs - 1) / segs;
  int seg = (int)(blockIdx.x % (unsigned)segs), seg_fails = 0;
  int64_t seg_lo = seg * seg_len, seg_hi = seg_lo + seg_len < n_queue ? seg_lo + seg_len : n_queue;
  int64_t qpos = seg_lo + (int64_t)(blockIdx.x / (unsigned)segs) * batch;
  int64_t batch_end = qpos + batch < seg_hi ? qpos + batch : seg_hi;
  while (true) {
    if (qpos >= batch_end) {
      bool drained = false;
      while (true) {
        unsigned long long* const ctr = segs == 1 ? S.queue : S.queue + DT_QSEG_OFF + seg * DT_QSEG_STRIDE;
        if (lane == 0) item_s = atomicAdd(ctr, (unsigned long long)batch);
        __syncthreads();
        // the segment's first batches belong to its home waves (blocks seg, seg + segs, ...)
        const int64_t home = ((int64_t)gridDim.x - seg + segs - 1) / segs;
        qpos = seg_lo + (int64_t)item_s + home * batch;
        __syncthreads();
        if (qpos < seg_hi) {
          batch_end = qpos + batch < seg_hi ? qpos + batch : seg_hi;
          seg_fails = 0;
          break;
        }
        if (++seg_fails >= segs) {
          drained = true;
          break;
        }
        seg = seg + 1 == segs ? 0 : seg + 1;
        seg_lo = seg * seg_len;
        seg_hi = seg_lo + seg_len < n_queue ? seg_lo + seg_len : n_queue;
      }
      if (drained) break;
    }
    if (qpos >= n_queue) break;
    const int64_t code = DT_AGAIN_QUEUE && P.sky_again == 2 ? (int64_t)S.again_list[qpos] : qpos;
    int64_t item = code;
    float* const outc = out;
    // P.chunk_items: the item is one 64-sample chunk of a pixel item (a listed sky item likewise)
    int chunk_lo = 0, chunk_hi = P.chunks;
    if (DT_CHUNK_ITEMS && P.chunk_items) {
      const uint32_t nck = (uint32_t)P.chunks, ci = (uint32_t)item;
      uint32_t pi, ck;
      if (P.chunk_items == 2) {   // chunk-major (host: n_items * chunks < 2^32)
        ck = ci / (uint32_t)P.n_items;
        pi = ci - ck * (uint32_t)P.n_items;
      } else {
        pi = ci / nck;
        ck = ci - pi * nck;
      }
      item = pi;
      chunk_lo = (int)ck;
      chunk_hi = chunk_lo + 1;
    }
    bool px_done = true;   // false for chunk items: dt_chunk_sum_kernel stores their pixels
    bool sky_again = false;
#if DT_AGAIN_QUEUE
    // the item's counters are taken back: the launch that listed it counted it already
    if (lane < WC_N) wc_snap[lane] = wc_lds[lane];
    const uint32_t wnodes0 = cnt.wnodes;
#endif

    const int group = P.ppw;
    const int spp = P.spp;
    // lanes: pixel slot j = lane / min(spp,64), sample = chunk*64 + lane % ...
    const int per = spp < DT_WAVE ? spp : DT_WAVE;
    const int j = lane / per;
    if (DT_PSUM_LDS == 1 || lane < 8) {   // pixel j's sums, in sample order
      psum[0][lane] = 0; psum[1][lane] = 0; psum[2][lane] = 0;
    }
    int px_x = 0, px_y = 0;
    int64_t px_off = 0;
    bool px_valid = false;
    pixel_of(P, item * group + (j < group ? j : 0), px_x, px_y, px_off, px_valid);
#ifdef DT_ITEM_TIMES
    const unsigned long long item_t0 = DT_ITEM_TIMES == 2 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
#endif

    for (int chunk = chunk_lo; chunk < chunk_hi; ++chunk) {
      const int sample = chunk * DT_WAVE + (lane - j * per);
      const bool valid = j < group && px_valid && sample < spp && (lane - j * per) < per;
      c.rng.pixel = (uint32_t)(px_y * P.xRes + px_x);
      c.rng.sample = (uint32_t)sample;

      DT_T(k0);
      // pass 0: the sample's rayColor tree; passes 1..blur_samples: motion-blur re-traces for
      // samples whose last hit was a moving shape (cpp:1095-1210). One call site so the DFS is
      // inlined once.
      V3 tmp_color = v3(0, 0, 0);
      bool hit0 = false, need_blur = false;
      for (int pass = 0; pass <= P.blur_samples; ++pass) {
        bool act = valid;
        float val = 0.0f;
        if (pass > 0) {
          if (!__ballot(need_blur)) break;
          act = need_blur;
          if (act) {
            double u0, u1;
            c.rng.draw(0, P_BLUR, (uint32_t)(pass - 1), u0, u1);
            float frame_sample = (float)((float)P.frame + u0 * P.frame_range);
            if (P.frame >= P.frame_prism) {   // below frame_prism the reference's val is unset (Q19): 0
              if (P.frame >= P.frame_blur)
                val = (float)(P.move_per_frame * (frame_sample - P.frame) +
                              P.accel_t * pw3((double)(frame_sample - P.frame)));
              else
                val = P.move_per_frame * (frame_sample - P.frame);
            }
          }
        }
        // camera ray (cpp:1044-1072), regenerated per pass from the counter RNG (same values)
        // so that it is not held in registers across the DFS
        V3 eye_sample = v3a(P.eye), ray0 = v3(0, 0, 0);
        DT_WK(DT_WK_CAMERA, act);
        if (act) camera_ray(c, P, px_x, px_y, eye_sample, ray0);
        PassOut po;
        ocol[0][lane] = 0; ocol[1][lane] = 0; ocol[2][lane] = 0;
        po.hit = pass > 0;
        po.in_motion = false;
        run_pass(c, act, ray0, eye_sample, root_key(pass), val, po, stack, cnt, nrec, ocol, tcol
#if DT_DONATE
                 , dn
#endif
                 );
        po.color = v3(ocol[0][lane], ocol[1][lane], ocol[2][lane]);
        if (pass == 0) {
          tmp_color = po.color;
          hit0 = po.hit;
          need_blur = valid && po.hit && po.in_motion;
        } else if (need_blur) {
          tmp_color = add(tmp_color, po.color);
        }
      }
      if (need_blur) tmp_color = divs(tmp_color, P.blur_samples + 1);
      DT_T(k1);
      DT_ACC(5, k0, k1);
      const bool miss = valid && !hit0;
      // sky for missing samples: computed once per pixel by the whole wave, or (1 spp,
      // P.sky_defer) flagged for dt_sky_miss_kernel
      if (P.sky_defer) {
        if (miss) S.sky_miss[item * group + j] = 1;
      } else if (DT_SKY_AGAIN && P.perlin_cloud) {
        if (__ballot(miss)) sky_again = true;   // rendered again by a build with the sky
      } else if (P.perlin_cloud) {
        for (int jj = 0; jj < group; ++jj) {
          if (__ballot(miss && j == jj)) {
            int qx, qy;
            int64_t qo;
            bool qv;
            pixel_of(P, item * group + jj, qx, qy, qo, qv);
            const V3 eye = v3a(P.eye), X = v3a(P.X), Y = v3a(P.Y), Z = v3a(P.Z);
            float aa = P.l + (P.r - P.l) * (float)qx / (float)P.xRes;
            float bb = P.b + (P.t - P.b) * (float)qy / (float)P.yRes;
            V3 rd = sub(add(mul(aa, X), mul(bb, Y)), mul(P.near_plane, Z));
            V3 fp = add(eye, mul(P.focal_length, rd));
            V3 pt;
            pt.x = ((P.sky_m[0][0] * fp.x + P.sky_m[0][1] * fp.y) + P.sky_m[0][2] * fp.z) + P.sky_m[0][3] * 1.0;
            pt.y = ((P.sky_m[1][0] * fp.x + P.sky_m[1][1] * fp.y) + P.sky_m[1][2] * fp.z) + P.sky_m[1][3] * 1.0;
            pt.z = ((P.sky_m[2][0] * fp.x + P.sky_m[2][1] * fp.y) + P.sky_m[2][2] * fp.z) + P.sky_m[2][3] * 1.0;
            V3 skyc = cloud_color_coop(P, S.cloud_z, pt, dens, chan);
            if (miss && j == jj) tmp_color = skyc;
            if (lane == 0) sky_px++;
          }
        }
      } else if (miss) {
        tmp_color = v3a(P.default_col);
      }
      DT_T(k2);
      DT_ACC(6, k1, k2);
      if (DT_CHUNK_ITEMS && P.chunk_items) {
        // chunk items: the chunk stores its sample colours in its pixel's slot, in sample order
        // (coalesced: 64 lanes x 24 B); dt_chunk_sum_kernel adds each pixel's colours up after the
        // launch (dt_api.cpp), so no item of this launch stores a pixel
        double* const slot = S.chunk_cols + ((int64_t)item * spp + chunk * DT_WAVE + lane) * 3;
        if (valid) {
          slot[0] = tmp_color.x;
          slot[1] = tmp_color.y;
          slot[2] = tmp_color.z;
        }
        px_done = false;
      } else {
        // ordered per-pixel sum (cpp:1212: color += tmp_color in sample order)
        red[lane * 3 + 0] = tmp_color.x;
        red[lane * 3 + 1] = tmp_color.y;
        red[lane * 3 + 2] = tmp_color.z;
        __syncthreads();
        int ns = spp - chunk * DT_WAVE;
        if (ns > per) ns = per;
        if (group * 3 <= DT_WAVE) {
          // lane 3 jj + ch sums channel ch of pixel jj: the three channels' chains run side by side
          // (the same additions in the same order as one lane adding the three: add() is componentwise)
          if (lane < group * 3) {
            const int jj = lane / 3, ch = lane - 3 * jj, base = jj * per;
            double ps = psum[ch][jj];
            for (int s = 0; s < ns; ++s) ps = ps + red[(base + s) * 3 + ch];
            psum[ch][jj] = ps;
          }
        } else if (lane < group) {   // (up to 64 pixels per wave: 1 or 2 spp)
          const int base = lane * per;
          V3 ps = v3(psum[0][lane], psum[1][lane], psum[2][lane]);
          for (int s = 0; s < ns; ++s) ps = add(ps, v3(red[(base + s) * 3], red[(base + s) * 3 + 1], red[(base + s) * 3 + 2]));
          psum[0][lane] = ps.x; psum[1][lane] = ps.y; psum[2][lane] = ps.z;
        }
        __syncthreads();
      }
    }
    DT_T(k3);
    const bool item_again = sky_again;
    if (lane < group && px_done) {
      int qx, qy;
      int64_t qo;
      bool qv;
      pixel_of(P, item * group + lane, qx, qy, qo, qv);
      if (qv && !item_again && !(P.sky_defer && S.sky_miss[item * group + lane])) {
        V3 color = divs(v3(psum[0][lane], psum[1][lane], psum[2][lane]), spp);
#ifdef DT_ITEM_TIMES   // diagnostic builds (tools/item_times.py): the item's wave cycles / 1e4, raw
        {
          const int64_t off = P.layout == DT_OUT_SLAB ? qo : 3 * ((int64_t)(P.yRes - 1 - qy) * P.xRes + qx);
#if DT_ITEM_TIMES == 2   // tools/tail.py: start and end on the 100 MHz clock, 24-bit pieces (exact in f32)
          const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
          outc[off] = (float)(uint32_t)(item_t0 & 0xFFFFFF);
          outc[off + 1] = (float)(uint32_t)(t1 & 0xFFFFFF);
          outc[off + 2] = (float)(uint32_t)((t1 >> 24) & 0xFFFFFF);
#else
          const float cyc = (float)(__builtin_amdgcn_s_memtime() - item_t0) * 1e-4f;
          outc[off] = cyc; outc[off + 1] = cyc; outc[off + 2] = cyc;
#endif
        }
#else
        store_pixel(P, outc, qx, qy, qo, color);
#endif
        if (isnan(color.x) || isnan(color.y) || isnan(color.z)) atomicAdd(S.stats + ST_NAN, 1ull);
      }
    }
#if DT_AGAIN_QUEUE
    // a listed item is counted by the launch that listed it: the *_sky build takes its counts back
    // (all but its sky and NaN pixels, which only this launch stores)
    if (P.sky_again == 2) {
      __syncthreads();
      if (lane < WC_N) wc_lds[lane] = wc_snap[lane];
      cnt.wnodes = wnodes0;
      __syncthreads();
    }
#endif
#if DT_SKY_AGAIN
    if (item_again && lane == 0) S.again_list[atomicAdd(S.again_n, 1u)] = (uint32_t)code;
#endif
#if DT_ITEM_TIMES == 2
    if (S.item_cost && lane == 0) S.item_cost[code] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - item_t0);
#endif
    if (P.prio_steps > 0) __builtin_amdgcn_s_setprio(0);
    ++qpos;
  }
  {
    __syncthreads();
#ifdef DT_WORK_COUNTERS
    __syncthreads();
    if (lane < DT_WK_N && wk_lds[lane]) atomicAdd(S.stats + ST_N + 1 + lane, (unsigned long long)wk_lds[lane]);
    if (lane == 0) {
      unsigned long long pr = 0;
      for (int k = DT_WK_HIT_SHAPE; k < DT_WK_HIT; ++k) pr += wk_lds[k];
      atomicAdd(S.stats + ST_BOX, (unsigned long long)wk_lds[DT_WK_BOX]);
      atomicAdd(S.stats + ST_PRIM, pr);
    }
#endif
#ifdef DT_STAMPS
    if (lane == 0)
      for (int k = 0; k < DT_PH_N; ++k) atomicAdd(S.stats + ST_N + 1 + k, cnt.ph[k]);
#endif
    // the wave's counters into one of DT_STAT_SLOTS copies of the block (dt_collect_stats adds them
    // up), one counter per lane: 5120 waves adding to the same words serialise on one L2 channel at
    // the launch's end (the sky-item launch, a few hundred waves, keeps slot 0)
    const int slot = DT_AGAIN_QUEUE && P.sky_again == 2 ? 0 : (int)(blockIdx.x % DT_STAT_SLOTS);
    unsigned long long* const stb = slot == 0 ? S.stats : S.queue + DT_STAT_SLOT_OFF + (slot - 1) * DT_STAT_SLOT_STRIDE;
    const int st_of[WC_N] = {ST_RAYS, ST_SHADOW, ST_TEX, ST_STACK, ST_REFL, ST_GLOSSY, ST_UV, ST_PRISM, ST_SPHL};
    const unsigned long long sky_w = __shfl(sky_px, 0);   // (lane 0's, as before: counted there)
    const unsigned int wn_w = __shfl((unsigned int)cnt.wnodes, 0);
    if (lane < WC_N) {
      const unsigned long long v = wc_lds[lane];
      if (v) atomicAdd(stb + st_of[lane], v);
    } else if (lane == WC_N) {
      if (wn_w) atomicAdd(stb + ST_WNODES, (unsigned long long)wn_w);
    } else if (lane == WC_N + 1) {
      if (sky_w) atomicAdd(stb + ST_SKY, sky_w);
    }

  }
}

#endif   // !DT_ISECT

#if DT_HELPERS
// The sky of the pixels a 1-spp trace launch flagged as missed (P.sky_defer): renderImage's miss
// branch (cpp:1074-1092: cloudColor of mcam * focalPoint) one pixel per lane, at the occupancy of a
// small kernel instead of inside the trace kernel's register budget. With one sample the pixel is
// that sample's colour (0 + c, then / 1: exact), so the store is the trace kernel's. Clears the flags.
extern "C" __global__ void __launch_bounds__(256)
dt_sky_miss_kernel(const DLaunch* __restrict__ Lp, float* __restrict__ out)
{
  const DParams& P = Lp->P;
  const DScene& S = Lp->S;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool mine = q < P.n_items * P.ppw && S.sky_miss[q];
  if (mine) {
    S.sky_miss[q] = 0;
    int x, y;
    int64_t so;
    bool valid;
    pixel_of(P, q, x, y, so, valid);
    const V3 eye = v3a(P.eye), X = v3a(P.X), Y = v3a(P.Y), Z = v3a(P.Z);
    float aa = P.l + (P.r - P.l) * (float)x / (float)P.xRes;
    float bb = P.b + (P.t - P.b) * (float)y / (float)P.yRes;
    V3 rd = sub(add(mul(aa, X), mul(bb, Y)), mul(P.near_plane, Z));
    V3 fp = add(eye, mul(P.focal_length, rd));
    V3 pt;
    pt.x = ((P.sky_m[0][0] * fp.x + P.sky_m[0][1] * fp.y) + P.sky_m[0][2] * fp.z) + P.sky_m[0][3] * 1.0;
    pt.y = ((P.sky_m[1][0] * fp.x + P.sky_m[1][1] * fp.y) + P.sky_m[1][2] * fp.z) + P.sky_m[1][3] * 1.0;
    pt.z = ((P.sky_m[2][0] * fp.x + P.sky_m[2][1] * fp.y) + P.sky_m[2][2] * fp.z) + P.sky_m[2][3] * 1.0;
    const V3 color = cloud_color_lane(P, S.cloud_z, pt);
    if (valid) {
      store_pixel(P, out, x, y, so, color);
      if (isnan(color.x) || isnan(color.y) || isnan(color.z)) atomicAdd(S.stats + ST_NAN, 1ull);
    }
  }
  const unsigned long long n = __popcll(__ballot(mine));
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(S.stats + ST_SKY, n);
}

// Chunk items (P.chunk_items, spp > 64): every pixel's spp sample colours, stored by its chunk items
// in sample order, added up in that order (cpp:1212: color += tmp_color; the same chain as the
// per-pixel items' sums in LDS), then / spp (cpp:1213) and clamp*255 (store_pixel). One pixel per
// thread, the three channels' chains side by side (add() is componentwise).
extern "C" __global__ void __launch_bounds__(256)
dt_chunk_sum_kernel(const DLaunch* __restrict__ Lp, float* __restrict__ out)
{
  const DParams& P = Lp->P;
  const DScene& S = Lp->S;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool nan = false;
  if (q < P.n_items) {
    int x, y;
    int64_t so;
    bool valid;
    pixel_of(P, q, x, y, so, valid);
    if (valid) {
      const double* __restrict__ c = S.chunk_cols + q * P.spp * 3;
      V3 ps = v3(0, 0, 0);
      for (int s = 0; s < P.spp; ++s) ps = add(ps, v3(c[3 * s], c[3 * s + 1], c[3 * s + 2]));
      const V3 color = divs(ps, P.spp);
      store_pixel(P, out, x, y, so, color);
      nan = isnan(color.x) || isnan(color.y) || isnan(color.z);
    }
  }
  const unsigned long long n = __popcll(__ballot(nan));
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(S.stats + ST_NAN, n);
}

// renderImageCloud (cpp:1224-1279): one pixel per lane
extern "C" __global__ void __launch_bounds__(256)
dt_sky_kernel(const DLaunch* __restrict__ Lp, float* __restrict__ out)
{
  const DParams& P = Lp->P;
  const float* __restrict__ zs = Lp->S.cloud_z;
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = P.n_owned_tiles * P.tw * P.th;
  if (q >= total) return;
  int x, y;
  int64_t so;
  bool valid;
  pixel_of(P, q, x, y, so, valid);
  if (!valid) return;
  V3 eye = v3a(P.eye), X = v3a(P.X), Y = v3a(P.Y), Z = v3a(P.Z);
  float a = P.l + (P.r - P.l) * (float)x / (float)P.xRes;
  float b = P.b + (P.t - P.b) * (float)y / (float)P.yRes;
  V3 rayDir = sub(add(mul(a, X), mul(b, Y)), mul(P.near_plane, Z));
  V3 fp = add(rayDir, eye);
  V3 pt;
  pt.x = ((P.sky_m[0][0] * fp.x + P.sky_m[0][1] * fp.y) + P.sky_m[0][2] * fp.z) + P.sky_m[0][3] * 1.0;
  pt.y = ((P.sky_m[1][0] * fp.x + P.sky_m[1][1] * fp.y) + P.sky_m[1][2] * fp.z) + P.sky_m[1][3] * 1.0;
  pt.z = ((P.sky_m[2][0] * fp.x + P.sky_m[2][1] * fp.y) + P.sky_m[2][2] * fp.z) + P.sky_m[2][3] * 1.0;
  V3 color = cloud_color_lane(P, zs, pt);
  store_pixel(P, out, x, y, so, color);
}

// slab -> image scatter (multi-GPU gather epilogue)
extern "C" __global__ void dt_unpack_kernel(const DLaunch* __restrict__ Lp, int world, int64_t slab_floats,
                                            const float* __restrict__ slabs, float* __restrict__ image)
{
  const DParams& P = Lp->P;
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over rank-major slab pixels
  int64_t per_rank = slab_floats / 3;
  int64_t total = per_rank * world;
  if (q >= total) return;
  int r = (int)(q / per_rank);
  int64_t local = q - (int64_t)r * per_rank;
  int64_t ntiles = (int64_t)P.tiles_x * ((P.y1 - P.y0 + P.th - 1) / P.th);
  int64_t owned = (ntiles + world - 1) / world;
  const int64_t tile_px = (int64_t)P.tw * P.th;
  int64_t slot = local / tile_px;
  int lp = (int)(local - slot * tile_px);
  int py = lp / P.tw, px = lp - py * P.tw;
  int64_t t = tile_of(slot, r, world);
  int ty = (int)(t / P.tiles_x), tx = (int)(t - (int64_t)ty * P.tiles_x);
  int x = P.x0 + tx * P.tw + px, y = P.y0 + ty * P.th + py;
  bool valid = slot < owned && t < ntiles && x < P.x1 && y < P.y1;
  if (!valid) return;
  int64_t off = 3 * ((int64_t)(P.yRes - 1 - y) * P.xRes + x);
  const float* s = slabs + (int64_t)r * slab_floats + local * 3;
  image[off] = s[0];
  image[off + 1] = s[1];
  image[off + 2] = s[2];
}

// the kernels' vector normalisation (dt_math.h normalized) on n vectors: the numerics check of
// its shared-reciprocal division against correctly rounded division (tests/test_gpu_numerics.py)
extern "C" __global__ void dt_normalize_kernel(const double* __restrict__ in, double* __restrict__ out, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3 v = normalized(v3(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
  out[3 * i] = v.x;
  out[3 * i + 1] = v.y;
  out[3 * i + 2] = v.z;
}

// ---- host-side launch wrappers ---------------------------------------------------------
extern "C" hipError_t dt_launch_normalize(const double* in, double* out, int64_t n, hipStream_t stream)
{
  hipLaunchKernelGGL(dt_normalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, in, out, n);
  return hipGetLastError();
}
extern "C" size_t dt_launch_size(void) { return sizeof(DLaunch); }
extern "C" size_t dt_scene_struct_offset(void) { return offsetof(DLaunch, S); }
extern "C" size_t dt_scene_struct_size(void) { return sizeof(DScene); }
extern "C" size_t dt_params_struct_offset(void) { return offsetof(DLaunch, P); }

extern "C" hipError_t dt_launch_sky_miss(const void* dev_launch, float* out, int64_t n_px, hipStream_t stream)
{
  int64_t blocks = (n_px + 255) / 256;
  hipLaunchKernelGGL(dt_sky_miss_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const DLaunch*)dev_launch, out);
  return hipGetLastError();
}
extern "C" hipError_t dt_launch_chunk_sum(const void* dev_launch, float* out, int64_t n_px, hipStream_t stream)
{
  int64_t blocks = (n_px + 255) / 256;
  hipLaunchKernelGGL(dt_chunk_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const DLaunch*)dev_launch, out);
  return hipGetLastError();
}
extern "C" hipError_t dt_launch_sky(const void* dev_launch, float* out, int64_t n_threads, hipStream_t stream)
{
  int64_t blocks = (n_threads + 255) / 256;
  hipLaunchKernelGGL(dt_sky_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const DLaunch*)dev_launch, out);
  return hipGetLastError();
}
extern "C" hipError_t dt_launch_unpack(const void* dev_launch, int world, int64_t slab_floats, const float* slabs,
                                       float* image, hipStream_t stream)
{
  int64_t total = slab_floats / 3 * world;
  int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(dt_unpack_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const DLaunch*)dev_launch,
                     world, slab_floats, slabs, image);
  return hipGetLastError();
}
#endif

#if !DT_ISECT
// every trace-kernel build: <kernel>_launch and <kernel>_ptr (dt_api.cpp's kernel table)
#define DT_CAT2(a, b) a##b
#define DT_CAT(a, b) DT_CAT2(a, b)
#if DT_W5
static_assert(DT_TRACE_MIN_WAVES == 5 && DT_PSUM_LDS == 2, "5-wave build: Makefile W5FLAGS");
#endif
extern "C" hipError_t DT_CAT(DT_TRACE_KERNEL, _launch)(const void* dev_launch, float* out, int grid, hipStream_t stream)
{
  hipLaunchKernelGGL(DT_TRACE_KERNEL, dim3(grid), dim3(64), 0, stream, (const DLaunch*)dev_launch, out);
  return hipGetLastError();
}
extern "C" const void* DT_CAT(DT_TRACE_KERNEL, _ptr)(void) { return (const void*)DT_TRACE_KERNEL; }
// bit 0: the build lists sky items for another launch (DT_SKY_AGAIN); bit 1: it runs chunk items
// (DT_CHUNK_ITEMS); bits 8..23: the scene features
// it handles (DT_FEATURES; dt_api.cpp launches it only for scenes within them)
extern "C" int DT_CAT(DT_TRACE_KERNEL, _traits)(void)
{
  return (DT_SKY_AGAIN ? 1 : 0) | (DT_CHUNK_ITEMS ? 2 : 0) | (int)(((DT_FEATURES) & 0xFFFFu) << 8);
}
#endif
#endif   // !DT_REPRO
