/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, gcc, -ffp-contract=off) of the reference's per-pixel
 * render loop. It is the parity checker for the HIP path and the CPU baseline leg of
 * bench.py; nothing in distraytracer_amd/ links or calls it. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 *
 * Pinning status:
 *   - value noise (noise.h:25-136) is pinned bit-for-bit against the reference's own
 *     noise.h compiled as-is (oracle/ref/noise_harness.cpp -> oracle/_ref/libref_noise.so)
 *     and against the hand-derived anchors of SURVEY §8c.
 *   - everything else (render_final_project.cpp, geometry.cpp, helpers.h) needs Eigen,
 *     which is absent from the image: the reference is unbuildable here, so those
 *     functions are "parity unpinned" beyond analytic anchors (tests/test_oracle_*.py).
 *
 * RNG: the reference draws from random_device-seeded mt19937 (F7) and cannot be
 * reproduced; oracle and device share the counter-based stream documented in
 * DESIGN.md §RNG (Philox4x32-10).
 */
#ifndef DT_ORACLE_H
#define DT_ORACLE_H

#include "../include/dt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* noise.h */
double or_noise3d(int i, int x, int y, int z);
double or_smoothed3d(int i, int x, int y, int z);
double or_interpolated_noise3d(int i, double x, double y, double z);
double or_value_noise3d(double x, double y, double z);

/* render_final_project.cpp:146-192 */
void or_sky_color(const dt_globals* g, const double ray[3], double out[3]);
void or_cloud_color(const dt_globals* g, const double ray[3], const double origin[3],
                    float frame, double out[3]);

/* counter RNG (shared definition with the device path) */
void or_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double or_u01(uint32_t w0, uint32_t w1);
double or_u32_01(uint32_t w);   /* area-light draws: one word per float */

/* renderImageCloud (cpp:1224-1279) on a pixel window / tile set */
int or_render_sky(const dt_globals* g, float frame, const dt_tiles* tiles, float* out,
                  int nthreads);

/* generateBVH (helpers.h:330-472) over all shapes */
int or_bvh(const dt_scene_desc* d, const dt_globals* g, dt_bvh_node* nodes, int cap,
           int* indices, int index_cap, int* n_nodes, int* n_indices);

/* renderImage pixel loop (cpp:965-1222) on a pixel window / tile set */
int or_render(const dt_scene_desc* d, const dt_globals* g, int frame, const dt_tiles* tiles,
              float* out, int nthreads, dt_stats* stats);

/* or_render, also adding the include/dt_work.h event counts of the reference's loop (every box
 * its gathers test, every intersect / intersectShadow call, light, BRDF, texel, sky march) into
 * work[DT_WK_N] (zeroed by the caller) */
int or_render_work(const dt_scene_desc* d, const dt_globals* g, int frame, const dt_tiles* tiles,
                   float* out, int nthreads, dt_stats* stats, uint64_t* work);

/* the intersection micro-benchmark's closest hits (include/dt.h dt_intersect_primary numbering) */
int or_primary_hit(const dt_scene_desc* d, const dt_globals* g, int frame, long long first, long long n,
                   int* shape, float* t, int nthreads);

/* one rayColor call tree for a single pixel-sample (debug / unit tests) */
int or_sample_color(const dt_scene_desc* d, const dt_globals* g, int frame, int x, int y,
                    int sample, double out_color[3], int* out_hit);

#ifdef __cplusplus
}
#endif
#endif
