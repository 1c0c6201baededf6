/*
 * dt_work.h — the algorithmic work unit of the render loop and its weight table.
 *
 * The render loop is VALU-bound (FP64/FP32 vector ALU plus the integer work of the counter RNG and
 * the value-noise hash), not HBM- or MFMA-bound. Its work is measured as a sum over event counts
 * times fixed weights:
 *
 *     work = sum_k count[k] * dt_work_weight[k]        (FP64-equivalent VALU operations)
 *
 * The events are the reference's own steps (the box test of BoundingVolume::intersect, each
 * primitive's intersect / intersectShadow, the shading of a hit, a light sample, a BRDF, a texel,
 * a cloudColor march, ...), so the same counters come out of
 *   - the device (a -DDT_WORK_COUNTERS build of libdt, dt_kernels.hip: the events the kernel
 *     executes, lane by lane, with its culling, grid lists and per-pixel sky cache), and
 *   - the oracle (oracle/oracle.c or_render_work: the events the reference's loop executes, which
 *     gathers every leaf its BVH boxes pass and marches the sky for every missing sample).
 * bench.py reports roofline.achieved = device work per launch / trace-kernel time against the
 * MI355X FP64 vector peak (78.6 TFLOP/s), and the oracle's count for the same frame beside it.
 *
 * Weights: the VALU operations of the device's implementation of each event (dt_kernels.hip; the
 * reference's per-call recomputations of constants, e.g. Rectangle::intersect normalising its
 * normal twice, are precomputed once and not counted), counted by inspection with
 *   +, -, *, compare, min/max, select, f32<->f64 conversion, integer op   1
 *   division, square root (f64, or correctly rounded f32)                 4
 *   transcendental (sin, cos, tan, acos, exp, pow, atan2)                20
 *   one Philox4x32-10 draw (10 rounds of 2 mul_hi, 2 mul, 2 xor, 2 add)  80
 * and the full path of each test (its early exits make the average smaller). A RectPrismWithCylinder
 * test is priced with one hole.
 */
#ifndef DT_WORK_H
#define DT_WORK_H

enum dt_work_event {
  DT_WK_BOX          = 0,   /* BoundingVolume::intersect slab test, one ray x one node (geometry.cpp:2657-2740) */
  DT_WK_HIT_SHAPE    = 1,   /* + dt_shape_type (1..9): GeoPrimitive::intersect calls (cpp:514-538) */
  DT_WK_SHADOW_SHAPE = 11,  /* + dt_shape_type (1..9): GeoPrimitive::intersectShadow calls (cpp:832-852) */
  DT_WK_HIT          = 21,  /* a closest hit: isectP, getNorm, normalized ray, fixNorm, eye direction (cpp:546-567) */
  DT_WK_LIGHT        = 22,  /* a light iteration: sampleRay, |sray|, normalized sray, shadow origins (cpp:800-806) */
  DT_WK_BRDF         = 23,  /* + dt_model (0..3): Phong, Oren-Nayar, Cook-Torrance, raw (cpp:894-948) */
  DT_WK_EMIT         = 27,  /* emissive falloff of a light shape (cpp:775-789) */
  DT_WK_TEX          = 28,  /* getUV + nearest-texel lookup (cpp:859-893) */
  DT_WK_SKY          = 29,  /* one cloudColor: skyColor + the 200-step, 4-octave value-noise march (cpp:146-192) */
  DT_WK_CAMERA       = 30,  /* one sample's camera ray in one pass: getDOFSamples, getPerspEyeRay, focal point, blur shift */
  DT_WK_GLOSSY_RECT  = 31,  /* the glossy sample rectangle of a hit and its squeeze loops (cpp:644-695) */
  DT_WK_GLOSSY       = 32,  /* one glossy sample attempt (samplePoint, validity test, child origin; cpp:696-762) */
  DT_WK_REFRACT      = 33,  /* refraction ray + Fresnel (cpp:592-626, helpers.h:284-303) */
  DT_WK_MIRROR       = 34,  /* mirror reflection ray and child origin (cpp:628-638, 765) */
  DT_WK_N            = 35
};

/* FP64-equivalent VALU operations per event (rules above). Index = dt_work_event. */
static const double dt_work_weight[DT_WK_N] = {
  /* BOX: 3 axes x (2 sub, 2 mul, 2 cvt, 2 min/max) + 4 compares/selects + cull bound */
  30,
  /* HIT_SHAPE 1..9: sphere, cylinder, triangle, rectangle, RectPrismV2 (6 rectangles), checkerboard,
     checkerboard with hole, checker cylinder, RectPrismWithCylinder */
  0, 48, 95, 61, 55, 330, 70, 125, 95, 160,
  /* SHADOW_SHAPE 1..9 */
  0, 44, 95, 58, 55, 330, 55, 110, 95, 150,
  /* HIT: isectP 6, normal ~30, normalized ray 21, fixNorm 12, eye direction 24 */
  93,
  /* LIGHT: sample (area: half a draw + 12; point: 3) ~45, |sray| 10, normalized 21, 2 origins 12 */
  88,
  /* BRDF: Phong 64, Oren-Nayar 170, Cook-Torrance 184, raw 3 */
  64, 170, 184, 3,
  /* EMIT: four distances, |centre - A|, division, pow5, scaling */
  80,
  /* TEX: getUV ~60, texel index 8, three /255 12 */
  80,
  /* SKY: 200 steps x 4 octaves x (8 smoothed x (27 hashes x 16 + 33) + 3 cos x 20 + 7 lerps x 4
     + 9) + skyColor and contrast ~100 */
  3076100,
  /* CAMERA: DoF draw 80, sincos 20, eye sample 14, pixel ray 23, focal point 6, ray 3 */
  146,
  /* GLOSSY_RECT: rectangle 110, squeeze checks 36 */
  146,
  /* GLOSSY: half a draw 40, samplePoint 15, validity 6, child origin 6 */
  67,
  /* REFRACT */
  110,
  /* MIRROR */
  25
};

/* MI355X peaks the fraction is taken against (vendor figures; /opt/skills/guides/MI355X_MICROARCH.md) */
#define DT_PEAK_FP64_VECTOR_TFLOPS 78.6
#define DT_PEAK_HBM_GBPS 8000.0

#endif /* DT_WORK_H */
