// TEST INFRASTRUCTURE ONLY. Compiles the reference's own noise.h, unmodified, from where it
// lies under /root/reference (include path set by oracle/Makefile), and exports its
// functions with C linkage so tests can pin oracle/oracle.c against it bit for bit.
// Output goes to oracle/_ref/ (git-ignored). No reference source is copied into the repo.
#include "noise.h"

extern "C" {
double ref_Noise3D(int i, int x, int y, int z) { return Noise3D(i, x, y, z); }
double ref_Smoothed3D(int i, int x, int y, int z) { return Smoothed3D(i, x, y, z); }
double ref_InterpolatedNoise3D(int i, double x, double y, double z)
{
  return InterpolatedNoise3D(i, x, y, z);
}
double ref_ValueNoise_3D(double x, double y, double z) { return ValueNoise_3D(x, y, z); }
double ref_cosInterpolate(double a, double b, double x) { return cosInterpolate(a, b, x); }
}
