// Minimal reproducer of the called-function defect: the sky of C5 frame 2200's pixels
// (buildFinal(2200) at 3840x2160, the deferred 1-spp sky of dt_sky_miss_kernel: cloudColor of
// mcam * focalPoint, render_final_project.cpp:164-192, 1074-1092) computed by cloud_color_lane inlined
// into one kernel and behind a real call in another (dt_kernels.hip DT_REPRO, compiled with the flags
// under test, tools/call_repro/build.sh). Prints how many pixels differ; exit 1 if any.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dt.h"
#include "../../distraytracer_amd/csrc/dt_scene_dev.h"

namespace dth {
int fill_params(const dt_globals& g, int frame, const dt_tiles* tiles, dtd::DParams& P, std::string& err);
std::vector<float> cloud_z_steps(const dt_globals& g);
}
extern "C" hipError_t dt_repro_launch(int call, const void* Pp, const float* zs, int x0, int y0, int w, int n,
                                      double* out);

int main(int argc, char** argv)
{
  const char* data = argc > 1 ? argv[1] : "data";
  const int frame = 2200;
  dt_globals g;
  dt_globals_default(&g);
  g.use_model = 0;
  dt_scene_desc* desc = nullptr;
  if (dt_build_scene("final", (float)frame, &g, data, &desc)) { fprintf(stderr, "build: %s\n", dt_last_error()); return 2; }
  g.xRes = 3840; g.yRes = 2160; g.antialias_samples = 1; g.max_depth = 10;
  dtd::DParams P;
  std::string err;
  if (dth::fill_params(g, frame, nullptr, P, err)) { fprintf(stderr, "params: %s\n", err.c_str()); return 2; }
  std::vector<float> zs = dth::cloud_z_steps(g);
  P.n_cloud_steps = (int)zs.size();
  // a window of the frame's sky: rows 1000..1063 over the full width (256k pixels)
  const int x0 = 0, y0 = 1000, w = 3840, n = w * 64;
  void *dP, *dz, *da, *db;
  if (hipMalloc(&dP, sizeof(P)) || hipMalloc(&dz, zs.size() * sizeof(float)) || hipMalloc(&da, 24 * (size_t)n) ||
      hipMalloc(&db, 24 * (size_t)n)) { fprintf(stderr, "hipMalloc failed\n"); return 2; }
  if (hipMemcpy(dP, &P, sizeof(P), hipMemcpyHostToDevice) ||
      hipMemcpy(dz, zs.data(), zs.size() * sizeof(float), hipMemcpyHostToDevice)) return 2;
  if (dt_repro_launch(0, dP, (const float*)dz, x0, y0, w, n, (double*)da) ||
      dt_repro_launch(1, dP, (const float*)dz, x0, y0, w, n, (double*)db) || hipDeviceSynchronize()) {
    fprintf(stderr, "launch failed\n");
    return 2;
  }
  std::vector<double> a(3 * (size_t)n), b(3 * (size_t)n);
  if (hipMemcpy(a.data(), da, 24 * (size_t)n, hipMemcpyDeviceToHost) ||
      hipMemcpy(b.data(), db, 24 * (size_t)n, hipMemcpyDeviceToHost)) return 2;
  long bad = 0;
  double mx = 0;
  int first = -1;
  for (int i = 0; i < n; ++i) {
    bool diff = memcmp(&a[3 * (size_t)i], &b[3 * (size_t)i], 24) != 0;
    if (diff) {
      if (first < 0) first = i;
      ++bad;
      for (int c = 0; c < 3; ++c) {
        const double d = a[3 * (size_t)i + c] - b[3 * (size_t)i + c];
        if (d > mx) mx = d;
        if (-d > mx) mx = -d;
      }
    }
  }
  printf("%s: %ld of %d pixels differ between the inlined and the called cloud_color_lane (max |diff| %.6g)",
         argc > 2 ? argv[2] : "repro", bad, n, mx);
  if (first >= 0)
    printf("; first at x=%d y=%d: inline (%.17g, %.17g, %.17g) call (%.17g, %.17g, %.17g)", x0 + first % w,
           y0 + first / w, a[3 * (size_t)first], a[3 * (size_t)first + 1], a[3 * (size_t)first + 2],
           b[3 * (size_t)first], b[3 * (size_t)first + 1], b[3 * (size_t)first + 2]);
  printf("\n");
  dt_scene_desc_free(desc);
  return bad ? 1 : 0;
}
