// dtrender — host CLI mirroring the reference's `./render` modes (render_final_project.cpp:
// 1386-1956) on top of the C-ABI: builds the scene with the host builders, renders on the
// current MI355X through libdt's HIP kernels, writes the PPM. The models and ./ads assets are
// absent: use_model is off, and the tunnel's ad frames are the procedural stand-ins
// of host_scenes.cpp.
//
//   dtrender                 default: 980x540, antialias 2, frame 30 -> buildFinal(240) (1410-1424)
//   dtrender final <n>       1920x1080, antialias 10, depth 10, buildFinal(n*8) (1446-1456)
//   dtrender frame <n>       400x300 preview, aperture 0, 1 spp, no reflection (1428-1444)
//   dtrender nodistr <n>     antialias 6 (1457-1469)
//   dtrender perlin <i>      renderImageCloud 640x480 (1685-1698)
//   dtrender spheres         buildSceneSpheres(0) 256x256 (config C1)
//   dtrender prismcyl <n>    BuildScenePrismCylinder(n) 640x480 (1711-1723)
// options (after the mode): --out FILE(.ppm|.png)  --spp N  --depth N  --res WxH  --seed S
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dt.h"

static int die(const char* what, int rc)
{
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, dt_last_error());
  return 1;
}

int main(int argc, char** argv)
{
  dt_globals g;
  dt_globals_default(&g);
  g.use_model = 0;   // ./models absent (F6)
  std::string mode = argc > 1 ? argv[1] : "";
  int arg = (argc > 2 && argv[2][0] != '-') ? atoi(argv[2]) : 0;
  std::string out;
  std::string data_dir = DT_DATA_DIR;
  int spp = -1, depth = -1, W = -1, H = -1;
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--out" && i + 1 < argc) out = argv[++i];
    else if (a == "--spp" && i + 1 < argc) spp = atoi(argv[++i]);
    else if (a == "--depth" && i + 1 < argc) depth = atoi(argv[++i]);
    else if (a == "--seed" && i + 1 < argc) g.seed = (uint32_t)strtoul(argv[++i], nullptr, 10);
    else if (a == "--data" && i + 1 < argc) data_dir = argv[++i];
    else if (a == "--res" && i + 1 < argc) sscanf(argv[++i], "%dx%d", &W, &H);
  }
  std::string scene = "final";
  float build_frame = 0;
  int frame = 0;
  char buf[256];
  if (mode.empty()) {
    g.xRes = 980; g.yRes = 540; g.antialias_samples = 2; g.brdf_samples = 2;
    frame = 30 * 8; build_frame = (float)frame;
    snprintf(buf, sizeof buf, "./frame.%04d.ppm", 30);
  } else if (mode == "final") {
    frame = arg * 8; build_frame = (float)frame;
    snprintf(buf, sizeof buf, "./final_frames/frame.%04d.ppm", arg);
  } else if (mode == "frame") {
    g.xRes = 400; g.yRes = 300; g.aperture = 0; g.antialias_samples = 1; g.reflect = 0;
    frame = arg * 8; build_frame = (float)frame;
    snprintf(buf, sizeof buf, "./preview_frames/frame.%04d.ppm", arg);
  } else if (mode == "nodistr") {
    g.antialias_samples = 6; g.brdf_samples = 2;
    frame = arg * 8; build_frame = (float)frame;
    snprintf(buf, sizeof buf, "./nodistr/frame.%04d.ppm", arg);
  } else if (mode == "perlin") {
    g.xRes = 640; g.yRes = 480; g.aperture = 0; g.antialias_samples = 1;
    snprintf(buf, sizeof buf, "./test_frames/perlin/frame.%04d.ppm", arg);
    if (W > 0) { g.xRes = W; g.yRes = H; }
    std::vector<float> img((size_t)3 * g.xRes * g.yRes, 0.0f);
    dt_stats st;
    int rc = dt_render_sky(&g, (float)arg, nullptr, img.data(), 0, nullptr, &st);
    if (rc) return die("dt_render_sky", rc);
    std::string fn = out.empty() ? std::string(buf) : out;
    rc = dt_write_ppm(fn.c_str(), g.xRes, g.yRes, img.data());
    if (rc) return die("dt_write_ppm", rc);
    printf("Finished perlin cloud frame %d in %.3f ms (kernel) -> %s\n", arg, st.kernel_ms, fn.c_str());
    return 0;
  } else if (mode == "spheres") {
    scene = "spheres";
    snprintf(buf, sizeof buf, "./spheres.ppm");
  } else if (mode == "prismcyl") {
    scene = "prismcyl";
    g.xRes = 640; g.yRes = 480;
    frame = arg; build_frame = (float)arg;
    snprintf(buf, sizeof buf, "./test_frames/prismcyl/frame.%04d.ppm", arg);
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  dt_scene_desc* desc = nullptr;
  int rc = dt_build_scene(scene.c_str(), build_frame, &g, data_dir.c_str(), &desc);
  if (rc) return die("dt_build_scene", rc);
  if (scene == "spheres") { g.xRes = 256; g.yRes = 256; g.antialias_samples = 1; g.max_depth = 1; }
  if (spp > 0) g.antialias_samples = spp;
  if (depth > 0) g.max_depth = depth;
  if (W > 0) { g.xRes = W; g.yRes = H; }
  dt_scene* s = nullptr;
  rc = dt_scene_create(desc, &g, &s);
  if (rc) return die("dt_scene_create", rc);
  std::vector<float> img((size_t)3 * g.xRes * g.yRes, 0.0f);
  dt_stats st;
  rc = dt_render(s, &g, frame, nullptr, img.data(), 0, nullptr, &st);
  if (rc) return die("dt_render", rc);
  std::string fn = out.empty() ? std::string(buf) : out;
  const bool png = fn.size() > 4 && fn.compare(fn.size() - 4, 4, ".png") == 0;
  rc = png ? dt_write_png(fn.c_str(), g.xRes, g.yRes, img.data()) : dt_write_ppm(fn.c_str(), g.xRes, g.yRes, img.data());
  if (rc) return die("dt_write_ppm/png", rc);
  double msps = st.samples / (st.kernel_ms * 1e-3) / 1e6;
  printf("Rendered %s frame %d: %dx%d, %d spp, depth %d in %.2f ms (kernel, %.1f Mpixel-samples/s) -> %s\n",
         scene.c_str(), frame, g.xRes, g.yRes, (int)st.samples / (g.xRes * g.yRes), g.max_depth, st.kernel_ms,
         msps, fn.c_str());
  dt_scene_destroy(s);
  dt_scene_desc_free(desc);
  return 0;
}
