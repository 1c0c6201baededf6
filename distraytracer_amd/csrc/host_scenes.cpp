// host_scenes.cpp — the reference's scene builders (scene.h), restated as host C++ that
// fills a dt_scene_desc. Host input generation: the renderer never sees these functions,
// only the flattened descriptor. Each builder mutates dt_globals exactly as the reference
// builder mutates its globals (fresh-process semantics = start from
// dt_globals_default).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "host_internal.h"

using namespace dtm;

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

namespace {

struct OwnedDesc {
  dt_scene_desc d;   // must stay first: dt_scene_desc_free casts back
  std::vector<dt_shape_desc> shapes;
  std::vector<dt_light_desc> lights;
  std::vector<dt_texture_desc> tex;
  std::vector<std::vector<uint8_t>> texdata;
  std::vector<dt_shape_desc> holes;   // RectPrismWithCylinder::holes of the scene's prisms
  void finish()
  {
    d.n_shapes = (int32_t)shapes.size();
    d.n_lights = (int32_t)lights.size();
    d.n_textures = (int32_t)tex.size();
    d.n_holes = (int32_t)holes.size();
    for (size_t i = 0; i < tex.size(); ++i) tex[i].pixels = texdata[i].data();
    d.shapes = shapes.empty() ? nullptr : shapes.data();
    d.lights = lights.empty() ? nullptr : lights.data();
    d.textures = tex.empty() ? nullptr : tex.data();
    d.holes = holes.empty() ? nullptr : holes.data();
  }
};

void set3(double* d, V3 v)
{
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}

int material_of(const std::string& m)
{
  if (m.empty()) return DT_MAT_NONE;
  if (m == "glass") return DT_MAT_GLASS;
  if (m == "steel") return DT_MAT_STEEL;
  if (m == "aluminum") return DT_MAT_ALUMINUM;
  if (m == "water") return DT_MAT_WATER;
  if (m == "linoleum") return DT_MAT_LINOLEUM;
  return DT_MAT_OTHER;
}

int model_of(const std::string& s)
{
  if (s == "oren-nayar") return DT_MODEL_OREN_NAYAR;
  if (s == "cook-torrance") return DT_MODEL_COOK_TORRANCE;
  if (s == "raw") return DT_MODEL_RAW;
  return DT_MODEL_PHONG;
}

dt_shape_desc blank(int type)
{
  dt_shape_desc s;
  memset(&s, 0, sizeof(s));
  s.type = type;
  s.tex_frame = -1;
  return s;
}

// Sphere(c, r, col, material, in_motion, shader)  geometry.cpp:94-104
dt_shape_desc Sphere(V3 c, float r, V3 col, const std::string& material = "", bool motion = false,
                     const std::string& shader = "lambert")
{
  dt_shape_desc s = blank(DT_SHAPE_SPHERE);
  set3(s.v[0], c);
  set3(s.center, c);
  s.radius = r;
  set3(s.color, col);
  s.material = material_of(material);
  s.model = model_of(shader);
  if (motion) s.flags |= DT_F_MOTION;
  return s;
}

// Cylinder(v1, v2, r, col, material, in_motion, shader)  geometry.cpp:226-240
dt_shape_desc Cylinder(V3 v1, V3 v2, float r, V3 col, const std::string& material = "", bool motion = false,
                       const std::string& shader = "lambert")
{
  dt_shape_desc s = blank(DT_SHAPE_CYLINDER);
  set3(s.v[0], v1);
  set3(s.v[1], v2);
  s.radius = r;
  set3(s.color, col);
  s.material = material_of(material);
  s.model = model_of(shader);
  if (motion) s.flags |= DT_F_MOTION;
  set3(s.center, divs(add(v1, v2), 2));
  return s;
}

// Rectangle(a, b, c, d, col, material, in_motion, texframe, shader)  geometry.cpp:621-638
dt_shape_desc Rectangle(V3 a, V3 b, V3 c, V3 d, V3 col, const std::string& material = "", bool motion = false,
                        int texframe = -1, const std::string& shader = "lambert")
{
  dt_shape_desc s = blank(DT_SHAPE_RECTANGLE);
  set3(s.v[0], a);
  set3(s.v[1], b);
  set3(s.v[2], c);
  set3(s.v[3], d);
  s.length = (float)norm(sub(b, a));
  s.width = (float)norm(sub(d, a));
  set3(s.color, col);
  s.material = material_of(material);
  s.model = model_of(shader);
  if (motion) s.flags |= DT_F_MOTION;
  set3(s.center, divs(add(add(add(a, b), c), d), 4));
  s.flags |= DT_F_NAMED_RECT;   // name = "rectangle"
  if (texframe >= 0) s.tex_frame = texframe;
  return s;
}

// RectPrismV2(a..h, col, material, in_motion, texframe, shader)  geometry.cpp:784-813
dt_shape_desc RectPrismV2(V3 a, V3 b, V3 c, V3 d, V3 e, V3 f, V3 g, V3 h, V3 col,
                          const std::string& material = "", bool motion = false, int texframe = -1,
                          const std::string& shader = "lambert")
{
  dt_shape_desc s = blank(DT_SHAPE_RECTPRISM_V2);
  V3 vv[8] = {a, b, c, d, e, f, g, h};
  for (int k = 0; k < 8; ++k) set3(s.v[k], vv[k]);
  s.length = (float)norm(sub(b, a));
  s.width = (float)norm(sub(d, a));
  set3(s.color, col);
  s.material = material_of(material);
  s.model = model_of(shader);
  if (motion) s.flags |= DT_F_MOTION;
  V3 ctr = a;
  for (int k = 1; k < 8; ++k) ctr = add(ctr, vv[k]);
  set3(s.center, divs(ctr, 8));
  if (texframe >= 0) s.tex_frame = texframe;
  return s;
}

// RectPrismWithCylinder(a..h, col, material, in_motion, texframe, shader)  geometry.cpp:1467-1505;
// its holes are appended to O.holes by the caller (tmp->holes.push_back, scene.h:3241)
dt_shape_desc RectPrismWithCylinder(V3 a, V3 b, V3 c, V3 d, V3 e, V3 f, V3 g, V3 h, V3 col,
                                    const std::string& material = "", bool motion = false, int texframe = -1,
                                    const std::string& shader = "lambert")
{
  dt_shape_desc s = RectPrismV2(a, b, c, d, e, f, g, h, col, material, motion, texframe, shader);
  s.type = DT_SHAPE_RECTPRISM_CYL;   // same vertex members, centre (A+..+H)/8 and float length/width
  return s;
}

// CheckerboardWithHole(a,b,c,d,col1,col2,S,hole,material,in_motion,shader)  geometry.cpp:2344-2364
dt_shape_desc CheckerboardWithHole(V3 a, V3 b, V3 c, V3 d, V3 col1, V3 col2, float S, V3 ha, V3 hb, V3 hc, V3 hd,
                                   const std::string& material = "", bool motion = false,
                                   const std::string& shader = "lambert")
{
  dt_shape_desc s = blank(DT_SHAPE_CHECKERBOARD_HOLE);
  set3(s.v[0], a);
  set3(s.v[1], b);
  set3(s.v[2], c);
  set3(s.v[3], d);
  set3(s.v[4], ha);
  set3(s.v[5], hb);
  set3(s.v[6], hc);
  set3(s.v[7], hd);
  s.length = (float)norm(sub(b, a));
  s.width = (float)norm(sub(d, a));
  set3(s.color, col1);
  set3(s.color1, col1);
  set3(s.color2, col2);
  s.S = S;
  s.material = material_of(material);
  s.model = model_of(shader);
  if (motion) s.flags |= DT_F_MOTION;
  set3(s.center, divs(add(add(add(a, b), c), d), 4));
  return s;
}

// CheckerCylinder(v1, v2, r, col, s, material, in_motion, shader)  geometry.cpp:2563-2586
dt_shape_desc CheckerCylinder(V3 v1, V3 v2, float r, V3 col, float S, const std::string& material = "",
                              bool motion = false, const std::string& shader = "lambert")
{
  dt_shape_desc s = Cylinder(v1, v2, r, col, material, motion, shader);
  s.type = DT_SHAPE_CHECKER_CYLINDER;
  s.S = S;
  return s;
}

// rectangleLight(a,b,c,d,col): Rectangle() default ctor + light fields (geometry.cpp:2829-2843)
void RectangleLight(OwnedDesc& O, V3 a, V3 b, V3 c, V3 d, V3 col)
{
  dt_shape_desc s = blank(DT_SHAPE_RECTANGLE);
  set3(s.v[0], a);
  set3(s.v[1], b);
  set3(s.v[2], c);
  set3(s.v[3], d);
  s.length = 1;   // default ctor values (geometry.cpp:608-609), never recomputed
  s.width = 1;
  set3(s.color, col);
  s.model = DT_MODEL_PHONG;
  s.material = DT_MAT_NONE;
  s.flags |= DT_F_LIGHT;
  s.emit = DT_EMIT_RECT;
  set3(s.center, divs(add(add(add(a, b), c), d), 4));
  dt_light_desc L;
  memset(&L, 0, sizeof(L));
  L.type = DT_LIGHT_RECT;
  L.shape_index = (int32_t)O.shapes.size() + 0;   // pushed to shapes right after lights
  set3(L.center, divs(add(add(add(a, b), c), d), 4));
  set3(L.color, col);
  set3(L.A, a);
  set3(L.B, b);
  set3(L.D, d);
  O.lights.push_back(L);
  O.shapes.push_back(s);
}

void PointLight(OwnedDesc& O, V3 c, V3 col)
{
  dt_light_desc L;
  memset(&L, 0, sizeof(L));
  L.type = DT_LIGHT_POINT;
  L.shape_index = -1;
  set3(L.center, c);
  set3(L.color, col);
  O.lights.push_back(L);
}

// helpers.h:222-229 (including its row-3 typo: anorm[1]*sin in R(2,0))
V3 rotate(V3 point, V3 axis, float theta)
{
  V3 a = normalized(axis);
  float ct = cosf(theta), st = sinf(theta);
  float omc = 1 - ct;
  double R[3][3];
  R[0][0] = ct + pow(a.x, 2) * omc;
  R[0][1] = a.x * a.y * omc - a.z * st;
  R[0][2] = a.x * a.z * omc + a.y * st;
  R[1][0] = a.y * a.x * omc + a.z * st;
  R[1][1] = ct + pow(a.y, 2) * omc;
  R[1][2] = a.y * a.z * omc - a.x * st;
  R[2][0] = a.z * a.y * omc - a.y * st;
  R[2][1] = a.z * a.y * omc + a.x * st;
  R[2][2] = ct + pow(a.z, 2) * omc;
  double p[3] = {point.x, point.y, point.z}, o[3];
  for (int i = 0; i < 3; ++i) o[i] = (R[i][0] * p[0] + R[i][1] * p[1]) + R[i][2] * p[2];
  return v3(o[0], o[1], o[2]);
}

bool load_rgb(const std::string& path, std::vector<uint8_t>& data, int& w, int& h, int& n)
{
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::string magic;
  f >> magic >> w >> h >> n;
  if (magic != "DTRGB" || w <= 0 || h <= 0 || n < 3) return false;
  f.get();
  data.resize((size_t)w * h * n);
  f.read((char*)data.data(), data.size());
  return (size_t)f.gcount() == data.size();
}

// loadTexture (helpers.h:92-113): appends to texture_frames, returns its index
int load_texture(OwnedDesc& O, const std::string& data_dir, const std::string& name, std::string& err)
{
  std::vector<uint8_t> d;
  int w, h, n;
  std::string p = data_dir + "/textures/" + name + ".rgb";
  if (!load_rgb(p, d, w, h, n)) {
    err = "Image loading failed for: " + p;
    return -1;
  }
  dt_texture_desc t;
  memset(&t, 0, sizeof(t));
  t.width = w;
  t.height = h;
  t.channels = n;
  O.tex.push_back(t);
  O.texdata.push_back(std::move(d));
  return (int)O.tex.size() - 1;
}

// Triangle(a, b, c, col, material, in_motion, shader)  geometry.cpp:434-445
dt_shape_desc Triangle(V3 a, V3 b, V3 c, V3 col, const std::string& material = "", bool motion = false,
                       const std::string& shader = "lambert")
{
  dt_shape_desc s = blank(DT_SHAPE_TRIANGLE);
  set3(s.v[0], a);
  set3(s.v[1], b);
  set3(s.v[2], c);
  set3(s.color, col);
  s.material = material_of(material);
  s.model = model_of(shader);
  if (motion) s.flags |= DT_F_MOTION;
  set3(s.center, divs(add(add(a, b), c), 3));
  return s;
}

// loadObj (objHelper.h:6-85, tinyobj): positions and texcoords as float (tinyobj real_t),
// triangle faces "f v[/vt[/vn]] x3" with 1-based indices. Only what finalBuildModels uses.
struct ObjMesh {
  std::vector<V3> v;
  std::vector<double> vt;            // pairs
  std::vector<int> vi, ti;           // 3 per triangle; ti = -1 without texcoords
};

bool load_obj(const std::string& path, ObjMesh& m, std::string& err)
{
  std::ifstream f(path);
  if (!f) {
    err = "TinyObjReader: cannot open " + path;
    return false;
  }
  std::string line;
  while (std::getline(f, line)) {
    if (line.size() < 2 || line[0] == '#') continue;
    const char* c = line.c_str();
    if (c[0] == 'v' && c[1] == ' ') {
      float x, y, z;
      if (sscanf(c + 2, "%f %f %f", &x, &y, &z) != 3) { err = "bad vertex: " + line; return false; }
      m.v.push_back(v3(x, y, z));
    } else if (c[0] == 'v' && c[1] == 't') {
      float u, w;
      if (sscanf(c + 3, "%f %f", &u, &w) != 2) { err = "bad texcoord: " + line; return false; }
      m.vt.push_back(u);
      m.vt.push_back(w);
    } else if (c[0] == 'f' && c[1] == ' ') {
      const char* q = c + 2;
      int got = 0;
      while (*q && got < 3) {
        while (*q == ' ') ++q;
        if (!*q) break;
        int vi = 0, ti = 0;
        int n = 0;
        if (sscanf(q, "%d/%d%n", &vi, &ti, &n) == 2) {
        } else if (sscanf(q, "%d%n", &vi, &n) == 1) {
          ti = 0;
        } else {
          err = "bad face: " + line;
          return false;
        }
        q += n;
        while (*q && *q != ' ') ++q;   // skip a trailing /vn
        m.vi.push_back(vi - 1);
        m.ti.push_back(ti - 1);
        ++got;
      }
      if (got != 3) { err = "non-triangle face: " + line; return false; }
    }
  }
  for (int i : m.vi)
    if (i < 0 || i >= (int)m.v.size()) { err = "vertex index out of range in " + path; return false; }
  for (int i : m.ti)
    if (i >= (int)(m.vt.size() / 2)) { err = "texcoord index out of range in " + path; return false; }
  return true;
}

// MATRIX4 * (p, 1), head<3>: sequential sums over k (Eigen fixed-size product)
V3 xform(const double M[3][4], V3 p)
{
  double o[3];
  for (int i = 0; i < 3; ++i) o[i] = ((M[i][0] * p.x + M[i][1] * p.y) + M[i][2] * p.z) + M[i][3] * 1.0;
  return v3(o[0], o[1], o[2]);
}

// finalBuildModels (scene.h:258-602) with the substitute assets of tools/gen_models.py
int final_build_models(dt_globals& g, const std::string& data_dir, OwnedDesc& O, std::string& err)
{
  const float min_y = (float)(0.301897 + g.tot_move);
  const std::string mdir = data_dir + "/models/";
  ObjMesh col;
  if (!load_obj(mdir + "Column_LP_obj/Column_LP.obj", col, err)) return DT_E_IO;
  // loadTexture(Marble_Base_Color) then the roughness map read raw with stbi_load
  std::vector<uint8_t> tex, rough;
  int tw, th, tn, rw, rh, rn;
  if (!load_rgb(mdir + "Column_LP_obj/Textures/Marble_Base_Color.jpg.rgb", tex, tw, th, tn) ||
      !load_rgb(mdir + "Column_LP_obj/Textures/Marble_Roughness.jpg.rgb", rough, rw, rh, rn)) {
    err = "Image loading failed for: " + mdir + "Column_LP_obj/Textures";
    return DT_E_IO;
  }
  dt_texture_desc td;
  memset(&td, 0, sizeof(td));
  td.width = tw;
  td.height = th;
  td.channels = tn;
  O.tex.push_back(td);
  O.texdata.push_back(std::move(tex));
  const int tex_index = (int)O.tex.size() - 1;
  for (int side = 0; side < 2; ++side) {   // left (-3) and right (+3) straddle columns
    const double M[3][4] = {{3, 0, 0, side ? 3.0 : -3.0}, {0, 3, 0, (double)min_y}, {0, 0, 3, 5}};
    std::vector<V3> pv(col.v.size());
    for (size_t i = 0; i < col.v.size(); ++i) pv[i] = xform(M, col.v[i]);
    for (size_t i = 0; i < col.vi.size() / 3; ++i) {
      const int* vi = &col.vi[3 * i];
      const int* ti = &col.ti[3 * i];
      if (ti[0] < 0 || ti[1] < 0 || ti[2] < 0) { err = "column mesh needs texcoords"; return DT_E_INVALID; }
      dt_shape_desc s = Triangle(pv[vi[0]], pv[vi[1]], pv[vi[2]], v3(0.75, 0.75, 0.75), "marble", false,
                                 "oren-nayar");
      double uv[3][2];
      for (int k = 0; k < 3; ++k) {
        uv[k][0] = col.vt[2 * ti[k]];
        uv[k][1] = col.vt[2 * ti[k] + 1];
        if (uv[k][0] > 1) uv[k][0] = uv[k][0] - (int)uv[k][0];   // scene.h:338-343
        if (uv[k][1] > 1) uv[k][1] = uv[k][1] - (int)uv[k][1];
      }
      if (!(uv[0][0] >= 0 && uv[0][1] <= 1 && uv[1][0] >= 0 && uv[1][1] <= 1 && uv[2][0] >= 0 && uv[2][1] <= 1)) {
        err = "Texcoords out of bounds";   // scene.h:346-356 throws
        return DT_E_INVALID;
      }
      for (int k = 0; k < 3; ++k) {
        s.uv[k][0] = uv[k][0];
        s.uv[k][1] = 1 - uv[k][1];   // scene.h:359-361
      }
      s.flags |= DT_F_UV_VERTS | DT_F_TEXTURE;
      s.tex_frame = tex_index;
      // roughness map read as raw bytes at the (unwrapped) texcoords, scene.h:373-376
      float r[3];
      for (int k = 0; k < 3; ++k) {
        double u = col.vt[2 * ti[k]], w = col.vt[2 * ti[k] + 1];
        long idx = (long)(u * (int)(rw - 1) + w * (int)(rh - 1) * (rw - 1));
        if (idx < 0 || idx >= (long)rough.size()) { err = "roughness index out of range"; return DT_E_INVALID; }
        r[k] = rough[(size_t)idx];
      }
      s.roughness = (r[0] + r[1] + r[2]) / (3 * 255);
      O.shapes.push_back(s);
    }
  }
  ObjMesh bust;
  if (!load_obj(mdir + "helios_statue/helios_20.obj", bust, err)) return DT_E_IO;
  for (int side = 0; side < 2; ++side) {   // scene.h:471-478, 517-521
    const double M[3][4] = {{1.8 * cos(M_PI), 0, 1.8 * sin(M_PI), side ? 3.0 : -3.0},
                            {0, 1.8, 0, 3.9 + min_y},
                            {-1.8 * sin(M_PI), 0, 1.8 * cos(M_PI), 4}};
    std::vector<V3> hv(bust.v.size());
    for (size_t i = 0; i < bust.v.size(); ++i) hv[i] = xform(M, bust.v[i]);
    for (size_t i = 2; i < bust.vi.size() / 3; ++i) {   // the reference starts at triangle 2
      const int* vi = &bust.vi[3 * i];
      dt_shape_desc s = Triangle(hv[vi[0]], hv[vi[1]], hv[vi[2]], v3(0.75, 0.75, 0.75), "marble", false,
                                 "oren-nayar");
      s.roughness = 0.5f;
      O.shapes.push_back(s);
    }
  }
  return DT_OK;
}

// ---- ./ads substitute --------------------------------------------------------
// The reference lists every ./ads/<campaign>/*.jpg into frame_paths (render_final_project.cpp:
// 90-95, 1401-1406) and the tunnel mesh picks frames from it. The assets are absent; the
// substitute is a fixed-size list of procedurally generated 80x45 "ad" frames, frame i being
// a deterministic function of i (a banner colour, stripes and blocks), generated on load.
const int kAdFrames = 2400;   // >= 1000 + (frame_cloud - frame_prism): every index stays in range
const int kAdW = 80, kAdH = 45;

uint32_t ad_hash(uint32_t x)
{
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

int load_ad_frame(OwnedDesc& O, int idx)
{
  std::vector<uint8_t> px((size_t)kAdW * kAdH * 3);
  const uint32_t h0 = ad_hash((uint32_t)idx * 2654435761u + 17u);
  const int br = 60 + (h0 & 127), bg = 60 + ((h0 >> 7) & 127), bb = 60 + ((h0 >> 14) & 127);
  const int stripe = 3 + ((h0 >> 21) & 7);
  for (int y = 0; y < kAdH; ++y)
    for (int x = 0; x < kAdW; ++x) {
      uint8_t* q = &px[((size_t)y * kAdW + x) * 3];
      const bool band = ((x + y + idx) / stripe) % 3 == 0;
      const bool block = x > 10 && x < 40 && y > 12 && y < 32;
      q[0] = (uint8_t)(block ? 255 - br : band ? br / 2 : br);
      q[1] = (uint8_t)(block ? 255 - bg : band ? bg / 2 : bg);
      q[2] = (uint8_t)(block ? 255 - bb : band ? bb / 2 : bb);
    }
  dt_texture_desc t;
  memset(&t, 0, sizeof(t));
  t.width = kAdW;
  t.height = kAdH;
  t.channels = 3;
  O.tex.push_back(t);
  O.texdata.push_back(std::move(px));
  return (int)O.tex.size() - 1;
}

// generateTrianglePrismMesh (scene.h:135-256): the ad-covered tunnel the camera falls through
void triangle_prism_mesh(OwnedDesc& O, const dt_globals& g, V3 a_cap0, V3 b_cap0, V3 c_cap0, V3 a_cap1, V3 b_cap1,
                         V3 c_cap1, int time_frame, bool texture, bool motion)
{
  std::uniform_int_distribution<> unif(0, kAdFrames - 1000);
  const V3 eye = v3a(g.eye);
  const float far = g.far_dist;
  O.shapes.push_back(Triangle(a_cap1, b_cap1, c_cap1, v3(1, 1, 1)));
  const int n_rect = 4;
  const float bounding_width = 0.1f;
  const float rect_height = (float)((norm(sub(a_cap0, b_cap0)) - bounding_width * n_rect) / n_rect);
  const float rect_width = (float)5 / 3 * rect_height;
  const V3 length_v = normalized(sub(c_cap1, c_cap0));
  const V3 ac_v = normalized(sub(a_cap0, c_cap0));
  const V3 ab_v = normalized(sub(a_cap0, b_cap0));
  const V3 bc_v = normalized(sub(c_cap0, b_cap0));
  V3 left_a = add(b_cap0, mul(bounding_width, length_v));
  V3 left_b = add(left_a, mul(rect_width, length_v));
  V3 left_c = add(left_b, mul(rect_height, ab_v));
  V3 left_d = add(left_a, mul(rect_height, ab_v));
  V3 right_b = add(c_cap0, mul(bounding_width, length_v));
  V3 right_a = add(right_b, mul(rect_width, length_v));
  V3 right_d = add(right_a, mul(rect_height, ac_v));
  V3 right_c = add(right_b, mul(rect_height, ac_v));
  V3 bottom_a = add(add(b_cap0, mul(bounding_width, length_v)), mul(bounding_width, bc_v));
  V3 bottom_b = add(bottom_a, mul(rect_width, length_v));
  V3 bottom_c = add(bottom_b, mul(rect_height, bc_v));
  V3 bottom_d = add(bottom_a, mul(rect_height, bc_v));
  const V3 adj_b0 = add(b_cap0, divs(mul(bounding_width, bc_v), 2));
  int seed_counter = 0;
  auto place = [&](V3 a, V3 b, V3 c, V3 d, V3 dir, int i, uint32_t seed) {
    std::mt19937 gen(seed);   // scene.h:57, reseeded per rectangle (local: dt_build_scene stays reentrant)
    const int frame_ind = unif(gen) + (time_frame - g.frame_prism);
    const int tex_index = load_ad_frame(O, frame_ind);
    const V3 off = mul((double)i, mul(bounding_width + rect_height, dir));
    dt_shape_desc r = Rectangle(add(a, off), add(b, off), add(c, off), add(d, off), v3(0, 1, 0), "", motion,
                                tex_index, "raw");
    if (motion) r.flags |= DT_F_MOTION;
    if (texture) r.flags |= DT_F_TEXTURE;
    O.shapes.push_back(r);
  };
  while (norm(sub(bottom_b, adj_b0)) <= norm(sub(c_cap1, c_cap0))) {
    for (int i = 0; i < n_rect; i++) {
      // skip rectangles behind the eye or beyond `far` (scene.h:187-188)
      if (!(left_b.y > eye.y && left_c.y > eye.y) & !(norm(sub(left_b, eye)) > far && norm(sub(left_c, eye)) > far))
        place(left_a, left_b, left_c, left_d, ab_v, i, (uint32_t)seed_counter);
      seed_counter++;
      if (!(right_a.y > eye.y && right_d.y > eye.y) & !(norm(sub(right_a, eye)) > far && norm(sub(right_d, eye)) > far))
        place(right_a, right_b, right_c, right_d, ac_v, i, (uint32_t)(seed_counter + 1));
      seed_counter++;
      if (!(bottom_b.y > eye.y && bottom_c.y > eye.y) &
          !(norm(sub(bottom_b, eye)) > far && norm(sub(bottom_c, eye)) > far))
        place(bottom_a, bottom_b, bottom_c, bottom_d, bc_v, i, (uint32_t)(seed_counter + 2));
      seed_counter++;
    }
    const V3 step = mul(rect_width + bounding_width, length_v);
    left_a = add(left_a, step); left_b = add(left_b, step); left_c = add(left_c, step); left_d = add(left_d, step);
    right_a = add(right_a, step); right_b = add(right_b, step); right_c = add(right_c, step);
    right_d = add(right_d, step);
    bottom_a = add(bottom_a, step); bottom_b = add(bottom_b, step); bottom_c = add(bottom_c, step);
    bottom_d = add(bottom_d, step);
  }
}

// ---- buildSceneSpheres (scene.h:4399-4420) --------------------------------------------
int build_spheres(float frame, dt_globals& g, OwnedDesc& O)
{
  V3 center = v3(0, 0.5, 1);
  float x = 0;
  V3 eye = v3a(g.eye);
  for (int i = 0; i < 4; i++) {
    float r = (float)(0.3 * pow(1.5, i));
    float width = (float)(g.aspect * tan(g.fov * M_PI / 360.0) * (x - eye.x));
    V3 center_adj = add(center, v3(x, 0, sin((i + 1) * frame / 180 * 2 * M_PI) * width));
    O.shapes.push_back(Sphere(center_adj, r, v3(1, 0, 0), "", true));
    x += r * 2 * (i + 1);
  }
  O.shapes.push_back(Sphere(v3(0.5, -1000, 1), 999, v3(0.5, 0.5, 0.5)));
  PointLight(O, eye, v3(0.9, 0.9, 0.9));
  return DT_OK;
}

// ---- buildSceneDOF (scene.h:4422-4449) --------------------------------------------------
int build_dof(float, dt_globals& g, OwnedDesc& O)
{
  V3 start = v3(0, 0.5, 1);
  float r = 0.3f;
  V3 dir = normalized(v3(1, 0, 1));
  O.shapes.push_back(Sphere(start, 0.3f, v3(1, 0, 0)));
  for (int i = 1; i < 8; i++) {
    V3 col = i % 2 == 0 ? v3(1, 0, 0) : v3(0, 1, 0);
    O.shapes.push_back(Sphere(add(start, mul(2 * i * r, dir)), 0.3f, col));
    O.shapes.push_back(Sphere(sub(start, mul(2 * i * r, dir)), 0.3f, col));
  }
  O.shapes.push_back(Sphere(v3(0.5, -1000, 1), 999, v3(0.5, 0.5, 0.5)));
  PointLight(O, v3a(g.eye), v3(0.9, 0.9, 0.9));
  return DT_OK;
}

// ---- buildSceneHW4 (scene.h:4451-4477) --------------------------------------------------
int build_hw4(float, dt_globals&, OwnedDesc& O)
{
  O.shapes.push_back(Sphere(v3(-3.5, 0, -10), 3, v3(1, 0.25, 0.25)));
  O.shapes.push_back(Sphere(v3(3.5, 0, -10), 3, v3(0.25, 0.25, 1)));
  O.shapes.push_back(Sphere(v3(0, -1000, -10), 997, v3(0.5, 0.5, 0.5)));
  PointLight(O, v3(10, 3, -5), v3(1, 1, 1));
  PointLight(O, v3(-10, 3, -7.5), v3(0.5, 0, 0));
  return DT_OK;
}

// ---- BuildScenePrismCylinder (scene.h:3227-3263), the `./render prismcyl` mode ----------------
// A 4x4x1 box (RectPrismWithCylinder) with one cylinder hole of radius 1 through it, a point light;
// the eye is rotated about itself (to_origin, rotation, from_origin around og_eye), which leaves it
// at og_eye up to the rounding of the 4x4 products (sequential sums, oracle.c header).
int build_prismcyl(float frame, dt_globals& g, OwnedDesc& O)
{
  const V3 A = v3(0, -2, -2), B = v3(0, -2, 2), C = v3(0, 2, 2), D = v3(0, 2, -2), back = v3(1, 0, 0);
  dt_shape_desc p = RectPrismWithCylinder(A, B, C, D, add(A, back), add(B, back), add(C, back), add(D, back),
                                          v3(1, 0, 0));
  const V3 c1 = divs(add(add(add(A, B), C), D), 4);
  const V3 c2 = add(c1, back);
  p.hole_first = (int32_t)O.holes.size();
  p.n_holes = 1;
  O.holes.push_back(Cylinder(c1, c2, 1, v3(0, 0, 1)));
  O.shapes.push_back(p);
  PointLight(O, v3(-5, 1, 0), v3(1, 1, 1));
  const double og[4] = {-6, 0.5, 1, 1};
  const float theta = (float)(M_PI * 2 * frame / 50);
  // cos(theta) / sin(theta) of a float: <cmath>'s float overloads (cosf / sinf)
  const double ct = cosf(theta), st = sinf(theta);
  const double to_origin[4][4] = {{1, 0, 0, -og[0]}, {0, 1, 0, -og[1]}, {0, 0, 1, -og[2]}, {0, 0, 0, 1}};
  const double rot[4][4] = {{ct, 0, st, 0}, {0, 1, 0, 0}, {-st, 0, ct, 0}, {0, 0, 0, 1}};
  const double from_origin[4][4] = {{1, 0, 0, og[0]}, {0, 1, 0, og[1]}, {0, 0, 1, og[2]}, {0, 0, 0, 1}};
  double m1[4][4], m2[4][4];
  auto mul4 = [](const double a[4][4], const double b[4][4], double r[4][4]) {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        double acc = a[i][0] * b[0][j];
        for (int k = 1; k < 4; ++k) acc = acc + a[i][k] * b[k][j];
        r[i][j] = acc;
      }
  };
  mul4(from_origin, rot, m1);
  mul4(m1, to_origin, m2);
  for (int i = 0; i < 3; ++i) {
    double acc = m2[i][0] * og[0];
    for (int k = 1; k < 4; ++k) acc = acc + m2[i][k] * og[k];
    g.eye[i] = acc;
  }
  return DT_OK;
}

// bone table written by tools/gen_bones.py from dt_mocap_bone_table
bool load_bones(const std::string& data_dir, int posture_frame, std::vector<double>& out, std::string& err)
{
  std::string p = data_dir + "/bones_90_16_v3.bin";
  std::ifstream f(p, std::ios::binary);
  if (!f) {
    err = "missing bone table " + p + " (tools/gen_bones.py)";
    return false;
  }
  std::string magic;
  int n_frames, n_bones, n_postures;
  f >> magic >> n_frames >> n_bones >> n_postures;
  f.get();
  if (magic != "DTBONES" || n_frames <= 0 || n_bones <= 0) {
    err = "bad bone table " + p;
    return false;
  }
  if (posture_frame >= n_postures) posture_frame = n_postures - 1;   // scene.h:121-125
  if (posture_frame < 0) posture_frame = 0;
  std::vector<int32_t> ids(n_frames);
  f.read((char*)ids.data(), sizeof(int32_t) * n_frames);
  for (int i = 0; i < n_frames; ++i) {
    if (ids[i] == posture_frame) {
      out.resize((size_t)n_bones * 6);
      f.seekg((std::streamoff)((size_t)i * n_bones * 6 * sizeof(double)), std::ios::cur);
      f.read((char*)out.data(), out.size() * sizeof(double));
      return (size_t)f.gcount() == out.size() * sizeof(double);
    }
  }
  err = "bone table has no posture " + std::to_string(posture_frame);
  return false;
}

// ---- buildFinal (scene.h:605-1100) ---------------------------------------------------------
int build_final(float frame, dt_globals& g, const std::string& data_dir, OwnedDesc& O, std::string& err)
{
  g.perlin_cloud = 1;
  std::vector<double> bones;
  if (!load_bones(data_dir, (int)frame, bones, err)) return DT_E_IO;
  const int nb = (int)bones.size() / 6;
  for (int x = 0; x < nb; ++x) {
    V3 l = v3(bones[x * 6 + 0], bones[x * 6 + 1], bones[x * 6 + 2]);
    V3 r = v3(bones[x * 6 + 3], bones[x * 6 + 4], bones[x * 6 + 5]);
    if (frame >= g.frame_cloud) {   // scene.h:646-651
      double dy = (double)(frame - g.frame_cloud);
      l.y = l.y - dy;
      r.y = r.y - dy;
    }
    O.shapes.push_back(Cylinder(l, r, 0.05f, v3(1, 0, 0)));
  }
  // camera choreography (scene.h:667-709)
  V3 init_eye = v3(-7, 9, -4), init_lookingAt = v3(8, 11, 6);
  V3 final_eye = v3(0.5, 8, 1.1), final_lookingAt = v3(0.5, 0.5, 1);
  V3 eye = v3a(g.eye), lookingAt = v3a(g.lookingAt), up = v3a(g.up);
  if (frame <= g.frame_prism) {
    eye = init_eye;
    lookingAt = init_lookingAt;
    float final_theta = (float)(M_PI * 9 / 8);
    float theta = fminr(final_theta, frame * final_theta / g.frame_move1);
    eye = rotate(eye, v3(0, 1, 0), theta);
    while (eye.x < -10 || eye.x > 10 || eye.z < -5 || eye.z > 8) eye = mul(0.999, eye);
    lookingAt = rotate(lookingAt, v3(0, 1, 0), theta);
    lookingAt = sub(lookingAt, v3(0, frame / g.frame_move1 * 10, 0));
  }
  if (frame <= g.frame_prism && frame >= g.frame_move1) {
    double f = dmin(1.0, (double)(frame - g.frame_move1) / (g.frame_move2 - g.frame_move1));
    eye = add(eye, mul(f, sub(final_eye, eye)));
    lookingAt = add(lookingAt, mul(f, sub(final_lookingAt, lookingAt)));
    float theta = (float)(-M_PI / 2 * f);
    up = rotate(up, v3(1, 0, 0), theta);
  }
  if (frame > g.frame_prism) {
    eye = final_eye;
    lookingAt = final_lookingAt;
    up = v3(0, 0, -1);
    g.focal_length = 20;
  }
  // movement (scene.h:711-733)
  float tunnel_transition = 20 * 8;
  float movement_multiplier = fmaxr(0.0f, frame - g.frame_prism);
  g.move_per_frame = (float)(0.1 / 8);
  g.move_per_frame *= (1 + fminr(2.0f, 2 * (movement_multiplier) / tunnel_transition));
  g.tot_move = movement_multiplier * g.move_per_frame;
  float accel_d = (float)(g.accel_t * pow(frame - g.frame_blur, 3));
  /* dist = 263 only sizes the tunnel mesh (frames >= frame_prism) */
  if (frame > g.frame_blur && frame <= g.frame_cloud) {
    g.tot_move += accel_d;
    g.move_per_frame += 0.1 / (2 * 64) * pow(frame - g.frame_blur, 2);
  }
  float min_y = (float)(0.301897 + g.tot_move);
  float xmin = -0.1f, xmax = 1.7f, zmin = -0.4f, zmax = 1.9f;
  V3 A = v3(xmin, min_y, zmax), B = v3((xmin + xmax) / 2, min_y, zmax), C = v3((xmin + xmax) / 2, min_y, zmin);
  V3 D = v3(xmin, min_y, zmin), E = v3(xmax, min_y, zmax), F = v3(xmax, min_y, zmin);
  V3 gA = v3(-10, min_y, -5), gB = v3(-10, min_y, 8), gC = v3(10, min_y, 8), gD = v3(10, min_y, -5);
  V3 gE = v3(-10, 10 + min_y, -5), gF = v3(-10, 10 + min_y, 8), gG = v3(10, 10 + min_y, 8),
     gH = v3(10, 10 + min_y, -5);
  V3 gEH = normalized(sub(gE, gH)), gEF = normalized(sub(gE, gF)), gAD = normalized(sub(gA, gD)),
     gCD = normalized(sub(gC, gD));
  // tunnel transition (scene.h:760-766)
  V3 tunnel_point = v3((xmin + xmax) / 2, 5, (zmin + zmax) / 2);
  V3 eye_path = normalized(sub(tunnel_point, eye));
  float accel = (float)(norm(sub(tunnel_point, eye)) / pow(tunnel_transition, 2));
  double mv = accel * pow(fminr(tunnel_transition, movement_multiplier), 2);
  eye = add(mul(mv, eye_path), eye);
  lookingAt = add(mul(mv, eye_path), lookingAt);
  // triangle prism caps (scene.h:772-781)
  V3 b_cap0 = v3(xmin, min_y, zmax), c_cap0 = v3(xmax, min_y, zmax);
  V3 a_cap0 = v3((xmin + xmax) / 2, min_y, (xmin - xmax) * sqrt(3) / 2 + zmax);
  V3 cap_center = divs(add(add(a_cap0, b_cap0), c_cap0), 3);
  set3(g.cap_center, cap_center);
  if (frame >= g.frame_prism + tunnel_transition) PointLight(O, eye, v3(1, 1, 1));
  set3(g.eye, eye);
  set3(g.lookingAt, lookingAt);
  set3(g.up, up);
  if (frame >= g.frame_cloud) {   // scene.h:788-803
    g.aperture = 0;
    g.antialias_samples = 1;
    V3 sunorange = v3(0.953, 0.51, 0.21), pastelpink = v3(1, 0.82, 0.863), violet = v3(0.541, 0.168, 0.886),
       indigo = v3(75.0 / 255, 0, 130.0 / 255), darkblue = v3(0.0667, 0.1137, 0.37);
    auto lerp = [&](double* c, V3 target) {
      V3 cur = v3a(c);
      set3(c, add(cur, divs(mul(frame - g.frame_cloud, sub(target, cur)), (g.total - g.frame_cloud))));
    };
    lerp(g.redsky, sunorange);
    lerp(g.bluesky, pastelpink);
    lerp(g.sun_outer, violet);
    lerp(g.sun_inner, indigo);
    lerp(g.sun_core, darkblue);
    return DT_OK;
  }
  // the tunnel (scene.h:776-781, 806-871): caps scaled x5 about their centre, pulled up by
  // the movement, rotated about +y, extruded 263 down; ads from the substitute frame list
  {
    const float dist = 263;
    a_cap0 = add(mul(5, sub(a_cap0, cap_center)), cap_center);
    b_cap0 = add(mul(5, sub(b_cap0, cap_center)), cap_center);
    c_cap0 = add(mul(5, sub(c_cap0, cap_center)), cap_center);
    a_cap0 = add(a_cap0, v3(0, g.tot_move, 0));
    b_cap0 = add(b_cap0, v3(0, g.tot_move, 0));
    c_cap0 = add(c_cap0, v3(0, g.tot_move, 0));
    const float rot_theta = (float)(movement_multiplier / 720.0 * M_PI);
    a_cap0 = add(rotate(sub(a_cap0, cap_center), v3(0, 1, 0), rot_theta), cap_center);
    b_cap0 = add(rotate(sub(b_cap0, cap_center), v3(0, 1, 0), rot_theta), cap_center);
    c_cap0 = add(rotate(sub(c_cap0, cap_center), v3(0, 1, 0), rot_theta), cap_center);
    const V3 a_cap1 = sub(a_cap0, v3(0, dist, 0)), b_cap1 = sub(b_cap0, v3(0, dist, 0)),
             c_cap1 = sub(c_cap0, v3(0, dist, 0));
    if (frame >= g.frame_prism)
      triangle_prism_mesh(O, g, a_cap0, b_cap0, c_cap0, a_cap1, b_cap1, c_cap1, (int)frame, true, true);
  }
  if ((min_y + g.tot_move <= eye.y + 2) || frame < g.frame_prism + tunnel_transition) {
    float angle = (float)(fminr(1.1f, movement_multiplier / (tunnel_transition)) * M_PI / 2);
    V3 B_left = add(rotate(sub(B, A), sub(D, A), angle), A);
    V3 C_left = add(rotate(sub(C, A), sub(D, A), angle), A);
    V3 B_right = add(rotate(sub(B, E), sub(F, E), -angle), E);
    V3 C_right = add(rotate(sub(C, E), sub(F, E), -angle), E);
    int tex = load_texture(O, data_dir, "sad_finder1_adj.jpg", err);
    if (tex < 0) return DT_E_IO;
    dt_shape_desc door1 = Rectangle(A, B_left, C_left, D, v3(0, 0, 0), "steel", false, tex, "cook-torrance");
    door1.roughness = 0.7f;
    door1.refr[0] = 2.75;
    door1.refr[1] = 3.79;
    door1.flags |= DT_F_GLOSSY | DT_F_TEXTURE;
    O.shapes.push_back(door1);
    tex = load_texture(O, data_dir, "sad_finder2_adj.jpg", err);
    if (tex < 0) return DT_E_IO;
    dt_shape_desc door2 = Rectangle(B_right, E, F, C_right, v3(0, 0, 0), "steel", false, tex, "cook-torrance");
    door2.roughness = 0.7f;
    door2.refr[0] = 2.75;
    door2.refr[1] = 3.79;
    door2.flags |= DT_F_GLOSSY | DT_F_TEXTURE;
    O.shapes.push_back(door2);
    tex = load_texture(O, data_dir, "floor.jpeg", err);
    if (tex < 0) return DT_E_IO;
    float s = 1;
    dt_shape_desc fl = CheckerboardWithHole(gA, gB, gC, gD, v3(0.58, 0.82, 1), v3(1, 0.416, 0.835), s, A, E, F, D);
    fl.tex_frame = tex;
    fl.borderwidth = 0.05f;
    set3(fl.bordercolor, v3(0.55, 0.55, 0.55));
    fl.flags |= DT_F_TEXTURE | DT_F_GLOSSY;
    fl.material = DT_MAT_LINOLEUM;
    fl.roughness = 0.6f;
    fl.refr[0] = 1.543;
    fl.refr[1] = 0;
    O.shapes.push_back(fl);
    V3 wall = v3(0, 0.81, 0.99);
    O.shapes.push_back(Rectangle(gA, gD, gH, gE, wall));
    O.shapes.push_back(Rectangle(gA, gB, gF, gE, wall));
    O.shapes.push_back(Rectangle(gD, gC, gG, gH, wall));
    // right wall with window (scene.h:931-981)
    V3 height_vector = normalized(sub(gF, gB));
    float height = (float)norm(sub(gF, gB));
    V3 length_vector = normalized(sub(gB, gC));
    float length = (float)norm(sub(gC, gB));
    V3 width_vector = normalized(sub(gB, gA));
    float width = 2;
    V3 gBp = add(gB, mul(width, width_vector)), gCp = add(gC, mul(width, width_vector));
    V3 gFp = add(gF, mul(width, width_vector)), gGp = add(gG, mul(width, width_vector));
    float window_size = 2;
    float mid_height = (height - window_size) / 2;
    float mid_length = (length - window_size) / 2;
    V3 a1 = add(gC, mul(mid_height, height_vector)), b1 = add(gB, mul(mid_height, height_vector));
    V3 c1 = add(gBp, mul(mid_height, height_vector)), d1 = add(gCp, mul(mid_height, height_vector));
    V3 am1 = add(a1, mul(mid_length, length_vector));
    V3 bm1 = add(am1, mul(window_size, length_vector));
    V3 cm1 = add(bm1, mul(width, width_vector));
    V3 dm1 = add(am1, mul(width, width_vector));
    V3 a2 = add(a1, mul(window_size, height_vector)), b2 = add(b1, mul(window_size, height_vector));
    V3 c2 = add(c1, mul(window_size, height_vector)), d2 = add(d1, mul(window_size, height_vector));
    V3 am2 = add(am1, mul(window_size, height_vector)), bm2 = add(bm1, mul(window_size, height_vector));
    V3 cm2 = add(cm1, mul(window_size, height_vector)), dm2 = add(dm1, mul(window_size, height_vector));
    V3 up3 = v3(0, 1e3, 0);
    O.shapes.push_back(RectPrismV2(gC, gB, gBp, gCp, add(a1, up3), add(b1, up3), add(c1, up3), add(d1, up3), wall));
    O.shapes.push_back(RectPrismV2(sub(a1, up3), sub(am1, up3), sub(dm1, up3), sub(d1, up3), a2, am2, dm2, d2, wall));
    O.shapes.push_back(RectPrismV2(sub(bm1, up3), sub(b1, up3), sub(c1, up3), sub(cm1, up3), bm2, b2, c2, cm2, wall));
    O.shapes.push_back(RectPrismV2(a2, b2, c2, d2, gG, gF, gFp, gGp, wall));
    V3 windowlight_c = add(divs(add(add(add(cm1, dm1), cm2), dm2), 4), v3(0, 0, 1));
    PointLight(O, windowlight_c, v3(1, 1, 1));
    // ceiling + 4 area lights (scene.h:987-1027)
    O.shapes.push_back(Rectangle(gE, gF, gG, gH, wall));
    int nlights = 4;
    V3 lightcol = v3(1, 1, 1);
    float lighth = (float)((gD.x - gA.x) / (nlights + (nlights + 2) / 2));
    float lightw = (float)((gB.z - gA.z) / (2 + 4.0 / 5));
    float wbound = lightw / 5;
    V3 cc = sub(divs(add(add(add(gE, gF), gG), gH), 4), v3(0, 0.05, 0));
    auto light_at = [&](V3 at) {
      RectangleLight(O, at, sub(at, mul(lighth, gEF)), sub(sub(at, mul(lighth, gEH)), mul(lighth, gEF)),
                     sub(at, mul(lighth, gEH)), lightcol);
    };
    light_at(sub(add(cc, mul(lighth + wbound, gEF)), mul(wbound, gAD)));
    light_at(sub(sub(cc, mul(wbound, gEF)), mul(wbound, gAD)));
    light_at(add(add(cc, mul(wbound + lighth, gEF)), mul(wbound + lighth, gAD)));
    light_at(add(sub(cc, mul(wbound, gEF)), mul(wbound + lighth, gAD)));
    // corner checker cylinder (scene.h:1030-1045)
    float l_prism = 2, w_prism = 3.0f / 4, h_prism = 1;
    float r = 4 * w_prism;
    V3 c_top = add(add(gH, mul(l_prism + r, gEH)), mul(w_prism, mul(1, gCD)));
    V3 c_bot = add(add(gD, mul(l_prism + r, gAD)), mul(w_prism, mul(1, gCD)));
    dt_shape_desc cyl = CheckerCylinder(c_top, c_bot, r, v3(1, 1, 1), s, "linoleum");
    cyl.tex_frame = tex;
    cyl.borderwidth = 0.05f;
    set3(cyl.bordercolor, v3(0.55, 0.55, 0.55));
    cyl.flags |= DT_F_TEXTURE | DT_F_GLOSSY;
    cyl.material = DT_MAT_LINOLEUM;
    cyl.roughness = 0.6f;
    cyl.refr[0] = 1.543;
    cyl.refr[1] = 0;
    O.shapes.push_back(cyl);
    // staircase (scene.h:1047-1088)
    V3 pink = v3(1, 0.44, 0.81);
    width_vector = normalized(v3(-1, 0, -0.8));
    length_vector = normalized(cross(v3(0, 1, 0), width_vector));
    height_vector = v3(0, 1, 0);
    V3 sd = add(mul(r, gAD), c_bot);
    V3 sa = add(sd, mul(w_prism, width_vector));
    V3 sb = add(sa, mul(l_prism, length_vector));
    V3 sc = add(sd, mul(l_prism, length_vector));
    V3 se = add(sa, mul(h_prism, height_vector)), sf = add(sb, mul(h_prism, height_vector));
    V3 sg = add(sc, mul(h_prism, height_vector)), sh = add(sd, mul(h_prism, height_vector));
    V3 tmp_center = c_bot;
    float theta = (float)acos(1 - pow(w_prism, 2) / pow(norm(sub(sa, tmp_center)), 2));
    int guard = 0;
    while (se.y <= 13 && dot(length_vector, gCD) > 0 && guard++ < 10000) {
      O.shapes.push_back(RectPrismV2(sa, sb, sc, sd, se, sf, sg, sh, pink));
      sa = add(add(rotate(sub(sa, tmp_center), height_vector, theta), tmp_center), mul(h_prism, height_vector));
      sb = add(add(rotate(sub(sb, tmp_center), height_vector, theta), tmp_center), mul(h_prism, height_vector));
      sc = add(add(rotate(sub(sc, tmp_center), height_vector, theta), tmp_center), mul(h_prism, height_vector));
      sd = add(add(rotate(sub(sd, tmp_center), height_vector, theta), tmp_center), mul(h_prism, height_vector));
      se = add(sa, mul(h_prism, height_vector));
      sf = add(sb, mul(h_prism, height_vector));
      sg = add(sc, mul(h_prism, height_vector));
      sh = add(sd, mul(h_prism, height_vector));
      tmp_center = add(tmp_center, height_vector);
      width_vector = normalized(sub(sa, sd));
      length_vector = normalized(sub(sb, sa));
      theta = (float)acos(1 - pow(w_prism, 2) / pow(norm(sub(sa, tmp_center)), 2));
    }
    if (g.use_model && frame < g.frame_prism) {   // scene.h:1095-1098 (substitute assets, F6)
      int rc = final_build_models(g, data_dir, O, err);
      if (rc) return rc;
    }
  }
  return DT_OK;
}

}  // namespace

extern "C" int dt_build_scene(const char* name, float frame, dt_globals* g, const char* data_dir, dt_scene_desc** out)
{
  if (!name || !g || !out) {
    dth::set_error("null argument");
    return DT_E_INVALID;
  }
  *out = nullptr;
  auto O = std::make_unique<OwnedDesc>();
  memset(&O->d, 0, sizeof(O->d));
  std::string err, dir = data_dir ? data_dir : "data";
  std::string n = name;
  int rc;
  if (n == "spheres") rc = build_spheres(frame, *g, *O);
  else if (n == "dof") rc = build_dof(frame, *g, *O);
  else if (n == "hw4") rc = build_hw4(frame, *g, *O);
  else if (n == "prismcyl") rc = build_prismcyl(frame, *g, *O);
  else if (n == "final") rc = build_final(frame, *g, dir, *O, err);
  else {
    err = "unknown scene " + n;
    rc = DT_E_INVALID;
  }
  if (rc) {
    dth::set_error(err.empty() ? "scene build failed" : err);
    return rc;
  }
  O->finish();
  *out = &O.release()->d;
  return DT_OK;
}

extern "C" void dt_scene_desc_free(dt_scene_desc* d)
{
  if (d) delete reinterpret_cast<OwnedDesc*>(d);
}

// the OBJ ingest as finalBuildModels sees it (load_obj above, objHelper.h:6-85): counts, then the
// vertices and texcoords as the floats tinyobj's real_t holds and 6 ints per triangle (vertex and
// texcoord indices, 0-based, texcoord -1 when absent). tests/test_oracle_obj.py compares it with
// the reference's own vendored tiny_obj_loader.h (oracle/ref/obj_parse.cpp).
extern "C" int dt_debug_load_obj(const char* path, float* v, int64_t cap_v, float* vt, int64_t cap_vt, int32_t* faces,
                                 int64_t cap_faces, int64_t counts[3])
{
  if (!path || !counts) {
    dth::set_error("null argument");
    return DT_E_INVALID;
  }
  ObjMesh m;
  std::string err;
  if (!load_obj(path, m, err)) {
    dth::set_error(err);
    return DT_E_IO;
  }
  const int64_t nv = (int64_t)m.v.size(), nt = (int64_t)m.vt.size() / 2, nf = (int64_t)m.vi.size() / 3;
  counts[0] = nv;
  counts[1] = nt;
  counts[2] = nf;
  if (v && cap_v >= nv)
    for (int64_t i = 0; i < nv; ++i) {
      v[3 * i] = (float)m.v[i].x;
      v[3 * i + 1] = (float)m.v[i].y;
      v[3 * i + 2] = (float)m.v[i].z;
    }
  if (vt && cap_vt >= nt)
    for (int64_t i = 0; i < 2 * nt; ++i) vt[i] = (float)m.vt[i];
  if (faces && cap_faces >= nf)
    for (int64_t f = 0; f < nf; ++f)
      for (int k = 0; k < 3; ++k) {
        faces[6 * f + k] = m.vi[3 * f + k];
        faces[6 * f + 3 + k] = m.ti[3 * f + k];
      }
  return DT_OK;
}
