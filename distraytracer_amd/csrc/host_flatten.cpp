// host_flatten.cpp — dt_scene_desc -> device layout, and per-render parameters.
//
// Every precomputed value is the exact IEEE result of the expression the reference
// evaluates on every call (cited per field), computed here once with the same operation
// order and no FMA contraction; the kernels therefore produce the same bits as if they
// recomputed it per ray.
#include <cfloat>
#include <cmath>
#include <cstring>

#include "host_internal.h"

using namespace dtm;
using dtd::DLight;
using dtd::DMat;
using dtd::DParams;
using dtd::DShapeHdr;

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

namespace dth {

namespace {

void put3(std::vector<double>& g, size_t at, V3 v)
{
  g[at] = v.x;
  g[at + 1] = v.y;
  g[at + 2] = v.z;
}

// Rectangle plane record (Rectangle::intersect, geometry.cpp:664-686)
void put_rect(std::vector<double>& g, size_t at, V3 A, V3 B, V3 C, V3 D)
{
  V3 n = normalized(normalized(cross(sub(B, A), sub(C, A))));  // getNorm(start).normalized()
  V3 V1 = sub(B, A), V2 = sub(D, A);
  put3(g, at + dtd::R_A, A);
  put3(g, at + dtd::R_N, n);
  put3(g, at + dtd::R_V1N, normalized(V1));
  put3(g, at + dtd::R_V2N, normalized(V2));
  g[at + dtd::R_LEN1] = norm(V1);
  g[at + dtd::R_LEN2] = norm(V2);
}

V3 VV(const dt_shape_desc& s, int k) { return v3a(s.v[k]); }

const int PRISM_FACES[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4}, {3, 0, 4, 7}, {1, 2, 6, 5}, {2, 3, 7, 6}};

}  // namespace

int flatten_scene(const dt_scene_desc& d, const dt_globals& g, FlatScene& out, std::string& err)
{
  out = FlatScene();
  if (d.n_shapes < 0 || d.n_lights < 0 || d.n_textures < 0 || (d.n_shapes > 0 && !d.shapes) ||
      (d.n_lights > 0 && !d.lights) || (d.n_textures > 0 && !d.textures)) {
    err = "invalid scene descriptor";
    return DT_E_INVALID;
  }
  if (d.n_holes < 0 || (d.n_holes > 0 && !d.holes)) {
    err = "invalid hole array";
    return DT_E_INVALID;
  }
  if (d.n_lights > 32) {   // the device keeps one visibility bit per light in a 32-bit mask
    err = "more than 32 lights";
    return DT_E_LIMIT;
  }
  // textures
  std::vector<int64_t> tex_off(d.n_textures);
  for (int i = 0; i < d.n_textures; ++i) {
    const dt_texture_desc& t = d.textures[i];
    if (t.width <= 0 || t.height <= 0 || t.channels < 3 || !t.pixels) {
      err = "invalid texture " + std::to_string(i);
      return DT_E_INVALID;
    }
    tex_off[i] = (int64_t)out.tex.size();
    out.tex.insert(out.tex.end(), t.pixels, t.pixels + (size_t)t.width * t.height * t.channels);
  }
  if (out.tex.empty()) out.tex.push_back(0);

  out.hdr.resize(d.n_shapes);
  out.mat.resize(d.n_shapes);
  for (int i = 0; i < d.n_shapes; ++i) {
    const dt_shape_desc& s = d.shapes[i];
    DShapeHdr& h = out.hdr[i];
    h.type = s.type;
    h.flags = s.flags;
    h._pad = 0;
    size_t at = out.geom.size();
    h.off = (int32_t)at;
    std::vector<double>& G = out.geom;
    switch (s.type) {
      case DT_SHAPE_SPHERE:
        G.resize(at + dtd::SP_SIZE);
        put3(G, at + dtd::SP_C, VV(s, 0));
        G[at + dtd::SP_R2] = pow((double)s.radius, 2.0);  // pow(radius, 2) (geometry.cpp:110)
        break;
      case DT_SHAPE_CYLINDER:
      case DT_SHAPE_CHECKER_CYLINDER: {
        G.resize(at + dtd::CY_SIZE, 0.0);
        V3 c1 = VV(s, 0), c2 = VV(s, 1);
        V3 axis = normalized(sub(c2, c1));  // Cylinder ctor (geometry.cpp:231)
        put3(G, at + dtd::CY_C1, c1);
        put3(G, at + dtd::CY_C2, c2);
        put3(G, at + dtd::CY_AX, axis);
        G[at + dtd::CY_R2] = pow((double)s.radius, 2.0);
        // CheckerCylinder objM = buildCOB(axis) * origin (geometry.cpp:27-41, 2579-2586)
        V3 w = normalized(axis);
        V3 u = normalized(cross(v3(1, 0, 0), w));
        if (is_approx_zero(u)) u = normalized(cross(v3(0, 1, 0), w));
        V3 v = normalized(cross(w, u));
        double cob[4][4] = {{u.x, u.y, u.z, 0}, {v.x, v.y, v.z, 0}, {w.x, w.y, w.z, 0}, {0, 0, 0, 1}};
        double org[4][4] = {{1, 0, 0, -c1.x}, {0, 1, 0, -c1.y}, {0, 0, 1, -c1.z}, {0, 0, 0, 1}};
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 4; ++c) {
            double acc = cob[r][0] * org[0][c];
            for (int k = 1; k < 4; ++k) acc = acc + cob[r][k] * org[k][c];
            G[at + dtd::CY_M + r * 4 + c] = acc;
          }
        G[at + dtd::CY_NAX] = norm(axis);
        float mud = (float)(s.S / (2 * M_PI * s.radius));   // geometry.cpp:2604
        float mvd = (float)(s.S / norm(axis));              // 2605
        float bw = s.borderwidth / (2 * s.S);                // 2617
        G[at + dtd::CY_MUD] = mud;
        G[at + dtd::CY_MVD] = mvd;
        G[at + dtd::CY_BW] = bw;
        break;
      }
      case DT_SHAPE_TRIANGLE: {
        G.resize(at + dtd::TR_SIZE);
        V3 A = VV(s, 0), B = VV(s, 1), C = VV(s, 2);
        put3(G, at + dtd::TR_A, A);
        put3(G, at + dtd::TR_B, B);
        put3(G, at + dtd::TR_C, C);
        put3(G, at + dtd::TR_R1, sub(B, A));
        put3(G, at + dtd::TR_R2, sub(C, A));
        put3(G, at + dtd::TR_MN, v3a(s.mesh_normal));
        for (int k = 0; k < 3; ++k) {
          G[at + dtd::TR_UV + 2 * k] = s.uv[k][0];
          G[at + dtd::TR_UV + 2 * k + 1] = s.uv[k][1];
        }
        break;
      }
      case DT_SHAPE_RECTANGLE: {
        G.resize(at + dtd::RC_SIZE);
        V3 A = VV(s, 0), B = VV(s, 1), C = VV(s, 2), D = VV(s, 3);
        put_rect(G, at + dtd::RC_R, A, B, C, D);
        put3(G, at + dtd::RC_A, A);
        put3(G, at + dtd::RC_B, B);
        put3(G, at + dtd::RC_C, C);
        put3(G, at + dtd::RC_D, D);
        V3 ad = sub(D, A), dc = sub(C, D);  // Rectangle::getUV (geometry.cpp:751-759)
        put3(G, at + dtd::RC_AD, ad);
        put3(G, at + dtd::RC_DC, dc);
        G[at + dtd::RC_NADC] = norm(ad) * norm(dc);
        break;
      }
      case DT_SHAPE_RECTPRISM_V2: {
        G.resize(at + dtd::PR_SIZE);
        for (int f = 0; f < 6; ++f) {
          const int* q = PRISM_FACES[f];
          put_rect(G, at + dtd::PR_F + f * dtd::R_SIZE, VV(s, q[0]), VV(s, q[1]), VV(s, q[2]), VV(s, q[3]));
        }
        V3 A = VV(s, 0), B = VV(s, 1), C = VV(s, 2), D = VV(s, 3), E = VV(s, 4), F = VV(s, 5), Gv = VV(s, 6),
           H = VV(s, 7);
        // RectPrismV2::getNorm (geometry.cpp:866-868)
        put3(G, at + dtd::PR_NBOT, neg(normalized(cross(sub(F, E), sub(H, E)))));
        put3(G, at + dtd::PR_NRIGHT, normalized(cross(sub(E, A), sub(D, A))));
        put3(G, at + dtd::PR_NFRONT, normalized(cross(sub(B, A), sub(E, A))));
        put3(G, at + dtd::PR_A, A);
        put3(G, at + dtd::PR_G, Gv);
        V3 ad = sub(D, A), dc = sub(C, D);  // faces[0]->getUV
        put3(G, at + dtd::PR_AD, ad);
        put3(G, at + dtd::PR_DC, dc);
        G[at + dtd::PR_NADC] = norm(ad) * norm(dc);
        put3(G, at + dtd::PR_D, D);
        break;
      }
      case DT_SHAPE_RECTPRISM_CYL: {
        // RectPrismWithCylinder (geometry.cpp:1467-1505) and its holes (Cylinder ctor, 227-240)
        if (s.n_holes < 0 || (s.n_holes > 0 && (!d.holes || s.hole_first < 0 || s.hole_first + s.n_holes > d.n_holes))) {
          err = "shape " + std::to_string(i) + ": hole range out of the descriptor's holes";
          return DT_E_INVALID;
        }
        G.resize(at + dtd::RP_H + (size_t)s.n_holes * dtd::RH_SIZE, 0.0);
        V3 lb, ub;
        shape_bounds(s, lb, ub);   // RectPrism::getBounds (1382-1401), the box intersect tests
        put3(G, at + dtd::RP_LB, lb);
        put3(G, at + dtd::RP_UB, ub);
        V3 A = VV(s, 0), B = VV(s, 1), C = VV(s, 2), D = VV(s, 3), E = VV(s, 4), F = VV(s, 5), H = VV(s, 7);
        // getNorm (1802-1804)
        put3(G, at + dtd::RP_NBOT, neg(normalized(cross(sub(F, E), sub(H, E)))));
        put3(G, at + dtd::RP_NRIGHT, normalized(cross(sub(E, A), sub(D, A))));
        put3(G, at + dtd::RP_NFRONT, normalized(cross(sub(B, A), sub(E, A))));
        put3(G, at + dtd::RP_A, A);
        V3 ad = sub(D, A), dc = sub(C, D);   // RectPrism::getUV (1445-1453)
        put3(G, at + dtd::RP_AD, ad);
        put3(G, at + dtd::RP_DC, dc);
        put3(G, at + dtd::RP_ADC, cross(ad, dc));
        G[at + dtd::RP_NADC] = norm(ad) * norm(dc);
        put3(G, at + dtd::RP_D, D);
        G[at + dtd::RP_NH] = s.n_holes;
        for (int k = 0; k < s.n_holes; ++k) {
          const dt_shape_desc& hs = d.holes[s.hole_first + k];
          const size_t o = at + dtd::RP_H + (size_t)k * dtd::RH_SIZE;
          V3 c1 = VV(hs, 0), c2 = VV(hs, 1);
          V3 axis = normalized(sub(c2, c1));
          put3(G, o + dtd::RH_C1, c1);
          put3(G, o + dtd::RH_C2, c2);
          put3(G, o + dtd::RH_AX, axis);
          G[o + dtd::RH_R2] = pow((double)hs.radius, 2.0);   // pow(radius, 2) (250)
          put3(G, o + dtd::RH_COL, v3a(hs.color));
          G[o + dtd::RH_C1A] = dot(c1, axis);   // c1.dot(axis) of intersectCap (307)
          G[o + dtd::RH_C2A] = dot(c2, axis);   // c2.dot(axis) (308)
        }
        break;
      }
      case DT_SHAPE_CHECKERBOARD:
      case DT_SHAPE_CHECKERBOARD_HOLE: {
        G.resize(at + dtd::CK_SIZE, 0.0);
        V3 A = VV(s, 0), B = VV(s, 1), C = VV(s, 2), D = VV(s, 3);
        put_rect(G, at + dtd::CK_R, A, B, C, D);
        put3(G, at + dtd::CK_GN, normalized(cross(sub(B, A), sub(C, A))));  // getNorm (edge test, 2274)
        put3(G, at + dtd::CK_A, A);
        put3(G, at + dtd::CK_B, B);
        put3(G, at + dtd::CK_C, C);
        put3(G, at + dtd::CK_D, D);
        if (s.type == DT_SHAPE_CHECKERBOARD_HOLE)
          put_rect(G, at + dtd::CK_HOLE, VV(s, 4), VV(s, 5), VV(s, 6), VV(s, 7));
        G[at + dtd::CK_S] = s.S;
        put3(G, at + dtd::CK_COL1, v3a(s.color1));
        put3(G, at + dtd::CK_COL2, v3a(s.color2));
        put3(G, at + dtd::CK_COL, v3a(s.color));
        V3 ad = sub(D, A), dc = sub(C, D);   // CheckerboardWithHole::getUV (2518-2521)
        put3(G, at + dtd::CK_AD, ad);
        put3(G, at + dtd::CK_DC, dc);
        G[at + dtd::CK_NADC] = norm(ad) * norm(dc);
        G[at + dtd::CK_MUD] = (float)(s.S / s.length);   // 2525
        G[at + dtd::CK_MVD] = (float)(s.S / s.width);    // 2526
        G[at + dtd::CK_BW] = (float)(s.borderwidth / (2 * s.S));
        break;
      }
      default:
        err = "shape " + std::to_string(i) + ": unsupported type " + std::to_string(s.type);
        return DT_E_UNSUPPORTED;
    }
    DMat& m = out.mat[i];
    memset(&m, 0, sizeof(m));
    m.model = s.model;
    m.material = s.material;
    m.emit = s.emit;
    m.flags = s.flags;
    m.tex = -1;
    if (s.flags & DT_F_TEXTURE) {
      if (s.tex_frame < 0 || s.tex_frame >= d.n_textures) {
        if (s.type == DT_SHAPE_RECTANGLE || s.type == DT_SHAPE_RECTPRISM_V2 || s.type == DT_SHAPE_TRIANGLE ||
            s.type == DT_SHAPE_CHECKERBOARD_HOLE || s.type == DT_SHAPE_CHECKER_CYLINDER ||
            s.type == DT_SHAPE_RECTPRISM_CYL) {
          err = "shape " + std::to_string(i) + ": texture index out of range";
          return DT_E_INVALID;
        }
      } else {
        const dt_texture_desc& t = d.textures[s.tex_frame];
        m.tex = s.tex_frame;
        m.tex_w = t.width;
        m.tex_h = t.height;
        m.tex_ch = t.channels;
        m.tex_off = tex_off[s.tex_frame];
      }
    }
    m.roughness = s.roughness;
    m.radius = s.radius;
    m.refr[0] = s.refr[0];
    m.refr[1] = s.refr[1];
    {
      const double r0 = m.refr[0], r1 = m.refr[1], rr = (double)m.roughness;
      m.ct_r0 = (float)(((r0 - 1) * (r0 - 1) + r1 * r1) / ((r0 + 1) * (r0 + 1) + r1 * r1));
      m.on_a = (float)(1.0 - (0.5 * (rr * rr)) / ((rr * rr) + 0.33));
      m.on_b = (float)((0.45 * (rr * rr)) / ((rr * rr) + 0.09));
      m._pad_m = 0;
    }
    for (int k = 0; k < 3; ++k) {
      m.color[k] = s.color[k];
      m.bordercolor[k] = s.bordercolor[k];
      m.center[k] = s.center[k];
    }
  }
  out.lights.resize(d.n_lights);
  for (int i = 0; i < d.n_lights; ++i) {
    const dt_light_desc& L = d.lights[i];
    DLight& o = out.lights[i];
    memset(&o, 0, sizeof(o));
    if (L.type != DT_LIGHT_POINT && L.type != DT_LIGHT_RECT && L.type != DT_LIGHT_SPHERE) {
      err = "light " + std::to_string(i) + ": unsupported type";
      return DT_E_UNSUPPORTED;
    }
    if (L.shape_index >= d.n_shapes) {
      err = "light " + std::to_string(i) + ": shape index out of range";
      return DT_E_INVALID;
    }
    o.type = L.type;
    o.shape_index = L.shape_index;
    o.use_baxis = !is_approx_zero(v3a(L.baxis));
    o.radius = L.radius;
    for (int k = 0; k < 3; ++k) {
      o.center[k] = L.center[k];
      o.color[k] = L.color[k];
      o.baxis[k] = L.baxis[k];
      o.A[k] = L.A[k];
      o.B[k] = L.B[k];
      o.D[k] = L.D[k];
    }
  }
  build_bvh(d, g, out.bvh);
  return DT_OK;
}

std::vector<float> cloud_z_steps(const dt_globals& g)
{
  std::vector<float> z;
  for (float v = g.clouddist; v > 0; v -= 0.05) {   // cpp:172 (float loop variable)
    z.push_back(v);
    if (z.size() > 1000000) break;
  }
  return z;
}

namespace {

void mat4_mul(const double A[4][4], const double B[4][4], double R[4][4])
{
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = A[i][0] * B[0][j];
      for (int k = 1; k < 4; ++k) s = s + A[i][k] * B[k][j];
      R[i][j] = s;
    }
}

int fill_tiles(const dt_globals& g, const dt_tiles* T, DParams& P, std::string& err)
{
  dt_tiles t;
  if (T) t = *T;
  else memset(&t, 0, sizeof(t));
  P.x0 = t.x0 < 0 ? 0 : t.x0;
  P.y0 = t.y0 < 0 ? 0 : t.y0;
  P.x1 = t.x1 > 0 ? (t.x1 < g.xRes ? t.x1 : g.xRes) : g.xRes;
  P.y1 = t.y1 > 0 ? (t.y1 < g.yRes ? t.y1 : g.yRes) : g.yRes;
  if (P.x1 <= P.x0 || P.y1 <= P.y0) {
    err = "empty pixel window";
    return DT_E_INVALID;
  }
  P.tw = t.tile_w > 0 ? t.tile_w : 32;
  P.th = t.tile_h > 0 ? t.tile_h : 32;
  P.world = t.world > 0 ? t.world : 1;
  P.rank = t.rank;
  if (P.rank < 0 || P.rank >= P.world) {
    err = "rank out of range";
    return DT_E_INVALID;
  }
  P.layout = t.layout;
  P.tiles_x = (P.x1 - P.x0 + P.tw - 1) / P.tw;
  int64_t tiles_y = (P.y1 - P.y0 + P.th - 1) / P.th;
  int64_t n_tiles = (int64_t)P.tiles_x * tiles_y;
  P.n_tiles = n_tiles;
  P.n_owned_tiles = (n_tiles + P.world - 1) / P.world;   // slots (dtd::tile_of): equal for every rank
  return DT_OK;
}

void camera(V3 eye, V3 lookingAt, V3 up, V3& X, V3& Y, V3& Z, bool& degenerate)
{
  Z = neg(normalized(sub(lookingAt, eye)));  // cpp:990
  X = normalized(cross(up, Z));               // 992
  degenerate = is_approx_zero(X);
  Y = normalized(cross(Z, X));                // 998
}

void near_plane(const dt_globals& g, DParams& P)
{
  P.t = (float)(tan(g.fov * M_PI / 360.0) * fabsf(g.near_plane));   // cpp:1024-1027
  P.b = -P.t;
  P.r = g.aspect * P.t;
  P.l = -P.r;
}

void common(const dt_globals& g, DParams& P)
{
  P.xRes = g.xRes;
  P.yRes = g.yRes;
  P.near_plane = g.near_plane;
  P.saturation = g.saturation;
  P.cloudhoff = g.cloudhoff;
  V3 sun = normalized(v3a(g.sundir));   // cpp:152
  for (int k = 0; k < 3; ++k) {
    P.sun[k] = (&sun.x)[k];
    P.sun_outer[k] = g.sun_outer[k];
    P.sun_inner[k] = g.sun_inner[k];
    P.sun_core[k] = g.sun_core[k];
    P.bluesky[k] = g.bluesky[k];
    P.redsky[k] = g.redsky[k];
    P.default_col[k] = g.default_col[k];
  }
  P.n_cloud_steps = (int32_t)cloud_z_steps(g).size();
}

}  // namespace

int fill_params(const dt_globals& g, int frame, const dt_tiles* tiles, DParams& P, std::string& err)
{
  memset(&P, 0, sizeof(P));
  for (int l = 0; l < DT_MAX_SGRID; ++l) P.sgb_base[l] = -1;   // no block subtrees (the scene sets them)
  P.sgb_bz = 1;
  if (g.xRes <= 0 || g.yRes <= 0 || g.antialias_samples < 1 || g.max_depth < 0 || g.brdf_samples < 0 ||
      g.blur_samples < 0) {
    err = "invalid globals";
    return DT_E_INVALID;
  }
  common(g, P);
  int rc = fill_tiles(g, tiles, P, err);
  if (rc) return rc;
  int n = (int)sqrt((double)g.antialias_samples);
  P.spp = (int)pow(n, 2);
  P.ppw = P.spp <= 64 ? 64 / P.spp : 1;
  P.chunks = (P.spp + 63) / 64;
  int64_t owned_px = P.n_owned_tiles * P.tw * P.th;
  P.n_items = (owned_px + P.ppw - 1) / P.ppw;
  P.max_depth = g.max_depth;
  P.brdf_samples = g.brdf_samples;
  P.blur_samples = g.blur_samples;
  P.frame_range = g.frame_range;
  P.frame = frame;
  P.frame_prism = g.frame_prism;
  P.frame_blur = g.frame_blur;
  P.frame_cloud = g.frame_cloud;
  P.reflect = g.reflect;
  P.nogloss = g.nogloss;
  P.perlin_cloud = g.perlin_cloud;
  P.seed = g.seed;
  P.aperture = g.aperture;
  P.focal_length = g.focal_length;
  P.refr_air = g.refr_air;
  P.refr_glass = g.refr_glass;
  P.phong = g.phong;
  P.move_per_frame = g.move_per_frame;
  P.accel_t = g.accel_t;
  P.frame_f = (float)frame;
  V3 X, Y, Z;
  bool degenerate;
  camera(v3a(g.eye), v3a(g.lookingAt), v3a(g.up), X, Y, Z, degenerate);
  if (degenerate) {
    err = "Gaze direction can't be equal to up vector";   // cpp:993-996
    return DT_E_INVALID;
  }
  V3 E = v3a(g.eye);
  for (int k = 0; k < 3; ++k) {
    P.eye[k] = (&E.x)[k];
    P.X[k] = (&X.x)[k];
    P.Y[k] = (&Y.x)[k];
    P.Z[k] = (&Z.x)[k];
  }
  near_plane(g, P);
  // mcam / new_mcam (cpp:1004-1021)
  V3 RX = X, RY = Y;
  if (frame >= g.frame_cloud) {
    V3 new_up = v3(-1, 0, 0);
    RX = normalized(cross(new_up, Z));
    RY = normalized(cross(Z, RX));
  }
  double cob[4][4] = {{RX.x, RX.y, RX.z, 0}, {RY.x, RY.y, RY.z, 0}, {Z.x, Z.y, Z.z, 0}, {0, 0, 0, 1}};
  double org[4][4] = {{1, 0, 0, -E.x}, {0, 1, 0, -E.y}, {0, 0, 1, -E.z}, {0, 0, 0, 1}};
  double M[4][4];
  mat4_mul(cob, org, M);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) P.sky_m[r][c] = M[r][c];
  return DT_OK;
}

int fill_sky_params(const dt_globals& g0, float frame, const dt_tiles* tiles, DParams& P, std::string& err)
{
  memset(&P, 0, sizeof(P));
  dt_globals g = g0;
  if (g.xRes <= 0 || g.yRes <= 0) {
    err = "invalid globals";
    return DT_E_INVALID;
  }
  // renderImageCloud overrides the camera (cpp:1227-1229)
  g.eye[0] = 0.5; g.eye[1] = 1.5; g.eye[2] = 1;
  g.up[0] = 0; g.up[1] = 0; g.up[2] = 1;
  g.lookingAt[0] = 0.5; g.lookingAt[1] = -1; g.lookingAt[2] = 1;
  common(g, P);
  int rc = fill_tiles(g, tiles, P, err);
  if (rc) return rc;
  P.frame_f = frame;
  V3 X, Y, Z;
  bool degenerate;
  camera(v3a(g.eye), v3a(g.lookingAt), v3a(g.up), X, Y, Z, degenerate);
  if (degenerate) {
    err = "Gaze direction can't be equal to up vector";
    return DT_E_INVALID;
  }
  V3 E = v3a(g.eye);
  for (int k = 0; k < 3; ++k) {
    P.eye[k] = (&E.x)[k];
    P.X[k] = (&X.x)[k];
    P.Y[k] = (&Y.x)[k];
    P.Z[k] = (&Z.x)[k];
  }
  near_plane(g, P);
  // cob rows X, Y, -Z (cpp:1262-1263)
  double cob[4][4] = {{X.x, X.y, X.z, 0}, {Y.x, Y.y, Y.z, 0}, {-Z.x, -Z.y, -Z.z, 0}, {0, 0, 0, 1}};
  double org[4][4] = {{1, 0, 0, -E.x}, {0, 1, 0, -E.y}, {0, 0, 1, -E.z}, {0, 0, 0, 1}};
  double M[4][4];
  mat4_mul(cob, org, M);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) P.sky_m[r][c] = M[r][c];
  P.spp = 1;
  P.ppw = 1;
  P.chunks = 1;
  P.n_items = P.n_owned_tiles * P.tw * P.th;
  return DT_OK;
}

}  // namespace dth
