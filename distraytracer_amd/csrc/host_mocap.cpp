// host_mocap.cpp — CMU ASF/AMC skeleton + forward kinematics that produce buildFinal's 30
// bone cylinders (scene.h:617-659). Host-side scene input generation,
// restating skeleton.cpp (ASF parse, RotateBoneDirToLocalCoordSystem,
// ComputeRotationToParentCoordSystem), motion.cpp (readAMCfile) and displaySkeleton.cpp
// (software GL matrix stack: DrawBone/Traverse/ComputeBonePositions), including their
// float casts. Eigen semantics: 4x4 products sum over k sequentially; AngleAxis is
// Eigen's toRotationMatrix formula.
//
// The reference's mocap files are inputs that do not exist on the GPU box, so
// tools/gen_bones.py runs this once here and commits the endpoints of the frames buildFinal
// uses (data/bones_90_16_v3.bin); dt_build_scene("final") reads that table.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <array>
#include <stack>
#include <string>
#include <vector>

#include "host_internal.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

namespace {

typedef double M4[4][4];

void ident(M4 m)
{
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) m[i][j] = i == j ? 1.0 : 0.0;
}
void mmul(const M4 A, const M4 B, M4 R)
{
  M4 T;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = A[i][0] * B[0][j];
      for (int k = 1; k < 4; ++k) s = s + A[i][k] * B[k][j];
      T[i][j] = s;
    }
  memcpy(R, T, sizeof(T));
}
// skeleton.cpp:16-53 (float angle; cosf/sinf)
void rotX(float theta, M4 R)
{
  memset(R, 0, sizeof(M4));
  R[0][0] = R[3][3] = 1;
  float c = cosf(theta), s = sinf(theta);
  R[1][1] = R[2][2] = c;
  R[1][2] = -s;
  R[2][1] = s;
}
void rotY(float theta, M4 R)
{
  memset(R, 0, sizeof(M4));
  R[1][1] = R[3][3] = 1;
  float c = cosf(theta), s = sinf(theta);
  R[0][0] = R[2][2] = c;
  R[0][2] = s;
  R[2][0] = -s;
}
void rotZ(float theta, M4 R)
{
  memset(R, 0, sizeof(M4));
  R[2][2] = R[3][3] = 1;
  float c = cosf(theta), s = sinf(theta);
  R[0][0] = R[1][1] = c;
  R[0][1] = -s;
  R[1][0] = s;
}
// Eigen AngleAxis<double>::toRotationMatrix, then transposeInPlace, into a 4x4
void angle_axis_T(double angle, const double ax[3], M4 out)
{
  double sa[3], c1a[3];
  double sn = sin(angle), c = cos(angle);
  for (int k = 0; k < 3; ++k) {
    sa[k] = sn * ax[k];
    c1a[k] = (1.0 - c) * ax[k];
  }
  double r[3][3];
  double tmp = c1a[0] * ax[1];
  r[0][1] = tmp - sa[2];
  r[1][0] = tmp + sa[2];
  tmp = c1a[0] * ax[2];
  r[0][2] = tmp + sa[1];
  r[2][0] = tmp - sa[1];
  tmp = c1a[1] * ax[2];
  r[1][2] = tmp - sa[0];
  r[2][1] = tmp + sa[0];
  for (int k = 0; k < 3; ++k) r[k][k] = c1a[k] * ax[k] + c;
  ident(out);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) out[i][j] = r[j][i];   // transposeInPlace + toMatrix4
}
void normalize3(double a[3])
{
  double n = (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2];
  if (n > 0) {
    double s = sqrt(n);
    a[0] /= s;
    a[1] /= s;
    a[2] /= s;
  }
}

struct Bone {
  int sibling = -1, child = -1;
  int idx = 0;
  double dir[3] = {0, 0, 0};
  double length = 0;
  double axis_x = 0, axis_y = 0, axis_z = 0;
  double aspx = 1, aspy = 1;
  int dof = 0;
  int dofrx = 0, dofry = 0, dofrz = 0, doftx = 0, dofty = 0, doftz = 0, doftl = 0;
  char name[256] = {0};
  double rpc[4][4];   // rot_parent_current
  double rx = 0, ry = 0, rz = 0, tx = 0, ty = 0, tz = 0, tl = 0;
  int dofo[8] = {0};
};

struct Skeleton {
  std::vector<Bone> b;
  int nbones = 1;

  int name2idx(const char* n) const
  {
    for (int i = 0; i < nbones; ++i)
      if (strcmp(b[i].name, n) == 0) return b[i].idx;
    return -1;
  }
  int num_in(int bone) const   // numBonesInSkel (skeleton.cpp:56-72)
  {
    int tmp = b[bone].sibling, n = 0;
    while (tmp >= 0) {
      if (b[tmp].child >= 0) n += num_in(b[tmp].child);
      n++;
      tmp = b[tmp].sibling;
    }
    if (b[bone].child >= 0) return n + 1 + num_in(b[bone].child);
    return n + 1;
  }
  int mov_in(int bone) const   // movBonesInSkel (80-101)
  {
    int tmp = b[bone].sibling, n = 0;
    if (b[bone].dof > 0) n++;
    while (tmp >= 0) {
      if (b[tmp].child >= 0) n += mov_in(b[tmp].child);
      if (b[tmp].dof > 0) n++;
      tmp = b[tmp].sibling;
    }
    if (b[bone].child >= 0) return n + mov_in(b[bone].child);
    return n;
  }
  void set_child(int parent, int child)   // setChildrenAndSibling
  {
    if (b[parent].child < 0) {
      b[parent].child = child;
    } else {
      int p = b[parent].child;
      while (b[p].sibling >= 0) p = b[p].sibling;
      b[p].sibling = child;
    }
  }
};

bool read_asf(const std::string& path, double scale, Skeleton& S, std::string& err)
{
  std::ifstream is(path);
  if (!is) {
    err = "cannot open " + path;
    return false;
  }
  S.b.assign(256, Bone());
  Bone& root = S.b[0];
  strcpy(root.name, "root");
  int o[7] = {4, 5, 6, 1, 2, 3, 0};
  memcpy(root.dofo, o, sizeof(o));
  root.idx = 0;
  root.length = 0.05;
  root.dof = 6;
  root.dofrx = root.dofry = root.dofrz = root.doftx = root.dofty = root.doftz = 1;
  S.nbones = 1;
  std::string line;
  auto kw = [](const std::string& l) {
    std::istringstream ss(l);
    std::string k;
    ss >> k;
    return k;
  };
  while (std::getline(is, line))
    if (kw(line) == ":bonedata") break;
  std::getline(is, line);   // begin
  bool done = false;
  for (int i = 1; !done && i < 256; ++i) {
    Bone& B = S.b[i];
    S.nbones++;
    double length = 0;
    while (std::getline(is, line)) {
      if (!line.empty() && line.back() == '\r') line.pop_back();
      std::string k = kw(line);
      if (k == "end") break;
      if (k == ":hierarchy") {
        S.nbones--;
        done = true;
        break;
      }
      std::istringstream ss(line);
      std::string t;
      ss >> t;
      if (k == "id") B.idx = S.nbones - 1;
      if (k == "name") ss >> B.name;
      if (k == "direction") ss >> B.dir[0] >> B.dir[1] >> B.dir[2];
      if (k == "length") ss >> length;
      if (k == "axis") ss >> B.axis_x >> B.axis_y >> B.axis_z;
      if (k == "dof") {
        std::string tok;
        while (ss >> tok) {
          int d = B.dof;
          if (tok == "rx") { B.dofrx = 1; B.dofo[d] = 1; }
          else if (tok == "ry") { B.dofry = 1; B.dofo[d] = 2; }
          else if (tok == "rz") { B.dofrz = 1; B.dofo[d] = 3; }
          else if (tok == "tx") { B.doftx = 1; B.dofo[d] = 4; }
          else if (tok == "ty") { B.dofty = 1; B.dofo[d] = 5; }
          else if (tok == "tz") { B.doftz = 1; B.dofo[d] = 6; }
          else if (tok == "l") { B.doftl = 1; B.dofo[d] = 7; }
          else continue;
          B.dof++;
          B.dofo[B.dof] = 0;
        }
      }
    }
    if (!done) B.length = length * scale;
  }
  // hierarchy
  std::getline(is, line);   // begin
  while (std::getline(is, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (kw(line) == "end") break;
    std::istringstream ss(line);
    std::string part;
    int j = 0, parent = 0;
    while (ss >> part) {
      if (j == 0) parent = S.name2idx(part.c_str());
      else S.set_child(parent, S.name2idx(part.c_str()));
      j++;
    }
  }
  // RotateBoneDirToLocalCoordSystem (skeleton.cpp:412-433)
  for (int i = 1; i < S.nbones; ++i) {
    Bone& B = S.b[i];
    M4 Rz, Ry, Rx, T1, T2;
    rotZ((float)(-B.axis_z * M_PI / 180.0), Rz);
    rotY((float)(-B.axis_y * M_PI / 180.0), Ry);
    rotX((float)(-B.axis_x * M_PI / 180.0), Rx);
    mmul(Rx, Ry, T1);
    mmul(T1, Rz, T2);
    double d4[4] = {B.dir[0], B.dir[1], B.dir[2], 1}, r[4];
    for (int q = 0; q < 4; ++q) {
      double s = T2[q][0] * d4[0];
      for (int k = 1; k < 4; ++k) s = s + T2[q][k] * d4[k];
      r[q] = s;
    }
    B.dir[0] = r[0];
    B.dir[1] = r[1];
    B.dir[2] = r[2];
  }
  // ComputeRotationToParentCoordSystem (skeleton.cpp:366-405)
  {
    M4 Rz, Ry, Rx, T1, T2;
    rotZ((float)(S.b[0].axis_z * M_PI / 180.0), Rz);
    rotY((float)(S.b[0].axis_y * M_PI / 180.0), Ry);
    rotX((float)(S.b[0].axis_x * M_PI / 180.0), Rx);
    mmul(Rz, Ry, T1);
    mmul(T1, Rx, T2);
    for (int x = 0; x < 4; ++x)
      for (int y = 0; y < 4; ++y) S.b[0].rpc[x][y] = T2[y][x];
  }
  auto rel = [&](int parent, int child) {
    const Bone& P = S.b[parent];
    Bone& C = S.b[child];
    M4 Rz, Ry, Rx, A1, tmp1, tmp2, tmp;
    rotZ((float)(-P.axis_z * M_PI / 180.0), Rz);
    rotY((float)(-P.axis_y * M_PI / 180.0), Ry);
    rotX((float)(-P.axis_x * M_PI / 180.0), Rx);
    mmul(Rx, Ry, A1);
    mmul(A1, Rz, tmp1);
    rotZ((float)(C.axis_z * M_PI / 180.0), Rz);
    rotY((float)(C.axis_y * M_PI / 180.0), Ry);
    rotX((float)(C.axis_x * M_PI / 180.0), Rx);
    mmul(Rz, Ry, A1);
    mmul(A1, Rx, tmp2);
    mmul(tmp1, tmp2, tmp);
    for (int x = 0; x < 4; ++x)
      for (int y = 0; y < 4; ++y) C.rpc[x][y] = tmp[y][x];
  };
  int numbones = S.num_in(0);
  for (int i = 0; i < numbones; ++i) {
    if (S.b[i].child >= 0) {
      rel(i, S.b[i].child);
      int tmp = S.b[S.b[i].child].sibling;
      while (tmp >= 0) {
        rel(i, tmp);
        tmp = S.b[tmp].sibling;
      }
    }
  }
  // set_bone_shape
  S.b[0].aspx = S.b[0].aspy = 1;
  for (int j = 1; j < numbones; ++j) S.b[j].aspx = S.b[j].aspy = 0.25;
  return true;
}

struct Posture {
  double rot[256][3];
  double trans[256][3];
  double len[256];
};

bool read_amc(const std::string& path, double scale, const Skeleton& S, std::vector<Posture>& post, std::string& err)
{
  std::ifstream f(path);
  if (!f) {
    err = "cannot open " + path;
    return false;
  }
  int n = 0;
  std::string line;
  while (std::getline(f, line))
    if (!line.empty() && line != "\r") n++;
  int movbones = S.mov_in(0);
  n = (n - 3) / (movbones + 1);
  f.clear();
  f.seekg(0);
  std::string tok;
  while (f >> tok)
    if (tok == ":DEGREES") break;
  post.assign(n, Posture());
  for (auto& p : post) {
    memset(&p, 0, sizeof(p));
  }
  for (int i = 0; i < n; ++i) {
    int frame_num;
    f >> frame_num;
    for (int j = 0; j < movbones; ++j) {
      f >> tok;
      int bi = -1;
      for (int q = 0; q < S.nbones; ++q)
        if (tok == S.b[q].name) { bi = S.b[q].idx; break; }
      if (bi < 0) {
        err = "unknown bone " + tok;
        return false;
      }
      Posture& P = post[i];
      P.rot[bi][0] = P.rot[bi][1] = P.rot[bi][2] = 0;
      for (int x = 0; x < S.b[bi].dof; ++x) {
        double v;
        f >> v;
        switch (S.b[bi].dofo[x]) {
          case 1: P.rot[bi][0] = v; break;
          case 2: P.rot[bi][1] = v; break;
          case 3: P.rot[bi][2] = v; break;
          case 4: P.trans[bi][0] = v * scale; break;
          case 5: P.trans[bi][1] = v * scale; break;
          case 6: P.trans[bi][2] = v * scale; break;
          case 7: P.len[bi] = v; break;
          default: x = S.b[bi].dof; break;
        }
      }
    }
  }
  return true;
}

// displaySkeleton.cpp software GL (lines 15-71) + DrawBone/Traverse (108-247)
struct FK {
  Skeleton* S;
  M4 cur;
  std::stack<std::vector<double>> stk;
  std::vector<std::array<double, 16>> rot;   // boneRotations (= currentTransform^T)
  std::vector<std::array<double, 3>> trans;  // boneTranslations
  void push()
  {
    stk.push(std::vector<double>(&cur[0][0], &cur[0][0] + 16));
  }
  void pop()
  {
    memcpy(cur, stk.top().data(), sizeof(cur));
    stk.pop();
  }
  void translatef(float x, float y, float z)
  {
    M4 T;
    ident(T);
    T[3][0] = x;
    T[3][1] = y;
    T[3][2] = z;
    mmul(T, cur, cur);
  }
  void rotatef(float degrees, float x, float y, float z)
  {
    double ax[3] = {x, y, z};
    normalize3(ax);
    float radians = (float)((degrees / 360.0) * 2.0 * M_PI);
    M4 R;
    angle_axis_T((double)radians, ax, R);
    mmul(R, cur, cur);
  }
  void mult(const double m[4][4])
  {
    M4 A;
    for (int x = 0; x < 4; ++x)
      for (int y = 0; y < 4; ++y) A[x][y] = m[x][y];
    mmul(A, cur, cur);
  }
  void draw(Bone& B)
  {
    mult(B.rpc);
    if (B.doftz) translatef(0.0f, 0.0f, (float)B.tz);
    if (B.dofty) translatef(0.0f, (float)B.ty, 0.0f);
    if (B.doftx) translatef((float)B.tx, 0.0f, 0.0f);
    if (B.dofrz) rotatef((float)B.rz, 0.0f, 0.0f, 1.0f);
    if (B.dofry) rotatef((float)B.ry, 0.0f, 1.0f, 0.0f);
    if (B.dofrx) rotatef((float)B.rx, 1.0f, 0.0f, 0.0f);
    push();
    double tx = B.dir[0] * B.length, ty = B.dir[1] * B.length, tz = B.dir[2] * B.length;
    if (B.idx != 0) {
      M4 ct;
      memcpy(ct, cur, sizeof(ct));
      const double z_dir[3] = {0, 0, 1};
      double r_axis[3] = {z_dir[1] * B.dir[2] - z_dir[2] * B.dir[1], z_dir[2] * B.dir[0] - z_dir[0] * B.dir[2],
                          z_dir[0] * B.dir[1] - z_dir[1] * B.dir[0]};
      double dot_prod = z_dir[0] * B.dir[0] + z_dir[1] * B.dir[1] + z_dir[2] * B.dir[2];
      double r_axis_len = sqrt(r_axis[0] * r_axis[0] + r_axis[1] * r_axis[1] + r_axis[2] * r_axis[2]);
      double theta = atan2(r_axis_len, dot_prod);
      double ax[3] = {r_axis[0], r_axis[1], r_axis[2]};
      normalize3(ax);
      M4 R, Sc, SR;
      angle_axis_T(theta, ax, R);
      ident(Sc);
      Sc[0][0] = B.aspx;
      Sc[1][1] = B.aspy;
      mmul(Sc, R, SR);
      mmul(SR, ct, ct);
      std::array<double, 3> t = {ct[3][0], ct[3][1], ct[3][2]};
      ct[3][0] = ct[3][1] = ct[3][2] = 0;
      std::array<double, 16> rT;
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) rT[i * 4 + j] = ct[j][i];
      rot[B.idx] = rT;
      trans[B.idx] = t;
    }
    pop();
    translatef((float)tx, (float)ty, (float)tz);
  }
  void traverse(int bi)
  {
    if (bi < 0) return;
    push();
    draw(S->b[bi]);
    traverse(S->b[bi].child);
    pop();
    traverse(S->b[bi].sibling);
  }
};

}  // namespace

extern "C" int dt_mocap_bone_table(const char* asf, const char* amc, const int32_t* frames, int32_t n_frames,
                                   double* out, int32_t* n_bones_out, int32_t* n_postures_out)
{
  Skeleton S;
  std::string err;
  const double scale = 0.06;   // MOCAP_SCALE (types.h:6)
  if (!read_asf(asf, scale, S, err)) {
    dth::set_error(err);
    return DT_E_IO;
  }
  std::vector<Posture> post;
  if (!read_amc(amc, scale, S, post, err)) {
    dth::set_error(err);
    return DT_E_IO;
  }
  int numbones = S.num_in(0);
  if (n_bones_out) *n_bones_out = numbones - 1;
  if (n_postures_out) *n_postures_out = (int32_t)post.size();
  if (!out) return DT_OK;
  for (int fi = 0; fi < n_frames; ++fi) {
    int pid = frames[fi];
    if (pid < 0) pid = 0;
    if (pid >= (int)post.size()) pid = (int)post.size() - 1;   // scene.h:121-125
    const Posture& P = post[pid];
    // Skeleton::setPosture (skeleton.cpp:476-508)
    for (int j = 0; j < S.nbones; ++j) {
      Bone& B = S.b[j];
      if (B.dofrx) B.rx = P.rot[j][0];
      if (B.doftx) B.tx = P.trans[j][0];
      if (B.dofry) B.ry = P.rot[j][1];
      if (B.dofty) B.ty = P.trans[j][1];
      if (B.dofrz) B.rz = P.rot[j][2];
      if (B.doftz) B.tz = P.trans[j][2];
      if (B.doftl) B.tl = P.len[j];
    }
    FK fk;
    fk.S = &S;
    fk.rot.assign(numbones, std::array<double, 16>{});
    fk.trans.assign(numbones, std::array<double, 3>{});
    ident(fk.cur);
    // ComputeBonePositions (displaySkeleton.cpp:256-290); skeleton-level translation and
    // rotation are always 0 (GetTranslation returns tx,ty,tz of the Skeleton, never set)
    fk.push();
    ident(fk.cur);
    fk.push();
    fk.translatef(0.0f, 0.0f, 0.0f);
    fk.rotatef(0.0f, 1.0f, 0.0f, 0.0f);
    fk.rotatef(0.0f, 0.0f, 1.0f, 0.0f);
    fk.rotatef(0.0f, 0.0f, 0.0f, 1.0f);
    fk.traverse(0);
    fk.pop();
    fk.pop();
    // buildFinal (scene.h:637-658): left = R*S*(0,0,0,1) + t ; right = R*S*(0,0,len,1) + t
    for (int x = 1; x < numbones; ++x) {
      const std::array<double, 16>& Rm = fk.rot[x];
      double Sm[4][4];
      ident(Sm);
      Sm[0][0] = S.b[x].aspx;
      Sm[1][1] = S.b[x].aspy;
      double RS[4][4];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          double s = Rm[i * 4 + 0] * Sm[0][j];
          for (int k = 1; k < 4; ++k) s = s + Rm[i * 4 + k] * Sm[k][j];
          RS[i][j] = s;
        }
      float len = (float)S.b[x].length;   // vector<float> lengths
      double lv[4] = {0, 0, 0, 1}, rv[4] = {0, 0, len, 1};
      double* o = out + ((size_t)fi * (numbones - 1) + (x - 1)) * 6;
      for (int i = 0; i < 3; ++i) {
        double sl = RS[i][0] * lv[0], sr = RS[i][0] * rv[0];
        for (int k = 1; k < 4; ++k) {
          sl = sl + RS[i][k] * lv[k];
          sr = sr + RS[i][k] * rv[k];
        }
        o[i] = sl + fk.trans[x][i];
        o[3 + i] = sr + fk.trans[x][i];
      }
    }
  }
  return DT_OK;
}
