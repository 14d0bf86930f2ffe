// oracle/pmvs_oracle.cpp -- TEST INFRASTRUCTURE ONLY (the oracle).
//
// Scalar CPU restatement of the reference PMVS2 hot path (robjermy/CMVS-PMVS @ 2025-02-04):
// image pyramid, camera projection, bilinear sampling, COptim::grabTex / normalize / dot /
// my_f / encode / decode / getPAxes / computeINCC / setINCCs, preProcess / refinePatch /
// postProcess and the image-selection helpers, each restated in the reference's operation
// order (float vs double exactly as the reference's C++ types and overloads resolve; the
// unqualified sin/cos/log/sqrt/asin/acos/atan/floor on float arguments in those TUs resolve to
// the double C functions -- probed with static_assert against the reference headers).
// Build with -ffp-contract=off (x86-64 baseline has no FMA; the reference never fuses).
//
// Parity pinning: camera setup/projection, CPatch serialisation and option parsing are pinned
// against the reference's own TUs compiled unmodified into oracle/_ref (see oracle/Makefile).
// optim.cpp itself is unbuildable here (it includes nlopt.hpp, absent), and CImage needs
// CImg.h (absent), so grabTex/normalize/my_f/... and buildImage are restated without a
// reference binary to compare against: "parity partially pinned" (DESIGN.md §Oracle).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this file.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/pmvs_amd.h"
#include "bobyqa_oracle.h"

namespace oracle {

constexpr int MAXL = PMVS_MAX_LEVEL + 3;

struct V3 {
  float v[3];
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
};
struct V4 {
  float v[4];
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
};

// TVec4 operator* (vec4.hpp:230-232): ((u0v0 + u1v1) + u2v2) + u3v3 in float.
static inline float dot4(const V4& a, const V4& b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}
static inline float dot3(const V3& a, const V3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline V4 sub4(const V4& a, const V4& b) { return {{a[0] - b[0], a[1] - b[1], a[2] - b[2], a[3] - b[3]}}; }
static inline V4 add4(const V4& a, const V4& b) { return {{a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]}}; }
static inline V3 sub3(const V3& a, const V3& b) { return {{a[0] - b[0], a[1] - b[1], a[2] - b[2]}}; }
static inline V3 add3(const V3& a, const V3& b) { return {{a[0] + b[0], a[1] + b[1], a[2] + b[2]}}; }
static inline V3 mul3(const V3& a, float s) { return {{a[0] * s, a[1] * s, a[2] * s}}; }
// vec3.hpp:222-229 cross
static inline V3 cross3(const V3& u, const V3& v) {
  return {{u[1] * v[2] - v[1] * u[2], -u[0] * v[2] + v[0] * u[2], u[0] * v[1] - v[0] * u[1]}};
}
// norm(): sqrt(norm2) -> double sqrt of a float, rounded back to float (exact either way).
static inline float norm3(const V3& a) { return (float)std::sqrt((double)dot3(a, a)); }
static inline float norm4(const V4& a) { return (float)std::sqrt((double)dot4(a, a)); }
// unitize (vec4.hpp:256-261, vec3.hpp:246-251): v /= sqrt(l) with the double converted to float.
static inline void unitize4(V4& v) {
  const float l = dot4(v, v);
  if (l != 1.0 && l != 0.0) {
    const float d = (float)std::sqrt((double)l);
    v[0] /= d; v[1] /= d; v[2] /= d; v[3] /= d;
  }
}
static inline void unitize3(V3& v) {
  const float l = dot3(v, v);
  if (l != 1.0 && l != 0.0) {
    const float d = (float)std::sqrt((double)l);
    v[0] /= d; v[1] /= d; v[2] /= d;
  }
}
// std::min / std::max argument order semantics.
template <class T> static inline T smin(T a, T b) { return (b < a) ? b : a; }
template <class T> static inline T smax(T a, T b) { return (a < b) ? b : a; }

struct OView {
  int w[MAXL], h[MAXL];
  std::vector<uint8_t> img[MAXL], mask[MAXL], edge[MAXL];
  float P[MAXL][3][4];
  V4 center, oaxis;
};

struct OScene {
  int num, tnum, level, maxLevel, csize, wsize, minImageNum, tau, sequence;
  float nccThreshold, nccThresholdBefore, maxAngle, angle0, angle1, quad;
  int depth;
  std::vector<OView> views;
  std::vector<std::vector<int>> visdata2;
  std::vector<int> bindexes;
  std::vector<V3> xaxes, yaxes, zaxes;
  std::vector<float> ipscales;
  std::vector<int> gwidths, gheights;
};

struct OPatch {
  V4 coord, normal;
  std::vector<int> images;
  std::vector<std::pair<int, int>> grids;
  float ncc = -1.0f, dscale = 0.0f, ascale = 0.0f, tmp = 0.0f;
  int timages = 0;
};

// Per-thread scratch: the reference's _centersT/_raysT/_indexesT/_dscalesT/_ascalesT/_texsT/_weightsT.
struct OCtx {
  V4 center, ray;
  std::vector<int> indexes;
  float dscale = 0, ascale = 0;
  std::vector<float> weights;
  std::vector<std::vector<float>> texs;
  int64_t evals = 0, tex_valid = 0, tex_grabs = 0;
};

// ------------------------------------------------------------------ image pyramid
// CImage::buildImage, image.cpp:228-325 (filter == 0): double accumulation, float denom,
// stored as (uchar)(int)floor(c + 0.5f).
static void build_image(OView& v, int maxLevel) {
  double mask[4][4] = {{1, 3, 3, 1}, {3, 9, 9, 3}, {3, 9, 9, 3}, {1, 3, 3, 1}};
  const float total = 64.0f;
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) mask[y][x] /= total;
  for (int level = 1; level < maxLevel; ++level) {
    const int W = v.w[level], H = v.h[level], Wp = v.w[level - 1], Hp = v.h[level - 1];
    v.img[level].assign((size_t)W * H * 3, 0);
    const uint8_t* src = v.img[level - 1].data();
    for (int y = 0; y < H; ++y) {
      for (int x = 0; x < W; ++x) {
        double c0 = 0, c1 = 0, c2 = 0;
        float denom = 0.0;
        for (int j = -1; j < 3; ++j) {
          const int ytmp = 2 * y + j;
          if (ytmp < 0 || Hp - 1 < ytmp) continue;
          for (int i = -1; i < 3; ++i) {
            const int xtmp = 2 * x + i;
            if (xtmp < 0 || Wp - 1 < xtmp) continue;
            const int index = (ytmp * Wp + xtmp) * 3;
            c0 += mask[j + 1][i + 1] * (double)src[index];
            c1 += mask[j + 1][i + 1] * (double)src[index + 1];
            c2 += mask[j + 1][i + 1] * (double)src[index + 2];
            denom += mask[j + 1][i + 1];
          }
        }
        const double dd = denom;
        c0 /= dd; c1 /= dd; c2 /= dd;
        const int index = (y * W + x) * 3;
        v.img[level][index] = (uint8_t)((int)std::floor(c0 + 0.5f));
        v.img[level][index + 1] = (uint8_t)((int)std::floor(c1 + 0.5f));
        v.img[level][index + 2] = (uint8_t)((int)std::floor(c2 + 0.5f));
      }
    }
  }
}

// CImage::buildMask / buildEdge, image.cpp:327-405 (any of the 2x2 children set -> 255).
static void build_binary(std::vector<uint8_t>* pyr, const int* w, const int* h, int maxLevel) {
  for (int level = 1; level < maxLevel; ++level) {
    pyr[level].assign((size_t)w[level] * h[level], 0);
    for (int y = 0; y < h[level]; ++y) {
      const int ys[2] = {2 * y, std::min(h[level - 1] - 1, 2 * y + 1)};
      for (int x = 0; x < w[level]; ++x) {
        const int xs[2] = {2 * x, std::min(w[level - 1] - 1, 2 * x + 1)};
        int in = 0;
        for (int j = 0; j < 2; ++j)
          for (int i = 0; i < 2; ++i)
            if (pyr[level - 1][ys[j] * w[level - 1] + xs[i]]) in++;
        pyr[level][y * w[level] + x] = (0 < in) ? 255 : 0;
      }
    }
  }
}

// ------------------------------------------------------------------ camera
// CCamera::project, camera.hpp:89-108.
static inline V3 project(const OScene& s, int index, const V4& c, int level) {
  const float(*P)[4] = s.views[index].P[level];
  float v0 = P[0][0] * c[0] + P[0][1] * c[1] + P[0][2] * c[2] + P[0][3] * c[3];
  float v1 = P[1][0] * c[0] + P[1][1] * c[1] + P[1][2] * c[2] + P[1][3] * c[3];
  float v2 = P[2][0] * c[0] + P[2][1] * c[1] + P[2][2] * c[2] + P[2][3] * c[3];
  if (v2 <= 0.0) return {{-0xffff, -0xffff, -1.0f}};
  const float d = v2;
  v0 /= d; v1 /= d; v2 /= d;
  const float lo = (float)(INT_MIN + 3.0f), hi = (float)(INT_MAX - 3.0f);
  v0 = smax(lo, smin(hi, v0));
  v1 = smax(lo, smin(hi, v1));
  return {{v0, v1, v2}};
}

// CCamera::updateProjection/updateCamera/getOpticalCenter, camera.cpp:56-173 (CONTOUR type).
static void setup_camera(OView& v, const float* p12, int maxLevel) {
  for (int y = 0; y < 3; ++y)
    for (int x = 0; x < 4; ++x) v.P[0][y][x] = p12[4 * y + x];
  for (int level = 1; level < maxLevel; ++level) {
    for (int i = 0; i < 3; ++i)
      for (int x = 0; x < 4; ++x) v.P[level][i][x] = v.P[level - 1][i][x];
    for (int x = 0; x < 4; ++x) {
      v.P[level][0][x] /= 2.0f;
      v.P[level][1][x] /= 2.0f;
    }
  }
  V4 oa = {{v.P[0][2][0], v.P[0][2][1], v.P[0][2][2], 0.0f}};
  const float ftmp = norm4(oa);
  oa[3] = v.P[0][2][3];
  for (int i = 0; i < 4; ++i) oa[i] /= ftmp;
  v.oaxis = oa;
  if (v.P[0][2][0] == 0.0 && v.P[0][2][1] == 0.0 && v.P[0][2][2] == 0.0) {
    V3 a = {{v.P[0][0][0], v.P[0][0][1], v.P[0][0][2]}}, b = {{v.P[0][1][0], v.P[0][1][1], v.P[0][1][2]}};
    V3 c = cross3(a, b);
    unitize3(c);
    v.center = {{c[0], c[1], c[2], 0.f}};
  } else {
    double A[3][3], b[3];
    for (int y = 0; y < 3; ++y) {
      for (int x = 0; x < 3; ++x) A[y][x] = v.P[0][y][x];
      b[y] = -(double)v.P[0][y][3];
    }
    // invert (mat3.hpp:275-292): rows of the adjoint are m1^m2, m2^m0, m0^m1.
    auto cr = [](const double* u, const double* w, double* o) {
      o[0] = u[1] * w[2] - w[1] * u[2];
      o[1] = -u[0] * w[2] + w[0] * u[2];
      o[2] = u[0] * w[1] - w[0] * u[1];
    };
    double ad[3][3];
    cr(A[1], A[2], ad[0]);
    cr(A[2], A[0], ad[1]);
    cr(A[0], A[1], ad[2]);
    const double det = ad[0][0] * A[0][0] + ad[0][1] * A[0][1] + ad[0][2] * A[0][2];
    double inv[3][3] = {{0}};
    if (det != 0.0)
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) inv[r][c] = ad[c][r] / det;
    double o[3];
    for (int r = 0; r < 3; ++r) o[r] = inv[r][0] * b[0] + inv[r][1] * b[1] + inv[r][2] * b[2];
    v.center = {{(float)o[0], (float)o[1], (float)o[2], 1.f}};
  }
}

// ------------------------------------------------------------------ image access
// CImage::getColor bilinear branch, image.hpp:435-476.
static inline V3 get_color(const OScene& s, int index, float x, float y, int level) {
  const OView& v = s.views[index];
  const int lx = (int)x, ly = (int)y;
  const int W = v.w[level];
  const int idx = 3 * (ly * W + lx);
  const float dx1 = x - lx, dx0 = 1.0f - dx1;
  const float dy1 = y - ly, dy0 = 1.0f - dy1;
  const float f00 = dx0 * dy0, f01 = dx0 * dy1, f10 = dx1 * dy0, f11 = dx1 * dy1;
  const int idx2 = idx + 3 * W;
  const uint8_t* p0 = v.img[level].data() + idx;
  const uint8_t* p1 = v.img[level].data() + idx2;
  float r = 0.0f, g = 0.0f, b = 0.0f;
  r += p0[0] * f00 + p1[0] * f01;
  g += p0[1] * f00 + p1[1] * f01;
  b += p0[2] * f00 + p1[2] * f01;
  r += p0[3] * f10 + p1[3] * f11;
  g += p0[4] * f10 + p1[4] * f11;
  b += p0[5] * f10 + p1[5] * f11;
  return {{r, g, b}};
}

// CPhoto::getEdge / CImage::getEdge, photo.hpp:50-58, image.hpp:554-581.
static inline int get_edge(const OScene& s, const V4& coord, int index, int level) {
  const OView& v = s.views[index];
  if (v.edge[level].empty()) return 1;
  const V3 ic = project(s, index, coord, level);
  if (ic[0] < 0 || v.w[level] - 1 <= ic[0] || ic[1] < 0 || v.h[level] - 1 <= ic[1]) return 0;
  const int ix = (int)std::floor(ic[0] + 0.5f), iy = (int)std::floor(ic[1] + 0.5f);
  if (ix < 0 || v.w[level] <= ix || iy < 0 || v.h[level] <= iy) return 1;
  return v.edge[level][iy * v.w[level] + ix];
}

// CPhotoSetS::getMask(coord, level) over all views, photoSetS.hpp:110-117; CPhoto::getMask photo.hpp:42-48.
static inline int get_mask_all(const OScene& s, const V4& coord, int level) {
  for (int index = 0; index < s.num; ++index) {
    const OView& v = s.views[index];
    if (v.mask[level].empty()) continue;
    const V3 ic = project(s, index, coord, level);
    const int ix = (int)std::floor(ic[0] + 0.5f), iy = (int)std::floor(ic[1] + 0.5f);
    if (ix < 0 || v.w[level] <= ix || iy < 0 || v.h[level] <= iy) continue;
    if (v.mask[level][iy * v.w[level] + ix] == 0) return 0;
  }
  return 1;
}

// CFindMatch::insideBimages, findMatch.cpp:109-118.
static inline int inside_bimages(const OScene& s, const V4& coord) {
  for (int index : s.bindexes) {
    const V3 ic = project(s, index, coord, s.level);
    if (ic[0] < 0.0 || s.views[index].w[s.level] - 1 < ic[0] || ic[1] < 0.0 || s.views[index].h[s.level] - 1 < ic[1])
      return 0;
  }
  return 1;
}

// ------------------------------------------------------------------ COptim helpers
// COptim::getUnit, optim.cpp:1116-1124.
static inline float get_unit(const OScene& s, int index, const V4& coord) {
  const float fz = norm4(sub4(coord, s.views[index].center));
  const float ftmp = s.ipscales[index];
  if (ftmp == 0.0) return 1.0;
  return (float)(2.0 * fz * (0x0001 << s.level) / ftmp);
}

// COptim::getPAxes, optim.cpp:1127-1144.
static inline void get_paxes(const OScene& s, int index, const V4& coord, const V4& normal, V4& px, V4& py) {
  const float pscale = get_unit(s, index, coord);
  V3 n3 = {{normal[0], normal[1], normal[2]}};
  V3 y3 = cross3(n3, s.xaxes[index]);
  unitize3(y3);
  V3 x3 = cross3(y3, n3);
  px = {{x3[0], x3[1], x3[2], 0.0f}};
  py = {{y3[0], y3[1], y3[2], 0.0f}};
  for (int i = 0; i < 4; ++i) { px[i] *= pscale; py[i] *= pscale; }
  const V3 c0 = project(s, index, coord, s.level);
  const float xdis = norm3(sub3(project(s, index, add4(coord, px), s.level), c0));
  const float ydis = norm3(sub3(project(s, index, add4(coord, py), s.level), c0));
  for (int i = 0; i < 4; ++i) { px[i] /= xdis; py[i] /= ydis; }
}

static const float kPow2[] = {0.0625, 0.125, 0.25, 0.5, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024};
static const float kLog2 = (float)std::log(2.0);  // static float Log2 = log(2.0f) (double log)

// (int) conversion of a double as x86-64 cvttsd2si does it (out of range / NaN -> INT_MIN).
static inline int cvt_int_x86(double d) {
  if (!(d > -2147483649.0 && d < 2147483648.0)) return INT_MIN;
  return (int)d;
}

// COptim::grabSafe, optim.cpp:783-805.
static inline int grab_safe(const OScene& s, int index, int size, const V3& c, const V3& dx, const V3& dy, int level) {
  const int margin = size / 2;
  const V3 dxm = mul3(dx, (float)margin), dym = mul3(dy, (float)margin);
  const V3 tl = sub3(sub3(c, dxm), dym);
  const V3 tr = sub3(add3(c, dxm), dym);
  const V3 bl = add3(sub3(c, dxm), dym);
  const V3 br = add3(add3(c, dxm), dym);
  const float minx = smin(tl[0], smin(tr[0], smin(bl[0], br[0])));
  const float maxx = smax(tl[0], smax(tr[0], smax(bl[0], br[0])));
  const float miny = smin(tl[1], smin(tr[1], smin(bl[1], br[1])));
  const float maxy = smax(tl[1], smax(tr[1], smax(bl[1], br[1])));
  const int margin2 = 3;
  if (minx < margin2 || s.views[index].w[level] - 1 - margin2 <= maxx || miny < margin2 ||
      s.views[index].h[level] - 1 - margin2 <= maxy)
    return 0;
  return 1;
}

// COptim::grabTex, optim.cpp:815-863.  Returns 0 and fills tex on success, 1 (empty tex) otherwise.
static int grab_tex(const OScene& s, const V4& coord, const V4& px, const V4& py, const V4& pz, int index,
                    int size, std::vector<float>& tex) {
  tex.clear();
  V4 ray = sub4(s.views[index].center, coord);
  unitize4(ray);
  const float weight = smax(0.0f, dot4(ray, pz));
  if (weight < std::cos((double)s.angle1)) return 1;
  const int margin = size / 2;
  V3 center = project(s, index, coord, s.level);
  V3 dx = sub3(project(s, index, add4(coord, px), s.level), center);
  V3 dy = sub3(project(s, index, add4(coord, py), s.level), center);
  const float ratio = (norm3(dx) + norm3(dy)) / 2.0f;
  int leveldif = cvt_int_x86(std::floor(std::log((double)ratio) / (double)kLog2 + 0.5f));
  leveldif = std::max(-s.level, std::min(2, leveldif));
  const float scale = kPow2[leveldif + 4];
  const int newlevel = s.level + leveldif;
  for (int i = 0; i < 3; ++i) { center[i] /= scale; dx[i] /= scale; dy[i] /= scale; }
  if (grab_safe(s, index, size, center, dx, dy, newlevel) == 0) return 1;
  const V3 dxm = mul3(dx, (float)margin), dym = mul3(dy, (float)margin);
  V3 left = sub3(sub3(center, dxm), dym);
  tex.resize(3 * size * size);
  float* t = tex.data();
  for (int y = 0; y < size; ++y) {
    V3 v = left;
    left = add3(left, dy);
    for (int x = 0; x < size; ++x) {
      const V3 c = get_color(s, index, v[0], v[1], newlevel);
      *t++ = c[0];
      *t++ = c[1];
      *t++ = c[2];
      v = add3(v, dx);
    }
  }
  return 0;
}

// COptim::normalize(vector<float>&), optim.cpp:1031-1067.
static void normalize(std::vector<float>& tex) {
  const int size = (int)tex.size();
  const int size3 = size / 3;
  float a0 = 0, a1 = 0, a2 = 0;
  for (int i = 0; i < size3; ++i) {
    a0 += tex[3 * i];
    a1 += tex[3 * i + 1];
    a2 += tex[3 * i + 2];
  }
  a0 /= (float)size3; a1 /= (float)size3; a2 /= (float)size3;
  float ave2 = 0.0;
  for (int i = 0; i < size3; ++i) {
    const float f0 = a0 - tex[3 * i], f1 = a1 - tex[3 * i + 1], f2 = a2 - tex[3 * i + 2];
    ave2 += f0 * f0 + f1 * f1 + f2 * f2;
  }
  ave2 = (float)std::sqrt((double)(ave2 / (float)size));
  if (ave2 == 0.0f) ave2 = 1.0f;
  for (int i = 0; i < size3; ++i) {
    tex[3 * i] -= a0; tex[3 * i] /= ave2;
    tex[3 * i + 1] -= a1; tex[3 * i + 1] /= ave2;
    tex[3 * i + 2] -= a2; tex[3 * i + 2] /= ave2;
  }
}

// COptim::dot, optim.cpp:1069-1077.
static inline float dot_tex(const std::vector<float>& a, const std::vector<float>& b) {
  const int size = (int)a.size();
  float ans = 0.0f;
  for (int i = 0; i < size; ++i) ans += a[i] * b[i];
  return ans / (float)size;
}

static inline float robustincc(float rhs) { return rhs / (1 + 3 * rhs); }   // optim.hpp:86
static inline float unrobustincc(float rhs) { return rhs / (1 - 3 * rhs); } // optim.hpp:90

// COptim::decode, optim.cpp:690-707.
static void decode(const OScene& s, const OCtx& c, V4& coord, V4& normal, const double* vect) {
  const double sc = (double)c.dscale * vect[0];
  const V4 step = {{(float)(c.ray[0] * sc), (float)(c.ray[1] * sc), (float)(c.ray[2] * sc), (float)(c.ray[3] * sc)}};
  coord = add4(c.center, step);
  const int image = c.indexes[0];
  const float angle1 = (float)(vect[1] * c.ascale);
  const float angle2 = (float)(vect[2] * c.ascale);
  const float fx = (float)(std::sin((double)angle1) * std::cos((double)angle2));
  const float fy = (float)std::sin((double)angle2);
  const float fz = (float)(-std::cos((double)angle1) * std::cos((double)angle2));
  const V3 t = add3(add3(mul3(s.xaxes[image], fx), mul3(s.yaxes[image], fy)), mul3(s.zaxes[image], fz));
  normal = {{t[0], t[1], t[2], 0.0f}};
}

// COptim::encode, optim.cpp:660-688.
static void encode(const OScene& s, const OCtx& c, const V4& coord, const V4& normal, double* vect) {
  vect[0] = dot4(sub4(coord, c.center), c.ray) / c.dscale;
  const int image = c.indexes[0];
  V3 n3 = {{normal[0], normal[1], normal[2]}};  // proj(normal), vec4.hpp:268-274
  if (normal[3] != 1.0 && normal[3] != 0.0) { n3[0] /= normal[3]; n3[1] /= normal[3]; n3[2] /= normal[3]; }
  const float fx = dot3(s.xaxes[image], n3);
  const float fy = dot3(s.yaxes[image], n3);
  const float fz = dot3(s.zaxes[image], n3);
  vect[2] = std::asin((double)smax(-1.0f, smin(1.0f, fy)));
  const float cosb = (float)std::cos(vect[2]);
  if (cosb == 0.0) {
    vect[1] = 0.0;
  } else {
    const float sina = fx / cosb;
    const float cosa = -fz / cosb;
    vect[1] = std::acos((double)smax(-1.0f, smin(1.0f, cosa)));
    if (sina < 0.0) vect[1] = -vect[1];
  }
  vect[1] = vect[1] / c.ascale;
  vect[2] = vect[2] / c.ascale;
}

// COptim::my_f, optim.cpp:507-578 (non-pairwise branch).
static double my_f(const OScene& s, OCtx& c, const double* x) {
  double xs[3] = {x[0], x[1], x[2]};
  V4 coord, normal, px, py;
  decode(s, c, coord, normal, xs);
  const int index = c.indexes[0];
  get_paxes(s, index, coord, normal, px, py);
  const int size = std::min(s.tau, (int)c.indexes.size());
  const int mininum = std::min(s.minImageNum, size);
  int nvalid = 0;
  for (int i = 0; i < size; ++i) {
    const int flag = grab_tex(s, coord, px, py, normal, c.indexes[i], s.wsize, c.texs[i]);
    c.tex_grabs++;
    if (flag == 0) {
      normalize(c.texs[i]);
      nvalid++;
    }
  }
  c.evals++;
  c.tex_valid += nvalid;
  if (c.texs[0].empty()) return 2.0;
  double ans = 0.0f;
  int denom = 0;
  for (int i = 1; i < size; ++i) {
    if (c.texs[i].empty()) continue;
    ans += robustincc((float)(1.0 - dot_tex(c.texs[0], c.texs[i])));
    denom++;
  }
  if (denom < mininum - 1) return 2.0f;
  return ans / denom;
}

// COptim::computeUnits (vector<float>& version), optim.cpp:446-471.
static void compute_units(const OScene& s, const OPatch& p, std::vector<float>& units) {
  units.resize(p.images.size());
  for (size_t i = 0; i < p.images.size(); ++i) {
    const int img = p.images[i];
    float u = get_unit(s, img, p.coord);
    V4 ray = sub4(s.views[img].center, p.coord);
    unitize4(ray);
    const float denom = dot4(ray, p.normal);
    if (0.0 < denom) u /= denom;
    else u = INT_MAX / 2;
    units[i] = u;
  }
}

// COptim::computeUnits (indexes/units/rays version), optim.cpp:473-494.
static void compute_units3(const OScene& s, const OPatch& p, std::vector<int>& idx, std::vector<float>& units,
                           std::vector<V4>& rays) {
  for (int img : p.images) {
    V4 ray = sub4(s.views[img].center, p.coord);
    unitize4(ray);
    const float d = dot4(ray, p.normal);
    if (d <= 0.0f) continue;
    const float scale = get_unit(s, img, p.coord);
    idx.push_back(img);
    units.push_back(scale / d);
    rays.push_back(ray);
  }
}

// COptim::computeINCC, optim.cpp:865-938 (weighted, reference-vs-others branch).
static double compute_incc(const OScene& s, OCtx& c, const V4& coord, const V4& normal,
                           const std::vector<int>& indexes, int robust) {
  if ((int)indexes.size() < 2) return 2.0;
  V4 px, py;
  get_paxes(s, indexes[0], coord, normal, px, py);
  const int size = std::min(s.tau, (int)indexes.size());
  for (int i = 0; i < size; ++i) {
    const int flag = grab_tex(s, coord, px, py, normal, indexes[i], s.wsize, c.texs[i]);
    c.tex_grabs++;
    if (flag == 0) normalize(c.texs[i]);
  }
  if (c.texs[0].empty()) return 2.0;
  double score = 0.0;
  float totalweight = 0.0;
  for (int i = 1; i < size; ++i) {
    if (!c.texs[i].empty()) {
      totalweight += c.weights[i];
      if (robust)
        score += robustincc((float)(1.0 - dot_tex(c.texs[0], c.texs[i]))) * c.weights[i];
      else
        score += (1.0 - dot_tex(c.texs[0], c.texs[i])) * c.weights[i];
    }
  }
  if (totalweight == 0.0) score = 2.0;
  else score /= totalweight;
  return score;
}

// COptim::setINCCs (vector version), optim.cpp:709-744.
static void set_inccs(const OScene& s, OCtx& c, const OPatch& p, std::vector<float>& inccs,
                      const std::vector<int>& indexes, int robust) {
  V4 px, py;
  get_paxes(s, indexes[0], p.coord, p.normal, px, py);
  const int size = (int)indexes.size();
  for (int i = 0; i < size; ++i) {
    const int flag = grab_tex(s, p.coord, px, py, p.normal, indexes[i], s.wsize, c.texs[i]);
    c.tex_grabs++;
    if (flag == 0) normalize(c.texs[i]);
  }
  inccs.assign(size, 0.0f);
  if (c.texs[0].empty()) {
    std::fill(inccs.begin(), inccs.end(), 2.0f);
    return;
  }
  for (int i = 0; i < size; ++i) {
    if (i == 0) inccs[i] = 0.0f;
    else if (!c.texs[i].empty()) {
      if (robust == 0) inccs[i] = 1.0f - dot_tex(c.texs[0], c.texs[i]);
      else inccs[i] = robustincc(1.0f - dot_tex(c.texs[0], c.texs[i]));
    } else
      inccs[i] = 2.0f;
  }
}

// COptim::setINCCs (matrix version), optim.cpp:746-781.
static void set_inccs2(const OScene& s, OCtx& c, const OPatch& p, std::vector<std::vector<float>>& inccs,
                       const std::vector<int>& indexes, int robust) {
  V4 px, py;
  get_paxes(s, indexes[0], p.coord, p.normal, px, py);
  const int size = (int)indexes.size();
  for (int i = 0; i < size; ++i) {
    const int flag = grab_tex(s, p.coord, px, py, p.normal, indexes[i], s.wsize, c.texs[i]);
    c.tex_grabs++;
    if (flag == 0) normalize(c.texs[i]);
  }
  inccs.assign(size, std::vector<float>(size, 0.0f));
  for (int i = 0; i < size; ++i) {
    inccs[i][i] = 0.0f;
    for (int j = i + 1; j < size; ++j) {
      if (!c.texs[i].empty() && !c.texs[j].empty()) {
        if (robust == 0) inccs[j][i] = inccs[i][j] = 1.0f - dot_tex(c.texs[i], c.texs[j]);
        else inccs[j][i] = inccs[i][j] = robustincc(1.0f - dot_tex(c.texs[i], c.texs[j]));
      } else
        inccs[j][i] = inccs[i][j] = 2.0f;
    }
  }
}

// COptim::addImages, optim.cpp:398-444.
static void add_images(const OScene& s, OPatch& p) {
  std::vector<int> used(s.num, 0);
  for (int img : p.images) used[img] = 1;
  const float athreshold = (float)std::cos((double)s.angle0);
  for (int img : s.visdata2[p.images[0]]) {
    if (used[img]) continue;
    const V3 ic = project(s, img, p.coord, s.level);
    if (ic[0] < 0.0f || s.views[img].w[s.level] - 1 <= ic[0] || ic[1] < 0.0f || s.views[img].h[s.level] - 1 <= ic[1])
      continue;
    if (get_edge(s, p.coord, img, s.level) == 0) continue;
    V4 ray = sub4(s.views[img].center, p.coord);
    unitize4(ray);
    const float ftmp = dot4(ray, p.normal);
    if (athreshold <= ftmp) p.images.push_back(img);
  }
}

// Near-threshold diagnostics (test infrastructure: how many decisions a parity workload puts close
// to a threshold, so a bit-exact match there means something).  [0] constraintImages tests,
// [1] those with |incc - (1 - thr)| < 0.02; [2] filterOutside gains, [3] those with |gain| < 0.05;
// [4] refined patches, [5] those with |ncc - nccThreshold| < 0.02.
static std::atomic<long long> g_diag[6];
static inline void diag(int k, bool near) {
  g_diag[k].fetch_add(1, std::memory_order_relaxed);
  if (near) g_diag[k + 1].fetch_add(1, std::memory_order_relaxed);
}

// Conversions to the C-ABI records (include/pmvs_amd.h): lists hold PMVS_MAX_IMAGES entries and
// pmvs_patch keeps 16-bit cell coordinates.  A longer list is not truncated: it raises
// g_list_overflow, which pyoracle turns into an exception.  A cell coordinate outside
// [-32767, 32767] (a projection far outside the image, so outside every cell grid) is stored as
// -32768, the rule the device uses too (pmvs_layout.h grid16).
static std::atomic<int> g_list_overflow{0};
static inline int list_len(size_t n) {
  if (n > (size_t)PMVS_MAX_IMAGES) {
    g_list_overflow = 1;
    return PMVS_MAX_IMAGES;
  }
  return (int)n;
}
static inline int16_t cell16(int v) { return (v < -32767 || v > 32767) ? (int16_t)-32768 : (int16_t)v; }

// COptim::constraintImages, optim.cpp:192-206.
static void constraint_images(const OScene& s, OCtx& c, OPatch& p, float thr) {
  std::vector<float> inccs;
  set_inccs(s, c, p, inccs, p.images, 0);
  std::vector<int> ni;
  ni.push_back(p.images[0]);
  for (int i = 1; i < (int)p.images.size(); ++i) {
    diag(0, std::fabs(inccs[i] - (1.0f - thr)) < 0.02f);
    if (inccs[i] < 1.0f - thr) ni.push_back(p.images[i]);
  }
  p.images.swap(ni);
}

// COptim::sortImages, optim.cpp:284-321 (newm == 1).
static void sort_images(const OScene& s, OPatch& p) {
  const float threshold = (float)(1.0f - std::cos(10.0 * M_PI / 180.0));
  std::vector<int> idx, idx2;
  std::vector<float> units, units2;
  std::vector<V4> rays, rays2;
  compute_units3(s, p, idx, units, rays);
  p.images.clear();
  if (idx.size() < 2) return;
  units[0] = 0.0f;
  while (!idx.empty()) {
    int index = 0;
    for (int k = 1; k < (int)units.size(); ++k)
      if (units[k] < units[index]) index = k;
    p.images.push_back(idx[index]);
    idx2.clear(); units2.clear(); rays2.clear();
    for (int j = 0; j < (int)rays.size(); ++j) {
      if (j == index) continue;
      idx2.push_back(idx[j]);
      rays2.push_back(rays[j]);
      const float ftmp = std::min(threshold, std::max(threshold / 2.0f, 1.0f - dot4(rays[index], rays[j])));
      units2.push_back(units[j] * (threshold / ftmp));
    }
    idx2.swap(idx); units2.swap(units); rays2.swap(rays);
  }
}

// CPatchOrganizerS::setScales, patchOrganizerS.cpp:663-684.
static void set_scales(const OScene& s, OPatch& p) {
  const float unit = get_unit(s, p.images[0], p.coord);
  const float unit2 = 2.0f * unit;
  V4 ray = sub4(p.coord, s.views[p.images[0]].center);
  unitize4(ray);
  const int inum = std::min(s.tau, (int)p.images.size());
  const V4 off = {{ray[0] * unit2, ray[1] * unit2, ray[2] * unit2, ray[3] * unit2}};
  for (int i = 1; i < inum; ++i) {
    const V3 diff = sub3(project(s, p.images[i], p.coord, s.level), project(s, p.images[i], sub4(p.coord, off), s.level));
    p.dscale += norm3(diff);
  }
  p.dscale /= (float)(inum - 1);
  p.dscale = unit2 / p.dscale;
  p.ascale = (float)std::atan((double)(p.dscale / (unit * s.wsize / 2.0f)));
}

// CPhotoSetS::checkAngles, photoSetS.cpp:164-189.
static int check_angles(const OScene& s, const V4& coord, const std::vector<int>& idx, float minA, float maxA) {
  int count = 0;
  std::vector<V4> rays(idx.size());
  for (size_t i = 0; i < idx.size(); ++i) {
    rays[i] = sub4(s.views[idx[i]].center, coord);
    unitize4(rays[i]);
  }
  for (size_t i = 0; i < idx.size(); ++i)
    for (size_t j = i + 1; j < idx.size(); ++j) {
      const float d = std::max(-1.0f, std::min(1.0f, dot4(rays[i], rays[j])));
      const float angle = (float)std::acos((double)d);
      if (minA < angle && angle < maxA) ++count;
    }
  return count < 1 ? 1 : 0;
}

// COptim::filterImagesByAngle, optim.cpp:124-148.
static void filter_images_by_angle(const OScene& s, OPatch& p) {
  std::vector<int> ni;
  const double ct = std::cos((double)s.angle1);
  for (size_t k = 0; k < p.images.size(); ++k) {
    const int img = p.images[k];
    V4 ray = sub4(s.views[img].center, p.coord);
    unitize4(ray);
    if (dot4(ray, p.normal) < ct) {
      if (k == 0) {
        p.images.clear();
        return;
      }
    } else
      ni.push_back(img);
  }
  p.images.swap(ni);
}

// CPatchOrganizerS::setGrids, patchOrganizerS.cpp:410-419.
static void set_grids(const OScene& s, OPatch& p) {
  p.grids.clear();
  for (int img : p.images) {
    const V3 ic = project(s, img, p.coord, s.level);
    const int ix = ((int)std::floor(ic[0] + 0.5f)) / s.csize;
    const int iy = ((int)std::floor(ic[1] + 0.5f)) / s.csize;
    p.grids.push_back({ix, iy});
  }
}

// COptim::setRefImage, optim.cpp:208-254.
static void set_ref_image(const OScene& s, OCtx& c, OPatch& p) {
  std::vector<int> indexes;
  for (int img : p.images)
    if (img < s.tnum) indexes.push_back(img);
  if (indexes.empty()) {
    p.images.clear();
    return;
  }
  std::vector<std::vector<float>> inccs;
  set_inccs2(s, c, p, inccs, indexes, 1);
  int refindex = -1;
  float refncc = INT_MAX / 2;
  for (int i = 0; i < (int)indexes.size(); ++i) {
    float sum = 0.0f;
    for (float v : inccs[i]) sum = sum + v;
    if (sum < refncc) {
      refncc = sum;
      refindex = i;
    }
  }
  const int refIndex = indexes[refindex];
  for (size_t i = 0; i < p.images.size(); ++i)
    if (p.images[i] == refIndex) {
      const int t = p.images[0];
      p.images[0] = refIndex;
      p.images[i] = t;
      break;
    }
}

// COptim::preProcess, optim.cpp:95-122.
static int pre_process(const OScene& s, OCtx& c, OPatch& p) {
  add_images(s, p);
  constraint_images(s, c, p, s.nccThresholdBefore);
  sort_images(s, p);
  if ((int)p.images.size() > 0) set_scales(s, p);
  if ((int)p.images.size() < s.minImageNum) return 1;
  if (check_angles(s, p.coord, p.images, s.maxAngle, s.angle1)) {
    p.images.clear();
    return 1;
  }
  return 0;
}

// COptim::refinePatchBFGS, optim.cpp:580-658; returns the optimizer result code.
static int refine_patch(const OScene& s, OCtx& c, OPatch& p, int* evals) {
  c.center = p.coord;
  c.ray = sub4(p.coord, s.views[p.images[0]].center);
  unitize4(c.ray);
  c.indexes = p.images;
  c.dscale = p.dscale;
  c.ascale = (float)(M_PI / 48.0f);
  compute_units(s, p, c.weights);
  for (int i = 1; i < (int)c.weights.size(); ++i) c.weights[i] = std::min(1.0f, c.weights[0] / c.weights[i]);
  c.weights[0] = 1.0f;
  double pv[3];
  encode(s, c, p.coord, p.normal, pv);
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999};
  const double ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  double x[3];
  for (int i = 0; i < 3; ++i) x[i] = std::max(std::min(pv[i], ub[i]), lb[i]);
  double minf = 0;
  int ne = 0;
  const int64_t ev0 = c.evals;
  const BqResult rc = bobyqa_minimize(x, lb, ub, 1.e-7, 1000, [&](const double* xx) { return my_f(s, c, xx); },
                                      &minf, &ne);
  *evals = (int)(c.evals - ev0);
  const bool success = (rc == BQ_SUCCESS || rc == BQ_STOPVAL || rc == BQ_FTOL || rc == BQ_XTOL);
  if (success) {
    decode(s, c, p.coord, p.normal, x);
    p.ncc = (float)(1.0 - unrobustincc((float)compute_incc(s, c, p.coord, p.normal, p.images, 1)));
    diag(4, std::fabs(p.ncc - s.nccThreshold) < 0.02f);
  }
  return (int)rc;
}

// COptim::postProcess, optim.cpp:150-190 (depth 0: no setVImagesVGrids / check).
static int post_process(const OScene& s, OCtx& c, OPatch& p) {
  if ((int)p.images.size() < s.minImageNum) return 1;
  if (get_mask_all(s, p.coord, s.level) == 0 || inside_bimages(s, p.coord) == 0) return 1;
  add_images(s, p);
  constraint_images(s, c, p, s.nccThreshold);
  filter_images_by_angle(s, p);
  if ((int)p.images.size() < s.minImageNum) return 1;
  set_grids(s, p);
  set_ref_image(s, c, p);
  if (p.images.empty()) return 1;  // reference would index an empty vector here (UB); reject
  constraint_images(s, c, p, s.nccThreshold);
  if ((int)p.images.size() < s.minImageNum) return 1;
  set_grids(s, p);
  p.timages = 0;
  for (int img : p.images)
    if (img < s.tnum) ++p.timages;
  p.tmp = std::max(0.0f, p.ncc - s.nccThreshold) * p.timages;
  return 0;
}

static void refine_one(const OScene& s, OCtx& c, const pmvs_candidate& in, pmvs_refined& out) {
  std::memset(&out, 0, sizeof(out));
  OPatch p;
  for (int i = 0; i < 4; ++i) { p.coord[i] = in.coord[i]; p.normal[i] = in.normal[i]; }
  p.dscale = in.dscale;
  p.images.assign(in.images, in.images + in.num_images);
  int status = PMVS_ACCEPTED;
  out.refine_code = 0;
  if (pre_process(s, c, p)) {
    status = PMVS_FAIL_PRE;
  } else {
    int ev = 0;
    out.refine_code = refine_patch(s, c, p, &ev);
    out.evals = ev;
    if (post_process(s, c, p)) status = PMVS_FAIL_POST;
  }
  out.status = status;
  for (int i = 0; i < 4; ++i) { out.coord[i] = p.coord[i]; out.normal[i] = p.normal[i]; }
  out.ncc = p.ncc; out.dscale = p.dscale; out.ascale = p.ascale; out.tmp = p.tmp; out.timages = p.timages;
  const int ni = list_len(p.images.size());
  out.num_images = ni;
  for (int i = 0; i < ni; ++i) out.images[i] = p.images[i];
  for (int i = 0; i < (int)p.grids.size() && i < PMVS_MAX_IMAGES; ++i) {
    out.grids[i][0] = p.grids[i].first;
    out.grids[i][1] = p.grids[i].second;
  }
}

static void init_ctx(const OScene& s, OCtx& c) {
  c.texs.assign(s.num, std::vector<float>());
  c.weights.clear();
}

}  // namespace oracle

#include "filter_oracle.h"
#include "expand_oracle.h"
#include "seed_oracle.h"

using namespace oracle;

extern "C" {

// CPatchOrganizerS::setGrids (patchOrganizerS.cpp:410-419) on pmvs_patch records, with the int16
// cell narrowing of the C-ABI (cell16); used by the cluster-exchange emulation in the tests.
void oracle_set_grids(void* h, pmvs_patch* patches, int n) {
  const OScene& s = *static_cast<const OScene*>(h);
  for (int i = 0; i < n; ++i) {
    pmvs_patch& a = patches[i];
    V4 c;
    for (int k = 0; k < 4; ++k) c[k] = a.coord[k];
    for (int k = 0; k < a.num_images; ++k) {
      const V3 ic = project(s, a.images[k], c, s.level);
      a.grids[k][0] = cell16(((int)std::floor(ic[0] + 0.5f)) / s.csize);
      a.grids[k][1] = cell16(((int)std::floor(ic[1] + 0.5f)) / s.csize);
    }
  }
}

// ---- organizer pieces, pinned to the reference's own patchOrganizerS.cpp / photoSetS.cpp compiled
// in oracle/_ref/organizer (tests/test_organizer_pinning.py).  Records: coords4[4 * i], image lists
// images[off[i] .. off[i + 1]).

// set_grids_images (expand_oracle.h) per record: out[i * (3 * PMVS_MAX_IMAGES + 1)] = kept entries,
// then (image, ix, iy) triples.
void oracle_set_grids_images(void* h, int n, const float* coords4, const int* off, const int* images, int* out) {
  const OScene& s = *static_cast<const OScene*>(h);
  const int stride = 3 * PMVS_MAX_IMAGES + 1;
  for (int i = 0; i < n; ++i) {
    FPatch c;
    for (int k = 0; k < 4; ++k) c.coord[k] = coords4[4 * i + k];
    set_grids_images(s, std::vector<int>(images + off[i], images + off[i + 1]), c);
    int* o = out + (size_t)i * stride;
    o[0] = (int)c.images.size();
    for (size_t k = 0; k < c.images.size() && k < (size_t)PMVS_MAX_IMAGES; ++k) {
      o[1 + 3 * k] = c.images[k];
      o[2 + 3 * k] = c.grids[k].first;
      o[3 + 3 * k] = c.grids[k].second;
    }
  }
}

// set_grids (CPatchOrganizerS::setGrids, full int cells) per record, out as oracle_set_grids_images.
void oracle_set_grids_full(void* h, int n, const float* coords4, const int* off, const int* images, int* out) {
  const OScene& s = *static_cast<const OScene*>(h);
  const int stride = 3 * PMVS_MAX_IMAGES + 1;
  for (int i = 0; i < n; ++i) {
    OPatch p;
    for (int k = 0; k < 4; ++k) p.coord[k] = coords4[4 * i + k];
    p.images.assign(images + off[i], images + off[i + 1]);
    set_grids(s, p);
    int* o = out + (size_t)i * stride;
    o[0] = (int)p.images.size();
    for (size_t k = 0; k < p.images.size() && k < (size_t)PMVS_MAX_IMAGES; ++k) {
      o[1 + 3 * k] = p.images[k];
      o[2 + 3 * k] = p.grids[k].first;
      o[3 + 3 * k] = p.grids[k].second;
    }
  }
}

// update_depth_maps (expand_oracle.h, CPatchOrganizerS::updateDepthMaps) for the n patches added in
// order to empty depth maps; out: every target's cells, row-major, concatenated (patch or -1).
void oracle_update_depth_maps(void* h, int n, const float* coords4, int* out) {
  const OScene& s = *static_cast<const OScene*>(h);
  Model m(s);
  std::vector<FPatch> P((size_t)n);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 4; ++k) P[i].coord[k] = coords4[4 * i + k];
    update_depth_maps(m, P, i);
  }
  size_t o = 0;
  for (int t = 0; t < s.tnum; ++t)
    for (int d : m.o.dpgrids[t]) out[o++] = d;
}

// isVisible0 at depth 0 as set_vimages_vgrids evaluates it: the patch's cell in image t, and
// is_visible (filter_oracle.h); out3: visible, ix, iy.
void oracle_is_visible0(void* h, int n, const float* coords4, const int* images, int* out3) {
  const OScene& s = *static_cast<const OScene*>(h);
  const Organizer o(s);
  const std::vector<FPatch> P;
  for (int i = 0; i < n; ++i) {
    FPatch q;
    for (int k = 0; k < 4; ++k) q.coord[k] = coords4[4 * i + k];
    const int t = images[i];
    const V3 ic = project(s, t, q.coord, s.level);
    const int ix = ((int)std::floor(ic[0] + 0.5f)) / s.csize;
    const int iy = ((int)std::floor(ic[1] + 0.5f)) / s.csize;
    out3[3 * i] = is_visible(o, P, q, t, ix, iy, 0.5f);
    out3[3 * i + 1] = ix;
    out3[3 * i + 2] = iy;
  }
}

// check_angles (CPhotoSetS::checkAngles) per record.
void oracle_check_angles(void* h, int n, const float* coords4, const int* off, const int* idx, float minA, float maxA,
                         int* out) {
  const OScene& s = *static_cast<const OScene*>(h);
  for (int i = 0; i < n; ++i) {
    V4 c;
    for (int k = 0; k < 4; ++k) c[k] = coords4[4 * i + k];
    out[i] = check_angles(s, c, std::vector<int>(idx + off[i], idx + off[i + 1]), minA, maxA);
  }
}

// set_distances (seed_oracle.h, CPhotoSetS::setDistances): num x num.
void oracle_distances(void* h, float* out) {
  const OScene& s = *static_cast<const OScene*>(h);
  std::vector<std::vector<float>> d;
  set_distances(s, d);
  for (int i = 0; i < s.num; ++i)
    for (int j = 0; j < s.num; ++j) out[(size_t)i * s.num + j] = d[i][j];
}

// 1 when a result list exceeded PMVS_MAX_IMAGES since the last reset (see list_len).
int oracle_list_overflow(int reset) {
  const int v = g_list_overflow.load();
  if (reset) g_list_overflow = 0;
  return v;
}

// Near-threshold decision counts accumulated since the last reset (see g_diag).
void oracle_diag(long long* out, int reset) {
  for (int k = 0; k < 6; ++k) {
    if (out) out[k] = g_diag[k].load();
    if (reset) g_diag[k] = 0;
  }
}

void* oracle_scene_create(const pmvs_scene_desc* d) {
  OScene* s = new OScene();
  s->num = d->num_views;
  s->tnum = d->num_targets;
  s->level = d->level;
  s->maxLevel = std::max(1, d->level + 3);
  s->csize = d->csize;
  s->wsize = d->wsize;
  s->minImageNum = d->min_image_num;
  s->tau = std::min(d->min_image_num * 2, d->num_views);
  s->sequence = d->sequence;
  s->nccThreshold = d->threshold;
  s->nccThresholdBefore = d->threshold - 0.3f;
  s->maxAngle = d->max_angle;
  s->angle0 = (float)(60.0f * M_PI / 180.0f);
  s->angle1 = (float)(60.0f * M_PI / 180.0f);
  s->quad = d->quad_threshold;
  s->depth = 0;
  s->views.resize(s->num);
  for (int i = 0; i < s->num; ++i) {
    OView& v = s->views[i];
    const pmvs_view_desc& vd = d->views[i];
    v.w[0] = vd.width;
    v.h[0] = vd.height;
    for (int l = 1; l < s->maxLevel; ++l) { v.w[l] = v.w[l - 1] / 2; v.h[l] = v.h[l - 1] / 2; }
    v.img[0].assign(vd.rgb, vd.rgb + (size_t)vd.width * vd.height * 3);
    build_image(v, s->maxLevel);
    if (vd.mask) {
      v.mask[0].resize((size_t)vd.width * vd.height);
      for (size_t k = 0; k < v.mask[0].size(); ++k) v.mask[0][k] = (127 < (int)vd.mask[k]) ? 255 : 0;
      build_binary(v.mask, v.w, v.h, s->maxLevel);
    }
    if (vd.edge) {
      v.edge[0].resize((size_t)vd.width * vd.height);
      for (size_t k = 0; k < v.edge[0].size(); ++k) v.edge[0][k] = (1 < vd.edge[k]) ? 255 : 0;
      build_binary(v.edge, v.w, v.h, s->maxLevel);
    }
    setup_camera(v, vd.projection, s->maxLevel);
  }
  s->visdata2.resize(s->num);
  for (int i = 0; i < s->num; ++i)
    for (int k = d->visdata2_offsets[i]; k < d->visdata2_offsets[i + 1]; ++k) s->visdata2[i].push_back(d->visdata2[k]);
  for (int i = 0; i < d->num_bindexes; ++i) s->bindexes.push_back(d->bindexes[i]);
  // COptim::setAxesScales, optim.cpp:43-64.
  s->xaxes.resize(s->num); s->yaxes.resize(s->num); s->zaxes.resize(s->num); s->ipscales.resize(s->num);
  for (int i = 0; i < s->num; ++i) {
    const OView& v = s->views[i];
    s->zaxes[i] = {{v.oaxis[0], v.oaxis[1], v.oaxis[2]}};
    s->xaxes[i] = {{v.P[0][0][0], v.P[0][0][1], v.P[0][0][2]}};
    s->yaxes[i] = cross3(s->zaxes[i], s->xaxes[i]);
    unitize3(s->yaxes[i]);
    s->xaxes[i] = cross3(s->yaxes[i], s->zaxes[i]);
    const V4 xa = {{s->xaxes[i][0], s->xaxes[i][1], s->xaxes[i][2], 0.0}};
    const V4 ya = {{s->yaxes[i][0], s->yaxes[i][1], s->yaxes[i][2], 0.0}};
    const V4 p0 = {{v.P[0][0][0], v.P[0][0][1], v.P[0][0][2], v.P[0][0][3]}};
    const V4 p1 = {{v.P[0][1][0], v.P[0][1][1], v.P[0][1][2], v.P[0][1][3]}};
    const float fx = dot4(xa, p0), fy = dot4(ya, p1);
    s->ipscales[i] = fx + fy;
  }
  s->gwidths.resize(s->num); s->gheights.resize(s->num);
  for (int i = 0; i < s->num; ++i) {
    s->gwidths[i] = (s->views[i].w[s->level] + s->csize - 1) / s->csize;
    s->gheights[i] = (s->views[i].h[s->level] + s->csize - 1) / s->csize;
  }
  return s;
}

void oracle_scene_destroy(void* p) { delete static_cast<OScene*>(p); }

void oracle_set_thresholds(void* p, float ncc, float before, int depth) {
  OScene* s = static_cast<OScene*>(p);
  s->nccThreshold = ncc;
  s->nccThresholdBefore = before;
  s->depth = depth;
}

int oracle_get_level(void* p, int view, int level, uint8_t* out, int* w, int* h) {
  const OScene* s = static_cast<const OScene*>(p);
  if (view < 0 || view >= s->num || level < 0 || level >= s->maxLevel) return 1;
  const OView& v = s->views[view];
  *w = v.w[level];
  *h = v.h[level];
  if (out) std::memcpy(out, v.img[level].data(), v.img[level].size());
  return 0;
}

// Camera/axes values for pinning against oracle/_ref: out[0..3] center, [4..7] oaxis,
// [8..10] xaxis, [11..13] yaxis, [14..16] zaxis, [17] ipscale, [18..29] P at `level`.
void oracle_camera(void* p, int view, int level, float* out) {
  const OScene* s = static_cast<const OScene*>(p);
  const OView& v = s->views[view];
  for (int i = 0; i < 4; ++i) { out[i] = v.center[i]; out[4 + i] = v.oaxis[i]; }
  for (int i = 0; i < 3; ++i) { out[8 + i] = s->xaxes[view][i]; out[11 + i] = s->yaxes[view][i]; out[14 + i] = s->zaxes[view][i]; }
  out[17] = s->ipscales[view];
  for (int y = 0; y < 3; ++y)
    for (int x = 0; x < 4; ++x) out[18 + 4 * y + x] = v.P[level][y][x];
}

void oracle_project(void* p, int view, int level, const float* coords4, int n, float* out3) {
  const OScene* s = static_cast<const OScene*>(p);
  for (int i = 0; i < n; ++i) {
    V4 c = {{coords4[4 * i], coords4[4 * i + 1], coords4[4 * i + 2], coords4[4 * i + 3]}};
    const V3 r = project(*s, view, c, level);
    out3[3 * i] = r[0]; out3[3 * i + 1] = r[1]; out3[3 * i + 2] = r[2];
  }
}

void oracle_grab_tex(void* p, const pmvs_tex_query* q, int n, float* out, int* valid) {
  const OScene* s = static_cast<const OScene*>(p);
  const int len = 3 * s->wsize * s->wsize;
  std::vector<float> tex;
  for (int i = 0; i < n; ++i) {
    V4 c, px, py, pz;
    for (int k = 0; k < 4; ++k) { c[k] = q[i].coord[k]; px[k] = q[i].pxaxis[k]; py[k] = q[i].pyaxis[k]; pz[k] = q[i].normal[k]; }
    const int flag = grab_tex(*s, c, px, py, pz, q[i].view, s->wsize, tex);
    valid[i] = (flag == 0);
    if (flag == 0) {
      if (q[i].normalize) normalize(tex);
      std::memcpy(out + (size_t)i * len, tex.data(), len * sizeof(float));
    } else {
      std::memset(out + (size_t)i * len, 0, len * sizeof(float));
    }
  }
}

// get_color at n (x, y) points of one view/level (pinned against the reference's inline
// CImage::getColor through oracle/_ref ref_get_color): out 3 floats per point.
void oracle_get_color(void* p, int view, int level, const float* xy, int n, float* out3) {
  const OScene* s = static_cast<const OScene*>(p);
  for (int i = 0; i < n; ++i) {
    const V3 c = get_color(*s, view, xy[2 * i], xy[2 * i + 1], level);
    out3[3 * i] = c[0]; out3[3 * i + 1] = c[1]; out3[3 * i + 2] = c[2];
  }
}

// The organizer's depth (optical axis . coord) per point, as the filter oracle's depth_of.
void oracle_depth(void* p, int view, const float* coords4, int n, float* out) {
  const OScene* s = static_cast<const OScene*>(p);
  for (int i = 0; i < n; ++i) {
    V4 c = {{coords4[4 * i], coords4[4 * i + 1], coords4[4 * i + 2], coords4[4 * i + 3]}};
    out[i] = dot4(s->views[view].oaxis, c);
  }
}

// findEmptyBlocks' candidate centres for all 6 directions of (coord, normal, radius):
// ortho() then candidate_coord(); out 24 floats per query.
void oracle_expand_dirs(const float* coord4, const float* normal4, const float* radius, int n, float* out) {
  for (int q = 0; q < n; ++q) {
    V4 c, nn, xd, yd;
    for (int k = 0; k < 4; ++k) { c[k] = coord4[4 * q + k]; nn[k] = normal4[4 * q + k]; }
    ortho4(nn, xd, yd);
    for (int i = 0; i < 6; ++i) {
      const V4 r = candidate_coord(c, xd, yd, radius[q], i, 6);
      for (int k = 0; k < 4; ++k) out[24 * q + 4 * i + k] = r[k];
    }
  }
}

// getPAxes for test queries: out 8 floats (pxaxis, pyaxis).
void oracle_paxes(void* p, int view, const float* coord, const float* normal, float* out) {
  const OScene* s = static_cast<const OScene*>(p);
  V4 c, n, px, py;
  for (int k = 0; k < 4; ++k) { c[k] = coord[k]; n[k] = normal[k]; }
  get_paxes(*s, view, c, n, px, py);
  for (int k = 0; k < 4; ++k) { out[k] = px[k]; out[4 + k] = py[k]; }
}

// Sets up the refinePatchBFGS state of each query (as refine_patch does, without the
// optimizer) and evaluates my_f at q.x.  Also returns the encode() of the query's own
// geometry in enc (3 doubles per query) if enc != NULL.
void oracle_incc_eval(void* p, const pmvs_eval_query* q, int n, double* out, double* enc) {
  const OScene* s = static_cast<const OScene*>(p);
  OCtx c;
  init_ctx(*s, c);
  for (int i = 0; i < n; ++i) {
    OPatch pt;
    for (int k = 0; k < 4; ++k) { pt.coord[k] = q[i].coord[k]; pt.normal[k] = q[i].normal[k]; }
    pt.dscale = q[i].dscale;
    pt.images.assign(q[i].images, q[i].images + std::min(q[i].num_images, (int)PMVS_MAX_TAU));
    c.center = pt.coord;
    c.ray = sub4(pt.coord, s->views[pt.images[0]].center);
    unitize4(c.ray);
    c.indexes = pt.images;
    c.dscale = pt.dscale;
    c.ascale = (float)(M_PI / 48.0f);
    if (enc) encode(*s, c, pt.coord, pt.normal, enc + 3 * i);
    out[i] = my_f(*s, c, q[i].x);
  }
}

// Full preProcess -> refinePatch -> postProcess over a batch with nthreads std::threads
// (the reference's threading model: one scratch context per thread, expand.cpp:41-52).
void oracle_refine_batch(void* p, const pmvs_candidate* in, int n, pmvs_refined* out, int nthreads,
                         pmvs_stats* st) {
  const OScene* s = static_cast<const OScene*>(p);
  if (nthreads < 1) nthreads = 1;
  std::atomic<int> next(0);
  std::vector<OCtx> ctx(nthreads);
  auto work = [&](int t) {
    OCtx& c = ctx[t];
    init_ctx(*s, c);
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= n) break;
      refine_one(*s, c, in[i], out[i]);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->candidates = n;
    for (int i = 0; i < n; ++i) {
      if (out[i].status == PMVS_ACCEPTED) st->accepted++;
      if (out[i].status == PMVS_FAIL_PRE) st->fail_pre++;
      if (out[i].status == PMVS_FAIL_POST) st->fail_post++;
      if (out[i].status != PMVS_FAIL_PRE && !(out[i].refine_code >= 1 && out[i].refine_code <= 4)) st->refine_failed++;
    }
    for (auto& c : ctx) { st->evals += c.evals; st->tex_valid += c.tex_valid; st->tex_grabs += c.tex_grabs; }
  }
}

// Standalone BOBYQA on test objectives (for the device-BOBYQA parity test):
// kind 0 = quadratic, 1 = Rosenbrock-3, 2 = bound-active quadratic. Records up to maxrec f values.
int oracle_bobyqa_test(int kind, const double* x0, int maxeval, double* xout, double* fout, double* frec,
                       int maxrec, int* nrec) {
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999}, ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  double x[3] = {x0[0], x0[1], x0[2]};
  int cnt = 0;
  auto f = [&](const double* v) {
    double r;
    if (kind == 0) r = (v[0] - 1.5) * (v[0] - 1.5) + 2 * (v[1] - 3) * (v[1] - 3) + 0.5 * (v[2] + 2) * (v[2] + 2) + 0.1 * v[0] * v[1];
    else if (kind == 1) {
      const double a = 1 - v[0], b = v[1] - v[0] * v[0], c = v[2] - v[1] * v[1];
      r = a * a + 100 * b * b + 100 * c * c;
    } else r = (v[0] - 1) * (v[0] - 1) + (v[1] - 40) * (v[1] - 40) + (v[2] + 50) * (v[2] + 50);
    if (cnt < maxrec) frec[cnt] = r;
    cnt++;
    return r;
  };
  double minf = 0;
  int ne = 0;
  const int rc = bobyqa_minimize(x, lb, ub, 1e-7, maxeval, f, &minf, &ne);
  for (int i = 0; i < 3; ++i) xout[i] = x[i];
  *fout = minf;
  *nrec = cnt;
  return rc;
}

// One CFilter::run pass (filter_oracle.h).  counts[4]: removed by outside/exact/neighbor/groups.
// Thread count of the filter's per-patch stages (filter_oracle.h g_threads); results are
// independent of it.
void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }

// CFindMatch::isNeighbor(lhs, rhs, hunit, thr) and isNeighborRadius (findMatch.cpp:125-185) as
// restated in filter_oracle.h (is_neighbor_h), on records of 21 floats (lhs coord[4] normal[4] dscale,
// rhs coord[4] normal[4] dscale, hunit, threshold, radius): out[2i] / out[2i + 1].  Pinned against
// the reference's own findMatch.cpp by tests/test_isneighbor_pinning.py.
void oracle_is_neighbor(const float* in, int n, int* out) {
  for (int i = 0; i < n; ++i) {
    const float* r = in + (size_t)i * 21;
    FPatch l, q;
    for (int k = 0; k < 4; ++k) {
      l.coord[k] = r[k]; l.normal[k] = r[4 + k];
      q.coord[k] = r[9 + k]; q.normal[k] = r[13 + k];
    }
    l.dscale = r[8];
    q.dscale = r[17];
    out[2 * i] = is_neighbor_h(l, q, r[18], r[19], 0.0f, false);
    out[2 * i + 1] = is_neighbor_h(l, q, r[18], r[19], r[20], true);
  }
}

void oracle_filter_run(void* h, pmvs_patch* patches, int n, int* keep, int* counts) {
  const OScene& s = *static_cast<const OScene*>(h);
  std::vector<FPatch> P(n);
  parallel_for(g_threads, (size_t)n, [&](int, size_t i) {
    const pmvs_patch& a = patches[i];
    FPatch& q = P[i];
    for (int k = 0; k < 4; ++k) { q.coord[k] = a.coord[k]; q.normal[k] = a.normal[k]; }
    q.ncc = a.ncc; q.dscale = a.dscale; q.ascale = a.ascale; q.tmp = a.tmp;
    q.timages = a.timages; q.flag = a.flag; q.fix = a.fix; q.dflag = a.dflag;
    for (int k = 0; k < a.num_images; ++k) { q.images.push_back(a.images[k]); q.grids.push_back({a.grids[k][0], a.grids[k][1]}); }
    for (int k = 0; k < a.num_vimages; ++k) { q.vimages.push_back(a.vimages[k]); q.vgrids.push_back({a.vgrids[k][0], a.vgrids[k][1]}); }
  });
  std::vector<int> kp;
  filter_run(s, P, kp, counts);
  parallel_for(g_threads, (size_t)n, [&](int, size_t ii) {
    const int i = (int)ii;
    pmvs_patch& a = patches[i];
    const FPatch& q = P[i];
    a.timages = q.timages;
    a.flag = q.flag;
    a.num_images = list_len(q.images.size());
    for (int k = 0; k < a.num_images; ++k) {
      a.images[k] = (int16_t)q.images[k]; a.grids[k][0] = cell16(q.grids[k].first); a.grids[k][1] = cell16(q.grids[k].second);
    }
    a.num_vimages = list_len(q.vimages.size());
    for (int k = 0; k < a.num_vimages; ++k) {
      a.vimages[k] = (int16_t)q.vimages[k]; a.vgrids[k][0] = cell16(q.vgrids[k].first); a.vgrids[k][1] = cell16(q.vgrids[k].second);
    }
    keep[i] = kp[i];
  });
}

// Diagnostic: filterNeighbor's neighbour-list sizes (raw with duplicates, unique) on the
// organizer state right before filterNeighbor in a pass that skips outside/exact.
void oracle_neighbor_sizes(void* h, pmvs_patch* patches, int n, int* raw, int* uniq) {
  const OScene& s = *static_cast<const OScene*>(h);
  std::vector<FPatch> P(n);
  for (int i = 0; i < n; ++i) {
    const pmvs_patch& a = patches[i];
    FPatch& q = P[i];
    for (int k = 0; k < 4; ++k) { q.coord[k] = a.coord[k]; q.normal[k] = a.normal[k]; }
    q.ncc = a.ncc; q.dscale = a.dscale; q.ascale = a.ascale; q.tmp = a.tmp;
    q.timages = a.timages; q.flag = a.flag; q.fix = a.fix;
    for (int k = 0; k < a.num_images; ++k) { q.images.push_back(a.images[k]); q.grids.push_back({a.grids[k][0], a.grids[k][1]}); }
  }
  Organizer o(s);
  for (int p = 0; p < n; ++p) add_patch_p(o, P, p);
  set_dm_vgrids(o, P, 0);
  for (int p = 0; p < n; ++p) {
    std::vector<int> nb;
    find_neighbors(o, P, P[p], nb, 4.0f, 2, 1);
    uniq[p] = (int)nb.size();
    raw[p] = 0;
  }
}

static void to_fpatch(const pmvs_patch& a, FPatch& q) {
  for (int k = 0; k < 4; ++k) { q.coord[k] = a.coord[k]; q.normal[k] = a.normal[k]; }
  q.ncc = a.ncc; q.dscale = a.dscale; q.ascale = a.ascale; q.tmp = a.tmp;
  q.timages = a.timages; q.flag = a.flag; q.fix = a.fix; q.dflag = a.dflag;
  q.images.clear(); q.grids.clear(); q.vimages.clear(); q.vgrids.clear();
  for (int k = 0; k < a.num_images; ++k) { q.images.push_back(a.images[k]); q.grids.push_back({a.grids[k][0], a.grids[k][1]}); }
  for (int k = 0; k < a.num_vimages; ++k) { q.vimages.push_back(a.vimages[k]); q.vgrids.push_back({a.vgrids[k][0], a.vgrids[k][1]}); }
}
static void from_fpatch(const FPatch& q, pmvs_patch& a) {
  std::memset(&a, 0, sizeof(a));
  for (int k = 0; k < 4; ++k) { a.coord[k] = q.coord[k]; a.normal[k] = q.normal[k]; }
  a.ncc = q.ncc; a.dscale = q.dscale; a.ascale = q.ascale; a.tmp = q.tmp;
  a.timages = q.timages; a.flag = q.flag; a.fix = q.fix; a.dflag = q.dflag;
  a.num_images = list_len(q.images.size());
  for (int k = 0; k < a.num_images; ++k) {
    a.images[k] = (int16_t)q.images[k]; a.grids[k][0] = cell16(q.grids[k].first); a.grids[k][1] = cell16(q.grids[k].second);
  }
  a.num_vimages = list_len(q.vimages.size());
  for (int k = 0; k < a.num_vimages; ++k) {
    a.vimages[k] = (int16_t)q.vimages[k]; a.vgrids[k][0] = cell16(q.vgrids[k].first); a.vgrids[k][1] = cell16(q.vgrids[k].second);
  }
}

// One CExpand::run (expand_oracle.h) on the model (patches[i], alive[i]).  Writes the updated
// model (old patches first, new ones appended) to out/alive_out (capacity cap); returns the new
// patch count or -1 when cap is too small.  stats: parents, candidates, fail_prep, fail_pre,
// fail_post, fail_commit, added, waves, wave_ns (9 entries).
int oracle_expand_run(void* h, const pmvs_patch* patches, const int* alive, int n, int wave, int cthr, int flags,
                      int min_cands, pmvs_patch* out, int* alive_out, int cap, int64_t* stats, int nthreads,
                      int64_t max_waves) {
  const OScene& s = *static_cast<const OScene*>(h);
  // the organizer's per-target loops (collect, depth maps, vpgrids) use the same pool size
  const int saved = g_threads;
  g_threads = std::max(g_threads, nthreads);
  std::vector<FPatch> P(n);
  std::vector<int> al(alive, alive + n);
  parallel_for(g_threads, (size_t)n, [&](int, size_t i) { to_fpatch(patches[i], P[i]); });
  ExpandStats st;
  expand_run(s, P, al, wave, cthr, flags, st, min_cands, nthreads, max_waves);
  if ((int)P.size() > cap) {
    g_threads = saved;
    return -1;
  }
  parallel_for(g_threads, P.size(), [&](int, size_t i) {
    from_fpatch(P[i], out[i]);
    alive_out[i] = al[i];
  });
  g_threads = saved;
  const int64_t v[9] = {st.parents, st.candidates, st.fail_prep, st.fail_pre, st.fail_post, st.fail_commit, st.added,
                        st.waves, st.wave_ns};
  for (int k = 0; k < 9; ++k) stats[k] = v[k];
  return (int)P.size();
}


// ---- seed phase (seed_oracle.h)
static std::vector<std::vector<SeedPoint>> split_points(const OScene& s, const pmvs_point* pts, const int* npts) {
  std::vector<std::vector<SeedPoint>> v(s.num);
  size_t k = 0;
  for (int i = 0; i < s.num; ++i)
    for (int q = 0; q < npts[i]; ++q, ++k) v[i].push_back({pts[k].x, pts[k].y, pts[k].response, pts[k].type});
  return v;
}

// CSeed::run (CPU 1) from the feature points of every view (pts: npts[0] points of view 0, then
// view 1, ...).  Writes the seed patches in addPatch order; returns their number, or -1 when cap
// is too small.  stats: trial, pass, fail0 (preProcess), fail1 (postProcess).
int oracle_seed_run(void* h, const pmvs_point* pts, const int* npts, pmvs_patch* out, int cap, int64_t* stats) {
  const OScene& s = *static_cast<const OScene*>(h);
  std::vector<pmvs_patch> seeds;
  int64_t st[4];
  seed_run(s, split_points(s, pts, npts), seeds, st);
  for (int k = 0; k < 4; ++k) stats[k] = st[k];
  if ((int)seeds.size() > cap) return -1;
  std::memcpy(out, seeds.data(), seeds.size() * sizeof(pmvs_patch));
  return (int)seeds.size();
}

// Diagnostics for the parity tests: collectImages of every view (tau entries max, -1 padded),
// the seed job order, and the sorted candidate list of one feature point against the empty
// model (view, point, cell, coord[4], response per entry; returns the count, -1 if cap is short).
void oracle_seed_images(void* h, int* out_images, int* out_order) {
  const OScene& s = *static_cast<const OScene*>(h);
  std::vector<std::vector<float>> dist;
  set_distances(s, dist);
  std::vector<int> idx;
  for (int i = 0; i < s.num; ++i) {
    collect_images(s, dist, i, idx);
    for (int k = 0; k < s.tau; ++k) out_images[i * s.tau + k] = k < (int)idx.size() ? idx[k] : -1;
  }
  const std::vector<int> order = seed_order(s.tnum);
  for (int i = 0; i < s.tnum; ++i) out_order[i] = order[i];
}

int oracle_seed_candidates(void* h, const pmvs_point* pts, const int* npts, int index, int point, int* out_int,
                           float* out_f, int cap) {
  const OScene& s = *static_cast<const OScene*>(h);
  SeedState st(s);
  st.pts = split_points(s, pts, npts);
  st.cells.resize(s.num);
  for (int i = 0; i < s.num; ++i) {
    st.cells[i].assign((size_t)s.gwidths[i] * s.gheights[i], std::vector<int>());
    for (int q = 0; q < (int)st.pts[i].size(); ++q) {
      const int ix = ((int)std::floor(st.pts[i][q].x + 0.5f)) / s.csize;
      const int iy = ((int)std::floor(st.pts[i][q].y + 0.5f)) / s.csize;
      st.cells[i][iy * s.gwidths[i] + ix].push_back(q);
    }
  }
  st.counts.resize(s.tnum);
  st.occupied.resize(s.tnum);
  for (int t = 0; t < s.tnum; ++t) {
    st.counts[t].assign((size_t)s.gwidths[t] * s.gheights[t], 0);
    st.occupied[t].assign((size_t)s.gwidths[t] * s.gheights[t], 0);
  }
  set_distances(s, st.dist);
  std::vector<int> idx;
  collect_images(s, st.dist, index, idx);
  std::vector<SeedCand> vcp;
  collect_candidates(st, index, idx, st.pts[index][point], vcp);
  if ((int)vcp.size() > cap) return -1;
  for (size_t k = 0; k < vcp.size(); ++k) {
    out_int[3 * k] = vcp[k].view; out_int[3 * k + 1] = vcp[k].point; out_int[3 * k + 2] = vcp[k].cell;
    for (int c = 0; c < 4; ++c) out_f[5 * k + c] = vcp[k].coord[c];
    out_f[5 * k + 4] = vcp[k].response;
  }
  return (int)vcp.size();
}

// Image::setF / computeEPD / CSeed::unproject on explicit inputs (pinned against the reference
// headers by tests/test_seed_pinning.py).
void oracle_seed_geometry(void* h, int i0, int i1, const float* xy0, const float* xy1, int n, double* F9, float* epd,
                          float* coords4) {
  const OScene& s = *static_cast<const OScene*>(h);
  double F[3][3];
  set_f(s, i0, i1, F);
  for (int i = 0; i < 9; ++i) F9[i] = F[i / 3][i % 3];
  for (int k = 0; k < n; ++k) {
    const double p0[3] = {xy0[2 * k], xy0[2 * k + 1], 1.0}, p1[3] = {xy1[2 * k], xy1[2 * k + 1], 1.0};
    epd[k] = compute_epd(F, p0, p1);
    const SeedPoint a{xy0[2 * k], xy0[2 * k + 1], 0.0f, 0}, b{xy1[2 * k], xy1[2 * k + 1], 0.0f, 0};
    const V4 c = unproject(s, i0, i1, a, b);
    for (int j = 0; j < 4; ++j) coords4[4 * k + j] = c[j];
  }
}


// Cmylapack::lls restated (filter_oracle.h lls5) on an n x 5 float system, for tests/test_lls.py.
void oracle_lls5(const float* A, const float* b, int n, float* x) {
  std::vector<std::array<float, 5>> a(n);
  std::vector<float> bb(b, b + n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 5; ++j) a[i][j] = A[5 * i + j];
  lls5(a, bb, x);
}

}  // extern "C"
