// pmvs_device.h -- device-side scene layout and the per-wave PMVS photo-consistency primitives.
//
// Layout in HBM (built once by pmvs_scene_create, pmvs_api.hip):
//   * pyr: every view's image pyramid (level+3 levels, CImage::_images, reference
//     image.cpp:113-140,228-325) re-packed as RGBA8 words (one 32-bit word per pixel, A = 0),
//     one contiguous slab per (view, level).  A bilinear sample (CImage::getColor,
//     image.hpp:435-476) is then 4 aligned dword loads instead of 12 byte loads.
//   * DView: per view, the 3x4 projection of every level (CCamera::_projection), optical
//     centre, the COptim::setAxesScales axes and ipscale (optim.cpp:43-64), level sizes.
//   * masks/edges (optional): one byte per pixel per level.
// Everything a COptim::my_f evaluation reads is here; nothing is re-uploaded per call.
//
// Numerics: every function below restates the reference's float/double operation order
// (see oracle/pmvs_oracle.cpp for the same restatement on the CPU).  Compiled with
// -ffp-contract=off and IEEE-rounded f32 division/sqrt so results are bit-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pmvs_layout.h"

namespace pmvsdev {

// ------------------------------------------------------------------ small vector math
// TVec4/TVec3 operator order (reference include/numeric/vec4.hpp, vec3.hpp).
__device__ __forceinline__ float dot4(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}
__device__ __forceinline__ float dot3(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
// norm(): sqrt of a float via the double C sqrt == correctly rounded f32 sqrt.  HIP's
// __fsqrt_rn is the 1-ulp native sqrt unless OCML_BASIC_ROUNDED_OPERATIONS is defined;
// __builtin_sqrtf lowers to v_sqrt_f32 + the neighbour-correction sequence (IEEE rounded).
__device__ __forceinline__ float fsqrt_rn(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ float norm3(const float* a) { return fsqrt_rn(dot3(a, a)); }
__device__ __forceinline__ float norm4(const float* a) { return fsqrt_rn(dot4(a, a)); }
__device__ __forceinline__ void unitize4(float* v) {
  const float l = dot4(v, v);
  if (l != 1.0f && l != 0.0f) {
    const float d = fsqrt_rn(l);
    v[0] = __fdiv_rn(v[0], d); v[1] = __fdiv_rn(v[1], d); v[2] = __fdiv_rn(v[2], d); v[3] = __fdiv_rn(v[3], d);
  }
}
__device__ __forceinline__ void unitize3(float* v) {
  const float l = dot3(v, v);
  if (l != 1.0f && l != 0.0f) {
    const float d = fsqrt_rn(l);
    v[0] = __fdiv_rn(v[0], d); v[1] = __fdiv_rn(v[1], d); v[2] = __fdiv_rn(v[2], d);
  }
}
__device__ __forceinline__ void cross3(const float* u, const float* v, float* o) {
  o[0] = u[1] * v[2] - v[1] * u[2];
  o[1] = -u[0] * v[2] + v[0] * u[2];
  o[2] = u[0] * v[1] - v[0] * u[1];
}
// std::min / std::max argument semantics.
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ int imin(int a, int b) { return (b < a) ? b : a; }
__device__ __forceinline__ int imax(int a, int b) { return (a < b) ? b : a; }
// (int) of a double as x86-64 cvttsd2si: NaN / out of range -> INT_MIN (the reference runs there).
__device__ __forceinline__ int cvt_int_x86(double d) {
  if (!(d > -2147483649.0 && d < 2147483648.0)) return (int)0x80000000;
  return (int)d;
}

// CCamera::project, camera.hpp:89-108.
__device__ __forceinline__ void project(const DView& v, const float* c, int level, float* out) {
  const float* P = v.P[level];
  float v0 = P[0] * c[0] + P[1] * c[1] + P[2] * c[2] + P[3] * c[3];
  float v1 = P[4] * c[0] + P[5] * c[1] + P[6] * c[2] + P[7] * c[3];
  float v2 = P[8] * c[0] + P[9] * c[1] + P[10] * c[2] + P[11] * c[3];
  if (v2 <= 0.0f) {
    out[0] = -65535.0f; out[1] = -65535.0f; out[2] = -1.0f;
    return;
  }
  const float d = v2;
  v0 = __fdiv_rn(v0, d); v1 = __fdiv_rn(v1, d); v2 = __fdiv_rn(v2, d);
  const float lo = -2147483648.0f, hi = 2147483648.0f;  // (float)(INT_MIN + 3.0f), (float)(INT_MAX - 3.0f)
  out[0] = smax(lo, smin(hi, v0));
  out[1] = smax(lo, smin(hi, v1));
  out[2] = v2;
}

// COptim::getUnit, optim.cpp:1116-1124.
__device__ __forceinline__ float get_unit(const DScene& s, const DView& v, const float* coord) {
  const float d[4] = {coord[0] - v.center[0], coord[1] - v.center[1], coord[2] - v.center[2], coord[3] - v.center[3]};
  const float fz = norm4(d);
  const float ftmp = v.ipscale;
  if (ftmp == 0.0f) return 1.0f;
  return (float)(2.0 * (double)fz * (double)(1 << s.level) / (double)ftmp);
}

// COptim::getPAxes, optim.cpp:1127-1144.
__device__ __forceinline__ void get_paxes(const DScene& s, const DView& v, const float* coord, const float* normal,
                                          float* px, float* py) {
  const float pscale = get_unit(s, v, coord);
  const float n3[3] = {normal[0], normal[1], normal[2]};
  float y3[3], x3[3];
  cross3(n3, v.xaxis, y3);
  unitize3(y3);
  cross3(y3, n3, x3);
  px[0] = x3[0] * pscale; px[1] = x3[1] * pscale; px[2] = x3[2] * pscale; px[3] = 0.0f * pscale;
  py[0] = y3[0] * pscale; py[1] = y3[1] * pscale; py[2] = y3[2] * pscale; py[3] = 0.0f * pscale;
  float c0[3], c1[3], c2[3], t[4];
  project(v, coord, s.level, c0);
  for (int i = 0; i < 4; ++i) t[i] = coord[i] + px[i];
  project(v, t, s.level, c1);
  for (int i = 0; i < 4; ++i) t[i] = coord[i] + py[i];
  project(v, t, s.level, c2);
  const float dx[3] = {c1[0] - c0[0], c1[1] - c0[1], c1[2] - c0[2]};
  const float dy[3] = {c2[0] - c0[0], c2[1] - c0[1], c2[2] - c0[2]};
  const float xdis = norm3(dx), ydis = norm3(dy);
  for (int i = 0; i < 4; ++i) {
    px[i] = __fdiv_rn(px[i], xdis);
    py[i] = __fdiv_rn(py[i], ydis);
  }
}

// CImage::getColor bilinear branch, image.hpp:435-476, on the RGBA8 pyramid.
__device__ __forceinline__ void get_color(const DScene& s, const DView& v, float x, float y, int level, float* rgb) {
  const int lx = (int)x, ly = (int)y;
  const int W = v.w[level];
  const uint32_t* base = s.pyr + v.pyr_off[level] + (long long)ly * W + lx;
  const uint32_t a0 = base[0], a1 = base[1], b0 = base[W], b1 = base[W + 1];
  const float dx1 = x - (float)lx, dx0 = 1.0f - dx1;
  const float dy1 = y - (float)ly, dy0 = 1.0f - dy1;
  const float f00 = dx0 * dy0, f01 = dx0 * dy1, f10 = dx1 * dy0, f11 = dx1 * dy1;
  float r = 0.0f, g = 0.0f, b = 0.0f;
  r += (float)(a0 & 0xff) * f00 + (float)(b0 & 0xff) * f01;
  g += (float)((a0 >> 8) & 0xff) * f00 + (float)((b0 >> 8) & 0xff) * f01;
  b += (float)((a0 >> 16) & 0xff) * f00 + (float)((b0 >> 16) & 0xff) * f01;
  r += (float)(a1 & 0xff) * f10 + (float)(b1 & 0xff) * f11;
  g += (float)((a1 >> 8) & 0xff) * f10 + (float)((b1 >> 8) & 0xff) * f11;
  b += (float)((a1 >> 16) & 0xff) * f10 + (float)((b1 >> 16) & 0xff) * f11;
  rgb[0] = r; rgb[1] = g; rgb[2] = b;
}

// CPhoto::getEdge, photo.hpp:50-58 + CImage::getEdge image.hpp:554-581.
__device__ __forceinline__ int get_edge(const DScene& s, const DView& v, const float* coord, int level) {
  if (v.edge_off[level] < 0) return 1;
  float ic[3];
  project(v, coord, level, ic);
  if (ic[0] < 0 || (float)(v.w[level] - 1) <= ic[0] || ic[1] < 0 || (float)(v.h[level] - 1) <= ic[1]) return 0;
  const int ix = (int)floorf(ic[0] + 0.5f), iy = (int)floorf(ic[1] + 0.5f);
  if (ix < 0 || v.w[level] <= ix || iy < 0 || v.h[level] <= iy) return 1;
  return s.edges[v.edge_off[level] + (long long)iy * v.w[level] + ix];
}

// CPhoto::getMask for one view, photo.hpp:42-48 + image.hpp:522-550.
__device__ __forceinline__ int get_mask(const DScene& s, const DView& v, const float* coord, int level) {
  if (v.mask_off[level] < 0) return 1;
  float ic[3];
  project(v, coord, level, ic);
  const int ix = (int)floorf(ic[0] + 0.5f), iy = (int)floorf(ic[1] + 0.5f);
  if (ix < 0 || v.w[level] <= ix || iy < 0 || v.h[level] <= iy) return 1;
  return s.masks[v.mask_off[level] + (long long)iy * v.w[level] + ix];
}

__device__ __forceinline__ float robustincc(float rhs) { return __fdiv_rn(rhs, 1.0f + 3.0f * rhs); }
__device__ __forceinline__ float unrobustincc(float rhs) { return __fdiv_rn(rhs, 1.0f - 3.0f * rhs); }

}  // namespace pmvsdev
