// pmvs_refine.h -- device pieces of refinePatchBFGS shared by the refine kernels' translation units
// (pmvs_kernels.hip: pre / wavefront / workgroup forms and post; pmvs_refine_split.hip: split form).
#pragma once
#include <hip/hip_runtime.h>

#include "bobyqa_dev.h"
#include "pmvs_device.h"

namespace pmvsdev {

constexpr int WAVE = 64;
__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

__device__ __forceinline__ int wave_excl_scan(int v) {
  const int lane = lane_id();
  int incl = v;
  for (int d = 1; d < WAVE; d <<= 1) {
    const int t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  return incl - v;
}

// ---------------------------------------------------------------- encode / decode
struct RefineSetup {
  float center[4], ray[4];
  float dscale, ascale;
  int ref;  // _indexesT[id][0]
};

// COptim::decode, optim.cpp:690-707.
__device__ __forceinline__ void decode(const DScene& s, const RefineSetup& R, const double* vect, float* coord,
                                       float* normal) {
  const double sc = (double)R.dscale * vect[0];
  for (int i = 0; i < 4; ++i) coord[i] = R.center[i] + (float)((double)R.ray[i] * sc);
  const DView& v = s.views[R.ref];
  const float angle1 = (float)(vect[1] * (double)R.ascale);
  const float angle2 = (float)(vect[2] * (double)R.ascale);
  const double ca2 = cos((double)angle2);
  const float fx = (float)(sin((double)angle1) * ca2);
  const float fy = (float)sin((double)angle2);
  const float fz = (float)(-cos((double)angle1) * ca2);
  for (int i = 0; i < 3; ++i) normal[i] = (v.xaxis[i] * fx + v.yaxis[i] * fy) + v.zaxis[i] * fz;
  normal[3] = 0.0f;
}

// setup, one thread per texture: grabTex optim.cpp:818-846 + grabSafe :783-805.  tex_geom computes a
// texture's sampling frame (validity, pyramid level, top-left sample, steps) from the request's
// geometry g (coord, normal, pxaxis, pyaxis); tex_setup stores it in the kernel's LDS slot.
struct TexGeom {
  int ok, W;
  long long base;
  float tl0, tl1, dx0, dx1, dy0, dy1;
};
template <int WS>
__device__ __forceinline__ TexGeom tex_geom(const DScene& s, const float* g, int index) {
  const float coord[4] = {g[0], g[1], g[2], g[3]}, pz[4] = {g[4], g[5], g[6], g[7]};
  const float px[4] = {g[8], g[9], g[10], g[11]}, py[4] = {g[12], g[13], g[14], g[15]};
  const DView& v = s.views[index];
  int ok = 1;
  float ray[4] = {v.center[0] - coord[0], v.center[1] - coord[1], v.center[2] - coord[2], v.center[3] - coord[3]};
  unitize4(ray);
  const float weight = smax(0.0f, dot4(ray, pz));
  if ((double)weight < s.cosAngle1) ok = 0;
  float center[3], c1[3], c2[3], tt[4];
  project(v, coord, s.level, center);
  for (int i = 0; i < 4; ++i) tt[i] = coord[i] + px[i];
  project(v, tt, s.level, c1);
  for (int i = 0; i < 4; ++i) tt[i] = coord[i] + py[i];
  project(v, tt, s.level, c2);
  float dx[3] = {c1[0] - center[0], c1[1] - center[1], c1[2] - center[2]};
  float dy[3] = {c2[0] - center[0], c2[1] - center[1], c2[2] - center[2]};
  const float ratio = __fdiv_rn(norm3(dx) + norm3(dy), 2.0f);
  int leveldif = cvt_int_x86(floor(log((double)ratio) / (double)s.log2f + (double)0.5f));
  leveldif = imax(-s.level, imin(2, leveldif));
  const float scale = (leveldif >= 0) ? (float)(1 << leveldif) : __fdiv_rn(1.0f, (float)(1 << (-leveldif)));
  const int newlevel = s.level + leveldif;
  for (int i = 0; i < 3; ++i) {
    center[i] = __fdiv_rn(center[i], scale);
    dx[i] = __fdiv_rn(dx[i], scale);
    dy[i] = __fdiv_rn(dy[i], scale);
  }
  const float fm = (float)(WS / 2);
  const float dxm[2] = {dx[0] * fm, dx[1] * fm}, dym[2] = {dy[0] * fm, dy[1] * fm};
  const float tl0 = (center[0] - dxm[0]) - dym[0], tl1 = (center[1] - dxm[1]) - dym[1];
  const float tr0 = (center[0] + dxm[0]) - dym[0], tr1 = (center[1] + dxm[1]) - dym[1];
  const float bl0 = (center[0] - dxm[0]) + dym[0], bl1 = (center[1] - dxm[1]) + dym[1];
  const float br0 = (center[0] + dxm[0]) + dym[0], br1 = (center[1] + dxm[1]) + dym[1];
  const float minx = smin(tl0, smin(tr0, smin(bl0, br0)));
  const float maxx = smax(tl0, smax(tr0, smax(bl0, br0)));
  const float miny = smin(tl1, smin(tr1, smin(bl1, br1)));
  const float maxy = smax(tl1, smax(tr1, smax(bl1, br1)));
  if (ok && (minx < 3.0f || (float)(v.w[newlevel] - 1 - 3) <= maxx || miny < 3.0f ||
             (float)(v.h[newlevel] - 1 - 3) <= maxy))
    ok = 0;
  TexGeom T;
  T.ok = ok;
  T.W = v.w[newlevel];
  T.base = v.pyr_off[newlevel];
  T.tl0 = tl0; T.tl1 = tl1;
  T.dx0 = dx[0]; T.dx1 = dx[1];
  T.dy0 = dy[0]; T.dy1 = dy[1];
  return T;
}
// The objective value of one request from its slots [off, off + sz): COptim::my_f
// (optim.cpp:527-577, need 1) or the robust weighted computeINCC (optim.cpp:875-938, need 2).
template <class L>
__device__ __forceinline__ double request_value(const DScene& s, const L& C, int off, int sz, int need,
                                                const RefineJob& J, unsigned long long& tex_valid) {
  const int ref = off;
  int nv = 0;
  for (int i = 0; i < sz; ++i) nv += C.jvalid[off + i];
  double f;
  if (need == 1) {
    const int mininum = imin(s.minImageNum, sz);
    tex_valid += nv;
    if (!C.jvalid[ref]) {
      f = 2.0;
    } else {
      double ans = 0.0f;
      int denom = 0;
      for (int i = 1; i < sz; ++i) {
        if (!C.jvalid[off + i]) continue;
        ans += (double)C.jres[off + i];
        denom++;
      }
      f = (denom < mininum - 1) ? 2.0f : ans / denom;
    }
  } else {
    if (!C.jvalid[ref]) {
      f = 2.0;
    } else {
      double score = 0.0;
      float totalweight = 0.0f;
      for (int i = 1; i < sz; ++i) {
        if (C.jvalid[off + i]) {
          const float w = J.weights[i];
          totalweight += w;
          score += (double)(C.jres[off + i] * w);
        }
      }
      f = (totalweight == 0.0f) ? 2.0 : score / (double)totalweight;
    }
  }
  return f;
}

// Wavefronts per SIMD the refine kernel's register budget is sized for: 2 (<= 256 VGPR+AGPR).  The
// out-of-line BOBYQA routines get the budget of their most permissive caller, so the self-test
// kernels that call them use the same value.  Measured on C2 (tools/sweep_variants.sh,
// profiles/r02g_sweeps.txt): 2 waves of 4 chains with 12 texture slots (19 KB LDS, 8 per CU)
// beat 1 wave of 8 chains with the 512-register inlined optimizer by 17 %; 3 or 4 waves per SIMD
// (168 / 128 registers) spill and lose 40-50 %.  With the compacted BqState (1736 B) and 12-byte
// texture samples, 6 chains x 12 slots fit the same 20 KB (default 1206, +6 %).
#ifndef REFINE_WPE
#define REFINE_WPE(NC) 2
#endif
#ifndef BQ_CALLER_WPE
#define BQ_CALLER_WPE 2
#endif
}  // namespace pmvsdev
