// pmvs_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the PMVS2 hot path.
//
// Mapping:
//   * one 64-lane wavefront (= one workgroup) owns one patch candidate at a time and pulls
//     candidates from a device work queue (persistent grid, one dequeue per candidate);
//   * texture gather (COptim::grabTex, optim.cpp:815-863): one lane per (texture, sample) --
//     tau*wsize^2 = 294 bilinear samples over 64 lanes -- into an LDS texture tile;
//   * normalize / dot (optim.cpp:1031-1077): one lane per texture (resp. texture pair) runs the
//     reference's sequential float reduction from LDS, so every sum has the reference's rounding
//     sequence (bit-exact); element-wise normalisation uses all lanes;
//   * BOBYQA (NLopt LN_BOBYQA, optim.cpp:621-644): reverse-communication state machine
//     (bobyqa_dev.h) stepped by lane 0 with its state in LDS, the wave evaluates my_f;
//   * pre/postProcess image selection (optim.cpp:95-254): lane-parallel predicates with
//     order-preserving ballot compaction; order-dependent scalar loops on lane 0.
// No MFMA: this is gather + small reductions (HBM/L2-gather bound), see DESIGN.md.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>

#include "bobyqa_dev.h"
#include "pmvs_device.h"
#include "pmvs_refine.h"

namespace pmvsdev {

#ifndef REFINE_TSLOTS
#define REFINE_TSLOTS 48
#endif

template <int WS>
struct WaveLds {
  static constexpr int S = WS * WS;
  float tex[TEXCAP][S][4];  // RGB(+pad) per sample, sample-major like the reference vector
  float ave[TEXCAP][4];     // per-texture channel means and ave2
  int valid[TEXCAP];
  int jview[TEXCAP], jlevel[TEXCAP];
  float jrow[TEXCAP][WS][2], jdx[TEXCAP][2], jdy[TEXCAP][2];  // jrow: each sample row's start (left)
  float res[TEXCAP];        // per-texture result (inccs)
  int images[PMVS_MAX_IMAGES];
  int nimg;
  int list2[PMVS_MAX_IMAGES];
  float fl[PMVS_MAX_IMAGES];
  float fl2[PMVS_MAX_IMAGES];
  float rays[PMVS_MAX_IMAGES][4];
  int grids[PMVS_MAX_IMAGES][2];
  int cand;
  int overflow;
};

// Order-preserving compaction across the wave: returns the position of this lane's kept element
// among kept elements of lanes < lane, and writes the number kept to *count.
__device__ __forceinline__ int ballot_prefix(bool keep, int* count) {
  const unsigned long long m = __ballot(keep);
  *count = __popcll(m);
  const unsigned long long below = (lane_id() == 0) ? 0ull : (m & ((~0ull) >> (64 - lane_id())));
  return __popcll(below);
}

// ---------------------------------------------------------------- texture batch
// Grabs cnt (<= TEXCAP) textures: view jv(j) into LDS slot js(j), j < cnt, at the wave-uniform
// geometry (coord, px, py, normal); normalises the valid ones.  lds.valid[slot] is set.
template <int WS>
__device__ void grab_batch(const DScene& s, WaveLds<WS>& L, int cnt, const int* views, int slot0,
                           const float* coord, const float* px, const float* py, const float* pz,
                           unsigned long long* grabs) {
  constexpr int S = WS * WS;
  const int lane = lane_id();
  // --- per-texture setup (grabTex lines 818-846), one lane per texture
  if (lane < cnt) {
    const int slot = slot0 + lane;
    const int index = views[lane];
    const DView& v = s.views[index];
    int ok = 1;
    float ray[4] = {v.center[0] - coord[0], v.center[1] - coord[1], v.center[2] - coord[2], v.center[3] - coord[3]};
    unitize4(ray);
    const float weight = smax(0.0f, dot4(ray, pz));
    if ((double)weight < s.cosAngle1) ok = 0;
    const int margin = WS / 2;
    float center[3], c1[3], c2[3], t[4];
    project(v, coord, s.level, center);
    for (int i = 0; i < 4; ++i) t[i] = coord[i] + px[i];
    project(v, t, s.level, c1);
    for (int i = 0; i < 4; ++i) t[i] = coord[i] + py[i];
    project(v, t, s.level, c2);
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
    // grabSafe, optim.cpp:783-805
    const float fm = (float)margin;
    const float dxm[2] = {dx[0] * fm, dx[1] * fm}, dym[2] = {dy[0] * fm, dy[1] * fm};
    const float tl0 = (center[0] - dxm[0]) - dym[0], tl1 = (center[1] - dxm[1]) - dym[1];
    const float tr0 = (center[0] + dxm[0]) - dym[0], tr1 = (center[1] + dxm[1]) - dym[1];
    const float bl0 = (center[0] - dxm[0]) + dym[0], bl1 = (center[1] - dxm[1]) + dym[1];
    const float br0 = (center[0] + dxm[0]) + dym[0], br1 = (center[1] + dxm[1]) + dym[1];
    const float minx = smin(tl0, smin(tr0, smin(bl0, br0)));
    const float maxx = smax(tl0, smax(tr0, smax(bl0, br0)));
    const float miny = smin(tl1, smin(tr1, smin(bl1, br1)));
    const float maxy = smax(tl1, smax(tr1, smax(bl1, br1)));
    if (ok) {
      if (minx < 3.0f || (float)(v.w[newlevel] - 1 - 3) <= maxx || miny < 3.0f || (float)(v.h[newlevel] - 1 - 3) <= maxy)
        ok = 0;
    }
    L.valid[slot] = ok;
    L.jview[slot] = index;
    L.jlevel[slot] = newlevel;
    float lx = tl0, ly = tl1;  // rows' starts: `left += dy` (optim.cpp:850-860), once per texture
    for (int r = 0; r < WS; ++r) {
      L.jrow[slot][r][0] = lx; L.jrow[slot][r][1] = ly;
      lx = lx + dy[0]; ly = ly + dy[1];
    }
    L.jdx[slot][0] = dx[0];
    L.jdx[slot][1] = dx[1];
    L.jdy[slot][0] = dy[0];
    L.jdy[slot][1] = dy[1];
  }
  if (lane == 0) *grabs += cnt;
  __syncthreads();
  // --- bilinear samples: one lane per (texture, sample); positions by the reference's
  // incremental float sums (left += dy per row, vftmp += dx per column, optim.cpp:846-859).
  // NB samples per lane at a time with all 4 * NB texel loads issued before use (get_color's
  // arithmetic per sample, as tex_gather does for the refine kernel)
  constexpr int NB = 4;
  const int total = cnt * S;
  for (int u0 = 0; u0 < total; u0 += WAVE * NB) {
    uint32_t a0[NB], a1[NB], b0[NB], b1[NB];
    float fx[NB], fy[NB];
    int lxs[NB], lys[NB];
    bool live[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int t = u0 + q * WAVE + lane;
      const int j = t / S, k = t - j * S;
      const int slot = slot0 + (t < total ? j : 0);
      live[q] = t < total && L.valid[slot];
      const uint32_t* p = s.pyr;
      int W = 0;
      float lx = 0.0f, ly = 0.0f;
      if (live[q]) {
        const int yy = k / WS, xx = k - yy * WS;
        lx = L.jrow[slot][yy][0];
        ly = L.jrow[slot][yy][1];
        const float dxx = L.jdx[slot][0], dxy = L.jdx[slot][1];
        for (int c = 0; c < xx; ++c) { lx = lx + dxx; ly = ly + dxy; }
        const DView& v = s.views[L.jview[slot]];
        const int level = L.jlevel[slot];
        W = v.w[level];
        p = s.pyr + v.pyr_off[level] + (long long)(int)ly * W + (int)lx;
      }
      fx[q] = lx; fy[q] = ly;
      lxs[q] = (int)lx; lys[q] = (int)ly;
      a0[q] = p[0]; a1[q] = p[1]; b0[q] = p[W]; b1[q] = p[W + 1];
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      if (!live[q]) continue;
      const int t = u0 + q * WAVE + lane;
      const int j = t / S, k = t - j * S;
      const int slot = slot0 + j;
      const float dx1 = fx[q] - (float)lxs[q], dx0 = 1.0f - dx1;
      const float dy1 = fy[q] - (float)lys[q], dy0 = 1.0f - dy1;
      const float f00 = dx0 * dy0, f01 = dx0 * dy1, f10 = dx1 * dy0, f11 = dx1 * dy1;
      float r = 0.0f, g = 0.0f, b = 0.0f;
      r += (float)(a0[q] & 0xff) * f00 + (float)(b0[q] & 0xff) * f01;
      g += (float)((a0[q] >> 8) & 0xff) * f00 + (float)((b0[q] >> 8) & 0xff) * f01;
      b += (float)((a0[q] >> 16) & 0xff) * f00 + (float)((b0[q] >> 16) & 0xff) * f01;
      r += (float)(a1[q] & 0xff) * f10 + (float)(b1[q] & 0xff) * f11;
      g += (float)((a1[q] >> 8) & 0xff) * f10 + (float)((b1[q] >> 8) & 0xff) * f11;
      b += (float)((a1[q] >> 16) & 0xff) * f10 + (float)((b1[q] >> 16) & 0xff) * f11;
      L.tex[slot][k][0] = r;
      L.tex[slot][k][1] = g;
      L.tex[slot][k][2] = b;
    }
  }
  __syncthreads();
  // --- normalize, optim.cpp:1031-1067: sequential channel sums, one lane per texture
  if (lane < cnt) {
    const int slot = slot0 + lane;
    if (L.valid[slot]) {
      float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
      #pragma unroll 7  // a bounded unroll: the full 49-step one held every texel in registers (pre / post spilled)
      for (int i = 0; i < S; ++i) {
        const float4 q = *reinterpret_cast<const float4*>(L.tex[slot][i]);
        a0 += q.x; a1 += q.y; a2 += q.z;
      }
      const float fs3 = (float)S;
      a0 = __fdiv_rn(a0, fs3); a1 = __fdiv_rn(a1, fs3); a2 = __fdiv_rn(a2, fs3);
      float ave2 = 0.0f;
      #pragma unroll 7
      for (int i = 0; i < S; ++i) {
        const float4 q = *reinterpret_cast<const float4*>(L.tex[slot][i]);
        const float f0 = a0 - q.x, f1 = a1 - q.y, f2 = a2 - q.z;
        ave2 += f0 * f0 + f1 * f1 + f2 * f2;
      }
      ave2 = fsqrt_rn(__fdiv_rn(ave2, (float)(3 * S)));
      if (ave2 == 0.0f) ave2 = 1.0f;
      L.ave[slot][0] = a0; L.ave[slot][1] = a1; L.ave[slot][2] = a2; L.ave[slot][3] = ave2;
    }
  }
  __syncthreads();
  for (int t = lane; t < cnt * S; t += WAVE) {
    const int j = t / S, k = t - j * S;
    const int slot = slot0 + j;
    if (!L.valid[slot]) continue;
    const float a2 = L.ave[slot][3];
    L.tex[slot][k][0] = __fdiv_rn(L.tex[slot][k][0] - L.ave[slot][0], a2);
    L.tex[slot][k][1] = __fdiv_rn(L.tex[slot][k][1] - L.ave[slot][1], a2);
    L.tex[slot][k][2] = __fdiv_rn(L.tex[slot][k][2] - L.ave[slot][2], a2);
  }
  __syncthreads();
}

// COptim::dot, optim.cpp:1069-1077: sequential over the 3*S floats, then / size.
template <int WS>
__device__ __forceinline__ float tex_dot(const WaveLds<WS>& L, int a, int b) {
  constexpr int S = WS * WS;
  float ans = 0.0f;
  #pragma unroll 7
  for (int i = 0; i < S; ++i) {
    const float4 p = *reinterpret_cast<const float4*>(L.tex[a][i]);
    const float4 q = *reinterpret_cast<const float4*>(L.tex[b][i]);
    ans += p.x * q.x;
    ans += p.y * q.y;
    ans += p.z * q.z;
  }
  return __fdiv_rn(ans, (float)(3 * S));
}

// COptim::encode, optim.cpp:660-688, up to its transcendental functions: vect[0] and the normal's
// components (fx, fy, fz) in the reference camera frame.  The angles -- asin(fy), cos of it, acos
// -- are the optimizer's start point as doubles, so they must carry glibc's bits (glibc 2.35's asin
// and acos are not correctly rounded: 0.27 % / 0.03 % of float arguments differ from the correctly
// rounded value by one ulp, and so would any device libm); encode_angles_host finishes them with the
// host's libm (launch_refine).
__device__ __forceinline__ void encode_dev(const DScene& s, const RefineSetup& R, const float* coord, const float* normal,
                                           double* vect0, float* fxyz) {
  const float d[4] = {coord[0] - R.center[0], coord[1] - R.center[1], coord[2] - R.center[2], coord[3] - R.center[3]};
  *vect0 = (double)__fdiv_rn(dot4(d, R.ray), R.dscale);
  const DView& v = s.views[R.ref];
  float n3[3] = {normal[0], normal[1], normal[2]};
  if (normal[3] != 1.0f && normal[3] != 0.0f) {
    n3[0] = __fdiv_rn(n3[0], normal[3]); n3[1] = __fdiv_rn(n3[1], normal[3]); n3[2] = __fdiv_rn(n3[2], normal[3]);
  }
  fxyz[0] = dot3(v.xaxis, n3);
  fxyz[1] = dot3(v.yaxis, n3);
  fxyz[2] = dot3(v.zaxis, n3);
}

// ---------------------------------------------------------------- objective
// COptim::my_f, optim.cpp:507-578 (non-pairwise).  Wave-uniform result.
template <int WS>
__device__ double my_f(const DScene& s, WaveLds<WS>& L, const RefineSetup& R, const int* idx, int nidx,
                       const double* x, unsigned long long* grabs, unsigned long long* nvalid_acc) {
  float coord[4], normal[4], px[4], py[4];
  decode(s, R, x, coord, normal);
  get_paxes(s, s.views[R.ref], coord, normal, px, py);
  const int size = imin(s.tau, nidx);
  const int mininum = imin(s.minImageNum, size);
  grab_batch<WS>(s, L, size, idx, 0, coord, px, py, normal, grabs);
  const int lane = lane_id();
  if (lane >= 1 && lane < size) {
    float r = 0.0f;
    if (L.valid[0] && L.valid[lane]) r = robustincc((float)(1.0 - (double)tex_dot<WS>(L, 0, lane)));
    L.res[lane] = r;
  }
  __syncthreads();
  double ret;
  int nv = 0;
  for (int i = 0; i < size; ++i) nv += L.valid[i];
  if (lane == 0) *nvalid_acc += nv;
  if (!L.valid[0]) {
    ret = 2.0;
  } else {
    double ans = 0.0f;
    int denom = 0;
    for (int i = 1; i < size; ++i) {
      if (!L.valid[i]) continue;
      ans += (double)L.res[i];
      denom++;
    }
    ret = (denom < mininum - 1) ? 2.0f : ans / denom;
  }
  __syncthreads();
  return ret;
}

// COptim::computeINCC (weighted, robust), optim.cpp:865-938.  weights in L.fl2[].
template <int WS>
__device__ double compute_incc(const DScene& s, WaveLds<WS>& L, const float* coord, const float* normal,
                               const int* idx, int nidx, unsigned long long* grabs) {
  if (nidx < 2) return 2.0;
  float px[4], py[4];
  get_paxes(s, s.views[idx[0]], coord, normal, px, py);
  const int size = imin(s.tau, nidx);
  grab_batch<WS>(s, L, size, idx, 0, coord, px, py, normal, grabs);
  const int lane = lane_id();
  if (lane >= 1 && lane < size) {
    float r = 0.0f;
    if (L.valid[0] && L.valid[lane]) r = robustincc((float)(1.0 - (double)tex_dot<WS>(L, 0, lane)));
    L.res[lane] = r;
  }
  __syncthreads();
  double score = 0.0;
  if (!L.valid[0]) {
    score = 2.0;
  } else {
    float totalweight = 0.0f;
    for (int i = 1; i < size; ++i) {
      if (L.valid[i]) {
        totalweight += L.fl2[i];
        score += (double)(L.res[i] * L.fl2[i]);
      }
    }
    if (totalweight == 0.0f) score = 2.0;
    else score /= (double)totalweight;
  }
  __syncthreads();
  return score;
}

// ---------------------------------------------------------------- image-list steps
// COptim::addImages, optim.cpp:398-444.  Appends in visdata2 order.
template <int WS>
__device__ void add_images(const DScene& s, WaveLds<WS>& L, const float* coord, const float* normal) {
  const int lane = lane_id();
  const int ref = L.images[0];
  const int nused = L.nimg;  // the reference's used[] is built before the loop
  const int b = s.vis_off[ref], e = s.vis_off[ref + 1];
  for (int base = b; base < e; base += WAVE) {
    bool keep = false;
    const int k = base + lane;
    if (k < e) {
      const int img = s.vis[k];
      bool used = false;
      for (int i = 0; i < nused; ++i) used |= (L.images[i] == img);
      if (!used) {
        const DView& v = s.views[img];
        float ic[3];
        project(v, coord, s.level, ic);
        if (!(ic[0] < 0.0f || (float)(v.w[s.level] - 1) <= ic[0] || ic[1] < 0.0f || (float)(v.h[s.level] - 1) <= ic[1])) {
          if (get_edge(s, v, coord, s.level) != 0) {
            float ray[4] = {v.center[0] - coord[0], v.center[1] - coord[1], v.center[2] - coord[2], v.center[3] - coord[3]};
            unitize4(ray);
            keep = (s.athreshold <= dot4(ray, normal));
          }
        }
      }
    }
    int cnt;
    const int pos = ballot_prefix(keep, &cnt);
    const int n0 = L.nimg;
    __syncthreads();
    if (keep) {
      if (n0 + pos < PMVS_MAX_IMAGES) L.images[n0 + pos] = s.vis[k];
      else L.overflow = 1;
    }
    __syncthreads();
    if (lane == 0) L.nimg = imin(n0 + cnt, PMVS_MAX_IMAGES);
    __syncthreads();
  }
}

// COptim::setINCCs (reference-vs-others) + constraintImages, optim.cpp:192-206, 709-744.
template <int WS>
__device__ void constraint_images(const DScene& s, WaveLds<WS>& L, const float* coord, const float* normal, float thr,
                                  unsigned long long* grabs) {
  const int lane = lane_id();
  const int n = L.nimg;
  float px[4], py[4];
  get_paxes(s, s.views[L.images[0]], coord, normal, px, py);
  // slot 0 = reference texture, the rest in batches of TEXCAP-1
  grab_batch<WS>(s, L, 1, L.images, 0, coord, px, py, normal, grabs);
  const int ok0 = L.valid[0];
  // keep flags in L.list2
  if (lane == 0) L.list2[0] = 1;
  for (int b = 1; b < n; b += TEXCAP - 1) {
    const int cnt = imin(TEXCAP - 1, n - b);
    if (ok0) grab_batch<WS>(s, L, cnt, L.images + b, 1, coord, px, py, normal, grabs);
    if (lane < cnt) {
      float incc = 2.0f;
      if (ok0 && L.valid[1 + lane]) incc = 1.0f - tex_dot<WS>(L, 0, 1 + lane);
      L.list2[b + lane] = (incc < 1.0f - thr) ? 1 : 0;
    }
    __syncthreads();
  }
  // order-preserving compaction of images[] by keep flags, 64 entries at a time (an entry is
  // only ever moved down, and a chunk's entries are read before any of its writes)
  int newn = 0;
  for (int c = 0; c < n; c += WAVE) {
    const int k = c + lane;
    const bool keep = k < n && L.list2[k];
    const int img = k < n ? L.images[k] : 0;
    int cnt;
    const int pos = ballot_prefix(keep, &cnt);
    __syncthreads();
    if (keep) L.images[newn + pos] = img;
    newn += cnt;
    __syncthreads();
  }
  if (lane == 0) L.nimg = newn;
  __syncthreads();
}

// COptim::sortImages (newm == 1), optim.cpp:284-321; computeUnits optim.cpp:473-494.
template <int WS>
__device__ void sort_images(const DScene& s, WaveLds<WS>& L, const float* coord, const float* normal) {
  const int lane = lane_id();
  const int n = L.nimg;
  int m = 0;
  for (int c = 0; c < n; c += WAVE) {
    const int k = c + lane;
    bool keep = false;
    float unit = 0.0f, ray[4] = {0, 0, 0, 0};
    int img = 0;
    if (k < n) {
      img = L.images[k];
      const DView& v = s.views[img];
      ray[0] = v.center[0] - coord[0]; ray[1] = v.center[1] - coord[1];
      ray[2] = v.center[2] - coord[2]; ray[3] = v.center[3] - coord[3];
      unitize4(ray);
      const float d = dot4(ray, normal);
      if (!(d <= 0.0f)) {
        keep = true;
        unit = __fdiv_rn(get_unit(s, v, coord), d);
      }
    }
    int cnt;
    const int pos = ballot_prefix(keep, &cnt);
    if (keep) {
      L.list2[m + pos] = img;
      L.fl[m + pos] = unit;
      for (int i = 0; i < 4; ++i) L.rays[m + pos][i] = ray[i];
    }
    m += cnt;
  }
  __syncthreads();
  if (lane == 0) {
    if (m < 2) {
      L.nimg = 0;
    } else {
      L.fl[0] = 0.0f;
      unsigned long long alive[PMVS_MAX_IMAGES / 64];  // bit k: entry k not yet taken
      for (int w = 0; w < PMVS_MAX_IMAGES / 64; ++w)
        alive[w] = (m >= 64 * (w + 1)) ? ~0ull : (m > 64 * w ? ((1ull << (m - 64 * w)) - 1ull) : 0ull);
      int out = 0;
      for (int it = 0; it < m; ++it) {
        int index = -1;
        for (int k = 0; k < m; ++k) {
          if (!((alive[k >> 6] >> (k & 63)) & 1ull)) continue;
          if (index < 0 || L.fl[k] < L.fl[index]) index = k;
        }
        L.images[out++] = L.list2[index];
        alive[index >> 6] &= ~(1ull << (index & 63));
        for (int j = 0; j < m; ++j) {
          if (!((alive[j >> 6] >> (j & 63)) & 1ull)) continue;
          const float ftmp = smin(s.sortThreshold, smax(__fdiv_rn(s.sortThreshold, 2.0f), 1.0f - dot4(L.rays[index], L.rays[j])));
          L.fl[j] = L.fl[j] * __fdiv_rn(s.sortThreshold, ftmp);
        }
      }
      L.nimg = m;
    }
  }
  __syncthreads();
}

// CPatchOrganizerS::setScales, patchOrganizerS.cpp:663-684 (lane 0).
__device__ void set_scales(const DScene& s, const int* images, int nimg, const float* coord, float* dscale, float* ascale) {
  const DView& v0 = s.views[images[0]];
  const float unit = get_unit(s, v0, coord);
  const float unit2 = 2.0f * unit;
  float ray[4] = {coord[0] - v0.center[0], coord[1] - v0.center[1], coord[2] - v0.center[2], coord[3] - v0.center[3]};
  unitize4(ray);
  const int inum = imin(s.tau, nimg);
  const float c2[4] = {coord[0] - ray[0] * unit2, coord[1] - ray[1] * unit2, coord[2] - ray[2] * unit2, coord[3] - ray[3] * unit2};
  float ds = *dscale;
  for (int i = 1; i < inum; ++i) {
    const DView& v = s.views[images[i]];
    float a[3], b[3];
    project(v, coord, s.level, a);
    project(v, c2, s.level, b);
    const float d[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
    ds += norm3(d);
  }
  ds = __fdiv_rn(ds, (float)(inum - 1));
  ds = __fdiv_rn(unit2, ds);
  *dscale = ds;
  *ascale = (float)atan((double)__fdiv_rn(ds, __fdiv_rn(unit * (float)s.wsize, 2.0f)));
}

// CPhotoSetS::checkAngles, photoSetS.cpp:164-189.  Returns 1 if no pair is in (minA, maxA).
template <int WS>
__device__ int check_angles(const DScene& s, WaveLds<WS>& L, const float* coord, float minA, float maxA) {
  const int lane = lane_id();
  const int n = L.nimg;
  for (int k = lane; k < n; k += WAVE) {
    const DView& v = s.views[L.images[k]];
    float r[4] = {v.center[0] - coord[0], v.center[1] - coord[1], v.center[2] - coord[2], v.center[3] - coord[3]};
    unitize4(r);
    for (int i = 0; i < 4; ++i) L.rays[k][i] = r[i];
  }
  __syncthreads();
  const int npairs = n * (n - 1) / 2;
  int count = 0;
  for (int base = 0; base < npairs; base += WAVE) {
    const int p = base + lane;
    bool hit = false;
    if (p < npairs) {
      // unrank p -> (i, j), i < j
      int i = 0, rem = p;
      while (rem >= n - 1 - i) { rem -= n - 1 - i; ++i; }
      const int j = i + 1 + rem;
      const float d = smax(-1.0f, smin(1.0f, dot4(L.rays[i], L.rays[j])));
      const float angle = (float)acos((double)d);
      hit = (minA < angle && angle < maxA);
    }
    count += __popcll(__ballot(hit));
  }
  __syncthreads();
  return count < 1 ? 1 : 0;
}

// COptim::filterImagesByAngle, optim.cpp:124-148.
template <int WS>
__device__ void filter_images_by_angle(const DScene& s, WaveLds<WS>& L, const float* coord, const float* normal) {
  const int lane = lane_id();
  const int n = L.nimg;
  bool refbad = false;
  int newn = 0;
  for (int c = 0; c < n; c += WAVE) {
    const int k = c + lane;
    bool keep = false;
    int img = 0;
    if (k < n) {
      img = L.images[k];
      const DView& v = s.views[img];
      float ray[4] = {v.center[0] - coord[0], v.center[1] - coord[1], v.center[2] - coord[2], v.center[3] - coord[3]};
      unitize4(ray);
      keep = !((double)dot4(ray, normal) < s.cosAngle1);
    }
    if (c == 0) refbad = !__shfl(keep ? 1 : 0, 0);
    int cnt;
    const int pos = ballot_prefix(keep, &cnt);
    __syncthreads();
    if (!refbad && keep) L.images[newn + pos] = img;
    newn += cnt;
    __syncthreads();
  }
  if (lane == 0) L.nimg = refbad ? 0 : newn;
  __syncthreads();
}

// CPatchOrganizerS::setGrids, patchOrganizerS.cpp:410-419.
template <int WS>
__device__ void set_grids(const DScene& s, WaveLds<WS>& L, const float* coord) {
  const int lane = lane_id();
  for (int k = lane; k < L.nimg; k += WAVE) {
    float ic[3];
    project(s.views[L.images[k]], coord, s.level, ic);
    L.grids[k][0] = ((int)floorf(ic[0] + 0.5f)) / s.csize;
    L.grids[k][1] = ((int)floorf(ic[1] + 0.5f)) / s.csize;
  }
  __syncthreads();
}

// COptim::setRefImage, optim.cpp:208-254, with setINCCs (pairwise, robust) optim.cpp:746-781.
// The m x m INCC matrix lives in this workgroup's global scratch slot.
template <int WS>
__device__ void set_ref_image(const DScene& s, WaveLds<WS>& L, const float* coord, const float* normal, float* mat,
                              unsigned long long* grabs) {
  const int lane = lane_id();
  const int n = L.nimg;
  int m = 0;
  for (int c = 0; c < n; c += WAVE) {
    const int k = c + lane;
    const bool tgt = k < n && L.images[k] < s.tnum;
    int cnt;
    const int pos = ballot_prefix(tgt, &cnt);
    if (tgt) L.list2[m + pos] = L.images[k];
    m += cnt;
  }
  __syncthreads();
  if (m == 0) {
    if (lane == 0) L.nimg = 0;
    __syncthreads();
    return;
  }
  float px[4], py[4];
  get_paxes(s, s.views[L.list2[0]], coord, normal, px, py);
  constexpr int B = TEXCAP / 2;
  if (m <= TEXCAP) {
    grab_batch<WS>(s, L, m, L.list2, 0, coord, px, py, normal, grabs);
    const int npairs = m * (m - 1) / 2;
    for (int base = 0; base < npairs; base += WAVE) {
      const int p = base + lane;
      if (p < npairs) {
        int i = 0, rem = p;
        while (rem >= m - 1 - i) { rem -= m - 1 - i; ++i; }
        const int j = i + 1 + rem;
        float v = 2.0f;
        if (L.valid[i] && L.valid[j]) v = robustincc(1.0f - tex_dot<WS>(L, i, j));
        mat[i * PMVS_MAX_IMAGES + j] = v;
        mat[j * PMVS_MAX_IMAGES + i] = v;
      }
    }
  } else {
    for (int bi = 0; bi < m; bi += B) {
      const int ci = imin(B, m - bi);
      grab_batch<WS>(s, L, ci, L.list2 + bi, 0, coord, px, py, normal, grabs);
      for (int bj = bi; bj < m; bj += B) {
        const int cj = imin(B, m - bj);
        if (bj != bi) grab_batch<WS>(s, L, cj, L.list2 + bj, B, coord, px, py, normal, grabs);
        const int np = (bj == bi) ? ci * (ci - 1) / 2 : ci * cj;
        for (int base = 0; base < np; base += WAVE) {
          const int p = base + lane;
          if (p < np) {
            int i, j, si, sj;
            if (bj == bi) {
              int a = 0, rem = p;
              while (rem >= ci - 1 - a) { rem -= ci - 1 - a; ++a; }
              i = a; j = a + 1 + rem; si = i; sj = j;
            } else {
              i = p / cj; j = p - i * cj; si = i; sj = B + j;
            }
            float v = 2.0f;
            if (L.valid[si] && L.valid[sj]) v = robustincc(1.0f - tex_dot<WS>(L, si, sj));
            const int gi = bi + i, gj = bj + j;
            mat[gi * PMVS_MAX_IMAGES + gj] = v;
            mat[gj * PMVS_MAX_IMAGES + gi] = v;
          }
        }
        __syncthreads();
      }
    }
  }
  for (int k = lane; k < m; k += WAVE) mat[k * PMVS_MAX_IMAGES + k] = 0.0f;
  __syncthreads();
  // row sums in j order (std::accumulate, float)
  for (int k = lane; k < m; k += WAVE) {
    float sum = 0.0f;
    for (int j = 0; j < m; ++j) sum = sum + mat[k * PMVS_MAX_IMAGES + j];
    L.fl[k] = sum;
  }
  __syncthreads();
  if (lane == 0) {
    int refindex = -1;
    float refncc = 1073741824.0f;  // (float)(INT_MAX/2)
    for (int i = 0; i < m; ++i) {
      if (L.fl[i] < refncc) {
        refncc = L.fl[i];
        refindex = i;
      }
    }
    const int refIndex = L.list2[refindex];
    for (int i = 0; i < L.nimg; ++i) {
      if (L.images[i] == refIndex) {
        const int t = L.images[0];
        L.images[0] = refIndex;
        L.images[i] = t;
        break;
      }
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- preProcess (kernel 1)
// COptim::preProcess (optim.cpp:95-122) + the refinePatchBFGS setup (optim.cpp:584-599,629-634)
// for one candidate; writes a RefineJob.  acc: [2] grabs.
template <int WS>
__device__ void pre_candidate(const DScene& s, WaveLds<WS>& L, const pmvs_candidate& cin, RefineJob& job,
                              float4& enc, unsigned long long* acc) {
  const int lane = lane_id();
  float coord[4], normal[4];
  for (int i = 0; i < 4; ++i) { coord[i] = cin.coord[i]; normal[i] = cin.normal[i]; }
  float dscale = cin.dscale, ascale = 0.0f;
  if (lane == 0) enc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // w = 0: no refinement, no angles
  const int n0 = imin(cin.num_images, PMVS_MAX_IMAGES);
  bool badidx = false;
  for (int k = lane; k < n0; k += WAVE) {
    const int img = cin.images[k];
    const bool bad = (img < 0 || img >= s.num);
    badidx |= bad;
    L.images[k] = bad ? 0 : img;
  }
  badidx = __ballot(badidx) != 0;
  if (lane == 0) { L.nimg = n0; L.overflow = (cin.num_images > PMVS_MAX_IMAGES || n0 < 1 || badidx); }
  __syncthreads();
  int status = PMVS_ACCEPTED;
  if (L.overflow) {
    status = PMVS_FAIL_OVERFLOW;
  } else {
    add_images<WS>(s, L, coord, normal);
    constraint_images<WS>(s, L, coord, normal, s.nccThresholdBefore, &acc[2]);
    sort_images<WS>(s, L, coord, normal);
    // setScales accumulates onto the candidate's _dscale (patchOrganizerS.cpp:672)
    if (lane == 0 && L.nimg > 0) {
      float ds = dscale, as = 0.0f;
      set_scales(s, L.images, L.nimg, coord, &ds, &as);
      L.fl2[0] = ds;
      L.fl2[1] = as;
    }
    __syncthreads();
    if (L.nimg > 0) { dscale = L.fl2[0]; ascale = L.fl2[1]; }
    __syncthreads();
    if (L.nimg < s.minImageNum) {
      status = PMVS_FAIL_PRE;
    } else if (check_angles<WS>(s, L, coord, s.maxAngle, s.angle1)) {
      status = PMVS_FAIL_PRE;
      if (lane == 0) L.nimg = 0;
      __syncthreads();
    }
    if (L.overflow) status = PMVS_FAIL_OVERFLOW;
  }
  const int ni = L.nimg;
  if (status == PMVS_ACCEPTED) {
    // weights: computeUnits(patch) (optim.cpp:446-471) then min(1, w0 / wi)
    for (int k = lane; k < ni; k += WAVE) {
      const DView& v = s.views[L.images[k]];
      float u = get_unit(s, v, coord);
      float ray[4] = {v.center[0] - coord[0], v.center[1] - coord[1], v.center[2] - coord[2], v.center[3] - coord[3]};
      unitize4(ray);
      const float den = dot4(ray, normal);
      if (0.0f < den) u = __fdiv_rn(u, den);
      else u = 1073741824.0f;  // (float)(INT_MAX/2)
      L.fl[k] = u;
    }
    __syncthreads();
    if (lane < ni && lane < PMVS_MAX_TAU) {
      const float w0 = L.fl[0];
      job.weights[lane] = (lane == 0) ? 1.0f : smin(1.0f, __fdiv_rn(w0, L.fl[lane]));
    }
    if (lane == 0) {
      RefineSetup R;
      const DView& vr = s.views[L.images[0]];
      for (int i = 0; i < 4; ++i) { R.center[i] = coord[i]; R.ray[i] = coord[i] - vr.center[i]; }
      unitize4(R.ray);
      R.dscale = dscale;
      R.ascale = s.ascale;
      R.ref = L.images[0];
      double p0;
      float f[3];
      encode_dev(s, R, coord, normal, &p0, f);
      job.x0[0] = p0;  // bounds (-inf, inf): std::max(std::min(p, ub), lb) keeps it
      enc = make_float4(f[0], f[1], f[2], 1.0f);  // x0[1], x0[2]: encode_angles_host + angles_kernel
      for (int i = 0; i < 4; ++i) { job.center[i] = R.center[i]; job.ray[i] = R.ray[i]; }
    }
  }
  for (int k = lane; k < ni; k += WAVE) job.images[k] = L.images[k];
  if (lane == 0) {
    for (int i = 0; i < 4; ++i) {
      job.coord[i] = coord[i]; job.normal[i] = normal[i];
      job.rcoord[i] = coord[i]; job.rnormal[i] = normal[i];
    }
    job.dscale = dscale;
    job.ascale = ascale;
    job.ncc = -1.0f;
    job.status = status;
    job.nimg = ni;
    job.refine_code = 0;
    job.evals = 0;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- postProcess (kernel 3)
// COptim::postProcess (optim.cpp:150-190) at depth 0 on the refined job; writes the final
// pmvs_refined.  acc: [2] grabs [3] accepted [4] fail_pre [5] fail_post [6] refine_failed.
template <int WS>
__device__ void post_candidate(const DScene& s, WaveLds<WS>& L, const RefineJob& job, pmvs_refined& cout, float* mat,
                               unsigned long long* acc) {
  const int lane = lane_id();
  float coord[4], normal[4];
  for (int i = 0; i < 4; ++i) { coord[i] = job.rcoord[i]; normal[i] = job.rnormal[i]; }
  const float ncc = job.ncc, dscale = job.dscale, ascale = job.ascale;
  int status = job.status, timages = 0;
  float tmp = 0.0f;
  const int ni = job.nimg;
  for (int k = lane; k < ni; k += WAVE) L.images[k] = job.images[k];
  if (lane == 0) { L.nimg = ni; L.overflow = 0; }
  __syncthreads();
  if (status == PMVS_ACCEPTED) {
    const int rc = job.refine_code;
    const bool success = (rc == BQR_SUCCESS || rc == 2 || rc == 3 || rc == BQR_XTOL);
    if (!success && lane == 0) acc[6] += 1;
    int pfail = 0;
    if (L.nimg < s.minImageNum) pfail = 1;
    if (!pfail) {
      bool bad = false;  // CPhotoSetS::getMask over all views + CFindMatch::insideBimages
      if (s.anyMask)
        for (int b = 0; b < s.num; b += WAVE)
          if (b + lane < s.num && get_mask(s, s.views[b + lane], coord, s.level) == 0) bad = true;
      for (int b = 0; b < s.nb; b += WAVE) {
        if (b + lane < s.nb) {
          const DView& v = s.views[s.bindexes[b + lane]];
          float ic[3];
          project(v, coord, s.level, ic);
          if (ic[0] < 0.0f || (float)(v.w[s.level] - 1) < ic[0] || ic[1] < 0.0f || (float)(v.h[s.level] - 1) < ic[1]) bad = true;
        }
      }
      if (__ballot(bad)) pfail = 1;
    }
    if (!pfail) {
      add_images<WS>(s, L, coord, normal);
      constraint_images<WS>(s, L, coord, normal, s.nccThreshold, &acc[2]);
      filter_images_by_angle<WS>(s, L, coord, normal);
      if (L.nimg < s.minImageNum) pfail = 1;
    }
    int ref_before = -1;
    if (!pfail) {
      ref_before = L.images[0];
      set_ref_image<WS>(s, L, coord, normal, mat, &acc[2]);
      if (L.nimg == 0) pfail = 1;
    }
    if (!pfail) {
      // optim.cpp:165.  With the reference image unchanged by setRefImage, this second pass is the
      // identity: every image it tests passed the first pass (optim.cpp:157) against the same reference
      // texture, with the same geometry and the same frame (getPAxes of images[0]), and nothing
      // between the passes re-admits an image.  Only its grabTex count is charged then.
      if (L.images[0] != ref_before) constraint_images<WS>(s, L, coord, normal, s.nccThreshold, &acc[2]);
      else if (lane == 0) acc[2] += (unsigned long long)L.nimg;
      if (L.nimg < s.minImageNum) pfail = 1;
    }
    if (!pfail) {
      set_grids<WS>(s, L, coord);
      int t = 0;
      for (int i = 0; i < L.nimg; ++i) t += (L.images[i] < s.tnum);
      timages = t;
      tmp = smax(0.0f, ncc - s.nccThreshold) * (float)timages;
    }
    if (pfail) status = PMVS_FAIL_POST;
    if (L.overflow) status = PMVS_FAIL_OVERFLOW;
  }
  const int nout = L.nimg;
  for (int k = lane; k < PMVS_MAX_IMAGES; k += WAVE) {  // the unused tail is zero: the record's bytes are defined
    cout.images[k] = (k < nout) ? L.images[k] : 0;
    cout.grids[k][0] = (k < nout && status == PMVS_ACCEPTED) ? L.grids[k][0] : 0;
    cout.grids[k][1] = (k < nout && status == PMVS_ACCEPTED) ? L.grids[k][1] : 0;
  }
  if (lane == 0) {
    cout.status = status;
    cout.refine_code = job.refine_code;
    cout.evals = job.evals;
    cout.num_images = nout;
    for (int i = 0; i < 4; ++i) { cout.coord[i] = coord[i]; cout.normal[i] = normal[i]; }
    cout.ncc = ncc;
    cout.dscale = dscale;
    cout.ascale = ascale;
    cout.tmp = tmp;
    cout.timages = timages;
    cout.reserved = 0;
    if (status == PMVS_ACCEPTED) acc[3]++;
    else if (status == PMVS_FAIL_POST) acc[5]++;
    else acc[4]++;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- refinePatchBFGS (kernel 2)
// One LANE per candidate runs the BOBYQA state machine (state in private memory); every
// round, the lanes that requested an objective value (COptim::my_f, or the final
// computeINCC) are evaluated cooperatively by the whole wavefront in chunks of <= TSLOTS
// textures: lane-per-texture setup, lane-per-(texture,sample) gather issued NB samples at a
// time, lane-per-texture sequential normalisation, lane-per-pair sequential dots.
template <int WS, int TSLOTS, int NC>
struct RefLds {
  static constexpr int S = WS * WS;
  static constexpr int SP = (S + 3) & ~3;  // channel rows padded to 16 B (float4 reads)
#if !defined(BQ_PRIVATE)
  BqState bq[NC];                    // optimizer state of the wave's NC chains (lane c owns bq[c])
#endif
  alignas(16) float tex[TSLOTS][3][SP];  // per texture: R, G, B rows of the S samples
  float ave[TSLOTS][4];
  long long jbase[TSLOTS];
  int jvalid[TSLOTS], jW[TSLOTS], jreq[TSLOTS], jidx[TSLOTS];
  float jrow[TSLOTS][WS][2], jdx[TSLOTS][2], jdy[TSLOTS][2];  // jrow: each sample row's start (left)
  float jres[TSLOTS];
  float geo[NC][16];                 // requesting lane: coord, normal, pxaxis, pyaxis
  unsigned short views[NC][PMVS_MAX_TAU];  // requesting lane: first size images
  int rsize[NC], rfirst[NC];
};

// Phase timers of the refine kernel (pmvs_stats.prof / cyc_opt / cyc_eval): diagnostic builds
// only (-DBQ_PROFILE, libpmvs_amd_prof.so); the product build keeps the counters' registers free.
#if defined(BQ_PROFILE)
#define PROF_NOW() __builtin_amdgcn_s_memtime()
#define PROF_MARK(slot)                                   \
  do {                                                    \
    const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    prof[slot] += _t - tprev;                             \
    tprev = _t;                                           \
  } while (0)
#else
#define PROF_NOW() 0ull
#define PROF_MARK(slot) \
  do {                  \
  } while (0)
#endif

// Per-texture steps of the cooperative objective evaluation, shared by the wavefront form
// (refine_v2_kernel) and the workgroup form (refine_wg_kernel).  L is the kernel's LDS layout
// (jreq / jidx / views / geo name the slot's request, tex / ave / j* hold the slot).
// setup, one thread per texture: tex_geom (pmvs_refine.h) computes the frame, tex_setup stores it.
template <int WS, class L>
__device__ __forceinline__ void tex_setup(const DScene& s, L& C, int t) {
  const int r = C.jreq[t];
  const TexGeom T = tex_geom<WS>(s, C.geo[r], C.views[r][C.jidx[t]]);
  C.jvalid[t] = T.ok;
  C.jW[t] = T.W;
  C.jbase[t] = T.base;
  // each row's start, by the reference's recurrence `left += dy` (optim.cpp:850-860), once per texture
  // instead of once per sample in the gather
  float lx = T.tl0, ly = T.tl1;
  for (int r = 0; r < WS; ++r) {
    C.jrow[t][r][0] = lx; C.jrow[t][r][1] = ly;
    lx = lx + T.dy0; ly = ly + T.dy1;
  }
  C.jdx[t][0] = T.dx0; C.jdx[t][1] = T.dx1;
  C.jdy[t][0] = T.dy0; C.jdy[t][1] = T.dy1;
}

// gather: thread `tid` of `NT` takes samples tid, tid + NT, ...; NB samples per thread at a time,
// all 4*NB texel loads issued before use
template <int WS, int NT, class L>
__device__ __forceinline__ void tex_gather(const DScene& s, L& C, int njobs, int tid) {
  constexpr int S = WS * WS;
  constexpr int NB = 4;
  const int total = njobs * S;
  for (int u0 = 0; u0 < total; u0 += NT * NB) {
    uint32_t a0[NB], a1[NB], b0[NB], b1[NB];
    float fx[NB], fy[NB];
    int lxs[NB], lys[NB];
    bool live[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int u = u0 + q * NT + tid;
      const int t = u / S, k = u - t * S;
      live[q] = (u < total) && C.jvalid[t < njobs ? t : 0];
      long long idx = 0;
      float lx = 0.f, ly = 0.f;
      if (live[q]) {
        const int yy = k / WS, xx = k - yy * WS;
        lx = C.jrow[t][yy][0]; ly = C.jrow[t][yy][1];
        const float dxx = C.jdx[t][0], dxy = C.jdx[t][1];
        for (int c = 0; c < xx; ++c) { lx = lx + dxx; ly = ly + dxy; }
        const int ix = (int)lx, iy = (int)ly;
        idx = C.jbase[t] + (long long)iy * C.jW[t] + ix;
        lxs[q] = ix; lys[q] = iy;
      } else {
        lxs[q] = 0; lys[q] = 0;
      }
      fx[q] = lx; fy[q] = ly;
      const int W = live[q] ? C.jW[t] : 0;
      const uint32_t* p = s.pyr + idx;
      a0[q] = p[0]; a1[q] = p[1]; b0[q] = p[W]; b1[q] = p[W + 1];
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      if (!live[q]) continue;
      const int u = u0 + q * NT + tid;
      const int t = u / S, k = u - t * S;
      const float dx1 = fx[q] - (float)lxs[q], dx0 = 1.0f - dx1;
      const float dy1 = fy[q] - (float)lys[q], dy0 = 1.0f - dy1;
      const float f00 = dx0 * dy0, f01 = dx0 * dy1, f10 = dx1 * dy0, f11 = dx1 * dy1;
      float r = 0.0f, g = 0.0f, b = 0.0f;
      r += (float)(a0[q] & 0xff) * f00 + (float)(b0[q] & 0xff) * f01;
      g += (float)((a0[q] >> 8) & 0xff) * f00 + (float)((b0[q] >> 8) & 0xff) * f01;
      b += (float)((a0[q] >> 16) & 0xff) * f00 + (float)((b0[q] >> 16) & 0xff) * f01;
      r += (float)(a1[q] & 0xff) * f10 + (float)(b1[q] & 0xff) * f11;
      g += (float)((a1[q] >> 8) & 0xff) * f10 + (float)((b1[q] >> 8) & 0xff) * f11;
      b += (float)((a1[q] >> 16) & 0xff) * f10 + (float)((b1[q] >> 16) & 0xff) * f11;
      C.tex[t][0][k] = r; C.tex[t][1][k] = g; C.tex[t][2][k] = b;
    }
  }
}

// normalize (optim.cpp:1031-1067) part 1, one thread per valid texture: channel means and ave2,
// each sum in sample order
template <int WS, class L>
__device__ __forceinline__ void tex_moments(L& C, int t) {
  constexpr int S = WS * WS;
  const float *X = C.tex[t][0], *Y = C.tex[t][1], *Z = C.tex[t][2];
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
  int i = 0;
  for (; i + 4 <= S; i += 4) {
    const float4 x = *reinterpret_cast<const float4*>(X + i), y = *reinterpret_cast<const float4*>(Y + i),
                 z = *reinterpret_cast<const float4*>(Z + i);
    a0 += x.x; a1 += y.x; a2 += z.x;
    a0 += x.y; a1 += y.y; a2 += z.y;
    a0 += x.z; a1 += y.z; a2 += z.z;
    a0 += x.w; a1 += y.w; a2 += z.w;
  }
  for (; i < S; ++i) { a0 += X[i]; a1 += Y[i]; a2 += Z[i]; }
  const float fs3 = (float)S;
  a0 = __fdiv_rn(a0, fs3); a1 = __fdiv_rn(a1, fs3); a2 = __fdiv_rn(a2, fs3);
  float ave2 = 0.0f;
  auto sq = [&](float x, float y, float z) {
    const float f0 = a0 - x, f1 = a1 - y, f2 = a2 - z;
    ave2 += f0 * f0 + f1 * f1 + f2 * f2;
  };
  for (i = 0; i + 4 <= S; i += 4) {
    const float4 x = *reinterpret_cast<const float4*>(X + i), y = *reinterpret_cast<const float4*>(Y + i),
                 z = *reinterpret_cast<const float4*>(Z + i);
    sq(x.x, y.x, z.x); sq(x.y, y.y, z.y); sq(x.z, y.z, z.z); sq(x.w, y.w, z.w);
  }
  for (; i < S; ++i) sq(X[i], Y[i], Z[i]);
  ave2 = fsqrt_rn(__fdiv_rn(ave2, (float)(3 * S)));
  if (ave2 == 0.0f) ave2 = 1.0f;
  C.ave[t][0] = a0; C.ave[t][1] = a1; C.ave[t][2] = a2; C.ave[t][3] = ave2;
}

// normalize part 2, element-wise over all threads
template <int WS, int NT, class L>
__device__ __forceinline__ void tex_scale(L& C, int njobs, int tid) {
  constexpr int S = WS * WS;
  const int total = njobs * S;
  for (int u = tid; u < total; u += NT) {
    const int t = u / S, k = u - t * S;
    if (!C.jvalid[t]) continue;
    const float a2 = C.ave[t][3];
    C.tex[t][0][k] = __fdiv_rn(C.tex[t][0][k] - C.ave[t][0], a2);
    C.tex[t][1][k] = __fdiv_rn(C.tex[t][1][k] - C.ave[t][1], a2);
    C.tex[t][2][k] = __fdiv_rn(C.tex[t][2][k] - C.ave[t][2], a2);
  }
}

// robust INCC of slot t against its request's reference slot (optim.cpp:561-567, 919-929)
template <int WS, class L>
__device__ __forceinline__ void tex_dot(L& C, int t) {
  constexpr int S = WS * WS;
  const int ref = C.rfirst[C.jreq[t]];
  float r = 0.0f;
  if (C.jvalid[ref] && C.jvalid[t]) {
    float ans = 0.0f;  // per sample R, G, B products, in sample order
    const float *PX = C.tex[ref][0], *PY = C.tex[ref][1], *PZ = C.tex[ref][2];
    const float *QX = C.tex[t][0], *QY = C.tex[t][1], *QZ = C.tex[t][2];
    int i = 0;
    for (; i + 4 <= S; i += 4) {
      const float4 px = *reinterpret_cast<const float4*>(PX + i), py = *reinterpret_cast<const float4*>(PY + i),
                   pz = *reinterpret_cast<const float4*>(PZ + i), qx = *reinterpret_cast<const float4*>(QX + i),
                   qy = *reinterpret_cast<const float4*>(QY + i), qz = *reinterpret_cast<const float4*>(QZ + i);
      ans += px.x * qx.x; ans += py.x * qy.x; ans += pz.x * qz.x;
      ans += px.y * qx.y; ans += py.y * qy.y; ans += pz.y * qz.y;
      ans += px.z * qx.z; ans += py.z * qy.z; ans += pz.z * qz.z;
      ans += px.w * qx.w; ans += py.w * qy.w; ans += pz.w * qz.w;
    }
    for (; i < S; ++i) {
      ans += PX[i] * QX[i];
      ans += PY[i] * QY[i];
      ans += PZ[i] * QZ[i];
    }
    r = robustincc((float)(1.0 - (double)__fdiv_rn(ans, (float)(3 * S))));
  }
  C.jres[t] = r;
}

template <int WS, int TSLOTS, int NC>
__device__ void eval_chunk(const DScene& s, RefLds<WS, TSLOTS, NC>& C, int njobs, unsigned long long* prof,
                           unsigned long long& tprev) {
  const int lane = lane_id();
  if (lane < njobs) tex_setup<WS>(s, C, lane);
  __syncthreads();
  PROF_MARK(3);
  tex_gather<WS, WAVE>(s, C, njobs, lane);
  __syncthreads();
  PROF_MARK(4);
  if (lane < njobs && C.jvalid[lane]) tex_moments<WS>(C, lane);
  __syncthreads();
  tex_scale<WS, WAVE>(C, njobs, lane);
  __syncthreads();
  PROF_MARK(5);
  if (lane < njobs && C.jidx[lane] >= 1) tex_dot<WS>(C, lane);
  __syncthreads();
  PROF_MARK(6);
}

template <int WS, int TSLOTS, int NC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(REFINE_WPE(NC)))) void refine_v2_kernel(
    DScene s, RefineJob* __restrict__ jobs, int n, DevStats* st) {
  __shared__ RefLds<WS, TSLOTS, NC> C;
  const int lane = lane_id();
#if defined(BQ_PRIVATE)
  BqState bq_priv;
  BQ_AS BqState& bq = *(BQ_AS BqState*)&bq_priv;
#else
  BQ_AS BqState& bq = *(BQ_AS BqState*)&C.bq[lane < NC ? lane : 0];
#endif
  RefineSetup R;
  int cand = -1, need = 0, evals = 0, size = 0, nimg = 0, rc = 0;
  bool exhausted = lane >= NC;  // lanes >= NC only help evaluate
  double fv = 0.0;
  float fcoord[4], fnormal[4];
  unsigned long long tex_valid = 0, grabs = 0, nevals = 0;
  unsigned long long cyc_opt = 0, cyc_eval = 0, rounds = 0, chunks = 0;
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = 0;
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999};
  const double ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  if (lane == 0) atomicMax(&st->t_first_inv, ~__builtin_amdgcn_s_memrealtime());
  for (;;) {
    const unsigned long long t0 = PROF_NOW();
    tprev = t0;
    // (a) refill idle lanes from the queue (skipping candidates that failed preProcess)
    while (cand < 0 && !exhausted) {
      const unsigned long long c = atomicAdd(&st->queue2, 1ull);
      if (c >= (unsigned long long)n) {
        exhausted = true;
        atomicMax(&st->t_drain_inv, ~__builtin_amdgcn_s_memrealtime());
        break;
      }
      const RefineJob& J = jobs[c];
      if (J.status != PMVS_ACCEPTED) continue;
      cand = (int)c;
      for (int i = 0; i < 4; ++i) { R.center[i] = J.center[i]; R.ray[i] = J.ray[i]; }
      R.dscale = J.dscale;
      R.ascale = s.ascale;
      R.ref = J.images[0];
      nimg = J.nimg;
      size = imin(s.tau, nimg);
      for (int i = 0; i < size; ++i) C.views[lane][i] = J.images[i];  // the chain's texture views
      C.rsize[lane] = size;
      evals = 0;
      const double x0[3] = {J.x0[0], J.x0[1], J.x0[2]};
      bq_begin(bq, x0, lb, ub, 1.e-7, 1000);
      fv = 0.0;
      need = 0;
    }
    PROF_MARK(0);
    // (b) advance BOBYQA of every lane that holds an objective value (or just started)
    if (cand >= 0 && need == 0) {
      const int r = (bq.resume < 0) ? BQ_DONE : bq_step(bq, fv);
      if (r == BQ_NEED_F) {
        need = 1;
        const double xe[3] = {bq.xeval[0], bq.xeval[1], bq.xeval[2]};
        decode(s, R, xe, fcoord, fnormal);
      } else {
        rc = bq.rc;
        const bool success = (rc == BQR_SUCCESS || rc == 2 || rc == 3 || rc == BQR_XTOL);
        RefineJob& J = jobs[cand];
        J.refine_code = rc;
        J.evals = evals;
        if (success) {
          const double xo[3] = {bq.xout[0], bq.xout[1], bq.xout[2]};
          decode(s, R, xo, fcoord, fnormal);
          if (nimg < 2) {  // computeINCC returns 2.0 without grabbing (optim.cpp:866)
            J.ncc = (float)(1.0 - (double)unrobustincc(2.0f));
            for (int i = 0; i < 4; ++i) { J.rcoord[i] = fcoord[i]; J.rnormal[i] = fnormal[i]; }
            cand = -1;
          } else {
            need = 2;  // final computeINCC (robust, weighted) at the refined geometry
          }
        } else {
          cand = -1;  // geometry and _ncc stay unrefined (optim.cpp:649-655)
        }
      }
    }
    PROF_MARK(1);
    // (c) publish requests
    const bool req = (cand >= 0 && need != 0);
    if (req) {
      float px[4], py[4];
      get_paxes(s, s.views[R.ref], fcoord, fnormal, px, py);
      for (int i = 0; i < 4; ++i) {
        C.geo[lane][i] = fcoord[i]; C.geo[lane][4 + i] = fnormal[i];
        C.geo[lane][8 + i] = px[i]; C.geo[lane][12 + i] = py[i];
      }
    }
    const unsigned long long reqmask = __ballot(req);
    const unsigned long long t1 = PROF_NOW();
    prof[2] += t1 - tprev;
    tprev = t1;
    cyc_opt += t1 - t0;
    rounds++;
    if (reqmask == 0ull) {
      if (__ballot(cand >= 0 || !exhausted) == 0ull) break;
      continue;
    }
    __syncthreads();
    // (d) evaluate all requests, packed into chunks of <= TSLOTS textures (lane order)
    bool pending = req;
    while (__ballot(pending) != 0ull) {
      const int sz = pending ? size : 0;
      const int off = wave_excl_scan(sz);
      const bool in = pending && (off + sz <= TSLOTS);
      const int njobs = __shfl(off + sz, 63 - __clzll(__ballot(in)));  // end of the last member
      if (in) {
        C.rfirst[lane] = off;
        for (int i = 0; i < sz; ++i) {
          C.jreq[off + i] = lane;
          C.jidx[off + i] = i;
        }
      }
      __syncthreads();
      PROF_MARK(7);
      eval_chunk<WS, TSLOTS, NC>(s, C, njobs, prof, tprev);
      chunks++;
      if (lane == 0) grabs += njobs;
      if (in) {
        // reduce this request's per-texture results in the reference's order
        fv = request_value(s, C, off, sz, need, jobs[cand], tex_valid);
        pending = false;
      }
      __syncthreads();
    }
    cyc_eval += PROF_NOW() - t1;
    // (e) consume results
    if (req) {
      if (need == 1) {
        evals++;
        nevals++;
        need = 0;
      } else {
        RefineJob& J = jobs[cand];
        J.ncc = (float)(1.0 - (double)unrobustincc((float)fv));
        for (int i = 0; i < 4; ++i) { J.rcoord[i] = fcoord[i]; J.rnormal[i] = fnormal[i]; }
        cand = -1;
        need = 0;
      }
    }
  }
  // wave-level reduction of the counters, one atomic each
  for (int d = 32; d >= 1; d >>= 1) {
    tex_valid += __shfl_xor(tex_valid, d);
    nevals += __shfl_xor(nevals, d);
  }
  if (lane == 0) {
    atomicAdd(&st->evals, nevals);
    atomicAdd(&st->tex_valid, tex_valid);
    atomicAdd(&st->tex_grabs, grabs);
    atomicAdd(&st->cyc_opt, cyc_opt);
    atomicAdd(&st->cyc_eval, cyc_eval);
    atomicAdd(&st->rounds, rounds);
    atomicAdd(&st->chunks, chunks);
    for (int i = 0; i < 8; ++i) atomicAdd(&st->prof[i], prof[i]);
    atomicMax(&st->t_last, __builtin_amdgcn_s_memrealtime());
  }
}

// ---------------------------------------------------------------- refinePatchBFGS, workgroup form
// One 256-thread workgroup (4 wavefronts, one per SIMD) owns NC chains whose optimizer states
// live in the workgroup's LDS.  Chain c is stepped by lane c % (NC/OW) of wavefront c / (NC/OW):
// with OW = 1 a single wavefront advances all NC chains in one instruction stream (NC lanes per
// f64 instruction instead of the wavefront form's 6), with OW = 4 every SIMD steps NC/4 of them.
// The requests of a round are packed, in chain order, into chunks of <= TS texture slots, and all
// 256 threads evaluate a chunk: thread-per-texture setup / moments / dot spread over the four
// wavefronts (consecutive slots per wavefront: conflict-free LDS rows), thread-per-sample gather
// and scaling.  Results, optimizer trajectories and counters equal the wavefront form's.
constexpr int WG_THREADS = 256;
constexpr int WG_LDS_BYTES = 160 * 1024;

template <int WS, int NC, int WGPC>
struct RefWgFit {  // texture slots (<= 64) that fit next to NC optimizer states, WGPC workgroups per CU
  static constexpr int SP = (WS * WS + 3) & ~3;
  static constexpr int per_slot = 3 * SP * 4 + 4 * 4 + 8 + 4 * 4 + (2 * WS + 4) * 4 + 4;
  static constexpr int fixed = NC * ((int)sizeof(BqState) + 16 * 4 + PMVS_MAX_TAU * 2 + 4 * 4) + 4 * (NC + 1) + 64;
  static constexpr int fit = (WG_LDS_BYTES / WGPC - fixed) / per_slot - 1;
  static constexpr int slots = fit < 64 ? fit : 64;
};

template <int WS, int NC, int TS>
struct RefWgLds {
  static constexpr int S = WS * WS;
  static constexpr int SP = (S + 3) & ~3;
  BqState bq[NC];                          // chain c's optimizer state
  alignas(16) float tex[TS][3][SP];       // slot: R, G, B rows of the S samples
  float ave[TS][4];
  long long jbase[TS];
  int jvalid[TS], jW[TS], jreq[TS], jidx[TS];
  float jrow[TS][WS][2], jdx[TS][2], jdy[TS][2];
  float jres[TS];
  float geo[NC][16];                       // requesting chain: coord, normal, pxaxis, pyaxis
  unsigned short views[NC][PMVS_MAX_TAU];  // chain: first size images
  int rsize[NC];                           // this round's request size (0: none)
  int rfirst[NC], rchunk[NC];              // its first slot and chunk
  int alive[NC];                           // chain holds a candidate or may still get one
  int chunk_jobs[NC + 1];
  int nchunk, live;
};

template <int WS, int NC, int TS, int OW>
__global__ __launch_bounds__(WG_THREADS) __attribute__((amdgpu_waves_per_eu(REFINE_WPE(NC)))) void refine_wg_kernel(
    DScene s, RefineJob* __restrict__ jobs, int n, int nc_active, DevStats* st) {
  constexpr int CPW = NC / OW;
  static_assert(NC % OW == 0 && NC <= WAVE && OW >= 1 && OW <= WG_THREADS / WAVE, "chain layout");
  static_assert(TS >= PMVS_MAX_TAU, "a request must fit one chunk");
  static_assert(sizeof(RefWgLds<WS, NC, TS>) <= WG_LDS_BYTES, "LDS");
  __shared__ RefWgLds<WS, NC, TS> C;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & (WAVE - 1);
  // chain c = lane * OW + wave: the first nc_active chains (small batches spread over more
  // workgroups) fall on every optimizer wavefront
  const int cidx = lane * OW + wave;
  const bool owner = wave < OW && lane < CPW && cidx < nc_active;
  const int c = owner ? cidx : 0;
  BQ_AS BqState& bq = *(BQ_AS BqState*)&C.bq[c];
  RefineSetup R;
  int cand = -1, need = 0, evals = 0, size = 0, nimg = 0, rc = 0;
  bool exhausted = !owner;
  double fv = 0.0;
  float fcoord[4], fnormal[4];
  unsigned long long tex_valid = 0, grabs = 0, nevals = 0, rounds = 0, chunks = 0;
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999};
  const double ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  // chains beyond nc_active never publish: they read as idle and dead (the packing and the loop's
  // exit test read every chain's entry)
  if (tid < NC) {
    C.rsize[tid] = 0;
    C.alive[tid] = 0;
  }
  if (tid == 0) atomicMax(&st->t_first_inv, ~__builtin_amdgcn_s_memrealtime());
  __syncthreads();
  for (;;) {
    bool req = false;
    if (owner) {
      // (a) refill an idle chain from the queue (skipping candidates that failed preProcess)
      while (cand < 0 && !exhausted) {
        const unsigned long long q = atomicAdd(&st->queue2, 1ull);
        if (q >= (unsigned long long)n) {
          exhausted = true;
          atomicMax(&st->t_drain_inv, ~__builtin_amdgcn_s_memrealtime());
          break;
        }
        const RefineJob& J = jobs[q];
        if (J.status != PMVS_ACCEPTED) continue;
        cand = (int)q;
        for (int i = 0; i < 4; ++i) { R.center[i] = J.center[i]; R.ray[i] = J.ray[i]; }
        R.dscale = J.dscale;
        R.ascale = s.ascale;
        R.ref = J.images[0];
        nimg = J.nimg;
        size = imin(s.tau, nimg);
        for (int i = 0; i < size; ++i) C.views[c][i] = J.images[i];
        evals = 0;
        const double x0[3] = {J.x0[0], J.x0[1], J.x0[2]};
        bq_begin(bq, x0, lb, ub, 1.e-7, 1000);
        fv = 0.0;
        need = 0;
      }
      // (b) advance BOBYQA when it holds an objective value (or just started)
      if (cand >= 0 && need == 0) {
        const int r = (bq.resume < 0) ? BQ_DONE : bq_step(bq, fv);
        if (r == BQ_NEED_F) {
          need = 1;
          const double xe[3] = {bq.xeval[0], bq.xeval[1], bq.xeval[2]};
          decode(s, R, xe, fcoord, fnormal);
        } else {
          rc = bq.rc;
          const bool success = (rc == BQR_SUCCESS || rc == 2 || rc == 3 || rc == BQR_XTOL);
          RefineJob& J = jobs[cand];
          J.refine_code = rc;
          J.evals = evals;
          if (success) {
            const double xo[3] = {bq.xout[0], bq.xout[1], bq.xout[2]};
            decode(s, R, xo, fcoord, fnormal);
            if (nimg < 2) {  // computeINCC returns 2.0 without grabbing (optim.cpp:866)
              J.ncc = (float)(1.0 - (double)unrobustincc(2.0f));
              for (int i = 0; i < 4; ++i) { J.rcoord[i] = fcoord[i]; J.rnormal[i] = fnormal[i]; }
              cand = -1;
            } else {
              need = 2;  // final computeINCC (robust, weighted) at the refined geometry
            }
          } else {
            cand = -1;  // geometry and _ncc stay unrefined (optim.cpp:649-655)
          }
        }
      }
      // (c) publish the request
      req = (cand >= 0 && need != 0);
      if (req) {
        float px[4], py[4];
        get_paxes(s, s.views[R.ref], fcoord, fnormal, px, py);
        for (int i = 0; i < 4; ++i) {
          C.geo[c][i] = fcoord[i]; C.geo[c][4 + i] = fnormal[i];
          C.geo[c][8 + i] = px[i]; C.geo[c][12 + i] = py[i];
        }
      }
      C.rsize[c] = req ? size : 0;
      C.alive[c] = (cand >= 0 || !exhausted) ? 1 : 0;
    }
    __syncthreads();
    // (d) pack the round's requests into chunks of <= TS slots, in chain order
    if (wave == 0) {
      const int sz = lane < NC ? C.rsize[lane] : 0;
      bool pending = sz > 0;
      int k = 0;
      while (__ballot(pending) != 0ull) {
        const int off = wave_excl_scan(pending ? sz : 0);
        const bool in = pending && (off + sz <= TS);
        const int nj = __shfl(off + sz, 63 - __clzll(__ballot(in)));
        if (in) {
          C.rfirst[lane] = off;
          C.rchunk[lane] = k;
        }
        if (lane == 0) C.chunk_jobs[k] = nj;
        pending = pending && !in;
        ++k;
      }
      const bool al = lane < NC && C.alive[lane] != 0;
      if (lane == 0) {
        C.nchunk = k;
        C.live = __ballot(al) != 0ull ? 1 : 0;
      }
    }
    __syncthreads();
    const int nchunk = C.nchunk;
    rounds++;
    if (nchunk == 0) {  // (nchunk / live are rewritten only after the next round's first barrier)
      if (!C.live) break;
      continue;
    }
    const int my_chunk = req ? C.rchunk[c] : -1;
    const int my_off = req ? C.rfirst[c] : 0;
    // (e) evaluate chunk by chunk
    for (int k = 0; k < nchunk; ++k) {
      if (my_chunk == k) {
        for (int i = 0; i < size; ++i) {
          C.jreq[my_off + i] = c;
          C.jidx[my_off + i] = i;
        }
      }
      __syncthreads();
      const int njobs = C.chunk_jobs[k];
      const int per = (njobs + 3) >> 2;  // slots per wavefront in the per-texture steps
      const int t = wave * per + lane;
      const bool mine = lane < per && t < njobs;
      if (mine) tex_setup<WS>(s, C, t);
      __syncthreads();
      tex_gather<WS, WG_THREADS>(s, C, njobs, tid);
      __syncthreads();
      if (mine && C.jvalid[t]) tex_moments<WS>(C, t);
      __syncthreads();
      tex_scale<WS, WG_THREADS>(C, njobs, tid);
      __syncthreads();
      if (mine && C.jidx[t] >= 1) tex_dot<WS>(C, t);
      __syncthreads();
      chunks++;
      grabs += njobs;
      if (my_chunk == k) fv = request_value(s, C, my_off, size, need, jobs[cand], tex_valid);
      __syncthreads();
    }
    // (f) consume the results
    if (req) {
      if (need == 1) {
        evals++;
        nevals++;
        need = 0;
      } else {
        RefineJob& J = jobs[cand];
        J.ncc = (float)(1.0 - (double)unrobustincc((float)fv));
        for (int i = 0; i < 4; ++i) { J.rcoord[i] = fcoord[i]; J.rnormal[i] = fnormal[i]; }
        cand = -1;
        need = 0;
      }
    }
  }
  // per-wavefront reduction of the chain counters, one atomic each
  for (int d = 32; d >= 1; d >>= 1) {
    tex_valid += __shfl_xor(tex_valid, d);
    nevals += __shfl_xor(nevals, d);
  }
  if (lane == 0 && wave < OW) {
    atomicAdd(&st->evals, nevals);
    atomicAdd(&st->tex_valid, tex_valid);
    atomicAdd(&st->tex_valid_wg, tex_valid);
  }
  if (tid == 0) {
    atomicAdd(&st->tex_grabs, grabs);
    atomicAdd(&st->rounds, rounds);
    atomicAdd(&st->chunks, chunks);
    atomicMax(&st->t_last, __builtin_amdgcn_s_memrealtime());
  }
}

// PMVS_REFINE_TAIL=1 (diagnostics): after each refine launch, its span (first wavefront start -> last
// end) and tail (first empty refill -> last end: chains still running while no new candidate
// starts) are added to DevStats' sums and the per-launch stamps cleared.
__global__ void refine_tail_kernel(DevStats* st, int form) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned long long last = st->t_last, first = ~st->t_first_inv, drain = ~st->t_drain_inv;
  if (st->t_last != 0 && st->t_first_inv != 0) {
    st->span_t[form] += last - first;
    st->tail_t[form] += (st->t_drain_inv != 0 && drain < last) ? last - drain : 0ull;
    st->tail_launches[form] += 1;
  }
  st->t_first_inv = 0;
  st->t_drain_inv = 0;
  st->t_last = 0;
}

}  // namespace pmvsdev

// ==================================================================== kernels
namespace pmvsdev {

// Kernel 1: preProcess, one wavefront per candidate, persistent with a device work queue.  Pre and
// post are latency-bound wave-per-candidate walks: a 256-register budget (2 waves per SIMD, the
// persistent grid's 8 per CU) instead of the 324 the inlined code would take (1 per SIMD).
// Round 5: with the texture loops' unroll bounded (grab_batch, tex_dot) they fit 188 / 150
// registers without spills, and 3 waves per SIMD measured best (r05w: pre 161 -> 144, post 207 ->
// 200 ms per C3 step against round 4's 2 waves with spills; 4 waves no better).  PMVS_PREPOST_WPE:
// the waves-per-SIMD target (timing variants).
#ifndef PMVS_PREPOST_WPE
#define PMVS_PREPOST_WPE 3
#endif
int prepost_waves() { return PMVS_PREPOST_WPE; }
template <int WS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PMVS_PREPOST_WPE))) void pre_kernel(DScene s, const pmvs_candidate* __restrict__ in,
                                                  RefineJob* __restrict__ jobs, float4* __restrict__ enc, int n,
                                                  DevStats* st) {
  __shared__ WaveLds<WS> L;
  unsigned long long acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const int lane = lane_id();
  for (;;) {
    if (lane == 0) {
      const unsigned long long c = atomicAdd(&st->queue, 1ull);
      L.cand = (c < (unsigned long long)n) ? (int)c : -1;
    }
    __syncthreads();
    const int c = __builtin_amdgcn_readfirstlane(L.cand);
    __syncthreads();
    if (c < 0) break;
    pre_candidate<WS>(s, L, in[c], jobs[c], enc[c], acc);
  }
  if (lane == 0) atomicAdd(&st->tex_grabs, acc[2]);
}

// Kernel 3: postProcess, one wavefront per candidate.
template <int WS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PMVS_PREPOST_WPE))) void post_kernel(DScene s, const RefineJob* __restrict__ jobs,
                                                   pmvs_refined* __restrict__ out, int n, DevStats* st) {
  __shared__ WaveLds<WS> L;
  unsigned long long acc[7] = {0, 0, 0, 0, 0, 0, 0};
  float* mat = s.scratch + (size_t)blockIdx.x * PMVS_MAX_IMAGES * PMVS_MAX_IMAGES;
  const int lane = lane_id();
  for (;;) {
    if (lane == 0) {
      const unsigned long long c = atomicAdd(&st->queue3, 1ull);
      L.cand = (c < (unsigned long long)n) ? (int)c : -1;
    }
    __syncthreads();
    const int c = __builtin_amdgcn_readfirstlane(L.cand);
    __syncthreads();
    if (c < 0) break;
    post_candidate<WS>(s, L, jobs[c], out[c], mat, acc);
  }
  if (lane == 0) {
    atomicAdd(&st->tex_grabs, acc[2]);
    atomicAdd(&st->accepted, acc[3]);
    atomicAdd(&st->fail_pre, acc[4]);
    atomicAdd(&st->fail_post, acc[5]);
    atomicAdd(&st->refine_failed, acc[6]);
  }
}

// One wavefront per query: refinePatchBFGS setup (optim.cpp:584-596) + one my_f evaluation.
template <int WS>
__global__ __launch_bounds__(64) void incc_eval_kernel(DScene s, const pmvs_eval_query* __restrict__ q, int n,
                                                        double* __restrict__ out, DevStats* st) {
  __shared__ WaveLds<WS> L;
  const int i = blockIdx.x;
  if (i >= n) return;
  const int lane = lane_id();
  const pmvs_eval_query& Q = q[i];
  RefineSetup R;
  const DView& vr = s.views[Q.images[0]];
  for (int k = 0; k < 4; ++k) { R.center[k] = Q.coord[k]; R.ray[k] = Q.coord[k] - vr.center[k]; }
  unitize4(R.ray);
  R.dscale = Q.dscale;
  R.ascale = s.ascale;
  R.ref = Q.images[0];
  int idx[PMVS_MAX_TAU];
  const int ni = imin(Q.num_images, PMVS_MAX_TAU);
  for (int k = 0; k < ni; ++k) idx[k] = Q.images[k];
  unsigned long long grabs = 0, nvalid = 0;
  const double f = my_f<WS>(s, L, R, idx, ni, Q.x, &grabs, &nvalid);
  if (lane == 0) {
    out[i] = f;
    atomicAdd(&st->evals, 1ull);
    atomicAdd(&st->tex_valid, nvalid);
    atomicAdd(&st->tex_grabs, grabs);
  }
}

// One wavefront per query: grabTex (+ normalize).
template <int WS>
__global__ __launch_bounds__(64) void grab_tex_kernel(DScene s, const pmvs_tex_query* __restrict__ q, int n,
                                                       float* __restrict__ out, int* __restrict__ valid) {
  __shared__ WaveLds<WS> L;
  constexpr int S = WS * WS;
  const int i = blockIdx.x;
  if (i >= n) return;
  const int lane = lane_id();
  const pmvs_tex_query& Q = q[i];
  unsigned long long grabs = 0;
  int view = Q.view;
  // grab without normalisation when asked: run the batch, then undo is impossible, so grab into
  // slot 0 and (re)compute raw samples when normalize == 0 by skipping the normalize pass below.
  if (Q.normalize) {
    grab_batch<WS>(s, L, 1, &view, 0, Q.coord, Q.pxaxis, Q.pyaxis, Q.normal, &grabs);
  } else {
    // raw samples: same setup + sampling as grab_batch, no normalisation
    grab_batch<WS>(s, L, 1, &view, 0, Q.coord, Q.pxaxis, Q.pyaxis, Q.normal, &grabs);
    // restore raw values from the normalisation constants: not exact, so recompute instead
    if (L.valid[0]) {
      for (int t = lane; t < S; t += WAVE) {
        const int yy = t / WS, xx = t - yy * WS;
        float lx = L.jrow[0][yy][0], ly = L.jrow[0][yy][1];
        for (int c = 0; c < xx; ++c) { lx = lx + L.jdx[0][0]; ly = ly + L.jdx[0][1]; }
        float rgb[3];
        get_color(s, s.views[L.jview[0]], lx, ly, L.jlevel[0], rgb);
        L.tex[0][t][0] = rgb[0];
        L.tex[0][t][1] = rgb[1];
        L.tex[0][t][2] = rgb[2];
      }
    }
    __syncthreads();
  }
  const int ok = L.valid[0];
  for (int t = lane; t < S; t += WAVE) {
    for (int c = 0; c < 3; ++c) out[(size_t)i * 3 * S + 3 * t + c] = ok ? L.tex[0][t][c] : 0.0f;
  }
  if (lane == 0) valid[i] = ok;
}

// CImage::buildImage (image.cpp:228-325, filter 0): one thread per output pixel, double
// accumulation in the reference's (j, i) order, float denominator, floor(c + 0.5f).
__global__ void build_level_kernel(const uint8_t* __restrict__ src, int Wp, int Hp, uint8_t* __restrict__ dst, int W,
                                   int H) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= W || y >= H) return;
  const double wts[4] = {1.0 / 64.0 * 1.0, 3.0 / 64.0, 3.0 / 64.0, 1.0 / 64.0};
  double c0 = 0, c1 = 0, c2 = 0;
  float denom = 0.0f;
  for (int j = -1; j < 3; ++j) {
    const int ytmp = 2 * y + j;
    if (ytmp < 0 || Hp - 1 < ytmp) continue;
    for (int i = -1; i < 3; ++i) {
      const int xtmp = 2 * x + i;
      if (xtmp < 0 || Wp - 1 < xtmp) continue;
      // mask[j][i] = outer(1 3 3 1)/64: values 1/64, 3/64, 9/64 are exact in double
      const double m = (double)((j == -1 || j == 2) ? 1 : 3) * (double)((i == -1 || i == 2) ? 1 : 3) / 64.0;
      const uint8_t* p = src + ((size_t)ytmp * Wp + xtmp) * 3;
      c0 += m * (double)p[0];
      c1 += m * (double)p[1];
      c2 += m * (double)p[2];
      denom = (float)((double)denom + m);
    }
  }
  (void)wts;
  const double dd = (double)denom;
  c0 /= dd; c1 /= dd; c2 /= dd;
  uint8_t* o = dst + ((size_t)y * W + x) * 3;
  o[0] = (uint8_t)((int)floor(c0 + (double)0.5f));
  o[1] = (uint8_t)((int)floor(c1 + (double)0.5f));
  o[2] = (uint8_t)((int)floor(c2 + (double)0.5f));
}

__global__ void pack_rgba_kernel(const uint8_t* __restrict__ rgb, uint32_t* __restrict__ out, long long npix) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t* p = rgb + 3 * i;
  out[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}

__global__ void unpack_rgba_kernel(const uint32_t* __restrict__ in, uint8_t* __restrict__ rgb, long long npix) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint32_t v = in[i];
  rgb[3 * i] = v & 0xff;
  rgb[3 * i + 1] = (v >> 8) & 0xff;
  rgb[3 * i + 2] = (v >> 16) & 0xff;
}

}  // namespace pmvsdev

// ==================================================================== launchers
#include "pmvs_launch.h"
#include "pmvs_hostpool.h"

namespace pmvsdev {

// The optimizer start point's angles (encode's transcendental tail, see encode_dev) with the host's
// libm, exactly as COptim::encode (optim.cpp:671-686) evaluates them, then std::max(std::min(x,
// ub), lb) with the angle bounds (optim.cpp:629-634).  Threads for large batches.
static void encode_angles_host(const float4* enc, int n, float ascale, double2* ang) {
  auto one = [&](int i) {
    const float4 e = enc[i];
    double v1 = 0.0, v2 = 0.0;
    if (e.w != 0.0f) {
      const float fx = e.x, fy = e.y, fz = e.z;
      const float cfy = (1.0f < fy) ? 1.0f : fy;       // std::min(1.0f, fy)
      v2 = std::asin((double)((cfy < -1.0f) ? -1.0f : cfy));  // std::max(-1.0f, .)
      const float cosb = (float)std::cos(v2);
      if (cosb == 0.0f) {
        v1 = 0.0;
      } else {
        const float sina = fx / cosb;
        const float cosa = -fz / cosb;
        const float cc = (1.0f < cosa) ? 1.0f : cosa;
        v1 = std::acos((double)((cc < -1.0f) ? -1.0f : cc));
        if (sina < 0.0f) v1 = -v1;
      }
      v1 = v1 / (double)ascale;
      v2 = v2 / (double)ascale;
      const double lb = -23.99999, ub = 23.99999;
      v1 = (ub < v1) ? ub : v1; v1 = (v1 < lb) ? lb : v1;
      v2 = (ub < v2) ? ub : v2; v2 = (v2 < lb) ? lb : v2;
    }
    ang[i] = make_double2(v1, v2);
  };
  // ~0.1 us of libm per candidate: a C3 expansion wave's 15-80 k candidates would hold the GPU for
  // 2-8 ms on one thread, so from 2048 on the work is split into contiguous ranges over <= 8 threads
  // of a persistent pool (no thread start per batch); a pool busy with another scene's batch is
  // not waited for
  const int nt = (n >= 2048) ? std::min(8, n / 1024) : 1;
  if (nt <= 1 || !HostPool::get().run(nt, [&](int t, int nthreads) {
        const int per = (n + nthreads - 1) / nthreads;
        for (int i = t * per; i < std::min(n, (t + 1) * per); ++i) one(i);
      }))
    for (int i = 0; i < n; ++i) one(i);
}

__global__ void angles_kernel(RefineJob* __restrict__ jobs, const double2* __restrict__ ang, const float4* __restrict__ enc,
                              int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || enc[i].w == 0.0f) return;
  jobs[i].x0[1] = ang[i].x;
  jobs[i].x0[2] = ang[i].y;
}

hipError_t RefineHost::ensure(size_t n) {
  if (n <= cap) return hipSuccess;
  release();
  cap = std::max(n, (size_t)4096);
  hipError_t e = hipMalloc((void**)&d_enc, cap * sizeof(float4));
  if (e == hipSuccess) e = hipMalloc((void**)&d_ang, cap * sizeof(double2));
  if (e == hipSuccess) e = hipHostMalloc((void**)&h_enc, cap * sizeof(float4));
  if (e == hipSuccess) e = hipHostMalloc((void**)&h_ang, cap * sizeof(double2));
  if (e != hipSuccess) cap = 0;
  return e;
}
void RefineHost::release() {
  if (ev_pre) (void)hipEventDestroy(ev_pre);
  ev_pre = nullptr;
  if (d_enc) (void)hipFree(d_enc);
  if (d_ang) (void)hipFree(d_ang);
  if (h_enc) (void)hipHostFree(h_enc);
  if (h_ang) (void)hipHostFree(h_ang);
  d_enc = nullptr; d_ang = nullptr; h_enc = nullptr; h_ang = nullptr;
  cap = 0;
}

// refine_v2_kernel instantiations (texture slots * 100 + chains per wavefront)
bool refine_config_supported(int tslots) {
  switch (tslots) {
    case 804: case 807: case 808: case 1201: case 1202: case 1203: case 1204: case 1206: case 1608: case 2408: return true;
    case 164011: case 164021: case 164041: case 148041: case 132022: case 132042: case 116042: return true;
#if defined(BQ_PRIVATE)
    case 1264: case 2464: case 1232: case 2432: case 1216: case 2448: case 3232: case 3248: case 3264: case 4832:
    case 4864: return true;
#endif
    default: return refine_split_supported(tslots) || refine_lane_supported(tslots);
  }
}

static bool refine_tail_on() {
  static const bool on = getenv("PMVS_REFINE_TAIL") != nullptr;
  return on;
}

// Diagnostics only (PMVS_DUMP_JOBS=<file>, tools/r06ad.sh): after the first four refine batches of at
// least 50 000 candidates, every refined job's preProcess outputs and its evaluation count are
// appended to <file> as float32 rows [batch, nimg, evals, refine_code, dscale, ascale, x0[0..2],
// weights[0..5], ncc] -- the data for a chain-length predictor.
static void dump_jobs(const RefineJob* d_jobs, int n, hipStream_t stream) {
  static const char* path = getenv("PMVS_DUMP_JOBS");
  static int batches = 0;
  if (!path || n < 50000 || batches >= 4) return;
  std::vector<RefineJob> h((size_t)n);
  if (hipStreamSynchronize(stream) != hipSuccess ||
      hipMemcpy(h.data(), d_jobs, (size_t)n * sizeof(RefineJob), hipMemcpyDeviceToHost) != hipSuccess)
    return;
  FILE* f = fopen(path, "ab");
  if (!f) return;
  for (const RefineJob& J : h) {
    if (J.status != PMVS_ACCEPTED) continue;
    float r[16] = {(float)batches, (float)J.nimg, (float)J.evals, (float)J.refine_code, J.dscale, J.ascale,
                   (float)J.x0[0], (float)J.x0[1], (float)J.x0[2], 0, 0, 0, 0, 0, 0, J.ncc};
    for (int i = 0; i < 6 && i < PMVS_MAX_TAU; ++i) r[9 + i] = J.weights[i];
    fwrite(r, sizeof(r), 1, f);
  }
  fclose(f);
  ++batches;
}

template <int WS>
static hipError_t launch_refine_ws(const DScene& s, const pmvs_candidate* d_in, RefineJob* d_jobs, pmvs_refined* d_out,
                                   int n, DevStats* d_st, int grid, int refine_grid, int tslots, hipStream_t stream,
                                   hipEvent_t* ev, RefineHost& rh) {
  // pre / post: the persistent grid (2 single-wave workgroups per SIMD) scaled to their residency
  const int gp = grid * PMVS_PREPOST_WPE / 2;
  const int g = gp < n ? gp : n;
  hipError_t e = rh.ensure((size_t)n);
  if (e != hipSuccess) return e;
  (void)hipEventRecord(ev[0], stream);
  hipLaunchKernelGGL((pre_kernel<WS>), dim3(g), dim3(64), 0, stream, s, d_in, d_jobs, rh.d_enc, n, d_st);
  if (rh.prof && (rh.ev_pre || hipEventCreate(&rh.ev_pre) == hipSuccess)) (void)hipEventRecord(rh.ev_pre, stream);
  // the start point's angles with the host's libm (encode_angles_host): one round trip per batch
  if ((e = hipMemcpyAsync(rh.h_enc, rh.d_enc, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess)
    return e;
  encode_angles_host(rh.h_enc, n, s.ascale, rh.h_ang);
  if ((e = hipMemcpyAsync(rh.d_ang, rh.h_ang, (size_t)n * sizeof(double2), hipMemcpyHostToDevice, stream)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(angles_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_jobs, rh.d_ang, rh.d_enc, n);
  (void)hipEventRecord(ev[1], stream);
  if (rh.prof && rh.ev_pre && hipEventSynchronize(ev[1]) == hipSuccess) {  // diagnostics only: one more wait
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, rh.ev_pre, ev[1]) == hipSuccess) rh.trip_ms += ms;
    ++rh.trips;
  }
  if (tslots >= 300000) {  // lane form (pmvs_refine_lane.hip)
    if ((e = launch_refine_lane(tslots, s, d_jobs, n, d_st, stream)) != hipSuccess) return e;
    if (refine_tail_on()) hipLaunchKernelGGL(refine_tail_kernel, dim3(1), dim3(64), 0, stream, d_st, 1);
    (void)hipEventRecord(ev[2], stream);
    hipLaunchKernelGGL((post_kernel<WS>), dim3(g), dim3(64), 0, stream, s, d_jobs, d_out, n, d_st);
    (void)hipEventRecord(ev[3], stream);
    return hipGetLastError();
  }
  // (before the tau check below, which then also applies to the fallback layout)
  if (tslots >= 200000 && tslots < 300000 && WS > 7) tslots = 1206;  // split form: a texture's 3 * 81 samples exceed its registers
  // a request's textures must fit one chunk (TSLOTS >= tau, tau <= PMVS_MAX_TAU = 16): smaller
  // chunk configs are only valid for small tau, otherwise the default 24-slot kernel runs
  if (tslots / 100 < s.tau) {
    tslots = 2408;
    refine_grid = refine_grid / 2 > 0 ? refine_grid / 2 : 1;  // 39 KB LDS: 4 resident per CU
  }
  const int nc = tslots % 100;
  const int rg = refine_grid < (n + nc - 1) / nc ? refine_grid : (n + nc - 1) / nc;
  if (tslots >= 200000) {  // split form (pmvs_refine_split.hip)
    if ((e = launch_refine_split(tslots, s, d_jobs, n, d_st, stream)) != hipSuccess) return e;
    if (refine_tail_on()) hipLaunchKernelGGL(refine_tail_kernel, dim3(1), dim3(64), 0, stream, d_st, 0);
    (void)hipEventRecord(ev[2], stream);
    hipLaunchKernelGGL((post_kernel<WS>), dim3(g), dim3(64), 0, stream, s, d_jobs, d_out, n, d_st);
    (void)hipEventRecord(ev[3], stream);
    dump_jobs(d_jobs, n, stream);
    return hipGetLastError();
  }
  if (tslots >= 100000) {  // workgroup form: 100000 + chains * 1000 + optimizer wavefronts * 10 + workgroups per CU
    const int ncw = (tslots / 1000) % 100, wgpc = tslots % 10;
    int dev = 0, cus = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess ||
        (e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
      return e;
    cus = cus > 0 ? cus : 1;
    // every CU gets a workgroup while the batch has candidates for them; a small batch runs fewer
    // chains per workgroup (nc_active) rather than fewer workgroups: its length is one chain's latency
    const int wgrid = cus * wgpc < n ? cus * wgpc : n;
    const int nca = (n + wgrid - 1) / wgrid < ncw ? (n + wgrid - 1) / wgrid : ncw;
#define PMVS_WG(NCc, OWc, WGPCc)                                                                                    \
  case 100000 + NCc * 1000 + OWc * 10 + WGPCc:                                                                       \
    hipLaunchKernelGGL((refine_wg_kernel<WS, NCc, RefWgFit<WS, NCc, WGPCc>::slots, OWc>), dim3(wgrid), dim3(WG_THREADS), \
                       0, stream, s, d_jobs, n, nca, d_st);                                                           \
    break;
    switch (tslots) {
      PMVS_WG(64, 1, 1)
      PMVS_WG(64, 2, 1)
      PMVS_WG(64, 4, 1)
      PMVS_WG(48, 4, 1)
      PMVS_WG(32, 2, 2)
      PMVS_WG(32, 4, 2)
      PMVS_WG(16, 4, 2)
      default: return hipErrorInvalidValue;
    }
#undef PMVS_WG
    if (refine_tail_on()) hipLaunchKernelGGL(refine_tail_kernel, dim3(1), dim3(64), 0, stream, d_st, 1);
    (void)hipEventRecord(ev[2], stream);
    hipLaunchKernelGGL((post_kernel<WS>), dim3(g), dim3(64), 0, stream, s, d_jobs, d_out, n, d_st);
    (void)hipEventRecord(ev[3], stream);
    return hipGetLastError();
  }
  // tslots = texture slots per objective chunk * 100 + optimizer chains per wavefront
  switch (tslots) {
    case 804: hipLaunchKernelGGL((refine_v2_kernel<WS, 8, 4>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 808: hipLaunchKernelGGL((refine_v2_kernel<WS, 8, 8>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 807: hipLaunchKernelGGL((refine_v2_kernel<WS, 8, 7>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1608: hipLaunchKernelGGL((refine_v2_kernel<WS, 16, 8>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 2408: hipLaunchKernelGGL((refine_v2_kernel<WS, 24, 8>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1204: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 4>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1201: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 1>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1202: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 2>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1203: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 3>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
#if defined(BQ_PRIVATE)
    case 1264: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 64>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 2464: hipLaunchKernelGGL((refine_v2_kernel<WS, 24, 64>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1232: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 32>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 2432: hipLaunchKernelGGL((refine_v2_kernel<WS, 24, 32>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 1216: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 16>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 2448: hipLaunchKernelGGL((refine_v2_kernel<WS, 24, 48>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 3232: hipLaunchKernelGGL((refine_v2_kernel<WS, 32, 32>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 3248: hipLaunchKernelGGL((refine_v2_kernel<WS, 32, 48>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 3264: hipLaunchKernelGGL((refine_v2_kernel<WS, 32, 64>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 4832: hipLaunchKernelGGL((refine_v2_kernel<WS, 48, 32>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
    case 4864: hipLaunchKernelGGL((refine_v2_kernel<WS, 48, 64>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
#endif
    default: hipLaunchKernelGGL((refine_v2_kernel<WS, 12, 6>), dim3(rg), dim3(64), 0, stream, s, d_jobs, n, d_st); break;
  }
  if (refine_tail_on()) hipLaunchKernelGGL(refine_tail_kernel, dim3(1), dim3(64), 0, stream, d_st, 0);
  (void)hipEventRecord(ev[2], stream);
  hipLaunchKernelGGL((post_kernel<WS>), dim3(g), dim3(64), 0, stream, s, d_jobs, d_out, n, d_st);
  (void)hipEventRecord(ev[3], stream);
  return hipGetLastError();
}

hipError_t launch_refine(const DScene& s, const pmvs_candidate* d_in, RefineJob* d_jobs, pmvs_refined* d_out, int n,
                         DevStats* d_st, int grid, int refine_grid, int tslots, hipStream_t stream, hipEvent_t* ev,
                         RefineHost& rh) {
  if (n <= 0) return hipSuccess;
  switch (s.wsize) {
    case 5: return launch_refine_ws<5>(s, d_in, d_jobs, d_out, n, d_st, grid, refine_grid, tslots, stream, ev, rh);
    case 7: return launch_refine_ws<7>(s, d_in, d_jobs, d_out, n, d_st, grid, refine_grid, tslots, stream, ev, rh);
    case 9: return launch_refine_ws<9>(s, d_in, d_jobs, d_out, n, d_st, grid, refine_grid, tslots, stream, ev, rh);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_incc_eval(const DScene& s, const pmvs_eval_query* d_q, int n, double* d_out, DevStats* d_st,
                            hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  switch (s.wsize) {
    case 5: hipLaunchKernelGGL((incc_eval_kernel<5>), dim3(n), dim3(64), 0, stream, s, d_q, n, d_out, d_st); break;
    case 7: hipLaunchKernelGGL((incc_eval_kernel<7>), dim3(n), dim3(64), 0, stream, s, d_q, n, d_out, d_st); break;
    case 9: hipLaunchKernelGGL((incc_eval_kernel<9>), dim3(n), dim3(64), 0, stream, s, d_q, n, d_out, d_st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_grab_tex(const DScene& s, const pmvs_tex_query* d_q, int n, float* d_out, int* d_valid,
                           hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  switch (s.wsize) {
    case 5: hipLaunchKernelGGL((grab_tex_kernel<5>), dim3(n), dim3(64), 0, stream, s, d_q, n, d_out, d_valid); break;
    case 7: hipLaunchKernelGGL((grab_tex_kernel<7>), dim3(n), dim3(64), 0, stream, s, d_q, n, d_out, d_valid); break;
    case 9: hipLaunchKernelGGL((grab_tex_kernel<9>), dim3(n), dim3(64), 0, stream, s, d_q, n, d_out, d_valid); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_build_level(const uint8_t* d_src, int Wp, int Hp, uint8_t* d_dst, int W, int H, hipStream_t stream) {
  if (W <= 0 || H <= 0) return hipSuccess;
  hipLaunchKernelGGL(build_level_kernel, dim3((W + 255) / 256, H), dim3(256), 0, stream, d_src, Wp, Hp, d_dst, W, H);
  return hipGetLastError();
}

hipError_t launch_pack_rgba(const uint8_t* d_rgb, uint32_t* d_out, long long npix, hipStream_t stream) {
  if (npix <= 0) return hipSuccess;
  hipLaunchKernelGGL(pack_rgba_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream, d_rgb, d_out, npix);
  return hipGetLastError();
}

hipError_t launch_unpack_rgba(const uint32_t* d_in, uint8_t* d_rgb, long long npix, hipStream_t stream) {
  if (npix <= 0) return hipSuccess;
  hipLaunchKernelGGL(unpack_rgba_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream, d_in, d_rgb, npix);
  return hipGetLastError();
}

}  // namespace pmvsdev

// ==================================================================== filterExact setRefImage
namespace pmvsdev {
// filterExact's "setRefImage(patch, 0); setGrids(patch)" (filter.cpp:340-343) for the listed
// patches: one wavefront per patch, the refine path's set_ref_image (pairwise INCC in the
// workgroup's global scratch), then CPatchOrganizerS::setGrids (patchOrganizerS.cpp:417-426).
// setRefImage's outcome applied to the record: the list as set_ref_image left it (images[0] swapped with
// the chosen reference, or emptied) and setGrids over it.
__device__ __forceinline__ void apply_ref_list(const DScene& s, pmvs_patch& q, const float* coord, int j, int img) {
  float ic[3];
  project(s.views[img], coord, s.level, ic);
  q.images[j] = (int16_t)img;
  q.grids[j][0] = grid16(((int)floorf(ic[0] + 0.5f)) / s.csize);
  q.grids[j][1] = grid16(((int)floorf(ic[1] + 0.5f)) / s.csize);
}

// refpos == nullptr: setRefImage + setGrids in place.  Otherwise (owner-partitioned filter pass) only
// the list entries whose reference image this rank owns (images[0] % world == rank) are evaluated and
// their outcome written to refpos[k] -- the list position swapped with position 0 (0: unchanged) or
// -1 (no target image: list cleared); apply_refpos_kernel applies the all-gathered outcomes.
template <int WS>
__global__ __launch_bounds__(64) void filter_refimage_kernel(DScene s, pmvs_patch* __restrict__ P,
                                                             const int* __restrict__ list, int m, int* __restrict__ refpos,
                                                             int rank, int world) {
  __shared__ WaveLds<WS> L;
  float* mat = s.scratch + (size_t)blockIdx.x * PMVS_MAX_IMAGES * PMVS_MAX_IMAGES;
  const int lane = lane_id();
  unsigned long long grabs = 0;
  for (int k = blockIdx.x; k < m; k += gridDim.x) {
    pmvs_patch& q = P[list[k]];
    const int n = q.num_images;
    if (refpos && __builtin_amdgcn_readfirstlane(q.images[0]) % world != rank) continue;  // wave-uniform
    for (int j = lane; j < n; j += WAVE) L.images[j] = q.images[j];
    if (lane == 0) { L.nimg = n; L.overflow = 0; }
    __syncthreads();
    float coord[4], normal[4];
    for (int i = 0; i < 4; ++i) { coord[i] = q.coord[i]; normal[i] = q.normal[i]; }
    set_ref_image<WS>(s, L, coord, normal, mat, &grabs);
    const int nn = L.nimg;
    if (refpos) {
      if (lane == 0) {
        int pos = -1;
        if (nn > 0) {
          pos = 0;
          for (int j = 1; j < n; ++j)
            if (q.images[j] == L.images[0]) pos = j;
        }
        refpos[k] = pos;
      }
      __syncthreads();
      continue;
    }
    for (int j = lane; j < nn; j += WAVE) apply_ref_list(s, q, coord, j, L.images[j]);
    if (lane == 0) q.num_images = nn;
    __syncthreads();
  }
}

// The owner-partitioned setRefImage's outcomes (all ranks' refpos, rank-major m ints each) applied on
// every rank: entry k's value comes from the rank owning its reference image.
__global__ void apply_refpos_kernel(DScene s, pmvs_patch* __restrict__ P, const int* __restrict__ list, int m,
                                    const int* __restrict__ allpos, int world) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  pmvs_patch& q = P[list[k]];
  const int pos = allpos[(size_t)(q.images[0] % world) * m + k];
  if (pos < 0) {
    q.num_images = 0;
    return;
  }
  if (pos > 0) {
    const int16_t t = q.images[0];
    q.images[0] = q.images[pos];
    q.images[pos] = t;
  }
  const float coord[4] = {q.coord[0], q.coord[1], q.coord[2], q.coord[3]};
  for (int j = 0; j < q.num_images; ++j) apply_ref_list(s, q, coord, j, q.images[j]);
}

hipError_t launch_filter_refimage(const DScene& s, pmvs_patch* P, const int* list, int m, int grid, hipStream_t stream,
                                  int* refpos, int rank, int world) {
  if (m <= 0) return hipSuccess;
  const int g = grid < m ? grid : m;
  switch (s.wsize) {
    case 5: hipLaunchKernelGGL((filter_refimage_kernel<5>), dim3(g), dim3(64), 0, stream, s, P, list, m, refpos, rank, world); break;
    case 7: hipLaunchKernelGGL((filter_refimage_kernel<7>), dim3(g), dim3(64), 0, stream, s, P, list, m, refpos, rank, world); break;
    case 9: hipLaunchKernelGGL((filter_refimage_kernel<9>), dim3(g), dim3(64), 0, stream, s, P, list, m, refpos, rank, world); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_apply_refpos(const DScene& s, pmvs_patch* P, const int* list, int m, const int* allpos, int world,
                               hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(apply_refpos_kernel, dim3((m + 255) / 256), dim3(256), 0, stream, s, P, list, m, allpos, world);
  return hipGetLastError();
}
}  // namespace pmvsdev

// ==================================================================== .ply colours
namespace pmvsdev {
// CPatchOrganizerS::writePLY colour mode 0 (patchOrganizerS.cpp:716-731): Vec3f sum of
// CPhotoSetS::getColor over the patch's images (project + bilinear at the scene level), divided
// by the image count, floor(c + 0.5f) clamped to 255.  One thread per patch.  Out-of-image
// projections (undefined reads in the reference) are clamped to the border texel.
__global__ void patch_colors_kernel(DScene s, int n, const float* __restrict__ coords, const int* __restrict__ off,
                                    const int* __restrict__ images, int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float c[4] = {coords[4 * i], coords[4 * i + 1], coords[4 * i + 2], coords[4 * i + 3]};
  float acc[3] = {0.0f, 0.0f, 0.0f};
  int denom = 0;
  for (int k = off[i]; k < off[i + 1]; ++k) {
    const DView& v = s.views[images[k]];
    float ic[3], rgb[3];
    project(v, c, s.level, ic);
    const float mx = (float)(v.w[s.level] - 2), my = (float)(v.h[s.level] - 2);
    const float x = ic[0] < 0.0f ? 0.0f : (ic[0] > mx ? mx : ic[0]);
    const float y = ic[1] < 0.0f ? 0.0f : (ic[1] > my ? my : ic[1]);
    get_color(s, v, x, y, s.level, rgb);
    acc[0] += rgb[0];
    acc[1] += rgb[1];
    acc[2] += rgb[2];
    denom++;
  }
  for (int j = 0; j < 3; ++j) {
    const float m = __fdiv_rn(acc[j], (float)denom);
    const int q = (int)floor((double)(m + 0.5f));
    out[3 * i + j] = q < 255 ? q : 255;
  }
}
hipError_t launch_patch_colors(const DScene& s, int n, const float* coords, const int* off, const int* images, int* out,
                               hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(patch_colors_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, s, n, coords, off, images, out);
  return hipGetLastError();
}
}  // namespace pmvsdev

// ==================================================================== model digest
namespace pmvsdev {
// pmvs_loop_hash: one wavefront per record at a time (grid-stride), its words read coalesced, each
// word mixed with its position and the record's index (splitmix64 finaliser); the per-lane sums
// and then every wavefront's sum are added (u64 addition: exact and order-free, so the digest does
// not depend on the schedule).
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(64) void model_digest_kernel(const uint32_t* __restrict__ recs, int n, int words,
                                                          unsigned long long* out) {
  const int lane = threadIdx.x;
  unsigned long long acc = 0;
  for (long long r = blockIdx.x; r < n; r += gridDim.x) {
    const uint32_t* p = recs + r * words;
    for (int w = lane; w < words; w += 64)
      acc += mix64((unsigned long long)p[w] ^ ((unsigned long long)w << 32) ^ ((unsigned long long)r * 0x9e3779b97f4a7c15ull));
  }
  for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d);
  if (lane == 0) atomicAdd(out, acc);
}

hipError_t launch_model_digest(const void* recs, int n, int record_bytes, unsigned long long* d_out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int dev = 0, cus = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev)) != hipSuccess ||
      (e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
    return e;
  const int grid = std::min(n, std::max(1, cus) * 32);
  hipLaunchKernelGGL(model_digest_kernel, dim3(grid), dim3(64), 0, stream, static_cast<const uint32_t*>(recs), n,
                     record_bytes / 4, d_out);
  return hipGetLastError();
}
}  // namespace pmvsdev

// ==================================================================== device math self-test
// Evaluates the device implementations of the libm functions the hot path uses, so tests can
// measure their agreement with the host libm (glibc) that the reference runs on.
namespace pmvsdev {
__global__ void math_selftest_kernel(int op, const double* __restrict__ in, double* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = in[i];
  double r;
  switch (op) {
    case 0: r = sqrt(x); break;
    case 1: r = sin(x); break;
    case 2: r = cos(x); break;
    case 3: r = asin(x); break;
    case 4: r = acos(x); break;
    case 5: r = atan(x); break;
    case 6: r = log(x); break;
    case 7: r = (double)__builtin_sqrtf((float)x); break;
    case 8: r = (double)__fdiv_rn((float)x, (float)in[(i + 1) % n]); break;
    case 9: r = floor(x); break;
    default: r = 0.0;
  }
  out[i] = r;
}
hipError_t launch_math_selftest(int op, const double* d_in, double* d_out, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(math_selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, op, d_in, d_out, n);
  return hipGetLastError();
}
}  // namespace pmvsdev

// ==================================================================== BOBYQA self-test
// Runs the device BOBYQA on analytic test objectives (same as oracle_bobyqa_test) so its
// trajectories can be checked against the CPU oracle and its cost measured.
//   mode 0: one problem per LANE, 64 per workgroup (state in LDS, as in the refine kernel)
//   mode 1: one problem per WAVE, lane 0 steps the state held in LDS (the v1 refine layout)
namespace pmvsdev {
__device__ __forceinline__ double bq_test_f(int kind, const double* v) {
  if (kind == 0) return (v[0] - 1.5) * (v[0] - 1.5) + 2 * (v[1] - 3) * (v[1] - 3) + 0.5 * (v[2] + 2) * (v[2] + 2) + 0.1 * v[0] * v[1];
  if (kind == 1) {
    const double a = 1 - v[0], b = v[1] - v[0] * v[0], c = v[2] - v[1] * v[1];
    return a * a + 100 * b * b + 100 * c * c;
  }
  if (kind == 3) {  // timing proxy of the refine objective: bounded, a basin plus a ripple
    const double q = 0.3 * (v[0] - 0.2) * (v[0] - 0.2) + 0.01 * (v[1] - 3) * (v[1] - 3) + 0.02 * (v[2] + 2) * (v[2] + 2);
    return 1.0 - exp(-q) + 0.02 * sin(3.0 * v[1]) * cos(2.0 * v[2]);
  }
  return (v[0] - 1) * (v[0] - 1) + (v[1] - 40) * (v[1] - 40) + (v[2] + 50) * (v[2] + 50);
}

// Lane-per-problem with the BOBYQA state resident in LDS (C problems per 64-lane workgroup).
template <int C>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BQ_CALLER_WPE))) void bobyqa_lds_kernel(int kind, const double* __restrict__ x0, int n, int maxeval,
                                                        double* __restrict__ out) {
  const int lane = threadIdx.x;
  const int i = blockIdx.x * C + lane;
#if defined(BQ_PRIVATE)
  BqState st_priv;
  if (lane >= C || i >= n) return;
  BQ_AS BqState& st = *(BQ_AS BqState*)&st_priv;
#else
  __shared__ BqState sts[C];
  if (lane >= C || i >= n) return;
  BQ_AS BqState& st = *(BQ_AS BqState*)&sts[lane];
#endif
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999}, ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  double x[3] = {x0[3 * i], x0[3 * i + 1], x0[3 * i + 2]};
  bq_begin(st, x, lb, ub, 1e-7, maxeval);
  double f = 0.0;
  while (bq_step(st, f) == BQ_NEED_F) f = bq_test_f(kind, st.xeval);
  out[6 * i + 0] = st.xout[0];
  out[6 * i + 1] = st.xout[1];
  out[6 * i + 2] = st.xout[2];
  out[6 * i + 3] = st.minf;
  out[6 * i + 4] = (double)st.nevals;
  out[6 * i + 5] = (double)st.rc;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BQ_CALLER_WPE))) void bobyqa_wave_kernel(int kind, const double* __restrict__ x0, int n, int maxeval,
                                                         double* __restrict__ out) {
#if defined(BQ_PRIVATE)
  BqState st_;  // lane 0's
#else
  __shared__ BqState st_;
#endif
  BQ_AS BqState& st = *(BQ_AS BqState*)&st_;
  __shared__ int stepv;
  __shared__ double fres, xes[3];
  const int i = blockIdx.x;
  if (i >= n) return;
  const int lane = threadIdx.x;
  if (lane == 0) {
    const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999}, ub[3] = {HUGE_VAL, 23.99999, 23.99999};
    double x[3] = {x0[3 * i], x0[3 * i + 1], x0[3 * i + 2]};
    bq_begin(st, x, lb, ub, 1e-7, maxeval);
    fres = 0.0;
  }
  __syncthreads();
  for (;;) {
    if (lane == 0) {
      stepv = bq_step(st, fres);
      for (int k = 0; k < 3; ++k) xes[k] = st.xeval[k];
    }
    __syncthreads();
    if (stepv != BQ_NEED_F) break;
    const double xe[3] = {xes[0], xes[1], xes[2]};
    const double f = bq_test_f(kind, xe);
    __syncthreads();
    if (lane == 0) fres = f;
    __syncthreads();
  }
  if (lane == 0) {
    out[6 * i + 0] = st.xout[0];
    out[6 * i + 1] = st.xout[1];
    out[6 * i + 2] = st.xout[2];
    out[6 * i + 3] = st.minf;
    out[6 * i + 4] = (double)st.nevals;
    out[6 * i + 5] = (double)st.rc;
  }
}

hipError_t launch_bobyqa_selftest(int mode, int kind, const double* d_x0, int n, int maxeval, double* d_out,
                                  hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (mode == 0)
    hipLaunchKernelGGL((bobyqa_lds_kernel<64>), dim3((n + 63) / 64), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  else if (mode == 1)
    hipLaunchKernelGGL(bobyqa_wave_kernel, dim3(n), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  else if (mode == 2)
    hipLaunchKernelGGL((bobyqa_lds_kernel<16>), dim3((n + 15) / 16), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  else if (mode == 3)
    hipLaunchKernelGGL((bobyqa_lds_kernel<32>), dim3((n + 31) / 32), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  else if (mode == 5)  // the wavefront form's chains per wave (timing)
    hipLaunchKernelGGL((bobyqa_lds_kernel<6>), dim3((n + 5) / 6), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  else if (mode == 6)
    hipLaunchKernelGGL((bobyqa_lds_kernel<48>), dim3((n + 47) / 48), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  else
    hipLaunchKernelGGL((bobyqa_lds_kernel<64>), dim3((n + 63) / 64), dim3(64), 0, stream, kind, d_x0, n, maxeval, d_out);
  return hipGetLastError();
}
}  // namespace pmvsdev

#if defined(BQ_PROFILE)
// Diagnostic build only: read and reset the optimizer sub-step profile.
extern "C" int pmvs_debug_bq_prof(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pmvsdev::bq_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(pmvsdev::bq_prof), z, sizeof(z)) != hipSuccess;
}
#endif
