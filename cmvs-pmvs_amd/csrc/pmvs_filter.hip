// pmvs_filter.hip -- one PMVS filter pass (PMVS3::CFilter::run, filter.cpp:13-27) on the device.
//
// The reference keeps CPatchOrganizerS cell lists of shared_ptrs (pgrids / vpgrids / dpgrids,
// patchOrganizerS.cpp) and walks them with CPU threads.  Here the organizer is rebuilt on the
// device from the patch array whenever it changes:
//   * registration masks: preg[p] (bit i = images[i] is registered in pgrids) and vreg[p]
//     (bit i = vimages[i] is registered in vpgrids) -- removePatch clears them;
//   * cell lists as CSR over a global cell index (target image offset + iy*gw + ix), built by
//     a radix sort of (cell << 32 | patch) keys, so each list is in patch-index (= insertion)
//     order exactly like the reference's vectors;
//   * collectPatches order = sort of (first registered cell << 32 | patch);
//   * depth maps (setDepthMaps) with a 64-bit atomicMin on (order-preserving depth bits << 32 |
//     collect rank): the smallest depth wins and ties go to the earlier patch, as the reference's
//     strict "depth < dtmp" over collect order.
// Kernels are one thread per patch (gains, vimages, visibility, small-group edges), one thread
// per cell entry (filterExact), one wavefront per patch (filterNeighbor: neighbour gather,
// sort/unique in LDS, Householder least squares in double), and the setRefImage of filterExact
// reuses the refine path's wavefront kernel (pmvs_kernels.hip).  The connected-component labels of
// filterSmallGroups are a breadth-first search over the device-computed, ordered edge lists on the
// host (the reference's label assignment is an order-dependent BFS; its cost is O(edges)).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <vector>

#include "pmvs_device.h"
#include "pmvs_launch.h"
#include "pmvs_layout.h"

namespace pmvsdev {

constexpr int NB_CAP = 1024;  // neighbours per patch in filterNeighbor (overflow is reported)
__device__ __forceinline__ int lane_id_w() { return threadIdx.x & 63; }

struct FilterDev {
  const DScene* dummy;
  pmvs_patch* P;
  int n;
  unsigned long long* preg;
  unsigned long long* vreg;
  const long long* tgoff;  // [tnum + 1] global cell offsets of the target images
  int tnum;
  // CSR organizer
  const int* pg_off; const int* pg_items;
  const int* vp_off; const int* vp_items;
  const unsigned long long* dpkey;
  const int* order;  // collect order -> patch
  const int* rank;   // patch -> collect rank or -1
  int nalive;
  const float* unit0;  // getUnit(images[0], coord) per patch
  long long ncells;
  int npg, nvp;        // entries in the pgrids / vpgrids lists
  int* err;            // [0] count, [1] first code (defensive bounds checks)
};



// --------------------------------------------------------------------------- small helpers
__device__ __forceinline__ unsigned int depth_bits(float d) {
  const unsigned int u = __float_as_uint(d);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float depth_of(const DView& v, const float* c) { return dot4(v.oaxis, c); }
__device__ __forceinline__ bool in_grid(const DScene& s, int t, int ix, int iy) {
  return 0 <= ix && ix < (s.views[t].w[s.level] + s.csize - 1) / s.csize && 0 <= iy &&
         iy < (s.views[t].h[s.level] + s.csize - 1) / s.csize;
}
__device__ __forceinline__ int gwidth(const DScene& s, int t) { return (s.views[t].w[s.level] + s.csize - 1) / s.csize; }
__device__ __forceinline__ int gheight(const DScene& s, int t) { return (s.views[t].h[s.level] + s.csize - 1) / s.csize; }

// CFindMatch::isNeighbor / isNeighborRadius (findMatch.cpp:125-185).
__device__ int is_neighbor_h(const pmvs_patch& l, const pmvs_patch& r, float hunit, float thr, float radius,
                             bool use_radius) {
  if ((double)dot4(l.normal, r.normal) < cos(120.0 * M_PI / 180.0)) return 0;
  float diff[4];
  for (int k = 0; k < 4; ++k) diff[k] = r.coord[k] - l.coord[k];
  const float vunit = l.dscale + r.dscale;
  const float f0 = dot4(l.normal, diff), f1 = dot4(r.normal, diff);
  float ftmp = (float)(((double)fabsf(f0) + (double)fabsf(f1)) / 2.0);
  ftmp = __fdiv_rn(ftmp, vunit);
  float v[4];
  for (int k = 0; k < 4; ++k) v[k] = (2.0f * diff[k] - l.normal[k] * f0) - r.normal[k] * f1;
  const float hsize = (float)((double)norm4(v) / 2.0 / (double)hunit);
  if (use_radius && __fdiv_rn(radius, hunit) < hsize) return 0;
  if (1.0 < hsize) ftmp = __fdiv_rn(ftmp, smin(2.0f, hsize));
  return ftmp < thr ? 1 : 0;
}
__device__ int is_neighbor(const DScene& s, const FilterDev& F, int a, int b, float thr) {
  const float hunit = (float)((double)(F.unit0[a] + F.unit0[b]) / 2.0 * s.csize);
  return is_neighbor_h(F.P[a], F.P[b], hunit, thr, 0.0f, false);
}

// CPatchOrganizerS::isVisible (patchOrganizerS.cpp:500-525).
__device__ int is_visible(const DScene& s, const FilterDev& F, int p, int t, int ix, int iy, float strict) {
  if (!in_grid(s, t, ix, iy)) return 0;
  if (s.depth == 0) return 1;
  const unsigned long long key = F.dpkey[F.tgoff[t] + (long long)iy * gwidth(s, t) + ix];
  if (key == ~0ull) return 1;
  const int d = F.order[(int)(key & 0xffffffffull)];
  const pmvs_patch& q = F.P[p];
  const DView& v = s.views[t];
  float ray[4] = {q.coord[0] - v.center[0], q.coord[1] - v.center[1], q.coord[2] - v.center[2], q.coord[3] - v.center[3]};
  unitize4(ray);
  float dd[4];
  for (int k = 0; k < 4; ++k) dd[k] = q.coord[k] - F.P[d].coord[k];
  const float diff = dot4(ray, dd);
  const double fd = 2.0 + (double)dot4(ray, q.normal);
  const float factor = (float)((fd < 2.0) ? fd : 2.0);  // std::min(2.0, .)
  return diff < get_unit(s, v, q.coord) * (float)s.csize * strict * factor ? 1 : 0;
}

// --------------------------------------------------------------------------- organizer build
// CPatchOrganizerS::addPatch (patchOrganizerS.cpp:308-324): register every target entry of the
// input patches (out-of-grid cells, undefined in the reference, are not registered).
__global__ void init_reg_kernel(DScene s, const pmvs_patch* __restrict__ P, int n, unsigned long long* __restrict__ preg,
                                unsigned long long* __restrict__ vreg) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const pmvs_patch& q = P[p];
  unsigned long long m = 0ull;
  for (int i = 0; i < q.num_images; ++i)
    if (q.images[i] < s.tnum && in_grid(s, q.images[i], q.grids[i][0], q.grids[i][1])) m |= 1ull << i;
  preg[p] = m;
  vreg[p] = 0ull;
}

__global__ void keep_kernel(int n, const unsigned long long* __restrict__ preg, const int* __restrict__ rank,
                            int* __restrict__ keep) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  keep[p] = (rank[p] >= 0) ? 1 : 0;
}

__global__ void count_entries_kernel(const pmvs_patch* __restrict__ P, int n, const unsigned long long* __restrict__ reg,
                                     int vis, int* __restrict__ cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  cnt[p] = __popcll(reg[p]);
}

__global__ void emit_entries_kernel(DScene s, const pmvs_patch* __restrict__ P, int n,
                                    const unsigned long long* __restrict__ reg, int vis, const int* __restrict__ off,
                                    const long long* __restrict__ tgoff, unsigned long long* __restrict__ keys) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  unsigned long long m = reg[p];
  int o = off[p];
  const pmvs_patch& q = P[p];
  while (m) {
    const int i = __builtin_ctzll(m);
    m &= m - 1;
    const int t = vis ? q.vimages[i] : q.images[i];
    const int ix = vis ? q.vgrids[i][0] : q.grids[i][0];
    const int iy = vis ? q.vgrids[i][1] : q.grids[i][1];
    const unsigned long long cell = (unsigned long long)(tgoff[t] + (long long)iy * gwidth(s, t) + ix);
    keys[o++] = (cell << 32) | (unsigned)p;
  }
}

__global__ void cell_hist_kernel(const unsigned long long* __restrict__ keys, int e, int* __restrict__ cnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e) return;
  atomicAdd(&cnt[(long long)(keys[i] >> 32)], 1);
}

__global__ void items_kernel(const unsigned long long* __restrict__ keys, int e, int* __restrict__ items) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e) return;
  items[i] = (int)(keys[i] & 0xffffffffull);
}

// first registered pgrids cell of each patch (collectPatches order key)
__global__ void first_cell_kernel(DScene s, const pmvs_patch* __restrict__ P, int n,
                                  const unsigned long long* __restrict__ preg, const long long* __restrict__ tgoff,
                                  unsigned long long* __restrict__ keys, int* __restrict__ nalive) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  unsigned long long m = preg[p];
  unsigned long long best = ~0ull;
  const pmvs_patch& q = P[p];
  while (m) {
    const int i = __builtin_ctzll(m);
    m &= m - 1;
    const int t = q.images[i];
    const unsigned long long cell = (unsigned long long)(tgoff[t] + (long long)q.grids[i][1] * gwidth(s, t) + q.grids[i][0]);
    if (cell < best) best = cell;
  }
  keys[p] = (best == ~0ull) ? ~0ull : ((best << 32) | (unsigned)p);
  if (best != ~0ull) atomicAdd(nalive, 1);
}

__global__ void rank_kernel(const unsigned long long* __restrict__ keys, int nalive, int* __restrict__ order,
                            int* __restrict__ rank) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nalive) return;
  const int p = (int)(keys[i] & 0xffffffffull);
  order[i] = p;
  rank[p] = i;
}

__global__ void unit0_kernel(DScene s, const pmvs_patch* __restrict__ P, int n, float* __restrict__ unit0) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  unit0[p] = P[p].num_images > 0 ? get_unit(s, s.views[P[p].images[0]], P[p].coord) : 0.0f;
}

// CFilter::setDepthMapsThread (filter.cpp:689-725): one thread per (collected patch, target).
__global__ void depth_map_kernel(DScene s, FilterDev F, unsigned long long* __restrict__ dpkey) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)F.nalive * F.tnum) return;
  const int i = (int)(g / F.tnum), t = (int)(g - (long long)i * F.tnum);
  const pmvs_patch& q = F.P[F.order[i]];
  const DView& v = s.views[t];
  float ic[3];
  project(v, q.coord, s.level, ic);
  const float fx = __fdiv_rn(ic[0], (float)s.csize), fy = __fdiv_rn(ic[1], (float)s.csize);
  const int xs[2] = {(int)floor((double)fx), (int)ceil((double)fx)};
  const int ys[2] = {(int)floor((double)fy), (int)ceil((double)fy)};
  const unsigned long long key = ((unsigned long long)depth_bits(depth_of(v, q.coord)) << 32) | (unsigned)i;
  const int gw = gwidth(s, t), gh = gheight(s, t);
  for (int j = 0; j < 2; ++j)
    for (int k = 0; k < 2; ++k) {
      if (xs[k] < 0 || gw <= xs[k] || ys[j] < 0 || gh <= ys[j]) continue;
      atomicMin(&dpkey[F.tgoff[t] + (long long)ys[j] * gw + xs[k]], key);
    }
}

// CPatchOrganizerS::setVImagesVGrids (patchOrganizerS.cpp:429-459) per collected patch;
// vreg = every vimages entry (addPatchVThread registers the first entry per image, and the
// list never holds an image twice).
__global__ void vimages_kernel(DScene s, FilterDev F, int additive, unsigned long long* __restrict__ vreg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F.nalive) return;
  const int p = F.order[i];
  pmvs_patch& q = F.P[p];
  if (!additive) q.num_vimages = 0;
  unsigned long long used = 0ull;  // bit t (tnum <= 64)
  for (int k = 0; k < q.num_images; ++k)
    if (q.images[k] < s.tnum) used |= 1ull << q.images[k];
  for (int k = 0; k < q.num_vimages; ++k) used |= 1ull << q.vimages[k];
  for (int t = 0; t < s.tnum; ++t) {
    if (used & (1ull << t)) continue;
    const DView& v = s.views[t];
    float ic[3];
    project(v, q.coord, s.level, ic);
    const int ix = ((int)floorf(ic[0] + 0.5f)) / s.csize;
    const int iy = ((int)floorf(ic[1] + 0.5f)) / s.csize;
    if (is_visible(s, F, p, t, ix, iy, 0.5f) == 0) continue;
    if (get_edge(s, v, q.coord, s.level) == 0) continue;
    if (q.num_vimages >= PMVS_MAX_IMAGES) break;
    q.vimages[q.num_vimages] = t;
    q.vgrids[q.num_vimages][0] = ix;
    q.vgrids[q.num_vimages][1] = iy;
    q.num_vimages++;
  }
  vreg[p] = (q.num_vimages >= 64) ? ~0ull : ((1ull << q.num_vimages) - 1ull);
}

// --------------------------------------------------------------------------- filterOutside
// CFilter::filterOutsideThread (filter.cpp:148-201), neighbourThreshold1 = 1.0.
__global__ void gain_kernel(DScene s, FilterDev F, int* __restrict__ remove) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F.nalive) return;
  const int p = F.order[i];
  const pmvs_patch& q = F.P[p];
  remove[p] = 0;
  if (q.fix) return;
  float gain = smax(0.0f, q.ncc - s.nccThreshold) * (float)q.timages;
  for (int k = 0; k < q.num_images; ++k) {
    const int t = q.images[k];
    if (s.tnum <= t) continue;
    const long long c = F.tgoff[t] + (long long)q.grids[k][1] * gwidth(s, t) + q.grids[k][0];
    float maxp = 0.0f;
    for (int e = F.pg_off[c]; e < F.pg_off[c + 1]; ++e) {
      const int j = F.pg_items[e];
      if (!is_neighbor(s, F, p, j, 1.0f)) maxp = smax(maxp, F.P[j].ncc - s.nccThreshold);
    }
    gain -= maxp;
  }
  for (int k = 0; k < q.num_vimages; ++k) {
    const int t = q.vimages[k];
    if (s.tnum <= t) continue;
    const float pdepth = depth_of(s.views[t], q.coord);
    const long long c = F.tgoff[t] + (long long)q.vgrids[k][1] * gwidth(s, t) + q.vgrids[k][0];
    float maxp = 0.0f;
    for (int e = F.pg_off[c]; e < F.pg_off[c + 1]; ++e) {
      const int j = F.pg_items[e];
      const float bdepth = depth_of(s.views[t], F.P[j].coord);
      if (pdepth < bdepth && !is_neighbor(s, F, p, j, 1.0f)) maxp = smax(maxp, F.P[j].ncc - s.nccThreshold);
    }
    gain -= maxp;
  }
  remove[p] = (gain < 0.0) ? 1 : 0;
}

__global__ void clear_fixed_kernel(const pmvs_patch* __restrict__ P, int n, int* __restrict__ flags) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (P[p].fix) flags[p] = 0;
}

__global__ void apply_remove_kernel(int n, const int* __restrict__ remove, unsigned long long* __restrict__ preg,
                                    unsigned long long* __restrict__ vreg, int* __restrict__ count) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (remove[p]) {
    preg[p] = 0ull;
    vreg[p] = 0ull;
    atomicAdd(count, 1);
  }
}

// --------------------------------------------------------------------------- filterExact
// filterExactThread (filter.cpp:291-340): one thread per registered pgrids entry; marks the
// patch's images[] positions that are safe (visible at the cell or one of its 4 neighbours).
__global__ void exact_entries_kernel(DScene s, FilterDev F, long long ncells, unsigned long long* __restrict__ safe) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncells) return;
  const int b = F.pg_off[c], e = F.pg_off[c + 1];
  if (b == e) return;
  int t = 0;
  while (F.tgoff[t + 1] <= c) ++t;
  const int gw = gwidth(s, t), h = gheight(s, t);
  const long long local = c - F.tgoff[t];
  const int y = (int)(local / gw), x = (int)(local - (long long)y * gw);
  for (int k = b; k < e; ++k) {
    const int p = F.pg_items[k];
    const pmvs_patch& q = F.P[p];
    if (q.fix) continue;
    int ok = 0;
    if (is_visible(s, F, p, t, x, y, 1.0f)) ok = 1;
    else if (0 < x && is_visible(s, F, p, t, x - 1, y, 1.0f)) ok = 1;
    else if (x < gw - 1 && is_visible(s, F, p, t, x + 1, y, 1.0f)) ok = 1;
    else if (0 < y && is_visible(s, F, p, t, x, y - 1, 1.0f)) ok = 1;
    else if (y < h - 1 && is_visible(s, F, p, t, x, y + 1, 1.0f)) ok = 1;
    if (ok)
      for (int i = 0; i < q.num_images; ++i)
        if (q.images[i] == t) {
          atomicOr(&safe[p], 1ull << i);
          break;
        }
  }
}

// filterExact (filter.cpp:234-348) per collected, non-fixed patch: new list = safe targets in
// increasing image order (the reference's image-major scan) with their cells, then the
// non-target images; _timages = #safe.  need_ref[p] = 1 when setRefImage + setGrids follow.
__global__ void exact_patch_kernel(DScene s, FilterDev F, const unsigned long long* __restrict__ safe,
                                   unsigned long long* __restrict__ preg, unsigned long long* __restrict__ vreg,
                                   int* __restrict__ need_ref, int* __restrict__ removed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F.nalive) return;
  const int p = F.order[i];
  pmvs_patch& q = F.P[p];
  need_ref[p] = 0;
  if (q.fix) return;
  const unsigned long long sm = safe[p] & preg[p];
  int ni = 0;
  int imgs[PMVS_MAX_IMAGES], grd[PMVS_MAX_IMAGES][2];
  for (int t = 0; t < s.tnum; ++t)
    for (int k = 0; k < q.num_images; ++k)
      if (q.images[k] == t && ((sm >> k) & 1ull)) {
        imgs[ni] = t;
        grd[ni][0] = q.grids[k][0];
        grd[ni][1] = q.grids[k][1];
        ni++;
      }
  q.timages = ni;
  for (int k = 0; k < q.num_images; ++k)
    if (s.tnum <= q.images[k]) {
      imgs[ni] = q.images[k];
      grd[ni][0] = q.grids[k][0];
      grd[ni][1] = q.grids[k][1];
      ni++;
    }
  for (int k = 0; k < ni; ++k) {
    q.images[k] = imgs[k];
    q.grids[k][0] = grd[k][0];
    q.grids[k][1] = grd[k][1];
  }
  q.num_images = ni;
  unsigned long long m = 0ull;
  for (int k = 0; k < q.timages; ++k) m |= 1ull << k;
  preg[p] = m;
  if (s.minImageNum <= ni) {
    need_ref[p] = 1;
  } else {
    preg[p] = 0ull;
    vreg[p] = 0ull;
    atomicAdd(removed, 1);
  }
}

// after setRefImage: registered = target entries of the (reordered) list; empty list -> removed
__global__ void exact_after_ref_kernel(DScene s, const pmvs_patch* __restrict__ P, const int* __restrict__ list, int m,
                                       unsigned long long* __restrict__ preg, unsigned long long* __restrict__ vreg,
                                       int* __restrict__ removed) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const int p = list[k];
  const pmvs_patch& q = P[p];
  if (q.num_images < s.minImageNum) {
    preg[p] = 0ull;
    vreg[p] = 0ull;
    atomicAdd(removed, 1);
    return;
  }
  unsigned long long r = 0ull;
  for (int i = 0; i < q.num_images; ++i)
    if (q.images[i] < s.tnum) r |= 1ull << i;
  preg[p] = r;
}

// --------------------------------------------------------------------------- filterNeighbor
struct NbLds {
  int nb[NB_CAP];
  float fx[NB_CAP], fy[NB_CAP], fz[NB_CAP];
  float units[PMVS_MAX_IMAGES];
  int cnt, overflow;
  double R[5][5], xs[5], f[5];
  float x[5];
};

// Householder least squares (the oracle's lls5, same operation order), rows in global scratch.
__device__ void lls5_wave(NbLds& L, double* M, double* r, int n) {
  const int lane = lane_id_w();
  for (int k = 0; k < 5; ++k) {
    if (lane == 0) {
      double nrm = 0.0;
      for (int i = k; i < n; ++i) nrm += M[(size_t)i * 5 + k] * M[(size_t)i * 5 + k];
      nrm = sqrt(nrm);
      const double akk = M[(size_t)k * 5 + k];
      const double alpha = (akk > 0.0) ? -nrm : nrm;
      M[(size_t)k * 5 + k] = akk - alpha;
      double vnorm2 = 0.0;
      for (int i = k; i < n; ++i) vnorm2 += M[(size_t)i * 5 + k] * M[(size_t)i * 5 + k];
      L.R[k][k] = alpha;
      L.f[0] = vnorm2;
    }
    __syncthreads();
    const double vnorm2 = L.f[0];
    if (vnorm2 > 0.0) {
      // columns j > k and the right-hand side: one lane each, sequential dot over rows
      const int j = k + 1 + lane;
      if (lane < 5 - k) {
        double dotv = 0.0;
        if (j < 5) {
          for (int i = k; i < n; ++i) dotv += M[(size_t)i * 5 + k] * M[(size_t)i * 5 + j];
          const double fj = 2.0 * dotv / vnorm2;
          for (int i = k; i < n; ++i) M[(size_t)i * 5 + j] -= fj * M[(size_t)i * 5 + k];
        } else {
          for (int i = k; i < n; ++i) dotv += M[(size_t)i * 5 + k] * r[i];
          const double fb = 2.0 * dotv / vnorm2;
          for (int i = k; i < n; ++i) r[i] -= fb * M[(size_t)i * 5 + k];
        }
      }
    }
    __syncthreads();
    if (lane == 0)
      for (int jj = k + 1; jj < 5; ++jj) L.R[k][jj] = M[(size_t)k * 5 + jj];
    __syncthreads();
  }
  if (lane == 0) {
    for (int k = 4; k >= 0; --k) {
      double v = r[k];
      for (int j = k + 1; j < 5; ++j) v -= L.R[k][j] * L.xs[j];
      L.xs[k] = (L.R[k][k] != 0.0) ? v / L.R[k][k] : 0.0;
    }
    for (int k = 0; k < 5; ++k) L.x[k] = (float)L.xs[k];
  }
  __syncthreads();
}

// Sort a[0..n) ascending (bitonic over the next power of two, padded with INT_MAX) and drop
// duplicates; returns the unique count.  All 64 lanes call it.
__device__ int sort_unique_lds(int* a, int n, int* cnt_slot) {
  const int lane = lane_id_w();
  int N = 1;
  while (N < n) N <<= 1;
  for (int i = n + lane; i < N; i += 64) a[i] = 0x7fffffff;
  __syncthreads();
  for (int k = 2; k <= N; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < N; i += 64) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const int x = a[i], y = a[ixj];
          if ((x > y) == up) { a[i] = y; a[ixj] = x; }
        }
      }
      __syncthreads();
    }
  if (lane == 0) {
    int u = 0;
    for (int i = 0; i < n; ++i)
      if (u == 0 || a[i] != a[u - 1]) a[u++] = a[i];
    *cnt_slot = u;
  }
  __syncthreads();
  return *cnt_slot;
}

// CFilter::filterNeighborThread (filter.cpp:358-385) + findNeighbors(..., 0, 4, 2, 1)
// (patchOrganizerS.cpp:527-631) + filterQuad (filter.cpp:387-446), one wavefront per patch.
__global__ __launch_bounds__(64) void neighbor_kernel(DScene s, FilterDev F, double* __restrict__ scratch,
                                                      int* __restrict__ reject, int* __restrict__ overflow,
                                                      int* __restrict__ queue, int* __restrict__ dbg_counts) {
  __shared__ NbLds L;
  const int lane = threadIdx.x;
  double* M = scratch + (size_t)blockIdx.x * NB_CAP * 6;
  double* r = M + (size_t)NB_CAP * 5;
  for (;;) {
    int i = 0;
    if (lane == 0) i = atomicAdd(queue, 1);
    i = __shfl(i, 0);  // work-queue index broadcast in registers
    if (i >= F.nalive) break;
    const int p = F.order[i];
    const pmvs_patch& q = F.P[p];
    if (q.fix) {
      if (lane == 0) reject[p] = 0;
      continue;
    }
    __syncthreads();  // the previous patch's LDS reads are complete before L is reused
    // computeRadius: 2nd smallest of computeUnits (optim.cpp:446-471) times csize
    int ni = q.num_images;
    if (ni < 1 || ni > PMVS_MAX_IMAGES) { if (lane == 0) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 31); } ni = 1; }
    if (lane < ni) {
      const DView& v = s.views[q.images[lane]];
      float u = get_unit(s, v, q.coord);
      float ray[4] = {v.center[0] - q.coord[0], v.center[1] - q.coord[1], v.center[2] - q.coord[2], v.center[3] - q.coord[3]};
      unitize4(ray);
      const float den = dot4(ray, q.normal);
      u = (0.0f < den) ? __fdiv_rn(u, den) : 1073741824.0f;
      L.units[lane] = u;
    }
    if (lane == 0) { L.cnt = 0; L.overflow = 0; }
    __syncthreads();
    float radius = 0.0f, unit = 0.0f;
    {
      float m1 = 3.0e38f, m2 = 3.0e38f;  // two smallest (nth_element(begin, begin + 1, end))
      for (int k = 0; k < ni; ++k) {
        const float u = L.units[k];
        if (u < m1) { m2 = m1; m1 = u; }
        else if (u < m2) m2 = u;
      }
      radius = (float)(1.5 * 2 * (double)(m2 * (float)s.csize));
      for (int k = 0; k < ni; ++k) unit += get_unit(s, s.views[q.images[k]], q.coord);
      unit = __fdiv_rn(unit, (float)ni);
      unit *= (float)s.csize;
    }
    const float thr = 0.5f * 4.0f;
    // gather: target entries of images[], 5x5 cells, pgrids then vpgrids
    for (int k = 0; k < ni; ++k) {
      const int t = q.images[k];
      if (s.tnum <= t) continue;
      const int gw = gwidth(s, t), gh = gheight(s, t);
      for (int dy = -2; dy <= 2; ++dy) {
        const int yt = q.grids[k][1] + dy;
        if (yt < 0 || gh <= yt) continue;
        for (int dx = -2; dx <= 2; ++dx) {
          const int xt = q.grids[k][0] + dx;
          if (xt < 0 || gw <= xt) continue;
          const long long c = F.tgoff[t] + (long long)yt * gw + xt;
          if (c < 0 || c >= F.ncells) { if (lane == 0) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 11); } continue; }
          for (int lst = 0; lst < 2; ++lst) {
            const int* off = lst ? F.vp_off : F.pg_off;
            const int* items = lst ? F.vp_items : F.pg_items;
            const int lim = lst ? F.nvp : F.npg;
            int b = off[c], e = off[c + 1];
            if (b < 0 || e > lim || b > e) {
              if (lane == 0) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 12 + lst); }
              b = 0; e = 0;
            }
            for (int base = b; base < e; base += 64) {
              const int idx = base + lane;
              bool hit = false;
              int j = 0;
              if (idx < e) {
                j = items[idx];
                if (j < 0 || j >= F.n) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 14); j = 0; }
                else hit = is_neighbor_h(q, F.P[j], unit, thr, radius, true) != 0;
              }
              const unsigned long long mask = __ballot(hit);
              const int before = __popcll(mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
              const int pos = L.cnt + before;
              if (hit) {
                if (pos < NB_CAP) L.nb[pos] = j;
                else L.overflow = 1;
              }
              __syncthreads();
              if (lane == 0) L.cnt += __popcll(mask);
              __syncthreads();
              // duplicates (one entry per image/cell registration) are compacted when the
              // buffer fills; the reference sorts and uniques once at the end (same set)
              if (L.cnt > NB_CAP - 64 && !L.overflow) sort_unique_lds(L.nb, imin(L.cnt, NB_CAP), &L.cnt);
            }
          }
        }
      }
    }
    int n = L.cnt < NB_CAP ? L.cnt : NB_CAP;
    n = sort_unique_lds(L.nb, n, &L.cnt);
    if (lane == 0 && L.overflow) atomicAdd(overflow, 1);
    if (lane == 0 && dbg_counts) dbg_counts[p] = L.overflow ? -n : n;
    __syncthreads();
    n = L.cnt;
    if (n > NB_CAP || n < 0) { if (lane == 0) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 21); } n = 0; }
    for (int a = lane; a < n; a += 64)
      if (L.nb[a] < 0 || L.nb[a] >= F.n) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 22); L.nb[a] = p; }
    __syncthreads();
    int rej = 0;
    if (n < 6) {
      rej = 1;
    } else {
      // filterQuad (filter.cpp:387-446)
      float xdir[4] = {0, 0, 0, 0}, ydir[4] = {0, 0, 0, 0};
      const float* z = q.normal;
      if (fabs((double)z[0]) > 0.5) { xdir[0] = z[1]; xdir[1] = -z[0]; xdir[2] = 0; }
      else if (fabs((double)z[1]) > 0.5) { xdir[1] = z[2]; xdir[2] = -z[1]; xdir[0] = 0; }
      else { xdir[2] = z[0]; xdir[0] = -z[2]; xdir[1] = 0; }
      unitize4(xdir);
      ydir[0] = z[1] * xdir[2] - z[2] * xdir[1];
      ydir[1] = z[2] * xdir[0] - z[0] * xdir[2];
      ydir[2] = z[0] * xdir[1] - z[1] * xdir[0];
      if (lane == 0) {
        float h = 0.0f;
        for (int a = 0; a < n; ++a) {
          float d[4];
          for (int k = 0; k < 4; ++k) d[k] = F.P[L.nb[a]].coord[k] - q.coord[k];
          h += norm4(d);
        }
        L.f[1] = (double)__fdiv_rn(h, (float)n);
      }
      __syncthreads();
      const float h = (float)L.f[1];
      for (int a = lane; a < n; a += 64) {
        float d[4];
        for (int k = 0; k < 4; ++k) d[k] = F.P[L.nb[a]].coord[k] - q.coord[k];
        const float fx = __fdiv_rn(dot4(d, xdir), h), fy = __fdiv_rn(dot4(d, ydir), h), fz = dot4(d, q.normal);
        L.fx[a] = fx; L.fy[a] = fy; L.fz[a] = fz;
        M[(size_t)a * 5 + 0] = (double)(fx * fx);
        M[(size_t)a * 5 + 1] = (double)(fy * fy);
        M[(size_t)a * 5 + 2] = (double)(fx * fy);
        M[(size_t)a * 5 + 3] = (double)fx;
        M[(size_t)a * 5 + 4] = (double)fy;
        r[a] = (double)fz;
      }
      __threadfence_block();
      __syncthreads();
      lls5_wave(L, M, r, n);
      if (lane == 0) {
        const int inum = imin(s.tau, q.num_images);
        float u2 = 0.0f;
        for (int k = 0; k < inum; ++k) u2 += get_unit(s, s.views[q.images[k]], q.coord);
        u2 = __fdiv_rn(u2, (float)inum);
        float residual = 0.0f;
        for (int a = 0; a < n; ++a) {
          const float fx = L.fx[a], fy = L.fy[a];
          const float res = L.x[0] * (fx * fx) + L.x[1] * (fy * fy) + L.x[2] * (fx * fy) + L.x[3] * fx + L.x[4] * fy - L.fz[a];
          residual = (float)((double)residual + fabs((double)res) / (double)u2);  // float += double
        }
        residual = __fdiv_rn(residual, (float)(n - 5));
        L.cnt = (residual < s.quad ? 0 : 1);
      }
      __syncthreads();
      rej = L.cnt;
    }
    if (lane == 0) reject[p] = rej;
    __syncthreads();
  }
}

// --------------------------------------------------------------------------- filterSmallGroups
// filterSmallGroupsSub (filter.cpp:630-666): ordered neighbour scan of the 3x3 cells around
// the reference-image cell, pgrids then vpgrids, isNeighbor(threshold2 = 1.0); pass 0 counts,
// pass 1 writes collect ranks.
__global__ void group_edges_kernel(DScene s, FilterDev F, int pass, const int* __restrict__ off, int* __restrict__ cnt,
                                   int* __restrict__ edges) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F.nalive) return;
  const int p = F.order[i];
  const pmvs_patch& q = F.P[p];
  const int t = q.images[0], ix = q.grids[0][0], iy = q.grids[0][1];
  const int gw = gwidth(s, t), gh = gheight(s, t);
  int k = 0;
  int o = pass ? off[i] : 0;
  for (int y = -1; y <= 1; ++y) {
    const int yt = iy + y;
    if (yt < 0 || gh <= yt) continue;
    for (int x = -1; x <= 1; ++x) {
      const int xt = ix + x;
      if (xt < 0 || gw <= xt) continue;
      const long long c = F.tgoff[t] + (long long)yt * gw + xt;
      for (int lst = 0; lst < 2; ++lst) {
        const int* off2 = lst ? F.vp_off : F.pg_off;
        const int* items = lst ? F.vp_items : F.pg_items;
        for (int e = off2[c]; e < off2[c + 1]; ++e) {
          const int j = items[e];
          if (is_neighbor(s, F, p, j, 1.0f)) {
            if (pass) edges[o + k] = F.rank[j];
            ++k;
          }
        }
      }
    }
  }
  if (!pass) cnt[i] = k;
}


// ============================================================================ host orchestration
#define FCHK(x)                          \
  do {                                   \
    hipError_t e_ = (x);                 \
    if (e_ != hipSuccess) return e_;     \
  } while (0)

static inline unsigned nblk(long long n, int b = 256) { return (unsigned)((n + b - 1) / b); }

static void dbg(hipStream_t st, const char* what) {
  static const bool on = getenv("PMVS_FILTER_DEBUG") != nullptr;
  if (!on) return;
  const hipError_t e = hipStreamSynchronize(st);
  fprintf(stderr, "[filter] %s: %s\n", what, hipGetErrorString(e));
  fflush(stderr);
}

template <class T>
static hipError_t dalloc(T*& p, size_t n) {
  if (p) (void)hipFree(p);
  p = nullptr;
  return hipMalloc((void**)&p, (n ? n : 1) * sizeof(T));
}

FilterBuffers::~FilterBuffers() {
  void* ps[] = {preg, vreg, tgoff, cnt, off, keys, keys2, cellcnt, pg_off, pg_items, vp_off, vp_items, dpkey,
                order, rank, unit0, flags, safe, need, list, scratch, counters, temp, edge_off, edges};
  for (void* p : ps)
    if (p) (void)hipFree(p);
}

hipError_t FilterBuffers::reserve(int n_, long long ncells_, int tnum_, int grid_) {
  if (n_ <= cap_n && ncells_ <= cap_cells && grid_ <= cap_grid) return hipSuccess;
  cap_n = std::max(n_, cap_n);
  cap_cells = std::max(ncells_, cap_cells);
  cap_grid = std::max(grid_, cap_grid);
  const size_t ne = (size_t)cap_n * PMVS_MAX_IMAGES;
  FCHK(dalloc(preg, cap_n)); FCHK(dalloc(vreg, cap_n)); FCHK(dalloc(tgoff, 65));
  FCHK(dalloc(cnt, cap_n + 1)); FCHK(dalloc(off, cap_n + 1));
  FCHK(dalloc(keys, std::max(ne, (size_t)cap_n))); FCHK(dalloc(keys2, std::max(ne, (size_t)cap_n)));
  FCHK(dalloc(cellcnt, cap_cells + 1)); FCHK(dalloc(pg_off, cap_cells + 1)); FCHK(dalloc(vp_off, cap_cells + 1));
  FCHK(dalloc(pg_items, ne)); FCHK(dalloc(vp_items, ne)); FCHK(dalloc(dpkey, cap_cells));
  FCHK(dalloc(order, cap_n)); FCHK(dalloc(rank, cap_n)); FCHK(dalloc(unit0, cap_n)); FCHK(dalloc(flags, cap_n));
  FCHK(dalloc(safe, cap_n)); FCHK(dalloc(need, cap_n)); FCHK(dalloc(list, cap_n));
  FCHK(dalloc(scratch, (size_t)cap_grid * NB_CAP * 6)); FCHK(dalloc(counters, 8));
  FCHK(dalloc(edge_off, cap_n + 1));
  size_t t1 = 0, t2 = 0;
  FCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, keys, keys2, (int)ne));
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, cellcnt, pg_off, (int)(cap_cells + 1)));
  size_t t3 = 0;
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t3, cnt, off, cap_n + 1));
  temp_bytes = std::max(t1, std::max(t2, t3));
  if (temp) (void)hipFree(temp);
  temp = nullptr;
  FCHK(hipMalloc(&temp, temp_bytes ? temp_bytes : 1));
  return hipSuccess;
}

namespace {

struct Ctx {
  const DScene& s;
  FilterBuffers& B;
  pmvs_patch* P;
  int n;
  long long ncells;
  int grid;
  hipStream_t st;
  int nalive = 0, npg = 0, nvp = 0;
  FilterDev dev() const {
    FilterDev F{};
    F.P = P; F.n = n; F.preg = B.preg; F.vreg = B.vreg; F.tgoff = B.tgoff; F.tnum = s.tnum;
    F.pg_off = B.pg_off; F.pg_items = B.pg_items; F.vp_off = B.vp_off; F.vp_items = B.vp_items;
    F.dpkey = B.dpkey; F.order = B.order; F.rank = B.rank; F.nalive = nalive; F.unit0 = B.unit0;
    F.ncells = ncells; F.npg = npg; F.nvp = nvp; F.err = B.counters + 6;
    return F;
  }
};

static hipError_t read_int(const int* d, int* h, hipStream_t st) {
  FCHK(hipMemcpyAsync(h, d, sizeof(int), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

// CSR cell lists from the registration masks (vis = 0: pgrids, 1: vpgrids)
static hipError_t build_lists(Ctx& c, int vis) {
  FilterBuffers& B = c.B;
  const unsigned long long* reg = vis ? B.vreg : B.preg;
  int* csr_off = vis ? B.vp_off : B.pg_off;
  int* items = vis ? B.vp_items : B.pg_items;
  hipLaunchKernelGGL(count_entries_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.P, c.n, reg, vis, B.cnt);
  FCHK(hipMemsetAsync(B.cnt + c.n, 0, sizeof(int), c.st));
  size_t tb = B.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cnt, B.off, c.n + 1, c.st));
  int e = 0;
  FCHK(read_int(B.off + c.n, &e, c.st));
  (vis ? c.nvp : c.npg) = e;
  hipLaunchKernelGGL(emit_entries_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.s, c.P, c.n, reg, vis, B.off, B.tgoff,
                     B.keys);
  tb = B.temp_bytes;
  if (e > 0) FCHK(hipcub::DeviceRadixSort::SortKeys(B.temp, tb, B.keys, B.keys2, e, 0, 64, c.st));
  FCHK(hipMemsetAsync(B.cellcnt, 0, (c.ncells + 1) * sizeof(int), c.st));
  if (e > 0) {
    hipLaunchKernelGGL(cell_hist_kernel, dim3(nblk(e)), dim3(256), 0, c.st, B.keys2, e, B.cellcnt);
    hipLaunchKernelGGL(items_kernel, dim3(nblk(e)), dim3(256), 0, c.st, B.keys2, e, items);
  }
  tb = B.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cellcnt, csr_off, (int)(c.ncells + 1), c.st));
  return hipGetLastError();
}

// CPatchOrganizerS::collectPatches: collect ranks and order
static hipError_t collect(Ctx& c) {
  FilterBuffers& B = c.B;
  FCHK(hipMemsetAsync(B.counters, 0, 8 * sizeof(int), c.st));
  hipLaunchKernelGGL(first_cell_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.s, c.P, c.n, B.preg, B.tgoff, B.keys,
                     B.counters);
  size_t tb = B.temp_bytes;
  FCHK(hipcub::DeviceRadixSort::SortKeys(B.temp, tb, B.keys, B.keys2, c.n, 0, 64, c.st));
  FCHK(read_int(B.counters, &c.nalive, c.st));
  FCHK(hipMemsetAsync(B.rank, 0xff, c.n * sizeof(int), c.st));
  if (c.nalive > 0)
    hipLaunchKernelGGL(rank_kernel, dim3(nblk(c.nalive)), dim3(256), 0, c.st, B.keys2, c.nalive, B.order, B.rank);
  hipLaunchKernelGGL(unit0_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.s, c.P, c.n, B.unit0);
  return hipGetLastError();
}

// CFilter::setDepthMapsVGridsVPGridsAddPatchV(additive) (filter.cpp:727-770)
static hipError_t set_dm_vgrids(Ctx& c, int additive) {
  FilterBuffers& B = c.B;
  FCHK(build_lists(c, 0));
  dbg(c.st, "  lists");
  FCHK(collect(c));
  dbg(c.st, "  collect");
  FCHK(hipMemsetAsync(B.dpkey, 0xff, c.ncells * sizeof(unsigned long long), c.st));
  if (c.nalive > 0)
    hipLaunchKernelGGL(depth_map_kernel, dim3(nblk((long long)c.nalive * c.s.tnum)), dim3(256), 0, c.st, c.s, c.dev(),
                       B.dpkey);
  dbg(c.st, "  depth");
  FCHK(hipMemsetAsync(B.vreg, 0, c.n * sizeof(unsigned long long), c.st));
  if (c.nalive > 0)
    hipLaunchKernelGGL(vimages_kernel, dim3(nblk(c.nalive)), dim3(256), 0, c.st, c.s, c.dev(), additive, B.vreg);
  dbg(c.st, "  vimages");
  FCHK(build_lists(c, 1));
  dbg(c.st, "  vlists");
  return hipGetLastError();
}

static hipError_t apply_flags(Ctx& c, int* removed) {
  FilterBuffers& B = c.B;
  FCHK(hipMemsetAsync(B.counters + 1, 0, sizeof(int), c.st));
  hipLaunchKernelGGL(apply_remove_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.n, B.flags, B.preg, B.vreg,
                     B.counters + 1);
  return read_int(B.counters + 1, removed, c.st);
}

}  // namespace

hipError_t filter_pass(const DScene& s, FilterBuffers& B, pmvs_patch* dP, int n, long long ncells, const long long* h_tgoff,
                       int grid, hipStream_t st, int counts[4], int* overflow, int* keep_dev) {
  dbg(st, "start");
  FCHK(B.reserve(n, ncells, s.tnum, grid));
  dbg(st, "reserve");
  FCHK(hipMemcpyAsync(B.tgoff, h_tgoff, (s.tnum + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
  Ctx c{s, B, dP, n, ncells, grid, st};
  for (int k = 0; k < 4; ++k) counts[k] = 0;
  *overflow = 0;
  hipLaunchKernelGGL(init_reg_kernel, dim3(nblk(n)), dim3(256), 0, st, s, dP, n, B.preg, B.vreg);
  FCHK(set_dm_vgrids(c, 0));
  dbg(st, "set_dm_vgrids(0)");
  // ---- filterOutside
  FCHK(hipMemsetAsync(B.flags, 0, n * sizeof(int), st));
  if (c.nalive) hipLaunchKernelGGL(gain_kernel, dim3(nblk(c.nalive)), dim3(256), 0, st, s, c.dev(), B.flags);
  FCHK(apply_flags(c, &counts[0]));
  dbg(st, "outside");
  FCHK(set_dm_vgrids(c, 1));
  // ---- filterExact
  FCHK(hipMemsetAsync(B.safe, 0, n * sizeof(unsigned long long), st));
  FCHK(hipMemsetAsync(B.counters + 2, 0, sizeof(int), st));
  hipLaunchKernelGGL(exact_entries_kernel, dim3(nblk(ncells)), dim3(256), 0, st, s, c.dev(), ncells, B.safe);
  FCHK(hipMemsetAsync(B.need, 0, n * sizeof(int), st));
  if (c.nalive)
    hipLaunchKernelGGL(exact_patch_kernel, dim3(nblk(c.nalive)), dim3(256), 0, st, s, c.dev(), B.safe, B.preg, B.vreg,
                       B.need, B.counters + 2);
  {
    std::vector<int> need(n);
    FCHK(hipMemcpyAsync(need.data(), B.need, n * sizeof(int), hipMemcpyDeviceToHost, st));
    FCHK(hipStreamSynchronize(st));
    std::vector<int> lst;
    for (int p = 0; p < n; ++p)
      if (need[p]) lst.push_back(p);
    const int m = (int)lst.size();
    if (m) {
      FCHK(hipMemcpyAsync(B.list, lst.data(), m * sizeof(int), hipMemcpyHostToDevice, st));
      FCHK(launch_filter_refimage(s, dP, B.list, m, grid, st));
      hipLaunchKernelGGL(exact_after_ref_kernel, dim3(nblk(m)), dim3(256), 0, st, s, dP, B.list, m, B.preg, B.vreg,
                         B.counters + 2);
    }
    FCHK(read_int(B.counters + 2, &counts[1], st));
  }
  dbg(st, "exact");
  FCHK(set_dm_vgrids(c, 1));
  dbg(st, "set_dm_vgrids(1) after exact");
  // ---- filterNeighbor(1)
  FCHK(hipMemsetAsync(B.flags, 0, n * sizeof(int), st));
  FCHK(hipMemsetAsync(B.counters + 3, 0, 5 * sizeof(int), st));
  if (c.nalive)
    hipLaunchKernelGGL(neighbor_kernel, dim3(std::min(grid, c.nalive)), dim3(64), 0, st, s, c.dev(), B.scratch, B.flags,
                       B.counters + 3, B.counters + 4, getenv("PMVS_FILTER_DEBUG") ? B.need : nullptr);
  dbg(st, "neighbor kernel");
  if (getenv("PMVS_FILTER_DEBUG")) {
    std::vector<int> cnts(n), ord(c.nalive);
    (void)hipMemcpy(cnts.data(), B.need, n * sizeof(int), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ord.data(), B.order, c.nalive * sizeof(int), hipMemcpyDeviceToHost);
    int mx = 0, ov = 0;
    for (int k = 0; k < c.nalive; ++k) {
      const int v = cnts[ord[k]];
      if (v < 0) ++ov;
      mx = std::max(mx, v < 0 ? -v : v);
    }
    fprintf(stderr, "[filter] neighbours: max unique %d, overflowed %d of %d; first: %d %d %d\n", mx, ov, c.nalive,
            cnts[ord[0]], c.nalive > 1 ? cnts[ord[1]] : 0, c.nalive > 2 ? cnts[ord[2]] : 0);
  }
  FCHK(read_int(B.counters + 3, overflow, st));
  {
    int errs[2] = {0, 0};
    FCHK(hipMemcpy(errs, B.counters + 6, 2 * sizeof(int), hipMemcpyDeviceToHost));
    if (errs[0]) {
      fprintf(stderr, "[filter] neighbor kernel bounds violations: %d (first code %d)\n", errs[0], errs[1]);
      return hipErrorIllegalAddress;
    }
  }
  FCHK(apply_flags(c, &counts[2]));
  FCHK(set_dm_vgrids(c, 1));
  // ---- filterSmallGroups
  if (c.nalive) {
    const int na = c.nalive;
    hipLaunchKernelGGL(group_edges_kernel, dim3(nblk(na)), dim3(256), 0, st, s, c.dev(), 0, B.edge_off, B.cnt, B.edges);
    FCHK(hipMemsetAsync(B.cnt + na, 0, sizeof(int), st));
    size_t tb = B.temp_bytes;
    FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cnt, B.edge_off, na + 1, st));
    int ne = 0;
    FCHK(read_int(B.edge_off + na, &ne, st));
    if ((size_t)ne > B.edges_cap) {
      if (B.edges) (void)hipFree(B.edges);
      B.edges = nullptr;
      B.edges_cap = (size_t)ne * 2;
      FCHK(hipMalloc((void**)&B.edges, B.edges_cap * sizeof(int)));
    }
    hipLaunchKernelGGL(group_edges_kernel, dim3(nblk(na)), dim3(256), 0, st, s, c.dev(), 1, B.edge_off, B.cnt, B.edges);
    std::vector<int> eoff(na + 1), edges(ne ? ne : 1), order(na), fixv(n);
    FCHK(hipMemcpyAsync(eoff.data(), B.edge_off, (na + 1) * sizeof(int), hipMemcpyDeviceToHost, st));
    if (ne) FCHK(hipMemcpyAsync(edges.data(), B.edges, ne * sizeof(int), hipMemcpyDeviceToHost, st));
    FCHK(hipMemcpyAsync(order.data(), B.order, na * sizeof(int), hipMemcpyDeviceToHost, st));
    FCHK(hipStreamSynchronize(st));
    // filterSmallGroups label BFS (filter.cpp:520-562) in collect order
    std::vector<int> label(na, -1);
    int id = -1;
    std::deque<int> q;
    for (int pid = 0; pid < na; ++pid) {
      if (label[pid] != -1) continue;
      label[pid] = ++id;
      q.push_back(pid);
      while (!q.empty()) {
        const int pt = q.front();
        q.pop_front();
        for (int e = eoff[pt]; e < eoff[pt + 1]; ++e) {
          const int j = edges[e];
          if (label[j] != -1) continue;
          label[j] = id;
          q.push_back(j);
        }
      }
    }
    std::vector<int> size(id + 1, 0);
    for (int l : label) ++size[l];
    const int threshold = std::max(20, na / 10000);
    std::vector<int> flags(n, 0);
    for (int k = 0; k < na; ++k)
      if (size[label[k]] < threshold) flags[order[k]] = 1;
    FCHK(hipMemcpyAsync(B.flags, flags.data(), n * sizeof(int), hipMemcpyHostToDevice, st));
    // fixed patches are never removed (filter.cpp:590)
    hipLaunchKernelGGL(clear_fixed_kernel, dim3(nblk(n)), dim3(256), 0, st, dP, n, B.flags);
    FCHK(apply_flags(c, &counts[3]));
  }
  dbg(st, "groups");
  FCHK(set_dm_vgrids(c, 1));
  FCHK(build_lists(c, 0));
  FCHK(collect(c));
  hipLaunchKernelGGL(keep_kernel, dim3(nblk(n)), dim3(256), 0, st, n, B.preg, B.rank, keep_dev);
  return hipGetLastError();
}

}  // namespace pmvsdev
