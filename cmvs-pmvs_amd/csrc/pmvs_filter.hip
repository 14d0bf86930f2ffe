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
// sort/unique in LDS, Cmylapack::lls with Eigen's JacobiSVD algorithm in double), and the setRefImage of filterExact
// reuses the refine path's wavefront kernel (pmvs_kernels.hip).  The connected-component labels of
// filterSmallGroups are a breadth-first search over the device-computed, ordered edge lists on the
// host (the reference's label assignment is an order-dependent BFS; its cost is O(edges)).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <new>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <deque>
#include <functional>
#include <mutex>
#include <unordered_map>
#include <queue>
#include <vector>

#include "pmvs_device.h"
#include "pmvs_launch.h"
#include "pmvs_layout.h"
#include "pmvs_queue.h"

namespace pmvsdev {

// Debug builds of the tests: PMVS_POISON_ALLOC=<byte> fills every new device allocation with that
// byte, so a read of memory no kernel wrote shows up as a result change (tests/test_gpu_poison.py).
inline void poison_alloc(void* p, size_t bytes) {
  static const int v = [] {
    const char* e = getenv("PMVS_POISON_ALLOC");
    return e ? atoi(e) : -1;
  }();
  if (v >= 0 && p && bytes) {
    (void)hipMemset(p, v & 0xff, bytes);
    (void)hipDeviceSynchronize();
  }
}

// Neighbours per patch the walks hold in LDS.  The NB_CAP form runs every walk; the few patches
// with more unique neighbours are walked again by the NB_CAP_BIG form (NbLdsT<16384>, about 130 KB
// of LDS, one workgroup per CU); only beyond NB_CAP_BIG is the run an error.
// PMVS_NB_CAP / PMVS_NB_GRID_MULT / PMVS_NB_WAVES_PER_EU: experiment variants only (tools/sweep_walks.sh,
// `make variant VARTU=pmvs_filter`); the product builds the defaults.
#ifndef PMVS_NB_CAP
#define PMVS_NB_CAP 1024
#endif
constexpr int NB_CAP = PMVS_NB_CAP;
constexpr int NB_CAP_BIG = PMVS_MAX_NEIGHBOURS;
// Global scratch per persistent workgroup of the neighbour walks (doubles): the lls rows M
// (5 CAP), its right-hand side r (CAP), then the filterQuad coordinates fx, fy, fz as floats
// (1.5 CAP).  Kept out of LDS so NbLds stays ~8 KB (occupancy of the latency-bound walks).
constexpr int NB_SCR = NB_CAP * 8;
constexpr int NB_GRID_BIG = 32;  // workgroups of the NB_CAP_BIG re-walks
// gather_neighbors: cell slots per lane per round, entries per lane per test round
#ifndef PMVS_NB_SK  // experiment variants only (tools/sweep_walks.sh)
#define PMVS_NB_SK 2
#endif
#ifndef PMVS_NB_NE
#define PMVS_NB_NE 2
#endif
constexpr int NB_SK = PMVS_NB_SK;
constexpr int NB_NE = PMVS_NB_NE;
// gather_neighbors' slots (round 6): 1 = one slot per ROW of a list's (2 margin + 1)^2 window -- the
// row's cells are consecutive in the CSR cell order, so their entries are the one range
// [off[c0], off[c0 + nx]) -- against 0 = one slot per cell (rounds 2-5).  The neighbour set is the
// same; a filterNeighbor walk loads 10 list bounds per image instead of 50.
#ifndef PMVS_NB_ROWS
#define PMVS_NB_ROWS 1
#endif
// Diagnostic build only (-DNB_PROFILE, tools/r06w.sh): shader cycles per phase of the neighbour walks,
// summed over wavefronts, per kernel (0 neighbor_kernel, 1 empty_blocks_kernel, 2 depth_post_kernel):
// [0] setup (radius, units, seen-set clear), [1] slot bounds, [2] entries (items, tests, appends),
// [3] delta chains, [4] final sort + unique, [5] the kernel's work after the walk, [6] queue / other.
// Printed to stderr after every filter pass and expansion (pmvs_filter.hip, nb_prof_dump).
#if defined(NB_PROFILE)
__device__ unsigned long long g_nb_prof[3][8];
#define NBP_NOW() __builtin_amdgcn_s_memtime()
#define NBP(ph)                                   \
  do {                                            \
    if (prof) {                                   \
      const unsigned long long _t = NBP_NOW();    \
      prof[ph] += _t - nbp_t;                     \
      nbp_t = _t;                                 \
    }                                             \
  } while (0)
#define NBP_FLUSH(kid)                                                    \
  do {                                                                    \
    if (threadIdx.x == 0)                                                 \
      for (int _i = 0; _i < 8; ++_i) atomicAdd(&g_nb_prof[kid][_i], prof[_i]); \
  } while (0)
#else
#define NBP_NOW() 0ull
#define NBP(ph) \
  do {          \
  } while (0)
#define NBP_FLUSH(kid) \
  do {                 \
  } while (0)
#endif
// Persistent workgroups per CU-grid unit for the NbLds kernels (neighbor_kernel, depth_post_kernel,
// empty_blocks_kernel): twice the organizer grid, since ~8 KB of LDS and <= 107 VGPRs leave room.
#ifndef PMVS_NB_GRID_MULT
#define PMVS_NB_GRID_MULT 2
#endif
constexpr int NB_GRID_MULT = PMVS_NB_GRID_MULT;
#ifdef PMVS_NB_WAVES_PER_EU
#define NB_WALK_ATTR __attribute__((amdgpu_waves_per_eu(PMVS_NB_WAVES_PER_EU)))
#else
#define NB_WALK_ATTR
#endif
__device__ __forceinline__ int lane_id_w() { return threadIdx.x & 63; }
// Wave-uniform copies (SGPR) of values that are uniform by construction but loaded from memory:
// every branch or loop around a barrier is driven by one of these, never by a VGPR value.
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float uni_f(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

__host__ __device__ inline Reg reg_zero() {
  Reg r;
  for (int k = 0; k < REGW; ++k) r.w[k] = 0ull;
  return r;
}
__host__ __device__ inline Reg reg_first(int n) {  // entries 0 .. n-1
  Reg r;
  for (int k = 0; k < REGW; ++k)
    r.w[k] = (n >= 64 * (k + 1)) ? ~0ull : (n > 64 * k ? ((1ull << (n - 64 * k)) - 1ull) : 0ull);
  return r;
}
__host__ __device__ inline void reg_set(Reg& r, int i) { r.w[i >> 6] |= 1ull << (i & 63); }
__host__ __device__ inline bool reg_test(const Reg& r, int i) { return (r.w[i >> 6] >> (i & 63)) & 1ull; }
__device__ inline int reg_popc(const Reg& r) {
  int c = 0;
  for (int k = 0; k < REGW; ++k) c += __popcll(r.w[k]);
  return c;
}
__host__ __device__ inline Reg reg_and(const Reg& a, const Reg& b) {
  Reg r;
  for (int k = 0; k < REGW; ++k) r.w[k] = a.w[k] & b.w[k];
  return r;
}
// visits the set entries in increasing order: for (int i = reg_next(m, -1); i >= 0; i = reg_next(m, i))
__device__ inline int reg_next(const Reg& r, int i) {
  for (int k = (i + 1) >> 6; k < REGW; ++k) {
    const int b = (k == ((i + 1) >> 6)) ? ((i + 1) & 63) : 0;
    const unsigned long long m = (b >= 64) ? 0ull : (r.w[k] & (~0ull << b));
    if (m) return 64 * k + __builtin_ctzll(m);
  }
  return -1;
}

struct FilterDev {
  const DScene* dummy;
  pmvs_patch* P;
  int n;
  Reg* preg;
  Reg* vreg;
  const long long* tgoff;  // [tnum + 1] global cell offsets of the target images
  int tnum;
  // CSR organizer
  const int* pg_off; const int* pg_items;
  const int* vp_off; const int* vp_items;
  const unsigned long long* dpkey;
  const int* order;  // collect order -> patch
  const int* rank;   // patch -> collect rank or -1
  int nalive;
  const PHot* hot;     // per patch: coord, normal, dscale, ncc, getUnit(images[0], coord)
  long long ncells;
  int npg, nvp;        // entries in the pgrids / vpgrids lists
  int* err;            // [0] count, [1] first code (defensive bounds checks)
  int* lovf;           // patches whose image / vimage list would exceed PMVS_MAX_IMAGES (an error, never a clamp)
  int nb_softcap;      // tests (PMVS_NB_SOFTCAP): neighbour capacity of the NB_CAP walks, to exercise the re-walks
  // Expansion only: registrations committed since the CSR lists were built, as per-cell chains
  // (head per cell, -1 = empty; item/next in a shared entry pool).  Every expansion reader is
  // insensitive to the order inside a cell list (findNeighbors sorts and uniques, computeGain
  // takes a max per cell, checkCounts tests occupancy), so chains need no insertion order.
  // nullptr in the filter pass.
  const int* pg_dhead; const int* vp_dhead;
  const int2* d_ent;  // {item, next} per pool entry
  // Filter pass only: the collected patches' coordinates in collect order (the dpkey payload),
  // so depth tests read 16 B instead of a patch record; nullptr in the expansion.
  const float4* coordc;
};


// filterNeighbor's deferred quadric fits (neighbor_kernel -> quad_lane_kernel): per job the rows'
// fx, fy, fz (3n floats at 3 * offset) and the solver's n x 5 system plus Q^T b (6n doubles at
// 6 * offset); offsets from a row counter, jobs {patch, offset, n}.  f == nullptr: no deferral.
struct QuadJobs {
  float* f;
  double* rows;
  int4* jobs;
  unsigned long long* rows_used;
  int* njobs;
  unsigned long long cap_rows;
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
template <class PL, class PR>
__device__ __forceinline__ int is_neighbor_h(const PL& l, const PR& r, float hunit, float thr, float radius, bool use_radius) {
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
  const PHot &ha = F.hot[a], &hb = F.hot[b];
  const float hunit = (float)((double)(ha.unit0 + hb.unit0) / 2.0 * s.csize);
  return is_neighbor_h(ha, hb, hunit, thr, 0.0f, false);
}

// CPatchOrganizerS::isVisible (patchOrganizerS.cpp:500-525).
template <class PQ>
__device__ __forceinline__ int is_visible_q(const DScene& s, const FilterDev& F, const PQ& q, int t, int ix, int iy, float strict) {
  if (!in_grid(s, t, ix, iy)) return 0;
  if (s.depth == 0) return 1;
  const unsigned long long key = F.dpkey[F.tgoff[t] + (long long)iy * gwidth(s, t) + ix];
  if (key == ~0ull) return 1;
  const int rk = (int)(key & 0xffffffffull);
  float pc[4];
  if (F.coordc) {
    const float4 c4 = F.coordc[rk];
    pc[0] = c4.x; pc[1] = c4.y; pc[2] = c4.z; pc[3] = c4.w;
  } else {
    const float* c = F.P[F.order[rk]].coord;
    for (int k = 0; k < 4; ++k) pc[k] = c[k];
  }
  const DView& v = s.views[t];
  float ray[4] = {q.coord[0] - v.center[0], q.coord[1] - v.center[1], q.coord[2] - v.center[2], q.coord[3] - v.center[3]};
  unitize4(ray);
  float dd[4];
  for (int k = 0; k < 4; ++k) dd[k] = q.coord[k] - pc[k];
  const float diff = dot4(ray, dd);
  const double fd = 2.0 + (double)dot4(ray, q.normal);
  const float factor = (float)((fd < 2.0) ? fd : 2.0);  // std::min(2.0, .)
  return diff < get_unit(s, v, q.coord) * (float)s.csize * strict * factor ? 1 : 0;
}
__device__ int is_visible(const DScene& s, const FilterDev& F, int p, int t, int ix, int iy, float strict) {
  return is_visible_q(s, F, F.P[p], t, ix, iy, strict);  // the caller reads this record anyway
}

// --------------------------------------------------------------------------- organizer build
// CPatchOrganizerS::addPatch (patchOrganizerS.cpp:308-324): register every target entry of the
// input patches (out-of-grid cells, undefined in the reference, are not registered).
// The list kernels below read a patch's image / cell lists with kLG lanes per patch (entry i on
// lane i mod kLG): one load instruction covers kLG consecutive entries of one record, so each list
// line is fetched once.  Thread-per-patch forms re-fetched the lines for every entry (a CU's
// thousands of in-flight records do not stay in L1 / L2 between one thread's iterations): 10.9 GB
// of HBM reads per first_cell launch and 6.2 GB per emit_entries launch on C3
// (profiles/r05j_pmc.json) against ~1.5 GB of list lines.
constexpr int kLG = 8;
__device__ __forceinline__ int reg_rank(const Reg& r, int i) {  // set entries below i
  return (i < 64) ? __popcll(r.w[0] & ((1ull << i) - 1ull)) : __popcll(r.w[0]) + __popcll(r.w[1] & ((1ull << (i - 64)) - 1ull));
}
__device__ __forceinline__ int reg_last(const Reg& r) {  // highest set entry, -1 if none
  return r.w[1] ? 127 - __clzll(r.w[1]) : (r.w[0] ? 63 - __clzll(r.w[0]) : -1);
}
__global__ void init_reg_kernel(DScene s, const pmvs_patch* __restrict__ P, int n, Reg* __restrict__ preg,
                                Reg* __restrict__ vreg) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int p = (int)(g / kLG), l = (int)(g % kLG);
  if (p >= n) return;  // whole lane groups
  const pmvs_patch& q = P[p];
  const int ni = q.num_images;
  unsigned long long w0 = 0ull, w1 = 0ull;
  for (int i = l; i < ni; i += kLG)
    if (q.images[i] < s.tnum && in_grid(s, q.images[i], q.grids[i][0], q.grids[i][1])) {
      if (i < 64) w0 |= 1ull << i;
      else w1 |= 1ull << (i - 64);
    }
  for (int d = 1; d < kLG; d <<= 1) {
    w0 |= __shfl_xor(w0, d);
    w1 |= __shfl_xor(w1, d);
  }
  if (l == 0) {
    Reg m;
    m.w[0] = w0;
    m.w[1] = w1;
    preg[p] = m;
    vreg[p] = reg_zero();
  }
}

__global__ void keep_kernel(int n, const Reg* __restrict__ preg, const int* __restrict__ rank,
                            int* __restrict__ keep) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  keep[p] = (rank[p] >= 0) ? 1 : 0;
}

__global__ void count_entries_kernel(const pmvs_patch* __restrict__ P, int n, const Reg* __restrict__ reg,
                                     int vis, int* __restrict__ cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  cnt[p] = reg_popc(reg[p]);
}

__global__ void emit_entries_kernel(DScene s, const pmvs_patch* __restrict__ P, int n,
                                    const Reg* __restrict__ reg, int vis, const int* __restrict__ off,
                                    const long long* __restrict__ tgoff, unsigned long long* __restrict__ keys) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int p = (int)(g / kLG), l = (int)(g % kLG);
  if (p >= n) return;
  const Reg m = reg[p];
  const int last = reg_last(m);
  if (last < 0) return;
  const int o = off[p];
  const pmvs_patch& q = P[p];
  for (int i = l; i <= last; i += kLG) {
    if (!reg_test(m, i)) continue;
    const int t = vis ? q.vimages[i] : q.images[i];
    const int ix = vis ? q.vgrids[i][0] : q.grids[i][0];
    const int iy = vis ? q.vgrids[i][1] : q.grids[i][1];
    const unsigned long long cell = (unsigned long long)(tgoff[t] + (long long)iy * gwidth(s, t) + ix);
    keys[o + reg_rank(m, i)] = (cell << 32) | (unsigned)p;
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
// Grid-stride over the patches (kLG lanes each), the collected count summed per wavefront and added
// with one atomic per wavefront of the grid: an atomic per wavefront of patches (525 k same-address
// atomics per C3 launch) made the lane-group form 4x slower than the thread-per-patch one.
__global__ void first_cell_kernel(DScene s, const pmvs_patch* __restrict__ P, int n,
                                  const Reg* __restrict__ preg, const long long* __restrict__ tgoff,
                                  unsigned long long* __restrict__ keys, int* __restrict__ nalive) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  int live = 0;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < (long long)n * kLG; g += stride) {
    const int p = (int)(g / kLG), l = (int)(g % kLG);  // stride is a multiple of kLG: groups stay whole
    const Reg m = preg[p];
    const int last = reg_last(m);
    unsigned long long best = ~0ull;
    const pmvs_patch& q = P[p];
    for (int i = l; i <= last; i += kLG) {
      if (!reg_test(m, i)) continue;
      const int t = q.images[i];
      const unsigned long long cell = (unsigned long long)(tgoff[t] + (long long)q.grids[i][1] * gwidth(s, t) + q.grids[i][0]);
      if (cell < best) best = cell;
    }
    for (int d = 1; d < kLG; d <<= 1) {
      const unsigned long long o = __shfl_xor(best, d);
      best = o < best ? o : best;
    }
    if (l == 0) {
      keys[p] = (best == ~0ull) ? ~0ull : ((best << 32) | (unsigned)p);
      live += (best != ~0ull);
    }
  }
  for (int d = 32; d >= 1; d >>= 1) live += __shfl_xor(live, d);
  if ((threadIdx.x & 63) == 0 && live) atomicAdd(nalive, live);
}

__global__ void rank_kernel(const unsigned long long* __restrict__ keys, int nalive, int* __restrict__ order,
                            int* __restrict__ rank) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nalive) return;
  const int p = (int)(keys[i] & 0xffffffffull);
  order[i] = p;
  rank[p] = i;
}

__device__ inline void write_hot(const DScene& s, const pmvs_patch& q, PHot& h) {
  PHot v;
  for (int k = 0; k < 4; ++k) { v.coord[k] = q.coord[k]; v.normal[k] = q.normal[k]; }
  v.dscale = q.dscale;
  v.ncc = q.ncc;
  v.unit0 = q.num_images > 0 ? get_unit(s, s.views[q.images[0]], q.coord) : 0.0f;
  for (int k = 0; k < 5; ++k) v.pad[k] = 0.0f;
  h = v;
}
__global__ void hot_kernel(DScene s, const pmvs_patch* __restrict__ P, int n, PHot* __restrict__ hot) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  write_hot(s, P[p], hot[p]);
}

// CFilter::setDepthMapsThread (filter.cpp:689-725): one thread per (collected patch, target).
// The collected patches' coordinates in collect order (the depth-map pass reads them once per
// target, coalesced, instead of re-reading 1.6 KB patch records).
__global__ void coordc_kernel(const pmvs_patch* __restrict__ P, const int* __restrict__ order, int na,
                              float4* __restrict__ coordc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na) return;
  const float* c = P[order[i]].coord;
  coordc[i] = make_float4(c[0], c[1], c[2], c[3]);
}

// XCD-aware block order: the hardware deals workgroups to the 8 XCDs round-robin (block b on XCD
// b % 8), each XCD with its own L2.  Remapping b to the logical block (b % 8) * (grid / 8) + b / 8
// (grid a multiple of 8: xcd_grid) gives each XCD one contiguous range of logical blocks, so
// threads that touch neighbouring cells share an L2.  Used by the vimages lists (round 3's
// patch-major vimages kernel: 8.6 -> 5.8 ms per launch); setDepthMaps keeps the hardware order, where this order measured
// slower (7.9 -> 10.6 ms: a contiguous range is ~6 whole target maps of atomics on one L2).
constexpr int kXcds = 8;
__device__ __forceinline__ long long xcd_block() {
  const unsigned b = blockIdx.x, per = gridDim.x / kXcds;
  return (long long)(b % kXcds) * per + b / kXcds;
}

// setDepthMaps: one thread per (target, collected patch), target-major so that neighbouring
// threads hold neighbouring patches (collect order is by image and cell) and their atomics hit
// nearby cells of the same map.
// Owner-partitioned filter pass (world > 1): only the targets rank owns (t = rank + world j) -- the
// other targets' maps are never read on this rank (its visibility tests are its own targets').
// tpt targets per thread (PMVS_DM_TARGETS, default 4): the patch's coordinate is read once for them.
__global__ void depth_map_kernel(DScene s, FilterDev F, const float4* __restrict__ coordc,
                                 unsigned long long* __restrict__ dpkey, int rank = 0, int world = 1, int tpt = 1) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // hardware order (r03k3: the XCD
  const int nown = (F.tnum - rank + world - 1) / world;                   // order made it 7.9 -> 10.6 ms)
  const int ngrp = (nown + tpt - 1) / tpt;
  if (g >= (long long)F.nalive * ngrp) return;
  const int jg = (int)(g / F.nalive), i = (int)(g - (long long)jg * F.nalive);
  const float4 c4 = coordc[i];
  const float coord[4] = {c4.x, c4.y, c4.z, c4.w};
  for (int u = 0; u < tpt; ++u) {
    const int j = jg * tpt + u;
    if (j >= nown) break;
    const int t = rank + world * j;
    const DView& v = s.views[t];
    float ic[3];
    project(v, coord, s.level, ic);
    const float fx = __fdiv_rn(ic[0], (float)s.csize), fy = __fdiv_rn(ic[1], (float)s.csize);
    const int xs[2] = {(int)floor((double)fx), (int)ceil((double)fx)};
    const int ys[2] = {(int)floor((double)fy), (int)ceil((double)fy)};
    const unsigned long long key = ((unsigned long long)depth_bits(depth_of(v, coord)) << 32) | (unsigned)i;
    const int gw = gwidth(s, t), gh = gheight(s, t);
    for (int y = 0; y < 2; ++y)
      for (int x = 0; x < 2; ++x) {
        if (xs[x] < 0 || gw <= xs[x] || ys[y] < 0 || gh <= ys[y]) continue;
        unsigned long long* cell = &dpkey[F.tgoff[t] + (long long)ys[y] * gw + xs[x]];
        // the stored minimum only decreases, so a (possibly stale) value <= key means the atomic
        // could not change the cell: skip it (most updates of a dense model)
        if (key < *cell) atomicMin(cell, key);
      }
  }
}

// setVImagesVGrids (patchOrganizerS.cpp:429-459) in two steps, target-major:
//   vis_rows_kernel   one thread per (target, collected patch), consecutive patches of one target per
//                     wavefront: isVisible0 + the edge test (the tests vimages_kernel makes) and a ballot,
//                     so row t holds one bit per collected patch -- while the grid works through target
//                     t, t's depth map and edge map stay in L2 (vimages_kernel walks all targets per
//                     patch, every wavefront in another map);
//   vis_lists_kernel  one thread per patch: the visible targets appended in target order, their cells.
// Owner-partitioned (world > 1): a rank computes the rows of the targets it owns
// (t = rank + world j), the rows are all-gathered, and every rank builds the same lists.
__global__ void normalc_kernel(const pmvs_patch* __restrict__ P, const int* __restrict__ order, int na,
                               float4* __restrict__ normalc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na) return;
  const float* c = P[order[i]].normal;
  normalc[i] = make_float4(c[0], c[1], c[2], c[3]);
}

// per collected patch: the targets already in its lists (images; vimages too when additive), kLG
// lanes per patch (the lists read as the list kernels read them), OR-reduced over the lane group
__global__ void used_kernel(DScene s, FilterDev F, int additive, unsigned long long* __restrict__ used) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(g / kLG), l = (int)(g % kLG);
  if (i >= F.nalive) return;  // whole lane groups
  const pmvs_patch& q = F.P[F.order[i]];
  unsigned long long u0 = 0ull, u1 = 0ull, u2 = 0ull, u3 = 0ull;  // registers (a dynamically indexed array went to scratch)
  auto add = [&](int t) {
    const unsigned long long b = 1ull << (t & 63);
    const int w = t >> 6;
    u0 |= (w == 0) ? b : 0ull;
    u1 |= (w == 1) ? b : 0ull;
    u2 |= (w == 2) ? b : 0ull;
    u3 |= (w == 3) ? b : 0ull;
  };
  static_assert(PMVS_MAX_TARGETS == 256, "four used words per patch");
  const int ni = q.num_images;
  for (int k = l; k < ni; k += kLG)
    if (q.images[k] < s.tnum) add(q.images[k]);
  if (additive) {
    const int nv = q.num_vimages;
    for (int k = l; k < nv; k += kLG) add(q.vimages[k]);
  }
  for (int d = 1; d < kLG; d <<= 1) {
    u0 |= __shfl_xor(u0, d);
    u1 |= __shfl_xor(u1, d);
    u2 |= __shfl_xor(u2, d);
    u3 |= __shfl_xor(u3, d);
  }
  // word-major (word w of every patch together): vis_rows_kernel's wavefronts read one word of 64
  // consecutive patches, contiguously
  if (l == 0) {
    const size_t na = (size_t)F.nalive;
    used[i] = u0;
    used[na + i] = u1;
    used[2 * na + i] = u2;
    used[3 * na + i] = u3;
  }
}

struct PCN {  // the fields isVisible reads of the tested patch
  float coord[4], normal[4];
};

// kVisT targets per thread: the patch's coordinate and normal are read once for them (round 4 read
// them once per target, 32 B x targets x patches per launch).
constexpr int kVisT = 4;
__global__ __launch_bounds__(256) void vis_rows_kernel(DScene s, FilterDev F, const float4* __restrict__ coordc,
                                                       const float4* __restrict__ normalc,
                                                       const unsigned long long* __restrict__ used, int rank, int world,
                                                       int nown, long long row_words, unsigned long long* __restrict__ rows) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long napad = row_words * 64;
  const int ngrp = (nown + kVisT - 1) / kVisT;
  if (g >= (long long)ngrp * napad) return;  // whole wavefronts: napad is a multiple of 64
  const int jg = (int)(g / napad), i = (int)(g - (long long)jg * napad);
  const bool live = i < F.nalive;
  PCN q{};
  if (live) {
    const float4 c4 = coordc[i], n4 = normalc[i];
    q = PCN{{c4.x, c4.y, c4.z, c4.w}, {n4.x, n4.y, n4.z, n4.w}};
  }
  for (int u = 0; u < kVisT; ++u) {
    const int j = jg * kVisT + u;
    if (j >= nown) break;  // wave-uniform
    const int t = rank + world * j;
    bool vis = false;
    if (live && !((used[(size_t)(t >> 6) * F.nalive + i] >> (t & 63)) & 1ull)) {
      const DView& v = s.views[t];
      float ic[3];
      project(v, q.coord, s.level, ic);
      const int ix = ((int)floorf(ic[0] + 0.5f)) / s.csize;
      const int iy = ((int)floorf(ic[1] + 0.5f)) / s.csize;
      vis = is_visible_q(s, F, q, t, ix, iy, 0.5f) != 0 && get_edge(s, v, q.coord, s.level) != 0;
    }
    const unsigned long long b = __ballot(vis);
    if ((threadIdx.x & 63) == 0) rows[(long long)j * row_words + i / 64] = b;
  }
}

// rows: world blocks (rank r: nown_max rows of row_words words; row j = target r + world j)
__global__ void vis_lists_kernel(DScene s, FilterDev F, int additive, int world, int nown_max, long long row_words,
                                 const unsigned long long* __restrict__ rows, Reg* __restrict__ vreg) {
  const int i = (int)(xcd_block() * blockDim.x + threadIdx.x);
  if (i >= F.nalive) return;
  const int p = F.order[i];
  pmvs_patch& q = F.P[p];
  if (!additive) q.num_vimages = 0;
  const long long blk = (long long)nown_max * row_words;
  for (int t = 0; t < s.tnum; ++t) {
    const unsigned long long w = rows[(long long)(t % world) * blk + (long long)(t / world) * row_words + i / 64];
    if (!((w >> (i & 63)) & 1ull)) continue;
    float ic[3];
    project(s.views[t], q.coord, s.level, ic);
    if (q.num_vimages >= PMVS_MAX_IMAGES) {  // more than PMVS_MAX_IMAGES targets see the patch: the pass fails
      atomicAdd(F.lovf, 1);
      break;
    }
    q.vimages[q.num_vimages] = (int16_t)t;
    q.vgrids[q.num_vimages][0] = grid16(((int)floorf(ic[0] + 0.5f)) / s.csize);
    q.vgrids[q.num_vimages][1] = grid16(((int)floorf(ic[1] + 0.5f)) / s.csize);
    q.num_vimages++;
  }
  vreg[p] = reg_first(q.num_vimages);
}

__global__ void or_bits_kernel(const unsigned* __restrict__ all, int world, size_t words, unsigned* __restrict__ out) {
  const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  unsigned v = 0u;
  for (int r = 0; r < world; ++r) v |= all[(size_t)r * words + w];
  out[w] = v;
}

// --------------------------------------------------------------------------- filterOutside
// CFilter::filterOutsideThread (filter.cpp:148-201), neighbourThreshold1 = 1.0.  Owner-partitioned
// (world > 1): the patches whose reference image this rank owns; the flags are all-gathered.
// kLG lanes per patch (as the list kernels): entry e of the patch's images-then-vimages sequence on
// lane e mod kLG computes its cell's max; the gain is then reduced in the reference's entry order by
// every lane of the group (the maxima come by shuffles), so the float result is the sequential one.
__global__ void gain_kernel(DScene s, FilterDev F, int* __restrict__ remove, int rank = 0, int world = 1) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(g / kLG), l = (int)(g % kLG);
  if (i >= F.nalive) return;  // whole lane groups
  const int p = F.order[i];
  const pmvs_patch& q = F.P[p];
  if (q.fix || q.images[0] % world != rank) {
    if (l == 0) remove[p] = 0;
    return;
  }
  float gain = smax(0.0f, q.ncc - s.nccThreshold) * (float)q.timages;
  const int ni = q.num_images, ne = ni + q.num_vimages;
  const int base = (int)(threadIdx.x & 63) & ~(kLG - 1);  // the group's first lane in the wavefront
  for (int c = 0; c < ne; c += kLG) {
    const int k = c + l;
    float maxp = 0.0f;
    if (k < ni) {
      const int t = q.images[k];
      if (t < s.tnum) {
        const long long cell = F.tgoff[t] + (long long)q.grids[k][1] * gwidth(s, t) + q.grids[k][0];
        for (int e = F.pg_off[cell]; e < F.pg_off[cell + 1]; ++e) {
          const int j = F.pg_items[e];
          if (!is_neighbor(s, F, p, j, 1.0f)) maxp = smax(maxp, F.hot[j].ncc - s.nccThreshold);
        }
      }
    } else if (k < ne) {
      const int t = q.vimages[k - ni];
      if (t < s.tnum) {
        const float pdepth = depth_of(s.views[t], q.coord);
        const long long cell = F.tgoff[t] + (long long)q.vgrids[k - ni][1] * gwidth(s, t) + q.vgrids[k - ni][0];
        for (int e = F.pg_off[cell]; e < F.pg_off[cell + 1]; ++e) {
          const int j = F.pg_items[e];
          const float bdepth = depth_of(s.views[t], F.hot[j].coord);
          if (pdepth < bdepth && !is_neighbor(s, F, p, j, 1.0f)) maxp = smax(maxp, F.hot[j].ncc - s.nccThreshold);
        }
      }
    }
    for (int u = 0; u < kLG && c + u < ne; ++u) gain -= __shfl(maxp, base + u);  // gain -= maxp, entry order
  }
  if (l == 0) remove[p] = (gain < 0.0) ? 1 : 0;
}

__global__ void clear_fixed_kernel(const pmvs_patch* __restrict__ P, int n, int* __restrict__ flags) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (P[p].fix) flags[p] = 0;
}

__global__ void apply_remove_kernel(int n, const int* __restrict__ remove, Reg* __restrict__ preg,
                                    Reg* __restrict__ vreg, int* __restrict__ count) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (remove[p]) {
    preg[p] = reg_zero();
    vreg[p] = reg_zero();
    atomicAdd(count, 1);
  }
}

// --------------------------------------------------------------------------- filterExact
// filterExactThread (filter.cpp:291-340): one thread per registered pgrids entry; marks the
// patch's images[] positions that are safe (visible at the cell or one of its 4 neighbours).
// Owner-partitioned (world > 1): the cells of the targets this rank owns; the safe bits are OR-merged
// over the ranks afterwards.
__global__ void exact_entries_kernel(DScene s, FilterDev F, long long ncells, Reg* __restrict__ safe, int rank = 0,
                                     int world = 1) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncells) return;
  const int b = F.pg_off[c], e = F.pg_off[c + 1];
  if (b == e) return;
  int t = 0;
  while (F.tgoff[t + 1] <= c) ++t;
  if (t % world != rank) return;
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
          atomicOr(&safe[p].w[i >> 6], 1ull << (i & 63));
          break;
        }
  }
}

// filterExact (filter.cpp:234-348) per collected, non-fixed patch: new list = safe targets in
// increasing image order (the reference's image-major scan) with their cells, then the
// non-target images; _timages = #safe.  need_ref[p] = 1 when setRefImage + setGrids follow.
// One wavefront per patch (4 per 256-lane block): lane l holds list entries l and l + 64.  A kept
// target entry goes to the number of kept target entries before it in (image, list position)
// order -- the reference loops over the targets and looks each up in the list, filter.cpp:305-330
// -- and a non-target entry to the kept count plus the non-target entries before it in list order.
// Every lane's entries are in registers before any lane writes, so the list is rewritten in place.
// (Round 4's thread-per-patch form staged the new list in 1.5 KB of per-thread arrays, which lived
// in scratch: 87 GB of HBM traffic per C3 launch, profiles/r05j_pmc.json.)
__global__ __launch_bounds__(256) void exact_patch_kernel(DScene s, FilterDev F, const Reg* __restrict__ safe,
                                                          Reg* __restrict__ preg, Reg* __restrict__ vreg,
                                                          int* __restrict__ need_ref, int* __restrict__ removed) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= F.nalive) return;  // wave-uniform; no barriers below
  const int p = F.order[i];
  pmvs_patch& q = F.P[p];
  if (q.fix) {
    if (lane == 0) need_ref[p] = 0;
    return;
  }
  const Reg sm = reg_and(safe[p], preg[p]);
  const int n0 = q.num_images;
  int t[2], g0[2], g1[2];
  bool kept[2], other[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int k = lane + 64 * u;
    t[u] = 0; g0[u] = 0; g1[u] = 0; kept[u] = false; other[u] = false;
    if (k < n0) {
      t[u] = q.images[k];
      g0[u] = q.grids[k][0];
      g1[u] = q.grids[k][1];
      kept[u] = t[u] < s.tnum && reg_test(sm, k);
      other[u] = s.tnum <= t[u];
    }
  }
  int pos[2] = {0, 0};
  for (int k2 = 0; k2 < n0; ++k2) {  // n0 is wave-uniform: every lane reads entry k2 by a shuffle
    const int t2 = __shfl(k2 < 64 ? t[0] : t[1], k2 & 63);
    const int kp2 = __shfl(k2 < 64 ? (int)kept[0] : (int)kept[1], k2 & 63);
#pragma unroll
    for (int u = 0; u < 2; ++u)
      pos[u] += (kp2 && (t2 < t[u] || (t2 == t[u] && k2 < lane + 64 * u)));  // ties in list order
  }
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const unsigned long long bk0 = __ballot(kept[0]), bk1 = __ballot(kept[1]);
  const unsigned long long bo0 = __ballot(other[0]), bo1 = __ballot(other[1]);
  const int nkept = __popcll(bk0) + __popcll(bk1);
  const int ni = nkept + __popcll(bo0) + __popcll(bo1);
  const int opos[2] = {nkept + (int)__popcll(bo0 & lt), nkept + (int)__popcll(bo0) + (int)__popcll(bo1 & lt)};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!kept[u] && !other[u]) continue;
    const int d = kept[u] ? pos[u] : opos[u];
    q.images[d] = (int16_t)t[u];
    q.grids[d][0] = (int16_t)g0[u];
    q.grids[d][1] = (int16_t)g1[u];
  }
  if (lane == 0) {
    q.timages = nkept;
    q.num_images = ni;
    if (s.minImageNum <= ni) {
      preg[p] = reg_first(nkept);
      need_ref[p] = 1;
    } else {
      preg[p] = reg_zero();
      vreg[p] = reg_zero();
      need_ref[p] = 0;
      atomicAdd(removed, 1);
    }
  }
}

// after setRefImage: registered = target entries of the (reordered) list; empty list -> removed
__global__ void exact_after_ref_kernel(DScene s, const pmvs_patch* __restrict__ P, const int* __restrict__ list, int m,
                                       Reg* __restrict__ preg, Reg* __restrict__ vreg,
                                       int* __restrict__ removed) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const int p = list[k];
  const pmvs_patch& q = P[p];
  if (q.num_images < s.minImageNum) {
    preg[p] = reg_zero();
    vreg[p] = reg_zero();
    atomicAdd(removed, 1);
    return;
  }
  Reg r = reg_zero();
  for (int i = 0; i < q.num_images; ++i)
    if (q.images[i] < s.tnum) reg_set(r, i);
  preg[p] = r;
}

// --------------------------------------------------------------------------- filterNeighbor
struct NbSmall {
  int sb[64 * NB_SK], so[64 * NB_SK];  // gather_neighbors: per-slot list start (bit 31: vpgrids), flattened offset
  float units[PMVS_MAX_IMAGES];
  int cnt, overflow;
  double f[5];
  double nu[5], nd[5], tau[5], den;  // lls5_wave: column norms (updated / direct), Householder taus
  int perm[5], big;
  float x[5];
  double jw[5][5], ju[5][5], jv[5][5], sv[5], jy[5];  // lls5_wave's Jacobi stage (lane 0)
};
template <int CAP>
struct NbLdsT : NbSmall {
  static_assert((CAP & (CAP - 1)) == 0 && CAP >= 64, "power of two");
  static constexpr int kCap = CAP;
  static constexpr int kLlsRows = (CAP * 2 * 4) / 8;  // doubles of nb + seq filterQuad's lls rows may use
  alignas(8) int nb[CAP];  // nb and seq are adjacent: filterQuad's lls rows reuse them
  float seq[CAP];          // values summed in the reference's order by one lane (filterQuad)
};
using NbLds = NbLdsT<NB_CAP>;

// Cmylapack::lls (mylapack.cpp:102-149, Eigen JacobiSVD(ThinU | ThinV).solve) with Eigen's algorithm,
// the same operation order as the oracle's lls5 (oracle/filter_oracle.h): column-pivoting
// Householder QR of the scaled n x 5 system (rows in global scratch; per-column sums by one lane
// each, in row order; elementwise updates spread over the lanes), then two-sided Jacobi, sorting
// and the rank-thresholded minimum-norm solve on the 5 x 5 factor by lane 0.
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ double dmaxd(double a, double b) { return (a < b) ? b : a; }  // std::max
// lls5_wave's 5 x 5 stage on lane 0 (two-sided Jacobi, signs, sort, rank-thresholded solve).
__device__ __attribute__((noinline)) void lls5_jacobi(NbSmall& L, const double* M, const double* r, double scale) {
  constexpr int N = 5;
  const double eps = 2.220446049250313e-16, dmin = 2.2250738585072014e-308;
    // L lives in LDS in every caller: LDS-typed pointers give 32-bit addresses with immediate offsets
    // (generic 64-bit addresses of the unrolled 5 x 5 loops were hoisted into ~200 registers, which
    // capped the occupancy of the calling neighbour walks; one lane runs this stage)
    lds_f64* W = (lds_f64*)&L.jw[0][0];
    lds_f64* U = (lds_f64*)&L.ju[0][0];
    lds_f64* V = (lds_f64*)&L.jv[0][0];
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        W[i * N + j] = (j >= i) ? M[(size_t)i * N + j] : 0.0;
        U[i * N + j] = V[i * N + j] = (i == j) ? 1.0 : 0.0;
      }
    double maxd = 0.0;
    for (int i = 0; i < N; ++i) maxd = dmaxd(maxd, fabs(W[(i) * N + (i)]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 100; ++sweep) {
      finished = true;
#pragma nounroll
      for (int p = 1; p < N; ++p)
#pragma nounroll
        for (int q = 0; q < p; ++q) {
          const double thr = dmaxd(dmin, 2.0 * eps * maxd);
          if (!(fabs(W[(p) * N + (q)]) > thr || fabs(W[(q) * N + (p)]) > thr)) continue;
          finished = false;
          double m00 = W[(p) * N + (p)], m01 = W[(p) * N + (q)], m10 = W[(q) * N + (p)], m11 = W[(q) * N + (q)];
          const double t = m00 + m11, d = m10 - m01;
          double c1 = 1.0, s1 = 0.0;
          if (!(fabs(d) < dmin)) {
            const double u = t / d;
            const double tmp = sqrt(1.0 + u * u);
            s1 = 1.0 / tmp;
            c1 = u / tmp;
          }
          {
            const double a0 = m00, a1 = m01, b0 = m10, b1 = m11;
            m00 = c1 * a0 + s1 * b0; m01 = c1 * a1 + s1 * b1;
            m10 = -s1 * a0 + c1 * b0; m11 = -s1 * a1 + c1 * b1;
          }
          double cr = 1.0, sr = 0.0;
          const double deno = 2.0 * fabs(m01);
          if (!(deno < dmin)) {
            const double tau_ = (m00 - m11) / deno;
            const double w = sqrt(tau_ * tau_ + 1.0);
            const double tt = (tau_ > 0.0) ? 1.0 / (tau_ + w) : 1.0 / (tau_ - w);
            const double sign_t = tt > 0.0 ? 1.0 : -1.0;
            const double nn = 1.0 / sqrt(tt * tt + 1.0);
            sr = -sign_t * (m01 / fabs(m01)) * fabs(tt) * nn;
            cr = nn;
          }
          const double cl = c1 * cr - s1 * (-sr);
          const double sl = c1 * (-sr) + s1 * cr;
          for (int j = 0; j < N; ++j) {  // W rows p, q by j_left
            const double xp = W[(p) * N + (j)], xq = W[(q) * N + (j)];
            W[(p) * N + (j)] = cl * xp + sl * xq;
            W[(q) * N + (j)] = -sl * xp + cl * xq;
          }
          for (int i = 0; i < N; ++i) {  // U columns p, q by j_left^T
            const double xp = U[(i) * N + (p)], xq = U[(i) * N + (q)];
            U[(i) * N + (p)] = cl * xp - (-sl) * xq;
            U[(i) * N + (q)] = (-sl) * xp + cl * xq;
          }
          for (int i = 0; i < N; ++i) {  // W columns p, q by j_right
            const double xp = W[(i) * N + (p)], xq = W[(i) * N + (q)];
            W[(i) * N + (p)] = cr * xp - sr * xq;
            W[(i) * N + (q)] = sr * xp + cr * xq;
          }
          for (int i = 0; i < N; ++i) {  // V columns p, q by j_right
            const double xp = V[(i) * N + (p)], xq = V[(i) * N + (q)];
            V[(i) * N + (p)] = cr * xp - sr * xq;
            V[(i) * N + (q)] = sr * xp + cr * xq;
          }
          maxd = dmaxd(maxd, dmaxd(fabs(W[(p) * N + (p)]), fabs(W[(q) * N + (q)])));
        }
    }
    lds_f64* sv = (lds_f64*)L.sv;
    for (int i = 0; i < N; ++i) {
      sv[i] = fabs(W[(i) * N + (i)]);
      if (W[(i) * N + (i)] < 0.0)
        for (int k = 0; k < N; ++k) U[(k) * N + (i)] = -U[(k) * N + (i)];
    }
    for (int i = 0; i < N; ++i) sv[i] *= scale;
    int nonzero = N;
    for (int i = 0; i < N; ++i) {
      int pos = i;
      for (int j = i + 1; j < N; ++j)
        if (sv[j] > sv[pos]) pos = j;
      if (sv[pos] == 0.0) {
        nonzero = i;
        break;
      }
      if (pos != i) {
        double t = sv[i]; sv[i] = sv[pos]; sv[pos] = t;
        for (int k = 0; k < N; ++k) {
          t = U[(k) * N + (i)]; U[(k) * N + (i)] = U[(k) * N + (pos)]; U[(k) * N + (pos)] = t;
          t = V[(k) * N + (i)]; V[(k) * N + (i)] = V[(k) * N + (pos)]; V[(k) * N + (pos)] = t;
        }
      }
    }
    int rank = 0;
    if (nonzero > 0) {
      const double pre = dmaxd(sv[0] * (N * eps), dmin);
      int i = nonzero - 1;
      while (i >= 0 && sv[i] < pre) --i;
      rank = i + 1;
    }
    lds_f64* y = (lds_f64*)L.jy;
    for (int i = 0; i < rank; ++i) {
      double t = 0.0;
      for (int k = 0; k < N; ++k) t += U[(k) * N + (i)] * r[k];
      y[i] = t / sv[i];
    }
    for (int k = 0; k < N; ++k) {
      double t = 0.0;
      for (int i = 0; i < rank; ++i) t += V[(k) * N + (i)] * y[i];
      L.x[L.perm[k]] = (float)t;
    }
}

// Out of line: its registers do not add to the latency-bound neighbour walks of the callers (whose
// occupancy is register-limited); M / r rows in global scratch, the 5 x 5 stage in NbLds.  The
// one-lane row loops are unrolled by 8 so their (independent) row loads are in flight together;
// the sums stay sequential in row order.
__device__ __attribute__((noinline)) void lls5_wave(NbSmall& L, double* M, double* r, int n) {
  constexpr int N = 5;
  const double eps = 2.220446049250313e-16, dmin = 2.2250738585072014e-308;
  const int lane = lane_id_w();
  auto bar = []() {
    __threadfence_block();
    __syncthreads();
  };
  // scale = max |a_ij| (exact in any order)
  double mx = 0.0;
  for (int u = lane; u < n * N; u += 64) mx = dmaxd(mx, fabs(M[u]));
  for (int d = 32; d >= 1; d >>= 1) mx = dmaxd(mx, __shfl_xor(mx, d));
  if (!isfinite(mx)) {
    if (lane == 0)
      for (int k = 0; k < N; ++k) L.x[k] = 0.0f;
    bar();
    return;
  }
  const double scale = (mx == 0.0) ? 1.0 : mx;
  for (int u = lane; u < n * N; u += 64) M[u] = M[u] / scale;
  bar();
  // column norms (one lane per column, rows in order)
  if (lane < N) {
    double sq = 0.0;
    #pragma unroll 8
    for (int i = 0; i < n; ++i) sq += M[(size_t)i * N + lane] * M[(size_t)i * N + lane];
    L.nu[lane] = L.nd[lane] = sqrt(sq);
    L.perm[lane] = lane;
  }
  bar();
  const double downdate = sqrt(eps);
  for (int k = 0; k < N; ++k) {
    if (lane == 0) {
      int big = k;
      for (int j = k + 1; j < N; ++j)
        if (L.nu[j] > L.nu[big]) big = j;
      L.big = big;
      if (big != k) {
        double t = L.nu[k]; L.nu[k] = L.nu[big]; L.nu[big] = t;
        t = L.nd[k]; L.nd[k] = L.nd[big]; L.nd[big] = t;
        const int pk = L.perm[k]; L.perm[k] = L.perm[big]; L.perm[big] = pk;
      }
    }
    bar();
    const int big = L.big;
    if (big != k)
      for (int i = lane; i < n; i += 64) {
        const double t = M[(size_t)i * N + k];
        M[(size_t)i * N + k] = M[(size_t)i * N + big];
        M[(size_t)i * N + big] = t;
      }
    bar();
    if (lane == 0) {  // makeHouseholderInPlace
      double tail = 0.0;
      #pragma unroll 8
      for (int i = k + 1; i < n; ++i) tail += M[(size_t)i * N + k] * M[(size_t)i * N + k];
      const double c0 = M[(size_t)k * N + k];
      double beta, tau, den = 0.0;
      if (tail <= dmin) {
        tau = 0.0;
        beta = c0;
      } else {
        beta = sqrt(c0 * c0 + tail);
        if (c0 >= 0.0) beta = -beta;
        den = c0 - beta;
        tau = (beta - c0) / beta;
      }
      L.tau[k] = tau;
      L.den = den;
      M[(size_t)k * N + k] = beta;
    }
    bar();
    const double tauk = L.tau[k], den = L.den;
    for (int i = k + 1 + lane; i < n; i += 64) M[(size_t)i * N + k] = (tauk == 0.0) ? 0.0 : M[(size_t)i * N + k] / den;
    bar();
    if (tauk != 0.0 && lane > k && lane < N) {  // applyHouseholderOnTheLeft, column j = lane
      const int j = lane;
      double t = 0.0;
      #pragma unroll 8
      for (int i = k + 1; i < n; ++i) t += M[(size_t)i * N + k] * M[(size_t)i * N + j];
      t += M[(size_t)k * N + j];
      M[(size_t)k * N + j] -= tauk * t;
      #pragma unroll 8
      for (int i = k + 1; i < n; ++i) M[(size_t)i * N + j] -= (tauk * M[(size_t)i * N + k]) * t;
    }
    bar();
    if (lane > k && lane < N && L.nu[lane] != 0.0) {  // norm downdating (LAPACK xGEQPF)
      const int j = lane;
      double t = fabs(M[(size_t)k * N + j]) / L.nu[j];
      t = (1.0 + t) * (1.0 - t);
      if (t < 0.0) t = 0.0;
      const double q = L.nu[j] / L.nd[j];
      const double t2 = t * (q * q);
      if (t2 <= downdate) {
        double sq = 0.0;
        #pragma unroll 8
        for (int i = k + 1; i < n; ++i) sq += M[(size_t)i * N + j] * M[(size_t)i * N + j];
        L.nd[j] = L.nu[j] = sqrt(sq);
      } else {
        L.nu[j] *= sqrt(t);
      }
    }
    bar();
  }
  // Q^T b
  for (int k = 0; k < N; ++k) {
    const double tauk = L.tau[k];
    if (tauk == 0.0) continue;
    if (lane == 0) {
      double t = 0.0;
      #pragma unroll 8
      for (int i = k + 1; i < n; ++i) t += M[(size_t)i * N + k] * r[i];
      t += r[k];
      L.den = t;
    }
    bar();
    const double t = L.den;
    if (lane == 0) r[k] -= tauk * t;
    for (int i = k + 1 + lane; i < n; i += 64) r[i] -= (tauk * M[(size_t)i * N + k]) * t;
    bar();
  }
  if (lane == 0) lls5_jacobi(L, M, r, scale);
  bar();
}

// Sort a[0..n) ascending (bitonic over the next power of two, padded with INT_MAX) and drop
// duplicates; returns the unique count.  All 64 lanes call it.
__device__ int sort_unique_lds(int* a, int n, int* cnt_slot) {
  const int lane = lane_id_w();
  n = uni(n);
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
  // unique, 64 per round: keep a[i] != a[i-1] (a[i-1] carried in a register across rounds, since
  // the compaction may already have overwritten it), positions by a wave prefix count.  Writes
  // land at or below the round's own reads, so one barrier between reads and writes suffices.
  int u = 0, carry = 0;
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const int x = (i < n) ? a[i] : 0x7fffffff;
    int prev = __shfl_up(x, 1);
    if (lane == 0) prev = carry;
    const bool keep = i < n && (i == 0 || x != prev);
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    carry = __shfl(x, 63);
    __syncthreads();
    if (keep) a[u + before] = x;
    u += __popcll(m);
    __syncthreads();
  }
  if (lane == 0) *cnt_slot = u;
  __syncthreads();
  return uni(u);
}

// CFilter::filterNeighborThread (filter.cpp:358-385) + findNeighbors(..., 0, 4, 2, 1)
// (patchOrganizerS.cpp:527-631) + filterQuad (filter.cpp:387-446), one wavefront per patch.
// CExpand::computeRadius (expand.cpp:182-198): second smallest of COptim::computeUnits
// (optim.cpp:446-471) times csize.  All lanes call; result in every lane.
// With the radius, findNeighbors' unit (patchOrganizerS.cpp:541-545) before its division: the images'
// getUnit summed in image order.  Lane k computes image k's getUnit once for both; the sum then reads
// them from LDS (the walks' setup had summed them in one lane-serial loop of dependent global loads).
struct RadUnit {
  float radius;  // computeRadius, csize included; < 0: not computed
  float usum;    // sum of getUnit(images[k], coord) over the images, in order
};
static_assert(PMVS_MAX_IMAGES <= 128, "compute_radius_unit: two images per lane");
__device__ RadUnit compute_radius_unit(const DScene& s, NbSmall& L, const pmvs_patch& q, bool want_usum) {
  const int lane = lane_id_w();
  const int ni = uni(q.num_images);
  __syncthreads();
  float raw0 = 0.0f, raw1 = 0.0f;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int k = lane + 64 * r;
    if (k < ni) {
      const DView& v = s.views[q.images[k]];
      float u = get_unit(s, v, q.coord);
      if (r == 0) raw0 = u;
      else raw1 = u;
      float ray[4] = {v.center[0] - q.coord[0], v.center[1] - q.coord[1], v.center[2] - q.coord[2], v.center[3] - q.coord[3]};
      unitize4(ray);
      const float den = dot4(ray, q.normal);
      u = (0.0f < den) ? __fdiv_rn(u, den) : 1073741824.0f;
      L.units[k] = u;
    }
  }
  __syncthreads();
  float m1 = 3.0e38f, m2 = 3.0e38f;  // two smallest (nth_element(begin, begin + 1, end))
  for (int k = 0; k < ni; ++k) {
    const float u = L.units[k];
    if (u < m1) { m2 = m1; m1 = u; }
    else if (u < m2) m2 = u;
  }
  RadUnit ru{m2 * (float)s.csize, 0.0f};
  if (want_usum) {
    __syncthreads();
    if (lane < ni) L.units[lane] = raw0;
    if (lane + 64 < ni) L.units[lane + 64] = raw1;
    __syncthreads();
    float us = 0.0f;
    for (int k = 0; k < ni; ++k) us += L.units[k];
    ru.usum = us;
  }
  return ru;
}
__device__ float compute_radius_wave(const DScene& s, NbSmall& L, const pmvs_patch& q) {
  return compute_radius_unit(s, L, q, false).radius;
}

// CPatchOrganizerS::findNeighbors(patch, neighbors, lock, scale, margin, skipvis)
// (patchOrganizerS.cpp:527-631) into L.nb[0..n), sorted by patch index and unique.  Returns n;
// L.overflow is set when more than NB_CAP unique neighbours exist.
__device__ __forceinline__ int wave_excl_scan_w(int v) {
  const int lane = lane_id_w();
  int x = v;
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x - v;
}

// The candidates a findNeighbors walk has already tested, as an open-addressing set over NbLds.seq
// (free during the walk; filterQuad writes it afterwards).  A patch registered in several of the
// walked images' cells is met once per image; isNeighbor(patch, j) does not depend on the cell it
// was found in, so only the first meeting is tested (the hit list's final sort + unique removes
// duplicates either way).  A crowded probe sequence just tests again.
template <int CAP>
__device__ __forceinline__ void nb_seen_clear(NbLdsT<CAP>& L) {
  int* tab = reinterpret_cast<int*>(L.seq);
  for (int i = lane_id_w(); i < CAP; i += 64) tab[i] = -1;
}
template <int CAP>
__device__ __forceinline__ bool nb_first_visit(NbLdsT<CAP>& L, int j) {
  int* tab = reinterpret_cast<int*>(L.seq);
  constexpr int kBits = __builtin_ctz(CAP);
  unsigned h = ((unsigned)j * 2654435761u) >> (32 - kBits);  // kBits bits: CAP slots
  for (int probe = 0; probe < 16; ++probe) {
    const int old = atomicCAS(&tab[h], -1, j);
    if (old == -1) return true;
    if (old == j) return false;
    h = (h + 1) & (CAP - 1);
  }
  return true;
}

// Appends the hits of one 64-lane round in lane order (ballot), compacting the buffer (sort +
// unique) when it nears capacity, as the reference's final sort/unique would (same set).
// cap: the capacity in use (CAP, or less under PMVS_NB_SOFTCAP in tests).
template <int CAP>
__device__ __forceinline__ void nb_append(NbLdsT<CAP>& L, bool hit, int j, int cap) {
  const int lane = lane_id_w();
  const unsigned long long mask = __ballot(hit);
  const int before = __popcll(mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
  const int pos = L.cnt + before;
  if (hit) {
    if (pos < cap) L.nb[pos] = j;
    else L.overflow = 1;
  }
  __syncthreads();
  if (lane == 0) L.cnt += __popcll(mask);
  __syncthreads();
  const int cnt = uni(L.cnt);
  if (cnt > cap - 64 && !uni(L.overflow)) sort_unique_lds(L.nb, imin(cnt, cap), &L.cnt);
}

// CPatchOrganizerS::findNeighbors(patch, neighbors, lock, scale, margin, skipvis)
// (patchOrganizerS.cpp:527-631) into L.nb[0..n), sorted by patch index and unique.  Returns n;
// L.overflow is set when more than NB_CAP unique neighbours exist.
// The (image list, dy, dx, pgrids/vpgrids) cells are visited 64 at a time, one per lane (their
// list bounds load in parallel); the cells' entries are then flattened and tested 64 per round.
// Expansion-time chain entries (FilterDev delta) are walked per lane.  The neighbour SET is the
// reference's; the visiting order only matters for the buffer's compaction points.
// CHM: the largest margin whose expansion-time chains the caller walks (0: the filter pass, which has
// none -- F.pg_dhead is nullptr there; chains met anyway are an error, code 16).
template <int CAP, int CHM>
__device__ __forceinline__ int gather_neighbors(const DScene& s, const FilterDev& F, NbLdsT<CAP>& L, const pmvs_patch& q, float scale,
                                int margin, int skipvis, unsigned long long* prof = nullptr, RadUnit pre = {-1.0f, 0.0f}) {
  const int lane = lane_id_w();
  unsigned long long nbp_t = NBP_NOW();
  (void)nbp_t;
  (void)prof;
  // the capacity in use: CAP (a test soft cap, F.nb_softcap, applies to the NB_CAP form only)
  const int cap = (CAP == NB_CAP && F.nb_softcap > 0) ? imin(CAP, F.nb_softcap) : CAP;
  const int ni = uni(q.num_images);
  const RadUnit ru = (pre.radius >= 0.0f) ? pre : compute_radius_unit(s, L, q, true);
  const float radius = (float)(1.5 * margin * (double)ru.radius);
  float unit = __fdiv_rn(ru.usum, (float)ni);
  unit *= (float)s.csize;
  const float thr = 0.5f * scale;
  if (lane == 0) { L.cnt = 0; L.overflow = 0; }
  nb_seen_clear(L);
  __syncthreads();
  const int nlists = skipvis ? ni : ni + uni(q.num_vimages);
  const int side = 2 * margin + 1;
#if PMVS_NB_ROWS
  const int per_list = side * 2;  // (row, pgrids / vpgrids)
#else
  const int per_list = side * side * 2;  // (row, column, pgrids / vpgrids)
#endif
  const bool chains = F.pg_dhead != nullptr;
  const int nslots = nlists * per_list;
  // NB_SK slots per lane per round (their list bounds load together), then the round's entries
  // NB_NE per lane at a time (their item and patch loads in flight together): fewer dependent
  // global-memory round trips per patch than one slot / one entry per lane.
  for (int base = 0; base < nslots; base += 64 * NB_SK) {
    // per slot: list start (bit 31: vpgrids) and length; for the expansion's chains its first cell
    // and the cells (bit dx) whose chain is not empty
    int bk[NB_SK], ck[NB_SK], hk[NB_SK];
    long long ck0[NB_SK];
#pragma unroll
    NBP(base == 0 ? 0 : 2);
    for (int k = 0; k < NB_SK; ++k) {
      const int slot = base + k * 64 + lane;
      int b = 0, e = 0, lst = 0, hm = 0;
      long long c0 = 0;
      if (slot < nslots) {
        const int li = slot / per_list;
        int r = slot - li * per_list;
#if PMVS_NB_ROWS
        const int dyi = r >> 1;
        lst = r & 1;
#else
        const int dyi = r / (2 * side);
        r -= dyi * 2 * side;
        const int dxi = r >> 1;
        lst = r & 1;
#endif
        const bool vis = li >= ni;
        const int t = vis ? q.vimages[li - ni] : q.images[li];
        if (t < s.tnum) {
          const int gw = gwidth(s, t), gh = gheight(s, t);
          const int yt = (vis ? q.vgrids[li - ni][1] : q.grids[li][1]) + dyi - margin;
          const int gx = vis ? q.vgrids[li - ni][0] : q.grids[li][0];
#if PMVS_NB_ROWS
          const int x0 = imax(gx - margin, 0), x1 = imin(gx + margin, gw - 1);
#else
          const int x0 = gx + dxi - margin, x1 = x0;
#endif
          if (0 <= yt && yt < gh && 0 <= x0 && x0 <= x1 && x1 < gw) {
            c0 = F.tgoff[t] + (long long)yt * gw + x0;
            const int nx = x1 - x0 + 1;
            const int* off = lst ? F.vp_off : F.pg_off;
            const int lim = lst ? F.nvp : F.npg;
            b = off[c0];
            e = off[c0 + nx];
            if (b < 0 || e > lim || b > e) {
              atomicAdd(&F.err[0], 1);
              atomicExch(&F.err[1], 12 + lst);
              b = 0;
              e = 0;
            }
            if (chains) {
              const int* dh = lst ? F.vp_dhead : F.pg_dhead;
              for (int dx = 0; dx < nx; ++dx) hm |= (dh[c0 + dx] >= 0 ? 1 : 0) << dx;
            }
          }
        }
      }
      bk[k] = b | (lst << 31);  // list start, list kind in bit 31
      ck[k] = e - b;
      hk[k] = hm;
      ck0[k] = c0;
    }
    // the round's CSR entries, flattened in (lane, k) order
    int mine = 0;
#pragma unroll
    for (int k = 0; k < NB_SK; ++k) mine += ck[k];
    const int offl = wave_excl_scan_w(mine);
    const int tot = uni(__shfl(offl + mine, 63));
    {
      int o = offl;
#pragma unroll
      for (int k = 0; k < NB_SK; ++k) {
        L.sb[lane * NB_SK + k] = bk[k];
        L.so[lane * NB_SK + k] = o;
        o += ck[k];
      }
    }
    __syncthreads();
    NBP(1);
    for (int ib = 0; ib < tot; ib += 64 * NB_NE) {
      int jv[NB_NE];
      bool hv[NB_NE];
#pragma unroll
      for (int u = 0; u < NB_NE; ++u) {
        const int idx = ib + u * 64 + lane;
        jv[u] = -1;
        if (idx < tot) {
          int sidx = 0;  // the last slot whose offset is <= idx (it holds idx)
          for (int step = 64 * NB_SK / 2; step >= 1; step >>= 1)
            if (sidx + step < 64 * NB_SK && L.so[sidx + step] <= idx) sidx += step;
          const int sb = L.sb[sidx];
          const int* items = (sb < 0) ? F.vp_items : F.pg_items;
          jv[u] = items[(sb & 0x7fffffff) + idx - L.so[sidx]];
        }
      }
#pragma unroll
      for (int u = 0; u < NB_NE; ++u) {
        const int j = jv[u];
        hv[u] = false;
        if (ib + u * 64 + lane < tot) {
          if (j < 0 || j >= F.n) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 14); jv[u] = 0; }
          else if (nb_first_visit(L, j)) hv[u] = is_neighbor_h(q, F.hot[j], unit, thr, radius, true) != 0;
        }
      }
#pragma unroll
      for (int u = 0; u < NB_NE; ++u)
        if (ib + u * 64 < tot) nb_append(L, hv[u], jv[u] < 0 ? 0 : jv[u], cap);
    }
    NBP(2);
    // entries committed by earlier expansion waves (per-cell chains, FilterDev delta): slot by slot,
    // every lane walks the chains of all the slot's row cells at once -- one cursor per cell, their
    // item / next loads in flight together -- so a round costs one dependent load per chain step, not
    // one per chain step of every cell in turn (round 6: iteration 1 of the C3 loop, where the whole
    // growing model is in chains, spent 69 % of findEmptyBlocks' cycles here cell by cell, r06w)
    int hany = 0;
#pragma unroll
    for (int k = 0; k < NB_SK; ++k) hany |= hk[k];
    if (chains && __ballot(hany != 0) != 0ull) {
      if (CHM == 0 || margin > CHM) {
        if (lane == 0) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 16); }
      } else {
        constexpr int MC = 2 * CHM + 1;
#pragma unroll
        for (int k = 0; k < NB_SK; ++k) {
        if (__ballot(hk[k] != 0) == 0ull) continue;
        int cur[MC];
#pragma unroll
        for (int dx = 0; dx < MC; ++dx) {
          const int* dh = (bk[k] < 0) ? F.vp_dhead : F.pg_dhead;
          cur[dx] = (dx < side && ((hk[k] >> dx) & 1)) ? dh[ck0[k] + dx] : -1;
        }
        for (;;) {
          int adds = 0;  // the round's appends at most: its live cursors over the wavefront
#pragma unroll
          for (int m = 0; m < MC; ++m) adds += __popcll(__ballot(cur[m] >= 0));
          if (adds == 0) break;
          const int cnt0 = uni(L.cnt);
          if (cnt0 + adds > cap && !uni(L.overflow)) sort_unique_lds(L.nb, imin(cnt0, cap), &L.cnt);
          int jm[MC];
#pragma unroll
          for (int m = 0; m < MC; ++m) {
            jm[m] = -2;
            if (cur[m] >= 0) {
              const int2 en = F.d_ent[cur[m]];
              jm[m] = en.x;
              cur[m] = en.y;
            }
          }
#pragma unroll
          for (int m = 0; m < MC; ++m) {
            const int j = jm[m];
            if (j == -2) continue;
            if (j < 0 || j >= F.n) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 15); continue; }
            if (nb_first_visit(L, j) && is_neighbor_h(q, F.hot[j], unit, thr, radius, true)) {
              const int pos = atomicAdd(&L.cnt, 1);
              if (pos < cap) L.nb[pos] = j;
              else L.overflow = 1;
            }
          }
          __syncthreads();
          if (lane == 0 && L.cnt > cap) L.cnt = cap;
          __syncthreads();
        }
        }
        const int cnt = uni(L.cnt);
        if (cnt > cap - 64 && !uni(L.overflow)) sort_unique_lds(L.nb, imin(cnt, cap), &L.cnt);
      }
    }
    __syncthreads();
    NBP(3);
  }
  const int n = imin(uni(L.cnt), cap);
#if defined(NBX_SKIP_SORT)  // timing experiment only (tools): the final sort skipped
  return n;
#else
  const int nu = sort_unique_lds(L.nb, n, &L.cnt);
  NBP(4);
  return nu;
#endif
}

// CFilter::filterQuad (filter.cpp:387-446) on the neighbours in L.nb[0..n); returns 1 = reject.
// fout != nullptr: the rows' fx[n], fy[n], fz[n] go there and the fit is left to quad_lane_kernel
// (returns -1).
template <int CAP>
__device__ __forceinline__ int filter_quad_wave(const DScene& s, const FilterDev& F, NbLdsT<CAP>& L, double* M, double* r,
                                const pmvs_patch& q, int n, float* fout = nullptr) {
  const int lane = lane_id_w();
  n = uni(n);
  float xdir[4] = {0, 0, 0, 0}, ydir[4] = {0, 0, 0, 0};
  const float* z = q.normal;
  if (fabs((double)z[0]) > 0.5) { xdir[0] = z[1]; xdir[1] = -z[0]; xdir[2] = 0; }
  else if (fabs((double)z[1]) > 0.5) { xdir[1] = z[2]; xdir[2] = -z[1]; xdir[0] = 0; }
  else { xdir[2] = z[0]; xdir[0] = -z[2]; xdir[1] = 0; }
  unitize4(xdir);
  ydir[0] = z[1] * xdir[2] - z[2] * xdir[1];
  ydir[1] = z[2] * xdir[0] - z[0] * xdir[2];
  ydir[2] = z[0] * xdir[1] - z[1] * xdir[0];
  float* gx = fout ? fout : reinterpret_cast<float*>(r + CAP);  // fx, fy, fz (workgroup's global scratch)
  float* gy = gx + (fout ? n : CAP);
  float* gz = gy + (fout ? n : CAP);
  for (int a = lane; a < n; a += 64) {  // the distances in parallel, their sum in order below
    float d[4];
    for (int k = 0; k < 4; ++k) d[k] = F.hot[L.nb[a]].coord[k] - q.coord[k];
    L.seq[a] = norm4(d);
  }
  __syncthreads();
  if (lane == 0) {
    float h = 0.0f;
    for (int a = 0; a < n; ++a) h += L.seq[a];
    L.f[1] = (double)__fdiv_rn(h, (float)n);
  }
  __syncthreads();
  const float h = (float)L.f[1];
  for (int a = lane; a < n; a += 64) {
    float d[4];
    for (int k = 0; k < 4; ++k) d[k] = F.hot[L.nb[a]].coord[k] - q.coord[k];
    const float fx = __fdiv_rn(dot4(d, xdir), h), fy = __fdiv_rn(dot4(d, ydir), h), fz = dot4(d, q.normal);
    gx[a] = fx; gy[a] = fy; gz[a] = fz;
  }
  if (fout) return -1;
  // The lls rows: in LDS over the neighbour list and seq[] (free until the residuals) when they
  // fit -- the solver's many wave barriers then drain LDS traffic only -- else in global scratch.
  __syncthreads();
  if (n * 6 <= NbLdsT<CAP>::kLlsRows) {
    M = reinterpret_cast<double*>(L.nb);
    r = M + (size_t)n * 5;
  }
  for (int a = lane; a < n; a += 64) {
    const float fx = gx[a], fy = gy[a], fz = gz[a];  // this lane's own stores
    M[(size_t)a * 5 + 0] = (double)(fx * fx);
    M[(size_t)a * 5 + 1] = (double)(fy * fy);
    M[(size_t)a * 5 + 2] = (double)(fx * fy);
    M[(size_t)a * 5 + 3] = (double)fx;
    M[(size_t)a * 5 + 4] = (double)fy;
    r[a] = (double)fz;
  }
  __threadfence_block();
  __syncthreads();
#if defined(NBX_SKIP_LLS)  // timing experiment only (tools): the quadric fit skipped
  if (lane < 5) L.x[lane] = 0.0f;
  __syncthreads();
#else
  lls5_wave(L, M, r, n);
#endif
  // The residual terms |r_a| / u2 in parallel (each lane its own rows; every lane computes the same
  // u2), into the lls rows' space (free now), then their float += double sum in the reference's order.
  const int inum = imin(s.tau, q.num_images);
  float u2 = 0.0f;
  for (int k = 0; k < inum; ++k) u2 += get_unit(s, s.views[q.images[k]], q.coord);
  u2 = __fdiv_rn(u2, (float)inum);
  double* term = M;
  for (int a = lane; a < n; a += 64) {
    const float fx = gx[a], fy = gy[a];
    const float ra = L.x[0] * (fx * fx) + L.x[1] * (fy * fy) + L.x[2] * (fx * fy) + L.x[3] * fx + L.x[4] * fy - gz[a];
    term[a] = fabs((double)ra) / (double)u2;
  }
  __threadfence_block();
  __syncthreads();
  if (lane == 0) {
    float residual = 0.0f;
    for (int a = 0; a < n; ++a)  // in the reference's order
      residual = (float)((double)residual + term[a]);  // float += double
    residual = __fdiv_rn(residual, (float)(n - 5));
    L.cnt = (residual < s.quad ? 0 : 1);
  }
  __syncthreads();
  return uni(L.cnt);
}

// CFilter::filterNeighborThread (filter.cpp:358-385): findNeighbors(patch, ., 0, 4, 2, 1), reject
// with fewer than 6 neighbours or a failed quadric fit.  One wavefront per patch.
// Sharded loop (world > 1): a rank tests only the patches whose reference image it owns
// (target t belongs to rank t mod world); the others are left to their owners
// and the reject flags are all-gathered afterwards (filter_pass).
// Overflow (more than CAP unique neighbours): with `ovf` (the NB_CAP form) the patch goes on the
// re-walk list ovf.items and the NB_CAP_BIG form (ovf.only: walks that list) decides it; without,
// it is counted in `overflow` (an error for the run).
struct NbOverflow {
  int* items = nullptr;        // NB_CAP form: the overflowed work items (patch / parent / candidate)
  int* count = nullptr;        // their number
  const int* only = nullptr;   // NB_CAP_BIG form: walk items only[0 .. *only_n)
  const int* only_n = nullptr;
};
template <int CAP>
__global__ __launch_bounds__(64) NB_WALK_ATTR void neighbor_kernel(DScene s, FilterDev F, double* __restrict__ scratch,
                                                      int* __restrict__ reject, int* __restrict__ overflow,
                                                      int* __restrict__ queue, int* __restrict__ dbg_counts, int rank,
                                                      int world, QuadJobs qj, NbOverflow ov) {
  __shared__ NbLdsT<CAP> L;
  const int lane = threadIdx.x;
  double* M = scratch + (size_t)blockIdx.x * (CAP * 8);
  double* r = M + (size_t)CAP * 5;
#if defined(NB_PROFILE)
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nbp_t = NBP_NOW();
#else
  unsigned long long* prof = nullptr;
#endif
  for (;;) {
    NBP(6);
    int i = 0;
    if (lane == 0) i = atomicAdd(queue, 1);
    i = __builtin_amdgcn_readfirstlane(i);  // work-queue index, wave-uniform (SGPR)
    if (i >= (ov.only ? *ov.only_n : F.nalive)) break;
    const int p = __builtin_amdgcn_readfirstlane(ov.only ? ov.only[i] : F.order[i]);
    const pmvs_patch& q = F.P[p];
    int rej = 0;  // _fix patches are kept; no early `continue` (see depth_post_kernel)
    const bool mine = world <= 1 || uni(q.images[0]) % world == rank;
    if (mine && !uni(q.fix)) {
      NBP(6);
      const int n = gather_neighbors<CAP, 0>(s, F, L, q, 4.0f, 2, 1, prof);
#if defined(NB_PROFILE)
      nbp_t = NBP_NOW();
#endif
      const bool rewalk = ov.items && uni(L.overflow);
      if (lane == 0 && rewalk) ov.items[atomicAdd(ov.count, 1)] = p;
      if (lane == 0 && L.overflow && !ov.items) atomicAdd(overflow, 1);
      if (lane == 0 && dbg_counts) dbg_counts[p] = L.overflow ? -n : n;
      if (rewalk) {
        rej = 0;  // decided by the NB_CAP_BIG re-walk
      } else if (n < 6) {
        rej = 1;
      } else {
        // room for the rows in the deferred-fit buffers? (else the fit runs here, same result)
        unsigned long long o = ~0ull;
        if (lane == 0 && qj.f) o = atomicAdd(qj.rows_used, (unsigned long long)n);
        const unsigned long long lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(o & 0xffffffffull));
        const unsigned long long hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(o >> 32));
        o = (hi << 32) | lo;
        if (o + (unsigned long long)n <= qj.cap_rows) {
          filter_quad_wave(s, F, L, M, r, q, n, qj.f + 3ull * o);
          if (lane == 0) {
            const int k = atomicAdd(qj.njobs, 1);
            qj.jobs[k] = make_int4(p, (int)o, n, 0);
          }
        } else {
          rej = filter_quad_wave(s, F, L, M, r, q, n);
        }
      }
    }
    if (lane == 0) reject[p] = rej;
    __syncthreads();
    NBP(5);
  }
  NBP_FLUSH(0);
}

// filterQuad's fit and residual test for the patches neighbor_kernel deferred, one lane per patch:
// Cmylapack::lls as the oracle's lls5 (oracle/filter_oracle.h, Eigen JacobiSVD semantics) in its
// sequential operation order -- which is also lls5_wave's (per-column sums in row order) -- so the
// decision is the same as the in-wave fit's.  Jobs run in descending row count (qsorted: 64-bit
// keys (2047 - n) << 32 | job), so a wavefront's 64 lanes have similar loop trips and its chunk of
// the row pool is 64 x (first lane's n) rows; element (row i, column j; j = 5 is Q^T b) of lane l
// sits at pool[6 * qoff[chunk] + (6 i + j) * 64 + l], so every column walk is a coalesced 512-B
// access.  The 5 x 5 Jacobi stage runs in registers.
__device__ __forceinline__ double dmaxd2(double a, double b) { return (a < b) ? b : a; }  // std::max
__global__ void quad_chunk_rows_kernel(const unsigned long long* __restrict__ qsorted, int njobs, int* __restrict__ crows) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c * 64 < njobs) crows[c] = 64 * (2047 - (int)(qsorted[(size_t)c * 64] >> 32));
}
__global__ void quad_keys_kernel(const int4* __restrict__ jobs, int njobs, unsigned long long* __restrict__ keys) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < njobs) keys[k] = ((unsigned long long)(2047 - jobs[k].z) << 32) | (unsigned)k;
}
__device__ inline void quad_lane_job(const DScene& s, const FilterDev& F, const QuadJobs& qj,
                                     const unsigned long long* __restrict__ qsorted, const int* __restrict__ qoff, int k,
                                     int* __restrict__ reject);
__device__ inline void quad_solve(const DScene& s, const FilterDev& F, const double* M, const int* perm, double scale,
                                  bool fin, int p, int n, const float* gx, const float* gy, const float* gz,
                                  int* __restrict__ reject);
__global__ __launch_bounds__(256) void quad_lane_kernel(DScene s, FilterDev F, QuadJobs qj, const unsigned long long* __restrict__ qsorted,
                                                        const int* __restrict__ qoff, int njobs, int* __restrict__ reject,
                                                        const int* __restrict__ klim) {
  // grid-stride over the jobs: a capped grid (PMVS_QUAD_WAVES_PER_CU) bounds the row working set
  // of the resident wavefronts.  klim: the jobs [0, *klim) (the rest go to quad_qr_kernel)
  const int kend = klim ? imin(njobs, *klim) : njobs;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < kend; k += gridDim.x * blockDim.x)
    quad_lane_job(s, F, qj, qsorted, qoff, k, reject);
}
__device__ inline void quad_lane_job(const DScene& s, const FilterDev& F, const QuadJobs& qj,
                                                                   const unsigned long long* __restrict__ qsorted,
                                                                   const int* __restrict__ qoff, int k, int* __restrict__ reject) {
  constexpr int N = 5;
  const double eps = 2.220446049250313e-16, dmin = 2.2250738585072014e-308;
  const int4 jb = qj.jobs[(int)(qsorted[k] & 0xffffffffull)];
  const int p = jb.x, n = jb.z;
  const size_t o = (size_t)jb.y;
  const float* gx = qj.f + 3 * o;
  const float* gy = gx + n;
  const float* gz = gy + n;
  double* base = qj.rows + 6 * (size_t)qoff[k >> 6] + (k & 63);
  double* M = base;  // at(i, j) = M[(6 i + j) * 64]
  double scale = 0.0;
  for (int i = 0; i < n; ++i) {
    const float fx = gx[i], fy = gy[i];
    const double a[5] = {(double)(fx * fx), (double)(fy * fy), (double)(fx * fy), (double)fx, (double)fy};
    for (int j = 0; j < N; ++j) {
      M[(size_t)(6 * i + j) * 64] = a[j];
      scale = dmaxd2(scale, fabs(a[j]));
    }
    M[(size_t)(6 * i + 5) * 64] = (double)gz[i];
  }
  const bool fin = isfinite(scale);
  int perm[N] = {0, 1, 2, 3, 4};
  if (fin) {
    if (scale == 0.0) scale = 1.0;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < N; ++j) M[(size_t)(6 * i + j) * 64] = M[(size_t)(6 * i + j) * 64] / scale;
    auto rr = [&](int i) -> double& { return M[(size_t)(6 * i + 5) * 64]; };
    auto at = [&](int i, int j) -> double& { return M[(size_t)(6 * i + j) * 64]; };
    // ---- column-pivoting Householder QR
    double nu[N], nd[N], tau[N];
    for (int j = 0; j < N; ++j) {
      perm[j] = j;
      double sq = 0.0;
      for (int i = 0; i < n; ++i) sq += at(i, j) * at(i, j);
      nd[j] = nu[j] = sqrt(sq);
    }
    const double downdate = sqrt(eps);
    for (int kk = 0; kk < N; ++kk) {
      int big = kk;
      for (int j = kk + 1; j < N; ++j)
        if (nu[j] > nu[big]) big = j;
      if (big != kk) {
        for (int i = 0; i < n; ++i) { const double t = at(i, kk); at(i, kk) = at(i, big); at(i, big) = t; }
        double t = nu[kk]; nu[kk] = nu[big]; nu[big] = t;
        t = nd[kk]; nd[kk] = nd[big]; nd[big] = t;
        const int pk = perm[kk]; perm[kk] = perm[big]; perm[big] = pk;
      }
      double tail = 0.0;
      for (int i = kk + 1; i < n; ++i) tail += at(i, kk) * at(i, kk);
      const double c0 = at(kk, kk);
      double beta;
      if (tail <= dmin) {
        tau[kk] = 0.0;
        beta = c0;
        for (int i = kk + 1; i < n; ++i) at(i, kk) = 0.0;
      } else {
        beta = sqrt(c0 * c0 + tail);
        if (c0 >= 0.0) beta = -beta;
        const double den = c0 - beta;
        for (int i = kk + 1; i < n; ++i) at(i, kk) = at(i, kk) / den;
        tau[kk] = (beta - c0) / beta;
      }
      at(kk, kk) = beta;
      if (tau[kk] != 0.0)
        for (int j = kk + 1; j < N; ++j) {
          double t = 0.0;
          for (int i = kk + 1; i < n; ++i) t += at(i, kk) * at(i, j);
          t += at(kk, j);
          at(kk, j) -= tau[kk] * t;
          for (int i = kk + 1; i < n; ++i) at(i, j) -= (tau[kk] * at(i, kk)) * t;
        }
      for (int j = kk + 1; j < N; ++j) {
        if (nu[j] == 0.0) continue;
        double t = fabs(at(kk, j)) / nu[j];
        t = (1.0 + t) * (1.0 - t);
        if (t < 0.0) t = 0.0;
        const double qq = nu[j] / nd[j];
        const double t2 = t * (qq * qq);
        if (t2 <= downdate) {
          double sq = 0.0;
          for (int i = kk + 1; i < n; ++i) sq += at(i, j) * at(i, j);
          nd[j] = nu[j] = sqrt(sq);
        } else {
          nu[j] *= sqrt(t);
        }
      }
    }
    for (int kk = 0; kk < N; ++kk) {  // Q^T b
      if (tau[kk] == 0.0) continue;
      double t = 0.0;
      for (int i = kk + 1; i < n; ++i) t += at(i, kk) * rr(i);
      t += rr(kk);
      rr(kk) -= tau[kk] * t;
      for (int i = kk + 1; i < n; ++i) rr(i) -= (tau[kk] * at(i, kk)) * t;
    }
  }
  quad_solve(s, F, M, perm, scale, fin, p, n, gx, gy, gz, reject);
}

// The two-sided Jacobi stage on R, the rank-thresholded minimum-norm solve and filterQuad's residual
// test, on a pivoted QR left in the lane layout (rows 0..4: R in the upper triangle, Q^T b in column 5).
__device__ inline void quad_solve(const DScene& s, const FilterDev& F, const double* M, const int* perm, double scale,
                                  bool fin, int p, int n, const float* gx, const float* gy, const float* gz,
                                  int* __restrict__ reject) {
  constexpr int N = 5;
  const double eps = 2.220446049250313e-16, dmin = 2.2250738585072014e-308;
  float x[N] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  if (fin) {
    auto rr = [&](int i) -> double { return M[(size_t)(6 * i + 5) * 64]; };
    auto at = [&](int i, int j) -> double { return M[(size_t)(6 * i + j) * 64]; };
    // ---- two-sided Jacobi on R
    double W[N][N], U[N][N], V[N][N];
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        W[i][j] = (j >= i) ? at(i, j) : 0.0;
        U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
      }
    double maxd = 0.0;
    for (int i = 0; i < N; ++i) maxd = dmaxd2(maxd, fabs(W[i][i]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 100; ++sweep) {
      finished = true;
#pragma unroll
      for (int pp = 1; pp < N; ++pp)
#pragma unroll
        for (int q = 0; q < pp; ++q) {
          const double thr = dmaxd2(dmin, 2.0 * eps * maxd);
          if (!(fabs(W[pp][q]) > thr || fabs(W[q][pp]) > thr)) continue;
          finished = false;
          double m00 = W[pp][pp], m01 = W[pp][q], m10 = W[q][pp], m11 = W[q][q];
          const double t = m00 + m11, d = m10 - m01;
          double c1 = 1.0, s1 = 0.0;
          if (!(fabs(d) < dmin)) {
            const double u = t / d;
            const double tmp = sqrt(1.0 + u * u);
            s1 = 1.0 / tmp;
            c1 = u / tmp;
          }
          {
            const double a0 = m00, a1 = m01, b0 = m10, b1 = m11;
            m00 = c1 * a0 + s1 * b0; m01 = c1 * a1 + s1 * b1;
            m10 = -s1 * a0 + c1 * b0; m11 = -s1 * a1 + c1 * b1;
          }
          double cr = 1.0, sr = 0.0;
          const double deno = 2.0 * fabs(m01);
          if (!(deno < dmin)) {
            const double tau_ = (m00 - m11) / deno;
            const double w = sqrt(tau_ * tau_ + 1.0);
            const double tt = (tau_ > 0.0) ? 1.0 / (tau_ + w) : 1.0 / (tau_ - w);
            const double sign_t = tt > 0.0 ? 1.0 : -1.0;
            const double nn = 1.0 / sqrt(tt * tt + 1.0);
            sr = -sign_t * (m01 / fabs(m01)) * fabs(tt) * nn;
            cr = nn;
          }
          const double cl = c1 * cr - s1 * (-sr);
          const double sl = c1 * (-sr) + s1 * cr;
#pragma unroll
          for (int j = 0; j < N; ++j) {  // W rows pp, q by j_left
            const double xp = W[pp][j], xq = W[q][j];
            W[pp][j] = cl * xp + sl * xq;
            W[q][j] = -sl * xp + cl * xq;
          }
#pragma unroll
          for (int i = 0; i < N; ++i) {  // U columns pp, q by j_left^T
            const double xp = U[i][pp], xq = U[i][q];
            U[i][pp] = cl * xp - (-sl) * xq;
            U[i][q] = (-sl) * xp + cl * xq;
          }
#pragma unroll
          for (int i = 0; i < N; ++i) {  // W columns pp, q by j_right
            const double xp = W[i][pp], xq = W[i][q];
            W[i][pp] = cr * xp - sr * xq;
            W[i][q] = sr * xp + cr * xq;
          }
#pragma unroll
          for (int i = 0; i < N; ++i) {  // V columns pp, q by j_right
            const double xp = V[i][pp], xq = V[i][q];
            V[i][pp] = cr * xp - sr * xq;
            V[i][q] = sr * xp + cr * xq;
          }
          maxd = dmaxd2(maxd, dmaxd2(fabs(W[pp][pp]), fabs(W[q][q])));
        }
    }
    // ---- singular values, signs, scale; sorted descending (selection, unrolled: register arrays)
    double sv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      sv[i] = fabs(W[i][i]);
      if (W[i][i] < 0.0)
#pragma unroll
        for (int kk = 0; kk < N; ++kk) U[kk][i] = -U[kk][i];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) sv[i] *= scale;
    int nonzero = N;
    bool stop = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (stop) continue;
      int pos = i;
#pragma unroll
      for (int j = i + 1; j < N; ++j)
        if (sv[j] > sv[pos]) pos = j;
      double svp = sv[i];
#pragma unroll
      for (int j = i + 1; j < N; ++j)
        if (pos == j) svp = sv[j];
      if (svp == 0.0) {
        nonzero = i;
        stop = true;
        continue;
      }
#pragma unroll
      for (int j = i + 1; j < N; ++j)
        if (pos == j) {
          double t = sv[i]; sv[i] = sv[j]; sv[j] = t;
#pragma unroll
          for (int kk = 0; kk < N; ++kk) {
            t = U[kk][i]; U[kk][i] = U[kk][j]; U[kk][j] = t;
            t = V[kk][i]; V[kk][i] = V[kk][j]; V[kk][j] = t;
          }
        }
    }
    int rank = 0;
    if (nonzero > 0) {
      const double pre = dmaxd2(sv[0] * (N * eps), dmin);
      int i = nonzero - 1;
#pragma unroll
      for (int c = N - 1; c >= 0; --c)
        if (c == i && sv[c] < pre) --i;
      rank = i + 1;
    }
    double y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      y[i] = 0.0;
      if (i < rank) {
        double t = 0.0;
#pragma unroll
        for (int kk = 0; kk < N; ++kk) t += U[kk][i] * rr(kk);
        y[i] = t / sv[i];
      }
    }
#pragma unroll
    for (int kk = 0; kk < N; ++kk) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (i < rank) t += V[kk][i] * y[i];
#pragma unroll
      for (int c = 0; c < N; ++c)
        if (perm[kk] == c) x[c] = (float)t;
    }
  }
  // filterQuad's residual test (as filter_quad_wave's tail)
  const pmvs_patch& q = F.P[p];
  const int inum = imin(s.tau, q.num_images);
  float u2 = 0.0f;
  for (int i = 0; i < inum; ++i) u2 += get_unit(s, s.views[q.images[i]], q.coord);
  u2 = __fdiv_rn(u2, (float)inum);
  float residual = 0.0f;
  for (int a = 0; a < n; ++a) {
    const float fx = gx[a], fy = gy[a];
    const float ra = x[0] * (fx * fx) + x[1] * (fy * fy) + x[2] * (fx * fy) + x[3] * fx + x[4] * fy - gz[a];
    residual = (float)((double)residual + fabs((double)ra) / (double)u2);  // float += double
  }
  residual = __fdiv_rn(residual, (float)(n - 5));
  reject[p] = (residual < s.quad ? 0 : 1);
}

// The fits with at most nq rows, eight lanes per job (QL) and the job's rows in LDS: the same
// column-pivoting Householder steps as quad_lane_job, with every column sum still one lane's
// in-order loop -- the lanes split the columns (the five norms, the five dot products with the
// Householder vector, Q^T b's among them as column 5), and the row-wise scalings, swaps and rank-1
// updates. Applying H_kk to b inside step kk is the same arithmetic as quad_lane_job's Q^T b loop
// after the QR: column kk is final once step kk ends (later pivots and updates touch columns > kk).
// The result (R, Q^T b, perm, scale) goes to rows 0..5 of the job's lane-layout chunk for
// quad_solve_kernel.  Jobs are in descending row count, so the fits above nq rows are the prefix
// [0, kb) (quad_split_kernel) left to quad_lane_kernel.
constexpr int QL = 8;
__global__ void quad_split_kernel(const unsigned long long* __restrict__ qsorted, int njobs, int nq, int* __restrict__ kb) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= njobs) return;
  const unsigned thr = 2047u - (unsigned)nq;  // n > nq  <=>  key >> 32 < thr
  const bool big = (unsigned)(qsorted[k] >> 32) < thr;
  const bool next = k + 1 < njobs && (unsigned)(qsorted[k + 1] >> 32) < thr;
  if (k == 0 && !big) *kb = 0;
  if (big && !next) *kb = k + 1;
}

__global__ __launch_bounds__(64) void quad_qr_kernel(QuadJobs qj, const unsigned long long* __restrict__ qsorted,
                                                     const int* __restrict__ qoff, const int* __restrict__ kb_ptr,
                                                     int njobs, int nq) {
  constexpr int N = 5;
  const double dmin = 2.2250738585072014e-308;
  const double downdate = sqrt(2.220446049250313e-16);
  extern __shared__ double qlds[];  // (64 / QL) jobs x nq rows x 6
  __shared__ double sh_nu[64 / QL][N], sh_nd[64 / QL][N], sh_t[64 / QL][N + 1], sh_c[64 / QL][3];
  __shared__ int sh_perm[64 / QL][N];
  const int lane = threadIdx.x, js = lane / QL, jl = lane % QL;
  const int kb = *kb_ptr;
  double* A = qlds + (size_t)js * nq * 6;  // at(i, j) = A[6 i + j], j = 5: b
  for (int k0 = kb + blockIdx.x * (64 / QL); k0 < njobs; k0 += gridDim.x * (64 / QL)) {
    const int k = k0 + js;
    int n = 0;
    const float* gx = nullptr;
    if (k < njobs) {
      const int4 jb = qj.jobs[(int)(qsorted[k] & 0xffffffffull)];
      n = jb.z;
      gx = qj.f + 3 * (size_t)jb.y;
    }
    const float* gy = gx + n;
    const float* gz = gy + n;
    double smax = 0.0;
    for (int i = jl; i < n; i += QL) {
      const float fx = gx[i], fy = gy[i];
      const double a[5] = {(double)(fx * fx), (double)(fy * fy), (double)(fx * fy), (double)fx, (double)fy};
      for (int j = 0; j < N; ++j) {
        A[6 * i + j] = a[j];
        smax = dmaxd2(smax, fabs(a[j]));  // the max of the non-NaN terms: any order gives it
      }
      A[6 * i + 5] = (double)gz[i];
    }
    for (int m = 1; m < QL; m <<= 1) smax = dmaxd2(smax, __shfl_xor(smax, m));
    const bool fin = isfinite(smax);
    const double scale = smax == 0.0 ? 1.0 : smax;
    const int nn = fin ? n : 0;  // the rows this job's QR walks (none: x = 0, as quad_lane_job)
    __syncthreads();
    for (int i = jl; i < nn; i += QL)
      for (int j = 0; j < N; ++j) A[6 * i + j] = A[6 * i + j] / scale;
    __syncthreads();
    if (jl < N) {
      double sq = 0.0;
      for (int i = 0; i < nn; ++i) sq += A[6 * i + jl] * A[6 * i + jl];
      sh_nd[js][jl] = sh_nu[js][jl] = sqrt(sq);
      sh_perm[js][jl] = jl;
    }
    __syncthreads();
    for (int kk = 0; kk < N; ++kk) {
      // pivot: the column of largest remaining norm (first on ties)
      int big = kk;
      for (int j = kk + 1; j < N; ++j)
        if (sh_nu[js][j] > sh_nu[js][big]) big = j;
      if (big != kk)
        for (int i = jl; i < nn; i += QL) {
          const double t = A[6 * i + kk];
          A[6 * i + kk] = A[6 * i + big];
          A[6 * i + big] = t;
        }
      __syncthreads();
      if (jl == 0 && nn) {
        if (big != kk) {
          double t = sh_nu[js][kk]; sh_nu[js][kk] = sh_nu[js][big]; sh_nu[js][big] = t;
          t = sh_nd[js][kk]; sh_nd[js][kk] = sh_nd[js][big]; sh_nd[js][big] = t;
          const int pk = sh_perm[js][kk]; sh_perm[js][kk] = sh_perm[js][big]; sh_perm[js][big] = pk;
        }
        double tail = 0.0;
        for (int i = kk + 1; i < nn; ++i) tail += A[6 * i + kk] * A[6 * i + kk];
        const double c0 = A[6 * kk + kk];
        double beta, tau = 0.0, den = 0.0;
        if (tail <= dmin) {
          beta = c0;
        } else {
          beta = sqrt(c0 * c0 + tail);
          if (c0 >= 0.0) beta = -beta;
          den = c0 - beta;
          tau = (beta - c0) / beta;
        }
        A[6 * kk + kk] = beta;
        sh_c[js][0] = tau;
        sh_c[js][1] = den;
        sh_c[js][2] = tail <= dmin ? 1.0 : 0.0;
      }
      __syncthreads();
      const double tau = sh_c[js][0], den = sh_c[js][1];
      const bool zero = sh_c[js][2] != 0.0;
      for (int i = kk + 1 + jl; i < nn; i += QL) A[6 * i + kk] = zero ? 0.0 : A[6 * i + kk] / den;
      __syncthreads();
      const bool upd = nn && tau != 0.0;
      if (upd && jl > kk && jl <= N) {  // column jl's dot product with the Householder vector
        double t = 0.0;
        for (int i = kk + 1; i < nn; ++i) t += A[6 * i + kk] * A[6 * i + jl];
        t += A[6 * kk + jl];
        A[6 * kk + jl] -= tau * t;
        sh_t[js][jl] = t;
      }
      __syncthreads();
      if (upd)
        for (int i = kk + 1 + jl; i < nn; i += QL) {
          const double v = tau * A[6 * i + kk];
          for (int j = kk + 1; j <= N; ++j) A[6 * i + j] -= v * sh_t[js][j];
        }
      __syncthreads();
      if (nn && jl > kk && jl < N) {  // norm downdate of column jl
        const double nuj = sh_nu[js][jl];
        if (nuj != 0.0) {
          double t = fabs(A[6 * kk + jl]) / nuj;
          t = (1.0 + t) * (1.0 - t);
          if (t < 0.0) t = 0.0;
          const double qq = nuj / sh_nd[js][jl];
          const double t2 = t * (qq * qq);
          if (t2 <= downdate) {
            double sq = 0.0;
            for (int i = kk + 1; i < nn; ++i) sq += A[6 * i + jl] * A[6 * i + jl];
            sh_nd[js][jl] = sh_nu[js][jl] = sqrt(sq);
          } else {
            sh_nu[js][jl] = nuj * sqrt(t);
          }
        }
      }
      __syncthreads();
    }
    // R, Q^T b and (row 5) scale (non-finite: no fit) and perm, to the job's lane-layout chunk
    if (k < njobs) {
      double* M = qj.rows + 6 * (size_t)qoff[k >> 6] + (k & 63);
      for (int e = jl; e < 36; e += QL) {
        const int i = e / 6, j = e % 6;
        double v;
        if (i < N) v = A[e];
        else if (j == 0) v = fin ? scale : smax;
        else v = (double)sh_perm[js][j - 1];
        M[(size_t)e * 64] = v;
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void quad_solve_kernel(DScene s, FilterDev F, QuadJobs qj,
                                                         const unsigned long long* __restrict__ qsorted,
                                                         const int* __restrict__ qoff, const int* __restrict__ kb_ptr,
                                                         int njobs, int* __restrict__ reject) {
  const int k = *kb_ptr + blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= njobs) return;
  const int4 jb = qj.jobs[(int)(qsorted[k] & 0xffffffffull)];
  const int n = jb.z;
  const float* gx = qj.f + 3 * (size_t)jb.y;
  const double* M = qj.rows + 6 * (size_t)qoff[k >> 6] + (k & 63);
  const double scale = M[(size_t)30 * 64];
  int perm[5];
  for (int j = 0; j < 5; ++j) perm[j] = (int)M[(size_t)(31 + j) * 64];
  quad_solve(s, F, M, perm, scale, isfinite(scale), jb.x, n, gx, gx + n, gx + 2 * n, reject);
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


// ============================================================================ expansion
// CExpand::findEmptyBlocks (expand.cpp:95-180), one wavefront per parent: the six angular
// bins around the patch that hold no neighbour (findNeighbors(patch, ., 1, 4.0f), margin 1,
// vimages included) and were not tried before (_dflag) get a candidate at `radius`.
template <int CAP>
__global__ __launch_bounds__(64) NB_WALK_ATTR void empty_blocks_kernel(DScene s, FilterDev F, const int* __restrict__ parents, int np,
                                                          float* __restrict__ cand_coord, int* __restrict__ cand_ok,
                                                          int* __restrict__ queue, int* __restrict__ overflow, NbOverflow ov) {
  __shared__ NbLdsT<CAP> L;
  const int lane = threadIdx.x;
#if defined(NB_PROFILE)
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nbp_t = NBP_NOW();
#else
  unsigned long long* prof = nullptr;
#endif
  for (;;) {
    NBP(5);
    int i = 0;
    if (lane == 0) i = atomicAdd(queue, 1);
    i = __builtin_amdgcn_readfirstlane(i);
    if (i >= (ov.only ? *ov.only_n : np)) break;
    const int k = ov.only ? __builtin_amdgcn_readfirstlane(ov.only[i]) : i;
    const pmvs_patch& q = F.P[parents[k]];
    const RadUnit ru = compute_radius_unit(s, L, q, true);
    const float radius = ru.radius;
    NBP(6);
#if defined(EBX_SKIP_WALK)  // timing experiment only (tools/eb_breakdown.sh): no neighbour walk
    const int n = 0;
    if (lane == 0) L.overflow = 0;
#else
    const int n = gather_neighbors<CAP, 1>(s, F, L, q, 4.0f, 1, 0, prof, ru);  // the radius and units computed once
#endif
#if defined(NB_PROFILE)
    nbp_t = NBP_NOW();
#endif
    // overflowed: this parent's bins are rewritten by the NB_CAP_BIG re-walk
    if (lane == 0 && L.overflow && ov.items) ov.items[atomicAdd(ov.count, 1)] = k;
    if (lane == 0 && L.overflow && !ov.items) atomicAdd(overflow, 1);
    float xdir[4] = {0, 0, 0, 0}, ydir[4] = {0, 0, 0, 0};
    const float* z = q.normal;
    if (fabs((double)z[0]) > 0.5) { xdir[0] = z[1]; xdir[1] = -z[0]; xdir[2] = 0; }
    else if (fabs((double)z[1]) > 0.5) { xdir[1] = z[2]; xdir[2] = -z[1]; xdir[0] = 0; }
    else { xdir[2] = z[0]; xdir[0] = -z[2]; xdir[1] = 0; }
    unitize4(xdir);
    ydir[0] = z[1] * xdir[2] - z[2] * xdir[1];
    ydir[1] = z[2] * xdir[0] - z[0] * xdir[2];
    ydir[2] = z[0] * xdir[1] - z[1] * xdir[0];
    const float radiuslow = __fdiv_rn(radius, 6.0f), radiushigh = radius * 2.5f;
    // fill[i] of the reference is a sum of non-negative terms compared with 0 (expand.cpp:160-176):
    // it is > 0 iff some term is > 0 and none is NaN, so the neighbours are scanned lane-parallel
    // and only those two facts per bin are reduced.
    unsigned pos = 0u, nan = 0u;
#if defined(EBX_SKIP_BIN)  // timing experiment only (tools/eb_breakdown.sh): the neighbours not binned
    for (int a = lane; a < 0; a += 64) {
#else
    for (int a = lane; a < n; a += 64) {
#endif
      float d[4];
      for (int c = 0; c < 4; ++c) d[c] = F.hot[L.nb[a]].coord[c] - q.coord[c];
      float f0 = dot4(d, xdir), f1 = dot4(d, ydir);
      const float len = (float)sqrt((double)(f0 * f0 + f1 * f1));
      if (len < radiuslow || radiushigh < len) continue;
      f0 = __fdiv_rn(f0, len);
      f1 = __fdiv_rn(f1, len);
      float angle = (float)atan2((double)f1, (double)f0);
      if (angle < 0.0) angle = (float)((double)angle + 2 * M_PI);
      const float findex = (float)((double)angle / (2 * M_PI / 6));
      const int lindex = (int)floor((double)findex);
      const int hindex = lindex + 1;
      const float t0 = (float)hindex - findex, t1 = findex - (float)lindex;
      const int b0 = ((lindex % 6) + 6) % 6, b1 = ((hindex % 6) + 6) % 6;
      if (t0 > 0.0f) pos |= 1u << b0;
      if (t0 != t0) nan |= 1u << b0;
      if (t1 > 0.0f) pos |= 1u << b1;
      if (t1 != t1) nan |= 1u << b1;
    }
    for (int d = 32; d >= 1; d >>= 1) {
      pos |= __shfl_xor(pos, d);
      nan |= __shfl_xor(nan, d);
    }
    if (lane == 0) {
      for (int i = 0; i < 6; ++i) {
        int ok = 1;
        if ((pos >> i & 1u) && !(nan >> i & 1u)) ok = 0;  // 0.0f < fill[i]
        if (q.dflag & (0x0001 << i)) ok = 0;
        cand_ok[6 * k + i] = ok;
        if (ok) {
          // expand.cpp:176-177: the angle is stored as float, then cos/sin run in double.
          const float angle = (float)(2 * M_PI * i / 6);
          const double cr = cos((double)angle) * (double)radius, sr = sin((double)angle) * (double)radius;
          for (int c = 0; c < 4; ++c)
            cand_coord[4 * (6 * k + i) + c] = (q.coord[c] + (float)((double)xdir[c] * cr)) + (float)((double)ydir[c] * sr);
        }
      }
    }
    __syncthreads();
  }
  NBP_FLUSH(1);
}

// findEmptyBlocks' re-walk of the parents whose neighbour set overflowed the NB_CAP walk (round 5:
// replaces the NB_CAP_BIG form, whose 16 384-entry LDS buffer could overflow in its turn on dense
// 8K clusters).  fill[] of the reference (expand.cpp:160-176) only needs, per angular bin, whether
// some term is > 0 and whether one is NaN; neither depends on the order of the neighbour list or on
// duplicates in it, so this walk bins each neighbour as it meets it: no buffer, no sort, no
// capacity.  As the only walk it measured 10 % slower (duplicates re-tested, 146 registers, branch
// exp-stream-walks); as the re-walk of a few parents its speed does not matter.
__device__ __forceinline__ void eb_bin(const float* hc, const float* qc, const float* xdir, const float* ydir, float rlow,
                                       float rhigh, unsigned& pos, unsigned& nan) {
  float d[4];
  for (int c = 0; c < 4; ++c) d[c] = hc[c] - qc[c];
  float f0 = dot4(d, xdir), f1 = dot4(d, ydir);
  const float len = (float)sqrt((double)(f0 * f0 + f1 * f1));
  if (len < rlow || rhigh < len) return;
  f0 = __fdiv_rn(f0, len);
  f1 = __fdiv_rn(f1, len);
  float angle = (float)atan2((double)f1, (double)f0);
  if (angle < 0.0) angle = (float)((double)angle + 2 * M_PI);
  const float findex = (float)((double)angle / (2 * M_PI / 6));
  const int lindex = (int)floor((double)findex);
  const int hindex = lindex + 1;
  const float t0 = (float)hindex - findex, t1 = findex - (float)lindex;
  const int b0 = ((lindex % 6) + 6) % 6, b1 = ((hindex % 6) + 6) % 6;
  if (t0 > 0.0f) pos |= 1u << b0;
  if (t0 != t0) nan |= 1u << b0;
  if (t1 > 0.0f) pos |= 1u << b1;
  if (t1 != t1) nan |= 1u << b1;
}

__global__ __launch_bounds__(64) NB_WALK_ATTR void empty_blocks_stream_kernel(DScene s, FilterDev F, const int* __restrict__ parents,
                                                                              float* __restrict__ cand_coord, int* __restrict__ cand_ok,
                                                                              int* __restrict__ queue, NbOverflow ov) {
  __shared__ NbSmall L;
  const int lane = threadIdx.x;
  constexpr int margin = 1;
  for (;;) {
    int i = 0;
    if (lane == 0) i = atomicAdd(queue, 1);
    i = __builtin_amdgcn_readfirstlane(i);
    if (i >= *ov.only_n) break;
    const int pk = __builtin_amdgcn_readfirstlane(ov.only[i]);  // an overflowed parent of the NB_CAP walk
    const pmvs_patch& q = F.P[parents[pk]];
    const float radius = compute_radius_wave(s, L, q);
    float xdir[4] = {0, 0, 0, 0}, ydir[4] = {0, 0, 0, 0};
    const float* z = q.normal;
    if (fabs((double)z[0]) > 0.5) { xdir[0] = z[1]; xdir[1] = -z[0]; xdir[2] = 0; }
    else if (fabs((double)z[1]) > 0.5) { xdir[1] = z[2]; xdir[2] = -z[1]; xdir[0] = 0; }
    else { xdir[2] = z[0]; xdir[0] = -z[2]; xdir[1] = 0; }
    unitize4(xdir);
    ydir[0] = z[1] * xdir[2] - z[2] * xdir[1];
    ydir[1] = z[2] * xdir[0] - z[0] * xdir[2];
    ydir[2] = z[0] * xdir[1] - z[1] * xdir[0];
    const float radiuslow = __fdiv_rn(radius, 6.0f), radiushigh = radius * 2.5f;
    // findNeighbors(patch, ., 1, 4.0f) (patchOrganizerS.cpp:527-631) as in gather_neighbors: the
    // cells NB_SK per lane per round, their entries NB_NE per lane at a time
    const int ni = uni(q.num_images);
    const float nradius = (float)(1.5 * margin * (double)radius);
    float unit = 0.0f;
    for (int k = 0; k < ni; ++k) unit += get_unit(s, s.views[q.images[k]], q.coord);
    unit = __fdiv_rn(unit, (float)ni);
    unit *= (float)s.csize;
    const float thr = 0.5f * 4.0f;
    const int nlists = ni + uni(q.num_vimages);
    constexpr int side = 2 * margin + 1, per_list = side * side * 2;
    const int nslots = nlists * per_list;
    unsigned pos = 0u, nan = 0u;
    for (int base = 0; base < nslots; base += 64 * NB_SK) {
      int bk[NB_SK], ck[NB_SK], hk[NB_SK];
#pragma unroll
      for (int k = 0; k < NB_SK; ++k) {
        const int slot = base + k * 64 + lane;
        int b = 0, e = 0, lst = 0, head = -1;
        if (slot < nslots) {
          const int li = slot / per_list;
          int r = slot - li * per_list;
          const int dyi = r / (2 * side);
          r -= dyi * 2 * side;
          const int dxi = r >> 1;
          lst = r & 1;
          const bool vis = li >= ni;
          const int t = vis ? q.vimages[li - ni] : q.images[li];
          if (t < s.tnum) {
            const int gw = gwidth(s, t), gh = gheight(s, t);
            const int yt = (vis ? q.vgrids[li - ni][1] : q.grids[li][1]) + dyi - margin;
            const int xt = (vis ? q.vgrids[li - ni][0] : q.grids[li][0]) + dxi - margin;
            if (0 <= yt && yt < gh && 0 <= xt && xt < gw) {
              const long long c = F.tgoff[t] + (long long)yt * gw + xt;
              const int* off = lst ? F.vp_off : F.pg_off;
              const int lim = lst ? F.nvp : F.npg;
              b = off[c];
              e = off[c + 1];
              if (b < 0 || e > lim || b > e) {
                atomicAdd(&F.err[0], 1);
                atomicExch(&F.err[1], 12 + lst);
                b = 0;
                e = 0;
              }
              if (F.pg_dhead) head = (lst ? F.vp_dhead : F.pg_dhead)[c];
            }
          }
        }
        bk[k] = b | (lst << 31);
        ck[k] = e - b;
        hk[k] = head;
      }
      int mine = 0;
#pragma unroll
      for (int k = 0; k < NB_SK; ++k) mine += ck[k];
      const int offl = wave_excl_scan_w(mine);
      const int tot = uni(__shfl(offl + mine, 63));
      {
        int o = offl;
#pragma unroll
        for (int k = 0; k < NB_SK; ++k) {
          L.sb[lane * NB_SK + k] = bk[k];
          L.so[lane * NB_SK + k] = o;
          o += ck[k];
        }
      }
      __syncthreads();
      for (int ib = 0; ib < tot; ib += 64 * NB_NE) {
        int jv[NB_NE];
#pragma unroll
        for (int u = 0; u < NB_NE; ++u) {
          const int idx = ib + u * 64 + lane;
          jv[u] = -1;
          if (idx < tot) {
            int sidx = 0;  // the last slot whose offset is <= idx (it holds idx)
            for (int step = 64 * NB_SK / 2; step >= 1; step >>= 1)
              if (sidx + step < 64 * NB_SK && L.so[sidx + step] <= idx) sidx += step;
            const int sb = L.sb[sidx];
            const int fi = (sb & 0x7fffffff) + idx - L.so[sidx];
            jv[u] = ((sb < 0) ? F.vp_items : F.pg_items)[fi];
          }
        }
#pragma unroll
        for (int u = 0; u < NB_NE; ++u) {
          const int j = jv[u];
          if (ib + u * 64 + lane >= tot) continue;
          if (j < 0 || j >= F.n) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 14); continue; }
          const PHot& h = F.hot[j];
          if (is_neighbor_h(q, h, unit, thr, nradius, true)) eb_bin(h.coord, q.coord, xdir, ydir, radiuslow, radiushigh, pos, nan);
        }
      }
      // entries committed by earlier expansion waves (short chains, walked per lane)
#pragma unroll
      for (int k = 0; k < NB_SK; ++k)
        for (int ent = hk[k]; ent >= 0;) {
          const int2 en = F.d_ent[ent];
          ent = en.y;
          const int j = en.x;
          if (j < 0 || j >= F.n) { atomicAdd(&F.err[0], 1); atomicExch(&F.err[1], 15); continue; }
          const PHot& h = F.hot[j];
          if (is_neighbor_h(q, h, unit, thr, nradius, true)) eb_bin(h.coord, q.coord, xdir, ydir, radiuslow, radiushigh, pos, nan);
        }
      __syncthreads();
    }
    for (int d = 32; d >= 1; d >>= 1) {
      pos |= __shfl_xor(pos, d);
      nan |= __shfl_xor(nan, d);
    }
    if (lane == 0) {
      for (int b = 0; b < 6; ++b) {
        int ok = 1;
        if ((pos >> b & 1u) && !(nan >> b & 1u)) ok = 0;  // 0.0f < fill[b]
        if (q.dflag & (0x0001 << b)) ok = 0;
        cand_ok[6 * pk + b] = ok;
        if (ok) {
          // expand.cpp:176-177: the angle is stored as float, then cos/sin run in double.
          const float angle = (float)(2 * M_PI * b / 6);
          const double cr = cos((double)angle) * (double)radius, sr = sin((double)angle) * (double)radius;
          for (int c = 0; c < 4; ++c)
            cand_coord[4 * (6 * pk + b) + c] = (q.coord[c] + (float)((double)xdir[c] * cr)) + (float)((double)ydir[c] * sr);
        }
      }
    }
    __syncthreads();
  }
}

// CExpand::expandSub up to the refine (expand.cpp:200-226), one thread per candidate slot:
// setGridsImages from the parent's images, mask / bimages, checkCounts, removeImagesEdge.
// status: -1 no candidate, 1 rejected, 0 goes to preProcess (pmvs_candidate written).
__global__ void prepare_kernel(DScene s, FilterDev F, const unsigned char* __restrict__ counts, const int* __restrict__ parents,
                               int np, const float* __restrict__ cand_coord, const int* __restrict__ cand_ok,
                               pmvs_candidate* __restrict__ cout_all, pmvs_patch* __restrict__ prep_all,
                               int* __restrict__ status, int cthr, int only, const int* __restrict__ cidx) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= np * 6) return;
  if (!cand_ok[slot] || (only >= 0 && slot != only)) { status[slot] = -1; return; }
  // candidate and prepared-patch records exist for the free directions only (compact index)
  const int ci = cidx[slot];
  const pmvs_patch& par = F.P[parents[slot / 6]];
  float coord[4];
  for (int c = 0; c < 4; ++c) coord[c] = cand_coord[4 * slot + c];
  pmvs_patch& q = prep_all[ci];
  for (int c = 0; c < 4; ++c) { q.coord[c] = coord[c]; q.normal[c] = par.normal[c]; }
  int ni = 0;
  for (int k = 0; k < par.num_images; ++k) {  // setGridsImages (patchOrganizerS.cpp:383-399)
    const int t = par.images[k];
    float ic[3];
    project(s.views[t], coord, s.level, ic);
    const int ix = ((int)floorf(ic[0] + 0.5f)) / s.csize;
    const int iy = ((int)floorf(ic[1] + 0.5f)) / s.csize;
    if (0 <= ix && ix < gwidth(s, t) && 0 <= iy && iy < gheight(s, t)) {
      q.images[ni] = (int16_t)t;
      q.grids[ni][0] = (int16_t)ix;  // in the grid: fits
      q.grids[ni][1] = (int16_t)iy;
      ni++;
    }
  }
  q.num_images = ni;
  int st = 0;
  if (ni == 0) st = 1;
  if (!st) {
    bool bad = false;
    if (s.anyMask)
      for (int v = 0; v < s.num; ++v)
        if (get_mask(s, s.views[v], coord, s.level) == 0) bad = true;
    for (int b = 0; b < s.nb; ++b) {
      const DView& v = s.views[s.bindexes[b]];
      float ic[3];
      project(v, coord, s.level, ic);
      if (ic[0] < 0.0f || (float)(v.w[s.level] - 1) < ic[0] || ic[1] < 0.0f || (float)(v.h[s.level] - 1) < ic[1]) bad = true;
    }
    if (bad) st = 1;
  }
  if (!st) {  // checkCounts (expand.cpp:268-323)
    int full = 0, empty = 0;
    for (int k = 0; k < ni; ++k) {
      const int t = q.images[k];
      if (s.tnum <= t) continue;
      const long long c = F.tgoff[t] + (long long)q.grids[k][1] * gwidth(s, t) + q.grids[k][0];
      if (F.pg_off[c + 1] > F.pg_off[c] || (F.pg_dhead && F.pg_dhead[c] >= 0)) { ++full; continue; }
      if (cthr <= counts[c]) ++full;
      else ++empty;
    }
    if (s.depth <= 1) { if (empty < s.minImageNum && full != 0) st = 1; }
    else if (empty < s.minImageNum - 1 && full != 0) st = 1;
  }
  int ne = 0;
  if (!st) {  // removeImagesEdge (optim.cpp:384-396)
    for (int k = 0; k < ni; ++k)
      if (get_edge(s, s.views[q.images[k]], coord, s.level)) cout_all[ci].images[ne++] = q.images[k];
    if (ne == 0) st = 1;
  }
  status[slot] = st;
  if (!st) {
    for (int c = 0; c < 4; ++c) { cout_all[ci].coord[c] = coord[c]; cout_all[ci].normal[c] = par.normal[c]; }
    cout_all[ci].dscale = 0.0f;
    cout_all[ci].num_images = ne;
  }
}

// COptim::postProcess depth >= 1 steps (optim.cpp:178-188) on refined candidates, one wavefront
// each: setVImagesVGrids against the model's depth maps and, at depth >= 2, check() =
// computeGain + findNeighbors(patch, ., 1, 4, 2) + filterQuad.  out_status: 0 accepted,
// 2 preProcess failed, 3 postProcess failed.
template <int CAP>
__global__ __launch_bounds__(64) NB_WALK_ATTR void depth_post_kernel(DScene s, FilterDev F, const pmvs_refined* __restrict__ res,
                                                        int m, pmvs_patch* __restrict__ outp, int* __restrict__ out_status,
                                                        double* __restrict__ scratch, int* __restrict__ queue,
                                                        int* __restrict__ overflow, NbOverflow ov) {
  __shared__ NbLdsT<CAP> L;
  __shared__ pmvs_patch Q;  // the patch is built in LDS and stored once (no global read-back)
  const int lane = threadIdx.x;
  double* M = scratch + (size_t)blockIdx.x * (CAP * 8);
  double* r = M + (size_t)CAP * 5;
  for (;;) {
    int i = 0;
    if (lane == 0) i = atomicAdd(queue, 1);
    i = __builtin_amdgcn_readfirstlane(i);
    if (i >= (ov.only ? *ov.only_n : m)) break;
    const int k = ov.only ? __builtin_amdgcn_readfirstlane(ov.only[i]) : i;
    const pmvs_refined& rr = res[k];
    pmvs_patch& q = Q;
    // wave-uniform (SGPR) status: the branch below holds barriers, so it must not be divergent
    // No `continue` out of a lane-divergent region anywhere in this loop: lanes that leave early
    // are not guaranteed to reconverge with lane 0 before the next ticket is broadcast.
    const int rstatus = uni(rr.status);
    int st = (rstatus == PMVS_FAIL_POST) ? 3 : 2;
    // an error for the run, never a reject.  The re-walk pass (ov.only: candidates whose neighbour list
    // overflowed NB_CAP) runs the whole body again, so the overflow counts are taken in the first pass only
    if (rstatus == PMVS_FAIL_OVERFLOW && lane == 0 && !ov.only) atomicAdd(overflow, 1);
    if (rstatus == PMVS_ACCEPTED) {
    st = 0;
    if (lane == 0) {
      for (int c = 0; c < 4; ++c) { q.coord[c] = rr.coord[c]; q.normal[c] = rr.normal[c]; }
      q.ncc = rr.ncc; q.dscale = rr.dscale; q.ascale = rr.ascale; q.tmp = rr.tmp; q.timages = rr.timages;
      q.flag = 1; q.fix = 0; q.dflag = 0; q.num_images = rr.num_images; q.num_vimages = 0;
    }
    for (int e = lane; e < PMVS_MAX_IMAGES; e += 64) {
      q.images[e] = (int16_t)((e < rr.num_images) ? rr.images[e] : 0);
      q.grids[e][0] = grid16((e < rr.num_images) ? rr.grids[e][0] : 0);
      q.grids[e][1] = grid16((e < rr.num_images) ? rr.grids[e][1] : 0);
      q.vimages[e] = 0;
      q.vgrids[e][0] = 0;
      q.vgrids[e][1] = 0;
    }
    __syncthreads();
    if (s.depth) {
      // setVImagesVGrids (patchOrganizerS.cpp:429-459): lane t tests target image t
      bool take = false;
      int ix = 0, iy = 0;
      for (int base = 0; base < s.tnum; base += 64) {
        const int t = base + lane;
        take = false;
        if (t < s.tnum) {
          bool used = false;
          for (int i = 0; i < q.num_images; ++i)
            if (q.images[i] == t) used = true;
          if (!used) {
            float ic[3];
            project(s.views[t], q.coord, s.level, ic);
            ix = ((int)floorf(ic[0] + 0.5f)) / s.csize;
            iy = ((int)floorf(ic[1] + 0.5f)) / s.csize;
            take = is_visible_q(s, F, q, t, ix, iy, 0.5f) && get_edge(s, s.views[t], q.coord, s.level);
          }
        }
        const unsigned long long mask = __ballot(take);
        const int pos = __popcll(mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        const int nv = q.num_vimages;
        __syncthreads();
        if (take && nv + pos < PMVS_MAX_IMAGES) {
          q.vimages[nv + pos] = (int16_t)t;
          q.vgrids[nv + pos][0] = grid16(ix);
          q.vgrids[nv + pos][1] = grid16(iy);
        }
        __syncthreads();
        // more than PMVS_MAX_IMAGES visible targets: counted as an overflow (the run fails), never clamped silently
        if (lane == 0 && !ov.only && nv + __popcll(mask) > PMVS_MAX_IMAGES) atomicAdd(overflow, 1);
        if (lane == 0) q.num_vimages = imin(PMVS_MAX_IMAGES, nv + __popcll(mask));
        __syncthreads();
      }
      if (2 <= s.depth) {
        // COptim::check (optim.cpp:363-381): computeGain (filter.cpp:88-146) ...
        const int ne = uni(q.num_images + q.num_vimages);
        const float u0 = get_unit(s, s.views[q.images[0]], q.coord);
        if (lane == 0) L.f[2] = (double)(smax(0.0f, q.ncc - s.nccThreshold) * (float)q.timages);
        for (int base = 0; base < ne; base += 64) {
          const int en = base + lane;
          float maxp = 0.0f;
          if (en < ne) {
            const bool vis = en >= q.num_images;
            const int t = vis ? q.vimages[en - q.num_images] : q.images[en];
            if (t < s.tnum) {
              const int gx = vis ? q.vgrids[en - q.num_images][0] : q.grids[en][0];
              const int gy = vis ? q.vgrids[en - q.num_images][1] : q.grids[en][1];
              const long long c = F.tgoff[t] + (long long)gy * gwidth(s, t) + gx;
              const float pdepth = depth_of(s.views[t], q.coord);
              const int eb = F.pg_off[c], ee = F.pg_off[c + 1];
              for (int e = eb, ent = F.pg_dhead ? F.pg_dhead[c] : -1; e < ee || ent >= 0;) {
                int j;
                if (e < ee) j = F.pg_items[e++];
                else { const int2 en = F.d_ent[ent]; j = en.x; ent = en.y; }
                const PHot& hj = F.hot[j];
                if (vis && !(pdepth < depth_of(s.views[t], hj.coord))) continue;
                const float hunit = (float)((double)(u0 + hj.unit0) / 2.0 * s.csize);
                if (!is_neighbor_h(q, hj, hunit, 1.0f, 0.0f, false)) maxp = smax(maxp, hj.ncc - s.nccThreshold);
              }
            }
          }
          L.units[lane] = maxp;
          __syncthreads();
          if (lane == 0) {
            float gain = (float)L.f[2];
            for (int i = 0; i < 64 && base + i < ne; ++i) gain -= L.units[i];
            L.f[2] = (double)gain;
          }
          __syncthreads();
        }
        if (lane == 0) q.tmp = (float)L.f[2];
        __syncthreads();
        if (uni_f((float)L.f[2]) < 0.0f) {
          st = 3;
        } else {
          // ... findNeighbors(patch, neighbors, 1, 4, 2) + filterQuad when more than 6 neighbours
          const int n = gather_neighbors<CAP, 2>(s, F, L, q, 4.0f, 2, 0);
          // overflowed: candidate k is rewritten by the NB_CAP_BIG re-walk
          if (lane == 0 && L.overflow && ov.items) ov.items[atomicAdd(ov.count, 1)] = k;
          if (lane == 0 && L.overflow && !ov.items) atomicAdd(overflow, 1);
          if (6 < n && filter_quad_wave(s, F, L, M, r, q, n)) st = 3;
        }
      }
    }
    const unsigned* src = reinterpret_cast<const unsigned*>(&Q);
    unsigned* dst = reinterpret_cast<unsigned*>(&outp[k]);
    for (int w = lane; w < (int)(sizeof(pmvs_patch) / 4); w += 64) dst[w] = src[w];
    }
    if (lane == 0) out_status[k] = st;
    __syncthreads();
  }
}

// CPatchOrganizerS::addPatch of the committed patches (patchOrganizerS.cpp:308-381): registration
// bits and depth-map updates; rank codes are larger than every loaded patch's, so equal depths
// keep the older patch as the reference's strict "depth < dtmp".
struct DeltaLists {  // the per-cell chains of FilterDev (expansion), writable
  int* pg_head;
  int* vp_head;
  int2* ent;  // {item, next}
};

__global__ void add_patches_kernel(DScene s, FilterDev F, int first, int count, int rank0, Reg* __restrict__ preg,
                                   Reg* __restrict__ vreg, int* __restrict__ order,
                                   unsigned long long* __restrict__ dpkey, PHot* __restrict__ hot) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)count * s.tnum) return;
  const int k = (int)(g / s.tnum), t = (int)(g - (long long)k * s.tnum);
  const int p = first + k;
  const pmvs_patch& q = F.P[p];
  if (t == 0) {
    Reg m = reg_zero();
    for (int i = 0; i < q.num_images; ++i)
      if (q.images[i] < s.tnum && in_grid(s, q.images[i], q.grids[i][0], q.grids[i][1])) reg_set(m, i);
    preg[p] = m;
    vreg[p] = reg_first(q.num_vimages);
    order[rank0 + k] = p;
    write_hot(s, q, hot[p]);
  }
  if (s.depth == 0) return;  // addPatch keeps no depth maps at depth 0 (patchOrganizerS.cpp:331)
  const DView& v = s.views[t];
  float ic[3];
  project(v, q.coord, s.level, ic);
  const float fx = __fdiv_rn(ic[0], (float)s.csize), fy = __fdiv_rn(ic[1], (float)s.csize);
  const int xs[2] = {(int)floor((double)fx), (int)ceil((double)fx)};
  const int ys[2] = {(int)floor((double)fy), (int)ceil((double)fy)};
  const unsigned long long key = ((unsigned long long)depth_bits(depth_of(v, q.coord)) << 32) | (unsigned)(rank0 + k);
  const int gw = gwidth(s, t), gh = gheight(s, t);
  for (int j = 0; j < 2; ++j)
    for (int i = 0; i < 2; ++i) {
      if (xs[i] < 0 || gw <= xs[i] || ys[j] < 0 || gh <= ys[j]) continue;
      unsigned long long* cell = &dpkey[F.tgoff[t] + (long long)ys[j] * gw + xs[i]];
      if (key < *cell) atomicMin(cell, key);  // as depth_map_kernel: a value <= key cannot change
    }
}

// addPatch's cell registrations of the committed patches into the per-cell chains (pgrids: the
// in-grid target images; vpgrids: the vimages), one wavefront per patch, straight from its commit
// record; entry slots eoff[k].. are assigned by the host (no shared allocation counter).
__global__ __launch_bounds__(64) void register_kernel(DeltaLists D, const int* __restrict__ acc, const int* __restrict__ eoff,
                                                      int nacc, int first, const int* __restrict__ rec, int rec_ints) {
  const int k = blockIdx.x;
  if (k >= nacc) return;
  const int* r = rec + (size_t)acc[k] * rec_ints;
  const int ni = r[3], nv = r[4];
  for (int i = threadIdx.x; i < ni + nv; i += 64) {
    const int e = eoff[k] + i;
    const bool vis = i >= ni;
    const int cell = vis ? r[5 + 2 * PMVS_MAX_IMAGES + (i - ni)] : r[5 + PMVS_MAX_IMAGES + i];
    const int nx = atomicExch(&(vis ? D.vp_head : D.pg_head)[cell], e);  // readers are later kernels
    D.ent[e] = make_int2(first + k, nx);
  }
}

__global__ void flag_rank_kernel(pmvs_patch* __restrict__ P, const int* __restrict__ order, int na) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < na) P[order[k]].flag = k;
}

// ============================================================================ host orchestration
// PMVS_TRACE_ERRORS=1: the first failing call of a pass is reported with its line and the free
// device memory (diagnosis of capacity / allocation failures at full scale)
static void trace_error(hipError_t e, int line) {
  static const bool on = getenv("PMVS_TRACE_ERRORS") != nullptr;
  if (!on) return;
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  fprintf(stderr, "[pmvs] pmvs_filter.hip:%d: %s (device memory free %.2f of %.2f GB)\n", line, hipGetErrorString(e),
          fr / 1e9, tot / 1e9);
}
#define FCHK(x)                          \
  do {                                   \
    hipError_t e_ = (x);                 \
    if (e_ != hipSuccess) {              \
      trace_error(e_, __LINE__);         \
      return e_;                         \
    }                                    \
  } while (0)

static inline unsigned nblk(long long n, int b = 256) { return (unsigned)((n + b - 1) / b); }
// The (cell << 32 | index) keys of the list builds, the collect order and the commit are written in
// index order, and hipcub's radix sort is stable: sorting only the cell bits [32, 32 + cell_bits)
// gives the full 64-bit order (ties by index = input order) in about half the passes.  2^cell_bits
// > ncells, so the collect's dead-patch keys (~0) still sort after every cell.
static int cell_bits(long long ncells) {
  int b = 1;
  while (b < 31 && (1ll << b) <= ncells) ++b;
  return b;
}
static int dm_tpt() {  // depth_map_kernel's targets per thread (PMVS_DM_TARGETS; 4: r05x, 134 -> 121 ms per C3 step)
  static const int v = getenv("PMVS_DM_TARGETS") ? std::max(1, std::min(16, atoi(getenv("PMVS_DM_TARGETS")))) : 4;
  return v;
}
// a grid for the XCD-remapped kernels (xcd_block): nblk rounded up to a multiple of the XCD count
static inline unsigned xcd_grid(long long n, int b = 256) { return (nblk(n, b) + kXcds - 1) / kXcds * kXcds; }

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
  const hipError_t e = hipMalloc((void**)&p, (n ? n : 1) * sizeof(T));
  if (e == hipSuccess) poison_alloc(p, (n ? n : 1) * sizeof(T));
  return e;
}

FilterBuffers::~FilterBuffers() {
  void* ps[] = {preg, vreg, tgoff, cnt, off, keys, keys2, cellcnt, pg_off, pg_items, vp_off, vp_items, dpkey,
                order, rank, hot, flags, safe, need, list, scratch, counters, temp, edge_off, edges, rbits, coordc,
                qf, qrows, qjobs, qctr, qkeys, qkeys2, qcrows, qoff, vrows, used, normalc, refpos, xr, ovf_items,
                scratch_big};
  for (void* p : ps)
    if (p) (void)hipFree(p);
}

void FilterBuffers::release() {
  this->~FilterBuffers();
  new (this) FilterBuffers();
}

hipError_t FilterBuffers::reserve(int n_, long long ncells_, int tnum_, int grid_) {
  if (n_ <= cap_n && ncells_ <= cap_cells && grid_ <= cap_grid) return hipSuccess;
  // 25 % headroom: the next loop iteration's expansion reserves its model plus a few waves, so an exact
  // capacity would free and reallocate every per-patch buffer (GBs) once per iteration
  cap_n = std::max(n_ + n_ / 4, cap_n);
  cap_cells = std::max(ncells_, cap_cells);
  cap_grid = std::max(grid_, cap_grid);
  // cell-list entries: about 16 per patch to start with (a C3 patch registers ~10-17), grown by
  // ensure_entries to what build_lists counts -- not cap_n x PMVS_MAX_IMAGES
  cap_e = std::max(cap_e, (size_t)cap_n * 16);
  cap_pi = cap_vi = cap_e;
  const size_t ne = cap_e;
  FCHK(dalloc(preg, cap_n)); FCHK(dalloc(vreg, cap_n)); FCHK(dalloc(tgoff, PMVS_MAX_TARGETS + 1));
  FCHK(dalloc(cnt, cap_n + 1)); FCHK(dalloc(off, cap_n + 1));
  FCHK(dalloc(keys, std::max(ne, (size_t)cap_n))); FCHK(dalloc(keys2, std::max(ne, (size_t)cap_n)));
  FCHK(dalloc(cellcnt, cap_cells + 1)); FCHK(dalloc(pg_off, cap_cells + 1)); FCHK(dalloc(vp_off, cap_cells + 1));
  FCHK(dalloc(pg_items, ne)); FCHK(dalloc(vp_items, ne)); FCHK(dalloc(dpkey, cap_cells));
  FCHK(dalloc(coordc, cap_n));
  FCHK(dalloc(order, cap_n)); FCHK(dalloc(rank, cap_n)); FCHK(dalloc(hot, cap_n)); FCHK(dalloc(flags, cap_n));
  FCHK(dalloc(safe, cap_n)); FCHK(dalloc(need, cap_n)); FCHK(dalloc(list, cap_n));
  FCHK(dalloc(scratch, (size_t)cap_grid * NB_SCR)); FCHK(dalloc(counters, 16));
  FCHK(dalloc(edge_off, cap_n + 1));
  // deferred filterQuad fits: up to 48 rows per patch on average, at most 2^27 rows (7.5 GB);
  // patches past the capacity are fitted in neighbor_kernel itself
  // quad_lane_kernel's row pool: jobs sorted by descending n, so the 64-lane chunks' rows
  // (64 x their first n) sum to at most every job's n plus 64 x NB_CAP
  cap_qrows = std::min((size_t)cap_n * 48, (size_t)1 << 27);
  FCHK(dalloc(qf, cap_qrows * 3)); FCHK(dalloc(qrows, (cap_qrows + 64 * (size_t)NB_CAP) * 6)); FCHK(dalloc(qjobs, cap_n));
  FCHK(dalloc(qctr, 3)); FCHK(dalloc(qkeys, cap_n)); FCHK(dalloc(qkeys2, cap_n));
  FCHK(dalloc(qcrows, cap_n / 64 + 2)); FCHK(dalloc(qoff, cap_n / 64 + 2));
  size_t t1 = 0, t2 = 0;
  FCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, keys, keys2, (int)ne));
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, cellcnt, pg_off, (int)(cap_cells + 1)));
  size_t t3 = 0;
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t3, cnt, off, cap_n + 1));
  size_t t4 = 0;
  FCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, t4, qkeys, qkeys2, cap_n, 0, 43));
  temp_bytes = std::max(std::max(t1, t4), std::max(t2, t3));
  if (temp) (void)hipFree(temp);
  temp = nullptr;
  FCHK(hipMalloc(&temp, temp_bytes ? temp_bytes : 1));
  return hipSuccess;
}

// Grows the cell-list entry buffers (and the sort's temp storage) to e entries; the other per-patch
// buffers keep their size.
hipError_t FilterBuffers::ensure_entries(size_t e, int vis) {
  size_t& ci = vis ? cap_vi : cap_pi;
  if (e > ci) {  // only the list being built: the other one's items stay valid
    ci = std::max(e, ci + ci / 2);
    FCHK(dalloc(vis ? vp_items : pg_items, ci));
  }
  if (e <= cap_e) return hipSuccess;
  cap_e = std::max(e, cap_e + cap_e / 2);
  const size_t ne = std::max(cap_e, (size_t)cap_n);
  FCHK(dalloc(keys, ne)); FCHK(dalloc(keys2, ne));
  size_t t1 = 0;
  FCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, keys, keys2, (int)ne));
  if (t1 > temp_bytes) {
    if (temp) (void)hipFree(temp);
    temp = nullptr;
    temp_bytes = t1;
    FCHK(hipMalloc(&temp, temp_bytes));
  }
  return hipSuccess;
}

template <class T>
static hipError_t fgrow(T*& p, size_t& cap, size_t need) {  // grown, contents not kept
  if (need <= cap && p) return hipSuccess;
  need = std::max(need, cap + cap / 4);
  FCHK(dalloc(p, need));
  cap = need;
  return hipSuccess;
}

// The neighbour walks' re-walk lists (NbOverflow): the NB_CAP walk appends its overflowed items to
// B.ovf_items (count at B.counters[10]); the NB_CAP_BIG form, launched right after it without a host
// sync (its workgroups leave at once when the list is empty), walks them (queue B.counters[11]).
static hipError_t nb_overflow_lists(FilterBuffers& B, size_t items, hipStream_t st, NbOverflow& walk, NbOverflow& rewalk) {
  FCHK(fgrow(B.ovf_items, B.cap_ovf, std::max<size_t>(items, 1)));
  if (!B.scratch_big) FCHK(hipMalloc((void**)&B.scratch_big, (size_t)NB_GRID_BIG * NB_CAP_BIG * 8 * sizeof(double)));
  FCHK(hipMemsetAsync(B.counters + 10, 0, 2 * sizeof(int), st));
  walk = NbOverflow{};
  walk.items = B.ovf_items;
  walk.count = B.counters + 10;
  rewalk = NbOverflow{};
  rewalk.only = B.ovf_items;
  rewalk.only_n = B.counters + 10;
  return hipSuccess;
}

namespace {

// All-gather of one owner-partitioned filter stage (see filter_pass_impl).
using FilterXchg = std::function<hipError_t(int value, const void* dsend, size_t bytes, void* drecv, long long* vsum)>;

struct Ctx {
  const DScene& s;
  FilterBuffers& B;
  pmvs_patch* P;
  int n;
  long long ncells;
  int grid;
  hipStream_t st;
  int rank = 0, world = 1;  // owner partition of the target images (world > 1: xchg is set)
  FilterXchg xchg;
  int nalive = 0, npg = 0, nvp = 0;
  const int *pg_dhead = nullptr, *vp_dhead = nullptr;
  const int2* d_ent = nullptr;
  const float4* coordc = nullptr;
  FilterDev dev() const {
    FilterDev F{};
    F.P = P; F.n = n; F.preg = B.preg; F.vreg = B.vreg; F.tgoff = B.tgoff; F.tnum = s.tnum;
    F.pg_off = B.pg_off; F.pg_items = B.pg_items; F.vp_off = B.vp_off; F.vp_items = B.vp_items;
    F.dpkey = B.dpkey; F.order = B.order; F.rank = B.rank; F.nalive = nalive; F.hot = B.hot;
    F.ncells = ncells; F.npg = npg; F.nvp = nvp; F.err = B.counters + 6; F.lovf = B.counters + 8;
    F.pg_dhead = pg_dhead; F.vp_dhead = vp_dhead; F.d_ent = d_ent;
    F.coordc = coordc;
    const char* sc = getenv("PMVS_NB_SOFTCAP");
    F.nb_softcap = sc ? atoi(sc) : 0;
    return F;
  }
};

// Device -> host reads of the loop's control values (counts, flags, per-wave status) through a
// pinned staging buffer.  Into pageable memory every hipMemcpyAsync is a staged copy with a wait of
// its own (about 75 us each between the C3 loop's kernels, profiles/r04h_kernel_trace gaps); here the
// reads of one point share one stream synchronisation.  Reads above kStageMax bytes go to their
// destination directly (bandwidth-bound anyway).
struct D2H {
  void* h;
  const void* d;
  size_t bytes;
};
constexpr size_t kStageMax = 256 << 10;
// Several small reads are first gathered on the device into one buffer by one kernel, so they cost
// one copy: each further hipMemcpyAsync was a blit of its own, about 64 us apart (r04m trace).
constexpr int kGatherMax = 8;
constexpr size_t kGatherBytes = 1024;  // per item (whole 4-byte words)
// The staging buffers belong to the stream they are used on, i.e. to one scene on one device (the
// gather buffer is device memory of the stream's device).  They are created on the stream's first
// read and freed by d2h_stage_release when the scene is destroyed (pmvs_scene_destroy), so a thread
// that drives scenes on two GPUs never gathers into another device's memory, and exiting threads
// leave nothing behind.
struct D2HStage {
  PinnedBuf pin;
  unsigned* dgather = nullptr;
};
static std::mutex g_stage_mu;
static std::unordered_map<hipStream_t, D2HStage*> g_stages;
static D2HStage& stage_for(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  D2HStage*& p = g_stages[st];
  if (!p) p = new D2HStage();
  return *p;
}
}  // namespace
void d2h_stage_release(hipStream_t st) {
  D2HStage* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    auto it = g_stages.find(st);
    if (it == g_stages.end()) return;
    p = it->second;
    g_stages.erase(it);
  }
  if (p->dgather) (void)hipFree(p->dgather);
  delete p;  // PinnedBuf frees the pinned buffer
}
namespace {
struct GatherArgs {
  const unsigned* src[kGatherMax];
  int words[kGatherMax], off[kGatherMax];
  int n;
};
__global__ void gather_words_kernel(GatherArgs a, unsigned* __restrict__ dst) {
  for (int i = 0; i < a.n; ++i)
    for (int w = threadIdx.x; w < a.words[i]; w += blockDim.x) dst[a.off[i] + w] = a.src[i][w];
}
static hipError_t d2h_sync(hipStream_t st, std::initializer_list<D2H> reads) {
  auto staged = [](const D2H& r) { return r.bytes <= kStageMax; };
  auto pad = [](size_t b) { return (b + 15) & ~(size_t)15; };
  size_t tot = 0;
  int small = 0;
  bool gatherable = true;
  for (const D2H& r : reads) {
    if (!r.bytes) continue;
    if (staged(r)) tot += pad(r.bytes);
    if (r.bytes <= kGatherBytes && r.bytes % 4 == 0) ++small;
    else gatherable = false;
  }
  D2HStage& sg = stage_for(st);
  PinnedBuf& pb = sg.pin;
  if (tot) FCHK(pb.ensure(tot));
  if (gatherable && small > 1 && small <= kGatherMax) {  // every read small: one kernel, one copy
    if (!sg.dgather) FCHK(hipMalloc((void**)&sg.dgather, kGatherMax * kGatherBytes));
    unsigned* const dstage = sg.dgather;
    GatherArgs a{};
    size_t o = 0;
    for (const D2H& r : reads) {
      if (!r.bytes) continue;
      a.src[a.n] = static_cast<const unsigned*>(r.d);
      a.words[a.n] = (int)(r.bytes / 4);
      a.off[a.n] = (int)(o / 4);
      ++a.n;
      o += pad(r.bytes);
    }
    hipLaunchKernelGGL(gather_words_kernel, dim3(1), dim3(256), 0, st, a, dstage);
    FCHK(hipMemcpyAsync(pb.p, dstage, o, hipMemcpyDeviceToHost, st));
  } else {
    size_t o = 0;
    for (const D2H& r : reads) {
      if (!r.bytes) continue;
      if (staged(r)) {
        FCHK(hipMemcpyAsync(pb.as<char>(o), r.d, r.bytes, hipMemcpyDeviceToHost, st));
        o += pad(r.bytes);
      } else {
        FCHK(hipMemcpyAsync(r.h, r.d, r.bytes, hipMemcpyDeviceToHost, st));
      }
    }
  }
  FCHK(hipStreamSynchronize(st));
  size_t o = 0;
  for (const D2H& r : reads)
    if (r.bytes && staged(r)) {
      std::memcpy(r.h, pb.as<char>(o), r.bytes);
      o += pad(r.bytes);
    }
  return hipSuccess;
}
static hipError_t read_int(const int* d, int* h, hipStream_t st) { return d2h_sync(st, {{h, d, sizeof(int)}}); }
// Host -> device copies of the per-wave index lists (parents, survivor slots, commit slots) through
// the scene's pinned staging buffer (ExpandBuffers::h2d): asynchronous for real, where a pageable
// source is staged by the runtime first.  The buffer is rewritten only after the previous copy from
// it has completed (its event; in the loop several stream synchronisations lie between two copies).
static hipError_t h2d_async(H2DStage& sg, void* d, const void* h, size_t bytes, hipStream_t st) {
  if (!bytes) return hipSuccess;
  if (bytes > kStageMax) return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);
  if (!sg.done) FCHK(hipEventCreateWithFlags(&sg.done, hipEventDisableTiming));
  if (sg.pending) FCHK(hipEventSynchronize(sg.done));
  FCHK(sg.pin.ensure(bytes));
  std::memcpy(sg.pin.p, h, bytes);
  FCHK(hipMemcpyAsync(d, sg.pin.p, bytes, hipMemcpyHostToDevice, st));
  FCHK(hipEventRecord(sg.done, st));
  sg.pending = true;
  return hipSuccess;
}

// CSR cell lists from the registration masks (vis = 0: pgrids, 1: vpgrids)
static hipError_t build_lists(Ctx& c, int vis) {
  FilterBuffers& B = c.B;
  const Reg* reg = vis ? B.vreg : B.preg;
  int* csr_off = vis ? B.vp_off : B.pg_off;
  int* items = vis ? B.vp_items : B.pg_items;
  hipLaunchKernelGGL(count_entries_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.P, c.n, reg, vis, B.cnt);
  FCHK(hipMemsetAsync(B.cnt + c.n, 0, sizeof(int), c.st));
  size_t tb = B.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cnt, B.off, c.n + 1, c.st));
  int e = 0;
  FCHK(read_int(B.off + c.n, &e, c.st));
  (vis ? c.nvp : c.npg) = e;
  FCHK(B.ensure_entries((size_t)e, vis));
  items = vis ? B.vp_items : B.pg_items;  // (re)allocated by ensure_entries
  hipLaunchKernelGGL(emit_entries_kernel, dim3(nblk((long long)c.n * kLG)), dim3(256), 0, c.st, c.s, c.P, c.n, reg, vis, B.off, B.tgoff,
                     B.keys);
  tb = B.temp_bytes;
  if (e > 0) FCHK(hipcub::DeviceRadixSort::SortKeys(B.temp, tb, B.keys, B.keys2, e, 32, 32 + cell_bits(c.ncells), c.st));
  FCHK(memset_big(B.cellcnt, 0, (c.ncells + 1) * sizeof(int), c.st));
  if (e > 0) {
    hipLaunchKernelGGL(cell_hist_kernel, dim3(nblk(e)), dim3(256), 0, c.st, B.keys2, e, B.cellcnt);
    hipLaunchKernelGGL(items_kernel, dim3(nblk(e)), dim3(256), 0, c.st, B.keys2, e, items);
  }
  tb = B.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cellcnt, csr_off, (int)(c.ncells + 1), c.st));
  return hipGetLastError();
}

// flags / scatter over the collect order: out lists the flagged patches in collect order (sorted by
// their first cell), so concurrent workgroups work on neighbouring patches
__global__ void flag_order_kernel(const int* __restrict__ v, const int* __restrict__ order, int na, int* __restrict__ f) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < na) f[i] = v[order[i]] != 0;
}
__global__ void scatter_order_kernel(const int* __restrict__ f, const int* __restrict__ off, const int* __restrict__ order,
                                     int na, int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < na && f[i]) out[off[i]] = order[i];
}

__global__ void pack_bits_kernel(const int* __restrict__ f, int n, unsigned* __restrict__ bits) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w * 32 >= n) return;
  unsigned v = 0u;
  for (int b = 0; b < 32 && w * 32 + b < n; ++b) v |= (f[w * 32 + b] != 0 ? 1u : 0u) << b;
  bits[w] = v;
}
__global__ void unpack_bits_kernel(const unsigned* __restrict__ bits, int n, int* __restrict__ f) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) f[k] = (bits[k >> 5] >> (k & 31)) & 1u;
}

// filterSmallGroups labels on the device (filter_pass): see the comment at the call.
static int lab_jump() {  // PMVS_LAB_JUMP: sweeps per all-vertex pointer jump (A/B knob)
  static const int v = getenv("PMVS_LAB_JUMP") ? std::max(1, atoi(getenv("PMVS_LAB_JUMP"))) : 1;
  return v;
}
__global__ void lab_init_kernel(int* __restrict__ lab, int* __restrict__ active, int na) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < na) {
    lab[i] = i;
    active[i] = 1;
  }
}
// One relaxation sweep over the vertices whose label dropped since they were last relaxed
// (active[i] != 0), or over every vertex (all = 1: the verifying sweep).  A lowered target is
// re-activated; the sweep's reads of other vertices' labels may already see this sweep's updates
// (labels only decrease, so any interleaving converges to the same fixpoint).
// jump: whether every vertex tries the pointer jump in this sweep (else only the active ones do: an
// inactive vertex then costs one coalesced flag read, not the jump's dependent gather).
__global__ void lab_relax_kernel(const int* __restrict__ eoff, const int* __restrict__ edges, int na, int* lab,
                                 int* active, int all, int* changed, int jump) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na) return;
  if (!all && !jump && active[i] == 0) return;
  // the pointer jump lab[i] = lab[lab[i]] (reachability is transitive), fused here (round 4 ran it as
  // its own full pass after every other sweep); a jumped vertex relaxes too
  const int l0 = lab[i], l1 = lab[l0];
  const bool jumped = l1 < l0 && atomicMin(&lab[i], l1) > l1;
  if (jumped) atomicOr(changed, 1);
  // a plain read first (a flag set during this sweep and read stale stays set for the next)
  if (!all && !jumped && active[i] == 0) return;
  if (atomicExch(&active[i], 0) == 0 && !all && !jumped) return;
  const int li = atomicAdd(&lab[i], 0);
  bool any = false;
  for (int e = eoff[i]; e < eoff[i + 1]; ++e) {
    const int j = edges[e];
    if (li < lab[j] && atomicMin(&lab[j], li) > li) {
      atomicOr(&active[j], 1);
      any = true;
    }
  }
  if (any) atomicOr(changed, 1);
}
// Most patches share a few labels (one big component per surface): the lanes holding the wave's
// first label add it with one atomic, the others one each (no same-address atomic storm).
__global__ void lab_count_kernel(const int* __restrict__ lab, int na, int* __restrict__ csize) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = (i < na) ? lab[i] : -1;
  const int l0 = __shfl(l, 0, 64);
  const unsigned long long same = __ballot(i < na && l == l0);
  if (i < na && l != l0) atomicAdd(&csize[l], 1);
  if ((threadIdx.x & 63) == 0 && same) atomicAdd(&csize[l0], (int)__popcll(same));
}
__global__ void lab_flags_kernel(const int* __restrict__ lab, const int* __restrict__ csize, const int* __restrict__ order,
                                 int na, int threshold, int* __restrict__ flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < na && csize[lab[i]] < threshold) flags[order[i]] = 1;
}

// CPatchOrganizerS::collectPatches: collect ranks and order
static hipError_t collect(Ctx& c) {
  FilterBuffers& B = c.B;
  FCHK(hipMemsetAsync(B.counters, 0, 8 * sizeof(int), c.st));
  hipLaunchKernelGGL(first_cell_kernel, dim3(std::min(nblk((long long)c.n * kLG), 2048u)), dim3(256), 0, c.st, c.s, c.P, c.n,
                     B.preg, B.tgoff, B.keys,
                     B.counters);
  size_t tb = B.temp_bytes;
  FCHK(hipcub::DeviceRadixSort::SortKeys(B.temp, tb, B.keys, B.keys2, c.n, 32, 32 + cell_bits(c.ncells), c.st));
  FCHK(read_int(B.counters, &c.nalive, c.st));
  FCHK(hipMemsetAsync(B.rank, 0xff, c.n * sizeof(int), c.st));
  if (c.nalive > 0)
    hipLaunchKernelGGL(rank_kernel, dim3(nblk(c.nalive)), dim3(256), 0, c.st, B.keys2, c.nalive, B.order, B.rank);
  hipLaunchKernelGGL(hot_kernel, dim3(nblk(c.n)), dim3(256), 0, c.st, c.s, c.P, c.n, B.hot);
  return hipGetLastError();
}

// CFilter::setDepthMapsVGridsVPGridsAddPatchV(additive) (filter.cpp:727-770)
static hipError_t set_dm_vgrids(Ctx& c, int additive) {
  FilterBuffers& B = c.B;
  FCHK(build_lists(c, 0));
  dbg(c.st, "  lists");
  FCHK(collect(c));
  dbg(c.st, "  collect");
  FCHK(memset_big(B.dpkey, 0xff, c.ncells * sizeof(unsigned long long), c.st));
  if (c.nalive > 0)
    hipLaunchKernelGGL(coordc_kernel, dim3(nblk(c.nalive)), dim3(256), 0, c.st, c.P, B.order, c.nalive, B.coordc);
  // owner-partitioned: this rank's targets only (t = rank + world j)
  const int nown = (c.s.tnum - c.rank + c.world - 1) / c.world;
  if (c.nalive > 0 && nown > 0)
    hipLaunchKernelGGL(depth_map_kernel, dim3(nblk((long long)c.nalive * ((nown + dm_tpt() - 1) / dm_tpt()))), dim3(256), 0,
                       c.st, c.s, c.dev(), B.coordc, B.dpkey, c.rank, c.world, dm_tpt());
  dbg(c.st, "  depth");
  FCHK(hipMemsetAsync(B.vreg, 0, c.n * sizeof(Reg), c.st));
  if (c.nalive > 0) {
    // setVImagesVGrids: visibility rows of this rank's targets (all targets at world 1), all-gathered
    // when the pass is owner-partitioned, then every rank's lists in target order
    const long long row_words = (c.nalive + 63) / 64;
    const int nown_max = (c.s.tnum + c.world - 1) / c.world;
    const size_t rwords = (size_t)nown_max * row_words;
    FCHK(fgrow(B.normalc, B.cap_normalc, (size_t)c.nalive));
    FCHK(fgrow(B.used, B.cap_used, (size_t)c.nalive * (PMVS_MAX_TARGETS / 64)));
    FCHK(fgrow(B.vrows, B.cap_vrows, rwords));
    hipLaunchKernelGGL(normalc_kernel, dim3(nblk(c.nalive)), dim3(256), 0, c.st, c.P, B.order, c.nalive, B.normalc);
    hipLaunchKernelGGL(used_kernel, dim3(nblk((long long)c.nalive * kLG)), dim3(256), 0, c.st, c.s, c.dev(), additive, B.used);
    if (nown > 0)
      hipLaunchKernelGGL(vis_rows_kernel, dim3(nblk((long long)((nown + kVisT - 1) / kVisT) * row_words * 64)), dim3(256), 0,
                         c.st, c.s, c.dev(),
                         B.coordc, B.normalc, B.used, c.rank, c.world, nown, row_words, B.vrows);
    const unsigned long long* rows = B.vrows;
    if (c.world > 1) {
      FCHK(fgrow(B.xr, B.cap_xr, rwords * 8 * c.world));
      FCHK(c.xchg(0, B.vrows, rwords * 8, B.xr, nullptr));
      rows = reinterpret_cast<const unsigned long long*>(B.xr);
    }
    hipLaunchKernelGGL(vis_lists_kernel, dim3(xcd_grid(c.nalive)), dim3(256), 0, c.st, c.s, c.dev(), additive, c.world,
                       nown_max, row_words, rows, B.vreg);
  } else if (c.world > 1) {
    FCHK(c.xchg(0, nullptr, 0, nullptr, nullptr));  // the exchange every rank makes here
  }
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

// Owner-partitioned pass (sh->world > 1): rank g owns the target images t with
// t mod world = g and the patches whose reference image it owns.  The per-target stages run on the
// owner and their results are all-gathered, so every rank ends the pass with the same model:
//   setDepthMaps          the owned targets' maps only (no other rank reads them);
//   setVImagesVGrids      visibility bits in the owned targets -> all-gather -> every rank appends the
//                         visible targets in target order (5 times per pass);
//   filterOutside         gains of the owned patches -> reject bits all-gathered;
//   filterExact           isVisible over the owned targets' cells -> safe bits all-gathered (OR);
//                         setRefImage of the owned patches -> the chosen swap all-gathered;
//   filterNeighbor        the owned patches' neighbour walks and fits -> reject bits all-gathered;
//   filterSmallGroups     replicated (O(edges) label fixpoint).
// Every exchange is an 8-byte header {error, value} all-gathered first, then (all fine) the payload,
// device to device over RCCL when the shard has it.  A rank that fails between exchanges leaves the
// pass and sends one header with its error (filter_pass), which its peers receive at their next
// header -- this pass's next exchange, or the loop's next one -- so every rank returns the error.
static hipError_t filter_pass_impl(const DScene& s, FilterBuffers& B, pmvs_patch* dP, int n, long long ncells,
                                   const long long* h_tgoff, int grid, hipStream_t st, int counts[4], int* overflow,
                                   int* keep_dev, const Shard* sh, bool& agreed) {
  const bool part = sh && sh->world > 1;
  agreed = false;
  // test hook (tests/test_gpu_expand.py): PMVS_TEST_SHARD_FAIL="rank:0:f|g" fails that rank's
  // filter pass before (f) or after (g) its filterNeighbor exchange
  int inj_rank = -1, inj_wave = -1;
  char inj_where = 0;
  if (const char* e = getenv("PMVS_TEST_SHARD_FAIL")) (void)sscanf(e, "%d:%d:%c", &inj_rank, &inj_wave, &inj_where);
  const bool inject = part && inj_rank == sh->rank;
  dbg(st, "start");
  FCHK(B.reserve(n, ncells, s.tnum, grid * NB_GRID_MULT));
  dbg(st, "reserve");
  FCHK(hipMemcpyAsync(B.tgoff, h_tgoff, (s.tnum + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
  Ctx c{s, B, dP, n, ncells, grid, st};
  c.coordc = B.coordc;  // written with every depth map of this pass (set_dm_vgrids)
  const int G = part ? sh->world : 1, R = part ? sh->rank : 0;
  if (part) {
    c.rank = R;
    c.world = G;
    c.xchg = [&](int value, const void* dsend, size_t bytes, void* drecv, long long* vsum) -> hipError_t {
      int h[2] = {0, value};
      std::vector<int> all(2 * (size_t)G, 0);
      agreed = true;  // a failure from here to the payload's end is every rank's
      if (sh->exchange(h, sizeof(h), all.data()) != 0) return hipErrorUnknown;
      long long sum = 0;
      for (int r = 0; r < G; ++r) {
        if (all[2 * r] != 0) return hipErrorUnknown;  // a peer failed since the last exchange
        sum += all[2 * r + 1];
      }
      if (vsum) *vsum = sum;
      if (bytes) {
        if (sh->exchange_dev) {
          if (sh->exchange_dev(dsend, bytes, drecv, st) != 0) return hipErrorUnknown;
        } else {
          std::vector<char> hs(bytes), hr(bytes * G);
          FCHK(hipMemcpyAsync(hs.data(), dsend, bytes, hipMemcpyDeviceToHost, st));
          FCHK(hipStreamSynchronize(st));
          if (sh->exchange(hs.data(), bytes, hr.data()) != 0) return hipErrorUnknown;
          FCHK(hipMemcpyAsync(drecv, hr.data(), bytes * G, hipMemcpyHostToDevice, st));
          FCHK(hipStreamSynchronize(st));
        }
      }
      agreed = false;
      return hipSuccess;
    };
  }
  // flags[0, n) of the patches this rank decided -> every rank's, OR-merged (one exchange)
  auto merge_flags = [&](int value, long long* vsum) -> hipError_t {
    const size_t nw = (size_t)(n + 31) / 32;
    FCHK(fgrow(B.rbits, B.cap_rbits, nw + 1));
    FCHK(fgrow(B.xr, B.cap_xr, (nw + 1) * 4 * G));
    if (nw) hipLaunchKernelGGL(pack_bits_kernel, dim3(nblk((long long)nw)), dim3(256), 0, st, B.flags, n, B.rbits);
    FCHK(c.xchg(value, B.rbits, nw * 4, B.xr, vsum));
    if (nw) {
      hipLaunchKernelGGL(or_bits_kernel, dim3(nblk((long long)nw)), dim3(256), 0, st, reinterpret_cast<const unsigned*>(B.xr),
                         G, nw, B.rbits);
      hipLaunchKernelGGL(unpack_bits_kernel, dim3(nblk(n)), dim3(256), 0, st, B.rbits, n, B.flags);
    }
    return hipGetLastError();
  };
  for (int k = 0; k < 4; ++k) counts[k] = 0;
  *overflow = 0;
  FCHK(hipMemsetAsync(B.counters + 8, 0, sizeof(int), st));  // vimages list overflows (vis_lists_kernel)
  hipLaunchKernelGGL(init_reg_kernel, dim3(nblk((long long)n * kLG)), dim3(256), 0, st, s, dP, n, B.preg, B.vreg);
  FCHK(set_dm_vgrids(c, 0));
  dbg(st, "set_dm_vgrids(0)");
  // ---- filterOutside
  FCHK(hipMemsetAsync(B.flags, 0, n * sizeof(int), st));
  if (c.nalive) hipLaunchKernelGGL(gain_kernel, dim3(nblk((long long)c.nalive * kLG)), dim3(256), 0, st, s, c.dev(), B.flags, R, G);
  if (part) FCHK(merge_flags(0, nullptr));
  FCHK(apply_flags(c, &counts[0]));
  dbg(st, "outside");
  FCHK(set_dm_vgrids(c, 1));
  // ---- filterExact
  FCHK(hipMemsetAsync(B.safe, 0, n * sizeof(Reg), st));
  FCHK(hipMemsetAsync(B.counters + 2, 0, sizeof(int), st));
  hipLaunchKernelGGL(exact_entries_kernel, dim3(nblk(ncells)), dim3(256), 0, st, s, c.dev(), ncells, B.safe, R, G);
  if (part) {  // safe bits of every rank's targets, OR-merged
    const size_t words = (size_t)n * (sizeof(Reg) / 4);
    FCHK(fgrow(B.xr, B.cap_xr, words * 4 * G));
    FCHK(c.xchg(0, B.safe, words * 4, B.xr, nullptr));
    hipLaunchKernelGGL(or_bits_kernel, dim3(nblk((long long)words)), dim3(256), 0, st, reinterpret_cast<const unsigned*>(B.xr), G,
                       words, reinterpret_cast<unsigned*>(B.safe));
  }
  FCHK(hipMemsetAsync(B.need, 0, n * sizeof(int), st));
  if (c.nalive)
    hipLaunchKernelGGL(exact_patch_kernel, dim3((c.nalive + 3) / 4), dim3(256), 0, st, s, c.dev(), B.safe, B.preg, B.vreg,
                       B.need, B.counters + 2);
  {
    // the patches that need setRefImage (all collected: exact_patch_kernel sets need over the collect
    // order), compacted on the device in collect order -- sorted by their first cell, so the
    // persistent grid's concurrent patches are neighbours and share their texels in L2 (index
    // order, round 4, scattered them: 68 GB of texel reads per C3 launch)
    const int na = c.nalive;
    int m = 0;
    if (na > 0) {
      hipLaunchKernelGGL(flag_order_kernel, dim3(nblk(na)), dim3(256), 0, st, B.need, B.order, na, B.cnt);
      FCHK(hipMemsetAsync(B.cnt + na, 0, sizeof(int), st));
      size_t tb = B.temp_bytes;
      FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cnt, B.off, na + 1, st));
      hipLaunchKernelGGL(scatter_order_kernel, dim3(nblk(na)), dim3(256), 0, st, B.cnt, B.off, B.order, na, B.list);
      FCHK(read_int(B.off + na, &m, st));
    }
    if (part) {  // the owners' setRefImage outcomes (m is the same on every rank)
      FCHK(fgrow(B.refpos, B.cap_refpos, (size_t)std::max(m, 1)));
      FCHK(fgrow(B.xr, B.cap_xr, (size_t)std::max(m, 1) * 4 * G));
      FCHK(launch_filter_refimage(s, dP, B.list, m, grid, st, B.refpos, R, G));
      FCHK(c.xchg(0, B.refpos, (size_t)m * 4, B.xr, nullptr));
      FCHK(launch_apply_refpos(s, dP, B.list, m, reinterpret_cast<const int*>(B.xr), G, st));
    } else if (m) {
      FCHK(launch_filter_refimage(s, dP, B.list, m, grid, st));
    }
    if (m)
      hipLaunchKernelGGL(exact_after_ref_kernel, dim3(nblk(m)), dim3(256), 0, st, s, dP, B.list, m, B.preg, B.vreg,
                         B.counters + 2);
    FCHK(read_int(B.counters + 2, &counts[1], st));
  }
  dbg(st, "exact");
  FCHK(set_dm_vgrids(c, 1));
  dbg(st, "set_dm_vgrids(1) after exact");
  // ---- filterNeighbor(1)
  if (inject && inj_where == 'f') return hipErrorOutOfMemory;
  FCHK(hipMemsetAsync(B.flags, 0, n * sizeof(int), st));
  FCHK(hipMemsetAsync(B.counters + 3, 0, 5 * sizeof(int), st));
  if (c.nalive) {
    // PMVS_QUAD_ROWS caps the deferred-fit rows (tests: 0 = every fit in the wave, small = a mix)
    QuadJobs qj{B.qf, B.qrows, B.qjobs, B.qctr, reinterpret_cast<int*>(B.qctr + 1), (unsigned long long)B.cap_qrows};
    if (const char* e = getenv("PMVS_QUAD_ROWS")) qj.cap_rows = std::min(qj.cap_rows, (unsigned long long)atoll(e));
    if (qj.cap_rows == 0) qj.f = nullptr;
    FCHK(hipMemsetAsync(B.qctr, 0, 2 * sizeof(unsigned long long), st));
    NbOverflow nbw, nbr;
    FCHK(nb_overflow_lists(B, (size_t)c.nalive, st, nbw, nbr));
    int* nbdbg = getenv("PMVS_FILTER_DEBUG") ? B.need : nullptr;
    hipLaunchKernelGGL(neighbor_kernel<NB_CAP>, dim3(std::min(grid * NB_GRID_MULT, c.nalive)), dim3(64), 0, st, s, c.dev(),
                       B.scratch, B.flags, B.counters + 3, B.counters + 4, nbdbg, R, G, qj, nbw);
    if (qj.f) {
      int nj = 0;
      FCHK(read_int(qj.njobs, &nj, st));
      if (nj > 0) {
        const int nch = (nj + 63) / 64;
        hipLaunchKernelGGL(quad_keys_kernel, dim3(nblk(nj)), dim3(256), 0, st, B.qjobs, nj, B.qkeys);
        size_t tb = B.temp_bytes;
        FCHK(hipcub::DeviceRadixSort::SortKeys(B.temp, tb, B.qkeys, B.qkeys2, nj, 0, 43, st));
        hipLaunchKernelGGL(quad_chunk_rows_kernel, dim3(nblk(nch)), dim3(256), 0, st, B.qkeys2, nj, B.qcrows);
        tb = B.temp_bytes;
        FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.qcrows, B.qoff, nch, st));
        int dev = 0, cus = 0;
        FCHK(hipGetDevice(&dev));
        FCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        // fits of at most nq rows: quad_qr_kernel (rows in LDS) + quad_solve_kernel; the rest (the
        // sorted prefix [0, kb)) one lane per job.  PMVS_QUAD_LDS_ROWS=0: every fit one lane per job.
        int nq = 96;
        if (const char* e = getenv("PMVS_QUAD_LDS_ROWS")) nq = std::max(0, std::min(160, atoi(e)));
        int* kb = reinterpret_cast<int*>(B.qctr + 2);
        if (nq > 0) hipLaunchKernelGGL(quad_split_kernel, dim3(nblk(nj)), dim3(256), 0, st, B.qkeys2, nj, nq, kb);
        unsigned qgrid = nblk(nj);
        if (const char* e = getenv("PMVS_QUAD_WAVES_PER_CU"))  // 0 = one lane per job, no cap
          if (atoi(e) > 0) qgrid = std::min(qgrid, (unsigned)std::max(1, cus * atoi(e) / 4));  // 4 wavefronts per 256-lane block
        hipLaunchKernelGGL(quad_lane_kernel, dim3(qgrid), dim3(256), 0, st, s, c.dev(), qj, B.qkeys2, B.qoff, nj,
                           B.flags, nq > 0 ? kb : nullptr);
        if (nq > 0) {
          int wpc = 4;
          if (const char* e = getenv("PMVS_QUAD_QR_WAVES_PER_CU")) wpc = std::max(1, atoi(e));
          const unsigned qrgrid = std::min((unsigned)(cus * wpc), (unsigned)((nj + 64 / QL - 1) / (64 / QL)));
          const size_t lds = (size_t)(64 / QL) * nq * 6 * sizeof(double);
          hipLaunchKernelGGL(quad_qr_kernel, dim3(qrgrid), dim3(64), lds, st, qj, B.qkeys2, B.qoff, kb, nj, nq);
          hipLaunchKernelGGL(quad_solve_kernel, dim3(nblk(nj)), dim3(256), 0, st, s, c.dev(), qj, B.qkeys2, B.qoff, kb,
                             nj, B.flags);
        }
      }
    }
  }
  if (c.nalive) {  // the patches with more than NB_CAP neighbours, walked again (fits in the wavefront)
    QuadJobs qnone{};
    NbOverflow nbr;
    nbr.only = B.ovf_items;
    nbr.only_n = B.counters + 10;
    hipLaunchKernelGGL(neighbor_kernel<NB_CAP_BIG>, dim3(NB_GRID_BIG), dim3(64), 0, st, s, c.dev(), B.scratch_big, B.flags,
                       B.counters + 3, B.counters + 11, getenv("PMVS_FILTER_DEBUG") ? B.need : nullptr, R, G, qnone, nbr);
  }
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
  if (part) {  // reject flags of every rank's patches; the overflow counts summed in the header
    long long ovf = 0;
    FCHK(merge_flags(*overflow, &ovf));
    *overflow = (int)ovf;
    if (inject && inj_where == 'g') return hipErrorOutOfMemory;
  }
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
    // filterSmallGroups' labelling (filter.cpp:520-562): a BFS from every unlabelled patch in
    // collect order over the directed neighbour edges.  The label it gives patch j is the
    // smallest collect index m from which j is reachable (m is unlabelled when its turn comes --
    // an earlier root reaching m would reach j -- and no node of a path m -> j can carry an
    // earlier label, for the same reason), so the labels are a fixpoint: lab[j] = min over edges
    // i -> j of lab[i], accelerated by lab[j] = lab[lab[j]] (reachability is transitive).  Computed
    // on the device; only the component sizes matter (threshold below).
    const int threshold = std::max(20, na / 10000);
    int* lab = B.need;   // free after filterExact
    int* csize = B.list;
    int* changed = B.counters + 5;
    // Relaxation sweeps visit only the vertices whose label dropped since their last sweep (the
    // late sweeps, a few thousand vertices, cost a launch instead of a pass over every edge); the
    // loop ends after a sweep over EVERY vertex changes nothing, i.e. at the fixpoint itself.
    int* active = B.list;  // csize's buffer, free until the counting below
    hipLaunchKernelGGL(lab_init_kernel, dim3(nblk(na)), dim3(256), 0, st, lab, active, na);
    // every lab_jump()-th active sweep jumps every vertex's pointer (1: every sweep, rounds 4-5)
    int sweep = 0;
    for (int it = 0;; ++it) {
      const bool verify = (it % 9) == 8;  // a full sweep after each 8 rounds of active sweeps that changed something
      FCHK(hipMemsetAsync(changed, 0, sizeof(int), st));
      for (int r = 0; r < (verify ? 1 : 8); ++r) {
        if (ne)
          hipLaunchKernelGGL(lab_relax_kernel, dim3(nblk(na)), dim3(256), 0, st, B.edge_off, B.edges, na, lab, active,
                             verify ? 1 : 0, changed, (sweep++ % lab_jump()) == 0 ? 1 : 0);
      }
      int ch = 0;
      FCHK(read_int(changed, &ch, st));
      if (verify && !ch) break;
      if (!verify && !ch) it = 9 * (it / 9) + 7;  // nothing moved: verify next
      if (it > 9 * (na + 1)) return hipErrorIllegalState;  // cannot happen: every round lowers some label
    }
    FCHK(hipMemsetAsync(csize, 0, na * sizeof(int), st));
    hipLaunchKernelGGL(lab_count_kernel, dim3(nblk(na)), dim3(256), 0, st, lab, na, csize);
    FCHK(hipMemsetAsync(B.flags, 0, n * sizeof(int), st));
    hipLaunchKernelGGL(lab_flags_kernel, dim3(nblk(na)), dim3(256), 0, st, lab, csize, B.order, na, threshold, B.flags);
    // _flag = collect index of every collected patch (filter.cpp:538-542)
    hipLaunchKernelGGL(flag_rank_kernel, dim3(nblk(na)), dim3(256), 0, st, dP, B.order, na);
    // fixed patches are never removed (filter.cpp:590)
    hipLaunchKernelGGL(clear_fixed_kernel, dim3(nblk(n)), dim3(256), 0, st, dP, n, B.flags);
    FCHK(apply_flags(c, &counts[3]));
  }
  dbg(st, "groups");
  FCHK(set_dm_vgrids(c, 1));
  FCHK(build_lists(c, 0));
  FCHK(collect(c));
  hipLaunchKernelGGL(keep_kernel, dim3(nblk(n)), dim3(256), 0, st, n, B.preg, B.rank, keep_dev);
  int lovf = 0;
  FCHK(read_int(B.counters + 8, &lovf, st));
  if (lovf) return hipErrorNotSupported;  // a vimages list would exceed PMVS_MAX_IMAGES (reported by the API)
  return hipGetLastError();
}

// Owner-partitioned (world > 1): a rank that fails outside an exchange sends one 8-byte error header
// here (see filter_pass_impl), so its peers fail at their next header instead of blocking.
// NB_PROFILE builds: the walk-phase cycle sums since the last dump, one JSON line on stderr, then cleared
static void nb_prof_dump(const char* what) {
#if defined(NB_PROFILE)
  unsigned long long h[3][8];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(g_nb_prof), sizeof(h)) != hipSuccess) return;
  fprintf(stderr, "{\"nb_prof\": \"%s\"", what);
  for (int k = 0; k < 3; ++k) {
    fprintf(stderr, ", \"k%d\": [", k);
    for (int i = 0; i < 8; ++i) fprintf(stderr, "%s%llu", i ? ", " : "", h[k][i]);
    fprintf(stderr, "]");
  }
  fprintf(stderr, "}\n");
  std::memset(h, 0, sizeof(h));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_nb_prof), h, sizeof(h));
#else
  (void)what;
#endif
}

hipError_t filter_pass(const DScene& s, FilterBuffers& B, pmvs_patch* dP, int n, long long ncells, const long long* h_tgoff,
                       int grid, hipStream_t st, int counts[4], int* overflow, int* keep_dev, const Shard* sh,
                       bool* handled) {
  bool agreed = false;
  hipError_t e = filter_pass_impl(s, B, dP, n, ncells, h_tgoff, grid, st, counts, overflow, keep_dev, sh, agreed);
  nb_prof_dump("filter");
  if (handled) *handled = true;
  if (e != hipSuccess && sh && sh->world > 1 && n > 0 && !agreed) {
    int h[2] = {1, 0};
    std::vector<int> all(2 * (size_t)sh->world, 0);
    (void)sh->exchange(h, sizeof(h), all.data());
  }
  return e;
}


// ============================================================================ expansion (host)
namespace {

static inline float __int_as_float_h(int v) {
  float f;
  std::memcpy(&f, &v, sizeof(f));
  return f;
}

// Queue entry: key = order-preserving bits of _tmp (-0 as +0) << 32 | ~seq, so that one unsigned
// compare is P_compare (patchOrganizerS.hpp:10-15: max _tmp) with ties to the earlier push.
// sum of n 0/1 flags into *out (one atomic per wavefront)
__global__ void count_ok_kernel(const int* __restrict__ ok, int n, int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long m = __ballot(i < n && ok[i] != 0);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(out, (int)__popcll(m));
}

__global__ void gather_slots_kernel(const int* __restrict__ slots, int m, const pmvs_candidate* __restrict__ cin,
                                    const pmvs_patch* __restrict__ prep, pmvs_candidate* __restrict__ cout,
                                    pmvs_patch* __restrict__ pout, const int* __restrict__ cidx) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  cout[k] = cin[cidx[slots[k]]];
  pout[k] = prep[cidx[slots[k]]];
}

// Collected patches: flag = 1 (clearFlags + collectPatches(queue), patchOrganizerS.cpp) and their
// _tmp in collect order (the queue's initial contents).
__global__ void collect_flags_kernel(pmvs_patch* __restrict__ P, const int* __restrict__ order, int na,
                                     float* __restrict__ qtmp, int* __restrict__ rank, int* __restrict__ foreign) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na) return;
  pmvs_patch& q = P[order[i]];
  q.flag = 1;
  const float t = q.tmp;
  qtmp[i] = (t == 0.0f) ? 0.0f : t;  // -0 as +0: the radix order then agrees with QCmp's `<`
  rank[i] = i;
  foreign[i] = (q.fix == PMVS_FIX_FOREIGN);  // another cluster's boundary patch: never expanded here
}

// The initial queue run in key order (pmvs_queue.h QItem / qkey), built on the device from the
// device-sorted _tmp keys: item j of the sorted order is {qkey(tmp, collect rank), patch index},
// kept unless the patch is another cluster's boundary patch; keep flags first, then the scatter to
// the kept items' positions (an exclusive scan of the flags).
struct DQItem {  // pmvs_queue.h QItem's layout
  unsigned long long key;
  int p, pad;
};
__device__ __forceinline__ unsigned long long dqkey(float tmp, long long seq) {
  unsigned u = __float_as_uint(tmp == 0.0f ? 0.0f : tmp);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (0xffffffffull - (unsigned long long)seq);
}
__global__ void queue_keep_kernel(const int* __restrict__ srank, const int* __restrict__ foreign, int n,
                                  int* __restrict__ keep) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) keep[j] = foreign[srank[j]] ? 0 : 1;
}
__global__ void queue_items_kernel(const float* __restrict__ tmp_sorted, const int* __restrict__ srank,
                                   const int* __restrict__ order, const int* __restrict__ keep,
                                   const int* __restrict__ pos, int n, DQItem* __restrict__ items) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !keep[j]) return;
  const int r = srank[j];
  DQItem q;
  q.key = dqkey(tmp_sorted[j], r);
  q.p = order[r];
  q.pad = 0;
  items[pos[j]] = q;
}

// The survivors of a wave's preparation (status 0) in (parent, direction) order, on the device:
// surv_flags_kernel flags them and counts the prepared candidates (status >= 0, one atomic per
// block); after an exclusive scan of the flags, surv_scatter_kernel writes slots[pos] = k and
// slot2[k] = pos (-1 for the others).
__global__ __launch_bounds__(256) void surv_flags_kernel(const int* __restrict__ status, int nk, int* __restrict__ flag,
                                                         int* __restrict__ nprep) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int v = k < nk ? status[k] : -1;
  if (k < nk) flag[k] = (v == 0) ? 1 : 0;
  const unsigned long long b = __ballot(v >= 0);
  __shared__ int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&cnt, __popcll(b));
  __syncthreads();
  if (threadIdx.x == 0 && cnt) atomicAdd(nprep, cnt);
}
__global__ void surv_scatter_kernel(const int* __restrict__ flag, const int* __restrict__ pos, int nk,
                                    int* __restrict__ slots, int* __restrict__ slot2) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  if (flag[k]) {
    slots[pos[k]] = k;
    slot2[k] = pos[k];
  } else {
    slot2[k] = -1;
  }
}

// Compact per-candidate record the host commit reads (instead of two full patch records):
// [status, tmp bits, nprep, nimg, nvis | prep cells[64] | image cells[64] | vimage cells[64]],
// cells as global target-cell indexes.  prep cells: the in-grid target entries of the prepared
// candidate (the commit-time checkCounts); image / vimage cells: the in-grid target entries of
// the refined patch (updateCounts, addPatch).  status 9 = a record the refine path cannot produce.
constexpr int kRecInts = 5 + 3 * PMVS_MAX_IMAGES;
__global__ void commit_rec_kernel(DScene s, const long long* __restrict__ tgoff, const pmvs_patch* __restrict__ outp,
                                  const int* __restrict__ ostatus, const pmvs_patch* __restrict__ prep, int m,
                                  int* __restrict__ rec) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  int* r = rec + (size_t)j * kRecInts;
  const pmvs_patch& pp = prep[j];
  int np = 0;
  for (int i = 0; i < pp.num_images && i < PMVS_MAX_IMAGES; ++i) {
    const int t = pp.images[i];
    if (t < s.tnum && in_grid(s, t, pp.grids[i][0], pp.grids[i][1]))
      r[5 + np++] = (int)(tgoff[t] + (long long)pp.grids[i][1] * gwidth(s, t) + pp.grids[i][0]);
  }
  r[2] = np;
  int st = ostatus[j];
  int ni = 0, nv = 0;
  if (st == 0) {
    const pmvs_patch& q = outp[j];
    if (q.num_images < 1 || q.num_images > PMVS_MAX_IMAGES || q.num_vimages < 0 || q.num_vimages > PMVS_MAX_IMAGES) {
      st = 9;
    } else {
      for (int i = 0; i < q.num_images; ++i) {
        const int t = q.images[i];
        if (t < 0 || t >= s.num) st = 9;
        else if (t < s.tnum && in_grid(s, t, q.grids[i][0], q.grids[i][1]))
          r[5 + PMVS_MAX_IMAGES + ni++] = (int)(tgoff[t] + (long long)q.grids[i][1] * gwidth(s, t) + q.grids[i][0]);
      }
      for (int i = 0; i < q.num_vimages; ++i) {
        const int t = q.vimages[i];
        if (t < 0 || t >= s.tnum) st = 9;
        else if (in_grid(s, t, q.vgrids[i][0], q.vgrids[i][1]))
          r[5 + 2 * PMVS_MAX_IMAGES + nv++] = (int)(tgoff[t] + (long long)q.vgrids[i][1] * gwidth(s, t) + q.vgrids[i][0]);
      }
      r[1] = __float_as_int(q.tmp);
    }
  }
  r[0] = st;
  r[3] = ni;
  r[4] = nv;
}

// Committed candidates appended to the model: P[first + k] = outp[acc[k]] with _flag = 1,
// _fix = 0, _dflag = 0 (CExpand::expandSub -> addPatch).  One wavefront per record.
__global__ __launch_bounds__(64) void append_kernel(pmvs_patch* __restrict__ P, int first, const int* __restrict__ acc,
                                                    int nacc, const pmvs_patch* __restrict__ outp) {
  const int k = blockIdx.x;
  if (k >= nacc) return;
  const unsigned* src = reinterpret_cast<const unsigned*>(&outp[acc[k]]);
  unsigned* dst = reinterpret_cast<unsigned*>(&P[first + k]);
  constexpr int kFlag = offsetof(pmvs_patch, flag) / 4, kFix = offsetof(pmvs_patch, fix) / 4,
                kDflag = offsetof(pmvs_patch, dflag) / 4;
  for (int w = threadIdx.x; w < (int)(sizeof(pmvs_patch) / 4); w += 64)
    dst[w] = (w == kFlag) ? 1u : (w == kFix || w == kDflag) ? 0u : src[w];
}

// _dflag |= bits of the parents whose directions failed this wave (distinct parents per wave).
__global__ void dflag_kernel(pmvs_patch* __restrict__ P, const int2* __restrict__ upd, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) P[upd[k].x].dflag |= upd[k].y;
}

__global__ void alive_reg_kernel(int n, const int* __restrict__ alive, Reg* __restrict__ preg,
                                 Reg* __restrict__ vreg, const pmvs_patch* __restrict__ P) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (!alive[p]) {
    preg[p] = reg_zero();
    vreg[p] = reg_zero();
  } else {
    vreg[p] = reg_first(P[p].num_vimages);
  }
}

// Host mirror of one target cell during an expansion run.
struct HostCell {
  unsigned char count, occ;
};
static_assert(sizeof(HostCell) == 2, "HostCell layout");
struct HostCells {  // 2 MB-aligned, transparent huge pages: the commit's accesses are random
  HostCell* p = nullptr;
  explicit HostCells(size_t n) {
    const size_t bytes = ((n * sizeof(HostCell)) + (2u << 20) - 1) & ~((size_t)(2u << 20) - 1);
    p = static_cast<HostCell*>(aligned_alloc(2u << 20, bytes ? bytes : (2u << 20)));
    if (p) (void)madvise(p, bytes, MADV_HUGEPAGE);
  }
  ~HostCells() { free(p); }
};

// {count 0, occupied = pgrids holds a patch} per cell, for the host mirror.
__global__ void cell_init_kernel(const int* __restrict__ pg_off, long long ncells, HostCell* __restrict__ out) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncells) out[c] = HostCell{0, (unsigned char)(pg_off[c + 1] > pg_off[c] ? 1 : 0)};
}

// CExpand::updateCounts results of one commit (host-computed): counts[cell] = value.
__global__ void counts_scatter_kernel(const int* __restrict__ cells, const unsigned char* __restrict__ vals, int n,
                                      unsigned char* __restrict__ counts) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) counts[cells[k]] = vals[k];
}

template <class T>
static hipError_t grow(T*& p, size_t& cap, size_t need) {
  if (need <= cap && p) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = need;
  const hipError_t e = hipMalloc((void**)&p, (need ? need : 1) * sizeof(T));
  if (e == hipSuccess) poison_alloc(p, (need ? need : 1) * sizeof(T));
  return e;
}

}  // namespace

void delete_commit_work(CommitWork* w);  // after CommitWork's definition
ExpandBuffers::~ExpandBuffers() {
  void* ps[] = {parents, cand_coord, cand_ok, cand, prep, status, slots, cand2, prep2, res, outp, ostatus, counts, alive,
                pg_head, vp_head, d_ent, pool_used, tcells, tvals, qtmp, crec, acc, dupd, cellinit, occ,
                qkey, qrank, qrank2, qsort_tmp, xsd, xrd, cidx, qkeep, qpos, qitems, sflag, spos, slot2};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  delete_commit_work(cm);
}

void ExpandBuffers::release() {
  this->~ExpandBuffers();
  new (this) ExpandBuffers();
}

// Grows a device array keeping its contents (the delta-chain entry pool, the per-patch arrays).
// 1.5x: old and new coexist during the copy, and at C5 scale the model alone is ~80 GB.
template <class T>
static hipError_t grow_keep(T*& p, size_t& cap, size_t need, size_t used, hipStream_t st) {
  if (need <= cap && p) return hipSuccess;
  const size_t ncap = std::max(need, cap + cap / 2 + 1024);
  T* q = nullptr;
  FCHK(hipMalloc((void**)&q, ncap * sizeof(T)));
  poison_alloc(q, ncap * sizeof(T));
  if (p && used) FCHK(hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, st));
  FCHK(hipStreamSynchronize(st));
  if (p) (void)hipFree(p);
  p = q;
  cap = ncap;
  return hipSuccess;
}

// ============================================================================ device commit
// CExpand's commit of a wave (expand.cpp:225-266 addPatch + checkCounts, :309-406 updateCounts) in
// (parent priority, direction) order k = 6 * parent + direction, on the device.  The decision of
// candidate k depends on the counts / occupancy of its cells as left by every earlier candidate
// that touches one of them; candidates that share no cell with an undecided earlier candidate
// are decided in the same round.  Every access (prep cells read by checkCounts, image / vimage
// cells written by updateCounts and addPatch) is sorted by (cell, k); a round marks, per cell,
// the first undecided candidate, and decides every candidate that is first in all of its cells
// (so each cell has one writer per round and plain stores suffice).  The result is the
// sequential commit exactly, in as many rounds as the longest chain of cell-sharing candidates.
struct CommitWork {
  int *stc = nullptr, *nacc = nullptr, *aoff = nullptr, *vals = nullptr, *vals2 = nullptr, *pos = nullptr,
      *head = nullptr, *segid = nullptr, *seghead = nullptr, *segptr = nullptr, *segfirst = nullptr,
      *slot2 = nullptr, *flag = nullptr, *scan = nullptr, *ctr = nullptr, *pbits = nullptr;
  unsigned long long *keys = nullptr, *keys2 = nullptr;
  unsigned char* dec = nullptr;
  int2* push = nullptr;
  void* temp = nullptr;
  size_t cap_k = 0, cap_a = 0, temp_bytes = 0;
  ~CommitWork() {
    void* ps[] = {stc, nacc, aoff, vals, vals2, pos, head, segid, seghead, segptr, segfirst, slot2, flag, scan, ctr,
                  pbits, keys, keys2, dec, push, temp};
    for (void* p : ps)
      if (p) (void)hipFree(p);
  }
};

void delete_commit_work(CommitWork* w) { delete w; }

// occupancy per target cell after the model load: pgrids holds a patch
__global__ void occ_init_kernel(const int* __restrict__ pg_off, long long ncells, unsigned char* __restrict__ occ) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncells) occ[c] = pg_off[c + 1] > pg_off[c] ? 1 : 0;
}

// per k: outcome so far (-1 no candidate, 1 prepare failed, 2 / 3 refine failed, 9 invalid record,
// 0 refined: to be decided) and its number of cell accesses
__global__ void cm_stage_kernel(const int* __restrict__ status, const int* __restrict__ slot2, const int* __restrict__ rec,
                                int nk, int* __restrict__ stc, int* __restrict__ nacc, unsigned char* __restrict__ dec,
                                int* __restrict__ nlive) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  int st = status[k], a = 0;
  unsigned char d = 1;
  if (st < 0) {
    st = -1;
  } else if (st == 0) {
    const int* r = rec + (size_t)slot2[k] * kRecInts;
    st = r[0];
    if (st == 0) {
      a = r[2] + r[3] + r[4];
      d = 0;
      atomicAdd(nlive, 1);
    }
  }
  stc[k] = st;
  nacc[k] = a;
  dec[k] = d;
}

__global__ void cm_emit_kernel(const int* __restrict__ stc, const int* __restrict__ slot2, const int* __restrict__ rec,
                               const int* __restrict__ aoff, int nk, unsigned long long* __restrict__ keys,
                               int* __restrict__ vals) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk || stc[k] != 0) return;
  const int* r = rec + (size_t)slot2[k] * kRecInts;
  int o = aoff[k];
  auto emit = [&](int cell) {
    keys[o] = ((unsigned long long)(unsigned int)cell << 32) | (unsigned int)k;
    vals[o] = o;
    ++o;
  };
  for (int i = 0; i < r[2]; ++i) emit(r[5 + i]);
  for (int i = 0; i < r[3]; ++i) emit(r[5 + PMVS_MAX_IMAGES + i]);
  for (int i = 0; i < r[4]; ++i) emit(r[5 + 2 * PMVS_MAX_IMAGES + i]);
}

__global__ void cm_head_kernel(const unsigned long long* __restrict__ keys, const int* __restrict__ vals, int na,
                               int* __restrict__ head, int* __restrict__ pos) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= na) return;
  head[p] = (p == 0 || (keys[p] >> 32) != (keys[p - 1] >> 32)) ? 1 : 0;
  pos[vals[p]] = p;
}

// segid = inclusive scan of head - 1; seghead[segment] = its first position, seghead[nseg] = na
__global__ void cm_seg_kernel(const int* __restrict__ head, int* __restrict__ segid, int na, int* __restrict__ seghead,
                              int* __restrict__ segptr, int* __restrict__ nseg) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= na) return;
  const int s = segid[p] - 1;
  segid[p] = s;
  if (head[p]) {
    seghead[s] = p;
    segptr[s] = p;
  }
  if (p == na - 1) {
    seghead[s + 1] = na;
    *nseg = s + 1;
  }
}

__device__ __forceinline__ void cm_first_at(int s, const unsigned long long* __restrict__ keys,
                                            const unsigned char* dec, const int* __restrict__ seghead,
                                            int* __restrict__ segptr, int* __restrict__ segfirst) {
  int p = segptr[s];
  const int end = seghead[s + 1];
  while (p < end && dec[(int)(keys[p] & 0xffffffffull)]) ++p;
  segptr[s] = p;
  segfirst[s] = (p < end) ? (int)(keys[p] & 0xffffffffull) : -1;
}
__global__ void cm_first_kernel(const unsigned long long* __restrict__ keys, const unsigned char* __restrict__ dec,
                                const int* __restrict__ seghead, const int* __restrict__ nsegp, int* __restrict__ segptr,
                                int* __restrict__ segfirst) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= *nsegp) return;
  cm_first_at(s, keys, dec, seghead, segptr, segfirst);
}

// The decision of candidate k (record r) once it is the first undecided candidate in all of its
// cells: checkCounts with the committed state (expand.cpp:309-322), then updateCounts
// (expand.cpp:325-406) + addPatch's pgrids registration.  ctr: [0] decided, [1] fail_commit.
__device__ __forceinline__ void cm_apply(const DScene& s, int k, const int* r, unsigned char* dec, int* stc, int* flag,
                                         unsigned char* counts, unsigned char* occ, int cthr, int check, int* ctr) {
  int st = 0;
  if (check) {
    int full = 0, empty = 0;
    for (int i = 0; i < r[2]; ++i) {
      const int c = r[5 + i];
      if (occ[c]) { ++full; continue; }
      if (cthr <= counts[c]) ++full;
      else ++empty;
    }
    const bool fail = (s.depth <= 1) ? (empty < s.minImageNum && full != 0) : (empty < s.minImageNum - 1 && full != 0);
    if (fail) st = 4;
  }
  if (st == 0) {
    int full = 0, empty = 0;
    auto touch = [&](int c) {
      const unsigned char cc = counts[c];
      if (cthr <= cc) ++full;
      else ++empty;
      counts[c] = (unsigned char)(cc + 1);
    };
    for (int i = 0; i < r[3]; ++i) touch(r[5 + PMVS_MAX_IMAGES + i]);
    for (int i = 0; i < r[4]; ++i) touch(r[5 + 2 * PMVS_MAX_IMAGES + i]);
    for (int i = 0; i < r[3]; ++i) occ[r[5 + PMVS_MAX_IMAGES + i]] = 1;
    flag[k] = (empty != 0) ? 3 : 1;  // bit 0 accepted, bit 1 pushed on the queue
  } else {
    stc[k] = st;
    flag[k] = 0;
    atomicAdd(&ctr[1], 1);
  }
  dec[k] = 1;
  atomicAdd(&ctr[0], 1);
}

// each access's segment (segid[pos[e]]), once per commit instead of once per round
__global__ void cm_segof_kernel(const int* __restrict__ pos, const int* __restrict__ segid, int na, int* __restrict__ segof) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < na) segof[e] = segid[pos[e]];
}

// Decides every undecided candidate that is the first undecided one in all of its cells (its
// accesses' segments, four loads in flight at a time).
// ctr: [0] decided this call, [1] fail_commit, [2] invalid.
__device__ __forceinline__ void cm_decide_at(const DScene& s, int k, const int* __restrict__ slot2,
                                             const int* __restrict__ rec, const int* __restrict__ aoff,
                                             const int* __restrict__ nacc, const int* __restrict__ segof,
                                             const int* segfirst, unsigned char* dec, int* __restrict__ stc,
                                             int* __restrict__ flag, unsigned char* counts, unsigned char* occ, int cthr,
                                             int check, int* ctr) {
  if (dec[k]) return;
  const int e0 = aoff[k], ee = e0 + nacc[k];
  for (int e = e0; e < ee; e += 4) {
    int sg[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) sg[u] = (e + u < ee) ? segof[e + u] : -1;
    bool first = true;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (sg[u] >= 0 && segfirst[sg[u]] != k) first = false;
    if (!first) return;
  }
  cm_apply(s, k, rec + (size_t)slot2[k] * kRecInts, dec, stc, flag, counts, occ, cthr, check, ctr);
}
__global__ void cm_decide_kernel(DScene s, int nk, const int* __restrict__ slot2, const int* __restrict__ rec,
                                 const int* __restrict__ aoff, const int* __restrict__ nacc, const int* __restrict__ segof,
                                 const int* __restrict__ segfirst, unsigned char* __restrict__ dec, int* __restrict__ stc,
                                 int* __restrict__ flag, unsigned char* __restrict__ counts, unsigned char* __restrict__ occ,
                                 int cthr, int check, int* __restrict__ ctr) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  cm_decide_at(s, k, slot2, rec, aoff, nacc, segof, segfirst, dec, stc, flag, counts, occ, cthr, check, ctr);
}

// the undecided candidates of a wave's commit, listed after its first rounds (device_commit)
__global__ void cm_undecided_kernel(const unsigned char* __restrict__ dec, int nk, int* __restrict__ f) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nk) f[k] = dec[k] ? 0 : 1;
}
__global__ void cm_list_kernel(const int* __restrict__ f, const int* __restrict__ pos, int nk, int* __restrict__ list,
                               int* __restrict__ cnt) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nk && f[k]) list[pos[k]] = k;
  if (k == nk - 1) *cnt = pos[k] + f[k];
}
// cm_decide_kernel over the listed candidates (grid-stride over *cnt)
__global__ void cm_decide_list_kernel(DScene s, const int* __restrict__ list, const int* __restrict__ cnt,
                                      const int* __restrict__ slot2, const int* __restrict__ rec, const int* __restrict__ aoff,
                                      const int* __restrict__ nacc, const int* __restrict__ segof,
                                      const int* __restrict__ segfirst, unsigned char* __restrict__ dec, int* __restrict__ stc,
                                      int* __restrict__ flag, unsigned char* __restrict__ counts, unsigned char* __restrict__ occ,
                                      int cthr, int check, int* __restrict__ ctr) {
  const int n = *cnt;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x)
    cm_decide_at(s, list[t], slot2, rec, aoff, nacc, segof, segfirst, dec, stc, flag, counts, occ, cthr, check, ctr);
}

// flags of the non-refined candidates (0) and the outcome counters: ctr[3] fail_prep, [4] fail_pre,
// [5] fail_post, [2] invalid records
__global__ void cm_noref_kernel(const int* __restrict__ stc, int nk, int* __restrict__ flag, int* __restrict__ ctr) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  const int st = stc[k];
  if (st != 0) flag[k] = 0;
  if (st == 1) atomicAdd(&ctr[3], 1);
  else if (st == 2) atomicAdd(&ctr[4], 1);
  else if (st == 3) atomicAdd(&ctr[5], 1);
  else if (st != 0 && st != -1 && st != 4) atomicAdd(&ctr[2], 1);
}

// acc list [slot | entry offset] of the accepted candidates in k order, their pushes, and each
// parent's failed-direction bits (applied to _dflag when apply_dflag, else kept for the host)
__global__ void cm_accept_scan_kernel(const int* __restrict__ flag, int nk, int* __restrict__ a, int* __restrict__ b,
                                      int* __restrict__ c, const int* __restrict__ slot2, const int* __restrict__ rec) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  const int f = flag[k];
  a[k] = f & 1;               // accepted
  b[k] = (f >> 1) & 1;        // pushed
  if (f & 1) {
    const int* r = rec + (size_t)slot2[k] * kRecInts;
    c[k] = r[3] + r[4];       // registration entries
  } else {
    c[k] = 0;
  }
}

__global__ void cm_write_kernel(const int* __restrict__ flag, int nk, const int* __restrict__ qa, const int* __restrict__ qb,
                                const int* __restrict__ qc, const int* __restrict__ slot2, const int* __restrict__ rec,
                                int pool0, int first, int* __restrict__ acc, int2* __restrict__ push) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  const int f = flag[k];
  if (!(f & 1)) return;
  const int nacc = qa[nk];  // accepted candidates: the end of the exclusive scan
  const int q = qa[k];
  acc[q] = slot2[k];
  acc[nacc + q] = pool0 + qc[k];
  if (f & 2) {
    const int* r = rec + (size_t)slot2[k] * kRecInts;
    push[qb[k]] = make_int2(r[1], first + q);
  }
}

// _dflag |= failed directions (stc > 0) of each parent of the wave
__global__ void cm_bits_kernel(const int* __restrict__ stc, int np, int* __restrict__ bits) {
  const int pi = blockIdx.x * blockDim.x + threadIdx.x;
  if (pi >= np) return;
  int b = 0;
  for (int d = 0; d < 6; ++d)
    if (stc[6 * pi + d] > 0) b |= 1 << d;
  bits[pi] = b;
}
__global__ void cm_dflag_kernel(pmvs_patch* __restrict__ P, const int* __restrict__ parents, const int* __restrict__ bits,
                                int np) {
  const int pi = blockIdx.x * blockDim.x + threadIdx.x;
  if (pi < np && bits[pi]) P[parents[pi]].dflag |= bits[pi];
}

// Small waves (the reference's wave = 1 schedule: one parent, <= 6 candidates per batch): the same
// commit by one lane in k order, with one small read-back.  out = [nacc, npush, entries, fail_prep,
// fail_pre, fail_post, fail_commit, invalid, bits of parent 0, pushes (tmp bits, new index) x nk].
constexpr int kSerialCommit = 64;
__global__ void cm_serial_kernel(DScene s, const int* __restrict__ status, const int* __restrict__ slot2,
                                 const int* __restrict__ rec, int nk, int np, unsigned char* __restrict__ counts,
                                 unsigned char* __restrict__ occ, int cthr, int check, int first, int pool0,
                                 int* __restrict__ acc, int* __restrict__ out, const int* __restrict__ parents,
                                 pmvs_patch* __restrict__ P, int apply_dflag) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int accs[kSerialCommit], ents[kSerialCommit];
  int nacc = 0, npush = 0, entries = 0, f[5] = {0, 0, 0, 0, 0};
  int bits[kSerialCommit / 6 + 1];
  for (int pi = 0; pi < np; ++pi) bits[pi] = 0;
  for (int k = 0; k < nk; ++k) {
    int st = status[k];
    if (st < 0) continue;
    const int* r = nullptr;
    if (st == 0) {
      r = rec + (size_t)slot2[k] * kRecInts;
      st = r[0];
    }
    if (st == 0 && check) {
      int full = 0, empty = 0;
      for (int i = 0; i < r[2]; ++i) {
        const int c = r[5 + i];
        if (occ[c]) { ++full; continue; }
        if (cthr <= counts[c]) ++full;
        else ++empty;
      }
      const bool fail = (s.depth <= 1) ? (empty < s.minImageNum && full != 0) : (empty < s.minImageNum - 1 && full != 0);
      if (fail) st = 4;
    }
    if (st != 0) {
      bits[k / 6] |= 1 << (k % 6);
      if (st >= 1 && st <= 4) f[st - 1]++;
      else f[4]++;
      continue;
    }
    int full = 0, empty = 0;
    auto touch = [&](int c) {
      const unsigned char cc = counts[c];
      if (cthr <= cc) ++full;
      else ++empty;
      counts[c] = (unsigned char)(cc + 1);
    };
    for (int i = 0; i < r[3]; ++i) touch(r[5 + PMVS_MAX_IMAGES + i]);
    for (int i = 0; i < r[4]; ++i) touch(r[5 + 2 * PMVS_MAX_IMAGES + i]);
    for (int i = 0; i < r[3]; ++i) occ[r[5 + PMVS_MAX_IMAGES + i]] = 1;
    accs[nacc] = slot2[k];
    ents[nacc] = entries;
    entries += r[3] + r[4];
    if (empty != 0) {
      out[9 + 2 * npush] = r[1];
      out[9 + 2 * npush + 1] = first + nacc;
      ++npush;
    }
    ++nacc;
  }
  for (int q = 0; q < nacc; ++q) {
    acc[q] = accs[q];
    acc[nacc + q] = pool0 + ents[q];
  }
  out[0] = nacc; out[1] = npush; out[2] = entries;
  out[3] = f[0]; out[4] = f[1]; out[5] = f[2]; out[6] = f[3]; out[7] = f[4];
  out[8] = bits[0];
  if (apply_dflag)
    for (int pi = 0; pi < np; ++pi)
      if (bits[pi]) P[parents[pi]].dflag |= bits[pi];
}

template <class T>
static hipError_t cm_grow(T*& p, size_t n) {
  if (p) (void)hipFree(p);
  p = nullptr;
  const hipError_t e = hipMalloc((void**)&p, (n ? n : 1) * sizeof(T));
  if (e == hipSuccess) poison_alloc(p, (n ? n : 1) * sizeof(T));
  return e;
}

struct CommitOut {
  int nacc = 0, pbits = 0;
  long long entries = 0, fail[4] = {0, 0, 0, 0};  // fail_prep, fail_pre, fail_post, fail_commit
  std::vector<int2> push;                          // (tmp bits, new patch index) in commit order
};

// One wave's commit on the device (see CommitWork).  slot2h[k]: survivor slot of candidate k
// (status[k] == 0).  Writes X.acc = [slot of accepted q | pool0 + entry offset], applies the
// failed-direction bits to _dflag (apply_dflag) or returns them (wave = 1: one parent).
static hipError_t device_commit(const DScene& s, ExpandBuffers& X, hipStream_t st, int np, const int* d_slot2, int m,
                                const int* d_ovf, int* ovf,
                                int cthr, bool check, int first, long long pool0, bool apply_dflag, pmvs_patch* dP,
                                CommitOut& out) {
  if (!X.cm) X.cm = new CommitWork();
  CommitWork& W = *X.cm;
  const int nk = np * 6;
  if ((size_t)nk + 1 > W.cap_k) {
    const size_t c = std::max((size_t)nk + 1, 2 * W.cap_k);
    FCHK(cm_grow(W.stc, c)); FCHK(cm_grow(W.nacc, c)); FCHK(cm_grow(W.aoff, c));
    FCHK(cm_grow(W.flag, c)); FCHK(cm_grow(W.scan, 6 * c)); FCHK(cm_grow(W.dec, c)); FCHK(cm_grow(W.pbits, c));
    FCHK(cm_grow(W.push, c));
    W.cap_k = c;
  }
  if (!W.ctr) FCHK(cm_grow(W.ctr, 9 + 2 * kSerialCommit));
  const int* slot2v = d_slot2;  // candidate -> survivor (surv_scatter_kernel)
  *ovf = 0;
  if (nk <= kSerialCommit) {
    FCHK(grow(X.acc, X.cap_acc, 2 * (size_t)nk));
    hipLaunchKernelGGL(cm_serial_kernel, dim3(1), dim3(64), 0, st, s, X.status, slot2v, X.crec, nk, np, X.counts, X.occ,
                       cthr, check ? 1 : 0, first, (int)pool0, X.acc, W.ctr, X.parents, dP, apply_dflag ? 1 : 0);
    int h[9 + 2 * kSerialCommit];
    FCHK(d2h_sync(st, {{h, W.ctr, sizeof(h)}, {ovf, d_ovf, d_ovf ? sizeof(int) : 0}}));
    if (*ovf) return hipSuccess;
    if (h[7] != 0) {
      fprintf(stderr, "expand: %d refined records are not valid patches\n", h[7]);
      return hipErrorIllegalState;
    }
    out.nacc = h[0];
    out.entries = h[2];
    for (int q = 0; q < 4; ++q) out.fail[q] = h[3 + q];
    out.pbits = apply_dflag ? 0 : h[8];
    out.push.resize(h[1]);
    for (int q = 0; q < h[1]; ++q) out.push[q] = make_int2(h[9 + 2 * q], h[9 + 2 * q + 1]);
    return hipGetLastError();
  }
  FCHK(hipMemsetAsync(W.ctr, 0, 8 * sizeof(int), st));
  hipLaunchKernelGGL(cm_stage_kernel, dim3(nblk(nk)), dim3(256), 0, st, X.status, slot2v, X.crec, nk, W.stc, W.nacc,
                     W.dec, W.ctr + 6);
  FCHK(hipMemsetAsync(W.nacc + nk, 0, sizeof(int), st));
  auto temp_need = [&](size_t bytes) -> hipError_t {
    if (bytes <= W.temp_bytes && W.temp) return hipSuccess;
    W.temp_bytes = std::max(bytes, 2 * W.temp_bytes);
    return cm_grow(reinterpret_cast<char*&>(W.temp), W.temp_bytes);
  };
  size_t tb = 0;
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, W.nacc, W.aoff, nk + 1, st));
  FCHK(temp_need(tb));
  tb = W.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(W.temp, tb, W.nacc, W.aoff, nk + 1, st));
  int hv[2] = {0, 0};
  FCHK(d2h_sync(st, {{&hv[0], W.aoff + nk, sizeof(int)}, {&hv[1], W.ctr + 6, sizeof(int)},
                     {ovf, d_ovf, d_ovf ? sizeof(int) : 0}}));
  if (*ovf) return hipSuccess;  // the caller reports the neighbour overflow of the wave's depth_post
  const int na = hv[0], nlive = hv[1];
  if (na > 0) {
    if ((size_t)na + 1 > W.cap_a) {
      const size_t c = std::max((size_t)na + 1, 2 * W.cap_a);
      FCHK(cm_grow(W.keys, c)); FCHK(cm_grow(W.keys2, c)); FCHK(cm_grow(W.vals, c)); FCHK(cm_grow(W.vals2, c));
      FCHK(cm_grow(W.pos, c)); FCHK(cm_grow(W.head, c)); FCHK(cm_grow(W.segid, c)); FCHK(cm_grow(W.seghead, c));
      FCHK(cm_grow(W.segptr, c)); FCHK(cm_grow(W.segfirst, c));
      W.cap_a = c;
    }
    hipLaunchKernelGGL(cm_emit_kernel, dim3(nblk(nk)), dim3(256), 0, st, W.stc, slot2v, X.crec, W.aoff, nk, W.keys,
                       W.vals);
    tb = 0;
    const int cb = X.ncells > 0 ? 32 + cell_bits(X.ncells) : 64;
    FCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, W.keys, W.keys2, W.vals, W.vals2, na, 32, cb, st));
    size_t tb2 = 0;
    FCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb2, W.head, W.segid, na, st));
    FCHK(temp_need(std::max(tb, tb2)));
    tb = W.temp_bytes;
    FCHK(hipcub::DeviceRadixSort::SortPairs(W.temp, tb, W.keys, W.keys2, W.vals, W.vals2, na, 32, cb, st));
    hipLaunchKernelGGL(cm_head_kernel, dim3(nblk(na)), dim3(256), 0, st, W.keys2, W.vals2, na, W.head, W.pos);
    tb = W.temp_bytes;
    FCHK(hipcub::DeviceScan::InclusiveSum(W.temp, tb, W.head, W.segid, na, st));
    hipLaunchKernelGGL(cm_seg_kernel, dim3(nblk(na)), dim3(256), 0, st, W.head, W.segid, na, W.seghead, W.segptr,
                       W.ctr + 8);  // the segment count stays on the device (cm_first_kernel reads it)
    // W.vals (the sort's input values) is free from here: each access's segment
    hipLaunchKernelGGL(cm_segof_kernel, dim3(nblk(na)), dim3(256), 0, st, W.pos, W.segid, na, W.vals);
  }
  // rounds: every round decides at least the lowest undecided candidate.  The first four rounds
  // decide most of a wave; the candidates still undecided are then listed once (W.scan is free
  // until the accept scans below) and the later rounds' decide steps visit only them.
  int decided = 0;
  bool listed = false;
  int* uflag = W.scan;
  int* upos = W.scan + (nk + 1);
  int* ulist = W.scan + 2 * (size_t)(nk + 1);
  int* ucnt = W.ctr + 9;  // free in this (non-serial) form
  const unsigned lgrid = std::min(nblk(nk), 1024u);
  static const bool trace = getenv("PMVS_COMMIT_TRACE") != nullptr;
  if (trace) {
    // diagnostic: decided count after every round (one read per round), to stderr
    fprintf(stderr, "[commit] nk=%d nlive=%d na=%d:", nk, nlive, na);
    int d = 0;
    for (int round = 0; d < nlive && round < 4 * (nlive + 2); ++round) {
      if (na > 0)
        hipLaunchKernelGGL(cm_first_kernel, dim3(nblk(na)), dim3(256), 0, st, W.keys2, W.dec, W.seghead, W.ctr + 8, W.segptr,
                           W.segfirst);
      hipLaunchKernelGGL(cm_decide_kernel, dim3(nblk(nk)), dim3(256), 0, st, s, nk, slot2v, X.crec, W.aoff, W.nacc, W.vals,
                         W.segfirst, W.dec, W.stc, W.flag, X.counts, X.occ, cthr, check ? 1 : 0, W.ctr);
      FCHK(read_int(W.ctr, &d, st));
      fprintf(stderr, " %d", nlive - d);
    }
    fprintf(stderr, "\n");
    decided = d;
  }
  for (int round = 0; decided < nlive; ) {
    for (int r = 0; r < 4; ++r, ++round) {
      if (na > 0)  // <= na segments
        hipLaunchKernelGGL(cm_first_kernel, dim3(nblk(na)), dim3(256), 0, st, W.keys2, W.dec, W.seghead, W.ctr + 8, W.segptr,
                           W.segfirst);
      if (listed)
        hipLaunchKernelGGL(cm_decide_list_kernel, dim3(lgrid), dim3(256), 0, st, s, ulist, ucnt, slot2v, X.crec, W.aoff, W.nacc,
                           W.vals, W.segfirst, W.dec, W.stc, W.flag, X.counts, X.occ, cthr, check ? 1 : 0, W.ctr);
      else
        hipLaunchKernelGGL(cm_decide_kernel, dim3(nblk(nk)), dim3(256), 0, st, s, nk, slot2v, X.crec, W.aoff, W.nacc, W.vals,
                           W.segfirst, W.dec, W.stc, W.flag, X.counts, X.occ, cthr, check ? 1 : 0, W.ctr);
    }
    FCHK(read_int(W.ctr, &decided, st));
    if (decided < nlive && !listed) {
      hipLaunchKernelGGL(cm_undecided_kernel, dim3(nblk(nk)), dim3(256), 0, st, W.dec, nk, uflag);
      FCHK(hipMemsetAsync(uflag + nk, 0, sizeof(int), st));
      size_t ub = 0;
      FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, ub, uflag, upos, nk + 1, st));
      FCHK(temp_need(ub));
      ub = W.temp_bytes;
      FCHK(hipcub::DeviceScan::ExclusiveSum(W.temp, ub, uflag, upos, nk + 1, st));
      hipLaunchKernelGGL(cm_list_kernel, dim3(nblk(nk)), dim3(256), 0, st, uflag, upos, nk, ulist, ucnt);
      listed = true;
    }
    if (round > 4 * (nlive + 2)) return hipErrorIllegalState;  // cannot happen (progress every round)
  }
  hipLaunchKernelGGL(cm_noref_kernel, dim3(nblk(nk)), dim3(256), 0, st, W.stc, nk, W.flag, W.ctr);
  // accepted / pushed / entries in k order
  int* qa = W.scan;
  int* qb = W.scan + (nk + 1);
  int* qc = W.scan + 2 * (size_t)(nk + 1);
  int* ia = W.scan + 3 * (size_t)(nk + 1);
  int* ib = W.scan + 4 * (size_t)(nk + 1);
  int* ic = W.scan + 5 * (size_t)(nk + 1);
  hipLaunchKernelGGL(cm_accept_scan_kernel, dim3(nblk(nk)), dim3(256), 0, st, W.flag, nk, ia, ib, ic, slot2v, X.crec);
  FCHK(hipMemsetAsync(ia + nk, 0, sizeof(int), st));
  FCHK(hipMemsetAsync(ib + nk, 0, sizeof(int), st));
  FCHK(hipMemsetAsync(ic + nk, 0, sizeof(int), st));
  tb = 0;
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ia, qa, nk + 1, st));
  FCHK(temp_need(tb));
  for (int t = 0; t < 3; ++t) {
    tb = W.temp_bytes;
    FCHK(hipcub::DeviceScan::ExclusiveSum(W.temp, tb, t == 0 ? ia : t == 1 ? ib : ic, t == 0 ? qa : t == 1 ? qb : qc,
                                          nk + 1, st));
  }
  // accepted / pushed / entries written in k order (the accepted count read on the device), then ONE
  // read of the totals, the counters, the pushes (at most the m survivors) and the parents' bits
  FCHK(grow(X.acc, X.cap_acc, 2 * (size_t)std::max(m, 1)));
  hipLaunchKernelGGL(cm_write_kernel, dim3(nblk(nk)), dim3(256), 0, st, W.flag, nk, qa, qb, qc, slot2v, X.crec, (int)pool0,
                     first, X.acc, W.push);
  hipLaunchKernelGGL(cm_bits_kernel, dim3(nblk(np)), dim3(256), 0, st, W.stc, np, W.pbits);
  if (apply_dflag) hipLaunchKernelGGL(cm_dflag_kernel, dim3(nblk(np)), dim3(256), 0, st, dP, X.parents, W.pbits, np);
  int tot[3], ctr[8];
  out.push.resize((size_t)std::max(m, 0));
  out.pbits = 0;
  FCHK(d2h_sync(st, {{&tot[0], qa + nk, sizeof(int)}, {&tot[1], qb + nk, sizeof(int)}, {&tot[2], qc + nk, sizeof(int)},
                     {ctr, W.ctr, 8 * sizeof(int)}, {out.push.data(), W.push, (size_t)std::max(m, 0) * sizeof(int2)},
                     {&out.pbits, W.pbits, apply_dflag ? 0 : sizeof(int)}}));
  if (ctr[2] != 0) {
    fprintf(stderr, "expand: %d refined records are not valid patches\n", ctr[2]);
    return hipErrorIllegalState;
  }
  if (tot[0] > m || tot[1] > m) return hipErrorIllegalState;  // cannot happen: only survivors are accepted
  out.nacc = tot[0];
  out.entries = tot[2];
  out.fail[0] = ctr[3]; out.fail[1] = ctr[4]; out.fail[2] = ctr[5]; out.fail[3] = ctr[1];
  out.push.resize(tot[1]);
  return hipGetLastError();
}

// PMVS_EXPAND_PROFILE=1: host wall time per expansion phase (synchronising at phase ends), to stderr.
struct PhaseTimer {
  bool on = getenv("PMVS_EXPAND_PROFILE") != nullptr;
  hipStream_t st;
  double acc[10] = {0};
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit PhaseTimer(hipStream_t s) : st(s) {}
  void mark(int k) {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    const auto now = std::chrono::steady_clock::now();
    acc[k] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
  ~PhaseTimer() {
    if (!on) return;
    static const char* names[10] = {"load", "pop", "empty_blocks", "prepare", "gather+refine", "depth_post+d2h",
                                    "exchange", "commit", "upload", "other"};
    fprintf(stderr, "[expand profile ms]");
    for (int k = 0; k < 10; ++k) fprintf(stderr, " %s=%.1f", names[k], acc[k]);
    fprintf(stderr, "\n");
  }
};

// One CExpand::run (expand.cpp:17-406) in waves on a device-resident model; see pmvs_amd.h
// (pmvs_expand_run) and DESIGN.md.  dP[0, n0) holds the model (d_alive marks the patches the
// organizer holds); on return dP[0, *n_out) holds it with the new patches appended and _flag /
// _dflag updated.  The host keeps only the queue, the per-cell counts and occupancy, and reads
// compact per-candidate commit records (commit_rec_kernel) -- no patch records cross PCIe on one
// rank.  Sharded (sh.world > 1): every rank holds the same model and runs the same schedule; the
// organizer steps (findEmptyBlocks, expandSub up to the refine) run on every rank, the refine +
// depth >= 1 postProcess of a wave's candidates is split into contiguous rank ranges, and the
// refined records are all-gathered (sh.exchange) before the identical commit -- so the model is
// bit-identical to the one-rank run with the same wave.
// Sharded error protocol: every rank makes the same sequence of exchanges.  Each refine batch
// all-gathers a 2-int header {error, overflow} before its payload; a rank that fails anywhere
// else (allocation, a device error between exchanges) leaves the pass and makes one terminal
// header exchange with its error (expand_pass), which its peers receive in place of their next
// batch header or of their own terminal exchange -- so all ranks return the error together
// instead of blocking in the next all-gather.  `agreed` = the pass ended on a header every rank saw.
// Test hook (tests/test_gpu_expand.py): PMVS_TEST_SHARD_FAIL="rank:wave:b|e|a" fails that rank at the
// given wave before its batch exchange (b), at its findEmptyBlocks candidate exchange (e) or right after
// its batch exchange (a).
static hipError_t expand_pass_impl(const DScene& s, FilterBuffers& B, ExpandBuffers& X, pmvs_patch*& dP, size_t& dP_cap,
                                   int n0, const int* d_alive, int cap, long long ncells, const long long* h_tgoff,
                                   int wave, int cthr, int flags, int grid, hipStream_t st, const RefineFn& refine,
                                   const Shard& sh, long long stats[8], int* n_out, int min_cands, bool& agreed) {
  agreed = false;
  int inj_rank = -1, inj_wave = -1;
  char inj_where = 0;
  if (const char* e = getenv("PMVS_TEST_SHARD_FAIL")) (void)sscanf(e, "%d:%d:%c", &inj_rank, &inj_wave, &inj_where);
  const bool inject = sh.world > 1 && inj_rank == sh.rank;
  for (int k = 0; k < 8; ++k) stats[k] = 0;
  *n_out = n0;
  PhaseTimer T(st);
  const int W = std::max(1, std::min(wave, kMaxWave));
  // device patch capacity: the model plus a few waves, doubled when the commits need more
  size_t pcap = std::min<size_t>((size_t)cap, (size_t)n0 + 12 * (size_t)W + 1024);
  FCHK(B.reserve((int)pcap, ncells, s.tnum, grid * NB_GRID_MULT));
  pcap = std::min<size_t>((size_t)B.cap_n, (size_t)cap);
  FCHK(grow_keep(dP, dP_cap, pcap, (size_t)n0, st));
  FCHK(hipMemcpyAsync(B.tgoff, h_tgoff, (s.tnum + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
  Ctx c{s, B, dP, n0, ncells, grid, st};
  X.ncells = ncells;
  // ---- model load (the state CFilter::run leaves): registrations, collect order, depth maps, lists
  hipLaunchKernelGGL(init_reg_kernel, dim3(nblk((long long)n0 * kLG)), dim3(256), 0, st, s, dP, n0, B.preg, B.vreg);
  hipLaunchKernelGGL(alive_reg_kernel, dim3(nblk(n0)), dim3(256), 0, st, n0, d_alive, B.preg, B.vreg, dP);
  FCHK(build_lists(c, 0));
  FCHK(collect(c));
  FCHK(memset_big(B.dpkey, 0xff, ncells * sizeof(unsigned long long), st));
  if (c.nalive > 0 && !(flags & 1))  // after the seed phase the depth maps are still empty
  {
    hipLaunchKernelGGL(coordc_kernel, dim3(nblk(c.nalive)), dim3(256), 0, st, dP, B.order, c.nalive, B.coordc);
    hipLaunchKernelGGL(depth_map_kernel, dim3(nblk((long long)c.nalive * ((s.tnum + dm_tpt() - 1) / dm_tpt()))), dim3(256), 0,
                       st, s, c.dev(), B.coordc, B.dpkey, 0, 1, dm_tpt());
  }
  FCHK(build_lists(c, 1));
  // ---- registrations committed by this run: per-cell chains (no per-wave rebuild of the CSR)
  FCHK(grow(X.pg_head, X.cap_pghead, (size_t)ncells));
  FCHK(grow(X.vp_head, X.cap_vphead, (size_t)ncells));
  FCHK(memset_big(X.pg_head, 0xff, ncells * sizeof(int), st));
  FCHK(memset_big(X.vp_head, 0xff, ncells * sizeof(int), st));
  size_t pool_need = 0;
  X.pool_host = 0;
  auto set_delta = [&]() {
    c.pg_dhead = X.pg_head; c.vp_dhead = X.vp_head; c.d_ent = X.d_ent;
  };
  set_delta();
  // ---- device state of the commit: CExpand's _counts (unsigned char, clearCounts) and whether
  // pgrids holds a patch, per target cell; the host keeps only the queue
  // The collected patches enter the queue in collect order (seq = collect rank); their max-_tmp
  // order (QCmp: _tmp descending, ties by seq) is a stable descending radix sort on the device.
  const size_t na1 = (size_t)std::max(1, c.nalive);
  FCHK(grow(X.qtmp, X.cap_qtmp, na1));
  FCHK(grow(X.qkey, X.cap_qkey, na1));
  FCHK(grow(X.qrank, X.cap_qrank, na1));
  FCHK(grow(X.qrank2, X.cap_qrank2, na1));
  FCHK(grow(X.occ, X.cap_occ, (size_t)ncells));
  if (c.nalive) {
    hipLaunchKernelGGL(collect_flags_kernel, dim3(nblk(c.nalive)), dim3(256), 0, st, dP, B.order, c.nalive, X.qtmp,
                       X.qrank, B.need);
    size_t tb = 0;
    FCHK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, X.qtmp, X.qkey, X.qrank, X.qrank2, c.nalive, 0, 32, st));
    if (tb > X.cap_qsort) {
      if (X.qsort_tmp) FCHK(hipFree(X.qsort_tmp));
      X.qsort_tmp = nullptr;
      X.cap_qsort = 0;
      FCHK(hipMalloc(&X.qsort_tmp, tb));
      X.cap_qsort = tb;
    }
    tb = X.cap_qsort;
    FCHK(hipcub::DeviceRadixSort::SortPairsDescending(X.qsort_tmp, tb, X.qtmp, X.qkey, X.qrank, X.qrank2, c.nalive, 0, 32,
                                                      st));
  }
  hipLaunchKernelGGL(occ_init_kernel, dim3(nblk(ncells)), dim3(256), 0, st, B.pg_off, ncells, X.occ);
  // the initial run built on the device (queue_items_kernel) and read as QItems: collectPatches(queue)
  // without other clusters' boundary patches, in key order
  int ninit = 0;
  if (c.nalive) {
    static_assert(sizeof(DQItem) == sizeof(QItem), "QItem layout");
    FCHK(grow(X.qkeep, X.cap_qkeep, na1 + 1));
    FCHK(grow(X.qpos, X.cap_qpos, na1 + 1));
    FCHK(grow(X.qitems, X.cap_qitems, na1 * sizeof(DQItem)));
    hipLaunchKernelGGL(queue_keep_kernel, dim3(nblk(c.nalive)), dim3(256), 0, st, X.qrank2, B.need, c.nalive, X.qkeep);
    size_t tb = 0;
    FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, X.qkeep, X.qpos, c.nalive + 1, st));
    if (tb > X.cap_qsort) {
      if (X.qsort_tmp) FCHK(hipFree(X.qsort_tmp));
      X.qsort_tmp = nullptr;
      X.cap_qsort = 0;
      FCHK(hipMalloc(&X.qsort_tmp, tb));
      X.cap_qsort = tb;
    }
    FCHK(hipMemsetAsync(X.qkeep + c.nalive, 0, sizeof(int), st));
    tb = X.cap_qsort;
    FCHK(hipcub::DeviceScan::ExclusiveSum(X.qsort_tmp, tb, X.qkeep, X.qpos, c.nalive + 1, st));
    hipLaunchKernelGGL(queue_items_kernel, dim3(nblk(c.nalive)), dim3(256), 0, st, X.qkey, X.qrank2, B.order, X.qkeep,
                       X.qpos, c.nalive, reinterpret_cast<DQItem*>(X.qitems));
    FCHK(read_int(X.qpos + c.nalive, &ninit, st));
  }
  FCHK(grow(X.counts, X.cap_cnt, (size_t)ncells));
  FCHK(memset_big(X.counts, 0, ncells, st));
  // The max-_tmp queue (P_compare; ties: earlier push first): the collected patches as a sorted
  // run, the patches pushed during the run in a heap, popped by merging the two.
  std::vector<QItem> initial(ninit);
  if (ninit) FCHK(hipMemcpyAsync(initial.data(), X.qitems, (size_t)ninit * sizeof(QItem), hipMemcpyDeviceToHost, st));
  FCHK(hipStreamSynchronize(st));
  RunQueue queue;
  queue.add_run(std::move(initial));
  std::vector<QItem> wave_run, sort_tmp;
  long long seq = c.nalive;
  auto q_empty = [&]() { return queue.empty(); };
  int rank_next = c.nalive;
  int nmodel = n0;
  const int G = std::max(1, sh.world), R = std::min(std::max(0, sh.rank), G - 1);
  std::vector<char> xsend, xrecv;
  CommitOut co;
  T.mark(0);
  const long long max_waves = (long long)((unsigned)flags >> 8);  // PMVS_EXPAND_MAX_WAVES (0 = unbounded)
  while (!q_empty() && (max_waves <= 0 || stats[7] < max_waves)) {
    stats[7]++;
    if (inject && inj_where == 'b' && stats[7] == inj_wave) return hipErrorOutOfMemory;
    // A wave: chunks of W parents (queue order) until it holds min_cands candidate directions
    // (findEmptyBlocks against the start-of-wave model; min_cands = 0 or W = 1: one chunk).
    std::vector<int> parents;
    long long ndirs = 0;
    c.n = nmodel;
    do {
      const int off = (int)parents.size();
      queue.pop_many(parents, (size_t)W);
      const int nc = (int)parents.size() - off;
      T.mark(1);
      FCHK(grow_keep(X.parents, X.cap_par, parents.size(), (size_t)off, st));
      FCHK(grow_keep(X.cand_coord, X.cap_coord, parents.size() * 24, (size_t)off * 24, st));
      FCHK(grow_keep(X.cand_ok, X.cap_ok, parents.size() * 6, (size_t)off * 6, st));
      FCHK(h2d_async(X.h2d, X.parents + off, parents.data() + off, nc * sizeof(int), st));
      FCHK(hipMemsetAsync(B.counters + 3, 0, 5 * sizeof(int), st));
      // Sharded (G > 1): findEmptyBlocks of a contiguous share of the chunk's parents per rank, the
      // candidates (24 floats + 6 flags per parent) all-gathered, so every rank holds the chunk's.
      const int pch = (nc + G - 1) / G;
      const int plo = (G > 1) ? std::min(nc, R * pch) : 0, phi = (G > 1) ? std::min(nc, plo + pch) : nc;
      if (phi > plo) {  // the NB_CAP walk, then the unbounded re-walk of the parents it overflowed on
        NbOverflow nbw, nbr;
        FCHK(nb_overflow_lists(B, (size_t)(phi - plo), st, nbw, nbr));
        hipLaunchKernelGGL(empty_blocks_kernel<NB_CAP>, dim3(std::min(grid * NB_GRID_MULT, phi - plo)), dim3(64), 0, st, s,
                           c.dev(), X.parents + off + plo, phi - plo, X.cand_coord + (size_t)(off + plo) * 24,
                           X.cand_ok + (size_t)(off + plo) * 6, B.counters + 4, B.counters + 3, nbw);
        hipLaunchKernelGGL(empty_blocks_stream_kernel, dim3(NB_GRID_BIG), dim3(64), 0, st, s, c.dev(), X.parents + off + plo,
                           X.cand_coord + (size_t)(off + plo) * 24, X.cand_ok + (size_t)(off + plo) * 6, B.counters + 11,
                           nbr);
      }
      if (G > 1) {
        hipError_t lerr = hipPeekAtLastError();
        int ovf = 0;
        if (lerr == hipSuccess) lerr = read_int(B.counters + 3, &ovf, st);
        if (inject && inj_where == 'e' && stats[7] == inj_wave) lerr = hipErrorOutOfMemory;
        const size_t pb = (size_t)pch * (24 * sizeof(float) + 6 * sizeof(int));
        const bool dev = (bool)sh.exchange_dev;
        auto pack = [&](char* dst, hipMemcpyKind kind) -> hipError_t {  // this rank's share: coords, then flags
          if (phi <= plo) return hipSuccess;
          hipError_t e = hipMemcpyAsync(dst, X.cand_coord + (size_t)(off + plo) * 24, (size_t)(phi - plo) * 24 * sizeof(float),
                                        kind, st);
          if (e == hipSuccess)
            e = hipMemcpyAsync(dst + (size_t)pch * 24 * sizeof(float), X.cand_ok + (size_t)(off + plo) * 6,
                               (size_t)(phi - plo) * 6 * sizeof(int), kind, st);
          return e;
        };
        if (dev) {
          if (lerr == hipSuccess) lerr = grow(X.xsd, X.cap_xsd, std::max<size_t>(pb, 1));
          if (lerr == hipSuccess) lerr = grow(X.xrd, X.cap_xrd, std::max<size_t>(pb * G, 1));
          if (lerr == hipSuccess) lerr = pack(X.xsd, hipMemcpyDeviceToDevice);
        } else {
          xsend.assign(pb, 0);
          xrecv.assign(pb * G, 0);
          if (lerr == hipSuccess) lerr = pack(xsend.data(), hipMemcpyDeviceToHost);
          if (lerr == hipSuccess) lerr = hipStreamSynchronize(st);
        }
        int hdr[2] = {(int)lerr, ovf};
        std::vector<int> hall(2 * (size_t)G, 0);
        agreed = true;  // the header below is this chunk's terminal exchange for a failing rank
        if (sh.exchange(hdr, sizeof(hdr), hall.data()) != 0) return hipErrorUnknown;
        for (int r = 0; r < G; ++r) {
          if (hall[2 * r] != 0 && lerr == hipSuccess) lerr = hipErrorUnknown;  // another rank failed
          ovf |= hall[2 * r + 1];
        }
        FCHK(lerr);
        if (ovf) { trace_error(kCapacityOverflow, __LINE__); return kCapacityOverflow; }  // more than NB_CAP neighbours (reported by the API)
        if (dev ? sh.exchange_dev(X.xsd, pb, X.xrd, st) != 0 : sh.exchange(xsend.data(), pb, xrecv.data()) != 0)
          return hipErrorUnknown;
        agreed = false;
        for (int r = 0; r < G; ++r) {
          const int rlo = std::min(nc, r * pch), rhi = std::min(nc, rlo + pch);
          if (r == R || rhi <= rlo) continue;
          const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
          const char* b = dev ? X.xrd + (size_t)r * pb : xrecv.data() + (size_t)r * pb;
          FCHK(hipMemcpyAsync(X.cand_coord + (size_t)(off + rlo) * 24, b, (size_t)(rhi - rlo) * 24 * sizeof(float), kind, st));
          FCHK(hipMemcpyAsync(X.cand_ok + (size_t)(off + rlo) * 6, b + (size_t)pch * 24 * sizeof(float),
                              (size_t)(rhi - rlo) * 6 * sizeof(int), kind, st));
        }
        if (!dev) FCHK(hipStreamSynchronize(st));  // xrecv is reused by the next exchange
      }
      if (W > 1 && min_cands > 0) {  // the chunk's free directions, summed on the device
        FCHK(hipMemsetAsync(B.counters + 9, 0, sizeof(int), st));
        hipLaunchKernelGGL(count_ok_kernel, dim3(nblk((long long)nc * 6)), dim3(256), 0, st, X.cand_ok + (size_t)off * 6,
                           nc * 6, B.counters + 9);
        int nfree = 0;
        FCHK(read_int(B.counters + 9, &nfree, st));
        ndirs += nfree;
      }
      T.mark(2);
    } while (W > 1 && ndirs < min_cands && !q_empty());
    const int np = (int)parents.size();
    stats[0] += np;
    // compact index of the free directions: the candidate / prepared-patch records are sized by
    // them, not by 6 x parents (late waves pop most of the queue, few directions are free)
    FCHK(grow(X.cidx, X.cap_cidx, (size_t)np * 6 + 1));
    FCHK(hipMemsetAsync(X.cidx + (size_t)np * 6, 0, sizeof(int), st));
    {
      size_t tb = 0;
      FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, X.cand_ok, X.cidx, np * 6, st));
      if (tb > X.cap_qsort) {
        if (X.qsort_tmp) FCHK(hipFree(X.qsort_tmp));
        X.qsort_tmp = nullptr;
        X.cap_qsort = 0;
        FCHK(hipMalloc(&X.qsort_tmp, tb));
        X.cap_qsort = tb;
      }
      tb = X.cap_qsort;
      FCHK(hipcub::DeviceScan::ExclusiveSum(X.qsort_tmp, tb, X.cand_ok, X.cidx, np * 6, st));
    }
    int nok = 0;
    if (W > 1 && min_cands > 0) {
      nok = (int)ndirs;  // the chunks' free directions, already counted (count_ok_kernel): no read
    } else {
      int last_ok = 0, last_idx = 0;
      FCHK(d2h_sync(st, {{&last_ok, X.cand_ok + (size_t)np * 6 - 1, sizeof(int)},
                         {&last_idx, X.cidx + (size_t)np * 6 - 1, sizeof(int)}}));
      nok = last_idx + (last_ok != 0);
    }
    FCHK(grow(X.cand, X.cap_cand, (size_t)std::max(nok, 1)));
    FCHK(grow(X.prep, X.cap_prep, (size_t)std::max(nok, 1)));
    FCHK(grow(X.status, X.cap_status, (size_t)np * 6));
    // wave = 1 is the reference's schedule: the parent's directions are prepared, refined and
    // committed one after the other (expand.cpp:92-101); wider waves batch every candidate.
    std::vector<int> batches{-1};
    if (W == 1) {
      std::vector<int> ok(6);
      FCHK(d2h_sync(st, {{ok.data(), X.cand_ok, 6 * sizeof(int)}}));
      batches.clear();
      for (int k = 0; k < 6; ++k)
        if (ok[k]) batches.push_back(k);
    }
    int pbits = 0;  // wave = 1: failed directions of the single parent, written after its batches
    for (const int only : batches) {
      c.n = nmodel;
      hipLaunchKernelGGL(prepare_kernel, dim3(nblk((long long)np * 6)), dim3(256), 0, st, s, c.dev(), X.counts, X.parents,
                         np, X.cand_coord, X.cand_ok, X.cand, X.prep, X.status, cthr, only, X.cidx);
      FCHK(hipPeekAtLastError());
      // the survivors compacted on the device (surv_*_kernel): slots, slot2 (candidate -> survivor)
      const int nk = np * 6;
      FCHK(grow(X.sflag, X.cap_sflag, (size_t)nk + 2));  // [nk]: 0 for the scan, [nk + 1]: prepared count
      FCHK(grow(X.spos, X.cap_spos, (size_t)nk + 1));
      FCHK(grow(X.slot2, X.cap_slot2, (size_t)nk));
      FCHK(grow(X.slots, X.cap_slots, (size_t)nk));
      FCHK(hipMemsetAsync(X.sflag + nk, 0, 2 * sizeof(int), st));
      hipLaunchKernelGGL(surv_flags_kernel, dim3(nblk(nk)), dim3(256), 0, st, X.status, nk, X.sflag, X.sflag + nk + 1);
      {
        size_t tb = 0;
        FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, X.sflag, X.spos, nk + 1, st));
        if (tb > X.cap_qsort) {
          if (X.qsort_tmp) FCHK(hipFree(X.qsort_tmp));
          X.qsort_tmp = nullptr;
          X.cap_qsort = 0;
          FCHK(hipMalloc(&X.qsort_tmp, tb));
          X.cap_qsort = tb;
        }
        tb = X.cap_qsort;
        FCHK(hipcub::DeviceScan::ExclusiveSum(X.qsort_tmp, tb, X.sflag, X.spos, nk + 1, st));
      }
      hipLaunchKernelGGL(surv_scatter_kernel, dim3(nblk(nk)), dim3(256), 0, st, X.sflag, X.spos, nk, X.slots, X.slot2);
      int sv[2] = {0, 0};
      FCHK(d2h_sync(st, {{&sv[0], X.spos + nk, sizeof(int)}, {&sv[1], X.sflag + nk + 1, sizeof(int)}}));
      stats[1] += sv[1];
      T.mark(3);
      const int m = sv[0];
      // this rank's contiguous share of the survivors
      const int chunk = (m + G - 1) / G;
      const int lo = std::min(m, R * chunk), hi = std::min(m, lo + chunk), mine = hi - lo;
      int ovf = 0;
      auto local = [&]() -> hipError_t {
        if (m > 0) {
          FCHK(grow(X.cand2, X.cap_cand2, (size_t)m));
          FCHK(grow(X.prep2, X.cap_prep2, (size_t)m));
          FCHK(grow(X.res, X.cap_res, (size_t)m));
          FCHK(grow(X.outp, X.cap_outp, (size_t)m));
          FCHK(grow(X.ostatus, X.cap_ost, (size_t)m));
          hipLaunchKernelGGL(gather_slots_kernel, dim3(nblk(m)), dim3(256), 0, st, X.slots, m, X.cand, X.prep, X.cand2, X.prep2,
                             X.cidx);
          if (mine > 0) {
            FCHK(refine(X.cand2 + lo, mine, X.res + lo));
            T.mark(4);
            FCHK(hipMemsetAsync(B.counters + 4, 0, sizeof(int), st));
            NbOverflow nbw, nbr;
            FCHK(nb_overflow_lists(B, (size_t)mine, st, nbw, nbr));
            hipLaunchKernelGGL(depth_post_kernel<NB_CAP>, dim3(std::min(grid * NB_GRID_MULT, mine)), dim3(64), 0, st, s, c.dev(),
                               X.res + lo, mine, X.outp + lo, X.ostatus + lo, B.scratch, B.counters + 4, B.counters + 3, nbw);
            hipLaunchKernelGGL(depth_post_kernel<NB_CAP_BIG>, dim3(NB_GRID_BIG), dim3(64), 0, st, s, c.dev(), X.res + lo, mine,
                               X.outp + lo, X.ostatus + lo, B.scratch_big, B.counters + 11, B.counters + 3, nbr);
            FCHK(hipPeekAtLastError());
          }
        }
        // one rank: the neighbour-overflow flag is read with the commit's first read (device_commit)
        return G > 1 ? read_int(B.counters + 3, &ovf, st) : hipPeekAtLastError();
      };
      hipError_t lerr = local();
      T.mark(5);
      if (G > 1) {
        // all-gather of the header {error, overflow}, then (every rank ok) of [status[chunk],
        // patch[chunk]] per rank; the other ranks' ranges are uploaded so every rank holds all m
        // refined records
        const size_t bytes = (size_t)chunk * (sizeof(int) + sizeof(pmvs_patch));
        const bool dev = (bool)sh.exchange_dev;  // RCCL: device to device on this stream
        if (dev) {
          if (lerr == hipSuccess) lerr = grow(X.xsd, X.cap_xsd, std::max<size_t>(bytes, 1));
          if (lerr == hipSuccess) lerr = grow(X.xrd, X.cap_xrd, std::max<size_t>(bytes * G, 1));
          if (lerr == hipSuccess && mine > 0) {
            lerr = hipMemcpyAsync(X.xsd, X.ostatus + lo, mine * sizeof(int), hipMemcpyDeviceToDevice, st);
            if (lerr == hipSuccess)
              lerr = hipMemcpyAsync(X.xsd + (size_t)chunk * sizeof(int), X.outp + lo, (size_t)mine * sizeof(pmvs_patch),
                                    hipMemcpyDeviceToDevice, st);
          }
        } else {
          xsend.assign(bytes, 0);
          xrecv.assign(bytes * G, 0);
        }
        if (!dev && lerr == hipSuccess && mine > 0) {
          lerr = hipMemcpyAsync(xsend.data(), X.ostatus + lo, mine * sizeof(int), hipMemcpyDeviceToHost, st);
          if (lerr == hipSuccess)
            lerr = hipMemcpyAsync(xsend.data() + (size_t)chunk * sizeof(int), X.outp + lo, (size_t)mine * sizeof(pmvs_patch),
                                  hipMemcpyDeviceToHost, st);
          if (lerr == hipSuccess) lerr = hipStreamSynchronize(st);
        }
        int hdr[2] = {(int)lerr, ovf};
        std::vector<int> hall(2 * (size_t)G, 0);
        agreed = true;  // from here on every return is seen by all ranks
        if (sh.exchange(hdr, sizeof(hdr), hall.data()) != 0) return hipErrorUnknown;
        for (int r = 0; r < G; ++r) {
          if (hall[2 * r] != 0 && lerr == hipSuccess) lerr = hipErrorUnknown;  // another rank failed
          ovf |= hall[2 * r + 1];
        }
        FCHK(lerr);
        if (ovf) { trace_error(kCapacityOverflow, __LINE__); return kCapacityOverflow; }  // more than NB_CAP neighbours (reported by the API)
        if (dev ? sh.exchange_dev(X.xsd, bytes, X.xrd, st) != 0 : sh.exchange(xsend.data(), bytes, xrecv.data()) != 0)
          return hipErrorUnknown;
        agreed = false;
        for (int r = 0; r < G; ++r) {
          const int rlo = std::min(m, r * chunk), rhi = std::min(m, rlo + chunk);
          if (r == R || rhi <= rlo) continue;
          const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
          const char* b = dev ? X.xrd + (size_t)r * bytes : xrecv.data() + (size_t)r * bytes;
          FCHK(hipMemcpyAsync(X.ostatus + rlo, b, (rhi - rlo) * sizeof(int), kind, st));
          FCHK(hipMemcpyAsync(X.outp + rlo, b + (size_t)chunk * sizeof(int), (size_t)(rhi - rlo) * sizeof(pmvs_patch),
                              kind, st));
        }
        if (inject && inj_where == 'a' && stats[7] == inj_wave) return hipErrorOutOfMemory;
      }
      FCHK(lerr);
      if (ovf) { trace_error(kCapacityOverflow, __LINE__); return kCapacityOverflow; }  // more than NB_CAP neighbours (reported by the API)
      if (m > 0) {
        FCHK(grow(X.crec, X.cap_crec, (size_t)m * kRecInts));
        hipLaunchKernelGGL(commit_rec_kernel, dim3(nblk(m)), dim3(256), 0, st, s, B.tgoff, X.outp, X.ostatus, X.prep2, m,
                           X.crec);
      }
      T.mark(6);
      // ---- commit in (parent priority, direction) order, on the device (device_commit)
      const int first = nmodel;
      int ovf2 = 0;
      FCHK(device_commit(s, X, st, np, X.slot2, m, G > 1 ? nullptr : B.counters + 3, &ovf2, cthr, only < 0, first,
                         (long long)X.pool_host, W > 1, dP, co));
      if (ovf2) { trace_error(kCapacityOverflow, __LINE__); return kCapacityOverflow; }  // more than NB_CAP neighbours
      for (int q = 0; q < 4; ++q) stats[2 + q] += co.fail[q];
      if (W == 1) pbits |= co.pbits;
      const int added = co.nacc;
      if (added > 0 && nmodel + added > cap) { trace_error(kCapacityOverflow, __LINE__); return kCapacityOverflow; }
      stats[6] += added;
      T.mark(7);
      if (added > 0) {
        pool_need = X.pool_host + (size_t)co.entries;
        FCHK(grow_keep(X.d_ent, X.cap_ent, pool_need, X.pool_host, st));
        set_delta();
        if ((size_t)(first + added) > pcap) {  // per-patch arrays the waves write, grown keeping their contents
          // 1.5x: the old and the new model coexist during the copy (at C5 scale ~50 M records of 1608 B)
          const size_t ncap = std::min<size_t>((size_t)cap, std::max((size_t)(first + added), pcap + pcap / 2));
          size_t c1 = pcap, c2 = pcap, c3 = pcap, c4 = pcap;
          FCHK(grow_keep(dP, dP_cap, ncap, (size_t)first, st));
          FCHK(grow_keep(B.preg, c1, ncap, (size_t)first, st));
          FCHK(grow_keep(B.vreg, c2, ncap, (size_t)first, st));
          FCHK(grow_keep(B.order, c3, ncap, (size_t)rank_next, st));
          FCHK(grow_keep(B.hot, c4, ncap, (size_t)first, st));
          B.cap_n = 0;  // the other per-patch buffers are re-reserved by the next pass
          pcap = ncap;
          c.P = dP;
        }
        hipLaunchKernelGGL(append_kernel, dim3(added), dim3(64), 0, st, dP, first, X.acc, added, X.outp);
        nmodel += added;
        c.n = nmodel;
        DeltaLists D{X.pg_head, X.vp_head, X.d_ent};
        hipLaunchKernelGGL(register_kernel, dim3(added), dim3(64), 0, st, D, X.acc, X.acc + added, added, first, X.crec,
                           kRecInts);
        hipLaunchKernelGGL(add_patches_kernel, dim3(nblk((long long)added * s.tnum)), dim3(256), 0, st, s, c.dev(), first,
                           added, rank_next, B.preg, B.vreg, B.order, B.dpkey, B.hot);
        X.pool_host = pool_need;
        rank_next += added;
      }
      // the wave's pushes as a sorted run of the queue, on the host while the GPU appends and
      // registers the wave's patches (the next pops come after this)
      wave_run.clear();
      for (const int2& u : co.push) wave_run.push_back({qkey(__int_as_float_h(u.x), seq++), u.y});
      RunQueue::sort_run(wave_run, sort_tmp);
      queue.add_run(std::vector<QItem>(wave_run));
      T.mark(8);
    }
    if (W == 1 && pbits) {
      const int2 u = make_int2(parents[0], pbits);
      FCHK(grow(X.dupd, X.cap_dupd, 1));
      FCHK(hipMemcpyAsync(X.dupd, &u, sizeof(int2), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(dflag_kernel, dim3(1), dim3(64), 0, st, dP, X.dupd, 1);
      FCHK(hipStreamSynchronize(st));
    }
  }
  *n_out = nmodel;
  return hipGetLastError();
}

hipError_t expand_pass(const DScene& s, FilterBuffers& B, ExpandBuffers& X, pmvs_patch*& dP, size_t& dP_cap, int n0,
                       const int* d_alive, int cap, long long ncells, const long long* h_tgoff, int wave, int cthr,
                       int flags, int grid, hipStream_t st, const RefineFn& refine, const Shard& sh, long long stats[8],
                       int* n_out, int min_cands) {
  bool agreed = false;
  hipError_t e = expand_pass_impl(s, B, X, dP, dP_cap, n0, d_alive, cap, ncells, h_tgoff, wave, cthr, flags, grid, st,
                                  refine, sh, stats, n_out, min_cands, agreed);
  nb_prof_dump("expand");
  if (sh.world > 1 && !agreed) {  // terminal header: a local failure reaches the peers, or theirs reach us
    const int G = sh.world;
    int hdr[2] = {(int)e, 0};
    std::vector<int> hall(2 * (size_t)G, 0);
    if (sh.exchange(hdr, sizeof(hdr), hall.data()) != 0) return e != hipSuccess ? e : hipErrorUnknown;
    for (int r = 0; r < G; ++r)
      if (hall[2 * r] != 0 && e == hipSuccess) e = hipErrorUnknown;  // a peer failed
  }
  return e;
}

// Self-test of lls5_wave (tests/test_gpu_lls.py): one workgroup per n x 5 system.
__global__ __launch_bounds__(64) void lls_selftest_kernel(const float* __restrict__ A, const float* __restrict__ b,
                                                          const int* __restrict__ off, int nsys, double* __restrict__ scratch,
                                                          float* __restrict__ x) {
  __shared__ NbLds L;
  const int sys = blockIdx.x;
  if (sys >= nsys) return;
  const int o = off[sys], n = off[sys + 1] - off[sys];
  double* M = scratch + (size_t)o * 6;
  double* r = M + (size_t)n * 5;
  for (int i = threadIdx.x; i < n; i += 64) {
    for (int j = 0; j < 5; ++j) M[(size_t)i * 5 + j] = (double)A[(size_t)(o + i) * 5 + j];
    r[i] = (double)b[o + i];
  }
  __threadfence_block();
  __syncthreads();
  lls5_wave(L, M, r, n);
  if (threadIdx.x < 5) x[(size_t)sys * 5 + threadIdx.x] = L.x[threadIdx.x];
}

hipError_t lls_selftest(const float* A, const float* b, const int* off, int nsys, int total, float* x) {
  float *dA = nullptr, *db = nullptr, *dx = nullptr;
  int* doff = nullptr;
  double* scr = nullptr;
  hipError_t e = hipMalloc((void**)&dA, (size_t)total * 5 * sizeof(float));
  if (e == hipSuccess) e = hipMalloc((void**)&db, (size_t)total * sizeof(float));
  if (e == hipSuccess) e = hipMalloc((void**)&dx, (size_t)nsys * 5 * sizeof(float));
  if (e == hipSuccess) e = hipMalloc((void**)&doff, (size_t)(nsys + 1) * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&scr, (size_t)total * 6 * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(dA, A, (size_t)total * 5 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(db, b, (size_t)total * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(doff, off, (size_t)(nsys + 1) * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(lls_selftest_kernel, dim3(nsys), dim3(64), 0, nullptr, dA, db, doff, nsys, scr, dx);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(x, dx, (size_t)nsys * 5 * sizeof(float), hipMemcpyDeviceToHost);
  for (void* p : {(void*)dA, (void*)db, (void*)dx, (void*)doff, (void*)scr})
    if (p) (void)hipFree(p);
  return e;
}

// ============================================================================ loop helpers
__global__ __launch_bounds__(64) void compact_kernel(const pmvs_patch* __restrict__ src, int n, const int* __restrict__ keep,
                                                     const int* __restrict__ pos, pmvs_patch* __restrict__ dst) {
  const int k = blockIdx.x;
  if (k >= n || !keep[k]) return;
  const unsigned* a = reinterpret_cast<const unsigned*>(&src[k]);
  unsigned* b = reinterpret_cast<unsigned*>(&dst[pos[k]]);
  for (int w = threadIdx.x; w < (int)(sizeof(pmvs_patch) / 4); w += 64) b[w] = a[w];
}

__global__ void fill_int_kernel(int* __restrict__ a, int n, int v) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) a[k] = v;
}

// The patches a filter pass kept (keep[k] = 1), in order, into dst (CFindMatch::run keeps the
// model in the organizer; here the removed records are dropped between passes).
hipError_t compact_model(FilterBuffers& B, const pmvs_patch* src, int n, const int* keep, const CompactDst& dst_for,
                         int* nkept, hipStream_t st) {
  *nkept = 0;
  if (n <= 0) return hipSuccess;
  FCHK(B.reserve(n, B.cap_cells, 0, B.cap_grid));
  FCHK(hipMemcpyAsync(B.cnt, keep, n * sizeof(int), hipMemcpyDeviceToDevice, st));
  FCHK(hipMemsetAsync(B.cnt + n, 0, sizeof(int), st));
  size_t tb = B.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.cnt, B.off, n + 1, st));
  FCHK(read_int(B.off + n, nkept, st));
  pmvs_patch* dst = nullptr;
  FCHK(dst_for(*nkept, &dst));  // the target is sized by the kept records, not by the source's capacity
  if (*nkept > 0) hipLaunchKernelGGL(compact_kernel, dim3(n), dim3(64), 0, st, src, n, keep, B.off, dst);
  return hipGetLastError();
}

hipError_t fill_int(int* a, int n, int v, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(fill_int_kernel, dim3(nblk(n)), dim3(256), 0, st, a, n, v);
  return hipGetLastError();
}

// ============================================================================ cluster exchange
// CMVS runs one pmvs2 per cluster (genOption.cpp:73-108); its clusters overlap in target images
// (CBundle::addImagesP, bundle.cpp:1003-1160), so the same surface is reconstructed by several
// runs.  With one cluster per GPU, after every loop iteration each rank all-gathers the patches
// it holds in shared target images and inserts the other ranks' ones as the reference's
// readPatches inserts another run's patches (patchOrganizerS.cpp:133-197: image2index, _vimages
// cleared, setGrids, addPatch), fixed (never filtered) and never expanded (PMVS_FIX_FOREIGN): they
// occupy their cells, so this rank's expansion does not duplicate them, and they take part in the
// depth maps and visibility tests of the filters.
__global__ void own_flags_kernel(const pmvs_patch* __restrict__ P, int n, int* __restrict__ keep) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) keep[p] = (P[p].fix != PMVS_FIX_FOREIGN) ? 1 : 0;
}

__global__ void boundary_flags_kernel(DScene s, const pmvs_patch* __restrict__ P, int n,
                                      const unsigned char* __restrict__ shared_t, int* __restrict__ f) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const pmvs_patch& q = P[p];
  int b = 0;
  if (q.fix != PMVS_FIX_FOREIGN)
    for (int k = 0; k < q.num_images; ++k) {
      const int t = q.images[k];
      if (t < s.tnum && shared_t[t] && in_grid(s, t, q.grids[k][0], q.grids[k][1])) b = 1;
    }
  f[p] = b;
}

__global__ void boundary_pack_kernel(const pmvs_patch* __restrict__ P, int n, const int* __restrict__ f,
                                     const int* __restrict__ pos, const int* __restrict__ ids, BRec* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n || !f[p]) return;
  const pmvs_patch& q = P[p];
  BRec& r = out[pos[p]];
  for (int c = 0; c < 4; ++c) { r.coord[c] = q.coord[c]; r.normal[c] = q.normal[c]; }
  r.ncc = q.ncc; r.dscale = q.dscale; r.ascale = q.ascale;
  r.num_images = q.num_images;
  for (int k = 0; k < q.num_images; ++k) r.ids[k] = ids[q.images[k]];
}

// slot j of the received block: rank j / M, record j % M (rank `me` and the padding are skipped)
__global__ void boundary_insert_kernel(DScene s, const BRec* __restrict__ in, int world, int M, int me,
                                       const int* __restrict__ cnts, const int* __restrict__ id2idx, int maxid,
                                       pmvs_patch* __restrict__ outp, int* __restrict__ ok) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (long long)world * M) return;
  const int r = (int)(j / M), k = (int)(j - (long long)r * M);
  ok[j] = 0;
  if (r == me || k >= cnts[r]) return;
  const BRec& b = in[j];
  auto map = [&](int id) { return (0 <= id && id <= maxid) ? id2idx[id] : -1; };
  if (b.num_images < 1 || b.num_images > PMVS_MAX_IMAGES || map(b.ids[0]) < 0) return;  // reference image not here
  pmvs_patch& q = outp[j];
  for (int c = 0; c < 4; ++c) { q.coord[c] = b.coord[c]; q.normal[c] = b.normal[c]; }
  q.ncc = b.ncc; q.dscale = b.dscale; q.ascale = b.ascale; q.tmp = 0.0f;
  q.flag = 1; q.fix = PMVS_FIX_FOREIGN; q.dflag = 0; q.num_vimages = 0;
  int ni = 0, nt = 0;
  for (int e = 0; e < b.num_images; ++e) {  // CPatchOrganizerS::image2index (patchOrganizerS.cpp:16-41)
    const int v = map(b.ids[e]);
    if (v < 0) continue;
    float ic[3];
    project(s.views[v], q.coord, s.level, ic);  // setGrids (patchOrganizerS.cpp:410-419)
    q.images[ni] = (int16_t)v;
    q.grids[ni][0] = grid16(((int)floorf(ic[0] + 0.5f)) / s.csize);
    q.grids[ni][1] = grid16(((int)floorf(ic[1] + 0.5f)) / s.csize);
    if (v < s.tnum && in_grid(s, v, q.grids[ni][0], q.grids[ni][1])) ++nt;
    ++ni;
  }
  q.num_images = ni;
  q.timages = 0;
  for (int e = 0; e < ni; ++e) q.timages += (q.images[e] < s.tnum);
  ok[j] = (nt > 0) ? 1 : 0;  // registered in none of this scene's cells: nothing to insert
}

ClusterBuffers::~ClusterBuffers() {
  void* ps[] = {send, recv, ins, flags, pos, cnts, temp};
  for (void* p : ps)
    if (p) (void)hipFree(p);
}

static hipError_t scan_count(ClusterBuffers& CB, const int* f, int* pos, int n, int* total, hipStream_t st) {
  size_t tb = 0;
  FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, f, pos, n + 1, st));
  if (tb > CB.temp_bytes) {
    if (CB.temp) (void)hipFree(CB.temp);
    CB.temp = nullptr;
    CB.temp_bytes = 0;
    FCHK(hipMalloc(&CB.temp, tb));
    CB.temp_bytes = tb;
  }
  tb = CB.temp_bytes;
  FCHK(hipcub::DeviceScan::ExclusiveSum(CB.temp, tb, f, pos, n + 1, st));
  return read_int(pos + n, total, st);
}

hipError_t drop_foreign(FilterBuffers& B, const pmvs_patch* src, int n, const CompactDst& dst_for, int* n_out,
                        hipStream_t st) {
  *n_out = 0;
  if (n <= 0) return hipSuccess;
  FCHK(B.reserve(n, B.cap_cells, 0, B.cap_grid));
  hipLaunchKernelGGL(own_flags_kernel, dim3(nblk(n)), dim3(256), 0, st, src, n, B.flags);
  return compact_model(B, src, n, B.flags, dst_for, n_out, st);
}

hipError_t cluster_exchange(const DScene& s, ClusterBuffers& CB, const ClusterMaps& cm, const pmvs_patch* src, int n,
                            pmvs_patch*& dst, size_t& dst_cap, int* n_out, const Shard& sh, hipStream_t st,
                            long long xstats[3], bool& agreed) {
  agreed = false;
  xstats[0] = xstats[1] = xstats[2] = 0;
  *n_out = n;
  const int G = sh.world, me = sh.rank;
  // ---- this rank's boundary patches
  int m = 0;
  hipError_t le = grow(CB.flags, CB.cap_flags, (size_t)n + 1);
  if (le == hipSuccess) le = grow(CB.pos, CB.cap_pos, (size_t)n + 1);
  if (le == hipSuccess && n > 0) {
    hipLaunchKernelGGL(boundary_flags_kernel, dim3(nblk(n)), dim3(256), 0, st, s, src, n, cm.shared_t, CB.flags);
    le = hipMemsetAsync(CB.flags + n, 0, sizeof(int), st);
    if (le == hipSuccess) le = scan_count(CB, CB.flags, CB.pos, n, &m, st);
  }
  if (le == hipSuccess) le = grow(CB.send, CB.cap_send, (size_t)std::max(m, 1));
  if (le == hipSuccess && m > 0) {
    hipLaunchKernelGGL(boundary_pack_kernel, dim3(nblk(n)), dim3(256), 0, st, src, n, CB.flags, CB.pos, cm.ids, CB.send);
    le = hipGetLastError();
  }
  // ---- header all-gather {error, count}: every rank learns every count (and any failure)
  int hdr[2] = {(int)le, m};
  std::vector<int> hall(2 * (size_t)G, 0);
  agreed = true;
  if (sh.exchange(hdr, sizeof(hdr), hall.data()) != 0) return hipErrorUnknown;
  int M = 0;
  std::vector<int> cnts(G, 0);
  for (int r = 0; r < G; ++r) {
    if (hall[2 * r] != 0 && le == hipSuccess) le = hipErrorUnknown;  // a peer failed
    cnts[r] = hall[2 * r + 1];
    M = std::max(M, cnts[r]);
  }
  FCHK(le);
  xstats[0] = m;
  for (int r = 0; r < G; ++r)
    if (r != me) xstats[1] += cnts[r];
  if (M == 0) return hipSuccess;
  // ---- records: fixed-size blocks of M per rank (device to device over RCCL when available)
  const size_t bytes = (size_t)M * sizeof(BRec);
  agreed = false;  // a local failure from here on is announced by the caller (loop header)
  FCHK(grow(CB.recv, CB.cap_recv, (size_t)M * G));
  if (sh.exchange_dev) {
    FCHK(grow_keep(CB.send, CB.cap_send, (size_t)M, (size_t)m, st));  // pad to M records (contents past m unused)
    if (sh.exchange_dev(CB.send, bytes, CB.recv, st) != 0) return hipErrorUnknown;
  } else {
    std::vector<char> hs(bytes, 0), hr(bytes * G);
    if (m) FCHK(hipMemcpy(hs.data(), CB.send, (size_t)m * sizeof(BRec), hipMemcpyDeviceToHost));
    if (sh.exchange(hs.data(), bytes, hr.data()) != 0) return hipErrorUnknown;
    FCHK(hipMemcpyAsync(CB.recv, hr.data(), bytes * G, hipMemcpyHostToDevice, st));
    FCHK(hipStreamSynchronize(st));
  }
  // ---- insertion (readPatches semantics), compacted in rank / record order after the model
  const size_t slots = (size_t)M * G;
  FCHK(grow(CB.ins, CB.cap_ins, slots));
  FCHK(grow(CB.flags, CB.cap_flags, slots + 1));
  FCHK(grow(CB.pos, CB.cap_pos, slots + 1));
  if (CB.cap_cnts < G) {
    if (CB.cnts) (void)hipFree(CB.cnts);
    CB.cnts = nullptr;
    FCHK(hipMalloc((void**)&CB.cnts, G * sizeof(int)));
    CB.cap_cnts = G;
  }
  FCHK(hipMemcpyAsync(CB.cnts, cnts.data(), G * sizeof(int), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(boundary_insert_kernel, dim3(nblk((long long)slots)), dim3(256), 0, st, s, CB.recv, G, M, me, CB.cnts,
                     cm.id2idx, cm.maxid, CB.ins, CB.flags);
  FCHK(hipMemsetAsync(CB.flags + slots, 0, sizeof(int), st));
  int added = 0;
  FCHK(scan_count(CB, CB.flags, CB.pos, (int)slots, &added, st));
  xstats[2] = added;
  if (added == 0) return hipSuccess;
  FCHK(grow_keep(dst, dst_cap, (size_t)n + added, (size_t)n, st));
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)slots), dim3(64), 0, st, CB.ins, (int)slots, CB.flags, CB.pos, dst + n);
  FCHK(hipGetLastError());
  *n_out = n + added;
  return hipSuccess;
}
}  // namespace pmvsdev
