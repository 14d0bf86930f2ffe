// pmvs_seed.hip -- the seed phase (PMVS3::CSeed, reference seed.cpp:11-414) on the device.
//
// The reference walks, per target image (std::shuffle(mt19937(42)) order, seed.cpp:53-60), every
// cell in raster order and every feature point of a cell; for each point it collects the
// feature points of the tau nearest images that lie within 2 px of the epipolar line
// (collectCells + computeEPD, seed.cpp:207-305), triangulates them (unproject, :340-384), sorts them
// by _response and refines them one after the other (initialMatchSub = preProcess -> refinePatch ->
// postProcess, :387-414) until two succeed, keeping the best.  Counts and cell occupancy written
// by earlier attempts decide which later cells/candidates are still tried (canAdd, :325-338).
//
// Device mapping:
//   * epipolar candidate collection -- one wavefront per (feature point, other image): lanes walk
//     the epipolar band row by row (64 rows at a time), test the feature points of the three
//     cells of a row (type, static mask, EPD < 2 in double) and emit them in the reference's
//     collection order through a wave prefix sum (count pass, scan, write pass).
//   * triangulation + checks + _response -- one thread per candidate (unproject in double, the
//     P[2]-depth test, getMask over all views, insideBimages).
//   * the per-point sort by _response -- a segmented radix sort of (_response, collection index)
//     keys (ties keep collection order; the reference sorts by heap address, seed.cpp:322, see
//     DESIGN.md).
//   * refinement -- the batched refine kernels (pmvs_kernels.hip).  A candidate's refinement
//     depends on the candidate only, so the host replays the reference's sequential control
//     (canAdd, counts, best selection, addPatch) exactly and refines SPECULATIVELY: each round it
//     requests, for the cells ahead of the replay cursor, the next few candidates whose outcome
//     is still unknown, refines them in one launch and replays as far as the results reach.  The
//     result is the CPU 1 result for any batch size.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstring>
#include <deque>
#include <memory>
#include <random>
#include <vector>

#include "pmvs_device.h"
#include "pmvs_launch.h"

namespace pmvsdev {

namespace {

constexpr int WAVE = 64;

#define SCHK(expr)                      \
  do {                                  \
    hipError_t e_ = (expr);             \
    if (e_ != hipSuccess) return e_;    \
  } while (0)

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (WAVE - 1)); }

// (int) of a float as x86-64 cvttss2si (out of range / NaN -> INT_MIN), the reference's platform.
__device__ __forceinline__ int cvt_int_x86f(float f) {
  if (!(f > -2147483904.0f && f < 2147483648.0f)) return (int)0x80000000;
  return (int)f;
}

// CImage::getMask(int, int, level), image.hpp:553-565.
__device__ __forceinline__ int mask_at(const DScene& s, const DView& v, int ix, int iy) {
  if (v.mask_off[s.level] < 0) return 1;
  if (ix < 0 || v.w[s.level] <= ix || iy < 0 || v.h[s.level] <= iy) return 1;
  return s.masks[v.mask_off[s.level] + (long long)iy * v.w[s.level] + ix];
}

// Image::computeEPD<double>, camera.hpp:119-127.
__device__ __forceinline__ float compute_epd(const double* F, double p0x, double p0y, double p1x, double p1y) {
  double l0 = F[0] * p1x + F[1] * p1y + F[2] * 1.0;
  double l1 = F[3] * p1x + F[4] * p1y + F[5] * 1.0;
  double l2 = F[6] * p1x + F[7] * p1y + F[8] * 1.0;
  const double f = __builtin_sqrt(l0 * l0 + l1 * l1);
  if (f == 0.0) return 0.0f;
  l0 /= f; l1 /= f; l2 /= f;
  return (float)fabs(l0 * p0x + l1 * p0y + l2 * 1.0);
}

// One (feature point, other image) pair of CSeed::collectCandidates (seed.cpp:271-306): the cell
// walk of collectCells (seed.cpp:207-267), canAdd's static mask test, the type test and the EPD
// test.  COUNT: cnt[pair] = hits.  !COUNT: hits written from out_off[pair] in collection order.
struct EpiArgs {
  const float* px;      // feature x of the pair's point (level coordinates), per pair source point
  const float* py;
  const int* ptype;
  int npairs, nidx;     // pairs = p0 * nidx + jj
  const int* p0pts;     // global point index of each p0
  const double* F;      // nidx x 9 (setF(index, indexes[jj]))
  const int* views;     // nidx image indexes
  const int* cell_off;  // per view base into cells: CSR offsets of points by cell (gw*gh+1 per view)
  const long long* view_cell_base;
  const int* cell_pts;  // global point indexes, grouped by cell, cell order then detector order
  int* cnt;
  const long long* out_off;
  int* out_pt;          // global point index of each hit
  int* out_cell;        // its cell in the other image
  int* out_view;
};

template <bool COUNT>
__global__ void __launch_bounds__(64) epi_kernel(DScene s, EpiArgs a) {
  const int lane = lane_id();
  for (int pair = blockIdx.x; pair < a.npairs; pair += gridDim.x) {
    const int p0 = pair / a.nidx, jj = pair % a.nidx;
    const int gp0 = a.p0pts[p0];
    const float x0 = a.px[gp0], y0 = a.py[gp0];
    const int type0 = a.ptype[gp0];
    const int j = a.views[jj];
    const DView& v = s.views[j];
    const int gw = (v.w[s.level] + s.csize - 1) / s.csize, gh = (v.h[s.level] + s.csize - 1) / s.csize;
    const double* F = a.F + 9 * jj;
    // transpose(F) * point
    const double pt0 = x0, pt1 = y0, pt2 = 1.0;
    const double l0 = F[0] * pt0 + F[3] * pt1 + F[6] * pt2;
    const double l1 = F[1] * pt0 + F[4] * pt1 + F[7] * pt2;
    const double l2 = F[2] * pt0 + F[5] * pt1 + F[8] * pt2;
    long long base = COUNT ? 0 : a.out_off[pair];
    int total = 0;
    if (!(l0 == 0.0 && l1 == 0.0)) {
      const bool vertical = fabs(l0) > fabs(l1);
      const int nrow = vertical ? gh : gw;
      const int* coff = a.cell_off + a.view_cell_base[j] + j;  // gw*gh+1 entries per view
      for (int r0 = 0; r0 < nrow; r0 += WAVE) {
        const int r = r0 + lane;
        int cells[3] = {-1, -1, -1};
        if (r < nrow) {
          const float lo = -2147483648.0f, hi = 2147483648.0f;
          const float f = (float)((r + 0.5) * s.csize - 0.5f);
          float g = vertical ? (float)((-l1 * f - l2) / l0) : (float)((-l0 * f - l2) / l1);
          g = smax(lo, smin(hi, g));
          const int ig = cvt_int_x86f(floorf(g + 0.5f)) / s.csize;
          const int lim = vertical ? gw : gh;
          const int cand[3] = {ig, ig - 1, ig + 1};
          for (int k = 0; k < 3; ++k) {
            const int c = cand[k];
            if (0 <= c && c < lim) {
              const int cx = vertical ? c : r, cy = vertical ? r : c;
              if (mask_at(s, v, s.csize * cx, s.csize * cy)) cells[k] = cy * gw + cx;
            }
          }
        }
        // hits of this lane's row, in cell order then point order
        int mine = 0;
        for (int k = 0; k < 3; ++k) {
          if (cells[k] < 0) continue;
          const int b = coff[cells[k]], e = coff[cells[k] + 1];
          for (int q = b; q < e; ++q) {
            const int gq = a.cell_pts[q];
            if (a.ptype[gq] != type0) continue;
            if (2.0f <= compute_epd(F, pt0, pt1, (double)a.px[gq], (double)a.py[gq])) continue;
            ++mine;
          }
        }
        // wave-ordered exclusive prefix of the per-lane counts
        int incl = mine;
        for (int d = 1; d < WAVE; d <<= 1) {
          const int t = __shfl_up(incl, d, WAVE);
          if (lane >= d) incl += t;
        }
        const int sum = __shfl(incl, WAVE - 1, WAVE);
        if (!COUNT && mine) {
          long long w = base + total + (incl - mine);
          for (int k = 0; k < 3; ++k) {
            if (cells[k] < 0) continue;
            const int b = coff[cells[k]], e = coff[cells[k] + 1];
            for (int q = b; q < e; ++q) {
              const int gq = a.cell_pts[q];
              if (a.ptype[gq] != type0) continue;
              if (2.0f <= compute_epd(F, pt0, pt1, (double)a.px[gq], (double)a.py[gq])) continue;
              a.out_pt[w] = gq;
              a.out_cell[w] = cells[k];
              a.out_view[w] = j;
              ++w;
            }
          }
        }
        total += sum;
      }
    }
    if (COUNT && lane == 0) a.cnt[pair] = total;
  }
}

// CSeed::unproject (seed.cpp:340-384) and the checks of collectCandidates (seed.cpp:310-320):
// the triangulated point, the reference view's P[2] depth test, CPhotoSetS::getMask over all
// views, CFindMatch::insideBimages, and _response.  key = _response (valid) or +inf (dropped).
__global__ void __launch_bounds__(256) tri_kernel(DScene s, int index, long long n, const int* p0_of, const int* p0pts,
                                                  const float* px, const float* py, const int* cpt, const int* cview,
                                                  float* coord4, unsigned long long* key) {
  for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < n; c += (long long)gridDim.x * blockDim.x) {
    const int g0 = p0pts[p0_of[c]], g1 = cpt[c];
    const float ax = px[g0], ay = py[g0], bx = px[g1], by = py[g1];
    const DView& v0 = s.views[index];
    const DView& v1 = s.views[cview[c]];
    const float* P0 = v0.P[s.level];
    const float* P1 = v1.P[s.level];
    double A[4][3], bb[4];
    for (int k = 0; k < 3; ++k) {
      A[0][k] = (double)(P0[k] - ax * P0[8 + k]);
      A[1][k] = (double)(P0[4 + k] - ay * P0[8 + k]);
      A[2][k] = (double)(P1[k] - bx * P1[8 + k]);
      A[3][k] = (double)(P1[4 + k] - by * P1[8 + k]);
    }
    bb[0] = (double)(ax * P0[11] - P0[3]);
    bb[1] = (double)(ay * P0[11] - P0[7]);
    bb[2] = (double)(bx * P1[11] - P1[3]);
    bb[3] = (double)(by * P1[11] - P1[7]);
    double M[3][3], r[3];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) M[i][j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
      r[i] = A[0][i] * bb[0] + A[1][i] * bb[1] + A[2][i] * bb[2] + A[3][i] * bb[3];
    }
    double ad[3][3];
    ad[0][0] = M[1][1] * M[2][2] - M[2][1] * M[1][2];
    ad[0][1] = -M[1][0] * M[2][2] + M[2][0] * M[1][2];
    ad[0][2] = M[1][0] * M[2][1] - M[2][0] * M[1][1];
    ad[1][0] = M[2][1] * M[0][2] - M[0][1] * M[2][2];
    ad[1][1] = -M[2][0] * M[0][2] + M[0][0] * M[2][2];
    ad[1][2] = M[2][0] * M[0][1] - M[0][0] * M[2][1];
    ad[2][0] = M[0][1] * M[1][2] - M[1][1] * M[0][2];
    ad[2][1] = -M[0][0] * M[1][2] + M[1][0] * M[0][2];
    ad[2][2] = M[0][0] * M[1][1] - M[1][0] * M[0][1];
    const double d = ad[0][0] * M[0][0] + ad[0][1] * M[0][1] + ad[0][2] * M[0][2];
    float co[4];
    for (int i = 0; i < 3; ++i) {
      double o = 0.0;
      if (d != 0.0) {
        const double i0 = ad[0][i] / d, i1 = ad[1][i] / d, i2 = ad[2][i] / d;
        o = i0 * r[0] + i1 * r[1] + i2 * r[2];
      }
      co[i] = (float)o;
    }
    co[3] = 1.0f;
    bool ok = !(dot4(P0 + 8, co) <= 0.0f);
    if (ok && s.anyMask)
      for (int k = 0; k < s.num && ok; ++k)
        if (get_mask(s, s.views[k], co, s.level) == 0) ok = false;
    for (int b = 0; b < s.nb && ok; ++b) {
      const DView& vb = s.views[s.bindexes[b]];
      float ic[3];
      project(vb, co, s.level, ic);
      if (ic[0] < 0.0f || (float)(vb.w[s.level] - 1) < ic[0] || ic[1] < 0.0f || (float)(vb.h[s.level] - 1) < ic[1]) ok = false;
    }
    float resp = __builtin_inff();
    if (ok) {
      const float d0[4] = {co[0] - v0.center[0], co[1] - v0.center[1], co[2] - v0.center[2], co[3] - v0.center[3]};
      const float d1[4] = {co[0] - v1.center[0], co[1] - v1.center[1], co[2] - v1.center[2], co[3] - v1.center[3]};
      resp = fabsf(norm4(d0) - norm4(d1));
    }
    for (int k = 0; k < 4; ++k) coord4[4 * c + k] = co[k];
    // sort key: _response bits (non-negative floats order as unsigned), dropped candidates last;
    // the low word keeps the collection index, so equal responses stay in collection order
    const unsigned int hi = ok ? __float_as_uint(resp) : 0xFFFFFFFFu;
    key[c] = ((unsigned long long)hi << 32) | (unsigned long long)(unsigned int)c;
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------ host
namespace {

// Image::setF<double> (camera.hpp:130-151) from the float level projections.
void set_f(const DView& a, const DView& b, int level, double* F) {
  double p0[3][4], p1[3][4];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) {
      p0[r][c] = a.P[level][4 * r + c];
      p1[r][c] = b.P[level][4 * r + c];
    }
  auto det4 = [](const double* A, const double* B, const double* Cc, const double* D) {
    const double d1 = (Cc[2] * D[3]) - (Cc[3] * D[2]);
    const double d2 = (Cc[1] * D[3]) - (Cc[3] * D[1]);
    const double d3 = (Cc[1] * D[2]) - (Cc[2] * D[1]);
    const double d4 = (Cc[0] * D[3]) - (Cc[3] * D[0]);
    const double d5 = (Cc[0] * D[2]) - (Cc[2] * D[0]);
    const double d6 = (Cc[0] * D[1]) - (Cc[1] * D[0]);
    const double x0 = -B[1] * d1 + B[2] * d2 - B[3] * d3;
    const double x1 = B[0] * d1 - B[2] * d4 + B[3] * d5;
    const double x2 = -B[0] * d2 + B[1] * d4 - B[3] * d6;
    const double x3 = B[0] * d3 - B[1] * d5 + B[2] * d6;
    return A[0] * x0 + A[1] * x1 + A[2] * x2 + A[3] * x3;
  };
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) F[3 * i + j] = det4(p0[(i + 1) % 3], p0[(i + 2) % 3], p1[(j + 1) % 3], p1[(j + 2) % 3]);
}

inline float hdot4(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3]; }

template <class T>
struct DArr {
  T* p = nullptr;
  size_t n = 0;
  hipError_t need(size_t m) {
    if (m <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = std::max<size_t>(m, 1);
    return hipMalloc((void**)&p, n * sizeof(T));
  }
  ~DArr() {
    if (p) (void)hipFree(p);
  }
};

struct Cand {       // one epipolar candidate of a feature point (static part)
  int view, point;  // image index, global point index
  int cell;         // its cell in that image
  float coord[4];
};

}  // namespace

hipError_t seed_pass(const DScene& s, const std::vector<DView>& hv, const SeedInput& in, hipStream_t st,
                     const RefineFn& refine, SeedOutput& out) {
  const auto t_start = std::chrono::steady_clock::now();
  const int num = s.num, tnum = s.tnum, csize = s.csize, level = s.level;
  out.seeds.clear();
  std::memset(out.stats, 0, sizeof(out.stats));
  std::vector<int> gw(num), gh(num);
  for (int i = 0; i < num; ++i) {
    gw[i] = (hv[i].w[level] + csize - 1) / csize;
    gh[i] = (hv[i].h[level] + csize - 1) / csize;
  }
  // ---- CSeed::readPoints (seed.cpp:24-35): points bucketed by cell, detector order per cell
  std::vector<long long> vbase(num + 1, 0), cbase(num + 1, 0);
  for (int i = 0; i < num; ++i) {
    vbase[i + 1] = vbase[i] + in.npts[i];
    cbase[i + 1] = cbase[i] + (long long)gw[i] * gh[i];
  }
  const long long NP = vbase[num];
  std::vector<float> hx(std::max<long long>(NP, 1)), hy(std::max<long long>(NP, 1));
  std::vector<int> htype(std::max<long long>(NP, 1)), pcell(std::max<long long>(NP, 1), -1);
  std::vector<int> coff(cbase[num] + num, 0);  // per view gw*gh+1 offsets (relative to the view's points)
  std::vector<int> cpts(std::max<long long>(NP, 1));
  for (int i = 0; i < num; ++i) {
    const long long ncell = (long long)gw[i] * gh[i];
    int* off = coff.data() + cbase[i] + i;
    std::vector<int> cnt(ncell + 1, 0);
    for (long long q = vbase[i]; q < vbase[i + 1]; ++q) {
      const pmvs_point& p = in.points[q];
      hx[q] = p.x;
      hy[q] = p.y;
      htype[q] = p.type;
      const int ix = ((int)std::floor(p.x + 0.5f)) / csize, iy = ((int)std::floor(p.y + 0.5f)) / csize;
      const long long c = (long long)iy * gw[i] + ix;  // the reference's index2 (seed.cpp:29-31)
      if (c < 0 || c >= ncell) continue;                // outside _ppoints[index]: undefined there; dropped
      pcell[q] = (int)c;
      cnt[c + 1]++;
    }
    for (long long c = 0; c < ncell; ++c) cnt[c + 1] += cnt[c];
    for (long long c = 0; c <= ncell; ++c) off[c] = (int)(vbase[i] + cnt[c]);
    std::vector<int> fillp(cnt.begin(), cnt.end() - 1);
    for (long long q = vbase[i]; q < vbase[i + 1]; ++q)
      if (pcell[q] >= 0) cpts[vbase[i] + fillp[pcell[q]]++] = (int)q;
  }
  // ---- CPhotoSetS::setDistances (photoSetS.cpp:195-234) and COptim::collectImages (optim.cpp:66-93)
  std::vector<std::vector<float>> dist(num, std::vector<float>(num, 0.0f));
  {
    float avedis = 0.0f;
    int denom = 0;
    for (int i = 0; i < num; ++i)
      for (int j = 0; j < num; ++j) {
        if (i == j) continue;
        const float d[4] = {hv[i].center[0] - hv[j].center[0], hv[i].center[1] - hv[j].center[1],
                            hv[i].center[2] - hv[j].center[2], hv[i].center[3] - hv[j].center[3]};
        const float f = (float)std::sqrt((double)hdot4(d, d));
        dist[i][j] = f;
        avedis += f;
        denom++;
      }
    if (denom > 0) {
      avedis /= denom;
      const float margin = (float)std::cos(10.0f * M_PI / 180.0f);
      for (int i = 0; i < num; ++i) {
        const float r0[4] = {hv[i].oaxis[0], hv[i].oaxis[1], hv[i].oaxis[2], 0.0f};
        for (int j = 0; j < num; ++j) {
          const float r1[4] = {hv[j].oaxis[0], hv[j].oaxis[1], hv[j].oaxis[2], 0.0f};
          dist[i][j] /= avedis;
          dist[i][j] += std::max(0.0f, 1.0f - hdot4(r0, r1) - margin);
        }
      }
    }
  }
  auto collect_images = [&](int index, std::vector<int>& idx) {
    idx.clear();
    const float r0[4] = {hv[index].oaxis[0], hv[index].oaxis[1], hv[index].oaxis[2], 0.0f};
    struct V2 { float a, b; };
    std::vector<V2> c;
    for (int k = in.vis_off[index]; k < in.vis_off[index + 1]; ++k) {
      const int t = in.vis[k];
      if (in.sequence != -1 && in.sequence < std::abs(index - t)) continue;
      const float r1[4] = {hv[t].oaxis[0], hv[t].oaxis[1], hv[t].oaxis[2], 0.0f};
      if ((double)hdot4(r0, r1) < std::cos((double)in.angle0)) continue;
      c.push_back({dist[index][t], (float)t});
    }
    std::sort(c.begin(), c.end(), [](const V2& l, const V2& r) { return l.a < r.a || (l.a == r.a && l.b < r.b); });
    for (int i = 0; i < std::min(s.tau, (int)c.size()); ++i) idx.push_back((int)c[i].b);
  };
  // ---- device copies of the points
  DArr<float> dx, dy;
  DArr<int> dtype, dcoff, dcpts, dviews, dp0pts, dcnt, dpt, dcell, dview, dp0of;
  DArr<long long> dvbase, doff;
  DArr<double> dF;
  DArr<float> dcoord;
  DArr<unsigned long long> dkey, dkey2;
  DArr<char> dtemp;
  SCHK(dx.need(hx.size()));
  SCHK(dy.need(hy.size()));
  SCHK(dtype.need(htype.size()));
  SCHK(dcoff.need(coff.size()));
  SCHK(dcpts.need(cpts.size()));
  SCHK(dvbase.need(cbase.size()));
  SCHK(hipMemcpyAsync(dx.p, hx.data(), hx.size() * sizeof(float), hipMemcpyHostToDevice, st));
  SCHK(hipMemcpyAsync(dy.p, hy.data(), hy.size() * sizeof(float), hipMemcpyHostToDevice, st));
  SCHK(hipMemcpyAsync(dtype.p, htype.data(), htype.size() * sizeof(int), hipMemcpyHostToDevice, st));
  SCHK(hipMemcpyAsync(dcoff.p, coff.data(), coff.size() * sizeof(int), hipMemcpyHostToDevice, st));
  SCHK(hipMemcpyAsync(dcpts.p, cpts.data(), cpts.size() * sizeof(int), hipMemcpyHostToDevice, st));
  SCHK(hipMemcpyAsync(dvbase.p, cbase.data(), cbase.size() * sizeof(long long), hipMemcpyHostToDevice, st));
  // ---- replay state (CPatchOrganizerS::_counts / _pgrids occupancy of the target images)
  std::vector<std::vector<unsigned char>> counts(tnum), occupied(tnum);
  for (int t = 0; t < tnum; ++t) {
    counts[t].assign((size_t)gw[t] * gh[t], 0);
    occupied[t].assign((size_t)gw[t] * gh[t], 0);
  }
  auto can_add = [&](int index, int x, int y) -> bool {  // CSeed::canAdd, seed.cpp:325-338
    const DView& v = hv[index];
    const int ix = csize * x, iy = csize * y;
    if (v.mask_off[level] >= 0 && !(ix < 0 || v.w[level] <= ix || iy < 0 || v.h[level] <= iy) &&
        !in.mask_level[index][(size_t)iy * v.w[level] + ix])
      return false;
    if (tnum <= index) return true;
    const size_t c = (size_t)y * gw[index] + x;
    if (occupied[index][c]) return false;
    if (2 <= counts[index][c]) return false;  // _countThreshold2
    return true;
  };
  // order of the target images (seed.cpp:53-60); std::shuffle with libstdc++, as the reference
  std::vector<int> order(tnum);
  for (int i = 0; i < tnum; ++i) order[i] = i;
  {
    std::mt19937 gen(42);
    std::shuffle(order.begin(), order.end(), gen);
  }
  DArr<pmvs_candidate> dcand;
  DArr<pmvs_refined> dres;
  std::vector<pmvs_candidate> hcand;
  std::vector<pmvs_refined> hres;
  const int budget = std::max(1, in.batch);
  const int per_cell = std::max(1, in.per_cell);
  const int lookahead = std::max(1, in.lookahead);
  const int spec_near = std::max(1, in.spec_near);
  long long refined = 0, rounds = 0;
  double gen_ms = 0.0, refine_wall_ms = 0.0;
  // ---- per target image: its epipolar candidates (gen) and its exact-replay state.  Images are
  // replayed one after the other in `order`; the speculation may already request candidates of the
  // next `lookahead - 1` images while the current one drains: a refine result is a pure function of
  // the candidate, and which results the replay will read depends only on the occupancy / counts,
  // which only grow -- a request made against the current state is a superset of the later need.
  struct Img {
    int index = -1;
    std::vector<int> p0pts, p0cell, cellstart, sorted, soff, accepted_slot, creq, vcp;
    std::vector<unsigned char> drained;  // per cell: a full walk found no unknown candidate left
    std::vector<Cand> cands;
    std::vector<unsigned char> state;  // per candidate: 0 unknown, 1 requested, 2 failed in preProcess,
                                       // 3 failed in postProcess, 4 accepted
    std::vector<pmvs_refined> accepted;
    int ci = 0, pi = 0, vi = 0, count = 0, best = -1;  // replay cursor
    int frontier = 0;                                   // first cell no speculation walk reached
    bool in_point = false;
    float best_score = 0.0f;
    int ncells() const { return (int)cellstart.size() - 1; }
  };
  std::vector<int> idx;
  auto gen = [&](int index, Img& w) -> hipError_t {  // w.index stays -1 for an image without work
    collect_images(index, idx);
    if ((int)idx.size() > s.tau) idx.resize(s.tau);
    if (idx.empty()) return hipSuccess;
    const int nidx = (int)idx.size();
    // replay order: cells with points in raster order, their points in cell order
    std::vector<int>& p0pts = w.p0pts;
    std::vector<int>& p0cell = w.p0cell;
    std::vector<int>& cellstart = w.cellstart;
    {
      const int* off = coff.data() + cbase[index] + index;
      const long long ncell = (long long)gw[index] * gh[index];
      for (long long c = 0; c < ncell; ++c) {
        if (off[c] == off[c + 1]) continue;
        cellstart.push_back((int)p0pts.size());
        for (int q = off[c]; q < off[c + 1]; ++q) {
          p0pts.push_back(cpts[q]);
          p0cell.push_back((int)c);
        }
      }
      cellstart.push_back((int)p0pts.size());
    }
    const int np0 = (int)p0pts.size();
    if (np0 == 0) return hipSuccess;
    const auto tg0 = std::chrono::steady_clock::now();
    // ---- epipolar candidates of every point of this image (device), sorted per point
    std::vector<double> F(9 * nidx);
    for (int jj = 0; jj < nidx; ++jj) set_f(hv[index], hv[idx[jj]], level, F.data() + 9 * jj);
    const long long npairs = (long long)np0 * nidx;
    SCHK(dviews.need(nidx));
    SCHK(dF.need(9 * nidx));
    SCHK(dp0pts.need(np0));
    SCHK(dcnt.need(npairs + 1));
    SCHK(doff.need(npairs + 1));
    SCHK(hipMemcpyAsync(dviews.p, idx.data(), nidx * sizeof(int), hipMemcpyHostToDevice, st));
    SCHK(hipMemcpyAsync(dF.p, F.data(), 9 * nidx * sizeof(double), hipMemcpyHostToDevice, st));
    SCHK(hipMemcpyAsync(dp0pts.p, p0pts.data(), np0 * sizeof(int), hipMemcpyHostToDevice, st));
    EpiArgs ea{};
    ea.px = dx.p; ea.py = dy.p; ea.ptype = dtype.p;
    ea.npairs = (int)npairs; ea.nidx = nidx; ea.p0pts = dp0pts.p; ea.F = dF.p; ea.views = dviews.p;
    ea.cell_off = dcoff.p; ea.view_cell_base = dvbase.p; ea.cell_pts = dcpts.p;
    ea.cnt = dcnt.p; ea.out_off = doff.p;
    const int egrid = (int)std::min<long long>(npairs, 1 << 20);
    hipLaunchKernelGGL((epi_kernel<true>), dim3(egrid), dim3(64), 0, st, s, ea);
    SCHK(hipGetLastError());
    std::vector<int> hcnt(npairs);
    SCHK(hipMemcpyAsync(hcnt.data(), dcnt.p, npairs * sizeof(int), hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    std::vector<long long> hoff(npairs + 1, 0);
    for (long long k = 0; k < npairs; ++k) hoff[k + 1] = hoff[k] + hcnt[k];
    const long long nc = hoff[npairs];
    std::vector<int>& sorted = w.sorted;  // candidate ids per point in _response order (valid ones), CSR by p0
    std::vector<int>& soff = w.soff;
    soff.assign(np0 + 1, 0);
    std::vector<Cand>& cands = w.cands;
    cands.resize(std::max<long long>(nc, 1));
    if (nc > 0) {
      if (nc > INT_MAX / 2) return hipErrorOutOfMemory;
      SCHK(hipMemcpyAsync(doff.p, hoff.data(), (npairs + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
      SCHK(dpt.need(nc)); SCHK(dcell.need(nc)); SCHK(dview.need(nc)); SCHK(dp0of.need(nc));
      SCHK(dkey.need(nc)); SCHK(dkey2.need(nc)); SCHK(dcoord.need(4 * nc));
      ea.out_pt = dpt.p; ea.out_cell = dcell.p; ea.out_view = dview.p;
      hipLaunchKernelGGL((epi_kernel<false>), dim3(egrid), dim3(64), 0, st, s, ea);
      SCHK(hipGetLastError());
      std::vector<int> p0of(nc);
      for (long long k = 0; k < npairs; ++k)
        for (long long c = hoff[k]; c < hoff[k + 1]; ++c) p0of[c] = (int)(k / nidx);
      SCHK(hipMemcpyAsync(dp0of.p, p0of.data(), nc * sizeof(int), hipMemcpyHostToDevice, st));
      const int tgrid = (int)std::min<long long>((nc + 255) / 256, 65536);
      hipLaunchKernelGGL(tri_kernel, dim3(tgrid), dim3(256), 0, st, s, index, nc, dp0of.p, dp0pts.p, dx.p, dy.p, dpt.p,
                         dview.p, dcoord.p, dkey.p);
      SCHK(hipGetLastError());
      // stable segmented sort by _response within each point's candidates
      std::vector<int> segb(np0 + 1);
      for (int p = 0; p <= np0; ++p) segb[p] = (int)hoff[(long long)p * nidx];
      DArr<int> dsegb;
      SCHK(dsegb.need(np0 + 1));
      SCHK(hipMemcpyAsync(dsegb.p, segb.data(), (np0 + 1) * sizeof(int), hipMemcpyHostToDevice, st));
      size_t tb = 0;
      SCHK(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tb, dkey.p, dkey2.p, (int)nc, np0, dsegb.p, dsegb.p + 1,
                                                      0, 64, st));
      SCHK(dtemp.need(tb));
      SCHK(hipcub::DeviceSegmentedRadixSort::SortKeys(dtemp.p, tb, dkey.p, dkey2.p, (int)nc, np0, dsegb.p, dsegb.p + 1,
                                                      0, 64, st));
      std::vector<unsigned long long> hkey(nc);
      std::vector<int> hpt(nc), hcell(nc), hview(nc);
      std::vector<float> hcoord(4 * nc);
      SCHK(hipMemcpyAsync(hkey.data(), dkey2.p, nc * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
      SCHK(hipMemcpyAsync(hpt.data(), dpt.p, nc * sizeof(int), hipMemcpyDeviceToHost, st));
      SCHK(hipMemcpyAsync(hcell.data(), dcell.p, nc * sizeof(int), hipMemcpyDeviceToHost, st));
      SCHK(hipMemcpyAsync(hview.data(), dview.p, nc * sizeof(int), hipMemcpyDeviceToHost, st));
      SCHK(hipMemcpyAsync(hcoord.data(), dcoord.p, 4 * nc * sizeof(float), hipMemcpyDeviceToHost, st));
      SCHK(hipStreamSynchronize(st));
      for (long long c = 0; c < nc; ++c) {
        Cand& k = cands[c];
        k.view = hview[c];
        k.point = hpt[c];
        k.cell = hcell[c];
        for (int q = 0; q < 4; ++q) k.coord[q] = hcoord[4 * c + q];
      }
      for (int p = 0; p < np0; ++p) {
        for (int c = segb[p]; c < segb[p + 1]; ++c)
          if ((hkey[c] >> 32) != 0xFFFFFFFFull) sorted.push_back((int)(hkey[c] & 0xFFFFFFFFull));
        soff[p + 1] = (int)sorted.size();
      }
    }
    gen_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tg0).count();
    out.stats[6] += nc;
    w.state.assign(std::max<long long>(nc, 1), 0);
    w.accepted_slot.assign(std::max<long long>(nc, 1), -1);
    w.creq.assign(std::max(w.ncells(), 1), 0);
    w.drained.assign(std::max(w.ncells(), 1), 0);
    w.index = index;
    return hipSuccess;
  };
  auto filtered = [&](const Img& w, int p, std::vector<int>& v) {  // canAdd filter of collectCandidates now
    v.clear();
    for (int k = w.soff[p]; k < w.soff[p + 1]; ++k) {
      const Cand& c = w.cands[w.sorted[k]];
      const int x = c.cell % gw[c.view], y = c.cell / gw[c.view];
      if (can_add(c.view, x, y)) v.push_back(w.sorted[k]);
    }
  };
  auto make_candidate = [&](const Img& w, int cid, pmvs_candidate& pc) {  // seed.cpp:167-173
    const Cand& c = w.cands[cid];
    std::memset(&pc, 0, sizeof(pc));
    float n[4] = {hv[w.index].center[0] - c.coord[0], hv[w.index].center[1] - c.coord[1],
                  hv[w.index].center[2] - c.coord[2], hv[w.index].center[3] - c.coord[3]};
    const float l = hdot4(n, n);
    if (l != 1.0 && l != 0.0) {
      const float d = (float)std::sqrt((double)l);
      for (int k = 0; k < 4; ++k) n[k] /= d;
    }
    n[3] = 0.0f;
    for (int k = 0; k < 4; ++k) { pc.coord[k] = c.coord[k]; pc.normal[k] = n[k]; }
    pc.dscale = 0.0f;
    pc.num_images = 2;
    pc.images[0] = w.index;
    pc.images[1] = c.view;
  };
  auto score = [&](const pmvs_refined& r) { return std::max(0.0f, r.ncc - s.nccThreshold) * r.num_images; };
  auto finish_point = [&](Img& w) {  // seed.cpp:194-199
    if (w.count != 0) {
      if (w.best >= 0) {
        const pmvs_refined& r = w.accepted[w.best];
        pmvs_patch pp;
        std::memset(&pp, 0, sizeof(pp));
        for (int k = 0; k < 4; ++k) { pp.coord[k] = r.coord[k]; pp.normal[k] = r.normal[k]; }
        pp.ncc = r.ncc; pp.dscale = r.dscale; pp.ascale = r.ascale; pp.tmp = r.tmp; pp.timages = r.timages;
        pp.num_images = r.num_images;
        for (int k = 0; k < r.num_images; ++k) {
          pp.images[k] = (int16_t)r.images[k];
          pp.grids[k][0] = grid16(r.grids[k][0]);
          pp.grids[k][1] = grid16(r.grids[k][1]);
          const int t = r.images[k];
          if (t < tnum && 0 <= r.grids[k][0] && r.grids[k][0] < gw[t] && 0 <= r.grids[k][1] && r.grids[k][1] < gh[t])
            occupied[t][(size_t)r.grids[k][1] * gw[t] + r.grids[k][0]] = 1;  // addPatch at depth 0
        }
        out.seeds.push_back(pp);
      }
      ++w.ci;  // break out of the point loop: next cell
      w.pi = 0;
    } else {
      ++w.pi;
    }
    w.in_point = false;
  };
  // the exact replay of image w (the current one); returns -1 when the image is done, else the
  // candidate whose result is needed
  auto replay = [&](Img& w) -> int {
    const int index = w.index;
    while (w.ci < w.ncells()) {
      if (!w.in_point) {
        const int npts_cell = w.cellstart[w.ci + 1] - w.cellstart[w.ci];
        if (w.pi == 0) {
          const int c = w.p0cell[w.cellstart[w.ci]];
          if (!can_add(index, c % gw[index], c / gw[index])) { ++w.ci; continue; }
        }
        if (w.pi >= npts_cell) { ++w.ci; w.pi = 0; continue; }
        filtered(w, w.cellstart[w.ci] + w.pi, w.vcp);
        w.vi = 0; w.count = 0; w.best = -1; w.best_score = 0.0f;
        w.in_point = true;
      }
      if (w.vi >= (int)w.vcp.size()) { finish_point(w); continue; }
      const int cid = w.vcp[w.vi];
      if (w.state[cid] < 2) return cid;
      const Cand& c = w.cands[cid];
      const int cell = w.p0cell[w.cellstart[w.ci]];
      ++counts[index][cell];
      if (c.view < tnum) ++counts[c.view][c.cell];
      out.stats[0]++;  // trial
      if (w.state[cid] == 2) { out.stats[2]++; ++w.vi; continue; }
      if (w.state[cid] == 3) { out.stats[3]++; ++w.vi; continue; }
      out.stats[1]++;  // pass
      ++w.count;
      const float sc = score(w.accepted[w.accepted_slot[cid]]);
      if (w.best_score < sc) { w.best_score = sc; w.best = w.accepted_slot[cid]; }
      if (2 <= w.count) { finish_point(w); continue; }
      ++w.vi;
    }
    return -1;
  };
  // requests for image w's cells from its cursor on, against the current state (read-only), until
  // `limit` requests.  A cell whose earlier requests all failed gets twice as many the next time
  // (creq: requests so far), so a point that tries many epipolar candidates before two succeed
  // costs O(log) rounds, not one round per per_cell candidates; the replay is exact whatever was
  // requested.
  std::vector<int> tmpv;
  // The walk covers the `near` cells from the cursor on (where the replay will block next, so their
  // doubling quotas matter) and then continues from the frontier, the first cell no walk has reached
  // yet: the cells in between were requested once and are re-walked when the cursor nears them,
  // which keeps a round's host work O(near + new cells) instead of O(cells left in the image).
  auto speculate = [&](Img& w, std::vector<int>& req, int limit) {
    req.clear();
    int c2 = w.ci, p2 = w.pi;
    bool first = true;
    const int index = w.index;
    const int near_end = (int)std::min<long long>(w.ncells(), (long long)w.ci + spec_near);
    while (c2 < w.ncells() && (int)req.size() < limit) {
      if (c2 == near_end && c2 < w.frontier) c2 = w.frontier;
      if (c2 >= w.ncells()) break;
      // a cell whose walk went through every point and found every candidate requested or
      // resolved stays so (states never return to unknown, and canAdd only removes candidates):
      // later walks skip it
      if (w.drained[c2] && !(first && w.in_point)) { ++c2; p2 = 0; first = false; continue; }
      const bool full_walk = !(first && w.in_point) && p2 == 0;
      int unknown = 0;
      const int quota = std::min(4096, std::max(per_cell, w.creq[c2]));
      bool cell_done = false;
      const int npts_cell = w.cellstart[c2 + 1] - w.cellstart[c2];
      if (!(first && w.in_point) && p2 == 0) {
        const int c = w.p0cell[w.cellstart[c2]];
        if (!can_add(index, c % gw[index], c / gw[index])) { ++c2; p2 = 0; first = false; continue; }
      }
      for (; p2 < npts_cell && !cell_done && unknown < quota; ++p2) {
        int v0 = 0, cnt = 0;
        const std::vector<int>* list;
        if (first && w.in_point) { list = &w.vcp; v0 = w.vi; cnt = w.count; }
        else { filtered(w, w.cellstart[c2] + p2, tmpv); list = &tmpv; }
        first = false;
        for (int k = v0; k < (int)list->size(); ++k) {
          const int cid = (*list)[k];
          if (w.state[cid] == 4) {
            if (2 <= ++cnt) break;
          } else if (w.state[cid] == 0) {
            w.state[cid] = 1;
            req.push_back(cid);
            if (++unknown >= quota) break;
          }
        }
        if (cnt > 0) cell_done = true;  // this point adds a patch: the cell is finished
      }
      // (not after a point with an accepted candidate ended the walk: canAdd may still drop that
      // candidate before the replay gets there, and the cell's later points then matter)
      if (full_walk && unknown == 0 && !cell_done) w.drained[c2] = 1;
      w.creq[c2] += unknown;
      first = false;
      ++c2;
      p2 = 0;
    }
    w.frontier = std::max(w.frontier, c2);
  };
  std::deque<std::unique_ptr<Img>> win;  // the current image and the look-ahead ones, in `order`
  size_t next = 0;
  auto fill = [&](size_t k) -> hipError_t {
    while (win.size() < k && next < order.size()) {
      auto w = std::make_unique<Img>();
      SCHK(gen(order[next++], *w));
      if (w->index >= 0) win.push_back(std::move(w));
    }
    return hipSuccess;
  };
  std::vector<int> req;
  std::vector<std::pair<Img*, int>> reqs;
  while (true) {
    SCHK(fill(1));
    if (win.empty()) break;
    Img& cur = *win.front();
    const int need = replay(cur);
    if (need < 0) {
      win.pop_front();
      continue;
    }
    reqs.clear();
    speculate(cur, req, budget);
    if (req.empty()) return hipErrorUnknown;  // cannot happen: `need` is unknown at the cursor
    for (const int cid : req) reqs.emplace_back(&cur, cid);
    if ((int)reqs.size() < budget && lookahead > 1) {
      SCHK(fill((size_t)lookahead));
      for (size_t k = 1; k < win.size() && (int)reqs.size() < budget; ++k) {
        speculate(*win[k], req, budget - (int)reqs.size());
        for (const int cid : req) reqs.emplace_back(win[k].get(), cid);
      }
    }
    const int m = (int)reqs.size();
    hcand.resize(m);
    for (int k = 0; k < m; ++k) make_candidate(*reqs[k].first, reqs[k].second, hcand[k]);
    SCHK(dcand.need(m));
    SCHK(dres.need(m));
    const auto tr0 = std::chrono::steady_clock::now();
    SCHK(hipMemcpyAsync(dcand.p, hcand.data(), m * sizeof(pmvs_candidate), hipMemcpyHostToDevice, st));
    SCHK(refine(dcand.p, m, dres.p));
    hres.resize(m);
    SCHK(hipMemcpyAsync(hres.data(), dres.p, m * sizeof(pmvs_refined), hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    refine_wall_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count();
    for (int k = 0; k < m; ++k) {
      Img& w = *reqs[k].first;
      const int cid = reqs[k].second;
      const pmvs_refined& r = hres[k];
      if (r.status == PMVS_ACCEPTED) {
        w.state[cid] = 4;
        w.accepted_slot[cid] = (int)w.accepted.size();
        w.accepted.push_back(r);
      } else {
        if (r.status == PMVS_FAIL_OVERFLOW) return hipErrorNotSupported;  // list capacity: an error, not a reject
        w.state[cid] = (r.status == PMVS_FAIL_PRE) ? 2 : 3;
      }
    }
    refined += m;
    ++rounds;
  }
  out.stats[4] = refined;
  out.stats[5] = rounds;
  out.gen_ms = gen_ms;
  out.refine_ms = refine_wall_ms;
  out.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  return hipSuccess;
}

}  // namespace pmvsdev
