// oracle/filter_oracle.h -- TEST INFRASTRUCTURE ONLY (included by pmvs_oracle.cpp).
//
// CPU restatement of one PMVS filter pass, PMVS3::CFilter::run (filter.cpp:13-27), over a
// patch set held in a CPatchOrganizerS-style cell organizer (patchOrganizerS.cpp):
//   setDepthMapsVGridsVPGridsAddPatchV(0)  filter.cpp:727-770 (+ setDepthMaps :668-725,
//                                           setVImagesVGrids patchOrganizerS.cpp:429-459,
//                                           addPatchV filter.cpp:795-827)
//   filterOutside                           filter.cpp:29-86, computeGain :88-146 / thread :148-201
//   filterExact                             filter.cpp:203-356
//   filterNeighbor(1)                       filter.cpp:358-518 (findNeighbors
//                                           patchOrganizerS.cpp:527-631, filterQuad :387-446)
//   filterSmallGroups                       filter.cpp:520-666
// each followed by setDepthMapsVGridsVPGridsAddPatchV(1).
//
// Ordering.  The reference's cell lists hold shared_ptrs in insertion order and several
// results depend on iteration order (depth-map ties, BFS labels in filterSmallGroups) or
// on pointer order (findNeighbors sorts neighbours by address, which feeds the float sums and
// the least-squares fit of filterQuad).  Here insertion order = patch array index, and
// neighbour lists are sorted by array index.  Cmylapack::lls (Eigen JacobiSVD, absent from the
// image) is restated with Eigen's algorithm (column-pivoting QR preconditioner, two-sided Jacobi,
// rank-thresholded minimum-norm solve; lls5 below): filterQuad decisions are "parity unpinned"
// against the reference binary (Eigen's vectorised reductions sum in another order).
#pragma once

#include <array>
#include <deque>

namespace oracle {

struct FPatch {
  V4 coord, normal;
  float ncc, dscale, ascale, tmp;
  int timages, flag, fix, dflag = 0;
  std::vector<int> images, vimages;
  std::vector<std::pair<int, int>> grids, vgrids;
  int id = -1;  // CPatch::_id (collectPatches order)
};

struct Organizer {
  const OScene& s;
  std::vector<std::vector<std::vector<int>>> pgrids, vpgrids;  // [target][cell] -> patch indexes
  std::vector<std::vector<int>> dpgrids;                         // [target][cell] -> patch or -1
  std::vector<int> ppatches;                                     // collectPatches order
  explicit Organizer(const OScene& sc) : s(sc) {
    pgrids.resize(s.tnum);
    vpgrids.resize(s.tnum);
    dpgrids.resize(s.tnum);
    for (int t = 0; t < s.tnum; ++t) {
      const size_t n = (size_t)s.gwidths[t] * s.gheights[t];
      pgrids[t].resize(n);
      vpgrids[t].resize(n);
      dpgrids[t].assign(n, -1);
    }
  }
  int cell(int t, int ix, int iy) const { return iy * s.gwidths[t] + ix; }
  bool in_grid(int t, int ix, int iy) const { return 0 <= ix && ix < s.gwidths[t] && 0 <= iy && iy < s.gheights[t]; }
};

static inline void erase_from(std::vector<int>& v, int p) { v.erase(std::remove(v.begin(), v.end(), p), v.end()); }

// CPatchOrganizerS::addPatch (patchOrganizerS.cpp:308-346) without the depth-map update (the
// filter rebuilds depth maps from scratch before every use).
static void add_patch_p(Organizer& o, const std::vector<FPatch>& P, int p) {
  const FPatch& q = P[p];
  for (size_t i = 0; i < q.images.size(); ++i) {
    const int t = q.images[i];
    if (o.s.tnum <= t) continue;
    if (!o.in_grid(t, q.grids[i].first, q.grids[i].second)) continue;  // out-of-grid: undefined in the reference
    o.pgrids[t][o.cell(t, q.grids[i].first, q.grids[i].second)].push_back(p);
  }
}

// CPatchOrganizerS::removePatch (patchOrganizerS.cpp:461-489).
static void remove_patch(Organizer& o, const std::vector<FPatch>& P, int p) {
  const FPatch& q = P[p];
  for (size_t i = 0; i < q.images.size(); ++i) {
    const int t = q.images[i];
    if (o.s.tnum <= t || !o.in_grid(t, q.grids[i].first, q.grids[i].second)) continue;
    erase_from(o.pgrids[t][o.cell(t, q.grids[i].first, q.grids[i].second)], p);
  }
  for (size_t i = 0; i < q.vimages.size(); ++i) {
    const int t = q.vimages[i];
    erase_from(o.vpgrids[t][o.cell(t, q.vgrids[i].first, q.vgrids[i].second)], p);
  }
}

template <class F>
static void parallel_for(int nthreads, size_t n, F&& f);
static int g_threads = 1;

// CPatchOrganizerS::collectPatches(target) (patchOrganizerS.cpp:218-248).  The cell walk of each
// target image runs in parallel (its entries in cell order); the first-occurrence numbering then
// walks those entries in target order, as the serial walk does.
static void collect_patches(Organizer& o, std::vector<FPatch>& P, int target) {
  o.ppatches.clear();
  for (auto& q : P) q.id = -1;
  std::vector<std::vector<int>> ent(o.s.tnum);
  parallel_for(g_threads, (size_t)o.s.tnum, [&](int, size_t t) {
    for (auto& cellv : o.pgrids[t]) ent[t].insert(ent[t].end(), cellv.begin(), cellv.end());
  });
  int count = 0;
  for (int t = 0; t < o.s.tnum; ++t)
    for (int p : ent[t])
      if (P[p].id == -1) {
        P[p].id = count++;
        if (target == 0 || P[p].fix == 0) o.ppatches.push_back(p);
      }
}

static inline float depth_of(const OScene& s, int t, const V4& c) { return dot4(s.views[t].oaxis, c); }

// CFilter::setDepthMaps / setDepthMapsThread (filter.cpp:668-725).
static void set_depth_maps(Organizer& o, const std::vector<FPatch>& P) {
  const OScene& s = o.s;
  parallel_for(g_threads, (size_t)s.tnum, [&](int, size_t tt) {  // setDepthMapsThread: one image per job
    const int t = (int)tt;
    std::fill(o.dpgrids[t].begin(), o.dpgrids[t].end(), -1);
    for (int p : o.ppatches) {
      const V3 ic = project(s, t, P[p].coord, s.level);
      const float fx = ic[0] / s.csize, fy = ic[1] / s.csize;
      const int xs[2] = {(int)std::floor(fx), (int)std::ceil(fx)};
      const int ys[2] = {(int)std::floor(fy), (int)std::ceil(fy)};
      const float depth = depth_of(s, t, P[p].coord);
      for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 2; ++i) {
          if (!o.in_grid(t, xs[i], ys[j])) continue;
          int& d = o.dpgrids[t][o.cell(t, xs[i], ys[j])];
          if (d == -1) d = p;
          else if (depth < depth_of(s, t, P[d].coord)) d = p;
        }
    }
  });
}

// CPatchOrganizerS::isVisible (patchOrganizerS.cpp:500-525).
static int is_visible(const Organizer& o, const std::vector<FPatch>& P, const FPatch& q, int t, int ix, int iy,
                      float strict) {
  const OScene& s = o.s;
  if (!o.in_grid(t, ix, iy)) return 0;
  if (s.depth == 0) return 1;
  const int d = o.dpgrids[t][o.cell(t, ix, iy)];
  if (d == -1) return 1;
  V4 ray = sub4(q.coord, s.views[t].center);
  unitize4(ray);
  const float diff = dot4(ray, sub4(q.coord, P[d].coord));
  const float factor = (float)std::min(2.0, 2.0 + (double)dot4(ray, q.normal));
  return diff < get_unit(s, t, q.coord) * s.csize * strict * factor ? 1 : 0;
}

// CPatchOrganizerS::setVImagesVGrids (patchOrganizerS.cpp:429-459) with isVisible0 (:491-498),
// neighbourThreshold 0.5 (findMatch.cpp:94).
static void set_vimages_vgrids(const Organizer& o, const std::vector<FPatch>& P, FPatch& q) {
  const OScene& s = o.s;
  std::vector<int> used(s.tnum, 0);
  for (int t : q.images)
    if (t < s.tnum) used[t] = 1;
  for (int t : q.vimages) used[t] = 1;
  for (int t = 0; t < s.tnum; ++t) {
    if (used[t]) continue;
    const V3 ic = project(s, t, q.coord, s.level);
    const int ix = ((int)std::floor(ic[0] + 0.5f)) / s.csize;
    const int iy = ((int)std::floor(ic[1] + 0.5f)) / s.csize;
    if (is_visible(o, P, q, t, ix, iy, 0.5f) == 0) continue;
    if (get_edge(s, q.coord, t, s.level) == 0) continue;
    q.vimages.push_back(t);
    q.vgrids.push_back({ix, iy});
  }
}

// Thread pool for the per-patch stages (the reference runs them on _CPU threads, filter.cpp:
// filterOutsideThread / filterExactThread / filterNeighborThread / setVImagesVGrids threads).  Each
// task writes only its own slot, so results do not depend on the thread count.
template <class F>
static void parallel_for(int nthreads, size_t n, F&& f) {
  if (nthreads <= 1 || n < 2) {
    for (size_t i = 0; i < n; ++i) f(0, i);
    return;
  }
  std::atomic<size_t> next(0);
  auto work = [&](int tid) {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) break;
      f(tid, i);
    }
  };
  std::vector<std::thread> th;
  const int T = (int)std::min<size_t>((size_t)nthreads, n);
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
}

// CFilter::setDepthMapsVGridsVPGridsAddPatchV (filter.cpp:727-770).
static void set_dm_vgrids(Organizer& o, std::vector<FPatch>& P, int additive) {
  collect_patches(o, P, 0);
  set_depth_maps(o, P);
  parallel_for(g_threads, o.vpgrids.size(), [&](int, size_t t) {
    for (auto& c : o.vpgrids[t]) c.clear();
  });
  if (additive == 0)
    for (int p : o.ppatches) {
      P[p].vimages.clear();
      P[p].vgrids.clear();
    }
  parallel_for(g_threads, o.ppatches.size(), [&](int, size_t k) { set_vimages_vgrids(o, P, P[o.ppatches[k]]); });
  parallel_for(g_threads, (size_t)o.s.tnum, [&](int, size_t tt) {  // addPatchVThread: one image per job,
    const int t = (int)tt;                                         // first matching entry only
    for (int p : o.ppatches) {
      const FPatch& q = P[p];
      for (size_t i = 0; i < q.vimages.size(); ++i)
        if (q.vimages[i] == t) {
          o.vpgrids[t][o.cell(t, q.vgrids[i].first, q.vgrids[i].second)].push_back(p);
          break;
        }
    }
  });
}

// CFindMatch::isNeighbor / isNeighborRadius (findMatch.cpp:125-185).
static int is_neighbor_h(const FPatch& l, const FPatch& r, float hunit, float thr, float radius, bool use_radius) {
  if ((double)dot4(l.normal, r.normal) < std::cos(120.0 * M_PI / 180.0)) return 0;
  const V4 diff = sub4(r.coord, l.coord);
  const float vunit = l.dscale + r.dscale;
  const float f0 = dot4(l.normal, diff), f1 = dot4(r.normal, diff);
  float ftmp = (float)(((double)std::fabs(f0) + (double)std::fabs(f1)) / 2.0);
  ftmp /= vunit;
  V4 v;
  for (int k = 0; k < 4; ++k) v[k] = (2.0f * diff[k] - l.normal[k] * f0) - r.normal[k] * f1;
  const float hsize = (float)((double)norm4(v) / 2.0 / (double)hunit);
  if (use_radius && radius / hunit < hsize) return 0;
  if (1.0 < hsize) ftmp /= std::min(2.0f, hsize);
  return ftmp < thr ? 1 : 0;
}
static int is_neighbor(const OScene& s, const FPatch& l, const FPatch& r, float thr) {
  const float hunit =
      (float)((double)(get_unit(s, l.images[0], l.coord) + get_unit(s, r.images[0], r.coord)) / 2.0 * s.csize);
  return is_neighbor_h(l, r, hunit, thr, 0.0f, false);
}

// CPatch::score2 (patch.hpp:49-51).
static inline float score2(const FPatch& q, float thr) { return std::max(0.0f, q.ncc - thr) * q.timages; }

// CFilter::filterOutsideThread gain (filter.cpp:148-201), neighbourThreshold1 = 1.0.
static float compute_gain(const Organizer& o, const std::vector<FPatch>& P, const FPatch& q) {
  const OScene& s = o.s;
  float gain = score2(q, s.nccThreshold);
  for (size_t i = 0; i < q.images.size(); ++i) {
    const int t = q.images[i];
    if (s.tnum <= t) continue;
    const int c = o.cell(t, q.grids[i].first, q.grids[i].second);
    float maxp = 0.0f;
    for (int j : o.pgrids[t][c])
      if (!is_neighbor(s, q, P[j], 1.0f)) maxp = std::max(maxp, P[j].ncc - s.nccThreshold);
    gain -= maxp;
  }
  for (size_t i = 0; i < q.vimages.size(); ++i) {
    const int t = q.vimages[i];
    if (s.tnum <= t) continue;
    const float pdepth = depth_of(s, t, q.coord);
    const int c = o.cell(t, q.vgrids[i].first, q.vgrids[i].second);
    float maxp = 0.0f;
    for (int j : o.pgrids[t][c]) {
      const float bdepth = depth_of(s, t, P[j].coord);
      if (pdepth < bdepth && !is_neighbor(s, q, P[j], 1.0f)) maxp = std::max(maxp, P[j].ncc - s.nccThreshold);
    }
    gain -= maxp;
  }
  return gain;
}

static int filter_outside(Organizer& o, std::vector<FPatch>& P) {
  collect_patches(o, P, 1);
  std::vector<float> gains(o.ppatches.size());
  parallel_for(g_threads, o.ppatches.size(), [&](int, size_t k) { gains[k] = compute_gain(o, P, P[o.ppatches[k]]); });
  int count = 0;
  for (size_t k = 0; k < o.ppatches.size(); ++k) diag(2, std::fabs(gains[k]) < 0.05f);
  for (size_t k = 0; k < o.ppatches.size(); ++k)
    if (gains[k] < 0.0) {
      remove_patch(o, P, o.ppatches[k]);
      count++;
    }
  return count;
}

// CFilter::filterExact (filter.cpp:203-356), neighbourThreshold1 = 1.0.
static int filter_exact(Organizer& o, std::vector<FPatch>& P, std::vector<OCtx>& ctxs) {
  const OScene& s = o.s;
  collect_patches(o, P, 0);
  const int psize = (int)o.ppatches.size();
  std::vector<std::vector<int>> newimages(psize), removeimages(psize);
  std::vector<std::vector<std::pair<int, int>>> newgrids(psize), removegrids(psize);
  // per target image (in parallel): (patch id, x, y, safe) in cell order; merged in image order
  std::vector<std::vector<std::array<int, 4>>> found(s.tnum);
  parallel_for(g_threads, (size_t)s.tnum, [&](int, size_t tt) {
    const int t = (int)tt;
    const int w = s.gwidths[t], h = s.gheights[t];
    int index = -1;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        ++index;
        for (int p : o.pgrids[t][index]) {
          const FPatch& q = P[p];
          if (q.fix) continue;
          int safe = 0;
          if (is_visible(o, P, q, t, x, y, 1.0f)) safe = 1;
          else if (0 < x && is_visible(o, P, q, t, x - 1, y, 1.0f)) safe = 1;
          else if (x < w - 1 && is_visible(o, P, q, t, x + 1, y, 1.0f)) safe = 1;
          else if (0 < y && is_visible(o, P, q, t, x, y - 1, 1.0f)) safe = 1;
          else if (y < h - 1 && is_visible(o, P, q, t, x, y + 1, 1.0f)) safe = 1;
          found[t].push_back({{q.id, x, y, safe}});
        }
      }
  });
  for (int t = 0; t < s.tnum; ++t)
    for (const auto& f : found[t]) {
      if (f[3]) {
        newimages[f[0]].push_back(t);
        newgrids[f[0]].push_back({f[1], f[2]});
      } else {
        removeimages[f[0]].push_back(t);
        removegrids[f[0]].push_back({f[1], f[2]});
      }
    }
  for (int k = 0; k < psize; ++k) {
    const int p = o.ppatches[k];
    if (P[p].fix) continue;
    for (size_t i = 0; i < removeimages[k].size(); ++i) {
      const int t = removeimages[k][i];
      erase_from(o.pgrids[t][o.cell(t, removegrids[k][i].first, removegrids[k][i].second)], p);
    }
  }
  parallel_for(g_threads, (size_t)psize, [&](int tid, size_t kk) {
    const int k = (int)kk;
    const int p = o.ppatches[k];
    FPatch& q = P[p];
    if (q.fix) return;
    q.timages = (int)newimages[k].size();
    for (size_t i = 0; i < q.images.size(); ++i)
      if (s.tnum <= q.images[i]) {
        newimages[k].push_back(q.images[i]);
        newgrids[k].push_back(q.grids[i]);
      }
    q.images.swap(newimages[k]);
    q.grids.swap(newgrids[k]);
    if (s.minImageNum <= (int)q.images.size()) {
      OPatch op;
      op.coord = q.coord; op.normal = q.normal; op.images = q.images; op.grids = q.grids;
      op.dscale = q.dscale; op.ascale = q.ascale; op.ncc = q.ncc;
      set_ref_image(s, ctxs[tid], op);
      q.images = op.images;
      OPatch g = op;
      set_grids(s, g);
      q.grids = g.grids;
    }
  });
  int count = 0;
  for (int k = 0; k < psize; ++k) {
    const int p = o.ppatches[k];
    FPatch& q = P[p];
    if (q.fix) continue;
    if ((int)q.images.size() < s.minImageNum) {
      remove_patch(o, P, p);
      count++;
    }
  }
  return count;
}

// CExpand::computeRadius (expand.cpp:182-198) with COptim::computeUnits (optim.cpp:446-471).
static float compute_radius(const OScene& s, const FPatch& q) {
  OPatch op;
  op.coord = q.coord; op.normal = q.normal; op.images = q.images;
  std::vector<float> units;
  compute_units(s, op, units);
  std::nth_element(units.begin(), units.begin() + 1, units.end());
  return units[1] * s.csize;
}

// CPatchOrganizerS::findNeighbors(patch, neighbors, lock, scale, margin, skipvis)
// (patchOrganizerS.cpp:527-631); neighbours sorted by patch index (reference: by address).
static void find_neighbors(const Organizer& o, const std::vector<FPatch>& P, const FPatch& q, std::vector<int>& out,
                           float scale, int margin, int skipvis) {
  const OScene& s = o.s;
  const float radius = (float)(1.5 * margin * (double)compute_radius(s, q));
  float unit = 0.0f;
  for (int t : q.images) unit += get_unit(s, t, q.coord);
  unit /= (int)q.images.size();
  unit *= s.csize;
  const float thr = 0.5f * scale;  // _neighborThreshold * scale
  auto scan = [&](int t, int ix, int iy) {
    for (int j = -margin; j <= margin; ++j) {
      const int yt = iy + j;
      if (yt < 0 || s.gheights[t] <= yt) continue;
      for (int i = -margin; i <= margin; ++i) {
        const int xt = ix + i;
        if (xt < 0 || s.gwidths[t] <= xt) continue;
        const int c = o.cell(t, xt, yt);
        for (int p : o.pgrids[t][c])
          if (is_neighbor_h(q, P[p], unit, thr, radius, true)) out.push_back(p);
        for (int p : o.vpgrids[t][c])
          if (is_neighbor_h(q, P[p], unit, thr, radius, true)) out.push_back(p);
      }
    }
  };
  for (size_t i = 0; i < q.images.size(); ++i)
    if (q.images[i] < s.tnum) scan(q.images[i], q.grids[i].first, q.grids[i].second);
  if (skipvis == 0)
    for (size_t i = 0; i < q.vimages.size(); ++i) scan(q.vimages[i], q.vgrids[i].first, q.vgrids[i].second);
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
}

// ortho (vec4.hpp:303-322) on the patch normal.
static void ortho4(const V4& z, V4& x, V4& y) {
  x = {{0, 0, 0, 0}};
  y = {{0, 0, 0, 0}};
  if (std::fabs((double)z[0]) > 0.5) {
    x[0] = z[1]; x[1] = -z[0]; x[2] = 0;
  } else if (std::fabs((double)z[1]) > 0.5) {
    x[1] = z[2]; x[2] = -z[1]; x[0] = 0;
  } else {
    x[2] = z[0]; x[0] = -z[2]; x[1] = 0;
  }
  unitize4(x);
  y[0] = z[1] * x[2] - z[2] * x[1];
  y[1] = z[2] * x[0] - z[0] * x[2];
  y[2] = z[0] * x[1] - z[1] * x[0];
}

// Cmylapack::lls (mylapack.cpp:102-149): x = A.jacobiSvd(ComputeThinU | ComputeThinV).solve(b) in
// double for an n x 5 system (n >= 6), restated with Eigen 3.3's JacobiSVD algorithm (Eigen is absent
// from the image; parity unpinned against it):
//   1. scale = max|a_ij| (1 if 0); the scaled matrix is reduced by a column-pivoting Householder
//      QR (ColPivHouseholderQRPreconditioner: pivot = largest updated column norm, LAPACK xGEQPF
//      norm downdating, makeHouseholder: beta = -sign(c0) |x|, tau = (beta - c0) / beta,
//      essential = tail / (c0 - beta));
//   2. two-sided Jacobi sweeps on the 5 x 5 R (pairs p > q, threshold max(DBL_MIN, 2 eps max|diag|),
//      real_2x2_jacobi_svd + makeJacobi rotations, left rotations accumulated into U, right into V);
//   3. singular values |diag| * scale (U column negated for a negative diagonal), sorted descending;
//   4. solve with rank = #{s_i >= max(s_0 * 5 eps, DBL_MIN)}: x = V_r diag(1/s_r) U_r^T b -- the
//      minimum-norm least-squares solution on rank-deficient neighbourhoods.
// Sums run in index order; U^T b is formed as (Q^T b)[0..4] rotated by the accumulated 5 x 5 U.
static void lls5(const std::vector<std::array<float, 5>>& A, const std::vector<float>& b, float x[5]) {
  const int n = (int)A.size();
  constexpr int N = 5;
  const double eps = 2.220446049250313e-16, dmin = 2.2250738585072014e-308;
  std::vector<double> M((size_t)n * N), r(n);
  double scale = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < N; ++j) scale = std::max(scale, std::fabs((double)A[i][j]));
  if (!std::isfinite(scale)) {  // Eigen reports InvalidInput; the solve then returns garbage: zeros here
    for (int k = 0; k < N; ++k) x[k] = 0.0f;
    return;
  }
  if (scale == 0.0) scale = 1.0;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < N; ++j) M[(size_t)i * N + j] = (double)A[i][j] / scale;
    r[i] = b[i];
  }
  auto at = [&](int i, int j) -> double& { return M[(size_t)i * N + j]; };
  // ---- 1. column-pivoting Householder QR
  int perm[N];
  double nu[N], nd[N], tau[N];
  for (int j = 0; j < N; ++j) {
    perm[j] = j;
    double sq = 0.0;
    for (int i = 0; i < n; ++i) sq += at(i, j) * at(i, j);
    nd[j] = nu[j] = std::sqrt(sq);
  }
  const double downdate = std::sqrt(eps);
  for (int k = 0; k < N; ++k) {
    int big = k;
    for (int j = k + 1; j < N; ++j)
      if (nu[j] > nu[big]) big = j;
    if (big != k) {
      for (int i = 0; i < n; ++i) std::swap(at(i, k), at(i, big));
      std::swap(nu[k], nu[big]);
      std::swap(nd[k], nd[big]);
      std::swap(perm[k], perm[big]);
    }
    double tail = 0.0;
    for (int i = k + 1; i < n; ++i) tail += at(i, k) * at(i, k);
    const double c0 = at(k, k);
    double beta;
    if (tail <= dmin) {
      tau[k] = 0.0;
      beta = c0;
      for (int i = k + 1; i < n; ++i) at(i, k) = 0.0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      const double den = c0 - beta;
      for (int i = k + 1; i < n; ++i) at(i, k) = at(i, k) / den;
      tau[k] = (beta - c0) / beta;
    }
    at(k, k) = beta;
    if (tau[k] != 0.0)
      for (int j = k + 1; j < N; ++j) {
        double t = 0.0;
        for (int i = k + 1; i < n; ++i) t += at(i, k) * at(i, j);
        t += at(k, j);
        at(k, j) -= tau[k] * t;
        for (int i = k + 1; i < n; ++i) at(i, j) -= (tau[k] * at(i, k)) * t;
      }
    for (int j = k + 1; j < N; ++j) {
      if (nu[j] == 0.0) continue;
      double t = std::fabs(at(k, j)) / nu[j];
      t = (1.0 + t) * (1.0 - t);
      if (t < 0.0) t = 0.0;
      const double q = nu[j] / nd[j];
      const double t2 = t * (q * q);
      if (t2 <= downdate) {
        double sq = 0.0;
        for (int i = k + 1; i < n; ++i) sq += at(i, j) * at(i, j);
        nd[j] = nu[j] = std::sqrt(sq);
      } else {
        nu[j] *= std::sqrt(t);
      }
    }
  }
  // Q^T b (H_0 first)
  for (int k = 0; k < N; ++k) {
    if (tau[k] == 0.0) continue;
    double t = 0.0;
    for (int i = k + 1; i < n; ++i) t += at(i, k) * r[i];
    t += r[k];
    r[k] -= tau[k] * t;
    for (int i = k + 1; i < n; ++i) r[i] -= (tau[k] * at(i, k)) * t;
  }
  // ---- 2. two-sided Jacobi on R
  double W[N][N], U[N][N], V[N][N];
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      W[i][j] = (j >= i) ? at(i, j) : 0.0;
      U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
    }
  double maxd = 0.0;
  for (int i = 0; i < N; ++i) maxd = std::max(maxd, std::fabs(W[i][i]));
  auto rot_left = [&](double (*X)[N], int p, int q, double c, double s_) {  // rows p, q
    for (int j = 0; j < N; ++j) {
      const double xp = X[p][j], xq = X[q][j];
      X[p][j] = c * xp + s_ * xq;
      X[q][j] = -s_ * xp + c * xq;
    }
  };
  auto rot_right = [&](double (*X)[N], int p, int q, double c, double s_) {  // columns p, q by (c, s)^T
    for (int i = 0; i < N; ++i) {
      const double xp = X[i][p], xq = X[i][q];
      X[i][p] = c * xp - s_ * xq;
      X[i][q] = s_ * xp + c * xq;
    }
  };
  bool finished = false;
  for (int sweep = 0; !finished && sweep < 100; ++sweep) {
    finished = true;
    for (int p = 1; p < N; ++p)
      for (int q = 0; q < p; ++q) {
        const double thr = std::max(dmin, 2.0 * eps * maxd);
        if (!(std::fabs(W[p][q]) > thr || std::fabs(W[q][p]) > thr)) continue;
        finished = false;
        // real_2x2_jacobi_svd on [[W_pp, W_pq], [W_qp, W_qq]]
        double m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
        const double t = m00 + m11, d = m10 - m01;
        double c1 = 1.0, s1 = 0.0;
        if (!(std::fabs(d) < dmin)) {
          const double u = t / d;
          const double tmp = std::sqrt(1.0 + u * u);
          s1 = 1.0 / tmp;
          c1 = u / tmp;
        }
        {  // m.applyOnTheLeft(0, 1, rot1)
          const double a0 = m00, a1 = m01, b0 = m10, b1 = m11;
          m00 = c1 * a0 + s1 * b0; m01 = c1 * a1 + s1 * b1;
          m10 = -s1 * a0 + c1 * b0; m11 = -s1 * a1 + c1 * b1;
        }
        double cr = 1.0, sr = 0.0;  // makeJacobi(m00, m01, m11)
        const double deno = 2.0 * std::fabs(m01);
        if (!(deno < dmin)) {
          const double tau_ = (m00 - m11) / deno;
          const double w = std::sqrt(tau_ * tau_ + 1.0);
          const double tt = (tau_ > 0.0) ? 1.0 / (tau_ + w) : 1.0 / (tau_ - w);
          const double sign_t = tt > 0.0 ? 1.0 : -1.0;
          const double nn = 1.0 / std::sqrt(tt * tt + 1.0);
          sr = -sign_t * (m01 / std::fabs(m01)) * std::fabs(tt) * nn;
          cr = nn;
        }
        // j_left = rot1 * j_right^T, with j_right^T = (cr, -sr)
        const double cl = c1 * cr - s1 * (-sr);
        const double sl = c1 * (-sr) + s1 * cr;
        rot_left(W, p, q, cl, sl);
        rot_right(U, p, q, cl, -sl);  // U.applyOnTheRight(p, q, j_left^T)
        rot_right(W, p, q, cr, sr);
        rot_right(V, p, q, cr, sr);
        maxd = std::max(maxd, std::max(std::fabs(W[p][p]), std::fabs(W[q][q])));
      }
  }
  // ---- 3. singular values, signs, scale; 4. sort descending
  double sv[N];
  for (int i = 0; i < N; ++i) {
    sv[i] = std::fabs(W[i][i]);
    if (W[i][i] < 0.0)
      for (int k = 0; k < N; ++k) U[k][i] = -U[k][i];
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
      std::swap(sv[i], sv[pos]);
      for (int k = 0; k < N; ++k) {
        std::swap(U[k][i], U[k][pos]);
        std::swap(V[k][i], V[k][pos]);
      }
    }
  }
  int rank = 0;
  if (nonzero > 0) {
    const double pre = std::max(sv[0] * (N * eps), dmin);
    int i = nonzero - 1;
    while (i >= 0 && sv[i] < pre) --i;
    rank = i + 1;
  }
  // ---- 5. x = P V_r diag(1/s_r) U_r^T (Q^T b)[0..4]
  double y[N], z[N];
  for (int i = 0; i < rank; ++i) {
    double t = 0.0;
    for (int k = 0; k < N; ++k) t += U[k][i] * r[k];
    y[i] = t / sv[i];
  }
  for (int k = 0; k < N; ++k) {
    double t = 0.0;
    for (int i = 0; i < rank; ++i) t += V[k][i] * y[i];
    z[k] = t;
  }
  for (int k = 0; k < N; ++k) x[perm[k]] = (float)z[k];
}

// CFilter::filterQuad (filter.cpp:387-446).
static int filter_quad(const OScene& s, const std::vector<FPatch>& P, const FPatch& q, const std::vector<int>& nb) {
  V4 xdir, ydir;
  ortho4(q.normal, xdir, ydir);
  const int nsize = (int)nb.size();
  float h = 0.0f;
  for (int n = 0; n < nsize; ++n) h += norm4(sub4(P[nb[n]].coord, q.coord));
  h /= nsize;
  std::vector<std::array<float, 5>> A(nsize);
  std::vector<float> b(nsize), fxs(nsize), fys(nsize), fzs(nsize);
  for (int n = 0; n < nsize; ++n) {
    const V4 diff = sub4(P[nb[n]].coord, q.coord);
    fxs[n] = dot4(diff, xdir) / h;
    fys[n] = dot4(diff, ydir) / h;
    fzs[n] = dot4(diff, q.normal);
    A[n] = {{fxs[n] * fxs[n], fys[n] * fys[n], fxs[n] * fys[n], fxs[n], fys[n]}};
    b[n] = fzs[n];
  }
  float x[5];
  lls5(A, b, x);
  const int inum = std::min(s.tau, (int)q.images.size());
  float unit = 0.0f;
  for (int i = 0; i < inum; ++i) unit += get_unit(s, q.images[i], q.coord);
  unit /= inum;
  float residual = 0.0f;
  for (int n = 0; n < nsize; ++n) {
    const float res = x[0] * (fxs[n] * fxs[n]) + x[1] * (fys[n] * fys[n]) + x[2] * (fxs[n] * fys[n]) +
                      x[3] * fxs[n] + x[4] * fys[n] - fzs[n];
    residual = (float)((double)residual + std::fabs((double)res) / (double)unit);  // float += double
  }
  residual /= (nsize - 5);
  return residual < s.quad ? 0 : 1;
}

static int filter_neighbor(Organizer& o, std::vector<FPatch>& P) {
  collect_patches(o, P, 1);
  std::vector<int> rejects(o.ppatches.size(), 0);
  parallel_for(g_threads, o.ppatches.size(), [&](int, size_t k) {
    const FPatch& q = P[o.ppatches[k]];
    std::vector<int> nb;
    find_neighbors(o, P, q, nb, 4.0f, 2, 1);
    if ((int)nb.size() < 6) rejects[k] = 1;
    else if (filter_quad(o.s, P, q, nb)) rejects[k] = 1;
  });
  int count = 0;
  for (size_t k = 0; k < o.ppatches.size(); ++k)
    if (rejects[k]) {
      count++;
      remove_patch(o, P, o.ppatches[k]);
    }
  return count;
}

// CFilter::filterSmallGroups + Sub (filter.cpp:520-666), neighbourThreshold2 = 1.0.
static int filter_small_groups(Organizer& o, std::vector<FPatch>& P) {
  const OScene& s = o.s;
  collect_patches(o, P, 0);
  const int psize = (int)o.ppatches.size();
  if (psize == 0) return 0;
  std::vector<int> label(psize, -1);
  for (int k = 0; k < psize; ++k) P[o.ppatches[k]].flag = k;
  int id = -1;
  for (int pid = 0; pid < psize; ++pid) {
    if (label[pid] != -1) continue;
    label[pid] = ++id;
    std::deque<int> ltmp;
    ltmp.push_back(pid);
    while (!ltmp.empty()) {
      const int ptmp = ltmp.front();
      ltmp.pop_front();
      const FPatch& q = P[o.ppatches[ptmp]];
      const int t = q.images[0], ix = q.grids[0].first, iy = q.grids[0].second;
      for (int y = -1; y <= 1; ++y) {
        const int yt = iy + y;
        if (yt < 0 || s.gheights[t] <= yt) continue;
        for (int x = -1; x <= 1; ++x) {
          const int xt = ix + x;
          if (xt < 0 || s.gwidths[t] <= xt) continue;
          const int c = o.cell(t, xt, yt);
          for (int lst = 0; lst < 2; ++lst)
            for (int p : (lst == 0 ? o.pgrids[t][c] : o.vpgrids[t][c])) {
              const int itmp = P[p].flag;
              if (label[itmp] != -1) continue;
              if (is_neighbor(s, q, P[p], 1.0f)) {
                label[itmp] = id;
                ltmp.push_back(itmp);
              }
            }
        }
      }
    }
  }
  id++;
  std::vector<int> size(id, 0);
  for (int l : label) ++size[l];
  const int threshold = std::max(20, psize / 10000);
  int count = 0;
  for (int k = 0; k < psize; ++k) {
    const int p = o.ppatches[k];
    if (P[p].fix) continue;
    if (size[label[k]] < threshold) {
      remove_patch(o, P, p);
      count++;
    }
  }
  return count;
}

// CFilter::run (filter.cpp:13-27).  counts[0..3] = removed by outside/exact/neighbor/groups.
static void filter_run(const OScene& s, std::vector<FPatch>& P, std::vector<int>& keep, int counts[4]) {
  // ORACLE_PROFILE=1: wall time of each stage on stderr (diagnostics of the checker's own cost)
  const bool prof = getenv("ORACLE_PROFILE") != nullptr;
  auto t = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!prof) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[oracle filter] %s %.2f s\n", what, std::chrono::duration<double>(now - t).count());
    t = now;
  };
  Organizer o(s);
  std::vector<OCtx> ctxs(std::max(1, g_threads));
  for (auto& c : ctxs) init_ctx(s, c);
  for (int p = 0; p < (int)P.size(); ++p) add_patch_p(o, P, p);
  mark("organizer");
  set_dm_vgrids(o, P, 0);
  mark("set_dm_vgrids");
  counts[0] = filter_outside(o, P);
  mark("outside");
  set_dm_vgrids(o, P, 1);
  mark("set_dm_vgrids");
  counts[1] = filter_exact(o, P, ctxs);
  mark("exact");
  set_dm_vgrids(o, P, 1);
  mark("set_dm_vgrids");
  counts[2] = filter_neighbor(o, P);
  mark("neighbor");
  set_dm_vgrids(o, P, 1);
  mark("set_dm_vgrids");
  counts[3] = filter_small_groups(o, P);
  mark("groups");
  set_dm_vgrids(o, P, 1);
  mark("set_dm_vgrids");
  collect_patches(o, P, 0);
  keep.assign(P.size(), 0);
  for (int p : o.ppatches) keep[p] = 1;
}

}  // namespace oracle
