// oracle/seed_oracle.h -- TEST INFRASTRUCTURE ONLY (included by pmvs_oracle.cpp).
//
// CPU restatement of the seed phase, PMVS3::CSeed (seed.cpp:11-414), run with the reference's
// single-thread job order (CPU 1): target images in std::shuffle(mt19937(42)) order
// (seed.cpp:53-60), every cell of an image in raster order, the feature points of a cell in
// detector order, and for each point the epipolar candidates sorted by _response.
//
// One documented deviation: the reference sorts the candidate vector of shared_ptr<CPoint> by
// pointer value (seed.cpp:322, heap-address order; CPoint::operator< is never used there).  This
// restatement (and the device path) orders candidates by ascending _response, ties by collection
// order.  Everything else -- epipolar cell walk, EPD test, triangulation,
// counts, canAdd, best-patch selection -- follows the cited lines.
//
// The refinement of a candidate is refine_one() (preProcess -> refinePatch -> postProcess at
// depth 0, seed.cpp:387-414) and depends on nothing but the candidate, which is what lets the
// device path refine speculatively in batches and still reproduce this sequential order.
#pragma once

#include <random>

namespace oracle {

// CPhotoSetS::setDistances, photoSetS.cpp:195-234.
static void set_distances(const OScene& s, std::vector<std::vector<float>>& dist) {
  dist.assign(s.num, std::vector<float>(s.num, 0.0f));
  float avedis = 0.0f;
  int denom = 0;
  for (int i = 0; i < s.num; ++i)
    for (int j = 0; j < s.num; ++j) {
      if (i == j) continue;
      const float f = norm4(sub4(s.views[i].center, s.views[j].center));
      dist[i][j] = f;
      avedis += f;
      denom++;
    }
  if (denom == 0) return;
  avedis /= denom;
  const float margin = (float)std::cos(10.0f * M_PI / 180.0f);
  for (int i = 0; i < s.num; ++i) {
    V4 r0 = s.views[i].oaxis;
    r0[3] = 0.0f;
    for (int j = 0; j < s.num; ++j) {
      V4 r1 = s.views[j].oaxis;
      r1[3] = 0.0f;
      dist[i][j] /= avedis;
      const float dis = std::max(0.0f, 1.0f - dot4(r0, r1) - margin);
      dist[i][j] += dis;
    }
  }
}

// COptim::collectImages, optim.cpp:66-93 (candidates sorted with Svec2cmp, vec2.hpp:254-258).
static void collect_images(const OScene& s, const std::vector<std::vector<float>>& dist, int index,
                           std::vector<int>& out) {
  out.clear();
  V4 r0 = s.views[index].oaxis;
  r0[3] = 0.0f;
  std::vector<std::pair<float, float>> cands;
  for (int k : s.visdata2[index]) {
    if (s.sequence != -1 && s.sequence < std::abs(index - k)) continue;
    V4 r1 = s.views[k].oaxis;
    r1[3] = 0.0f;
    if ((double)dot4(r0, r1) < std::cos((double)s.angle0)) continue;
    cands.push_back({dist[index][k], (float)k});
  }
  std::sort(cands.begin(), cands.end(), [](const std::pair<float, float>& a, const std::pair<float, float>& b) {
    return a.first < b.first || (a.first == b.first && a.second < b.second);
  });
  for (int i = 0; i < std::min(s.tau, (int)cands.size()); ++i) out.push_back((int)cands[i].second);
}

// det(TMat4<double>) = m0 . cross(m1, m2, m3) (mat4.hpp:244-246, vec4.hpp:216-231).
static inline double det4(const double* a, const double* b, const double* c, const double* d) {
  const double d1 = (c[2] * d[3]) - (c[3] * d[2]);
  const double d2 = (c[1] * d[3]) - (c[3] * d[1]);
  const double d3 = (c[1] * d[2]) - (c[2] * d[1]);
  const double d4 = (c[0] * d[3]) - (c[3] * d[0]);
  const double d5 = (c[0] * d[2]) - (c[2] * d[0]);
  const double d6 = (c[0] * d[1]) - (c[1] * d[0]);
  const double x0 = -b[1] * d1 + b[2] * d2 - b[3] * d3;
  const double x1 = b[0] * d1 - b[2] * d4 + b[3] * d5;
  const double x2 = -b[0] * d2 + b[1] * d4 - b[3] * d6;
  const double x3 = b[0] * d3 - b[1] * d5 + b[2] * d6;
  return a[0] * x0 + a[1] * x1 + a[2] * x2 + a[3] * x3;
}

// Image::setF<double>, camera.hpp:130-151: rows of the level projections promoted to double.
static void set_f(const OScene& s, int i0, int i1, double F[3][3]) {
  double p0[3][4], p1[3][4];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) {
      p0[r][c] = s.views[i0].P[s.level][r][c];
      p1[r][c] = s.views[i1].P[s.level][r][c];
    }
  const double* A[3] = {p0[0], p0[1], p0[2]};
  const double* B[3] = {p1[0], p1[1], p1[2]};
  // F[i][j] = det(lhs row (i+1)%3, lhs row (i+2)%3, rhs row (j+1)%3, rhs row (j+2)%3)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) F[i][j] = det4(A[(i + 1) % 3], A[(i + 2) % 3], B[(j + 1) % 3], B[(j + 2) % 3]);
}

// Image::computeEPD<double>, camera.hpp:119-127.
static inline float compute_epd(const double F[3][3], const double* p0, const double* p1) {
  double l[3];
  for (int i = 0; i < 3; ++i) l[i] = F[i][0] * p1[0] + F[i][1] * p1[1] + F[i][2] * p1[2];
  const double f = std::sqrt(l[0] * l[0] + l[1] * l[1]);
  if (f == 0.0) return 0.0f;
  for (int i = 0; i < 3; ++i) l[i] /= f;
  return (float)std::fabs(l[0] * p0[0] + l[1] * p0[1] + l[2] * p0[2]);
}

struct SeedPoint {
  float x, y, response;
  int type;
};

struct SeedCand {
  int view, point, cell;  // image index, point id in that image, its cell
  V4 coord;
  float response;
};

struct SeedState {
  const OScene& s;
  std::vector<std::vector<SeedPoint>> pts;         // per view, detector order
  std::vector<std::vector<std::vector<int>>> cells;  // _ppoints[index][cell] -> point ids
  std::vector<std::vector<unsigned char>> counts;  // _counts (unsigned char) per target cell
  std::vector<std::vector<unsigned char>> occupied;  // _pgrids[index][cell] non-empty
  std::vector<std::vector<float>> dist;
  int64_t trial = 0, pass = 0, fail0 = 0, fail1 = 0;
  explicit SeedState(const OScene& sc) : s(sc) {}
};

// CImage::getMask(int, int, level), image.hpp:553-565.
static inline int mask_at(const OScene& s, int index, int ix, int iy) {
  const OView& v = s.views[index];
  if (v.mask[s.level].empty()) return 1;
  if (ix < 0 || v.w[s.level] <= ix || iy < 0 || v.h[s.level] <= iy) return 1;
  return v.mask[s.level][iy * v.w[s.level] + ix];
}

// CSeed::canAdd, seed.cpp:325-338.
static inline int can_add(const SeedState& st, int index, int x, int y) {
  const OScene& s = st.s;
  if (!mask_at(s, index, s.csize * x, s.csize * y)) return 0;
  if (s.tnum <= index) return 1;
  const int c = y * s.gwidths[index] + x;
  if (st.occupied[index][c]) return 0;
  if (2 <= st.counts[index][c]) return 0;  // _countThreshold2 = 2 (findMatch.cpp:97)
  return 1;
}

// CSeed::collectCells, seed.cpp:207-267.
static void collect_cells(const OScene& s, const double F[3][3], const SeedPoint& p0, int index1,
                          std::vector<std::pair<int, int>>& cells) {
  const double pt[3] = {p0.x, p0.y, 1.0};
  const int gw = s.gwidths[index1], gh = s.gheights[index1];
  double line[3];
  for (int i = 0; i < 3; ++i) line[i] = F[0][i] * pt[0] + F[1][i] * pt[1] + F[2][i] * pt[2];  // transpose(F) * point
  if (line[0] == 0.0 && line[1] == 0.0) return;
  const float lo = (float)(INT_MIN + 3.0f), hi = (float)(INT_MAX - 3.0f);
  if (std::fabs(line[0]) > std::fabs(line[1])) {
    for (int y = 0; y < gh; ++y) {
      const float fy = (float)((y + 0.5) * s.csize - 0.5f);
      float fx = (float)((-line[1] * fy - line[2]) / line[0]);
      fx = std::max(lo, std::min(hi, fx));
      const int ix = ((int)std::floor(fx + 0.5f)) / s.csize;
      if (0 <= ix && ix < gw) cells.push_back({ix, y});
      if (0 <= ix - 1 && ix - 1 < gw) cells.push_back({ix - 1, y});
      if (0 <= ix + 1 && ix + 1 < gw) cells.push_back({ix + 1, y});
    }
  } else {
    for (int x = 0; x < gw; ++x) {
      const float fx = (float)((x + 0.5) * s.csize - 0.5f);
      float fy = (float)((-line[0] * fx - line[2]) / line[1]);
      fy = std::max(lo, std::min(hi, fy));
      const int iy = ((int)std::floor(fy + 0.5f)) / s.csize;
      if (0 <= iy && iy < gh) cells.push_back({x, iy});
      if (0 <= iy - 1 && iy - 1 < gh) cells.push_back({x, iy - 1});
      if (0 <= iy + 1 && iy + 1 < gh) cells.push_back({x, iy + 1});
    }
  }
}

// CSeed::unproject, seed.cpp:340-384: 4x3 linear system from two views, normal equations in
// double (A entries are float expressions), solved with invert(Mat3) (mat3.hpp:275-292).
static V4 unproject(const OScene& s, int i0, int i1, const SeedPoint& a, const SeedPoint& b) {
  const float(*P0)[4] = s.views[i0].P[s.level];
  const float(*P1)[4] = s.views[i1].P[s.level];
  double A[4][3], bb[4];
  for (int c = 0; c < 3; ++c) {
    A[0][c] = (double)(P0[0][c] - a.x * P0[2][c]);
    A[1][c] = (double)(P0[1][c] - a.y * P0[2][c]);
    A[2][c] = (double)(P1[0][c] - b.x * P1[2][c]);
    A[3][c] = (double)(P1[1][c] - b.y * P1[2][c]);
  }
  // A is a Mat4 whose 4th column is 0 (default-constructed TMat4); b likewise a Vec4.
  bb[0] = (double)(a.x * P0[2][3] - P0[0][3]);
  bb[1] = (double)(a.y * P0[2][3] - P0[1][3]);
  bb[2] = (double)(b.x * P1[2][3] - P1[0][3]);
  bb[3] = (double)(b.y * P1[2][3] - P1[1][3]);
  // ATA(i,j) = AT[i] . A.col(j) = sum_k A[k][i] * A[k][j] (k = 0..3, left to right); ATb likewise.
  double M[3][3], r[3];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) M[i][j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
    r[i] = A[0][i] * bb[0] + A[1][i] * bb[1] + A[2][i] * bb[2] + A[3][i] * bb[3];
  }
  auto cr = [](const double* u, const double* w, double* o) {
    o[0] = u[1] * w[2] - w[1] * u[2];
    o[1] = -u[0] * w[2] + w[0] * u[2];
    o[2] = u[0] * w[1] - w[0] * u[1];
  };
  double ad[3][3];
  cr(M[1], M[2], ad[0]);
  cr(M[2], M[0], ad[1]);
  cr(M[0], M[1], ad[2]);
  const double d = ad[0][0] * M[0][0] + ad[0][1] * M[0][1] + ad[0][2] * M[0][2];
  double inv[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  // invert() leaves iATA3 untouched (zero) when d == 0
  if (d != 0.0)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) inv[i][j] = ad[j][i] / d;
  V4 out;
  for (int i = 0; i < 3; ++i) out[i] = (float)(inv[i][0] * r[0] + inv[i][1] * r[1] + inv[i][2] * r[2]);
  out[3] = 1.0f;
  return out;
}

// CSeed::collectCandidates, seed.cpp:271-323 (candidates ordered by _response, see header).
static void collect_candidates(SeedState& st, int index, const std::vector<int>& indexes, const SeedPoint& p,
                               std::vector<SeedCand>& vcp) {
  const OScene& s = st.s;
  vcp.clear();
  const double p0[3] = {p.x, p.y, 1.0};
  std::vector<std::pair<int, int>> cells;
  for (int j : indexes) {
    double F[3][3];
    set_f(s, index, j, F);
    cells.clear();
    collect_cells(s, F, p, j, cells);
    for (const auto& c : cells) {
      if (!can_add(st, j, c.first, c.second)) continue;
      const int cell = c.second * s.gwidths[j] + c.first;
      for (int q : st.cells[j][cell]) {
        const SeedPoint& rhs = st.pts[j][q];
        if (p.type != rhs.type) continue;
        const double p1[3] = {rhs.x, rhs.y, 1.0};
        if (2.0f <= compute_epd(F, p0, p1)) continue;  // _epThreshold = 2.0f (findMatch.cpp:106)
        vcp.push_back({j, q, cell, V4{}, 0.0f});
      }
    }
  }
  std::vector<SeedCand> keep;
  for (SeedCand& c : vcp) {
    c.coord = unproject(s, index, c.view, p, st.pts[c.view][c.point]);
    const float(*P)[4] = s.views[index].P[s.level];
    const V4 row2 = {{P[2][0], P[2][1], P[2][2], P[2][3]}};
    if (dot4(row2, c.coord) <= 0.0) continue;
    if (get_mask_all(s, c.coord, s.level) == 0 || inside_bimages(s, c.coord) == 0) continue;
    c.response = std::fabs(norm4(sub4(c.coord, s.views[index].center)) - norm4(sub4(c.coord, s.views[c.view].center)));
    keep.push_back(c);
  }
  std::stable_sort(keep.begin(), keep.end(), [](const SeedCand& a, const SeedCand& b) { return a.response < b.response; });
  vcp.swap(keep);
}

// The patch a seed candidate starts from (seed.cpp:167-173) as a refine-batch candidate.
static void seed_candidate(const OScene& s, int index, const SeedCand& c, pmvs_candidate& out) {
  std::memset(&out, 0, sizeof(out));
  V4 n = sub4(s.views[index].center, c.coord);
  unitize4(n);
  n[3] = 0.0f;
  for (int k = 0; k < 4; ++k) { out.coord[k] = c.coord[k]; out.normal[k] = n[k]; }
  out.dscale = 0.0f;
  out.num_images = 2;
  out.images[0] = index;
  out.images[1] = c.view;
}

// Patch::CPatch::score, patch.hpp:46-48.
static inline float seed_score(const pmvs_refined& r, float thr) { return std::max(0.0f, r.ncc - thr) * r.num_images; }

// CSeed::initialMatch, seed.cpp:133-205.
static void initial_match(SeedState& st, OCtx& ctx, int index, std::vector<pmvs_patch>& out) {
  const OScene& s = st.s;
  std::vector<int> indexes;
  collect_images(s, st.dist, index, indexes);
  if (s.tau < (int)indexes.size()) indexes.resize(s.tau);
  if (indexes.empty()) return;
  const int gw = s.gwidths[index], gh = s.gheights[index];
  std::vector<SeedCand> vcp;
  int cell = -1;
  for (int y = 0; y < gh; ++y)
    for (int x = 0; x < gw; ++x) {
      ++cell;
      if (!can_add(st, index, x, y)) continue;
      for (int pid : st.cells[index][cell]) {
        collect_candidates(st, index, indexes, st.pts[index][pid], vcp);
        int count = 0;
        bool have_best = false;
        pmvs_refined best;
        float best_score = 0.0f;  // a default CPatch scores max(0, -1 - thr) * 0 = 0
        for (const SeedCand& c : vcp) {
          ++st.counts[index][cell];
          if (c.view < s.tnum) ++st.counts[c.view][c.cell];
          pmvs_candidate cand;
          seed_candidate(s, index, c, cand);
          pmvs_refined r;
          refine_one(s, ctx, cand, r);
          ++st.trial;
          if (r.status == PMVS_FAIL_PRE) { ++st.fail0; continue; }
          if (r.status != PMVS_ACCEPTED) { ++st.fail1; continue; }
          ++st.pass;
          ++count;
          const float sc = seed_score(r, s.nccThreshold);
          if (best_score < sc) { best_score = sc; best = r; have_best = true; }
          if (2 <= count) break;  // _countThreshold0 = 2 (findMatch.cpp:95)
        }
        if (count != 0) {
          // addPatch(bestpatch), patchOrganizerS.cpp:308-331 at depth 0; a default CPatch
          // (no image scored above 0) registers nowhere and never reaches the model.
          if (have_best) {
            pmvs_patch pp;
            std::memset(&pp, 0, sizeof(pp));
            for (int k = 0; k < 4; ++k) { pp.coord[k] = best.coord[k]; pp.normal[k] = best.normal[k]; }
            pp.ncc = best.ncc; pp.dscale = best.dscale; pp.ascale = best.ascale; pp.tmp = best.tmp;
            pp.timages = best.timages;
            pp.num_images = best.num_images;
            for (int k = 0; k < best.num_images; ++k) {
              pp.images[k] = (int16_t)best.images[k];
              pp.grids[k][0] = cell16(best.grids[k][0]);
              pp.grids[k][1] = cell16(best.grids[k][1]);
              const int t = best.images[k];
              if (t < s.tnum) {
                const int gx = best.grids[k][0], gy = best.grids[k][1];
                // the reference indexes _pgrids without a bounds check; grids of accepted patches
                // lie inside the image (the patch projects inside every image it keeps)
                if (0 <= gx && gx < s.gwidths[t] && 0 <= gy && gy < s.gheights[t])
                  st.occupied[t][gy * s.gwidths[t] + gx] = 1;
              }
            }
            out.push_back(pp);
          }
          break;
        }
      }
    }
}

// The target-image order of CSeed::run (seed.cpp:53-60).
static std::vector<int> seed_order(int tnum) {
  std::vector<int> v(tnum);
  for (int i = 0; i < tnum; ++i) v[i] = i;
  std::mt19937 gen(42);
  std::shuffle(v.begin(), v.end(), gen);
  return v;
}

// CSeed::init + readPoints + run (seed.cpp:11-107) with CPU = 1.
static void seed_run(const OScene& s, const std::vector<std::vector<SeedPoint>>& points, std::vector<pmvs_patch>& out,
                     int64_t stats[4]) {
  SeedState st(s);
  st.pts = points;
  st.cells.resize(s.num);
  for (int i = 0; i < s.num; ++i) {
    st.cells[i].assign((size_t)s.gwidths[i] * s.gheights[i], std::vector<int>());
    for (int q = 0; q < (int)points[i].size(); ++q) {
      const int ix = ((int)std::floor(points[i][q].x + 0.5f)) / s.csize;
      const int iy = ((int)std::floor(points[i][q].y + 0.5f)) / s.csize;
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
  OCtx ctx;
  init_ctx(s, ctx);
  out.clear();
  for (int index : seed_order(s.tnum)) initial_match(st, ctx, index, out);
  stats[0] = st.trial; stats[1] = st.pass; stats[2] = st.fail0; stats[3] = st.fail1;
}

}  // namespace oracle
