// oracle/expand_oracle.h -- TEST INFRASTRUCTURE ONLY (included by pmvs_oracle.cpp after
// filter_oracle.h).
//
// CPU restatement of one expansion run, PMVS3::CExpand::run (expand.cpp:17-406), on the model
// a filter pass leaves behind (alive patches + their cell registrations + depth maps), with the
// depth >= 1 steps of COptim::postProcess (optim.cpp:178-188: setVImagesVGrids and, at depth
// >= 2, check() = computeGain + findNeighbors + filterQuad, optim.cpp:363-381).
//
// Scheduling.  The reference pops the max-_tmp patch from a shared priority queue, one patch per
// thread at a time (P_compare, patchOrganizerS.hpp:10-15), and every expandSub sees whatever the
// other threads committed so far.  Here expansion proceeds in WAVES: the `wave` highest-priority
// queue entries (ties: earlier push first) are expanded against the model as it stood at the
// start of the wave, their candidates refined, and the results committed in (parent priority,
// direction) order, re-running checkCounts at commit time so two candidates of one wave cannot
// both claim a cell.  wave = 1 is the reference's single-thread (CPU 1) schedule exactly.
#pragma once

#include <queue>

namespace oracle {

struct ExpandStats {
  int64_t parents = 0, candidates = 0, fail_prep = 0, fail_pre = 0, fail_post = 0, fail_commit = 0, added = 0,
          waves = 0;
  int64_t wave_ns = 0;  // wall time of the waves (after the model load and queue setup)
};

struct Model {
  const OScene& s;
  Organizer o;
  std::vector<std::vector<unsigned char>> counts;  // CPatchOrganizerS::_counts per target cell
  explicit Model(const OScene& sc) : s(sc), o(sc) {
    counts.resize(s.tnum);
    for (int t = 0; t < s.tnum; ++t) counts[t].assign((size_t)s.gwidths[t] * s.gheights[t], 0);
  }
};

// Organizer state of a model given by its alive patches (as CFilter::run leaves it:
// pgrids = target entries, dpgrids = setDepthMaps over collect order, vpgrids = addPatchV).
static void model_load(Model& m, std::vector<FPatch>& P, const std::vector<int>& alive, bool depth_maps) {
  for (int p = 0; p < (int)P.size(); ++p)
    if (alive[p]) add_patch_p(m.o, P, p);
  collect_patches(m.o, P, 0);
  if (depth_maps) set_depth_maps(m.o, P);  // none after the seed phase (addPatch at depth 0)
  parallel_for(g_threads, (size_t)m.s.tnum, [&](int, size_t tt) {  // one target image per job
    const int t = (int)tt;
    for (int p : m.o.ppatches) {
      const FPatch& q = P[p];
      for (size_t i = 0; i < q.vimages.size(); ++i)
        if (q.vimages[i] == t) {
          if (m.o.in_grid(t, q.vgrids[i].first, q.vgrids[i].second))
            m.o.vpgrids[t][m.o.cell(t, q.vgrids[i].first, q.vgrids[i].second)].push_back(p);
          break;
        }
    }
  });
}

// CPatchOrganizerS::updateDepthMaps (patchOrganizerS.cpp:348-381).
static void update_depth_maps(Model& m, const std::vector<FPatch>& P, int p) {
  const OScene& s = m.s;
  for (int t = 0; t < s.tnum; ++t) {
    const V3 ic = project(s, t, P[p].coord, s.level);
    const float fx = ic[0] / s.csize, fy = ic[1] / s.csize;
    const int xs[2] = {(int)std::floor(fx), (int)std::ceil(fx)};
    const int ys[2] = {(int)std::floor(fy), (int)std::ceil(fy)};
    const float depth = depth_of(s, t, P[p].coord);
    for (int j = 0; j < 2; ++j)
      for (int i = 0; i < 2; ++i) {
        if (!m.o.in_grid(t, xs[i], ys[j])) continue;
        int& d = m.o.dpgrids[t][m.o.cell(t, xs[i], ys[j])];
        if (d == -1) d = p;
        else if (depth < depth_of(s, t, P[d].coord)) d = p;
      }
  }
}

// CPatchOrganizerS::addPatch (patchOrganizerS.cpp:308-346) at depth > 0.
static void model_add(Model& m, std::vector<FPatch>& P, int p) {
  add_patch_p(m.o, P, p);
  if (m.s.depth == 0) return;  // addPatch: no vpgrids / depth maps at depth 0 (patchOrganizerS.cpp:331)
  const FPatch& q = P[p];
  for (size_t i = 0; i < q.vimages.size(); ++i)
    m.o.vpgrids[q.vimages[i]][m.o.cell(q.vimages[i], q.vgrids[i].first, q.vgrids[i].second)].push_back(p);
  update_depth_maps(m, P, p);
}

// The candidate centre of direction i (expand.cpp:176-177): `const float angle = 2*M_PI*i/dnum;`
// then coord + cos(angle)*radius*xdir + sin(angle)*radius*ydir, where the float angle goes to the
// double cos/sin (unqualified cos(float) resolves to ::cos(double) in that TU; probed), the
// double scalar times a Vec4f rounds each component to float (vec4.hpp:177-184), and the two
// Vec4f sums run left to right.
static V4 candidate_coord(const V4& coord, const V4& xdir, const V4& ydir, float radius, int i, int dnum) {
  const float angle = (float)(2 * M_PI * i / dnum);
  const double cr = std::cos((double)angle) * (double)radius, sr = std::sin((double)angle) * (double)radius;
  V4 c;
  for (int k = 0; k < 4; ++k) c[k] = (coord[k] + (float)((double)xdir[k] * cr)) + (float)((double)ydir[k] * sr);
  return c;
}

// CExpand::findEmptyBlocks (expand.cpp:95-180): free directions of a patch.
static void find_empty_blocks(const Model& m, const std::vector<FPatch>& P, const FPatch& q, int dflag,
                              std::vector<std::pair<int, V4>>& out) {
  const OScene& s = m.s;
  const int dnum = 6;
  V4 xdir, ydir;
  ortho4(q.normal, xdir, ydir);
  float fill[6] = {0, 0, 0, 0, 0, 0};
  const float radius = compute_radius(s, q);
  const float radiuslow = radius / 6.0f, radiushigh = radius * 2.5f;
  std::vector<int> nb;
  find_neighbors(m.o, P, q, nb, 4.0f, 1, 0);
  for (int j : nb) {
    const V4 diff = sub4(P[j].coord, q.coord);
    float f2[2] = {dot4(diff, xdir), dot4(diff, ydir)};
    const float len = (float)std::sqrt((double)(f2[0] * f2[0] + f2[1] * f2[1]));
    if (len < radiuslow || radiushigh < len) continue;
    f2[0] /= len;
    f2[1] /= len;
    float angle = (float)std::atan2((double)f2[1], (double)f2[0]);
    if (angle < 0.0) angle = (float)((double)angle + 2 * M_PI);
    const float findex = (float)((double)angle / (2 * M_PI / dnum));
    const int lindex = (int)std::floor((double)findex);
    const int hindex = lindex + 1;
    fill[lindex % dnum] += hindex - findex;
    fill[hindex % dnum] += findex - lindex;
  }
  for (int i = 0; i < dnum; ++i) {
    if (0.0f < fill[i]) continue;
    if (dflag & (0x0001 << i)) continue;
    out.push_back({i, candidate_coord(q.coord, xdir, ydir, radius, i, dnum)});
  }
}

// CExpand::checkCounts (expand.cpp:268-323).
static int check_counts(const Model& m, const FPatch& q, int cthr, int depth) {
  const OScene& s = m.s;
  int full = 0, empty = 0;
  for (size_t i = 0; i < q.images.size(); ++i) {
    const int t = q.images[i];
    if (s.tnum <= t) continue;
    const int ix = q.grids[i].first, iy = q.grids[i].second;
    if (!m.o.in_grid(t, ix, iy)) continue;
    const int c = m.o.cell(t, ix, iy);
    if (!m.o.pgrids[t][c].empty()) {
      ++full;
      continue;
    }
    if (cthr <= m.counts[t][c]) ++full;
    else ++empty;
  }
  if (depth <= 1) return (empty < s.minImageNum && full != 0) ? 1 : 0;
  return (empty < s.minImageNum - 1 && full != 0) ? 1 : 0;
}

// CExpand::updateCounts (expand.cpp:325-406).
static int update_counts(Model& m, const FPatch& q, int cthr) {
  const OScene& s = m.s;
  int full = 0, empty = 0;
  auto touch = [&](int t, int ix, int iy) {
    if (!m.o.in_grid(t, ix, iy)) return;
    unsigned char& c = m.counts[t][m.o.cell(t, ix, iy)];
    if (cthr <= c) ++full;
    else ++empty;
    ++c;
  };
  for (size_t i = 0; i < q.images.size(); ++i)
    if (q.images[i] < s.tnum) touch(q.images[i], q.grids[i].first, q.grids[i].second);
  for (size_t i = 0; i < q.vimages.size(); ++i) touch(q.vimages[i], q.vgrids[i].first, q.vgrids[i].second);
  return empty != 0 ? 1 : 0;
}

struct Cand {
  int parent, dir;
  V4 coord;                      // findEmptyBlocks' canCoord
  FPatch prep;                   // after setGridsImages (the checkCounts input)
  std::vector<int> edge_images;  // after removeImagesEdge (the preProcess input)
  FPatch out;                    // refined patch
  int status;                    // 0 ok, 1 prep fail, 2 preProcess fail, 3 postProcess fail
};

// CPatchOrganizerS::setGridsImages (patchOrganizerS.cpp:383-399): c.images / c.grids := the entries of
// `images` whose cell at c.coord lies in the target's grid.  Pinned to the reference's own
// patchOrganizerS.cpp (tests/test_organizer_pinning.py).
static void set_grids_images(const OScene& s, const std::vector<int>& images, FPatch& c) {
  c.images.clear();
  c.grids.clear();
  for (int t : images) {
    const V3 ic = project(s, t, c.coord, s.level);
    const int ix = ((int)std::floor(ic[0] + 0.5f)) / s.csize;
    const int iy = ((int)std::floor(ic[1] + 0.5f)) / s.csize;
    if (0 <= ix && ix < s.gwidths[t] && 0 <= iy && iy < s.gheights[t]) {
      c.images.push_back(t);
      c.grids.push_back({ix, iy});
    }
  }
}

// expandSub up to the refine (expand.cpp:200-226): returns 0 when the candidate goes on.
static int prepare_candidate(const Model& m, const FPatch& par, const V4& coord, int cthr, int depth, FPatch& c,
                             std::vector<int>& edge_images) {
  const OScene& s = m.s;
  c = FPatch();
  c.coord = coord;
  c.normal = par.normal;
  c.flag = 1;
  c.ncc = -1.0f; c.dscale = 0.0f; c.ascale = 0.0f; c.tmp = 0.0f; c.timages = 0; c.fix = 0;
  set_grids_images(s, par.images, c);
  if (c.images.empty()) return 1;
  if (get_mask_all(s, coord, s.level) == 0 || inside_bimages(s, coord) == 0) return 1;
  if (check_counts(m, c, cthr, depth)) return 1;
  edge_images.clear();  // COptim::removeImagesEdge (optim.cpp:384-396)
  for (int t : c.images)
    if (get_edge(s, coord, t, s.level)) edge_images.push_back(t);
  if (edge_images.empty()) return 1;
  return 0;
}

// preProcess -> refinePatch -> postProcess (+ depth >= 1 steps) for one prepared candidate.
static int refine_candidate(const Model& m, const std::vector<FPatch>& P, OCtx& ctx, const FPatch& c,
                            const std::vector<int>& images, FPatch& out) {
  const OScene& s = m.s;
  OPatch p;
  p.coord = c.coord;
  p.normal = c.normal;
  p.images = images;
  p.dscale = 0.0f;
  p.ncc = -1.0f;
  out = c;
  if (pre_process(s, ctx, p)) return 2;
  int ev = 0;
  refine_patch(s, ctx, p, &ev);
  const int post = post_process(s, ctx, p);
  out.coord = p.coord; out.normal = p.normal; out.images = p.images; out.grids = p.grids;
  out.ncc = p.ncc; out.dscale = p.dscale; out.ascale = p.ascale; out.tmp = p.tmp; out.timages = p.timages;
  out.vimages.clear();
  out.vgrids.clear();
  if (post) return 3;
  if (s.depth) {
    set_vimages_vgrids(m.o, P, out);
    if (2 <= s.depth) {  // COptim::check (optim.cpp:363-381)
      const float gain = compute_gain(m.o, P, out);
      out.tmp = gain;
      if (gain < 0.0) return 3;
      std::vector<int> nb;
      find_neighbors(m.o, P, out, nb, 4.0f, 2, 0);
      if (6 < (int)nb.size() && filter_quad(s, P, out, nb)) return 3;
    }
  }
  return 0;
}

struct QItem {
  float tmp;
  int64_t seq;
  int p;
};
struct QCmp {
  bool operator()(const QItem& a, const QItem& b) const {  // max-heap on tmp, then earliest push
    if (a.tmp != b.tmp) return a.tmp < b.tmp;
    return a.seq > b.seq;
  }
};

// CExpand::run (expand.cpp:17-72) in waves.
// A wave is `wave` parents, extended by further chunks of `wave` parents (popped in queue order,
// their free directions found against the same start-of-wave model) while it holds fewer than
// `min_cands` candidate directions: late passes, where most parents are already surrounded, then
// batch enough refinements per wave.  min_cands = 0 (or wave = 1) keeps plain waves.
// nthreads > 1 runs findEmptyBlocks, the candidate preparation and the refinements of one wave
// on a std::thread pool (one scratch context per thread, the reference's threading model,
// expand.cpp:41-52); they only read the start-of-wave model, so the result is identical for every
// thread count.  max_waves > 0 stops after that many waves (bounded CPU-baseline samples).
static void expand_run(const OScene& s, std::vector<FPatch>& P, std::vector<int>& alive, int wave, int cthr, int flags,
                       ExpandStats& st, int min_cands = 0, int nthreads = 1, int64_t max_waves = 0) {
  Model m(s);
  nthreads = std::max(1, nthreads);
  std::vector<OCtx> ctxs(nthreads);
  for (auto& c : ctxs) init_ctx(s, c);
  model_load(m, P, alive, (flags & 1) == 0);
  for (int p : m.o.ppatches) P[p].flag = 0;  // clearFlags
  std::priority_queue<QItem, std::vector<QItem>, QCmp> queue;
  int64_t seq = 0;
  for (int t = 0; t < s.tnum; ++t)  // collectPatches(queue), patchOrganizerS.cpp:250-262
    for (auto& cellv : m.o.pgrids[t])
      for (int p : cellv)
        if (P[p].flag == 0) {
          P[p].flag = 1;
          // another cluster's boundary patch (pmvs_scene_set_cluster, fix = PMVS_FIX_FOREIGN) is never expanded here
          if (P[p].fix != PMVS_FIX_FOREIGN) queue.push({P[p].tmp, seq++, p});
        }
  const int W = std::max(1, wave);
  const auto t_waves = std::chrono::steady_clock::now();
  while (!queue.empty() && (max_waves <= 0 || st.waves < max_waves)) {
    st.waves++;
    // Every parent's free directions are found against the model at the start of the wave
    // (expand.cpp:92-93); wave = 1 then prepares, refines and commits them one after the other
    // (expand.cpp:95-101, the single-thread schedule), wider waves do so as one batch and
    // re-run checkCounts at commit.
    std::vector<int> parents;
    std::vector<Cand> dirs;
    do {
      std::vector<int> chunk;
      while (!queue.empty() && (int)chunk.size() < W) {
        chunk.push_back(queue.top().p);
        queue.pop();
      }
      std::vector<std::vector<std::pair<int, V4>>> found(chunk.size());
      parallel_for(W > 1 ? nthreads : 1, chunk.size(),
                   [&](int, size_t k) { find_empty_blocks(m, P, P[chunk[k]], P[chunk[k]].dflag, found[k]); });
      for (size_t k = 0; k < chunk.size(); ++k) {
        const int par = chunk[k];
        for (auto& x : found[k]) {
          Cand c;
          c.parent = par;
          c.dir = x.first;
          c.coord = x.second;
          dirs.push_back(std::move(c));
        }
      }
      parents.insert(parents.end(), chunk.begin(), chunk.end());
    } while (W > 1 && (int64_t)dirs.size() < min_cands && !queue.empty());
    st.parents += (int64_t)parents.size();
    auto batch = [&](size_t b, size_t e, bool recheck) {
      const int T = e - b > 1 ? nthreads : 1;
      parallel_for(T, e - b, [&](int, size_t k) {
        Cand& c = dirs[b + k];
        c.status = prepare_candidate(m, P[c.parent], c.coord, cthr, s.depth, c.prep, c.edge_images) ? 1 : 0;
      });
      st.candidates += (int64_t)(e - b);
      parallel_for(T, e - b, [&](int tid, size_t k) {
        Cand& c = dirs[b + k];
        if (c.status == 0) c.status = refine_candidate(m, P, ctxs[tid], c.prep, c.edge_images, c.out);
      });
      for (size_t i = b; i < e; ++i) {
        Cand& c = dirs[i];
        int status = c.status;
        if (status == 0 && recheck && check_counts(m, c.prep, cthr, s.depth)) status = 4;
        if (status != 0) {
          P[c.parent].dflag |= 0x0001 << c.dir;
          if (status == 1) st.fail_prep++;
          else if (status == 2) st.fail_pre++;
          else if (status == 3) st.fail_post++;
          else st.fail_commit++;
          continue;
        }
        FPatch np = c.out;
        np.flag = 1;
        np.fix = 0;
        np.dflag = 0;
        const int add = update_counts(m, np, cthr);
        P.push_back(np);
        alive.push_back(1);
        const int id = (int)P.size() - 1;
        model_add(m, P, id);
        st.added++;
        if (add) queue.push({P[id].tmp, seq++, id});
      }
    };
    if (W == 1)
      for (size_t i = 0; i < dirs.size(); ++i) batch(i, i + 1, false);
    else
      batch(0, dirs.size(), true);
  }
  st.wave_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_waves).count();
}

}  // namespace oracle
