// tests/csrc/integration_example.cpp -- TEST INFRASTRUCTURE: the reference-side binding that
// INTEGRATION.md shows, as one translation unit.  tests/test_integration_doc.py checks that every
// ```cpp block of INTEGRATION.md occurs in this file and, where /root/reference exists (the build
// container), compiles it with -fsyntax-only against the reference's own headers and
// include/pmvs_amd.h -- so the documented binding type-checks against both sides of the boundary.
#include <algorithm>
#include <iostream>
#include <memory>
#include <vector>

#include "pmvs/findMatch.hpp"
#include "pmvs_amd.h"

namespace pmvs_integration {

// ---- §1 scene setup
pmvs_scene* make_scene(PMVS3::CFindMatch& fm, int device) {
  const int n = fm.NumImages();                // targets first, then other images
  std::vector<pmvs_view_desc> views(n);
  for (int i = 0; i < n; ++i) {
    const Image::CPhoto& ph = fm._pss._photos[i];
    views[i].width = ph.getWidth(0);
    views[i].height = ph.getHeight(0);
    views[i].rgb = ph.getImage(0).data();      // level-0 RGB8, row-major
    views[i].mask = ph.isMask() ? ph.Image::CImage::getMask(0).data() : nullptr;
    views[i].edge = ph.isEdge() ? ph.Image::CImage::getEdge(0).data() : nullptr;
    for (int y = 0; y < 3; ++y)                // level-0 projection rows (camera.cpp:56-68)
      for (int x = 0; x < 4; ++x) views[i].projection[4 * y + x] = ph.ProjectionMatrix()[0][y][x];
  }
  std::vector<int> vis_off, vis;               // SOption::_visdata2 as CSR
  vis_off.push_back(0);
  for (const auto& row : fm._visdata2) { vis.insert(vis.end(), row.begin(), row.end()); vis_off.push_back((int)vis.size()); }

  pmvs_scene_desc d{};
  d.num_views = n;            d.num_targets = fm.NumTargetImages();
  d.level = fm._level;        d.csize = fm._csize;         d.wsize = fm._wsize;
  d.min_image_num = fm._minImageNumThreshold;
  d.threshold = fm._nccThreshold;  d.max_angle = fm._maxAngleThreshold;
  d.quad_threshold = fm._quadThreshold;  d.sequence = fm._sequenceThreshold;
  d.visdata2_offsets = vis_off.data();  d.visdata2 = vis.data();
  d.num_bindexes = (int)fm._bindexes.size();  d.bindexes = fm._bindexes.data();
  d.views = views.data();

  pmvs_scene* s = nullptr;
  if (pmvs_scene_create(&d, device, &s) != PMVS_OK) {
    std::cerr << "pmvs_scene_create: " << pmvs_last_error() << std::endl;
    return nullptr;
  }
  return s;
}

// ---- §2 seed call site (CSeed::initialMatchSub, seed.cpp:387-414), depth 0
// status[i]: 0 accepted, 1 rejected by preProcess (_fcounts0), 2 rejected by postProcess (_fcounts1)
int refine_seed_candidates(pmvs_scene* scene, std::vector<Patch::CPatch>& batch, std::vector<int>& status) {
  std::vector<pmvs_candidate> in(batch.size());
  for (size_t i = 0; i < batch.size(); ++i) {
    const Patch::CPatch& p = batch[i];
    for (int k = 0; k < 4; ++k) { in[i].coord[k] = p._coord[k]; in[i].normal[k] = p._normal[k]; }
    in[i].dscale = p._dscale;
    in[i].num_images = (int)p._images.size();
    std::copy(p._images.begin(), p._images.end(), in[i].images);
  }
  std::vector<pmvs_refined> out(batch.size());
  pmvs_stats st{};
  if (pmvs_refine_batch(scene, in.data(), (int)in.size(), out.data(), &st) != PMVS_OK) {
    std::cerr << "pmvs_refine_batch: " << pmvs_last_error() << std::endl;
    return 1;
  }
  status.assign(batch.size(), 0);
  for (size_t i = 0; i < batch.size(); ++i) {
    const pmvs_refined& r = out[i];
    if (r.status == PMVS_FAIL_PRE) { status[i] = 1; continue; }
    if (r.status != PMVS_ACCEPTED) { status[i] = 2; continue; }
    Patch::CPatch& p = batch[i];
    for (int k = 0; k < 4; ++k) { p._coord[k] = r.coord[k]; p._normal[k] = r.normal[k]; }
    p._ncc = r.ncc;  p._dscale = r.dscale;  p._ascale = r.ascale;
    p._tmp = r.tmp;  p._timages = r.timages;
    p._images.assign(r.images, r.images + r.num_images);
    p._grids.resize(r.num_images);
    for (int k = 0; k < r.num_images; ++k) p._grids[k] = TVec2<int>(r.grids[k][0], r.grids[k][1]);
  }
  return 0;
}

// ---- §3 expansion call site: one CExpand::run (expand.cpp:17-72, whose expandSub at
// expand.cpp:200-266 needs the organizer at depth >= 1) becomes one pmvs_expand_run
// pmvs_patch keeps its lists as int16 (include/pmvs_amd.h): a cell coordinate outside the int16
// range (a projection far outside the image) is stored as -32768, which no in-grid test accepts
static int16_t cell16(int v) { return (v < -32767 || v > 32767) ? (int16_t)-32768 : (int16_t)v; }

// returns false when a list is longer than PMVS_MAX_IMAGES (never truncated)
static bool to_pmvs(const Patch::CPatch& p, pmvs_patch& a) {
  a = pmvs_patch{};
  if (p._images.size() > PMVS_MAX_IMAGES || p._vimages.size() > PMVS_MAX_IMAGES) return false;
  for (int k = 0; k < 4; ++k) { a.coord[k] = p._coord[k]; a.normal[k] = p._normal[k]; }
  a.ncc = p._ncc;  a.dscale = p._dscale;  a.ascale = p._ascale;  a.tmp = p._tmp;
  a.timages = p._timages;  a.flag = p._flag;  a.fix = p._fix;  a.dflag = p._dflag;
  a.num_images = (int)p._images.size();
  for (int k = 0; k < a.num_images; ++k) {
    a.images[k] = (int16_t)p._images[k];  a.grids[k][0] = cell16(p._grids[k][0]);  a.grids[k][1] = cell16(p._grids[k][1]);
  }
  a.num_vimages = (int)p._vimages.size();
  for (int k = 0; k < a.num_vimages; ++k) {
    a.vimages[k] = (int16_t)p._vimages[k];  a.vgrids[k][0] = cell16(p._vgrids[k][0]);  a.vgrids[k][1] = cell16(p._vgrids[k][1]);
  }
  return true;
}

static void from_pmvs(const pmvs_patch& a, Patch::CPatch& p) {
  for (int k = 0; k < 4; ++k) { p._coord[k] = a.coord[k]; p._normal[k] = a.normal[k]; }
  p._ncc = a.ncc;  p._dscale = a.dscale;  p._ascale = a.ascale;  p._tmp = a.tmp;
  p._timages = a.timages;  p._flag = a.flag;  p._fix = (char)a.fix;  p._dflag = (unsigned char)a.dflag;
  p._images.assign(a.images, a.images + a.num_images);
  p._grids.clear();
  for (int k = 0; k < a.num_images; ++k) p._grids.push_back(TVec2<int>(a.grids[k][0], a.grids[k][1]));
  p._vimages.assign(a.vimages, a.vimages + a.num_vimages);
  p._vgrids.clear();
  for (int k = 0; k < a.num_vimages; ++k) p._vgrids.push_back(TVec2<int>(a.vgrids[k][0], a.vgrids[k][1]));
}

// ---- §2b the whole seed phase: CSeed::run (seed.cpp:40-107) on the device, from the points
// CDetectFeatures produced (or pmvs_detect_features); the seeds are added as CSeed does
int seeds_on_device(PMVS3::CFindMatch& fm, pmvs_scene* scene, const std::vector<std::vector<PMVS3::CPoint>>& points) {
  std::vector<pmvs_point> flat;
  std::vector<int32_t> counts;
  for (const auto& view : points) {            // one entry per image index, detector order
    counts.push_back((int32_t)view.size());
    for (const PMVS3::CPoint& p : view) flat.push_back({p._icoord[0], p._icoord[1], p._response, p._type});
  }
  int32_t n = 0;
  pmvs_seed_stats st{};
  // out = NULL, cap = 0: the scene keeps the seeds until pmvs_seed_fetch (sized from n)
  if (pmvs_seed_run(scene, flat.data(), counts.data(), /*batch*/ 0, nullptr, 0, &n, &st) != PMVS_OK) {
    std::cerr << "pmvs_seed_run: " << pmvs_last_error() << std::endl;
    return 1;
  }
  std::vector<pmvs_patch> seeds(std::max(n, 1));
  if (pmvs_seed_fetch(scene, seeds.data(), n) != PMVS_OK) return 1;
  for (int i = 0; i < n; ++i) {                // addPatch order of the reference's CPU 1 run
    Patch::PPatch pp(new Patch::CPatch());
    from_pmvs(seeds[i], *pp);
    fm._pos.addPatch(pp);
  }
  return 0;
}

int expand_on_device(PMVS3::CFindMatch& fm, pmvs_scene* scene, bool after_seeds) {
  fm._pos.collectPatches();                    // the model = _ppatches (patchOrganizerS.cpp:228-248)
  const int n = (int)fm._pos._ppatches.size();
  std::vector<pmvs_patch> model(n);
  std::vector<int32_t> alive(n, 1);
  for (int i = 0; i < n; ++i)
    if (!to_pmvs(*fm._pos._ppatches[i], model[i])) return 1;  // list > PMVS_MAX_IMAGES
  pmvs_set_thresholds(scene, fm._nccThreshold, fm._nccThresholdBefore, fm._depth);
  int32_t n_out = 0;
  pmvs_expand_stats st{};
  if (pmvs_expand_run(scene, model.data(), alive.data(), n, /*wave*/ 32768, /*min_candidates*/ 131072,
                      fm._countThreshold1, after_seeds ? PMVS_EXPAND_AFTER_SEEDS : 0, nullptr, nullptr,
                      /*cap*/ 1 << 30, &n_out, &st) != PMVS_OK) {
    std::cerr << "pmvs_expand_run: " << pmvs_last_error() << std::endl;
    return 1;
  }
  std::vector<pmvs_patch> out(n_out);
  std::vector<int32_t> alive_out(n_out);
  pmvs_expand_fetch(scene, out.data(), alive_out.data(), n_out);
  for (int i = 0; i < n; ++i) {                // old patches: _flag / _dflag updated
    fm._pos._ppatches[i]->_flag = out[i].flag;
    fm._pos._ppatches[i]->_dflag = (unsigned char)out[i].dflag;
  }
  for (int i = n; i < n_out; ++i) {            // new patches, in commit order
    Patch::PPatch pp(new Patch::CPatch());
    from_pmvs(out[i], *pp);
    fm._pos.addPatch(pp);
  }
  return 0;
}

// ---- §4 the whole loop (findMatch.cpp:196-217 after the seed phase)
int run_loop_on_device(PMVS3::CFindMatch& fm, pmvs_scene* scene, std::vector<pmvs_patch>& model) {
  fm._pos.collectPatches();
  std::vector<pmvs_patch> seeds(fm._pos._ppatches.size());
  for (size_t i = 0; i < seeds.size(); ++i)
    if (!to_pmvs(*fm._pos._ppatches[i], seeds[i])) return 1;
  std::vector<pmvs_loop_iter> it(3);
  int32_t n = 0;
  if (pmvs_run_loop(scene, seeds.data(), (int)seeds.size(), fm._nccThreshold, /*iterations*/ 3,
                    /*wave*/ 32768, /*min_candidates*/ 131072, PMVS_EXPAND_AFTER_SEEDS,
                    /*cap*/ 1 << 30, &n, it.data()) != PMVS_OK) {
    std::cerr << "pmvs_run_loop: " << pmvs_last_error() << std::endl;
    return 1;
  }
  model.resize(n);
  return pmvs_loop_fetch(scene, model.data(), n) == PMVS_OK ? 0 : 1;
}

}  // namespace pmvs_integration
