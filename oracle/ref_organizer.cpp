// oracle/ref_organizer.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Runs pieces of the reference's own CPatchOrganizerS and CPhotoSetS, compiled unmodified from
// $(REF)/source/pmvs/patchOrganizerS.cpp and $(REF)/source/image/photoSetS.cpp (with camera.cpp and
// patch.cpp) by oracle/Makefile, so the restatements in oracle/expand_oracle.h, filter_oracle.h,
// seed_oracle.h and pmvs_oracle.cpp are pinned to reference object code
// (tests/test_organizer_pinning.py):
//   op 1  CPatchOrganizerS::setGridsImages   patchOrganizerS.cpp:383-399
//   op 2  CPatchOrganizerS::setGrids         patchOrganizerS.cpp:405-415
//   op 3  CPatchOrganizerS::updateDepthMaps  patchOrganizerS.cpp:351-381 (patches added in order)
//   op 4  CPatchOrganizerS::isVisible0       patchOrganizerS.cpp:479-486 at _depth == 0
//   op 5  CPhotoSetS::checkAngles            photoSetS.cpp:164-189
//   op 6  CPhotoSetS::setDistances           photoSetS.cpp:195-234
//   also  CPatchOrganizerS::init             patchOrganizerS.cpp:50-82 (the cell grids every op uses)
//
// No CFindMatch can be constructed here: its COptim / CSeed / CExpand / CFilter members live in TUs
// that need nlopt, CImg and Eigen, and so does CPhoto's constructor (its CImage base, image.cpp).
// Those symbols stay unresolved (non-PIE, --unresolved-symbols=ignore-all) and are never called; no
// stand-in is written for any of them.  Instead the members the functions above read are
// materialised in raw storage of the classes' sizes, each by its own (reference) constructor or
// initialiser where one exists: CCamera's constructor and init (camera.cpp) for every view's camera
// base, CPhotoSetS's constructor, CPatchOrganizerS's constructor and init.  The CImage part of a
// CPhoto holds only its level sizes (_widths / _heights / _alloc, which getWidth / getHeight read),
// named through a probe subclass as oracle/ref_driver.cpp does.  Out of reach: isVisible at _depth
// > 0 calls COptim::getUnit (optim.cpp, nlopt) -- DESIGN.md §6.
//
// stdin (little-endian int32 / float32):
//   num, tnum, level, csize, maxLevel, then per view: path length, path bytes (a CONTOUR camera
//   file), widths[maxLevel], heights[maxLevel]; then operations until EOF:
//   1/2: n, then n x {coord[4], m, images[m]}      -> per record: m', then m' x {image, ix, iy}
//   3:   n, then n x coord[4]                      -> per target: gw*gh cells (patch index or -1)
//   4:   n, then n x {coord[4], image}             -> n x {visible, ix, iy}
//   5:   n, minAngle, maxAngle, then n x {coord[4], m, indexes[m]} -> n x result
//   6:   (nothing)                                 -> num x num float32
#include <cstdint>
#include <cstdio>
#include <new>
#include <shared_mutex>
#include <string>
#include <vector>

#include "pmvs/findMatch.hpp"

namespace {
struct FmProbe : public PMVS3::CFindMatch {
  static auto tnum() { return &FmProbe::_tnum; }
  static auto num() { return &FmProbe::_num; }
  static auto locks() { return &FmProbe::_imageLocks; }
};
struct ImgProbe : public Image::CImage {
  static auto widths() { return &ImgProbe::_widths; }
  static auto heights() { return &ImgProbe::_heights; }
  static auto alloc() { return &ImgProbe::_alloc; }
};

bool rd(void* p, size_t n) { return std::fread(p, 1, n, stdin) == n; }
int32_t ri() {
  int32_t v = 0;
  if (!rd(&v, 4)) throw 1;
  return v;
}
float rf() {
  float v = 0;
  if (!rd(&v, 4)) throw 1;
  return v;
}
void wi(int32_t v) { std::fwrite(&v, 4, 1, stdout); }
Vec4f rcoord() {
  float c[4];
  if (!rd(c, 16)) throw 1;
  return Vec4f(c[0], c[1], c[2], c[3]);
}
}  // namespace

int main() {
  try {
    const int num = ri(), tnum = ri(), level = ri(), csize = ri(), maxLevel = ri();
    alignas(PMVS3::CFindMatch) static unsigned char raw[sizeof(PMVS3::CFindMatch)];
    PMVS3::CFindMatch& fm = *reinterpret_cast<PMVS3::CFindMatch*>(raw);
    fm._level = level;
    fm._csize = csize;
    fm._depth = 0;
    fm.*FmProbe::tnum() = tnum;
    fm.*FmProbe::num() = num;
    new (&(fm.*FmProbe::locks())) std::vector<std::shared_mutex*>();
    for (int i = 0; i < num; ++i) (fm.*FmProbe::locks()).push_back(new std::shared_mutex());
    new (&fm._pss) Image::CPhotoSetS();
    fm._pss._num = num;
    fm._pss._photos.reserve(num);  // storage only: a CPhoto cannot be constructed (see the header)
    Image::CPhoto* photos = fm._pss._photos.data();
    for (int v = 0; v < num; ++v) {
      const int len = ri();
      std::string path((size_t)len, '\0');
      if (!rd(&path[0], (size_t)len)) return 2;
      Image::CCamera* cam = static_cast<Image::CCamera*>(&photos[v]);
      new (cam) Image::CCamera();
      cam->init(path, maxLevel);
      Image::CImage* im = static_cast<Image::CImage*>(&photos[v]);
      std::vector<int> w((size_t)maxLevel), h((size_t)maxLevel);
      for (int l = 0; l < maxLevel; ++l) w[l] = ri();
      for (int l = 0; l < maxLevel; ++l) h[l] = ri();
      new (&(im->*ImgProbe::widths())) std::vector<int>(w);
      new (&(im->*ImgProbe::heights())) std::vector<int>(h);
      im->*ImgProbe::alloc() = 1;
    }
    PMVS3::CPatchOrganizerS org(fm);
    org.init();

    int32_t op = 0;
    while (rd(&op, 4)) {
      if (op == 1 || op == 2) {
        const int n = ri();
        for (int r = 0; r < n; ++r) {
          Patch::CPatch p;
          p._coord = rcoord();
          const int m = ri();
          std::vector<int> images((size_t)m);
          for (int k = 0; k < m; ++k) images[k] = ri();
          if (op == 1) {
            org.setGridsImages(p, images);
          } else {
            p._images = images;
            org.setGrids(p);
          }
          wi((int32_t)p._images.size());
          for (size_t k = 0; k < p._images.size(); ++k) {
            wi(p._images[k]);
            wi(p._grids[k][0]);
            wi(p._grids[k][1]);
          }
        }
      } else if (op == 3) {
        const int n = ri();
        std::vector<Patch::PPatch> pp((size_t)n);
        for (int r = 0; r < n; ++r) {
          pp[r].reset(new Patch::CPatch());
          pp[r]->_coord = rcoord();
          org.updateDepthMaps(pp[r]);
        }
        for (int t = 0; t < tnum; ++t)
          for (const Patch::PPatch& d : org._dpgrids[t]) {
            int32_t idx = -1;
            if (d != PMVS3::CPatchOrganizerS::_MAXDEPTH)
              for (int r = 0; r < n; ++r)
                if (pp[r] == d) {
                  idx = r;
                  break;
                }
            wi(idx);
          }
        // back to the initial state for the next operation
        for (int t = 0; t < tnum; ++t)
          for (Patch::PPatch& d : org._dpgrids[t]) d = PMVS3::CPatchOrganizerS::_MAXDEPTH;
      } else if (op == 4) {
        const int n = ri();
        for (int r = 0; r < n; ++r) {
          Patch::CPatch p;
          p._coord = rcoord();
          const int image = ri();
          int ix = 0, iy = 0;
          const int vis = org.isVisible0(p, image, ix, iy, fm._neighborThreshold, 1);
          wi(vis);
          wi(ix);
          wi(iy);
        }
      } else if (op == 5) {
        const int n = ri();
        const float minA = rf(), maxA = rf();
        for (int r = 0; r < n; ++r) {
          const Vec4f c = rcoord();
          const int m = ri();
          std::vector<int> idx((size_t)m);
          for (int k = 0; k < m; ++k) idx[k] = ri();
          wi(fm._pss.checkAngles(c, idx, minA, maxA, 0));
        }
      } else if (op == 6) {
        fm._pss.setDistances();
        for (int i = 0; i < num; ++i)
          std::fwrite(fm._pss._distances[i].data(), 4, (size_t)num, stdout);
      } else {
        return 2;
      }
    }
    std::fflush(stdout);
    std::_Exit(0);  // the raw-storage objects are never destroyed (their CImage / CFindMatch
                    // destructors live in the unbuilt TUs)
  } catch (int) {
    return 2;
  }
}
