// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver around the reference's own, unmodified translation units that
// compile in this image without any stand-in headers (see oracle/Makefile):
//   /root/reference/source/image/camera.cpp  (CCamera: CONTOUR parsing, per-level projections,
//                                             optical centre/axis, camera axes)
//   /root/reference/source/pmvs/option.cpp   (SOption: pmvs2 option-file parsing, vis.dat)
//   /root/reference/source/pmvs/patch.cpp    (CPatch text serialisation, operator<< / >>)
//   /root/reference/source/pmvs/{harris,dog,detector,point}.cpp  (the feature detectors)
// plus the header-only numeric library (include/numeric/*.hpp) and the inline
// CCamera::project (include/image/camera.hpp:89-108).  The resulting oracle/_ref/libpmvs_ref.so
// pins the oracle restatement and the product's host plumbing bit-for-bit on those pieces.
// It is built only in the build container (where /root/reference exists) and is never
// linked into the product.
#define _USE_MATH_DEFINES
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <limits>
#include <sstream>
#include <string>

#include <new>
#include <vector>

#include <set>

#include "image/camera.hpp"
#include "numeric/mat3.hpp"
#include "numeric/mat4.hpp"
#include "image/image.hpp"
#include "pmvs/dog.hpp"
#include "pmvs/harris.hpp"
#include "pmvs/option.hpp"
#include "pmvs/patch.hpp"

namespace {
// Exposes the protected camera axes computed by CCamera::updateCamera (camera.cpp:117-121),
// which are the same formulas COptim::setAxesScales uses (optim.cpp:48-52).
struct CamProbe : public Image::CCamera {
  void axes(float* out) const {
    for (int i = 0; i < 3; ++i) {
      out[i] = _xaxis[i];
      out[3 + i] = _yaxis[i];
      out[6 + i] = _zaxis[i];
    }
  }
};
// CImage's constructor and destructor live in image.cpp, which needs CImg.h (absent here), so
// a CImage object cannot be constructed in this recipe.  CImage::getColor
// (image.hpp:435-476, bilinear branch) and CImage::isSafe (image.hpp:165-178) are header-inline,
// non-virtual, and read only _images / _widths / _heights.  ImgProbe names those protected
// members; ref_get_color placement-constructs exactly those three vectors inside raw storage
// of CImage's size and calls the reference's own inline functions on it (no stand-in header,
// no restated code: the arithmetic executed is the unmodified header's).
struct ImgProbe : public Image::CImage {
  static auto images() { return &ImgProbe::_images; }
  static auto widths() { return &ImgProbe::_widths; }
  static auto heights() { return &ImgProbe::_heights; }
};

struct RawImage {
  alignas(Image::CImage) unsigned char raw[sizeof(Image::CImage)];
  Image::CImage* im() { return reinterpret_cast<Image::CImage*>(raw); }
  RawImage(const unsigned char* rgb, int w, int h) {
    using VU = std::vector<std::vector<unsigned char>>;
    using VI = std::vector<int>;
    new (&(im()->*ImgProbe::images())) VU(1, std::vector<unsigned char>(rgb, rgb + (size_t)3 * w * h));
    new (&(im()->*ImgProbe::widths())) VI(1, w);
    new (&(im()->*ImgProbe::heights())) VI(1, h);
  }
  ~RawImage() {
    using VU = std::vector<std::vector<unsigned char>>;
    using VI = std::vector<int>;
    (im()->*ImgProbe::images()).~VU();
    (im()->*ImgProbe::widths()).~VI();
    (im()->*ImgProbe::heights()).~VI();
  }
};
}  // namespace

extern "C" {

// CImage::getColor(fx, fy, level 0) of an RGB8 image (w x h, row-major, 3 B/pixel) at n
// points xy[2*i]; out 3 floats per point.  safe[i] = CImage::isSafe(Vec3f(x, y, 1), 0).
// getColor is only evaluated where isSafe holds (the reference never samples elsewhere:
// grabSafe, optim.cpp:783-805, guards every grabTex).
int ref_get_color(const unsigned char* rgb, int w, int h, const float* xy, int n, float* out3, int* safe) {
  RawImage R(rgb, w, h);
  const Image::CImage& im = *R.im();
  for (int i = 0; i < n; ++i) {
    const Vec3f ic(xy[2 * i], xy[2 * i + 1], 1.0f);
    safe[i] = im.isSafe(ic, 0);
    Vec3f c(0.0f, 0.0f, 0.0f);
    if (safe[i]) c = im.getColor(xy[2 * i], xy[2 * i + 1], 0);
    out3[3 * i] = c[0];
    out3[3 * i + 1] = c[1];
    out3[3 * i + 2] = c[2];
  }
  return 0;
}

// CCamera::computeDepth (camera.cpp:445-452), the depth the organizer's depth maps and
// isVisible compare (CPhotoSetS::computeDepth): out 1 float per point.
int ref_camera_depth(const char* txt, int max_level, const float* coords4, int n, float* out) {
  Image::CCamera cam;
  cam.init(txt, max_level);
  for (int i = 0; i < n; ++i) {
    const Vec4f c(coords4[4 * i], coords4[4 * i + 1], coords4[4 * i + 2], coords4[4 * i + 3]);
    out[i] = cam.computeDepth(c);
  }
  return 0;
}

// out: [0..3] center, [4..7] oaxis, [8..16] x/y/z axes, [17..28] P at `level`.
int ref_camera(const char* txt, int max_level, int level, float* out) {
  CamProbe cam;
  cam.init(txt, max_level);
  const Vec4f c = cam.OpticalCenter(), a = cam.OpticalAxis();
  for (int i = 0; i < 4; ++i) {
    out[i] = c[i];
    out[4 + i] = a[i];
  }
  cam.axes(out + 8);
  const auto P = cam.ProjectionMatrix();
  for (int y = 0; y < 3; ++y)
    for (int x = 0; x < 4; ++x) out[17 + 4 * y + x] = P[level][y][x];
  return 0;
}

int ref_project(const char* txt, int max_level, int level, const float* coords4, int n, float* out3) {
  Image::CCamera cam;
  cam.init(txt, max_level);
  for (int i = 0; i < n; ++i) {
    const Vec4f c(coords4[4 * i], coords4[4 * i + 1], coords4[4 * i + 2], coords4[4 * i + 3]);
    const Vec3f r = cam.project(c, level);
    out3[3 * i] = r[0];
    out3[3 * i + 1] = r[1];
    out3[3 * i + 2] = r[2];
  }
  return 0;
}

// SOption::init(prefix, option).  Scalars: [level, csize, wsize, minImageNum, CPU, useBound,
// useVisData, sequence, tflag, oflag] in iout[0..9]; [threshold, setEdge, maxAngle, quad] in
// fout[0..3].  timages/oimages/bindexes and visdata2 (CSR) written to the arrays given
// (capacity cap each); counts in iout[10..13] = ntimages, noimages, nbindexes, nvis.
int ref_option(const char* prefix, const char* option, int* iout, float* fout, int* timages, int* oimages,
               int* bindexes, int* vis_off, int* vis, int cap) {
  PMVS3::SOption o;
  o.init(prefix, option);
  iout[0] = o._level; iout[1] = o._csize; iout[2] = o._wsize; iout[3] = o._minImageNum; iout[4] = o._CPU;
  iout[5] = o._useBound; iout[6] = o._useVisData; iout[7] = o._sequence; iout[8] = o._tflag; iout[9] = o._oflag;
  fout[0] = o._threshold; fout[1] = o._setEdge; fout[2] = o._maxAngleThreshold; fout[3] = o._quadThreshold;
  iout[10] = (int)o._timages.size();
  iout[11] = (int)o._oimages.size();
  iout[12] = (int)o._bindexes.size();
  for (int i = 0; i < (int)o._timages.size() && i < cap; ++i) timages[i] = o._timages[i];
  for (int i = 0; i < (int)o._oimages.size() && i < cap; ++i) oimages[i] = o._oimages[i];
  for (int i = 0; i < (int)o._bindexes.size() && i < cap; ++i) bindexes[i] = o._bindexes[i];
  int k = 0;
  vis_off[0] = 0;
  for (int r = 0; r < (int)o._visdata2.size(); ++r) {
    for (int v : o._visdata2[r])
      if (k < cap) vis[k++] = v;
    vis_off[r + 1] = k;
  }
  iout[13] = k;
  return 0;
}

// CPatch serialisation exactly as CPatchOrganizerS::writePatches2 emits it
// (patchOrganizerS.cpp:98-116: setprecision(max_digits10), "PATCHES\n<n>\n", patch << "\n").
// Each patch: coord[4], normal[4], ncc, dscale, ascale (11 floats at fin[11*p]); image ids in
// ids (nimg[p] each) and vimage ids in vids (nvimg[p] each).  Returns bytes written to out.
int ref_write_patches(int n, const float* fin, const int* nimg, const int* ids, const int* nvimg,
                      const int* vids, char* out, int cap) {
  std::ostringstream ofstr;
  ofstr << std::setprecision(std::numeric_limits<double>::max_digits10);
  ofstr << "PATCHES" << std::endl << n << std::endl;
  int ki = 0, kv = 0;
  for (int p = 0; p < n; ++p) {
    Patch::CPatch patch;
    const float* f = fin + 11 * p;
    patch._coord = Vec4f(f[0], f[1], f[2], f[3]);
    patch._normal = Vec4f(f[4], f[5], f[6], f[7]);
    patch._ncc = f[8];
    patch._dscale = f[9];
    patch._ascale = f[10];
    for (int i = 0; i < nimg[p]; ++i) patch._images.push_back(ids[ki++]);
    for (int i = 0; i < nvimg[p]; ++i) patch._vimages.push_back(vids[kv++]);
    ofstr << patch << "\n";
  }
  const std::string s = ofstr.str();
  const int len = (int)s.size();
  if (len < cap) std::memcpy(out, s.data(), len + 1);
  return len;
}

// .pset lines (patchOrganizerS.cpp:118-131): default stream precision.
int ref_write_pset(int n, const float* fin, char* out, int cap) {
  std::ostringstream ofstr;
  for (int p = 0; p < n; ++p) {
    const float* f = fin + 11 * p;
    ofstr << f[0] << ' ' << f[1] << ' ' << f[2] << ' ' << f[4] << ' ' << f[5] << ' ' << f[6] << "\n";
  }
  const std::string s = ofstr.str();
  const int len = (int)s.size();
  if (len < cap) std::memcpy(out, s.data(), len + 1);
  return len;
}

// The candidate centres of CExpand::findEmptyBlocks (expand.cpp:114-115, 176-177), evaluated
// in a TU with expand.cpp's own includes so the reference's overload resolution applies:
// unqualified cos/sin on the float angle, TVec4 operator*(N, TVec4) (vec4.hpp:177) and
// operator+ (vec4.hpp:149).  expand.cpp itself cannot be linked here (it needs COptim from
// optim.cpp, i.e. nlopt); this evaluates its two lines with the reference's headers.
void ref_expand_dirs(const float* coord4, const float* normal4, const float* radius_in, int n, float* out) {
  const int dnum = 6;
  for (int q = 0; q < n; ++q) {
    const Vec4f coord(coord4[4 * q], coord4[4 * q + 1], coord4[4 * q + 2], coord4[4 * q + 3]);
    const Vec4f normal(normal4[4 * q], normal4[4 * q + 1], normal4[4 * q + 2], normal4[4 * q + 3]);
    const float radius = radius_in[q];
    Vec4f xdir, ydir;
    ortho(normal, xdir, ydir);
    for (int i = 0; i < dnum; ++i) {
      const float angle = 2 * M_PI * i / dnum;
      Vec4f canCoord = coord + cos(angle) * radius * xdir + sin(angle) * radius * ydir;
      for (int k = 0; k < 4; ++k) out[24 * q + 4 * i + k] = canCoord[k];
    }
  }
}

// The two detectors of CDetectFeatures::runThread (detectFeatures.cpp:77-108) -- the
// reference's own CHarris::run (sigma 4) and CDifferenceOfGaussians::run (scales 1, 3) from
// harris.cpp / dog.cpp / detector.cpp / point.cpp, compiled unmodified -- on one RGB8 image with
// optional mask / edge bytes, each result multiset read from its end as detectFeatures.cpp does.
// out: 4 floats per point (x, y, response, type); returns the point count (<= cap written).
int ref_detect_features(const unsigned char* rgb, const unsigned char* mask, const unsigned char* edge, int w, int h,
                        int fcsize, float* out, int cap) {
  const std::vector<unsigned char> image(rgb, rgb + (size_t)3 * w * h);
  std::vector<unsigned char> m, e;
  if (mask) m.assign(mask, mask + (size_t)w * h);
  if (edge) e.assign(edge, edge + (size_t)w * h);
  std::vector<PMVS3::CPoint> pts;
  {
    PMVS3::CHarris harris;
    std::multiset<PMVS3::CPoint> result;
    harris.run(image, m, e, w, h, fcsize, 4.0f, result);
    for (auto it = result.rbegin(); it != result.rend(); ++it) pts.push_back(*it);
  }
  {
    PMVS3::CDifferenceOfGaussians dog;
    std::multiset<PMVS3::CPoint> result;
    dog.run(image, m, e, w, h, fcsize, 1.0f, 3.0f, result);
    for (auto it = result.rbegin(); it != result.rend(); ++it) pts.push_back(*it);
  }
  for (int i = 0; i < (int)pts.size() && i < cap; ++i) {
    out[4 * i] = pts[i]._icoord[0];
    out[4 * i + 1] = pts[i]._icoord[1];
    out[4 * i + 2] = pts[i]._response;
    out[4 * i + 3] = (float)pts[i]._type;
  }
  return (int)pts.size();
}

// Header-only numeric library: ortho (vec4.hpp:303-322) used by CExpand::findEmptyBlocks.
void ref_ortho(const float* z, float* out) {
  Vec4f zz(z[0], z[1], z[2], z[3]), x, y;
  ortho(zz, x, y);
  for (int i = 0; i < 4; ++i) {
    out[i] = x[i];
    out[4 + i] = y[i];
  }
}

// Seed-phase geometry on the reference's own CCamera (camera.cpp) and header templates:
// Image::setF<double> and Image::computeEPD<double> (camera.hpp:119-151) are called as they are;
// the triangulation of CSeed::unproject (seed.cpp:340-384, a CSeed member that cannot be
// instantiated without CFindMatch) is evaluated with the reference's TMat4/TMat3/TVec types and
// operators (transpose, Mat4 * Mat4, Mat4 * Vec4, invert(Mat3), Mat3 * Vec3), so the operation
// order is the headers'.  out: F9 (row-major), epd[n], coords4[4n].
int ref_seed_geometry(const char* txt0, const char* txt1, int max_level, int level, const float* xy0, const float* xy1,
                      int n, double* F9, float* epd, float* coords4) {
  Image::CCamera c0, c1;
  c0.init(txt0, max_level);
  c1.init(txt1, max_level);
  Mat3 F;
  Image::setF(c0, c1, F, level);
  for (int i = 0; i < 9; ++i) F9[i] = F[i / 3][i % 3];
  const std::vector<Vec4f> P0 = c0.ProjectionMatrix()[level];
  const std::vector<Vec4f> P1 = c1.ProjectionMatrix()[level];
  for (int k = 0; k < n; ++k) {
    const Vec3f a(xy0[2 * k], xy0[2 * k + 1], 1.0f), b(xy1[2 * k], xy1[2 * k + 1], 1.0f);
    const Vec3 p0(a[0], a[1], a[2]), p1(b[0], b[1], b[2]);
    epd[k] = Image::computeEPD(F, p0, p1);
    Mat4 A;
    for (int j = 0; j < 3; ++j) {
      A[0][j] = P0[0][j] - a[0] * P0[2][j];
      A[1][j] = P0[1][j] - a[1] * P0[2][j];
      A[2][j] = P1[0][j] - b[0] * P1[2][j];
      A[3][j] = P1[1][j] - b[1] * P1[2][j];
    }
    Vec4 bb;
    bb[0] = a[0] * P0[2][3] - P0[0][3];
    bb[1] = a[1] * P0[2][3] - P0[1][3];
    bb[2] = b[0] * P1[2][3] - P1[0][3];
    bb[3] = b[1] * P1[2][3] - P1[1][3];
    const Mat4 AT = transpose(A);
    const Mat4 ATA = AT * A;
    const Vec4 ATb = AT * bb;
    Mat3 M3;
    Vec3 r3;
    for (int y = 0; y < 3; ++y) {
      for (int x = 0; x < 3; ++x) M3[y][x] = ATA[y][x];
      r3[y] = ATb[y];
    }
    Mat3 iM3;
    invert(iM3, M3);
    const Vec3 ans = iM3 * r3;
    for (int y = 0; y < 3; ++y) coords4[4 * k + y] = ans[y];
    coords4[4 * k + 3] = 1.0f;
  }
  return 0;
}
}
