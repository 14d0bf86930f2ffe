// pmvs_io.cpp -- host-side input/output surface of the pmvs2 pipeline (SURVEY.md §8 a19 and
// §8(b) "external boundary"): the option file (+ vis.dat, bimages.dat), camera txt files,
// binary PPM images, and the .patch / .pset / .ply writers.  Plain C++; no GPU involved except
// pmvs_patch_colors (pmvs_api.cpp), which samples the device pyramids.
//
// Each function restates the reference routine it replaces, with the same tokenisation and
// arithmetic, but reports errors through pmvs_status instead of exit(1).
#include <dlfcn.h>
#include <setjmp.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <limits>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pmvs_amd.h"

// libjpeg's API types (the image's libjpeg 9 headers); the library itself is loaded at run time
// (dlopen), so the product has no link-time JPEG dependency and reports PMVS_EUNSUPPORTED for
// .jpg inputs where libjpeg is absent.
// The Makefile finds jpeglib.h (JPEG_INC) and warns when it is missing.
#if __has_include(<jpeglib.h>)
#include <jpeglib.h>
#define PMVS_HAVE_JPEG_HEADERS 1
#endif

pmvs_status pmvs_io_fail(pmvs_status st, const char* fmt, ...);  // pmvs_api.cpp

namespace {

// ------------------------------------------------------------------ camera txt
// Image::CCamera::init (camera.cpp:13-54) + setProjection (camera.cpp:256-310) +
// setProjectionSub (camera.cpp:312-360) + q2proj (camera.cpp:407-426).  All arithmetic in
// double as the reference's Mat3/Mat4 (TMat<double>) with row-by-column products
// (mat3.hpp:262-272, mat4.hpp:364-375: A(i,j) = n[i] * m.col(j), left-to-right dot).
struct M4 { double a[4][4]; };
struct M3 { double a[3][3]; };

M4 mul4(const M4& n, const M4& m) {
  M4 r;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      r.a[i][j] = n.a[i][0] * m.a[0][j] + n.a[i][1] * m.a[1][j] + n.a[i][2] * m.a[2][j] + n.a[i][3] * m.a[3][j];
  return r;
}
M3 mul3(const M3& n, const M3& m) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.a[i][j] = n.a[i][0] * m.a[0][j] + n.a[i][1] * m.a[1][j] + n.a[i][2] * m.a[2][j];
  return r;
}
M3 tr3(const M3& m) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.a[i][j] = m.a[j][i];
  return r;
}

void q2proj(const double q[6], M4& mat) {
  const double a = q[0] * M_PI / 180.0;
  const double b = q[1] * M_PI / 180.0;
  const double g = q[2] * M_PI / 180.0;
  const double s1 = sin(a), s2 = sin(b), s3 = sin(g);
  const double c1 = cos(a), c2 = cos(b), c3 = cos(g);
  mat.a[0][0] = c2 * c3; mat.a[0][1] = c3 * s2 * s1 - s3 * c1;
  mat.a[1][0] = s3 * c2; mat.a[1][1] = s3 * s2 * s1 + c3 * c1;
  mat.a[2][0] = -s2;     mat.a[2][1] = c2 * s1;
  mat.a[0][2] = c3 * s2 * c1 + s3 * s1; mat.a[0][3] = q[3];
  mat.a[1][2] = s3 * s2 * c1 - c3 * s1; mat.a[1][3] = q[4];
  mat.a[2][2] = c2 * c1;                mat.a[2][3] = q[5];
  mat.a[3][0] = mat.a[3][1] = mat.a[3][2] = 0.0;
  mat.a[3][3] = 1.0;
}

void projection_sub(const double p[9], float out[12]) {
  const double rx = p[6] * M_PI / 180.0, ry = p[7] * M_PI / 180.0, rz = p[8] * M_PI / 180.0;
  const double fovx = p[0] * M_PI / 180.0;
  const double f = p[1] / 2.0 / tan(fovx / 2.0);
  M3 K = {{{f, 0.0, 0.0}, {0.0, f, 0.0}, {0.0, 0.0, -1.0}}};
  const M3 trans = {{{1.0, 0.0, p[1] / 2.0}, {0.0, -1.0, p[2] / 2.0}, {0.0, 0.0, 1.0}}};
  K = mul3(trans, K);
  const M3 Rx = {{{1.0, 0.0, 0.0}, {(double)0.0f, cos(rx), -sin(rx)}, {0.0, sin(rx), cos(rx)}}};
  const M3 Ry = {{{cos(ry), 0, sin(ry)}, {0.0, 1.0, 0.0}, {-sin(ry), 0, cos(ry)}}};
  const M3 Rz = {{{cos(rz), -sin(rz), 0.0}, {sin(rz), cos(rz), 0.0}, {0.0, 0.0, 1.0}}};
  const M3 R = mul3(mul3(tr3(Rx), tr3(Ry)), tr3(Rz));
  const double t[3] = {p[3], p[4], p[5]};
  const M3 left = mul3(K, R);
  double Rt[3], right[3];
  for (int i = 0; i < 3; ++i) Rt[i] = R.a[i][0] * t[0] + R.a[i][1] * t[1] + R.a[i][2] * t[2];
  for (int i = 0; i < 3; ++i)  // -K * (R*t): (-K) row . (R*t)
    right[i] = (-K.a[i][0]) * Rt[0] + (-K.a[i][1]) * Rt[1] + (-K.a[i][2]) * Rt[2];
  for (int y = 0; y < 3; ++y) {
    for (int x = 0; x < 3; ++x) out[4 * y + x] = (float)left.a[y][x];
    out[4 * y + 3] = (float)right[y];
  }
  // projection[0..1] /= (0x0001 << 0): Vec4f /= int at level 0
  for (int x = 0; x < 4; ++x) {
    out[x] /= (float)1;
    out[4 + x] /= (float)1;
  }
}

}  // namespace

// ==================================================================== C-ABI
extern "C" {

pmvs_status pmvs_camera_load(const char* txt_path, float projection[12]) {
  if (!txt_path || !projection) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  std::ifstream ifstr(txt_path);
  if (!ifstr.is_open()) return pmvs_io_fail(PMVS_EINVAL, "cannot open camera file %s", txt_path);
  std::string header;
  ifstr >> header;
  int type;
  if (header == "CONTOUR") type = 0;
  else if (header == "CONTOUR2") type = 2;
  else if (header == "CONTOUR3") type = 3;
  else return pmvs_io_fail(PMVS_EINVAL, "Unrecognizable txt format: %s", txt_path);
  float intr[6], extr[6];
  for (int i = 0; i < 6; ++i) ifstr >> intr[i];
  for (int i = 0; i < 6; ++i) ifstr >> extr[i];
  if (ifstr.fail()) return pmvs_io_fail(PMVS_EINVAL, "truncated camera file %s", txt_path);
  double params[12];
  for (int i = 0; i < 6; ++i) {
    params[i] = intr[i];
    params[6 + i] = extr[i];
  }
  if (type == 0) {
    for (int k = 0; k < 12; ++k) projection[k] = (float)params[k];
  } else if (type == 2) {
    M4 K;
    std::memset(&K, 0, sizeof(K));
    K.a[0][0] = params[0]; K.a[1][1] = params[1];
    K.a[0][1] = params[2]; K.a[0][2] = params[3];
    K.a[1][2] = params[4]; K.a[2][2] = 1.0;
    K.a[3][3] = 1.0;
    M4 m;
    q2proj(&params[6], m);
    m = mul4(K, m);
    for (int y = 0; y < 3; ++y)
      for (int x = 0; x < 4; ++x) projection[4 * y + x] = (float)m.a[y][x];
  } else {
    const double p2[9] = {params[0], params[1], params[2], params[6], params[7],
                          params[8], params[9], params[10], params[11]};
    projection_sub(p2, projection);
  }
  return PMVS_OK;
}

// Binary PPM (P6, maxval 255) -- the PNM branch of CImage::readAnyImage (image.cpp:473-506,
// which delegates to CImg's load_pnm); pixel bytes are passed through unchanged.
pmvs_status pmvs_ppm_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgb) {
  if (!path || !width || !height) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return pmvs_io_fail(PMVS_EINVAL, "cannot open image %s", path);
  auto token = [&](long* v) -> bool {
    int c = std::fgetc(f);
    while (c != EOF) {
      if (c == '#') {
        while (c != EOF && c != '\n') c = std::fgetc(f);
      } else if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
        c = std::fgetc(f);
      } else {
        break;
      }
    }
    if (c == EOF || c < '0' || c > '9') return false;
    long x = 0;
    while (c >= '0' && c <= '9') {
      x = 10 * x + (c - '0');
      c = std::fgetc(f);
    }
    *v = x;  // the single whitespace after maxval has been consumed
    return true;
  };
  char magic[3] = {0, 0, 0};
  long w = 0, h = 0, maxval = 0;
  const bool ok = std::fread(magic, 1, 2, f) == 2 && magic[0] == 'P' && magic[1] == '6' && token(&w) &&
                  token(&h) && token(&maxval);
  if (!ok || w <= 0 || h <= 0 || maxval != 255) {
    std::fclose(f);
    return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: only binary 8-bit PPM (P6, maxval 255) is supported", path);
  }
  *width = (int32_t)w;
  *height = (int32_t)h;
  if (rgb) {
    const size_t n = (size_t)w * h * 3;
    if (std::fread(rgb, 1, n, f) != n) {
      std::fclose(f);
      return pmvs_io_fail(PMVS_EINVAL, "%s: truncated pixel data", path);
    }
  }
  std::fclose(f);
  return PMVS_OK;
}

// ------------------------------------------------------------------ JPEG (dlopen'ed libjpeg)
#ifdef PMVS_HAVE_JPEG_HEADERS
namespace {
struct JpegApi {
  void* h = nullptr;
  struct jpeg_error_mgr* (*std_error)(struct jpeg_error_mgr*);
  void (*create)(j_decompress_ptr, int, size_t);
  void (*stdio_src)(j_decompress_ptr, FILE*);
  int (*read_header)(j_decompress_ptr, boolean);
  boolean (*start)(j_decompress_ptr);
  JDIMENSION (*read_scanlines)(j_decompress_ptr, JSAMPARRAY, JDIMENSION);
  boolean (*finish)(j_decompress_ptr);
  void (*destroy)(j_decompress_ptr);
  std::once_flag once;
  bool ok = false;
  bool load() {  // thread-safe: pmvs2 decodes views on a pool of host threads
    std::call_once(once, [this]() { ok = open(); });
    return ok;
  }
  bool open() {
    for (const char* name : {"libjpeg.so.9", "/opt/conda/lib/libjpeg.so.9", "libjpeg.so"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
    std_error = (decltype(std_error))dlsym(h, "jpeg_std_error");
    create = (decltype(create))dlsym(h, "jpeg_CreateDecompress");
    stdio_src = (decltype(stdio_src))dlsym(h, "jpeg_stdio_src");
    read_header = (decltype(read_header))dlsym(h, "jpeg_read_header");
    start = (decltype(start))dlsym(h, "jpeg_start_decompress");
    read_scanlines = (decltype(read_scanlines))dlsym(h, "jpeg_read_scanlines");
    finish = (decltype(finish))dlsym(h, "jpeg_finish_decompress");
    destroy = (decltype(destroy))dlsym(h, "jpeg_destroy_decompress");
    return std_error && create && stdio_src && read_header && start && read_scanlines && finish && destroy;
  }
};
JpegApi g_jpeg;
struct JpegErr {
  struct jpeg_error_mgr pub;
  jmp_buf jb;
};
void jpeg_err_exit(j_common_ptr c) { longjmp(reinterpret_cast<JpegErr*>(c->err)->jb, 1); }

// CImg::load_jpeg (cimg_use_jpeg) as CImage::readAnyImage uses it (image.cpp:473-506): libjpeg
// defaults (islow IDCT, fancy upsampling), 3-component output copied in (x, y, c) order.
pmvs_status jpeg_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgb) {
  if (!g_jpeg.load()) return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: libjpeg (libjpeg.so.9) is not available", path);
  FILE* f = std::fopen(path, "rb");
  if (!f) return pmvs_io_fail(PMVS_EINVAL, "cannot open image %s", path);
  struct jpeg_decompress_struct ci;
  JpegErr err;
  ci.err = g_jpeg.std_error(&err.pub);
  err.pub.error_exit = jpeg_err_exit;
  std::vector<uint8_t> row;
  if (setjmp(err.jb)) {
    g_jpeg.destroy(&ci);
    std::fclose(f);
    return pmvs_io_fail(PMVS_EINVAL, "%s: corrupt JPEG", path);
  }
  g_jpeg.create(&ci, JPEG_LIB_VERSION, sizeof(ci));
  g_jpeg.stdio_src(&ci, f);
  g_jpeg.read_header(&ci, TRUE);
  g_jpeg.start(&ci);
  const int nc = ci.output_components;
  if (nc < 3) {
    g_jpeg.destroy(&ci);
    std::fclose(f);
    // the reference prints "Unsufficient components (not a color image)" and leaves the image empty
    return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: %d components (not a color image)", path, nc);
  }
  *width = (int32_t)ci.output_width;
  *height = (int32_t)ci.output_height;
  if (rgb) {
    row.resize((size_t)ci.output_width * nc);
    JSAMPROW rp = row.data();
    for (uint32_t y = 0; y < ci.output_height; ++y) {
      g_jpeg.read_scanlines(&ci, &rp, 1);
      uint8_t* o = rgb + (size_t)y * ci.output_width * 3;
      for (uint32_t x = 0; x < ci.output_width; ++x)
        for (int c = 0; c < 3; ++c) o[3 * x + c] = row[(size_t)x * nc + c];
    }
    g_jpeg.finish(&ci);
  }
  g_jpeg.destroy(&ci);
  std::fclose(f);
  return PMVS_OK;
}
}  // namespace
#endif

static bool has_suffix(const std::string& s, const char* suf) {
  const size_t n = std::strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// CImage::readAnyImage (image.cpp:473-506): the colour image of a view, by extension (.ppm / .jpg).
pmvs_status pmvs_image_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgb) {
  if (!path || !width || !height) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  const std::string p(path);
  if (has_suffix(p, ".ppm")) return pmvs_ppm_load(path, width, height, rgb);
  if (has_suffix(p, ".jpg") || has_suffix(p, ".jpeg") || has_suffix(p, ".JPG")) {
#ifdef PMVS_HAVE_JPEG_HEADERS
    return jpeg_load(path, width, height, rgb);
#else
    return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: built without JPEG support", path);
#endif
  }
  return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: unsupported image format (ppm, jpg)", path);
}

// CImage::readPGMImage (image.cpp:622-670, binary P5) / readPBMImage (image.cpp:508-560, P4: bit 1
// -> 0, bit 0 -> 255), as the mask and edge readers of CImage::alloc (image.cpp:143-180).  The
// raw bytes are returned; the 127 / 1 thresholds are applied by pmvs_scene_create.
pmvs_status pmvs_pnm_mask_load(const char* path, int32_t* width, int32_t* height, uint8_t* out) {
  if (!path || !width || !height) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  const std::string p(path);
  const bool pgm = has_suffix(p, "pgm"), pbm = has_suffix(p, "pbm");
  if (!pgm && !pbm) return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: masks/edges are .pgm or .pbm", path);
  std::ifstream ifstr(path, std::ios::binary);
  if (!ifstr.is_open()) return pmvs_io_fail(PMVS_EINVAL, "cannot open %s", path);
  std::string header;
  unsigned char uc;
  ifstr >> header;
  ifstr.read((char*)&uc, 1);
  if (header != (pgm ? "P5" : "P4")) return pmvs_io_fail(PMVS_EUNSUPPORTED, "%s: only binary %s", path, pgm ? "pgm" : "pbm");
  while (true) {
    ifstr.read((char*)&uc, 1);
    ifstr.putback(uc);
    if (uc == '#') {
      char buffer[1024];
      ifstr.getline(buffer, 1024);
    } else {
      break;
    }
  }
  int w = 0, h = 0, maxv = 0;
  ifstr >> w >> h;
  if (pgm) ifstr >> maxv;
  ifstr.read((char*)&uc, 1);
  if (!ifstr || w <= 0 || h <= 0) return pmvs_io_fail(PMVS_EINVAL, "%s: bad header", path);
  *width = w;
  *height = h;
  if (!out) return PMVS_OK;
  const size_t n = (size_t)w * h;
  if (pgm) {
    ifstr.read((char*)out, (std::streamsize)n);
    if ((size_t)ifstr.gcount() != n) return pmvs_io_fail(PMVS_EINVAL, "%s: truncated", path);
  } else {
    // bit stream over the whole image (no per-row padding), as the reference reads it
    size_t bcount = n;
    if (bcount % 8 != 0) bcount++;
    size_t count = 0;
    for (size_t i = 0; i < bcount && count < n; ++i) {
      ifstr.read((char*)&uc, 1);
      if (!ifstr) return pmvs_io_fail(PMVS_EINVAL, "%s: truncated", path);
      for (int j = 0; j < 8 && count < n; ++j, ++count) {
        out[count] = (uc >> 7) ? 0 : 255;
        uc <<= 1;
      }
    }
  }
  return PMVS_OK;
}

// CImage::setEdge (image.cpp:407-460, option setEdge != 0): squared RGB central differences,
// separable Gaussian filterG (sigma 3, image.cpp:1013-1056, border renormalised), threshold.
pmvs_status pmvs_set_edge(const uint8_t* rgb, int32_t width, int32_t height, float threshold, uint8_t* edge_out) {
  if (!rgb || !edge_out || width < 1 || height < 1) return pmvs_io_fail(PMVS_EINVAL, "invalid argument");
  const int W = width, H = height;
  std::vector<float> a((size_t)W * H, 0.0f), b((size_t)W * H, 0.0f);
  for (int y = 1; y < H - 1; ++y)
    for (int x = 1; x < W - 1; ++x) {
      const int index = 3 * (y * W + x);
      const int r = index + 3, l = index - 3, t = index - 3 * W, bo = index + 3 * W;
      float& v = a[(size_t)y * W + x];
      for (int i = 0; i < 3; ++i) {
        const int i0 = std::abs(rgb[r + i] - rgb[l + i]);
        v += i0 * i0;
        const int i1 = std::abs(rgb[bo + i] - rgb[t + i]);
        v += i1 * i1;
      }
    }
  const float sigma = 3.f;
  const float sigma2 = 2.f * sigma * sigma;
  const int margin = (int)std::floor(2 * sigma);
  std::vector<float> filter(2 * margin + 1);
  for (int i = -margin; i <= margin; ++i) filter[i + margin] = (float)std::exp((double)(-i * i / sigma2));
  // vertical into b, horizontal back into a
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      float acc = 0.0f, denom = 0.0f;
      for (int j = -margin; j <= margin; ++j) {
        const int yt = y + j;
        if (yt < 0 || H <= yt) continue;
        acc += filter[j + margin] * a[(size_t)yt * W + x];
        denom += filter[j + margin];
      }
      b[(size_t)y * W + x] = acc / denom;
    }
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      float acc = 0.0f, denom = 0.0f;
      for (int i = -margin; i <= margin; ++i) {
        const int xt = x + i;
        if (xt < 0 || W <= xt) continue;
        acc += filter[i + margin] * b[(size_t)y * W + xt];
        denom += filter[i + margin];
      }
      a[(size_t)y * W + x] = acc / denom;
    }
  const float nt = threshold * threshold * (2 * margin + 1) * (2 * margin + 1) / 3.0f;
  for (size_t k = 0; k < (size_t)W * H; ++k) edge_out[k] = (nt < a[k]) ? 255 : 0;
  return PMVS_OK;
}

// ------------------------------------------------------------------ options
struct pmvs_options_store {
  pmvs_options pub;
  std::vector<int> timages, oimages, bindexes, vis_off, vis;
};

static void read_vis(std::ifstream& ifstr, int& num2, std::vector<std::vector<int>>& rows) {
  std::string header;
  ifstr >> header >> num2;
  rows.assign(num2 > 0 ? num2 : 0, {});
  for (int c = 0; c < num2; ++c) {
    int itmp;
    ifstr >> itmp >> itmp;
    for (int i = 0; i < itmp; ++i) {
      int v;
      ifstr >> v;
      rows[c].push_back(v);
    }
  }
}

// PMVS3::SOption::SOption + SOption::init (option.cpp:10-160) with initOimages (:162-198),
// initVisdata (:201-221), initVisdata2 (:224-283) and initBindexes (:285-307).
pmvs_status pmvs_options_load(const char* prefix, const char* option_file, pmvs_options** out) {
  if (!prefix || !option_file || !out) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  *out = nullptr;
  auto* st = new pmvs_options_store();
  pmvs_options& o = st->pub;
  o.level = 1; o.csize = 2; o.threshold = 0.7f; o.wsize = 7; o.min_image_num = 3; o.cpu = 4;
  o.set_edge = 0.0f; o.use_bound = 0; o.use_vis_data = 0; o.sequence = -1; o.tflag = -10; o.oflag = -10;
  o.max_angle = (float)(10.0f * M_PI / 180.0f);
  o.quad = 2.5f;
  auto bail = [&](pmvs_status s) { delete st; return s; };
  const std::string pre(prefix);
  std::ifstream ifstr((pre + option_file).c_str());
  if (!ifstr.is_open()) return bail(pmvs_io_fail(PMVS_EINVAL, "cannot open option file %s%s", prefix, option_file));
  while (true) {
    std::string name;
    ifstr >> name;
    if (ifstr.eof()) break;
    if (name[0] == '#') {
      char buffer[1024];
      ifstr.putback('#');
      ifstr.getline(buffer, 1024);
      continue;
    }
    if (name == "level") ifstr >> o.level;
    else if (name == "csize") ifstr >> o.csize;
    else if (name == "threshold") ifstr >> o.threshold;
    else if (name == "wsize") ifstr >> o.wsize;
    else if (name == "minImageNum") ifstr >> o.min_image_num;
    else if (name == "CPU") ifstr >> o.cpu;
    else if (name == "setEdge") ifstr >> o.set_edge;
    else if (name == "useBound") ifstr >> o.use_bound;
    else if (name == "useVisData") ifstr >> o.use_vis_data;
    else if (name == "sequence") ifstr >> o.sequence;
    else if (name == "timages") {
      ifstr >> o.tflag;
      if (o.tflag == -1) {
        int a, b;
        ifstr >> a >> b;
        for (int i = a; i < b; ++i) st->timages.push_back(i);
      } else if (0 < o.tflag) {
        for (int i = 0; i < o.tflag; ++i) {
          int v;
          ifstr >> v;
          st->timages.push_back(v);
        }
      } else {
        return bail(pmvs_io_fail(PMVS_EINVAL, "tflag is not valid: %d", o.tflag));
      }
    } else if (name == "oimages") {
      ifstr >> o.oflag;
      if (o.oflag == -1) {
        int a, b;
        ifstr >> a >> b;
        for (int i = a; i < b; ++i) st->oimages.push_back(i);
      } else if (0 <= o.oflag) {
        for (int i = 0; i < o.oflag; ++i) {
          int v;
          ifstr >> v;
          st->oimages.push_back(v);
        }
      } else if (o.oflag != -2 && o.oflag != -3) {
        return bail(pmvs_io_fail(PMVS_EINVAL, "oflag is not valid: %d", o.oflag));
      }
    } else if (name == "quad") ifstr >> o.quad;
    else if (name == "maxAngle") {
      ifstr >> o.max_angle;
      o.max_angle *= M_PI / 180.0f;
    } else {
      return bail(pmvs_io_fail(PMVS_EINVAL, "Unrecognizable option: %s", name.c_str()));
    }
  }
  if (o.tflag == -10 || o.oflag == -10)
    return bail(pmvs_io_fail(PMVS_EINVAL, "_tflag and _oflag not specified: %d %d", o.tflag, o.oflag));

  std::map<int, int> dict;
  for (int i = 0; i < (int)st->timages.size(); ++i) dict[st->timages[i]] = i;

  // initOimages: oimages from vis.dat rows of target images
  if (o.oflag == -2) {
    std::ifstream v((pre + "vis.dat").c_str());
    if (!v.is_open()) return bail(pmvs_io_fail(PMVS_EINVAL, "No vis.dat although specified to initOimages: %svis.dat", prefix));
    int num2 = 0;
    std::vector<std::vector<int>> rows;
    read_vis(v, num2, rows);
    st->oimages.clear();
    for (int c = 0; c < num2; ++c) {
      if (dict.find(c) == dict.end()) continue;
      for (int x : rows[c])
        if (dict.find(x) == dict.end()) st->oimages.push_back(x);
    }
    std::sort(st->oimages.begin(), st->oimages.end());
    st->oimages.erase(std::unique(st->oimages.begin(), st->oimages.end()), st->oimages.end());
  }

  // initVisdata / initVisdata2: visdata2 rows over the view list (timages then oimages)
  const int tnum = (int)st->timages.size(), onum = (int)st->oimages.size(), num = tnum + onum;
  std::vector<std::vector<int>> vis2(num);
  if (o.use_vis_data == 0) {
    for (int y = 0; y < num; ++y)
      for (int x = 0; x < num; ++x)
        if (x != y) vis2[y].push_back(x);
  } else {
    std::vector<int> images(st->timages);
    images.insert(images.end(), st->oimages.begin(), st->oimages.end());
    std::map<int, int> dict2;
    for (int i = 0; i < (int)images.size(); ++i) dict2[images[i]] = i;
    std::ifstream v((pre + "vis.dat").c_str());
    if (!v.is_open()) return bail(pmvs_io_fail(PMVS_EINVAL, "No vis.dat although specified to initVisdata2: %svis.dat", prefix));
    int num2 = 0;
    std::vector<std::vector<int>> rows;
    read_vis(v, num2, rows);
    for (int c = 0; c < num2; ++c) {
      auto i0 = dict2.find(c);
      if (i0 == dict2.end()) continue;
      for (int x : rows[c]) {
        auto i1 = dict2.find(x);
        if (i1 != dict2.end()) vis2[i0->second].push_back(i1->second);
      }
    }
  }
  st->vis_off.push_back(0);
  for (const auto& r : vis2) {
    st->vis.insert(st->vis.end(), r.begin(), r.end());
    st->vis_off.push_back((int)st->vis.size());
  }

  if (o.use_bound) {
    std::ifstream b((pre + "bimages.dat").c_str());
    if (!b.is_open()) return bail(pmvs_io_fail(PMVS_EINVAL, "File not found: %sbimages.dat", prefix));
    int cnt;
    b >> cnt;
    for (int i = 0; i < cnt; ++i) {
      int v;
      b >> v;
      auto it = dict.find(v);
      if (it != dict.end()) st->bindexes.push_back(it->second);
    }
  }
  o.num_timages = tnum;
  o.num_oimages = onum;
  o.num_bindexes = (int)st->bindexes.size();
  o.timages = st->timages.data();
  o.oimages = st->oimages.data();
  o.bindexes = st->bindexes.data();
  o.visdata2_offsets = st->vis_off.data();
  o.visdata2 = st->vis.data();
  *out = &st->pub;
  return PMVS_OK;
}

void pmvs_options_free(pmvs_options* o) {
  if (o) delete reinterpret_cast<pmvs_options_store*>(o);  // pub is the first member
}

// ------------------------------------------------------------------ writers
// CPatchOrganizerS::writePatches2 .patch branch (patchOrganizerS.cpp:98-116) with
// Patch::operator<< (patch.cpp:31-48): precision max_digits10, "PATCHS", coord, normal,
// "ncc dscale ascale", image ids, vimage ids.
pmvs_status pmvs_write_patches(const char* path, int32_t n, const float* fields, const int32_t* nimg,
                               const int32_t* ids, const int32_t* nvimg, const int32_t* vids) {
  if (!path || n < 0 || (n > 0 && (!fields || !nimg || !nvimg))) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  std::ofstream ofstr(path);
  if (!ofstr.is_open()) return pmvs_io_fail(PMVS_EINVAL, "cannot write %s", path);
  ofstr << std::setprecision(std::numeric_limits<double>::max_digits10);
  ofstr << "PATCHES" << std::endl << n << std::endl;
  size_t ki = 0, kv = 0;
  for (int p = 0; p < n; ++p) {
    const float* f = fields + 11 * (size_t)p;
    ofstr << "PATCHS" << std::endl
          << f[0] << " " << f[1] << " " << f[2] << " " << f[3] << std::endl
          << f[4] << " " << f[5] << " " << f[6] << " " << f[7] << std::endl
          << f[8] << ' ' << f[9] << ' ' << f[10] << std::endl
          << nimg[p] << std::endl;
    for (int i = 0; i < nimg[p]; ++i) ofstr << ids[ki++] << ' ';
    ofstr << std::endl;
    ofstr << nvimg[p] << std::endl;
    for (int i = 0; i < nvimg[p]; ++i) ofstr << vids[kv++] << ' ';
    ofstr << std::endl;
    ofstr << "\n";
  }
  return ofstr.good() ? PMVS_OK : pmvs_io_fail(PMVS_EINVAL, "write failed: %s", path);
}

// .pset branch (patchOrganizerS.cpp:118-131): default stream precision.
pmvs_status pmvs_write_pset(const char* path, int32_t n, const float* fields) {
  if (!path || n < 0 || (n > 0 && !fields)) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  std::ofstream ofstr(path);
  if (!ofstr.is_open()) return pmvs_io_fail(PMVS_EINVAL, "cannot write %s", path);
  for (int p = 0; p < n; ++p) {
    const float* f = fields + 11 * (size_t)p;
    ofstr << f[0] << ' ' << f[1] << ' ' << f[2] << ' ' << f[4] << ' ' << f[5] << ' ' << f[6] << "\n";
  }
  return ofstr.good() ? PMVS_OK : pmvs_io_fail(PMVS_EINVAL, "write failed: %s", path);
}

// CPatchOrganizerS::writePLY (patchOrganizerS.cpp:687-776), colour mode 0; colours come from
// pmvs_patch_colors.
pmvs_status pmvs_write_ply(const char* path, int32_t n, const float* fields, const int32_t* colors) {
  if (!path || n < 0 || (n > 0 && (!fields || !colors))) return pmvs_io_fail(PMVS_EINVAL, "null argument");
  std::ofstream ofstr(path);
  if (!ofstr.is_open()) return pmvs_io_fail(PMVS_EINVAL, "cannot write %s", path);
  ofstr << std::setprecision(std::numeric_limits<double>::max_digits10);
  ofstr << "ply" << '\n' << "format ascii 1.0" << '\n' << "element vertex " << n << '\n'
        << "property float x" << '\n' << "property float y" << '\n' << "property float z" << '\n'
        << "property float nx" << '\n' << "property float ny" << '\n' << "property float nz" << '\n'
        << "property uchar diffuse_red" << '\n' << "property uchar diffuse_green" << '\n'
        << "property uchar diffuse_blue" << '\n' << "property float quality" << '\n' << "end_header" << '\n';
  for (int p = 0; p < n; ++p) {
    const float* f = fields + 11 * (size_t)p;
    const int32_t* c = colors + 3 * (size_t)p;
    ofstr << f[0] << ' ' << f[1] << ' ' << f[2] << ' ' << f[4] << ' ' << f[5] << ' ' << f[6] << ' ' << c[0] << ' '
          << c[1] << ' ' << c[2] << ' ' << f[8] << '\n';
  }
  return ofstr.good() ? PMVS_OK : pmvs_io_fail(PMVS_EINVAL, "write failed: %s", path);
}

}  // extern "C"
