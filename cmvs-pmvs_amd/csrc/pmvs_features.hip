// pmvs_features.hip -- feature detection on the device: PMVS3::CDetectFeatures::run
// (detectFeatures.cpp:47-124) = CHarris::run (harris.cpp) then CDifferenceOfGaussians::run
// (dog.cpp) on one view's pyramid level, with its mask / edge images.
//
// Layout: the level's RGBA8 pyramid slab (DScene::pyr) is expanded to float4 (r, g, b, 0) maps
// (CDetector::_image, Vec3f per pixel) in a per-scene scratch arena; every separable convolution
// is one pass over a float4 or float map (CDetector::convolveX / convolveY with the mask and the
// clamped border, detector.hpp:23-94).  The block selection (at most 4 points per
// 2*fcsize-pixel block, a std::multiset per block) is sequential per block in the reference's
// scan order, one thread per block.  The final per-detector ordering (the result multiset read
// from its largest element, detectFeatures.cpp:84-88,103-107) is done by the host.
//
// Numerics follow the reference's float / double operations: f32 sums in tap order,
// -ffp-contract=off, the response D - 0.06*tr*tr evaluated in double (harris.cpp:176), IEEE
// sqrt for norm() (dog.cpp setRes), filter weights computed on the host exactly as
// CDetector::setGaussI (detector.cpp:29-49).  Zero signs of masked pixels may differ from the
// reference's `buffer *= 0.0` (which keeps the sign of the buffer's previous contents); no
// comparison or selected response depends on the sign of a zero.
#include <hip/hip_runtime.h>

#include "pmvs_features.h"

namespace pmvsdev {

namespace {

constexpr int kBlock = 256;

__global__ void feat_load_kernel(const uint32_t* __restrict__ pyr, const uint8_t* __restrict__ mask,
                                 const uint8_t* __restrict__ edge, int npix, float4* __restrict__ img,
                                 uint8_t* __restrict__ m) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint32_t v = pyr[i];
  // CHarris::init / CDifferenceOfGaussians::init: ((int)image[k]) / 255.0f
  img[i] = make_float4((float)(int)(v & 0xffu) / 255.0f, (float)(int)((v >> 8) & 0xffu) / 255.0f,
                       (float)(int)((v >> 16) & 0xffu) / 255.0f, 0.0f);
  if (m) {
    uint8_t b;
    if (!mask) b = edge[i];
    else if (!edge) b = mask[i];
    else b = (mask[i] && edge[i]) ? (uint8_t)255 : (uint8_t)0;
    m[i] = b;
  }
}

__device__ __forceinline__ float4 fma4(float w, float4 v, float4 acc) {  // acc += w * v, per component
  acc.x = acc.x + w * v.x;
  acc.y = acc.y + w * v.y;
  acc.z = acc.z + w * v.z;
  return acc;
}
__device__ __forceinline__ float fma1(float w, float v, float acc) { return acc + w * v; }

// convolveX / convolveY with a mask (detector.hpp:23-94): output 0 where the mask is 0, taps at
// masked pixels skipped, the tap position clamped to the image.
template <typename T, bool Y>
__global__ void conv_kernel(const T* __restrict__ in, T* __restrict__ out, const uint8_t* __restrict__ m, int W, int H,
                            FeatFilter f) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= W) return;
  const int margin = f.n / 2;
  T acc;
  if constexpr (sizeof(T) == sizeof(float4)) acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  else acc = 0.0f;
  const size_t row = (size_t)y * W;
  if (!m || m[row + x] != 0) {
    for (int j = 0; j < f.n; ++j) {
      int xt = x, yt = y;
      if (Y) {
        yt = y + j - margin;
        yt = yt < 0 ? 0 : (H <= yt ? H - 1 : yt);
      } else {
        xt = x + j - margin;
        xt = xt < 0 ? 0 : (W <= xt ? W - 1 : xt);
      }
      const size_t k = (size_t)yt * W + xt;
      if (m && m[k] == 0) continue;
      if constexpr (sizeof(T) == sizeof(float4)) acc = fma4(f.w[j], in[k], acc);
      else acc = fma1(f.w[j], in[k], acc);
    }
  }
  out[row + x] = acc;
}

// CHarris::preprocess2 products (harris.cpp:75-86): Vec3f dot products, 0 where masked.
__global__ void harris_products_kernel(const float4* __restrict__ dx, const float4* __restrict__ dy,
                                       const uint8_t* __restrict__ m, int npix, float* __restrict__ xx,
                                       float* __restrict__ yy, float* __restrict__ xy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  float a = 0.0f, b = 0.0f, c = 0.0f;
  if (!m || m[i] != 0) {
    const float4 u = dx[i], v = dy[i];
    a = u.x * u.x + u.y * u.y + u.z * u.z;
    b = v.x * v.x + v.y * v.y + v.z * v.z;
    c = u.x * v.x + u.y * v.y + u.z * v.z;
  }
  xx[i] = a;
  yy[i] = b;
  xy[i] = c;
}

// CHarris::setResponse (harris.cpp:166-198): response, then suppression of pixels smaller than a
// 4-neighbour (interior only).
__global__ void harris_response_kernel(const float* __restrict__ xx, const float* __restrict__ yy,
                                       const float* __restrict__ xy, const uint8_t* __restrict__ m, int npix,
                                       float* __restrict__ r) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  float v = 0.0f;
  if (!m || m[i] != 0) {
    const float D = xx[i] * yy[i] - xy[i] * xy[i];
    const float tr = xx[i] + yy[i];
    v = (float)((double)D - 0.06 * (double)tr * (double)tr);
  }
  r[i] = v;
}

__global__ void harris_nms_kernel(const float* __restrict__ r, float* __restrict__ out, int W, int H) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= W) return;
  const size_t i = (size_t)y * W + x;
  const float v = r[i];
  float o = v;
  if (1 <= y && y < H - 1 && 1 <= x && x < W - 1)
    if (v < r[i + 1] || v < r[i - 1] || v < r[i + W] || v < r[i - W]) o = 0.0f;
  out[i] = o;
}

// CDifferenceOfGaussians::setRes (dog.cpp:214-235): norm() of the blurred Vec3f image.
__global__ void dog_norm_kernel(const float4* __restrict__ in, int npix, float* __restrict__ res) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const float4 v = in[i];
  res[i] = __builtin_sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
}

// A std::multiset<CPoint> of at most 4 (+1 transient) points ordered by _response; equal
// responses keep insertion order (insert places an element after its equals; erase(begin())
// removes the earliest of the smallest).
struct SmallSet {
  float r[5];
  int x[5], y[5];
  int n;
  __device__ void insert(float v, int px, int py) {
    int pos = n;
    while (pos > 0 && v < r[pos - 1]) {  // upper_bound: after every element <= v
      r[pos] = r[pos - 1];
      x[pos] = x[pos - 1];
      y[pos] = y[pos - 1];
      --pos;
    }
    r[pos] = v;
    x[pos] = px;
    y[pos] = py;
    ++n;
  }
  __device__ void erase_first() {
    for (int k = 1; k < n; ++k) {
      r[k - 1] = r[k];
      x[k - 1] = x[k];
      y[k - 1] = y[k];
    }
    --n;
  }
};

__device__ __forceinline__ void write_block(const SmallSet& s, int b, FeatPoint* __restrict__ out, int* __restrict__ cnt) {
  for (int k = 0; k < s.n; ++k) out[4 * b + k] = FeatPoint{(float)s.x[k], (float)s.y[k], s.r[k], 0};
  cnt[b] = s.n;
}

// CHarris::run selection (harris.cpp:225-249): pixels in [margin, W-margin) x [margin, H-margin)
// in raster order; a block keeps its 4 largest (insert when not full or larger than the smallest).
__global__ void harris_select_kernel(const float* __restrict__ r, int W, int H, int margin, int gsize, int bw, int bh,
                                     FeatPoint* __restrict__ out, int* __restrict__ cnt) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= bw * bh) return;
  const int bx = b % bw, by = b / bw;
  SmallSet s;
  s.n = 0;
  const int y0 = max(by * gsize, margin), y1 = min(by * gsize + gsize, H - margin);
  const int x0 = max(bx * gsize, margin), x1 = min(bx * gsize + gsize, W - margin);
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x) {
      const float v = r[(size_t)y * W + x];
      if (v == 0.0f) continue;
      if (s.n < 4 || s.r[0] < v) {
        s.insert(v, x, y);
        if (4 < s.n) s.erase_first();
      }
    }
  write_block(s, b, out, cnt);
}

__device__ __forceinline__ float dogv(const float* a, const float* b, size_t i) { return b[i] - a[i]; }  // setDOG

// CDifferenceOfGaussians::isLocalMax (dog.cpp:25-76) on the three DoG layers p = r1 - r0,
// c = r2 - r1, n = r3 - r2; flag[i] |= bit when pixel i is detected on this layer and was not on
// an earlier one (alreadydetected, dog.cpp:167-175).
__global__ void dog_detect_kernel(const float* __restrict__ r0, const float* __restrict__ r1, const float* __restrict__ r2,
                                  const float* __restrict__ r3, int W, int H, int margin, uint8_t bit,
                                  uint8_t* __restrict__ flag) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= W || y < margin || H - margin <= y || x < margin || W - margin <= x) return;
  const size_t i = (size_t)y * W + x;
  if (flag[i]) return;
  const float v = dogv(r1, r2, i);
  if (v == 0.0f) return;
  const size_t nb[8] = {i - W - 1, i - 1, i + W - 1, i - W, i + W, i - W + 1, i + 1, i + W + 1};
  int f = 0;
  if (0.0f < v) {
    f = 1;
    for (int k = 0; k < 8; ++k)
      if (!(dogv(r1, r2, nb[k]) < v)) f = 0;
  } else {
    f = -1;
    for (int k = 0; k < 8; ++k)
      if (!(dogv(r1, r2, nb[k]) > v)) f = 0;
  }
  const float p = dogv(r0, r1, i), n = dogv(r2, r3, i);
  int ok = 0;
  if (f == 1) ok = (p < v && n < v);
  else if (f == -1) ok = (v < p && v < n);
  if (ok) flag[i] = bit;
}

// CDifferenceOfGaussians::run selection (dog.cpp:164-190): detections of layer 1 (raster order)
// then layer 2, every detection inserted and the smallest erased beyond 4.  Response |c|.
__global__ void dog_select_kernel(const uint8_t* __restrict__ flag, const float* __restrict__ ra,
                                  const float* __restrict__ rb, const float* __restrict__ rc, int W, int H,
                                  int margin1, int margin2, int gsize, int bw, int bh, FeatPoint* __restrict__ out,
                                  int* __restrict__ cnt) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= bw * bh) return;
  const int bx = b % bw, by = b / bw;
  SmallSet s;
  s.n = 0;
  for (int layer = 1; layer <= 2; ++layer) {
    const int margin = layer == 1 ? margin1 : margin2;
    const float* lo = layer == 1 ? ra : rb;
    const float* hi = layer == 1 ? rb : rc;
    const int y0 = max(by * gsize, margin), y1 = min(by * gsize + gsize, H - margin);
    const int x0 = max(bx * gsize, margin), x1 = min(bx * gsize + gsize, W - margin);
    for (int y = y0; y < y1; ++y)
      for (int x = x0; x < x1; ++x) {
        const size_t i = (size_t)y * W + x;
        if (flag[i] != layer) continue;
        s.insert(fabsf(dogv(lo, hi, i)), x, y);
        if (4 < s.n) s.erase_first();
      }
  }
  write_block(s, b, out, cnt);
}

inline dim3 grid1(long long n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

template <typename T>
hipError_t conv(const T* in, T* out, const uint8_t* m, int W, int H, const FeatFilter& f, bool y, hipStream_t st) {
  const dim3 g((W + kBlock - 1) / kBlock, H);
  if (y) hipLaunchKernelGGL((conv_kernel<T, true>), g, dim3(kBlock), 0, st, in, out, m, W, H, f);
  else hipLaunchKernelGGL((conv_kernel<T, false>), g, dim3(kBlock), 0, st, in, out, m, W, H, f);
  return hipGetLastError();
}

}  // namespace

#define FCHK(x)                        \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

hipError_t FeatBuffers::reserve(long long npix, int nblocks) {
  if (npix > cap_pix) {
    release_pix();
    const size_t f4 = (size_t)npix * sizeof(float4), f1 = (size_t)npix * sizeof(float);
    FCHK(hipMalloc(&img, f4));
    FCHK(hipMalloc(&a4, f4));
    FCHK(hipMalloc(&b4, f4));
    FCHK(hipMalloc(&c4, f4));
    for (int k = 0; k < 6; ++k) FCHK(hipMalloc(&f[k], f1));
    FCHK(hipMalloc(&mask, (size_t)npix));
    FCHK(hipMalloc(&flag, (size_t)npix));
    cap_pix = npix;
  }
  if (nblocks > cap_blocks) {
    if (pts) (void)hipFree(pts);
    if (cnt) (void)hipFree(cnt);
    pts = nullptr;
    cnt = nullptr;
    FCHK(hipMalloc(&pts, (size_t)nblocks * 2 * 4 * sizeof(FeatPoint)));
    FCHK(hipMalloc(&cnt, (size_t)nblocks * 2 * sizeof(int)));
    cap_blocks = nblocks;
  }
  return hipSuccess;
}

void FeatBuffers::release_pix() {
  for (float4** p : {&img, &a4, &b4, &c4})
    if (*p) (void)hipFree(*p), *p = nullptr;
  for (int k = 0; k < 6; ++k)
    if (f[k]) (void)hipFree(f[k]), f[k] = nullptr;
  if (mask) (void)hipFree(mask), mask = nullptr;
  if (flag) (void)hipFree(flag), flag = nullptr;
  cap_pix = 0;
}

FeatBuffers::~FeatBuffers() {
  release_pix();
  if (pts) (void)hipFree(pts);
  if (cnt) (void)hipFree(cnt);
}

hipError_t detect_features(const FeatJob& j, FeatBuffers& B, hipStream_t st) {
  const int W = j.W, H = j.H;
  const long long npix = (long long)W * H;
  const int nb = j.bw * j.bh;
  FCHK(B.reserve(npix, nb));
  const bool has_mask = j.mask || j.edge;
  uint8_t* m = has_mask ? B.mask : nullptr;
  hipLaunchKernelGGL(feat_load_kernel, grid1(npix), dim3(kBlock), 0, st, j.pyr, j.mask, j.edge, (int)npix, B.img, m);
  FCHK(hipGetLastError());

  // ---- Harris (harris.cpp:142-164, 75-121, 166-198, 225-249)
  FCHK(conv(B.img, B.a4, m, W, H, j.dfilter, false, st));  // dIdx = convolveY(ifilter, convolveX(dfilter, I))
  FCHK(conv(B.a4, B.b4, m, W, H, j.ifilter, true, st));
  FCHK(conv(B.img, B.a4, m, W, H, j.ifilter, false, st));  // dIdy = convolveY(dfilter, convolveX(ifilter, I))
  FCHK(conv(B.a4, B.c4, m, W, H, j.dfilter, true, st));
  hipLaunchKernelGGL(harris_products_kernel, grid1(npix), dim3(kBlock), 0, st, B.b4, B.c4, m, (int)npix, B.f[0], B.f[1],
                     B.f[2]);
  FCHK(hipGetLastError());
  for (int k = 0; k < 3; ++k) {  // blur with gaussI, X then Y (preprocess2)
    FCHK(conv(B.f[k], B.f[3], m, W, H, j.gaussI, false, st));
    FCHK(conv(B.f[3], B.f[k], m, W, H, j.gaussI, true, st));
  }
  hipLaunchKernelGGL(harris_response_kernel, grid1(npix), dim3(kBlock), 0, st, B.f[0], B.f[1], B.f[2], m, (int)npix,
                     B.f[3]);
  FCHK(hipGetLastError());
  hipLaunchKernelGGL(harris_nms_kernel, dim3((W + kBlock - 1) / kBlock, H), dim3(kBlock), 0, st, B.f[3], B.f[4], W, H);
  FCHK(hipGetLastError());
  hipLaunchKernelGGL(harris_select_kernel, grid1(nb), dim3(kBlock), 0, st, B.f[4], W, H, j.harris_margin, j.gsize,
                     j.bw, j.bh, B.pts, B.cnt);
  FCHK(hipGetLastError());

  // ---- DoG (dog.cpp:130-190): res maps r0..r4 at firstScale * scalestep^k
  float* r[5] = {B.f[0], B.f[1], B.f[2], B.f[3], B.f[5]};
  for (int k = 0; k < 5; ++k) {
    FCHK(conv(B.img, B.a4, m, W, H, j.dog_gauss[k], false, st));
    FCHK(conv(B.a4, B.b4, m, W, H, j.dog_gauss[k], true, st));
    hipLaunchKernelGGL(dog_norm_kernel, grid1(npix), dim3(kBlock), 0, st, B.b4, (int)npix, r[k]);
    FCHK(hipGetLastError());
  }
  FCHK(hipMemsetAsync(B.flag, 0, (size_t)npix, st));
  const dim3 g2((W + kBlock - 1) / kBlock, H);
  hipLaunchKernelGGL(dog_detect_kernel, g2, dim3(kBlock), 0, st, r[0], r[1], r[2], r[3], W, H, j.dog_margin[0],
                     (uint8_t)1, B.flag);
  FCHK(hipGetLastError());
  hipLaunchKernelGGL(dog_detect_kernel, g2, dim3(kBlock), 0, st, r[1], r[2], r[3], r[4], W, H, j.dog_margin[1],
                     (uint8_t)2, B.flag);
  FCHK(hipGetLastError());
  hipLaunchKernelGGL(dog_select_kernel, grid1(nb), dim3(kBlock), 0, st, B.flag, r[1], r[2], r[3], W, H,
                     j.dog_margin[0], j.dog_margin[1], j.gsize, j.bw, j.bh, B.pts + 4 * nb, B.cnt + nb);
  return hipGetLastError();
}

}  // namespace pmvsdev
