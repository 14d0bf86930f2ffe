// pmvs_features.h -- host interface of the feature-detection kernels (pmvs_features.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmvsdev {

// A 1-D filter (CDetector::setGaussI weights, or the [-0.5 0 0.5] / [1/3 1/3 1/3] derivative
// filters of CHarris::preprocess); at most 32 taps.
struct FeatFilter {
  float w[32];
  int n;
};

struct FeatPoint {  // CPoint: _icoord (x, y), _response, _type
  float x, y, response;
  int type;
};

struct FeatJob {
  const uint32_t* pyr;   // the view's RGBA8 slab at the option level
  const uint8_t* mask;   // level mask (NULL if none)
  const uint8_t* edge;   // level edge map (NULL if none)
  int W, H;
  int gsize, bw, bh;     // selection block size (2 * fcsize) and block grid
  int harris_margin;     // (int)_gaussD.size() / 2
  FeatFilter dfilter, ifilter, gaussI;
  FeatFilter dog_gauss[5];  // setGaussI(firstScale * scalestep^k), k = 0..4
  int dog_margin[2];        // (int)ceil(2 * cscale) of the two detection layers
};

struct FeatBuffers {
  float4 *img = nullptr, *a4 = nullptr, *b4 = nullptr, *c4 = nullptr;
  float* f[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  uint8_t *mask = nullptr, *flag = nullptr;
  FeatPoint* pts = nullptr;  // [2][nblocks][4]: Harris blocks, then DoG blocks
  int* cnt = nullptr;        // [2][nblocks]
  long long cap_pix = 0;
  int cap_blocks = 0;
  hipError_t reserve(long long npix, int nblocks);
  void release_pix();
  ~FeatBuffers();
};

// Runs both detectors of one view; per-block results land in B.pts / B.cnt (block raster order,
// each block's points in ascending multiset order).
hipError_t detect_features(const FeatJob& job, FeatBuffers& B, hipStream_t st);

}  // namespace pmvsdev
