// pmvs_layout.h -- device-resident scene layout shared by the kernels and the host API.
// (Plain structs only: included by host-only code too.)
#pragma once
#include <stdint.h>

#include "../../include/pmvs_amd.h"

#if defined(__HIPCC__)
#define PMVS_HD __host__ __device__
#else
#define PMVS_HD
#endif

namespace pmvsdev {

// A cell coordinate as pmvs_patch stores it (int16): values outside [-32767, 32767] -- only ever
// projections far outside the image, hence outside every cell grid (< 32768 cells wide / high,
// checked at scene creation) -- become -32768, which no in-grid test accepts either.
PMVS_HD inline int16_t grid16(int v) { return (v < -32767 || v > 32767) ? (int16_t)-32768 : (int16_t)v; }

constexpr int MAXL = PMVS_MAX_LEVEL + 3;

// Registration mask of one patch in the device organizer: bit i = list entry i is registered in a
// cell list (PMVS_MAX_IMAGES entries, 64 per word).
constexpr int REGW = PMVS_MAX_IMAGES / 64;
struct Reg {
  unsigned long long w[REGW];
};
constexpr int TEXCAP = 16;  // textures resident in LDS per wave (>= PMVS_MAX_TAU)

struct DView {
  float P[MAXL][12];
  float center[4];
  float oaxis[4];             // CCamera::_oaxis (optical axis, [3] = P[0][2][3] / |P[0][2][0..2]|)
  float xaxis[3], yaxis[3], zaxis[3];
  float ipscale;
  int w[MAXL], h[MAXL];
  long long pyr_off[MAXL];   // word offset of (view, level) in DScene::pyr
  long long mask_off[MAXL];  // byte offset in DScene::masks, -1 if no mask
  long long edge_off[MAXL];  // byte offset in DScene::edges, -1 if no edge map
};

struct DScene {
  const DView* views;
  const uint32_t* pyr;
  const uint8_t* masks;
  const uint8_t* edges;
  const int* vis_off;
  const int* vis;
  const int* bindexes;
  float* scratch;  // per-workgroup pairwise-INCC matrices (PMVS_MAX_IMAGES^2 floats each)
  int nb;
  int num, tnum, level, csize, wsize, minImageNum, tau, anyMask;
  float nccThreshold, nccThresholdBefore, maxAngle, angle1;
  float athreshold;     // (float)cos((double)_angleThreshold0)     optim.cpp:416
  double cosAngle1;     // cos((double)_angleThreshold1)            optim.cpp:134,823
  float sortThreshold;  // (float)(1.0f - cos(10.0*M_PI/180.0))      optim.cpp:287
  float ascale;         // (float)(M_PI / 48.0f)                      optim.cpp:590
  float log2f;          // static float Log2 = log(2.0f)              optim.cpp:813
  float quad;           // _quadThreshold (filterQuad)                 filter.cpp:443
  int depth;            // CFindMatch::_depth (isVisible, postProcess)  findMatch.hpp
  int pad2;
};

// One candidate between the three refine-batch kernels (pre -> refine -> post), in HBM.
struct RefineJob {
  float coord[4], normal[4];   // geometry after preProcess (refine input)
  float center[4], ray[4];     // refinePatchBFGS setup: _centersT, _raysT (optim.cpp:584-586)
  float dscale, ascale;        // _dscale/_ascale set by setScales in preProcess
  float ncc;                   // refine output _ncc (-1 when not refined)
  int status;                  // PMVS_ACCEPTED: refine; PMVS_FAIL_PRE / PMVS_FAIL_OVERFLOW: done
  int nimg, refine_code, evals, pad;
  float weights[PMVS_MAX_TAU]; // _weightsT (optim.cpp:592-596), first min(tau, nimg)
  double x0[3];                // encode()d start point, clamped to the bounds
  float rcoord[4], rnormal[4]; // refine output geometry (decoded on success, else the input)
  int images[PMVS_MAX_IMAGES];
};

// One boundary patch as the cluster exchange sends it (pmvs_scene_set_cluster): the fields the
// reference's readPatches reads from another run's output (patchOrganizerS.cpp:133-197, Patch
// operator>> patch.cpp:6-28) with image NUMBERS (global ids), 560 bytes.
struct BRec {
  float coord[4], normal[4];
  float ncc, dscale, ascale;
  int num_images;
  int ids[PMVS_MAX_IMAGES];
};

struct DevStats {
  unsigned long long evals, tex_valid, tex_grabs, accepted, fail_pre, fail_post, refine_failed;
  unsigned long long queue;   // dynamic work-queue heads of the three kernels
  unsigned long long queue2;
  unsigned long long queue3;
  unsigned long long cyc_opt, cyc_eval, rounds, chunks;  // refine-kernel phase profile (lane 0 of each wave)
  unsigned long long prof[8];  // refill, step, publish, chunk setup, gather, normalize, dot, reduce
  unsigned long long tex_valid_wg;  // the part of tex_valid the workgroup-form kernel evaluated
  // launch tail (s_memrealtime, 100 MHz): per launch the first wavefront's start (as ~t, so atomicMax
  // keeps the minimum), the first refill that found the queue empty (~t) and the last wavefront's
  // end; refine_tail_kernel folds them into the sums below ([0] wavefront form, [1] workgroup form)
  unsigned long long t_first_inv, t_drain_inv, t_last;
  unsigned long long tail_t[2], span_t[2], tail_launches[2];
};

}  // namespace pmvsdev
