// pmvs_refine_lane.hip -- refinePatchBFGS (optim.cpp:580-658), lane form: ONE candidate per wavefront,
// its BOBYQA state spread over the wavefront's lanes (bobyqa_lane.h) and every objective evaluation
// done by the same wavefront in place.
//
// Why: a refine launch of a few thousand candidates (iterations 2-3 of the C3 loop, the seed phase) lasts
// as long as its slowest chain -- about 150 BOBYQA rounds -- and in the LDS-state forms a round is a
// serial chain of LDS round trips on one lane (tens of microseconds).  Here the step's
// loops over the 7 interpolation points are one instruction each, the state never leaves registers,
// and there is no handshake between optimizer and evaluator: the wavefront steps, evaluates, steps.
//
// The objective of one request (my_f, optim.cpp:507-578; the final robust weighted computeINCC,
// optim.cpp:865-938) is evaluated with LP lanes per texture, texture t = lane / LP: the setup
// (grabTex's frame, optim.cpp:815-846) on every lane of the texture, samples [sub*K, sub*K + K) gathered
// in sample order by the reference's `left += dy` / `+= dx` recurrences (optim.cpp:850-860), and each
// sequential sum of normalize (optim.cpp:1031-1067) and of the robust dot (optim.cpp:1069-1077) in LP
// stages, lane sub continuing lane sub - 1's partial sum, so every sum is the reference's one
// left-to-right chain.  The request's value is reduced in request_value's order (pmvs_refine.h).
// Results, optimizer trajectories and counters equal every other refine form's
// (tests/test_gpu_parity.py::test_refine_configs_bit_exact).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "bobyqa_lane.h"
#include "pmvs_device.h"
#include "pmvs_launch.h"
#include "pmvs_refine.h"

namespace pmvsdev {

#ifndef LANE_WPE
#define LANE_WPE 2
#endif
constexpr int LANE_THREADS = 256;  // four independent wavefronts per workgroup

__device__ __forceinline__ float readlane_f(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
// Lane l - 1's value (row_shr:1 DPP; a texture's LP <= 8 lanes never straddle a 16-lane row), for the
// LP-stage hand-off of an ordered sum: no LDS round trip (ds_bpermute) on the sum's chain.
__device__ __forceinline__ float shr1_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false));
}
// The last lane of each LP-lane group's value, to every lane of the group (ds_swizzle bit mode:
// lane (i & ~(LP-1)) | (LP-1) within each 32-lane half).
template <int LP>
__device__ __forceinline__ float group_last_f(float v) {
  constexpr int pattern = (0x1f & ~(LP - 1)) | ((LP - 1) << 5);
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), pattern));
}

// One request of the wavefront's candidate: the objective at the geometry geo (coord, normal, pxaxis,
// pyaxis), over its first `size` textures; need 1 = my_f, need 2 = the final computeINCC.  Every lane
// returns the value.
template <int WS, int LP>
__device__ __forceinline__ double lane_request(const DScene& s, const float* geo, int myview, int size, int need,
                                               const RefineJob& J, unsigned long long& tex_valid) {
  constexpr int S = WS * WS;
  constexpr int K = (S + LP - 1) / LP;
  constexpr int NB = 7;  // samples whose texel loads are in flight together
  const int lane = lane_id();
  const int t = lane / LP, sub = lane - t * LP;
  const int k0 = sub * K;
  const int kn = k0 < S ? (S - k0 < K ? S - k0 : K) : 0;
  const bool mine = t < size;
  TexGeom T;
  T.ok = 0;
  if (mine) T = tex_geom<WS>(s, geo, myview);
  float X[K], Y[K], Z[K];
#pragma unroll
  for (int q = 0; q < K; ++q) { X[q] = 0.0f; Y[q] = 0.0f; Z[q] = 0.0f; }
  if (T.ok && kn > 0) {
    const uint32_t* pyr = s.pyr + T.base;
    const int yy0 = k0 / WS;
    int xx = k0 - yy0 * WS;
    float rx = T.tl0, ry = T.tl1;
    for (int r = 0; r < yy0; ++r) { rx = rx + T.dy0; ry = ry + T.dy1; }
    float lx = rx, ly = ry;
    for (int c = 0; c < xx; ++c) { lx = lx + T.dx0; ly = ly + T.dx1; }
#pragma unroll
    for (int b0 = 0; b0 < K; b0 += NB) {
      uint32_t q00[NB], q01[NB], q10[NB], q11[NB];
      float fx[NB], fy[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int q = b0 + u;
        if (q < K && q < kn) {
          fx[u] = lx; fy[u] = ly;
          const int ix = (int)lx, iy = (int)ly;
          const uint32_t* p = pyr + (iy * T.W + ix);  // within one level: < 2^31 texels
          q00[u] = p[0]; q10[u] = p[1]; q01[u] = p[T.W]; q11[u] = p[T.W + 1];
          if (++xx == WS) {
            xx = 0;
            rx = rx + T.dy0; ry = ry + T.dy1;
            lx = rx; ly = ry;
          } else {
            lx = lx + T.dx0; ly = ly + T.dx1;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int q = b0 + u;
        if (q < K && q < kn) {
          const float dx1 = fx[u] - (float)(int)fx[u], dx0 = 1.0f - dx1;
          const float dy1 = fy[u] - (float)(int)fy[u], dy0 = 1.0f - dy1;
          const float f00 = dx0 * dy0, f01 = dx0 * dy1, f10 = dx1 * dy0, f11 = dx1 * dy1;
          float r = 0.0f, gg = 0.0f, bb = 0.0f;
          r += (float)(q00[u] & 0xff) * f00 + (float)(q01[u] & 0xff) * f01;
          gg += (float)((q00[u] >> 8) & 0xff) * f00 + (float)((q01[u] >> 8) & 0xff) * f01;
          bb += (float)((q00[u] >> 16) & 0xff) * f00 + (float)((q01[u] >> 16) & 0xff) * f01;
          r += (float)(q10[u] & 0xff) * f10 + (float)(q11[u] & 0xff) * f11;
          gg += (float)((q10[u] >> 8) & 0xff) * f10 + (float)((q11[u] >> 8) & 0xff) * f11;
          bb += (float)((q10[u] >> 16) & 0xff) * f10 + (float)((q11[u] >> 16) & 0xff) * f11;
          X[q] = r; Y[q] = gg; Z[q] = bb;
        }
      }
    }
  }
  // normalize (optim.cpp:1031-1067), the channel sums in LP stages
  const bool ok = T.ok != 0;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (ok && sub == j) {
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < kn) { a0 += X[q]; a1 += Y[q]; a2 += Z[q]; }
    }
    if (j + 1 < LP) {
      const float u0 = shr1_f(a0), u1 = shr1_f(a1), u2 = shr1_f(a2);
      if (sub == j + 1) { a0 = u0; a1 = u1; a2 = u2; }
    }
  }
  a0 = group_last_f<LP>(a0); a1 = group_last_f<LP>(a1); a2 = group_last_f<LP>(a2);
  const float fs3 = (float)S;
  a0 = __fdiv_rn(a0, fs3); a1 = __fdiv_rn(a1, fs3); a2 = __fdiv_rn(a2, fs3);
  float ave2 = 0.0f;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (ok && sub == j) {
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < kn) {
          const float f0 = a0 - X[q], f1 = a1 - Y[q], f2 = a2 - Z[q];
          ave2 += f0 * f0 + f1 * f1 + f2 * f2;
        }
    }
    if (j + 1 < LP) {
      const float u = shr1_f(ave2);
      if (sub == j + 1) ave2 = u;
    }
  }
  ave2 = group_last_f<LP>(ave2);
  ave2 = fsqrt_rn(__fdiv_rn(ave2, (float)(3 * S)));
  if (ave2 == 0.0f) ave2 = 1.0f;
  if (ok) {
#pragma unroll
    for (int q = 0; q < K; ++q)
      if (q < kn) {
        X[q] = __fdiv_rn(X[q] - a0, ave2);
        Y[q] = __fdiv_rn(Y[q] - a1, ave2);
        Z[q] = __fdiv_rn(Z[q] - a2, ave2);
      }
  }
  // robust INCC against the reference texture (texture 0, optim.cpp:561-567, 919-929): its normalised
  // samples read one at a time from its lane with the same part, the products summed in sample order
  // (R, G, B per sample) in LP stages
  // (stage j: the reference texture's part j is lane j's registers, read by readlane -- wave-uniform)
  float ans = 0.0f;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (sub == j) {
      const int knj = j * K < S ? (S - j * K < K ? S - j * K : K) : 0;  // samples of part j
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < knj) {
          const float px = readlane_f(X[q], j), py = readlane_f(Y[q], j), pz = readlane_f(Z[q], j);
          if (ok) {
            ans += px * X[q];
            ans += py * Y[q];
            ans += pz * Z[q];
          }
        }
    }
    if (j + 1 < LP) {
      const float u = shr1_f(ans);
      if (sub == j + 1) ans = u;
    }
  }
  // per texture: validity (bit t * LP of vmask) and the robust value on its last lane
  const unsigned long long vmask = __ballot(mine && sub == 0 && ok);
  const bool refok = (vmask & 1ull) != 0ull;
  float jr = 0.0f;
  if (mine && sub == LP - 1 && t >= 1 && refok && ok) jr = robustincc((float)(1.0 - (double)__fdiv_rn(ans, (float)(3 * S))));
  // request_value (pmvs_refine.h), in its order
  double f;
  if (need == 1) {
    const int mininum = imin(s.minImageNum, size);
    tex_valid += (unsigned long long)__popcll(vmask);
    if (!refok) {
      f = 2.0;
    } else {
      double sum = 0.0f;
      int denom = 0;
      for (int i = 1; i < size; ++i) {
        if (!((vmask >> (i * LP)) & 1ull)) continue;
        sum += (double)readlane_f(jr, i * LP + LP - 1);
        denom++;
      }
      f = (denom < mininum - 1) ? 2.0f : sum / denom;
    }
  } else {
    if (!refok) {
      f = 2.0;
    } else {
      double score = 0.0;
      float totalweight = 0.0f;
      for (int i = 1; i < size; ++i) {
        if ((vmask >> (i * LP)) & 1ull) {
          const float w = J.weights[i];
          totalweight += w;
          score += (double)(readlane_f(jr, i * LP + LP - 1) * w);
        }
      }
      f = (totalweight == 0.0f) ? 2.0 : score / (double)totalweight;
    }
  }
  return f;
}

// One objective request out of line (LANE_EVAL_CALL): decode, getPAxes and lane_request from the job
// record, so the evaluation's code exists once instead of once per CALFUN site of the optimizer (4
// copies inlined), and its registers are allocated apart from the optimizer's.
#ifndef LANE_EVAL_CALL
#define LANE_EVAL_CALL 0
#endif
struct LaneEval {
  double f;
  unsigned nvalid;
};
template <int WS, int LP>
__device__ __noinline__ LaneEval lane_eval(const DScene& s, const RefineJob* __restrict__ J, double x0, double x1,
                                           double x2, int need, int myview, int size) {
  RefineSetup R;
  for (int i = 0; i < 4; ++i) { R.center[i] = J->center[i]; R.ray[i] = J->ray[i]; }
  R.dscale = J->dscale;
  R.ascale = s.ascale;
  R.ref = __builtin_amdgcn_readfirstlane(J->images[0]);
  const double xe[3] = {x0, x1, x2};
  float fc[4], fn[4], geo[16], px[4], py[4];
  decode(s, R, xe, fc, fn);
  get_paxes(s, s.views[R.ref], fc, fn, px, py);
  for (int i = 0; i < 4; ++i) {
    geo[i] = fc[i]; geo[4 + i] = fn[i];
    geo[8 + i] = px[i]; geo[12 + i] = py[i];
  }
  unsigned long long tv = 0;
  const double f = lane_request<WS, LP>(s, geo, myview, size, need, *J, tv);
  return {f, (unsigned)tv};
}

// One wavefront per candidate, persistent: candidates from the launch's queue (DevStats::queue2), the
// ones preProcess rejected skipped.
template <int WS, int LP>
__global__ __launch_bounds__(LANE_THREADS) __attribute__((amdgpu_waves_per_eu(LANE_WPE))) void refine_lane_kernel(
    DScene s, RefineJob* __restrict__ jobs, int n, DevStats* st) {
  static_assert(WAVE / LP >= PMVS_MAX_TAU / (LP > 4 ? 2 : 1), "textures per request");
  __shared__ bql::BqlU ustate[LANE_THREADS / WAVE];  // the optimizer's wave-uniform state, one slot per wavefront
  // the slot index through readfirstlane: the compiler then knows the state's addresses, hence every value
  // and branch of the optimizer, are wave-uniform (scalar branches instead of exec-masked regions)
  BQL_AS bql::BqlU& U = *(BQL_AS bql::BqlU*)&ustate[__builtin_amdgcn_readfirstlane(threadIdx.x / WAVE)];
  const int lane = lane_id();
  const int t = lane / LP;
  unsigned long long nevals = 0, tex_valid = 0, grabs = 0, nreq = 0;
#if defined(LANE_PROFILE)
  // diagnostic build (tools: make variant VAR=laneprof VARTU=pmvs_refine_lane VARFLAGS=-DLANE_PROFILE):
  // shader cycles per wavefront in the optimizer step, the objective evaluations, whole candidates
  unsigned long long prof_step = 0, prof_eval = 0, prof_cand = 0, prof_mark = 0;
#endif
  bql::BqlProf bprof;
  if (threadIdx.x == 0) atomicMax(&st->t_first_inv, ~__builtin_amdgcn_s_memrealtime());
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999};
  const double ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  for (;;) {
    unsigned long long q = 0;
    if (lane == 0) q = atomicAdd(&st->queue2, 1ull);
    q = __builtin_amdgcn_readfirstlane((unsigned)q) | ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(q >> 32)) << 32);
    if (q >= (unsigned long long)n) {
      if (lane == 0) atomicMax(&st->t_drain_inv, ~__builtin_amdgcn_s_memrealtime());
      break;
    }
    RefineJob& J = jobs[q];
    if (__builtin_amdgcn_readfirstlane(J.status) != PMVS_ACCEPTED) continue;
    RefineSetup R;
    for (int i = 0; i < 4; ++i) { R.center[i] = J.center[i]; R.ray[i] = J.ray[i]; }
    R.dscale = J.dscale;
    R.ascale = s.ascale;
    R.ref = __builtin_amdgcn_readfirstlane(J.images[0]);
    const int nimg = __builtin_amdgcn_readfirstlane(J.nimg);
    const int size = imin(s.tau, nimg);
    const int myview = t < size ? J.images[t] : 0;
    const double x0[3] = {J.x0[0], J.x0[1], J.x0[2]};
    auto request = [&](const float* fc, const float* fn, int need) -> double {
      float geo[16], px[4], py[4];
      get_paxes(s, s.views[R.ref], fc, fn, px, py);
      for (int i = 0; i < 4; ++i) {
        geo[i] = fc[i]; geo[4 + i] = fn[i];
        geo[8 + i] = px[i]; geo[12 + i] = py[i];
      }
      grabs += size;
      ++nreq;
      return lane_request<WS, LP>(s, geo, myview, size, need, J, tex_valid);
    };
    auto fobj = [&](const double* xe) -> double {
#if defined(LANE_PROFILE)
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
#if LANE_EVAL_CALL
      const LaneEval e = lane_eval<WS, LP>(s, &J, xe[0], xe[1], xe[2], 1, myview, size);
      tex_valid += e.nvalid;
      grabs += size;
      ++nreq;
      const double fv = e.f;
#else
      float fc[4], fn[4];
      decode(s, R, xe, fc, fn);
      const double fv = request(fc, fn, 1);
#endif
#if defined(LANE_PROFILE)
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      prof_eval += t1 - t0;
      prof_step += t0 - prof_mark;
      prof_mark = t1;
#endif
      return fv;
    };
    double xo[3], minf = 0.0;
    int nev = 0;
#if defined(LANE_PROFILE)
    prof_mark = __builtin_amdgcn_s_memtime();
    const unsigned long long tc0 = prof_mark;
#endif
    const int rc = bql::bobyqa(U, fobj, x0, lb, ub, 1.e-7, 1000, xo, &minf, &nev, bprof);
    nevals += (unsigned long long)nev;
#if defined(LANE_PROFILE)
    {
      const unsigned long long tc1 = __builtin_amdgcn_s_memtime();
      prof_step += tc1 - prof_mark;  // the optimizer's tail after its last evaluation
      prof_cand += tc1 - tc0;
    }
#endif
    const bool success = (rc == BQR_SUCCESS || rc == 2 || rc == 3 || rc == BQR_XTOL);
    float fc[4], fn[4];
    float ncc = 0.0f;
    if (success) {
      decode(s, R, xo, fc, fn);
      if (nimg < 2)  // computeINCC returns 2.0 without grabbing (optim.cpp:866)
        ncc = (float)(1.0 - (double)unrobustincc(2.0f));
      else {  // final computeINCC (robust, weighted) at the refined geometry
#if LANE_EVAL_CALL
        const LaneEval e = lane_eval<WS, LP>(s, &J, xo[0], xo[1], xo[2], 2, myview, size);
        grabs += size;
        ++nreq;
        ncc = (float)(1.0 - (double)unrobustincc((float)e.f));
#else
        ncc = (float)(1.0 - (double)unrobustincc((float)request(fc, fn, 2)));
#endif
      }
    }
    if (lane == 0) {
      J.refine_code = rc;
      J.evals = nev;
      if (success) {
        J.ncc = ncc;
        for (int i = 0; i < 4; ++i) { J.rcoord[i] = fc[i]; J.rnormal[i] = fn[i]; }
      }
    }
  }
  if (lane == 0) {
    atomicAdd(&st->evals, nevals);
    atomicAdd(&st->tex_valid, tex_valid);
    atomicAdd(&st->tex_valid_wg, tex_valid);
    atomicAdd(&st->tex_grabs, grabs);
    atomicAdd(&st->rounds, nreq);
    atomicAdd(&st->chunks, nreq);
    atomicMax(&st->t_last, __builtin_amdgcn_s_memrealtime());
#if defined(LANE_PROFILE)
    atomicAdd(&st->prof[0], prof_step);
    atomicAdd(&st->prof[1], prof_eval);
    atomicAdd(&st->prof[2], prof_cand);
    atomicAdd(&st->prof[3], bprof.t[0]);
    atomicAdd(&st->prof[4], bprof.t[1]);
    atomicAdd(&st->prof[5], bprof.t[2]);
#endif
  }
}

// config 300000 + LP: the lane form with LP lanes per texture (4: up to 16 textures per request, 8: up
// to 8); 300000 picks LP from the scene's tau
bool refine_lane_supported(int config) { return config == 300000 || config == 300004 || config == 300008; }

template <int WS>
static hipError_t launch_lane_ws(int config, const DScene& s, RefineJob* d_jobs, int n, DevStats* d_st, hipStream_t stream) {
  int lp = config % 100;
  if (lp == 0) lp = s.tau <= 8 ? 8 : 4;
  if (WAVE / lp < s.tau) lp = 4;
  if (WAVE / lp < s.tau) return hipErrorInvalidValue;
  int dev = 0, cus = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev)) != hipSuccess ||
      (e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
    return e;
  cus = cus > 0 ? cus : 1;
  // persistent: LANE_WPE wavefronts per SIMD on every CU (PMVS_LANE_WPS: fewer, for latency
  // experiments), no more than the batch needs
  static const int wps = [] {
    const char* e = getenv("PMVS_LANE_WPS");
    const int v = e ? atoi(e) : LANE_WPE;
    return v >= 1 && v <= LANE_WPE ? v : LANE_WPE;
  }();
  const int waves = cus * 4 * wps;
  const int need = (n + 3) / 4;
  const int grid = need < waves / 4 ? need : waves / 4;
  if (lp == 8)
    hipLaunchKernelGGL((refine_lane_kernel<WS, 8>), dim3(grid), dim3(LANE_THREADS), 0, stream, s, d_jobs, n, d_st);
  else
    hipLaunchKernelGGL((refine_lane_kernel<WS, 4>), dim3(grid), dim3(LANE_THREADS), 0, stream, s, d_jobs, n, d_st);
  return hipGetLastError();
}

hipError_t launch_refine_lane(int config, const DScene& s, RefineJob* d_jobs, int n, DevStats* d_st, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  switch (s.wsize) {
    case 5: return launch_lane_ws<5>(config, s, d_jobs, n, d_st, stream);
    case 7: return launch_lane_ws<7>(config, s, d_jobs, n, d_st, stream);
    case 9: return launch_lane_ws<9>(config, s, d_jobs, n, d_st, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmvsdev
