// pmvs_refine_split.hip -- refinePatchBFGS (optim.cpp:580-658), split form: optimizer and evaluator
// wavefronts of one workgroup per CU.  A translation unit of its own
// because it is compiled without SLP vectorisation (Makefile): packing the evaluator's per-texture
// float arithmetic into pairs made its 147 sample registers spill (1.6 KB per lane against 0.4 KB).
#include <hip/hip_runtime.h>

#include "bobyqa_dev.h"
#include "pmvs_device.h"
#include "pmvs_launch.h"
#include "pmvs_refine.h"

namespace pmvsdev {

// Diagnostic build only (-DBQ_PROFILE, libpmvs_amd_prof.so): wave time per role and phase in
// DevStats::prof -- optimizer: [0] refill, [1] BOBYQA step, [2] publish, [3] waiting for its
// chunks (its own chunk evaluations excluded); evaluator: [4] setup + gather + normalize, [6] dot +
// reduction, [7] idle.
#if defined(BQ_PROFILE)
#define SP_NOW() __builtin_amdgcn_s_memtime()
#define SP_MARK(slot)                                      \
  do {                                                     \
    const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    prof[slot] += _t - tprev;                              \
    tprev = _t;                                            \
  } while (0)
#else
#define SP_NOW() 0ull
#define SP_MARK(slot) \
  do {                \
  } while (0)
#endif

// ---------------------------------------------------------------- refinePatchBFGS, split form
// One 512-thread workgroup per CU (8 wavefronts, 2 per SIMD), persistent, pulling candidates from
// the launch's queue.  Its wavefronts have two roles:
//   * G optimizer wavefronts: wavefront g steps CG chains, one lane each, their BqStates in LDS, so
//     one instruction stream of the divergent f64 BOBYQA step serves up to CG chains (the wavefront
//     form serves 6).  After a step it publishes its chains' objective requests, packed in chain
//     order into chunks of at most 64 / LP textures, then evaluates unclaimed chunks of its own
//     group until every chunk of the round is done.
//   * 8 - G evaluator wavefronts: they claim chunks of any group (split_chunk).
// A chunk is evaluated with LP lanes per texture and everything in registers: the setup, the
// texture's samples gathered in sample order, normalize's moments and the robust INCC against the
// request's reference texture (its normalised samples read from the lanes holding them), each
// sequential sum in the reference's order; the reference texture's lane then reduces the request as
// request_value does.  Results, optimizer trajectories and counters equal the wavefront form's.
// While one group's requests are evaluated, the other groups step, so a CU's optimizer and texture
// work overlap instead of alternating inside each wavefront.  Handshake through LDS: per group,
// `avail` (chunks not yet claimed: set by the group's atomic exchange after its tables are written,
// taken by atomic decrements; a stale decrement only drives it below 0) and `done` (chunks
// evaluated).  No workgroup barrier after the start.  DESIGN.md §5c.
// Wavefronts per SIMD (register budget) and workgroup size: 2 and 512 (8 wavefronts, 256 VGPRs); an
// experiment build (SPLIT_WPE=1, SPLIT_THREADS=256) gives 4 wavefronts 512 registers each.
#ifndef SPLIT_WPE
#define SPLIT_WPE 2
#endif
#ifndef SPLIT_THREADS_
#define SPLIT_THREADS_ 512
#endif
constexpr int SPLIT_THREADS = SPLIT_THREADS_;
constexpr int SPLIT_TS = 64;  // texture slots per chunk at most (LP = 1)

template <int WS, int G, int CG>
struct RefSplitLds {
  static constexpr int NCH = G * CG;
  static constexpr int SLOTS = CG * PMVS_MAX_TAU;  // a group's slots per round (<= 16 textures per request)
  BqState bq[NCH];
  float geo[NCH][16];                       // requesting chain: coord, normal, pxaxis, pyaxis
  double fv[NCH];                           // the chain's objective value, written by its evaluator
  int cand[NCH];                            // the chain's candidate (need 2 reads its weights)
  unsigned short views[NCH][PMVS_MAX_TAU];  // chain: first size images
  unsigned char need[NCH], size[NCH];
  unsigned char sreq[G][SLOTS], sidx[G][SLOTS];  // slot -> chain within the group, texture index
  short choff[G][CG + 1];                   // chunk k of group g: slots [choff[g][k], choff[g][k + 1])
  int nchunk[G];
  int avail[G], done[G];
  int live;                                 // optimizer wavefronts still running
  int ejvalid[8][SPLIT_TS];                 // per wavefront: its chunk's per-texture results for the reduction
  float ejres[8][SPLIT_TS];
};

#define SPLIT_AS __attribute__((address_space(3)))
__device__ __forceinline__ int lds_load_acq(SPLIT_AS int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One chunk (group g, chunk k) evaluated by the calling wavefront -- an evaluator, or an optimizer
// wavefront waiting for its own group.  TS = 64 / LP textures, LP lanes per texture: lane `sub` of a
// texture holds its samples [sub * K, sub * K + K) (K = ceil(S / LP)) in registers.  Gather, bilinear
// weights and the element-wise normalisation are per lane; each of normalize's and dot's sequential
// sums runs in LP stages, lane sub continuing the partial sum of lane sub - 1, so every sum is the
// reference's single left-to-right chain (optim.cpp:1031-1077).  LP > 1 shortens a chunk, whose
// instruction count is what the optimizer waits for.  Returns the valid textures its my_f requests
// counted (request_value) and signals the chunk done.
template <int WS, int G, int CG, int LP>
__device__ __forceinline__ unsigned long long split_chunk_body(const DScene& s, SPLIT_AS RefSplitLds<WS, G, CG>& C,
                                                               RefineJob* __restrict__ jobs, int g, int k,
                                                               unsigned long long* prof) {
  constexpr int S = WS * WS;
  constexpr int K = (S + LP - 1) / LP;
  constexpr int NB = 7;  // samples whose texel loads are in flight together
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & (WAVE - 1);
  const int t = lane / LP, sub = lane - t * LP;  // the lane's texture slot and part of it
  const int k0 = sub * K;
  const int kn = k0 < S ? (S - k0 < K ? S - k0 : K) : 0;  // samples of this lane
  SPLIT_AS int* ejvalid = C.ejvalid[wave];
  SPLIT_AS float* ejres = C.ejres[wave];
  unsigned long long tex_valid = 0;
  unsigned long long tprev = SP_NOW();
  (void)prof;
  const int o0 = C.choff[g][k], nj = C.choff[g][k + 1] - o0;
  const bool mine = t < nj;
  const int chain = mine ? (int)C.sreq[g][o0 + t] : 0;
  const int idx = mine ? (int)C.sidx[g][o0 + t] : 0;
  const int cc = g * CG + chain;
  // setup (every lane of the texture computes it)
  TexGeom T;
  T.ok = 0;
  if (mine) T = tex_geom<WS>(s, (const float*)C.geo[cc], C.views[cc][idx]);
  // gather: samples in sample order, rows by the `left += dy` recurrence, columns by `+= dx`
  // (optim.cpp:850-860) -- the lane's first sample reached by the same additions
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
      __builtin_amdgcn_sched_barrier(0);  // one batch of loads in flight at a time: bounded registers
    }
  }
  // normalize (optim.cpp:1031-1067), the channel sums in LP stages
  const bool ok = T.ok != 0;
  const int last = t * LP + LP - 1;  // the lane that ends a texture's sums
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (ok && sub == j) {
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < kn) { a0 += X[q]; a1 += Y[q]; a2 += Z[q]; }
    }
    if (j + 1 < LP) {
      const float u0 = __shfl_up(a0, 1), u1 = __shfl_up(a1, 1), u2 = __shfl_up(a2, 1);
      if (sub == j + 1) { a0 = u0; a1 = u1; a2 = u2; }
    }
  }
  a0 = __shfl(a0, last); a1 = __shfl(a1, last); a2 = __shfl(a2, last);
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
      const float u = __shfl_up(ave2, 1);
      if (sub == j + 1) ave2 = u;
    }
  }
  ave2 = __shfl(ave2, last);
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
  SP_MARK(4);
  // robust INCC against the reference texture (optim.cpp:561-567, 919-929): the reference texture's
  // normalised samples from its lane with the same part, the products summed in sample order
  // (R, G, B per sample) in LP stages
  const int rt = mine ? t - idx : t;  // the request's reference texture (index 0)
  const int src = rt * LP + sub;
  const int refok = __shfl(T.ok, src);
  float ans = 0.0f;
#if !defined(SPLIT_DOT_STREAM)  // the reference texture's samples pulled at once (A/B r05m: equal)
  float px[K], py[K], pz[K];
#pragma unroll
  for (int q = 0; q < K; ++q) { px[q] = __shfl(X[q], src); py[q] = __shfl(Y[q], src); pz[q] = __shfl(Z[q], src); }
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (ok && sub == j) {
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < kn) {
          ans += px[q] * X[q];
          ans += py[q] * Y[q];
          ans += pz[q] * Z[q];
        }
    }
    if (j + 1 < LP) {
      const float u = __shfl_up(ans, 1);
      if (sub == j + 1) ans = u;
    }
  }
#else
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    // stage j: the lanes with sub == j, whose reference lanes (same sub) are active with them, read the
    // reference samples one at a time (no K-wide copy of them in registers)
    if (sub == j) {
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < kn) {
          const float px = __shfl(X[q], src), py = __shfl(Y[q], src), pz = __shfl(Z[q], src);
          if (ok) {
            ans += px * X[q];
            ans += py * Y[q];
            ans += pz * Z[q];
          }
        }
    }
    if (j + 1 < LP) {
      const float u = __shfl_up(ans, 1);
      if (sub == j + 1) ans = u;
    }
  }
#endif
  if (mine && sub == LP - 1) {
    float jr = 0.0f;
    if (idx >= 1 && refok && ok) jr = robustincc((float)(1.0 - (double)__fdiv_rn(ans, (float)(3 * S))));
    ejvalid[t] = T.ok;
    ejres[t] = jr;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // the request's value on its reference texture's last lane, in request_value's order
  if (mine && idx == 0 && sub == LP - 1) {
    struct {
      SPLIT_AS int* jvalid;
      SPLIT_AS float* jres;
    } V = {ejvalid, ejres};
    const int need = C.need[cc];
    C.fv[cc] = request_value(s, V, t, C.size[cc], need, jobs[C.cand[cc]], tex_valid);
  }
  SP_MARK(6);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_fetch_add(&C.done[g], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  return tex_valid;
}
// Out of line for the optimizer wavefronts (inlined there, the chunk's registers and the optimizer's
// spilled); the call saves and restores the callee-saved registers the chunk uses (78 per lane at
// LP = 2), so the evaluators inline the body instead.
template <int WS, int G, int CG, int LP>
__device__ __noinline__ unsigned long long split_chunk(const DScene& s, SPLIT_AS RefSplitLds<WS, G, CG>& C,
                                                       RefineJob* __restrict__ jobs, int g, int k, unsigned long long* prof) {
  return split_chunk_body<WS, G, CG, LP>(s, C, jobs, g, k, prof);
}

// The roles and the chunk as separate functions, so that each gets its own register allocation
// (inlined into one body, the chunk's sample registers and the optimizer's call sites spilled).
template <int WS, int G, int CG, int LP>
__device__ __noinline__ void split_optimizer(const DScene& s, SPLIT_AS RefSplitLds<WS, G, CG>& C, RefineJob* __restrict__ jobs,
                                             int n, int nc_active, DevStats* st) {
  constexpr int TS = WAVE / LP;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & (WAVE - 1);
  const int g = wave;
  const bool owner = lane < CG && lane < nc_active;
  const int c = g * CG + (lane < CG ? lane : 0);
  BQ_AS BqState& bq = *(BQ_AS BqState*)&C.bq[c];
  RefineSetup R;
  int cand = -1, need = 0, evals = 0, size = 0, nimg = 0, rc = 0;
  bool exhausted = !owner;
  double fv = 0.0;
  float fcoord[4], fnormal[4];
  unsigned long long nevals = 0, rounds = 0, tex_valid = 0, grabs = 0, chunks = 0;
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999};
  const double ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = SP_NOW();
  for (;;) {
    // (a) refill an idle chain from the queue (skipping candidates that failed preProcess)
    while (cand < 0 && !exhausted) {
      const unsigned long long q = atomicAdd(&st->queue2, 1ull);
      if (q >= (unsigned long long)n) {
        exhausted = true;
        atomicMax(&st->t_drain_inv, ~__builtin_amdgcn_s_memrealtime());
        break;
      }
      const RefineJob& J = jobs[q];
      if (J.status != PMVS_ACCEPTED) continue;
      cand = (int)q;
      for (int i = 0; i < 4; ++i) { R.center[i] = J.center[i]; R.ray[i] = J.ray[i]; }
      R.dscale = J.dscale;
      R.ascale = s.ascale;
      R.ref = J.images[0];
      nimg = J.nimg;
      size = imin(s.tau, nimg);
      for (int i = 0; i < size; ++i) C.views[c][i] = (unsigned short)J.images[i];
      C.cand[c] = cand;
      evals = 0;
      const double x0[3] = {J.x0[0], J.x0[1], J.x0[2]};
      bq_begin(bq, x0, lb, ub, 1.e-7, 1000);
      fv = 0.0;
      need = 0;
    }
    SP_MARK(0);
    // (b) advance BOBYQA when the chain holds an objective value (or just started)
    if (cand >= 0 && need == 0) {
      const int r = (bq.resume < 0) ? BQ_DONE : bq_step(bq, fv);
      if (r == BQ_NEED_F) {
        need = 1;
        const double xe[3] = {bq.xeval[0], bq.xeval[1], bq.xeval[2]};
        decode(s, R, xe, fcoord, fnormal);
      } else {
        rc = bq.rc;
        const bool success = (rc == BQR_SUCCESS || rc == 2 || rc == 3 || rc == BQR_XTOL);
        RefineJob& J = jobs[cand];
        J.refine_code = rc;
        J.evals = evals;
        if (success) {
          const double xo[3] = {bq.xout[0], bq.xout[1], bq.xout[2]};
          decode(s, R, xo, fcoord, fnormal);
          if (nimg < 2) {  // computeINCC returns 2.0 without grabbing (optim.cpp:866)
            J.ncc = (float)(1.0 - (double)unrobustincc(2.0f));
            for (int i = 0; i < 4; ++i) { J.rcoord[i] = fcoord[i]; J.rnormal[i] = fnormal[i]; }
            cand = -1;
          } else {
            need = 2;  // final computeINCC (robust, weighted) at the refined geometry
          }
        } else {
          cand = -1;  // geometry and _ncc stay unrefined (optim.cpp:649-655)
        }
      }
    }
    SP_MARK(1);
    // (c) publish the requests: geometry, then the chunk tables, then `avail`
    const bool req = (cand >= 0 && need != 0);
    if (req) {
      float px[4], py[4];
      get_paxes(s, s.views[R.ref], fcoord, fnormal, px, py);
      for (int i = 0; i < 4; ++i) {
        C.geo[c][i] = fcoord[i]; C.geo[c][4 + i] = fnormal[i];
        C.geo[c][8 + i] = px[i]; C.geo[c][12 + i] = py[i];
      }
      C.need[c] = (unsigned char)need;
      C.size[c] = (unsigned char)size;
    }
    bool pending = req;
    int k = 0, base = 0;
    while (__ballot(pending) != 0ull) {
      const int sz = pending ? size : 0;
      const int off = wave_excl_scan(sz);
      const bool in = pending && (off + sz <= TS);
      const int nj = __shfl(off + sz, 63 - __clzll(__ballot(in)));
      if (in) {
        for (int i = 0; i < sz; ++i) {
          C.sreq[g][base + off + i] = (unsigned char)lane;
          C.sidx[g][base + off + i] = (unsigned char)i;
        }
      }
      if (lane == 0) C.choff[g][k] = (short)base;
      base += nj;
      pending = pending && !in;
      ++k;
    }
    rounds++;
    if (k == 0) {
      if (__ballot(cand >= 0 || !exhausted) == 0ull) break;
      continue;
    }
    if (lane == 0) {
      C.choff[g][k] = (short)base;
      C.nchunk[g] = k;
      C.done[g] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_exchange(&C.avail[g], k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    SP_MARK(2);
    // (d) wait for the evaluators, evaluating this group's unclaimed chunks meanwhile
    while (lds_load_acq(&C.done[g]) < k) {
      int got = -1;
      if (lane == 0 && lds_load_acq(&C.avail[g]) > 0) {
        const int old = __hip_atomic_fetch_add(&C.avail[g], -1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old > 0) got = C.nchunk[g] - old;
      }
      got = __shfl(got, 0);
      if (got >= 0) {
        SP_MARK(3);
        tex_valid += split_chunk<WS, G, CG, LP>(s, C, jobs, g, got, prof);
        tprev = SP_NOW();
        grabs += C.choff[g][got + 1] - C.choff[g][got];
        chunks++;
      } else {
        __builtin_amdgcn_s_sleep(2);
      }
    }
    SP_MARK(3);
    // (e) consume the results
    if (req) {
      fv = C.fv[c];
      if (need == 1) {
        evals++;
        nevals++;
        need = 0;
      } else {
        RefineJob& J = jobs[cand];
        J.ncc = (float)(1.0 - (double)unrobustincc((float)fv));
        for (int i = 0; i < 4; ++i) { J.rcoord[i] = fcoord[i]; J.rnormal[i] = fnormal[i]; }
        cand = -1;
        need = 0;
      }
    }
  }
  if (lane == 0) __hip_atomic_fetch_add(&C.live, -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int d = 32; d >= 1; d >>= 1) {
    nevals += __shfl_xor(nevals, d);
    tex_valid += __shfl_xor(tex_valid, d);
  }
  if (lane == 0) {
#if defined(BQ_PROFILE)
    for (int i = 0; i < 4; ++i) atomicAdd(&st->prof[i], prof[i]);
#endif
    atomicAdd(&st->evals, nevals);
    atomicAdd(&st->tex_valid, tex_valid);
    atomicAdd(&st->tex_grabs, grabs);
    atomicAdd(&st->chunks, chunks);
    atomicAdd(&st->rounds, rounds);
    atomicMax(&st->t_last, __builtin_amdgcn_s_memrealtime());
  }
}

// An evaluator wavefront: claims chunks of any group, groups scanned from a per-wavefront start.
template <int WS, int G, int CG, int LP>
__device__ __noinline__ void split_evaluator(const DScene& s, SPLIT_AS RefSplitLds<WS, G, CG>& C, RefineJob* __restrict__ jobs,
                                             DevStats* st) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & (WAVE - 1);
  const int ew = wave - G;
  unsigned long long tex_valid = 0, grabs = 0, chunks = 0;
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = SP_NOW();
  for (int it = 0;; ++it) {
    // claim a chunk: groups scanned from a per-wavefront start so the evaluators spread
    int g = -1, k = -1;
    for (int i = 0; i < G && g < 0; ++i) {
      const int gg = (ew + it + i) % G;
      int got = -1;
      if (lane == 0 && lds_load_acq(&C.avail[gg]) > 0) {
        const int old = __hip_atomic_fetch_add(&C.avail[gg], -1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old > 0) got = C.nchunk[gg] - old;
      }
      got = __shfl(got, 0);
      if (got >= 0) {
        g = gg;
        k = got;
      }
    }
    if (g < 0) {
      if (lds_load_acq(&C.live) == 0) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    SP_MARK(7);
#if defined(SPLIT_EVAL_CALL)
    tex_valid += split_chunk<WS, G, CG, LP>(s, C, jobs, g, k, prof);
#else
    tex_valid += split_chunk_body<WS, G, CG, LP>(s, C, jobs, g, k, prof);
#endif
    tprev = SP_NOW();
    grabs += C.choff[g][k + 1] - C.choff[g][k];
    chunks++;
  }
  SP_MARK(7);
  for (int d = 32; d >= 1; d >>= 1) tex_valid += __shfl_xor(tex_valid, d);
  if (lane == 0) {
#if defined(BQ_PROFILE)
    for (int i = 4; i < 8; ++i) atomicAdd(&st->prof[i], prof[i]);
#endif
    atomicAdd(&st->tex_valid, tex_valid);
    atomicAdd(&st->tex_grabs, grabs);
    atomicAdd(&st->chunks, chunks);
  }
}

template <int WS, int G, int CG, int LP>
__global__ __launch_bounds__(SPLIT_THREADS) __attribute__((amdgpu_waves_per_eu(SPLIT_WPE))) void refine_split_kernel(
    DScene s, RefineJob* __restrict__ jobs, int n, int nc_active, DevStats* st) {
  using L = RefSplitLds<WS, G, CG>;
  static_assert(G >= 1 && G <= SPLIT_THREADS / WAVE && CG <= WAVE && CG <= 255, "roles");
  static_assert(sizeof(L) <= 160 * 1024, "LDS");
  __shared__ L C;
  const int tid = threadIdx.x, wave = tid >> 6;
  if (tid < G) {
    C.avail[tid] = 0;
    C.done[tid] = 0;
    C.nchunk[tid] = 0;
  }
  if (tid == 0) {
    C.live = G;
    atomicMax(&st->t_first_inv, ~__builtin_amdgcn_s_memrealtime());
  }
  __syncthreads();
  if (wave < G)
    split_optimizer<WS, G, CG, LP>(s, *(SPLIT_AS RefSplitLds<WS, G, CG>*)&C, jobs, n, nc_active, st);
  else
    split_evaluator<WS, G, CG, LP>(s, *(SPLIT_AS RefSplitLds<WS, G, CG>*)&C, jobs, st);
}


// config = 200000 + LP * 10000 + optimizer wavefronts * 1000 + chains per optimizer wavefront, LP =
// lanes per texture in the evaluators (0 reads as 1); WS <= 7
#if SPLIT_THREADS_ == 512
#define PMVS_SPLIT_CONFIGS(X) X(0, 2, 32) X(0, 4, 16) X(2, 4, 16) X(2, 5, 16) X(2, 6, 12) X(2, 6, 14) X(2, 7, 12) \
  X(2, 8, 10) X(3, 6, 14) X(4, 5, 16) X(4, 6, 14) X(4, 7, 12) X(4, 8, 10) X(8, 8, 10)
#else
#define PMVS_SPLIT_CONFIGS(X) X(2, 4, 20) X(4, 4, 20) X(8, 4, 20) X(2, 2, 40) X(4, 3, 24)
#endif
bool refine_split_supported(int config) {
#define PMVS_SPLIT_CASE(LPc, Gc, CGc) case 200000 + LPc * 10000 + Gc * 1000 + CGc:
  switch (config) {
    PMVS_SPLIT_CONFIGS(PMVS_SPLIT_CASE)
    return true;
    default: return false;
  }
#undef PMVS_SPLIT_CASE
}

template <int WS>
static hipError_t launch_split_ws(int config, const DScene& s, RefineJob* d_jobs, int n, DevStats* d_st, hipStream_t stream) {
  const int gw = (config / 1000) % 10, cg = config % 1000;
  int dev = 0, cus = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev)) != hipSuccess ||
      (e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
    return e;
  cus = cus > 0 ? cus : 1;
  // one workgroup per CU; a small batch runs fewer chains per optimizer wavefront on every CU
  const int sgrid = cus < (n + gw - 1) / gw ? cus : (n + gw - 1) / gw;
  const int per = (n + sgrid * gw - 1) / (sgrid * gw);
  const int nca = per < cg ? per : cg;
#define PMVS_SPLIT_LAUNCH(LPc, Gc, CGc)                                                                                   \
  case 200000 + LPc * 10000 + Gc * 1000 + CGc:                                                                             \
    hipLaunchKernelGGL((refine_split_kernel<WS, Gc, CGc, (LPc > 0 ? LPc : 1)>), dim3(sgrid), dim3(SPLIT_THREADS), 0, stream, \
                       s, d_jobs, n, nca, d_st);                                                                           \
    break;
  switch (config) {
    PMVS_SPLIT_CONFIGS(PMVS_SPLIT_LAUNCH)
    default: return hipErrorInvalidValue;
  }
#undef PMVS_SPLIT_LAUNCH
  return hipGetLastError();
}

hipError_t launch_refine_split(int config, const DScene& s, RefineJob* d_jobs, int n, DevStats* d_st, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  switch (s.wsize) {
    case 5: return launch_split_ws<5>(config, s, d_jobs, n, d_st, stream);
    case 7: return launch_split_ws<7>(config, s, d_jobs, n, d_st, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmvsdev
