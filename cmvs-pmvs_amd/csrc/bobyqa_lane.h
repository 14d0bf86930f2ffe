// bobyqa_lane.h -- BOBYQA (Powell, DAMTP 2009/NA06) with the NLopt 2.6.1 LN_BOBYQA driver semantics
// the reference relies on (reference source/pmvs/optim.cpp:615-647: n = 3, xtol_rel = 1e-7,
// maxeval = 1000), LANE-DISTRIBUTED: one optimisation chain per wavefront, its state spread over the
// wavefront's lanes instead of one lane's LDS.
//
//   * Every array Powell indexes by interpolation point k (xpt, fval, pq, zmat, w) or by bmat / vlag
//     row lives in one register per lane: lane k - 1 holds element k (xpt and bmat as three
//     column registers).  A loop over k whose iterations are independent is one instruction stream
//     in which every lane does its own k (`par`): one VALU instruction per element-wise operation.
//   * A sum over k keeps Powell's left-to-right order: the per-k terms are computed lane-parallel,
//     then added in order by a uniform chain of readlanes (`bc`).  Arg-max scans (knew, ksav, the
//     angle search) are the same in-order scans over the lanes' values.
//   * The n-vectors (xopt, gopt, d, ...) and Powell's scalars are wave-uniform values in registers;
//     a run-time index into them goes through selects (bq_get / bq_set), never through memory.
//   * The objective is called in place (CALFUN), so there is no reverse-communication state to
//     save, no LDS round trip on the step's critical path and no out-of-line call.
// The arithmetic is bobyqa_dev.h's -- itself Powell's, operation for operation -- so trajectories are
// identical.  This header also compiles for the host (g++): a wavefront is then emulated by
// 64-element arrays and `par` loops over the lanes (tests/csrc/bql_host.cpp checks the host build
// against bobyqa_dev.h's, which tests/test_bobyqa_host.py pins to oracle/bobyqa_oracle.h).
#pragma once

#include "bobyqa_dev.h"

namespace pmvsdev {
namespace bql {

// Diagnostic builds (-DLANE_PROFILE): shader cycles per optimizer phase, accumulated in registers of
// the caller's BqlProf: [0] TRSBOX, [1] ALTMOV, [2] UPDATE.
struct BqlProf {
  unsigned long long t[4] = {0, 0, 0, 0};
};
#if defined(LANE_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#define BQL_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define BQL_T1(slot, v) prof.t[slot] += __builtin_amdgcn_s_memtime() - v
#else
#define BQL_T0(v)
#define BQL_T1(slot, v)
#endif

// Host tests only (-DBQL_COUNT): how often each rare branch ran, so the tests can show they covered them.
#if defined(BQL_COUNT) && !defined(__HIPCC__)
extern long long bql_hits[16];
#define BQL_HIT(i) (++bql_hits[i])
#else
#define BQL_HIT(i) ((void)0)
#endif

constexpr int N = BQN, NPT = BQNPT, NP = BQNP, NPTM = BQNPTM, NDIM = BQNDIM, NH = BQNH;
static_assert(NDIM <= 64 && NPT <= 64, "one lane per interpolation point / bmat row");

#if defined(__HIP_DEVICE_COMPILE__)
#define BQL_HD __host__ __device__ inline __attribute__((always_inline))
// one register per lane
struct V {
  double x;
  BQL_HD double& operator[](int) { return x; }
  BQL_HD const double& operator[](int) const { return x; }
};
BQL_HD int lane() { return (int)__lane_id(); }
template <class F>
BQL_HD void par(F&& f) { f(lane()); }
template <class F>
BQL_HD unsigned long long ballot(F&& f) { return __ballot(f(lane()) ? 1 : 0); }
// lane k's value (k wave-uniform)
BQL_HD double bc(const V& v, int k) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v.x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), k);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
#else
#if defined(__HIPCC__)
#define BQL_HD __host__ __device__ inline
#else
#define BQL_HD inline
#endif
// host emulation of a wavefront: lane L is element L
struct V {
  double x[64];
  BQL_HD double& operator[](int L) { return x[L]; }
  BQL_HD const double& operator[](int L) const { return x[L]; }
};
template <class F>
BQL_HD void par(F&& f) {
  for (int L = 0; L < 64; ++L) f(L);
}
template <class F>
BQL_HD unsigned long long ballot(F&& f) {
  unsigned long long m = 0;
  for (int L = 0; L < 64; ++L)
    if (f(L)) m |= 1ull << L;
  return m;
}
BQL_HD double bc(const V& v, int k) { return v.x[k]; }
#endif

// The wave-uniform part of the state (Powell's n-vectors and scalars) lives in the wavefront's slot of
// LDS (BQL_AS, 32-bit ds addressing), not in registers: kept in VGPR pairs (the same value in every
// lane) it held ~110 doubles live across the whole optimizer and spilled 3 KB per lane.  Each phase
// (TRSBOX, ALTMOV, UPDATE, the driver's blocks) loads what it uses, and BQL_FENCE at the phase
// boundaries and around every objective call keeps the compiler from carrying values across them, so
// the registers hold the lane arrays and the current phase's temporaries only.
#if defined(__HIP_DEVICE_COMPILE__)
#define BQL_AS __attribute__((address_space(3)))
#define BQL_FENCE() __asm__ volatile("" ::: "memory")
#else
#define BQL_AS
#define BQL_FENCE() ((void)0)
#endif
struct BqlU {
  double x[N + 1], xl[N + 1], xu[N + 1], sc[N + 1], xbase[N + 1], xopt[N + 1], gopt[N + 1], hq[NH + 1], sl[N + 1],
      su[N + 1], xnew[N + 1], xalt[N + 1], d[N + 1], gnew[N + 1], pa1[N + 1], pa2[N + 1], wu[N + 1], wn[N + 1];
  double rhobeg, rhoend, f, fbeg, fsave, xoptsq, rho, delta, diffa, diffb, diffc, dnorm, distsq, dsq, crvmin, adelt,
      alpha, cauchy, beta, denom, fopt, vquad, diff, ratio, stepa, stepb, minf, rs_fbase;
  int nf, kopt, kbase, nresc, ntrits, itest, nfsav, knew, nevals, rc;
};

// element k of a lane array (k wave-uniform) := val
BQL_HD void put(V& v, int k, double val) {
  par([&](int L) {
    if (L == k) v[L] = val;
  });
}
// Element i (run-time, 1..N) of a small 1-based register array, and its store.  Plain selects over the
// constant positions (bq_get / bq_set) get folded back into an indexed load / store by the compiler,
// which then puts the array in scratch; the empty asm makes each candidate value opaque to that fold.
#if defined(__HIP_DEVICE_COMPILE__)
#define BQL_OPAQUE(v) __asm__("" : "+v"(v))
#else
#define BQL_OPAQUE(v) ((void)0)
#endif
template <int M>
BQL_HD double lget(const double (&a)[M], int i) {
  double r = a[1];
  BQL_OPAQUE(r);
#pragma unroll
  for (int k = 2; k < M; ++k) {
    double v = a[k];
    BQL_OPAQUE(v);
    r = (i == k) ? v : r;
  }
  return r;
}
template <int M>
BQL_HD void lset(double (&a)[M], int i, double val) {
#pragma unroll
  for (int k = 1; k < M; ++k) {
    double v = a[k];
    BQL_OPAQUE(v);
    a[k] = (i == k) ? val : v;
  }
}

// Lane k of column c of a 3-column lane array (c, k wave-uniform, c run-time): selects over the
// columns, so the array stays in registers (a run-time index would put it in scratch).
BQL_HD double bc3(const V (&A)[N], int c, int k) {
  const double a0 = bc(A[0], k), a1 = bc(A[1], k), a2 = bc(A[2], k);
  return c == 1 ? a1 : (c == 2 ? a2 : a0);
}
BQL_HD void put3(V (&A)[N], int c, int k, double val) {
  par([&](int L) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (L == k && j == c) A[j][L] = val;
  });
}
static_assert(N == 3 && NPTM == 3, "bc3 / put3 select over three columns");

// acc + v[0] + v[1] + ... + v[n-1], left to right (lanes whose bit of m is clear skipped)
BQL_HD double osum(double acc, const V& v, int n, unsigned long long m = ~0ull) {
#pragma unroll
  for (int k = 0; k < NDIM; ++k) {
    if (k < n) {
      const double t = bc(v, k);
      acc = ((m >> k) & 1ull) ? acc + t : acc;
    }
  }
  return acc;
}
// acc + a[0] + b[0] + a[1] + b[1] + ..., left to right: Powell's `sum = sum + p + q` per k
BQL_HD double osum2(double acc, const V& a, const V& b, int n) {
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (k < n) {
      const double ta = bc(a, k), tb = bc(b, k);
      acc = acc + ta;
      acc = acc + tb;
    }
  }
  return acc;
}

// a[i] / a[i] := v for a run-time i of an LDS-homed n-vector
template <class P>
BQL_HD double getp(P a, int i) { return a[i]; }
template <class P>
BQL_HD void setp(P a, int i, double v) { a[i] = v; }

// ---------------------------------------------------------------- TRSBOX (bobyqa_dev.h bq_trsbox)
BQL_HD void trsbox(const V (&XP)[N], const V& PQ, const BQL_AS double* xopt_m, const BQL_AS double* gopt_m,
                   const BQL_AS double* hq_m, const BQL_AS double* sl_m, const BQL_AS double* su_m, double delta,
                   BQL_AS double* xnew, BQL_AS double* d_out, BQL_AS double* gnew_out, BQL_AS double* dsq_out,
                   BQL_AS double* crvmin_out) {
  const double half = 0.5, one = 1.0, onemin = -1.0, zero = 0.0;
  double xopt[N + 1], gopt[N + 1], hq[NH + 1], sl[N + 1], su[N + 1];
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    xopt[i] = xopt_m[i];
    gopt[i] = gopt_m[i];
    sl[i] = sl_m[i];
    su[i] = su_m[i];
  }
#pragma unroll
  for (int i = 1; i <= NH; ++i) hq[i] = hq_m[i];
  double d[N + 1], gnew[N + 1];
  double xbdi[N + 1], s[N + 1], hs[N + 1], hred[N + 1];
  int iterc = 0, nact = 0, itermax = 0, itcsav = 0, iact = 0, isav = 0, iu = 0;
  double delsq, qred, crvmin, beta = 0, stepsq = 0, gredsq = 0, resid, ds, shs = 0, temp, blen = 0, stplen = 0, xsum,
                                sdec, ggsav = 0, dredsq = 0, dredg = 0, sredg = 0, angbd = 0, tempa, tempb, ssq, xsav = 0,
                                dhs = 0, dhd = 0, redmax, redsav, angt = 0, sth, rednew, rdprev = 0, rdnext = 0, cth;
  // the Hessian products' k terms need pq[k] != 0 (Powell skips the others)
  const unsigned long long mpq = ballot([&](int L) { return L < NPT && PQ[L] != zero; });
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    xbdi[i] = zero;
    if (xopt[i] <= sl[i]) {
      if (gopt[i] >= zero) xbdi[i] = onemin;
    } else if (xopt[i] >= su[i]) {
      if (gopt[i] <= zero) xbdi[i] = one;
    }
    if (xbdi[i] != zero) ++nact;
    d[i] = zero;
    gnew[i] = gopt[i];
  }
  hs[0] = hred[0] = s[0] = 0.0;
#pragma unroll
  for (int i = 1; i <= N; ++i) hs[i] = hred[i] = s[i] = 0.0;
  delsq = delta * delta;
  qred = zero;
  crvmin = onemin;
L20:
  beta = zero;
L30:
  stepsq = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] != zero) s[i] = zero;
    else if (beta == zero) s[i] = -gnew[i];
    else s[i] = beta * s[i] - gnew[i];
    stepsq += s[i] * s[i];
  }
  if (stepsq == zero) goto L190;
  if (beta == zero) {
    gredsq = stepsq;
    itermax = iterc + N - nact;
  }
  if (gredsq * delsq <= qred * 1e-4 * qred) goto L190;
  goto L210;
L50:
  resid = delsq;
  ds = zero;
  shs = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] == zero) {
      resid -= d[i] * d[i];
      ds += s[i] * d[i];
      shs += s[i] * hs[i];
    }
  }
  if (resid <= zero) goto L90;
  temp = sqrt(stepsq * resid + ds * ds);
  if (ds < zero) blen = (temp - ds) / stepsq;
  else blen = resid / (temp + ds);
  stplen = blen;
  if (shs > zero) stplen = bq_min(blen, gredsq / shs);
  iact = 0;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (s[i] != zero) {
      xsum = xopt[i] + d[i];
      if (s[i] > zero) temp = (su[i] - xsum) / s[i];
      else temp = (sl[i] - xsum) / s[i];
      if (temp < stplen) {
        stplen = temp;
        iact = i;
      }
    }
  }
  sdec = zero;
  if (stplen > zero) {
    ++iterc;
    temp = shs / stepsq;
    if (iact == 0 && temp > zero) {
      crvmin = bq_min(crvmin, temp);
      if (crvmin == onemin) crvmin = temp;
    }
    ggsav = gredsq;
    gredsq = zero;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      gnew[i] += stplen * hs[i];
      if (xbdi[i] == zero) gredsq += gnew[i] * gnew[i];
      d[i] += stplen * s[i];
    }
    sdec = bq_max(stplen * (ggsav - half * stplen * shs), zero);
    qred += sdec;
  }
  if (iact > 0) {
    ++nact;
    lset(xbdi, iact, lget(s, iact) < zero ? onemin : one);
    {
      const double di = lget(d, iact);
      delsq -= di * di;
    }
    if (delsq <= zero) goto L90;
    goto L20;
  }
  if (stplen < blen) {
    if (iterc == itermax) goto L190;
    if (sdec <= qred * .01) goto L190;
    beta = gredsq / ggsav;
    goto L30;
  }
L90:
  crvmin = zero;
L100:
  if (nact >= N - 1) goto L190;
  dredsq = zero;
  dredg = zero;
  gredsq = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] == zero) {
      dredsq += d[i] * d[i];
      dredg += d[i] * gnew[i];
      gredsq += gnew[i] * gnew[i];
      s[i] = d[i];
    } else {
      s[i] = zero;
    }
  }
  itcsav = iterc;
  goto L210;
L120:
  ++iterc;
  temp = gredsq * dredsq - dredg * dredg;
  if (temp <= qred * 1e-4 * qred) goto L190;
  temp = sqrt(temp);
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] == zero) s[i] = (dredg * d[i] - dredsq * gnew[i]) / temp;
    else s[i] = zero;
  }
  sredg = -temp;
  angbd = one;
  iact = 0;
  {
    // Powell's loop leaves for L100 at the first free i whose step reaches a bound; the angle bound is
    // updated for the i before it only.  Written with a first-hit flag instead of a goto out of the
    // loop so that the loop unrolls (and xbdi / d / s stay in registers).
    int ihit = 0;
    double xhit = zero;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      if (ihit == 0 && xbdi[i] == zero) {
        tempa = xopt[i] + d[i] - sl[i];
        tempb = su[i] - xopt[i] - d[i];
        if (tempa <= zero) {
          ihit = i;
          xhit = onemin;
        } else if (tempb <= zero) {
          ihit = i;
          xhit = one;
        } else {
          ssq = d[i] * d[i] + s[i] * s[i];
          temp = xopt[i] - sl[i];
          temp = ssq - temp * temp;
          if (temp > zero) {
            temp = sqrt(temp) - s[i];
            if (angbd * temp > tempa) {
              angbd = tempa / temp;
              iact = i;
              xsav = onemin;
            }
          }
          temp = su[i] - xopt[i];
          temp = ssq - temp * temp;
          if (temp > zero) {
            temp = sqrt(temp) + s[i];
            if (angbd * temp > tempb) {
              angbd = tempb / temp;
              iact = i;
              xsav = one;
            }
          }
        }
      }
    }
    if (ihit != 0) {
      ++nact;
      lset(xbdi, ihit, xhit);
      goto L100;
    }
  }
  goto L210;
L150:
  shs = zero;
  dhs = zero;
  dhd = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] == zero) {
      shs += s[i] * hs[i];
      dhs += d[i] * hs[i];
      dhd += d[i] * hred[i];
    }
  }
  redmax = zero;
  isav = 0;
  redsav = zero;
  iu = (int)(angbd * 17. + 3.1);
  BQL_HIT(7);
  if (iu >= 1 && iu <= 64) {
    // Powell's iu angles, one per lane (their reductions are independent), then his in-order scan
    V RR;
    par([&](int L) {
      const double at = angbd * (double)(L + 1) / (double)iu;
      const double st = (at + at) / (one + at * at);
      const double tp = shs + at * (at * dhd - dhs - dhs);
      RR[L] = st * (at * dredg - sredg - half * st * tp);
    });
    for (int i = 1; i <= iu; ++i) {
      rednew = bc(RR, i - 1);
      if (rednew > redmax) {
        redmax = rednew;
        isav = i;
        rdprev = redsav;
      } else if (i == isav + 1) {
        rdnext = rednew;
      }
      redsav = rednew;
    }
    angt = angbd * (double)iu / (double)iu;
  } else {
    for (int i = 1; i <= iu; ++i) {
      angt = angbd * (double)i / (double)iu;
      sth = (angt + angt) / (one + angt * angt);
      temp = shs + angt * (angt * dhd - dhs - dhs);
      rednew = sth * (angt * dredg - sredg - half * sth * temp);
      if (rednew > redmax) {
        redmax = rednew;
        isav = i;
        rdprev = redsav;
      } else if (i == isav + 1) {
        rdnext = rednew;
      }
      redsav = rednew;
    }
  }
  if (isav == 0) goto L190;
  if (isav < iu) {
    temp = (rdnext - rdprev) / (redmax + redmax - rdprev - rdnext);
    angt = angbd * ((double)isav + half * temp) / (double)iu;
  }
  cth = (one - angt * angt) / (one + angt * angt);
  sth = (angt + angt) / (one + angt * angt);
  temp = shs + angt * (angt * dhd - dhs - dhs);
  sdec = sth * (angt * dredg - sredg - half * sth * temp);
  if (sdec <= zero) goto L190;
  dredg = zero;
  gredsq = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    gnew[i] = gnew[i] + (cth - one) * hred[i] + sth * hs[i];
    if (xbdi[i] == zero) {
      d[i] = cth * d[i] + sth * s[i];
      dredg += d[i] * gnew[i];
      gredsq += gnew[i] * gnew[i];
    }
    hred[i] = cth * hred[i] + sth * hs[i];
  }
  qred += sdec;
  if (iact > 0 && isav == iu) {
    ++nact;
    lset(xbdi, iact, xsav);
    goto L100;
  }
  if (sdec > qred * .01) goto L120;
L190 : {
  double dsq = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    double xn = bq_max(bq_min(xopt[i] + d[i], su[i]), sl[i]);
    if (xbdi[i] == onemin) xn = sl[i];
    if (xbdi[i] == one) xn = su[i];
    xnew[i] = xn;
    d[i] = xn - xopt[i];
    dsq += d[i] * d[i];
  }
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    d_out[i] = d[i];
    gnew_out[i] = gnew[i];
  }
  *dsq_out = dsq;
  *crvmin_out = crvmin;
  return;
}
L210 : {
  int ih = 0;
#pragma unroll
  for (int j = 1; j <= N; ++j) {
    hs[j] = zero;
#pragma unroll
    for (int i = 1; i <= j; ++i) {
      ++ih;
      if (i < j) hs[j] += hq[ih] * s[i];
      hs[i] += hq[ih] * s[j];
    }
  }
  // k terms pq[k] (xpt[k] . s) xpt[k], added to hs in k order
  V P0, P1, P2;
  par([&](int L) {
    double t = zero;
    t += XP[0][L] * s[1];
    t += XP[1][L] * s[2];
    t += XP[2][L] * s[3];
    t *= PQ[L];
    P0[L] = t * XP[0][L];
    P1[L] = t * XP[1][L];
    P2[L] = t * XP[2][L];
  });
  hs[1] = osum(hs[1], P0, NPT, mpq);
  hs[2] = osum(hs[2], P1, NPT, mpq);
  hs[3] = osum(hs[3], P2, NPT, mpq);
  if (crvmin != zero) goto L50;
  if (iterc > itcsav) goto L150;
#pragma unroll
  for (int i = 1; i <= N; ++i) hred[i] = hs[i];
  goto L120;
}
}

// ---------------------------------------------------------------- ALTMOV (bobyqa_dev.h bq_altmov)
BQL_HD void altmov(const V (&XP)[N], const BQL_AS double* xopt_m, const V (&BM)[N], const V (&ZM)[NPTM],
                   const BQL_AS double* sl_m, const BQL_AS double* su_m, int kopt, int knew, double adelt,
                   BQL_AS double* xnew_m, BQL_AS double* xalt_m, BQL_AS double* alpha, BQL_AS double* cauchy) {
  const double half = 0.5, one = 1.0, zero = 0.0;
  double xopt[N + 1], sl[N + 1], su[N + 1], xnew[N + 1], xalt[N + 1];
#pragma unroll
  for (int i = 0; i <= N; ++i) {
    xopt[i] = i ? xopt_m[i] : 0.0;
    sl[i] = i ? sl_m[i] : 0.0;
    su[i] = i ? su_m[i] : 0.0;
    xnew[i] = xalt[i] = 0.0;
  }
  const double cnst = one + sqrt(2.0);
  double glag[N + 1], w[2 * N + 1];
  double temp, step = 0, tempa, tempb, bigstp, wfixsq, ggfree, wsqsav, gw, curv, scale, csave = 0, presav;
  int ksav = 0, ibdsav = 0, iflag;
  const int kn = knew - 1;
  // hcol[k] = sum_j zmat[knew][j] zmat[k][j]
  const double zk0 = bc(ZM[0], kn), zk1 = bc(ZM[1], kn), zk2 = bc(ZM[2], kn);
  V HC;
  par([&](int L) {
    double h = zero;
    h += zk0 * ZM[0][L];
    h += zk1 * ZM[1][L];
    h += zk2 * ZM[2][L];
    HC[L] = h;
  });
  *alpha = bc(HC, kn);
  const double ha = half * *alpha;
#pragma unroll
  for (int i = 1; i <= N; ++i) glag[i] = bc(BM[i - 1], kn);
  {
    V G0, G1, G2;
    par([&](int L) {
      double t = zero;
      t += XP[0][L] * xopt[1];
      t += XP[1][L] * xopt[2];
      t += XP[2][L] * xopt[3];
      t = HC[L] * t;
      G0[L] = t * XP[0][L];
      G1[L] = t * XP[1][L];
      G2[L] = t * XP[2][L];
    });
    glag[1] = osum(glag[1], G0, NPT);
    glag[2] = osum(glag[2], G1, NPT);
    glag[3] = osum(glag[3], G2, NPT);
  }
  // every point k != kopt: its step, bound and predicted value, lane-parallel; then Powell's scan
  V PRED, STEP, ISBD;
  par([&](int L) {
    const int k = L + 1;
    double dderiv = zero, distsq = zero, t;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      t = XP[i - 1][L] - xopt[i];
      dderiv += glag[i] * t;
      distsq += t * t;
    }
    double subd = adelt / sqrt(distsq);
    double slbd = -subd;
    int ilbd = 0, iubd = 0, isbd;
    const double sumin = bq_min(one, subd);
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      t = XP[i - 1][L] - xopt[i];
      if (t > zero) {
        if (slbd * t < sl[i] - xopt[i]) {
          slbd = (sl[i] - xopt[i]) / t;
          ilbd = -i;
        }
        if (subd * t > su[i] - xopt[i]) {
          subd = bq_max(sumin, (su[i] - xopt[i]) / t);
          iubd = i;
        }
      } else if (t < zero) {
        if (slbd * t > su[i] - xopt[i]) {
          slbd = (su[i] - xopt[i]) / t;
          ilbd = i;
        }
        if (subd * t < sl[i] - xopt[i]) {
          subd = bq_max(sumin, (sl[i] - xopt[i]) / t);
          iubd = -i;
        }
      }
    }
    double stp, vlag;
    if (k == knew) {
      const double diff = dderiv - one;
      stp = slbd;
      vlag = slbd * (dderiv - slbd * diff);
      isbd = ilbd;
      t = subd * (dderiv - subd * diff);
      if (fabs(t) > fabs(vlag)) {
        stp = subd;
        vlag = t;
        isbd = iubd;
      }
      const double tempd = half * dderiv;
      const double ta = tempd - diff * slbd;
      const double tb = tempd - diff * subd;
      if (ta * tb < zero) {
        t = tempd * tempd / diff;
        if (fabs(t) > fabs(vlag)) {
          stp = tempd / diff;
          vlag = t;
          isbd = 0;
        }
      }
    } else {
      stp = slbd;
      vlag = slbd * (one - slbd);
      isbd = ilbd;
      t = subd * (one - subd);
      if (fabs(t) > fabs(vlag)) {
        stp = subd;
        vlag = t;
        isbd = iubd;
      }
      if (subd > half) {
        if (fabs(vlag) < .25) {
          stp = half;
          vlag = .25;
          isbd = 0;
        }
      }
      vlag *= dderiv;
    }
    t = stp * (one - stp) * distsq;
    PRED[L] = vlag * vlag * (vlag * vlag + ha * t * t);
    STEP[L] = stp;
    ISBD[L] = (double)isbd;
  });
  presav = zero;
#pragma unroll
  for (int k = 1; k <= NPT; ++k) {
    if (k == kopt) continue;
    const double predsq = bc(PRED, k - 1);
    if (predsq > presav) {
      presav = predsq;
      ksav = k;
      ibdsav = (int)bc(ISBD, k - 1);
    }
  }
  const double stpsav = ksav > 0 ? bc(STEP, ksav - 1) : 0.0;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    const double xk = ksav > 0 ? bc(XP[i - 1], ksav - 1) : 0.0;
    temp = xopt[i] + stpsav * (xk - xopt[i]);
    xnew[i] = bq_max(sl[i], bq_min(su[i], temp));
  }
  if (ibdsav < 0) lset(xnew, -ibdsav, lget(sl, -ibdsav));
  if (ibdsav > 0) lset(xnew, ibdsav, lget(su, ibdsav));
  bigstp = adelt + adelt;
  iflag = 0;
L100:
  wfixsq = zero;
  ggfree = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    w[i] = zero;
    tempa = bq_min(xopt[i] - sl[i], glag[i]);
    tempb = bq_max(xopt[i] - su[i], glag[i]);
    if (tempa > zero || tempb < zero) {
      w[i] = bigstp;
      ggfree += glag[i] * glag[i];
    }
  }
  if (ggfree == zero) {
    *cauchy = zero;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      xnew_m[i] = xnew[i];
      xalt_m[i] = xalt[i];
    }
    return;
  }
L120:
  temp = adelt * adelt - wfixsq;
  if (temp > zero) {
    wsqsav = wfixsq;
    step = sqrt(temp / ggfree);
    ggfree = zero;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      if (w[i] == bigstp) {
        temp = xopt[i] - step * glag[i];
        if (temp <= sl[i]) {
          w[i] = sl[i] - xopt[i];
          wfixsq += w[i] * w[i];
        } else if (temp >= su[i]) {
          w[i] = su[i] - xopt[i];
          wfixsq += w[i] * w[i];
        } else {
          ggfree += glag[i] * glag[i];
        }
      }
    }
    if (wfixsq > wsqsav && ggfree > zero) goto L120;
  }
  gw = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    if (w[i] == bigstp) {
      w[i] = -step * glag[i];
      xalt[i] = bq_max(sl[i], bq_min(su[i], xopt[i] + w[i]));
    } else if (w[i] == zero) {
      xalt[i] = xopt[i];
    } else if (glag[i] > zero) {
      xalt[i] = sl[i];
    } else {
      xalt[i] = su[i];
    }
    gw += glag[i] * w[i];
  }
  {
    V CV;
    par([&](int L) {
      double t = zero;
      t += XP[0][L] * w[1];
      t += XP[1][L] * w[2];
      t += XP[2][L] * w[3];
      CV[L] = HC[L] * t * t;
    });
    curv = osum(zero, CV, NPT);
  }
  if (iflag == 1) curv = -curv;
  if (curv > -gw && curv < -cnst * gw) {
    scale = -gw / curv;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      temp = xopt[i] + scale * w[i];
      xalt[i] = bq_max(sl[i], bq_min(su[i], temp));
    }
    temp = half * gw * scale;
    *cauchy = temp * temp;
  } else {
    temp = gw + half * curv;
    *cauchy = temp * temp;
  }
  if (iflag == 0) {
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      glag[i] = -glag[i];
      w[N + i] = xalt[i];
    }
    csave = *cauchy;
    iflag = 1;
    goto L100;
  }
  if (csave > *cauchy) {
#pragma unroll
    for (int i = 1; i <= N; ++i) xalt[i] = w[N + i];
    *cauchy = csave;
  }
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    xnew_m[i] = xnew[i];
    xalt_m[i] = xalt[i];
  }
}


// ---------------------------------------------------------------- UPDATE (bobyqa_dev.h bq_update)
// W1 = w[1..npt] (lanes 0..npt-1), W2 = w[npt+1..2npt]: update writes w[npt+1..npt+n] (lanes 0..n-1).
BQL_HD void update(V (&BM)[N], V (&ZM)[NPTM], V& VL, double beta, double denom, int knew, V& W1, V& W2) {
  const double one = 1.0, zero = 0.0;
  const int kn = knew - 1;
  double ztest = zero, temp, tempa, tempb, alpha, tau;
  {
    // Powell's max over zmat in (k, j) order.  Without NaNs the max does not depend on the order, so
    // each lane folds its row and the rows are folded in k order; a NaN keeps the element order.
    const unsigned long long nan =
        ballot([&](int L) { return L < NPT && (ZM[0][L] != ZM[0][L] || ZM[1][L] != ZM[1][L] || ZM[2][L] != ZM[2][L]); });
    if (nan == 0ull) {
      V RM;
      par([&](int L) { RM[L] = bq_max(bq_max(fabs(ZM[0][L]), fabs(ZM[1][L])), fabs(ZM[2][L])); });
#pragma unroll
      for (int k = 0; k < NPT; ++k) ztest = bq_max(ztest, bc(RM, k));
    } else {
#pragma unroll
      for (int k = 0; k < NPT; ++k)
#pragma unroll
        for (int j = 0; j < NPTM; ++j) ztest = bq_max(ztest, fabs(bc(ZM[j], k)));
    }
  }
  ztest *= 1e-20;
#pragma unroll
  for (int j = 2; j <= NPTM; ++j) {
    const double zj = bc(ZM[j - 1], kn);
    if (fabs(zj) > ztest) {
      const double d1 = bc(ZM[0], kn), d2 = zj;
      temp = sqrt(d1 * d1 + d2 * d2);
      tempa = d1 / temp;
      tempb = d2 / temp;
      par([&](int L) {
        if (L < NPT) {
          const double t = tempa * ZM[0][L] + tempb * ZM[j - 1][L];
          ZM[j - 1][L] = tempa * ZM[j - 1][L] - tempb * ZM[0][L];
          ZM[0][L] = t;
        }
      });
    }
    put(ZM[j - 1], kn, zero);
  }
  const double zk1 = bc(ZM[0], kn);
  par([&](int L) {
    if (L < NPT) W1[L] = zk1 * ZM[0][L];
  });
  alpha = bc(W1, kn);
  tau = bc(VL, kn);
  put(VL, kn, tau - one);
  temp = sqrt(denom);
  tempb = zk1 / temp;
  tempa = tau / temp;
  par([&](int L) {
    if (L < NPT) ZM[0][L] = tempa * ZM[0][L] - tempb * VL[L];
  });
  double wj[N + 1];
#pragma unroll
  for (int j = 1; j <= N; ++j) {
    const int jp = NPT + j;
    wj[j] = bc(BM[j - 1], kn);
    put(W2, j - 1, wj[j]);
    const double vjp = bc(VL, jp - 1);
    tempa = (alpha * vjp - tau * wj[j]) / denom;
    tempb = (-beta * wj[j] - tau * vjp) / denom;
    // rows 1..jp of column j; w[i] is W1 for i <= npt and w[npt+j'] = wj[j'] above
    par([&](int L) {
      if (L < jp) {
        double wi = W1[L];
#pragma unroll
        for (int jj = 1; jj <= N; ++jj)
          if (L == NPT + jj - 1) wi = wj[jj];
        BM[j - 1][L] = BM[j - 1][L] + tempa * VL[L] + tempb * wi;
      }
    });
    // bmat[jp][i - npt] = bmat[i][j] for i = npt+1 .. jp (the symmetric part)
#pragma unroll
    for (int c = 1; c < j; ++c) put(BM[c - 1], jp - 1, bc(BM[j - 1], NPT + c - 1));
  }
}

// ---------------------------------------------------------------- the driver
// nlopt_optimize -> bobyqa() -> BOBYQB (+ PRELIM, RESCUE), bobyqa_dev.h bq_begin + bq_step_impl with
// every CALFUN a call of f(xe) (xe unscaled, wave-uniform).  Returns the NLopt result code; xout
// (unscaled) and *minf as bq_step leaves st.xout / st.minf; *nevals the evaluations made.
template <class F>
BQL_HD int bobyqa(BQL_AS BqlU& U, F&& fobj, const double* x0, const double* lb, const double* ub, double xtol_rel,
                  int maxeval, double* xout, double* minf_out, int* nevals_out, BqlProf& prof) {
  (void)prof;
  const double half = 0.5, one = 1.0, ten = 10.0, tenth = 0.1, two = 2.0, zero = 0.0;
  // ---- bq_begin
  BQL_AS double* const sc = U.sc;
  BQL_AS double *const x = U.x, *const xl = U.xl, *const xu = U.xu, *const xbase = U.xbase, *const xopt = U.xopt,
                       *const gopt = U.gopt, *const hq = U.hq, *const sl = U.sl, *const su = U.su, *const xnew = U.xnew,
                       *const xalt = U.xalt, *const d = U.d, *const gnew = U.gnew, *const pa1 = U.pa1,
                       *const pa2 = U.pa2, *const wu = U.wu, *const wn = U.wn;
  BQL_AS double &rhobeg = U.rhobeg, &rhoend = U.rhoend, &f = U.f, &fbeg = U.fbeg, &fsave = U.fsave,
                &xoptsq = U.xoptsq, &rho = U.rho, &delta = U.delta, &diffa = U.diffa, &diffb = U.diffb,
                &diffc = U.diffc, &dnorm = U.dnorm, &distsq = U.distsq, &dsq = U.dsq, &crvmin = U.crvmin,
                &adelt = U.adelt, &alpha = U.alpha, &cauchy = U.cauchy, &beta = U.beta, &denom = U.denom,
                &fopt = U.fopt, &vquad = U.vquad, &diff = U.diff, &ratio = U.ratio, &stepa = U.stepa,
                &stepb = U.stepb, &minf = U.minf, &rs_fbase = U.rs_fbase;
  BQL_AS int &nf = U.nf, &kopt = U.kopt, &kbase = U.kbase, &nresc = U.nresc, &ntrits = U.ntrits, &itest = U.itest,
             &nfsav = U.nfsav, &knew = U.knew, &nevals = U.nevals, &rc = U.rc;
  f = fbeg = fsave = xoptsq = rho = delta = diffa = diffb = diffc = dnorm = distsq = dsq = crvmin = adelt = alpha =
      cauchy = beta = denom = fopt = vquad = diff = ratio = stepa = stepb = minf = rs_fbase = 0.0;
  nf = 0;
  kopt = kbase = 1;
  nresc = ntrits = itest = nfsav = knew = nevals = 0;
  rc = BQR_SUCCESS;
  V XP[N], FV, PQ, ZM[NPTM], BM[N], VL, W1, W2, W3, PID;
#pragma unroll
  for (int i = 0; i <= N; ++i) {
    x[i] = xl[i] = xu[i] = xbase[i] = xopt[i] = gopt[i] = sl[i] = su[i] = xnew[i] = xalt[i] = d[i] = gnew[i] = 0.0;
    pa1[i] = pa2[i] = wu[i] = wn[i] = sc[i] = 0.0;
  }
#pragma unroll
  for (int i = 0; i <= NH; ++i) hq[i] = 0.0;
  par([&](int L) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      XP[j][L] = 0.0;
      BM[j][L] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < NPTM; ++j) ZM[j][L] = 0.0;
    FV[L] = PQ[L] = VL[L] = W1[L] = W2[L] = W3[L] = PID[L] = 0.0;
  });
  {
    double dxs[N];
#pragma unroll
    for (int i = 0; i < N; ++i) dxs[i] = bq_default_step(x0[i], lb[i], ub[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) sc[i] = 1.0;
    int i = 1;
    for (; i < N && dxs[i] == dxs[i - 1]; ++i) {
    }
    if (i < N)
      for (i = 1; i < N; ++i) sc[i] = dxs[i] / dxs[0];
    for (i = 0; i < N; ++i) {
      x[i + 1] = x0[i] / sc[i];
      xl[i + 1] = lb[i] / sc[i];
      xu[i + 1] = ub[i] / sc[i];
    }
    rhobeg = fabs(dxs[0] / sc[0]);
    rhoend = xtol_rel * rhobeg;
  }
#pragma unroll
  for (int j = 1; j <= N; ++j) {
    const double temp = xu[j] - xl[j];
    if (temp < rhobeg + rhobeg) {
#pragma unroll
      for (int i = 0; i < N; ++i) xout[i] = x0[i];
      *minf_out = 0.0;
      *nevals_out = 0;
      return BQR_INVALID_ARGS;
    }
    sl[j] = xl[j] - x[j];
    su[j] = xu[j] - x[j];
    if (sl[j] >= -rhobeg) {
      if (sl[j] >= 0.0) {
        x[j] = xl[j];
        sl[j] = 0.0;
        su[j] = temp;
      } else {
        x[j] = xl[j] + rhobeg;
        sl[j] = -rhobeg;
        su[j] = bq_max(xu[j] - x[j], rhobeg);
      }
    } else if (su[j] <= rhobeg) {
      if (su[j] <= 0.0) {
        x[j] = xu[j];
        sl[j] = -temp;
        su[j] = 0.0;
      } else {
        x[j] = xu[j] - rhobeg;
        sl[j] = bq_min(xl[j] - x[j], -rhobeg);
        su[j] = rhobeg;
      }
    }
  }
  // an evaluation at the rescaled point P (1-based): nlopt's rescale_fun unscales it
  auto calfun = [&](const BQL_AS double* P) -> double {
    double xe[N];
#pragma unroll
    for (int i = 0; i < N; ++i) xe[i] = P[i + 1] * sc[i];
    ++nevals;
    BQL_FENCE();
    const double fv = fobj(xe);
    BQL_FENCE();
    return fv;
  };
  double temp, sum, suma, sumb, bsum, dx, delsq, scaden, biglsq, den, errbig, frhosq, bdtol, bdtest, curv, fracsq, sumpq,
      pqold, gqsq, gisq, dist, densav;
  int ih, ksav;
  // ---- PRELIM
#pragma unroll
  for (int j = 1; j <= N; ++j) xbase[j] = x[j];
  nf = 0;
  kopt = 1;
  {
    const double rhosq = rhobeg * rhobeg;
    for (;;) {
      const int nfm = nf, nfx = nf - N;
      ++nf;
      if (nfm <= 2 * N) {
        if (nfm >= 1 && nfm <= N) {
          stepa = rhobeg;
          if (getp(su, nfm) == zero) stepa = -stepa;
          put3(XP, nfm - 1, nf - 1, stepa);
        } else if (nfm > N) {
          stepa = bc3(XP, nfx - 1, nf - N - 1);
          stepb = -rhobeg;
          if (getp(sl, nfx) == zero) stepb = bq_min(two * rhobeg, getp(su, nfx));
          if (getp(su, nfx) == zero) stepb = bq_max(-two * rhobeg, getp(sl, nfx));
          put3(XP, nfx - 1, nf - 1, stepb);
        }
      }
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        const double xp = bc(XP[j - 1], nf - 1);
        x[j] = bq_min(bq_max(xl[j], xbase[j] + xp), xu[j]);
        if (xp == sl[j]) x[j] = xl[j];
        if (xp == su[j]) x[j] = xu[j];
      }
      f = calfun(x);
      put(FV, nf - 1, f);
      if (nf == 1) {
        fbeg = f;
        kopt = 1;
      } else if (f < bc(FV, kopt - 1)) {
        kopt = nf;
      }
      if (nf <= 2 * N + 1) {
        if (nf >= 2 && nf <= N + 1) {
          setp(gopt, nfm, (f - fbeg) / stepa);
          if (NPT < nf + N) {
            put3(BM, nfm - 1, 0, -one / stepa);
            put3(BM, nfm - 1, nf - 1, one / stepa);
            put3(BM, nfm - 1, NPT + nfm - 1, -half * rhosq);
          }
        } else if (nf >= N + 2) {
          ih = nfx * (nfx + 1) / 2;
          temp = (f - fbeg) / stepb;
          diff = stepb - stepa;
          hq[ih] = two * (temp - getp(gopt, nfx)) / diff;
          setp(gopt, nfx, (getp(gopt, nfx) * stepb - temp * stepa) / diff);
          if (stepa * stepb < zero) {
            const double fo = bc(FV, nf - N - 1);
            if (f < fo) {
              put(FV, nf - 1, fo);
              put(FV, nf - N - 1, f);
              if (kopt == nf) kopt = nf - N;
              put3(XP, nfx - 1, nf - N - 1, stepb);
              put3(XP, nfx - 1, nf - 1, stepa);
            }
          }
          const double b1 = -(stepa + stepb) / (stepa * stepb);
          const double bn = -half / bc3(XP, nfx - 1, nf - N - 1);
          put3(BM, nfx - 1, 0, b1);
          put3(BM, nfx - 1, nf - 1, bn);
          put3(BM, nfx - 1, nf - N - 1, -b1 - bn);
          const double z1 = sqrt(two) / (stepa * stepb);
          const double zn = sqrt(half) / rhosq;
          put3(ZM, nfx - 1, 0, z1);
          put3(ZM, nfx - 1, nf - 1, zn);
          put3(ZM, nfx - 1, nf - N - 1, -z1 - zn);
        }
      }
      if (maxeval > 0 && nevals >= maxeval) {
        rc = BQR_MAXEVAL;
        break;
      }
      if (nf >= NPT) break;
    }
  }
  xoptsq = zero;
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    xopt[i] = bc(XP[i - 1], kopt - 1);
    xoptsq += xopt[i] * xopt[i];
  }
  fsave = bc(FV, 0);
  if (rc != BQR_SUCCESS) goto L720;
  kbase = 1;
  rho = rhobeg;
  delta = rho;
  nresc = nf;
  ntrits = 0;
  diffa = zero;
  diffb = zero;
  diffc = zero;
  ratio = zero;
  itest = 0;
  nfsav = nf;
  knew = 0;
L20:
  if (kopt != kbase) {
    ih = 0;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
#pragma unroll
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) gopt[j] += hq[ih] * xopt[i];
        gopt[i] += hq[ih] * xopt[j];
      }
    }
    if (nf > NPT) {
      V G0, G1, G2;
      par([&](int L) {
        double t = zero;
        t += XP[0][L] * xopt[1];
        t += XP[1][L] * xopt[2];
        t += XP[2][L] * xopt[3];
        t = PQ[L] * t;
        G0[L] = t * XP[0][L];
        G1[L] = t * XP[1][L];
        G2[L] = t * XP[2][L];
      });
      gopt[1] = osum(gopt[1], G0, NPT);
      gopt[2] = osum(gopt[2], G1, NPT);
      gopt[3] = osum(gopt[3], G2, NPT);
    }
  }
L60:
  BQL_FENCE();
  {
    BQL_T0(t0);
    trsbox(XP, PQ, xopt, gopt, hq, sl, su, delta, xnew, d, gnew, &dsq, &crvmin);
    BQL_T1(0, t0);
  }
  BQL_FENCE();
  dnorm = bq_min(delta, sqrt(dsq));
  if (dnorm < half * rho) {
    ntrits = -1;
    temp = ten * rho;
    distsq = temp * temp;
    if (nf <= nfsav + 2) goto L650;
    errbig = bq_max(bq_max(diffa, diffb), diffc);
    frhosq = rho * .125 * rho;
    if (crvmin > zero && errbig > frhosq * crvmin) goto L650;
    bdtol = errbig / rho;
    {
      // (goto L650 at the first j that passes both tests: a flag, so the loop unrolls)
      bool hit = false;
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        if (!hit) {
          bdtest = bdtol;
          if (xnew[j] == sl[j]) bdtest = gnew[j];
          if (xnew[j] == su[j]) bdtest = -gnew[j];
          if (bdtest < bdtol) {
            curv = hq[(j + j * j) / 2];
            V CT;
            par([&](int L) { CT[L] = PQ[L] * (XP[j - 1][L] * XP[j - 1][L]); });
            curv = osum(curv, CT, NPT);
            bdtest += half * curv * rho;
            if (bdtest < bdtol) hit = true;
          }
        }
      }
      if (hit) goto L650;
    }
    goto L680;
  }
  ++ntrits;
L90:
  if (dsq <= xoptsq * .001) {
    BQL_HIT(1);
    fracsq = xoptsq * .25;
    sumpq = osum(zero, PQ, NPT);
    // per k: w[npt+k] = sum, and the rank-two terms of bmat's lower block
    V SM, TV;
    par([&](int L) {
      double sm = -half * xoptsq;
#pragma unroll
      for (int i = 1; i <= N; ++i) sm += XP[i - 1][L] * xopt[i];
      SM[L] = sm;
      TV[L] = fracsq - half * sm;
    });
    par([&](int L) {
      if (L < NPT) W2[L] = SM[L];
    });
    // bmat[npt+i][j] += w[i] vlag[j] + vlag[i] w[j] over k, w[i] = bmat[k][i], vlag[i] = sum xpt[k][i] + temp xopt[i]
#pragma unroll
    for (int i = 1; i <= N; ++i) {
#pragma unroll
      for (int j = 1; j <= i; ++j) {
        V PA, PB;
        par([&](int L) {
          const double vj = SM[L] * XP[j - 1][L] + TV[L] * xopt[j];
          const double vi = SM[L] * XP[i - 1][L] + TV[L] * xopt[i];
          PA[L] = BM[i - 1][L] * vj;
          PB[L] = vi * BM[j - 1][L];
        });
        put(BM[j - 1], NPT + i - 1, osum2(bc(BM[j - 1], NPT + i - 1), PA, PB, NPT));
      }
    }
    // Powell leaves w[1..n] = bmat[npt][.] and vlag[1..n] from k = npt
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      wu[i] = bc(BM[i - 1], NPT - 1);
      put(VL, i - 1, bc(SM, NPT - 1) * bc(XP[i - 1], NPT - 1) + bc(TV, NPT - 1) * xopt[i]);
    }
#pragma unroll
    for (int jj = 1; jj <= NPTM; ++jj) {
      V VZ;
      par([&](int L) { VZ[L] = W2[L] * ZM[jj - 1][L]; });
      const double sumz = osum(zero, ZM[jj - 1], NPT);
      const double sumw = osum(zero, VZ, NPT);
      par([&](int L) {
        if (L < NPT) VL[L] = VZ[L];
      });
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        V PV;
        par([&](int L) { PV[L] = VL[L] * XP[j - 1][L]; });
        sum = (fracsq * sumz - half * sumw) * xopt[j];
        sum = osum(sum, PV, NPT);
        wu[j] = sum;
        par([&](int L) {
          if (L < NPT) BM[j - 1][L] += sum * ZM[jj - 1][L];
        });
      }
#pragma unroll
      for (int i = 1; i <= N; ++i) {
        const int ip = i + NPT;
        temp = wu[i];
#pragma unroll
        for (int j = 1; j <= i; ++j) put(BM[j - 1], ip - 1, bc(BM[j - 1], ip - 1) + temp * wu[j]);
      }
    }
    ih = 0;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      V PX;
      par([&](int L) { PX[L] = PQ[L] * XP[j - 1][L]; });
      wu[j] = -half * sumpq * xopt[j];
      wu[j] = osum(wu[j], PX, NPT);
      const double xj = xopt[j];
      par([&](int L) {
        if (L < NPT) XP[j - 1][L] -= xj;
      });
#pragma unroll
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] = hq[ih] + wu[i] * xopt[j] + xopt[i] * wu[j];
        put(BM[j - 1], NPT + i - 1, bc(BM[i - 1], NPT + j - 1));
      }
    }
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      xbase[i] += xopt[i];
      xnew[i] -= xopt[i];
      sl[i] -= xopt[i];
      su[i] -= xopt[i];
      xopt[i] = zero;
    }
    xoptsq = zero;
  }
  if (ntrits == 0) goto L210;
  goto L230;

L190:  // ---- RESCUE
  BQL_HIT(0);
  nfsav = nf;
  kbase = kopt;
  {
    const double sfrac = half / (double)NP;
    double winc = zero, bet2 = 0, den2 = 0, dsqmin, vlmxsq;
    int nrem, kold, kn;
    {
      V DS;
      par([&](int L) {
        double ds = zero;
#pragma unroll
        for (int j = 1; j <= N; ++j) {
          if (L < NPT) XP[j - 1][L] -= xopt[j];
          ds += XP[j - 1][L] * XP[j - 1][L];
        }
        DS[L] = ds;
        if (L < NPT) {
          W3[L] = ds;
#pragma unroll
          for (int j = 0; j < NPTM; ++j) ZM[j][L] = zero;
        }
      });
      sumpq = osum(zero, PQ, NPT);
#pragma unroll
      for (int k = 0; k < NPT; ++k) winc = bq_max(winc, bc(DS, k));
      distsq = bc(DS, NPT - 1);
    }
    ih = 0;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      V PX;
      par([&](int L) { PX[L] = PQ[L] * XP[j - 1][L]; });
      wu[j] = half * sumpq * xopt[j];
      wu[j] = osum(wu[j], PX, NPT);
#pragma unroll
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] = hq[ih] + wu[i] * xopt[j] + wu[j] * xopt[i];
      }
    }
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      xbase[j] += xopt[j];
      sl[j] -= xopt[j];
      su[j] -= xopt[j];
      xopt[j] = zero;
      pa1[j] = bq_min(delta, su[j]);
      pa2[j] = bq_max(-delta, sl[j]);
      if (pa1[j] + pa2[j] < zero) {
        temp = pa1[j];
        pa1[j] = pa2[j];
        pa2[j] = temp;
      }
      if (fabs(pa2[j]) < half * fabs(pa1[j])) pa2[j] = half * pa1[j];
    }
    par([&](int L) {
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (L < NDIM) BM[j][L] = zero;
    });
    rs_fbase = bc(FV, kopt - 1);
    put(PID, 0, sfrac);
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      const int jp = j + 1, jpn = jp + N;
      put(PID, jp - 1, (double)j + sfrac);
      if (jpn <= NPT) {
        put(PID, jpn - 1, (double)j / (double)NP + sfrac);
        temp = one / (pa1[j] - pa2[j]);
        const double bjp = -temp + one / pa1[j];
        const double bjpn = temp + one / pa2[j];
        put(BM[j - 1], jp - 1, bjp);
        put(BM[j - 1], jpn - 1, bjpn);
        put(BM[j - 1], 0, -bjp - bjpn);
        const double z1 = sqrt(2.) / fabs(pa1[j] * pa2[j]);
        put(ZM[j - 1], 0, z1);
        put(ZM[j - 1], jp - 1, z1 * pa2[j] * temp);
        put(ZM[j - 1], jpn - 1, -z1 * pa1[j] * temp);
      } else {
        put(BM[j - 1], 0, -one / pa1[j]);
        put(BM[j - 1], jp - 1, one / pa1[j]);
        put(BM[j - 1], j + NPT - 1, -half * (pa1[j] * pa1[j]));
      }
    }
    nrem = NPT;
    kold = 1;
    kn = kopt;
  R80:
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double a = bc(BM[j], kold - 1), b = bc(BM[j], kn - 1);
      put(BM[j], kold - 1, b);
      put(BM[j], kn - 1, a);
    }
#pragma unroll
    for (int j = 0; j < NPTM; ++j) {
      const double a = bc(ZM[j], kold - 1), b = bc(ZM[j], kn - 1);
      put(ZM[j], kold - 1, b);
      put(ZM[j], kn - 1, a);
    }
    put(PID, kold - 1, bc(PID, kn - 1));
    put(PID, kn - 1, zero);
    put(W3, kn - 1, zero);
    --nrem;
    if (kn != kopt) {
      const double a = bc(VL, kold - 1), b = bc(VL, kn - 1);
      put(VL, kold - 1, b);
      put(VL, kn - 1, a);
      BQL_FENCE();
      update(BM, ZM, VL, bet2, den2, kn, W1, W2);
      BQL_FENCE();
#pragma unroll
      for (int j = 1; j <= N; ++j) wn[j] = bc(W2, j - 1);
      if (nrem == 0) goto R350;
      par([&](int L) {
        if (L < NPT) W3[L] = fabs(W3[L]);
      });
    }
  R120:
    dsqmin = zero;
#pragma unroll
    for (int k = 1; k <= NPT; ++k) {
      const double wk = bc(W3, k - 1);
      if (wk > zero) {
        if (dsqmin == zero || wk < dsqmin) {
          kn = k;
          dsqmin = wk;
        }
      }
    }
    if (dsqmin == zero) goto R260;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      wn[j] = bc(XP[j - 1], kn - 1);
      put(W2, j - 1, wn[j]);
    }
    {
      V DN, ZH;
      const int kop = kopt;
      par([&](int L) {
        const int k = L + 1;
        double sm = zero;
        const double pid = PID[L];
        if (k == kop) {
        } else if (pid == zero) {
#pragma unroll
          for (int j = 1; j <= N; ++j) sm += wn[j] * XP[j - 1][L];
        } else {
          const int ip = (int)pid;
          if (ip > 0) sm = getp(wn, ip) * getp(pa1, ip);
          const int iq = (int)((double)NP * pid - (double)(ip * NP));
          if (iq > 0) {
            const double pq2 = (ip == 0) ? getp(pa2, iq) : getp(pa1, iq);
            sm += getp(wn, iq) * pq2;
          }
        }
        if (L < NPT) W1[L] = half * sm * sm;
        double v = zero;
#pragma unroll
        for (int j = 1; j <= N; ++j) v += BM[j - 1][L] * wn[j];
        if (L < NPT) VL[L] = v;
        double hd = zero;
#pragma unroll
        for (int j = 0; j < NPTM; ++j) hd += ZM[j][L] * ZM[j][L];
        ZH[L] = hd;
        DN[L] = zero;
      });
      bet2 = zero;
#pragma unroll
      for (int j = 1; j <= NPTM; ++j) {
        V PZ;
        par([&](int L) { PZ[L] = ZM[j - 1][L] * W1[L]; });
        sum = osum(zero, PZ, NPT);
        bet2 -= sum * sum;
        par([&](int L) {
          if (L < NPT) VL[L] += sum * ZM[j - 1][L];
        });
      }
      bsum = zero;
      distsq = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        V PB;
        par([&](int L) { PB[L] = BM[j - 1][L] * W1[L]; });
        sum = osum(zero, PB, NPT);
        const int jp = j + NPT;
        bsum += sum * wn[j];
#pragma unroll
        for (int ipp = NPT + 1; ipp <= NDIM; ++ipp) sum += bc(BM[j - 1], ipp - 1) * wn[ipp - NPT];
        bsum += sum * wn[j];
        put(VL, jp - 1, sum);
        distsq += wn[j] * wn[j];
      }
      bet2 = half * distsq * distsq + bet2 - bsum;
      put(VL, kopt - 1, bc(VL, kopt - 1) + one);
      den2 = zero;
      vlmxsq = zero;
      par([&](int L) { DN[L] = bet2 * ZH[L] + VL[L] * VL[L]; });
#pragma unroll
      for (int k = 1; k <= NPT; ++k) {
        const double vk = bc(VL, k - 1);
        if (bc(PID, k - 1) != zero) {
          const double den_ = bc(DN, k - 1);
          if (den_ > den2) {
            kold = k;
            den2 = den_;
          }
        }
        vlmxsq = bq_max(vlmxsq, vk * vk);
      }
    }
    if (den2 <= vlmxsq * .01) {
      BQL_HIT(4);
      put(W3, kn - 1, -bc(W3, kn - 1) - winc);
      goto R120;
    }
    goto R80;
  }
R260:
#pragma unroll
  for (int kpt = 1; kpt <= NPT; ++kpt) {
    const double pidk = bc(PID, kpt - 1);
    if (pidk == zero) continue;
    BQL_HIT(5);
    if (maxeval > 0 && nevals >= maxeval) {
      nf = -1;
      goto R350;
    }
    ih = 0;
    const double pqk = bc(PQ, kpt - 1);
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      wu[j] = bc(XP[j - 1], kpt - 1);
      put(XP[j - 1], kpt - 1, zero);
      temp = pqk * wu[j];
#pragma unroll
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] += temp * wu[i];
      }
    }
    put(PQ, kpt - 1, zero);
    const int ip = (int)pidk;
    const int iq = (int)((double)NP * pidk - (double)(ip * NP));
    int ihp = 0, ihq;
    double xp = 0, xq = 0, vq;
    if (ip > 0) {
      xp = getp(pa1, ip);
      put3(XP, ip - 1, kpt - 1, xp);
    }
    if (iq > 0) {
      xq = getp(pa1, iq);
      if (ip == 0) xq = getp(pa2, iq);
      put3(XP, iq - 1, kpt - 1, xq);
    }
    vq = rs_fbase;
    if (ip > 0) {
      ihp = (ip + ip * ip) / 2;
      vq += xp * (getp(gopt, ip) + half * xp * hq[ihp]);
    }
    if (iq > 0) {
      ihq = (iq + iq * iq) / 2;
      vq += xq * (getp(gopt, iq) + half * xq * hq[ihq]);
      if (ip > 0) {
        const int iw = (ihp > ihq ? ihp : ihq) - (ip > iq ? ip - iq : iq - ip);
        vq += xp * xq * hq[iw];
      }
    }
    {
      V PT;
      par([&](int L) {
        double t = zero;
        if (ip > 0) {
          double xk = XP[0][L];
          if (ip == 2) xk = XP[1][L];
          if (ip == 3) xk = XP[2][L];
          t += xp * xk;
        }
        if (iq > 0) {
          double xk = XP[0][L];
          if (iq == 2) xk = XP[1][L];
          if (iq == 3) xk = XP[2][L];
          t += xq * xk;
        }
        PT[L] = half * PQ[L] * t * t;
      });
      vq = osum(vq, PT, NPT);
    }
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      const double xk = bc(XP[i - 1], kpt - 1);
      wu[i] = bq_min(bq_max(xl[i], xbase[i] + xk), xu[i]);
      if (xk == sl[i]) wu[i] = xl[i];
      if (xk == su[i]) wu[i] = xu[i];
    }
    ++nf;
    f = calfun(wu);
    put(FV, kpt - 1, f);
    if (f < bc(FV, kopt - 1)) kopt = kpt;
    diff = f - vq;
#pragma unroll
    for (int i = 1; i <= N; ++i) gopt[i] += diff * bc(BM[i - 1], kpt - 1);
    {
      const double zk0 = bc(ZM[0], kpt - 1), zk1 = bc(ZM[1], kpt - 1), zk2 = bc(ZM[2], kpt - 1);
      V TT;
      par([&](int L) {
        double sm = zero;
        sm += ZM[0][L] * zk0;
        sm += ZM[1][L] * zk1;
        sm += ZM[2][L] * zk2;
        const double t = diff * sm;
        TT[L] = t;
        if (L < NPT && PID[L] == zero) PQ[L] += t;
      });
#pragma unroll
      for (int k = 1; k <= NPT; ++k) {
        const double pid = bc(PID, k - 1);
        if (pid == zero) continue;
        const double t = bc(TT, k - 1);
        const int ipk = (int)pid;
        const int iqk = (int)((double)NP * pid - (double)(ipk * NP));
        const int ihqk = (iqk * iqk + iqk) / 2;
        if (ipk == 0) {
          const double a2 = getp(pa2, iqk);
          hq[ihqk] = hq[ihqk] + t * (a2 * a2);
        } else {
          const int ihpk = (ipk * ipk + ipk) / 2;
          const double a1 = getp(pa1, ipk);
          hq[ihpk] = hq[ihpk] + t * (a1 * a1);
          if (iqk > 0) {
            const double a1q = getp(pa1, iqk);
            hq[ihqk] = hq[ihqk] + t * (a1q * a1q);
            const int iw = (ihpk > ihqk ? ihpk : ihqk) - (iqk > ipk ? iqk - ipk : ipk - iqk);
            hq[iw] = hq[iw] + t * a1 * a1q;
          }
        }
      }
    }
    put(PID, kpt - 1, zero);
  }
R350:
  xoptsq = zero;
  if (kopt != kbase) {
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      xopt[i] = bc(XP[i - 1], kopt - 1);
      xoptsq += xopt[i] * xopt[i];
    }
  }
  if (nf < 0) {
    nf = maxeval;
    rc = BQR_MAXEVAL;
    goto L720;
  }
  nresc = nf;
  if (nfsav < nf) {
    nfsav = nf;
    goto L20;
  }
  if (ntrits > 0) goto L60;
L210:
  BQL_FENCE();
  {
    BQL_T0(t0);
    altmov(XP, xopt, BM, ZM, sl, su, kopt, knew, adelt, xnew, xalt, &alpha, &cauchy);
    BQL_T1(1, t0);
  }
  BQL_FENCE();
#pragma unroll
  for (int i = 1; i <= N; ++i) d[i] = xnew[i] - xopt[i];
L230:
  {
    par([&](int L) {
      double sa = zero, sb = zero, sm = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        sa += XP[j - 1][L] * d[j];
        sb += XP[j - 1][L] * xopt[j];
        sm += BM[j - 1][L] * d[j];
      }
      if (L < NPT) {
        W1[L] = sa * (half * sa + sb);
        VL[L] = sm;
        W2[L] = sa;
      }
    });
    beta = zero;
#pragma unroll
    for (int jj = 1; jj <= NPTM; ++jj) {
      V PZ;
      par([&](int L) { PZ[L] = ZM[jj - 1][L] * W1[L]; });
      sum = osum(zero, PZ, NPT);
      beta -= sum * sum;
      par([&](int L) {
        if (L < NPT) VL[L] += sum * ZM[jj - 1][L];
      });
    }
    dsq = zero;
    bsum = zero;
    dx = zero;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      dsq += d[j] * d[j];
      V PB;
      par([&](int L) { PB[L] = W1[L] * BM[j - 1][L]; });
      sum = osum(zero, PB, NPT);
      bsum += sum * d[j];
      const int jp = NPT + j;
#pragma unroll
      for (int i = 1; i <= N; ++i) sum += bc(BM[i - 1], jp - 1) * d[i];
      put(VL, jp - 1, sum);
      bsum += sum * d[j];
      dx += d[j] * xopt[j];
    }
    beta = dx * dx + dsq * (xoptsq + dx + dx + half * dsq) + beta - bsum;
    put(VL, kopt - 1, bc(VL, kopt - 1) + one);
  }
  if (ntrits == 0) {
    const double vk = bc(VL, knew - 1);
    denom = vk * vk + alpha * beta;
    if (denom < cauchy && cauchy > zero) {
      BQL_HIT(3);
#pragma unroll
      for (int i = 1; i <= N; ++i) {
        xnew[i] = xalt[i];
        d[i] = xnew[i] - xopt[i];
      }
      cauchy = zero;
      goto L230;
    }
    if (denom <= half * (vk * vk)) {
      if (nf > nresc) goto L190;
      BQL_HIT(9);
      rc = BQR_ROUNDOFF;
      goto L720;
    }
  } else {
    delsq = delta * delta;
    scaden = zero;
    biglsq = zero;
    knew = 0;
    V DEN, DN, DST, TVL;
    par([&](int L) {
      double hd = zero;
#pragma unroll
      for (int jj = 0; jj < NPTM; ++jj) hd += ZM[jj][L] * ZM[jj][L];
      const double dn = beta * hd + VL[L] * VL[L];
      double ds = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        const double t = XP[j - 1][L] - xopt[j];
        ds += t * t;
      }
      double t = ds / delsq;
      t = bq_max(one, t * t);
      DEN[L] = t * dn;
      DN[L] = dn;
      DST[L] = ds;
      TVL[L] = t * (VL[L] * VL[L]);
    });
#pragma unroll
    for (int k = 1; k <= NPT; ++k) {
      if (k == kopt) continue;
      const double td = bc(DEN, k - 1);
      distsq = bc(DST, k - 1);
      if (td > scaden) {
        scaden = td;
        knew = k;
        denom = bc(DN, k - 1);
      }
      biglsq = bq_max(biglsq, bc(TVL, k - 1));
    }
    if (scaden <= half * biglsq) {
      if (nf > nresc) goto L190;
      rc = BQR_ROUNDOFF;
      goto L720;
    }
  }
L360:
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    x[i] = bq_min(bq_max(xl[i], xbase[i] + xnew[i]), xu[i]);
    if (xnew[i] == sl[i]) x[i] = xl[i];
    if (xnew[i] == su[i]) x[i] = xu[i];
  }
  if (maxeval > 0 && nevals >= maxeval) {
    rc = BQR_MAXEVAL;
    goto L720;
  }
  ++nf;
  f = calfun(x);
  if (ntrits == -1) {
    fsave = f;
    rc = BQR_XTOL;
    if (fsave < bc(FV, kopt - 1)) {
      BQL_HIT(10);
      minf = f;
#pragma unroll
      for (int i = 0; i < N; ++i) xout[i] = x[i + 1] * sc[i];
      *minf_out = minf;
      *nevals_out = nevals;
      return rc;
    }
    goto L720;
  }
  fopt = bc(FV, kopt - 1);
  vquad = zero;
  ih = 0;
#pragma unroll
  for (int j = 1; j <= N; ++j) {
    vquad += d[j] * gopt[j];
#pragma unroll
    for (int i = 1; i <= j; ++i) {
      ++ih;
      temp = d[i] * d[j];
      if (i == j) temp = half * temp;
      vquad += hq[ih] * temp;
    }
  }
  {
    V PV;
    par([&](int L) { PV[L] = half * PQ[L] * (W2[L] * W2[L]); });
    vquad = osum(vquad, PV, NPT);
  }
  diff = f - fopt - vquad;
  diffc = diffb;
  diffb = diffa;
  diffa = fabs(diff);
  if (dnorm > rho) nfsav = nf;
  if (ntrits > 0) {
    if (vquad >= zero) {
      rc = BQR_ROUNDOFF;
      goto L720;
    }
    ratio = (f - fopt) / vquad;
    if (ratio <= tenth) delta = bq_min(half * delta, dnorm);
    else if (ratio <= .7) delta = bq_max(half * delta, dnorm);
    else delta = bq_max(half * delta, dnorm + dnorm);
    if (delta <= rho * 1.5) delta = rho;
    if (f < fopt) {
      ksav = knew;
      densav = denom;
      delsq = delta * delta;
      scaden = zero;
      biglsq = zero;
      knew = 0;
      V DEN, DN, DST, TVL;
      par([&](int L) {
        double hd = zero;
#pragma unroll
        for (int jj = 0; jj < NPTM; ++jj) hd += ZM[jj][L] * ZM[jj][L];
        const double dn = beta * hd + VL[L] * VL[L];
        double ds = zero;
#pragma unroll
        for (int j = 1; j <= N; ++j) {
          const double t = XP[j - 1][L] - xnew[j];
          ds += t * t;
        }
        double t = ds / delsq;
        t = bq_max(one, t * t);
        DEN[L] = t * dn;
        DN[L] = dn;
        DST[L] = ds;
        TVL[L] = t * (VL[L] * VL[L]);
      });
#pragma unroll
      for (int k = 1; k <= NPT; ++k) {
        const double td = bc(DEN, k - 1);
        distsq = bc(DST, k - 1);
        if (td > scaden) {
          scaden = td;
          knew = k;
          denom = bc(DN, k - 1);
        }
        biglsq = bq_max(biglsq, bc(TVL, k - 1));
      }
      if (scaden <= half * biglsq) {
        BQL_HIT(6);
        knew = ksav;
        denom = densav;
      }
    }
  }
  BQL_FENCE();
  {
    BQL_T0(t0);
    update(BM, ZM, VL, beta, denom, knew, W1, W2);
    BQL_T1(2, t0);
  }
  BQL_FENCE();
  ih = 0;
  pqold = bc(PQ, knew - 1);
  put(PQ, knew - 1, zero);
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    temp = pqold * bc(XP[i - 1], knew - 1);
#pragma unroll
    for (int j = 1; j <= i; ++j) {
      ++ih;
      hq[ih] += temp * bc(XP[j - 1], knew - 1);
    }
  }
  {
    const double t0 = diff * bc(ZM[0], knew - 1), t1 = diff * bc(ZM[1], knew - 1), t2 = diff * bc(ZM[2], knew - 1);
    par([&](int L) {
      if (L < NPT) {
        PQ[L] += t0 * ZM[0][L];
        PQ[L] += t1 * ZM[1][L];
        PQ[L] += t2 * ZM[2][L];
      }
    });
  }
  put(FV, knew - 1, f);
#pragma unroll
  for (int i = 1; i <= N; ++i) {
    put(XP[i - 1], knew - 1, xnew[i]);
    wu[i] = bc(BM[i - 1], knew - 1);
  }
  {
    const double zk0 = bc(ZM[0], knew - 1), zk1 = bc(ZM[1], knew - 1), zk2 = bc(ZM[2], knew - 1);
    V G0, G1, G2;
    par([&](int L) {
      double sa = zero;
      sa += zk0 * ZM[0][L];
      sa += zk1 * ZM[1][L];
      sa += zk2 * ZM[2][L];
      double sb = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) sb += XP[j - 1][L] * xopt[j];
      const double t = sa * sb;
      G0[L] = t * XP[0][L];
      G1[L] = t * XP[1][L];
      G2[L] = t * XP[2][L];
    });
    wu[1] = osum(wu[1], G0, NPT);
    wu[2] = osum(wu[2], G1, NPT);
    wu[3] = osum(wu[3], G2, NPT);
  }
#pragma unroll
  for (int i = 1; i <= N; ++i) gopt[i] += diff * wu[i];
  if (f < fopt) {
    kopt = knew;
    xoptsq = zero;
    ih = 0;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      xopt[j] = xnew[j];
      xoptsq += xopt[j] * xopt[j];
#pragma unroll
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) gopt[j] += hq[ih] * d[i];
        gopt[i] += hq[ih] * d[j];
      }
    }
    V G0, G1, G2;
    par([&](int L) {
      double t = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) t += XP[j - 1][L] * d[j];
      t = PQ[L] * t;
      G0[L] = t * XP[0][L];
      G1[L] = t * XP[1][L];
      G2[L] = t * XP[2][L];
    });
    gopt[1] = osum(gopt[1], G0, NPT);
    gopt[2] = osum(gopt[2], G1, NPT);
    gopt[3] = osum(gopt[3], G2, NPT);
  }
  if (ntrits > 0) {
    const double fk = bc(FV, kopt - 1);
    par([&](int L) {
      if (L < NPT) {
        VL[L] = FV[L] - fk;
        W1[L] = zero;
      }
    });
#pragma unroll
    for (int j = 1; j <= NPTM; ++j) {
      V PZ;
      par([&](int L) { PZ[L] = ZM[j - 1][L] * VL[L]; });
      sum = osum(zero, PZ, NPT);
      par([&](int L) {
        if (L < NPT) W1[L] += sum * ZM[j - 1][L];
      });
    }
    par([&](int L) {
      double sm = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) sm += XP[j - 1][L] * xopt[j];
      if (L < NPT) {
        W2[L] = W1[L];
        W1[L] = sm * W1[L];
      }
    });
    gqsq = zero;
    gisq = zero;
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      V PA, PB;
      par([&](int L) {
        PA[L] = BM[i - 1][L] * VL[L];
        PB[L] = XP[i - 1][L] * W1[L];
      });
      sum = osum2(zero, PA, PB, NPT);
      if (xopt[i] == sl[i]) {
        temp = bq_min(zero, gopt[i]);
        gqsq += temp * temp;
        temp = bq_min(zero, sum);
        gisq += temp * temp;
      } else if (xopt[i] == su[i]) {
        temp = bq_max(zero, gopt[i]);
        gqsq += temp * temp;
        temp = bq_max(zero, sum);
        gisq += temp * temp;
      } else {
        gqsq += gopt[i] * gopt[i];
        gisq += sum * sum;
      }
      put(VL, NPT + i - 1, sum);
    }
    ++itest;
    if (gqsq < ten * gisq) itest = 0;
    if (itest >= 3) {
      BQL_HIT(2);
#pragma unroll
      for (int i = 1; i <= N; ++i) gopt[i] = bc(VL, NPT + i - 1);
      par([&](int L) {
        if (L < NPT) PQ[L] = W2[L];
      });
#pragma unroll
      for (int i = 1; i <= NH; ++i) hq[i] = zero;
      itest = 0;
    }
  }
  if (ntrits == 0) goto L60;
  if (f <= fopt + tenth * vquad) goto L60;
  {
    const double t1 = two * delta, t2 = ten * rho;
    distsq = bq_max(t1 * t1, t2 * t2);
  }
L650:
  knew = 0;
  {
    V DS;
    par([&](int L) {
      double sm = zero;
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        const double t = XP[j - 1][L] - xopt[j];
        sm += t * t;
      }
      DS[L] = sm;
    });
#pragma unroll
    for (int k = 1; k <= NPT; ++k) {
      const double sm = bc(DS, k - 1);
      if (sm > distsq) {
        knew = k;
        distsq = sm;
      }
    }
  }
  if (knew > 0) {
    dist = sqrt(distsq);
    if (ntrits == -1) {
      delta = bq_min(tenth * delta, half * dist);
      if (delta <= rho * 1.5) delta = rho;
    }
    ntrits = 0;
    adelt = bq_max(bq_min(tenth * dist, delta), rho);
    dsq = adelt * adelt;
    goto L90;
  }
  if (ntrits == -1) goto L680;
  if (ratio > zero) goto L60;
  if (bq_max(delta, dnorm) > rho) goto L60;
L680:
  if (rho > rhoend) {
    delta = half * rho;
    ratio = rho / rhoend;
    if (ratio <= 16.) rho = rhoend;
    else if (ratio <= 250.) rho = sqrt(ratio) * rhoend;
    else rho = tenth * rho;
    delta = bq_max(delta, rho);
    ntrits = 0;
    nfsav = nf;
    goto L60;
  }
  if (ntrits == -1) goto L360;
  BQL_HIT(8);
  rc = BQR_XTOL;
L720:
  if (bc(FV, kopt - 1) <= fsave) {
#pragma unroll
    for (int i = 1; i <= N; ++i) {
      x[i] = bq_min(bq_max(xl[i], xbase[i] + xopt[i]), xu[i]);
      if (xopt[i] == sl[i]) x[i] = xl[i];
      if (xopt[i] == su[i]) x[i] = xu[i];
    }
    f = bc(FV, kopt - 1);
  }
  minf = f;
#pragma unroll
  for (int i = 0; i < N; ++i) xout[i] = x[i + 1] * sc[i];
  *minf_out = minf;
  *nevals_out = nevals;
  return rc;
}

}  // namespace bql
}  // namespace pmvsdev
