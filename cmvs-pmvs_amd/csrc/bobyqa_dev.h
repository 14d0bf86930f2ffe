// bobyqa_dev.h -- BOBYQA (Powell, DAMTP 2009/NA06) with the NLopt 2.6.1 LN_BOBYQA driver
// semantics the reference relies on (reference source/pmvs/optim.cpp:615-647: n = 3,
// xtol_rel = 1e-7, maxeval = 1000, bounds +-23.99999 on the two angles), written as a
// REVERSE-COMMUNICATION state machine for the GPU:
//
//   BqState st;  bq_begin(st, x0, lb, ub, xtol_rel, maxeval);
//   while (bq_step(st, f) == BQ_NEED_F) f = objective(st.xeval);   // xeval is unscaled
//   result: st.rc (NLopt numbering), st.xout[0..2]
//
// All of Powell's locals live in BqState so the optimizer can yield at each CALFUN site
// (PRELIM, the main loop's label 360 and RESCUE) and resume.  One lane owns a BqState while
// the whole wavefront evaluates the objective (cmvs-pmvs_amd/csrc/pmvs_kernels.hip).  The
// arithmetic is Powell's, operation for operation; parity against the CPU oracle
// (oracle/bobyqa_oracle.h) is tested trajectory-for-trajectory in tests/test_gpu_bobyqa.py (device)
// and tests/test_bobyqa_host.py (this header compiled for the host).
#pragma once

#if defined(__HIPCC__)
#define BQ_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define BQ_HD inline
#endif
// The optimizer's state lives in LDS on the device (one BqState per chain, RefLds::bq).  Its big
// routines are called out of line with LDS-typed pointers (BQ_AS): 32-bit ds addressing with
// immediate offsets, and a register peak of the routine itself rather than of the whole inlined
// kernel (the inlined optimizer hoisted state into ~470 VGPR+AGPR and capped the refine kernel at
// one wavefront per SIMD).  Host builds (tests/csrc/bq_host.cpp) see plain pointers.
// -DBQ_PRIVATE (experiment builds): the state lives in per-lane private memory (scratch) instead,
// so a wavefront can hold 64 chains.
#if defined(__HIP_DEVICE_COMPILE__) && defined(BQ_PRIVATE)
#define BQ_AS __attribute__((address_space(5)))
#elif defined(__HIP_DEVICE_COMPILE__)
#define BQ_AS __attribute__((address_space(3)))
#else
#define BQ_AS
#endif
#if defined(__HIPCC__) && !defined(BQ_INLINE)
#define BQ_NI __host__ __device__ inline __attribute__((noinline))
#else
#define BQ_NI BQ_HD
#endif

#include <math.h>

// The routines' array arguments are distinct BqState members (no two alias), so ALTMOV's and
// UPDATE's are declared restrict: loads of read-only arrays (xpt, bmat, zmat, ...) may then stay in
// registers across the stores to xnew / xalt / w instead of being re-read from LDS after each of
// them (UPDATE: 132 -> 40 LDS reads, ALTMOV: 206 -> 127, gfx950 ISA).  TRSBOX keeps plain pointers:
// hoisting its xpt / hq / pq reads out of the Hessian-product loops overflows its 256 registers
// (944 B of scratch per lane) -- BQ_RST is empty unless -DBQ_TRSBOX_RESTRICT.
#if defined(BQ_NO_RESTRICT)
#define BQ_RS
#else
#define BQ_RS __restrict__
#endif
#if defined(BQ_TRSBOX_RESTRICT)
#define BQ_RST __restrict__
#else
#define BQ_RST
#endif

namespace pmvsdev {

// Diagnostic build only (-DBQ_PROFILE, tools/bq_profile.sh): wave-time spent in the optimizer's
// sub-steps, accumulated once per wavefront that executes the block.
#if defined(BQ_PROFILE) && defined(__HIPCC__)
__device__ unsigned long long bq_prof[8];
#endif
#if defined(BQ_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#define BQ_PT(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define BQ_PA(slot, v)                                                                 \
  do {                                                                                 \
    const unsigned long long _d = __builtin_amdgcn_s_memtime() - v;                    \
    if ((int)__lane_id() == (int)__builtin_ctzll(__ballot(1))) atomicAdd(&bq_prof[slot], _d); \
  } while (0)
#else
#define BQ_PT(v)
#define BQ_PA(slot, v)
#endif

enum { BQ_NEED_F = 1, BQ_DONE = 0 };
enum {
  BQR_SUCCESS = 1, BQR_XTOL = 4, BQR_MAXEVAL = 5, BQR_INVALID_ARGS = -2, BQR_ROUNDOFF = -4
};

constexpr int BQN = 3;
constexpr int BQNPT = 2 * BQN + 1;
constexpr int BQNP = BQN + 1;
constexpr int BQNPTM = BQNPT - BQNP;
constexpr int BQNDIM = BQNPT + BQN;
constexpr int BQNH = BQN * BQNP / 2;

BQ_HD double bq_min(double a, double b) { return (a <= b) ? a : b; }  // NLopt MIN2
BQ_HD double bq_max(double a, double b) { return (a >= b) ? a : b; }  // NLopt MAX2
// Run-time-indexed access to a small local array through selects over its constant positions, so
// the array stays in registers: a dynamic index (TRSBOX's xbdi[iact], ALTMOV's hcol[knew]) otherwise
// puts the whole array in scratch, and its hot loops then read scratch (global-memory latency).
template <int N>
BQ_HD double bq_get(const double (&a)[N], int i) {
  double r = a[0];
#pragma unroll
  for (int k = 1; k < N; ++k) r = (i == k) ? a[k] : r;
  return r;
}
template <int N>
BQ_HD void bq_set(double (&a)[N], int i, double v) {
#pragma unroll
  for (int k = 0; k < N; ++k) a[k] = (i == k) ? v : a[k];
}

struct BqState {
  // Powell's 1-based arrays stored without their unused row/column 0 (2216 -> 1736 bytes: the
  // state of a chain lives in LDS); bq_begin / bq_step_impl address them through 1-based aliases
  // (BQ_ALIASES).
  // problem (rescaled space)
  double x_[BQN], xl_[BQN], xu_[BQN], s[BQN];
  double rhobeg, rhoend;
  int maxeval, nevals;
  // BOBYQB arrays
  double xbase_[BQN], xpt_[BQNPT][BQN], fval_[BQNPT], xopt_[BQN], gopt_[BQN], hq_[BQNH], pq_[BQNPT],
      bmat_[BQNDIM][BQN], zmat_[BQNPT][BQNPTM], sl_[BQN], su_[BQN], xnew_[BQN], xalt_[BQN], d_[BQN],
      vlag_[BQNDIM], w_[BQNDIM + BQNPT];
  double gnew_[BQN];  // TRSBOX's GNEW (Powell's W(1..N) after TRSBOX)
  double ptsaux_[2][BQN], ptsid_[BQNPT];
  // BOBYQB scalars
  double f, fbeg, fsave, xoptsq, rho, delta, diffa, diffb, diffc, dnorm, distsq, dsq, crvmin,
      adelt, alpha, cauchy, beta, denom, fopt, vquad, diff, ratio, stepa, stepb;
  int nf, kopt, kbase, nresc, ntrits, itest, nfsav, knew;
  // PRELIM / RESCUE loop state kept across CALFUN
  int nfm, nfx, kpt, rs_ip, rs_iq;
  double rs_xp, rs_xq, rs_vq, rs_fbase;
  int rc;
  int resume;
  double xeval[BQN];  // unscaled point whose f is requested
  double xout[BQN];   // unscaled final point
  double minf;
};

// 1-based views of a BqState's arrays (Powell's indexing; element 0 / row 0 / column 0 are never
// touched), as the subroutines take them.
#define BQ_A1(name) BQ_AS double* const name = (st).name##_ - 1
#define BQ_A2(name, C) BQ_AS double(*const name)[C] = (BQ_AS double(*)[C])(&(st).name##_[0][0] - (C) - 1)
#define BQ_ALIASES(st)                                                                                         \
  BQ_A1(x); BQ_A1(xl); BQ_A1(xu); BQ_A1(xbase); BQ_A1(fval); BQ_A1(xopt); BQ_A1(gopt); BQ_A1(hq); BQ_A1(pq); \
  BQ_A1(sl); BQ_A1(su); BQ_A1(xnew); BQ_A1(xalt); BQ_A1(d); BQ_A1(vlag); BQ_A1(w); BQ_A1(gnew); BQ_A1(ptsid); \
  BQ_A2(xpt, BQN); BQ_A2(bmat, BQN); BQ_A2(zmat, BQNPTM); BQ_A2(ptsaux, BQN)

// ---------------------------------------------------------------- TRSBOX
// The small state arrays TRSBOX reads are copied into registers at entry (xopt, hq, pq, sl, su; xpt
// stays in LDS: with it the routine exceeds 256 registers) and d / gnew are kept there until the
// exit, so its loops run on registers instead of chains of dependent LDS round trips; the
// arithmetic is unchanged.
BQ_NI void bq_trsbox(const BQ_AS double (*BQ_RST xpt)[BQN], const BQ_AS double* BQ_RST xopt_m, const BQ_AS double* BQ_RST gopt,
                     const BQ_AS double* BQ_RST hq_m, const BQ_AS double* BQ_RST pq_m, const BQ_AS double* BQ_RST sl_m,
                     const BQ_AS double* BQ_RST su_m, double delta, BQ_AS double* BQ_RST xnew, BQ_AS double* BQ_RST d_m,
                     BQ_AS double* BQ_RST gnew_m, BQ_AS double* BQ_RST dsq_out, BQ_AS double* BQ_RST crvmin_out) {
  const double half = 0.5, one = 1.0, onemin = -1.0, zero = 0.0;
#if !defined(BQ_TRSBOX_LDS)
  double xopt[BQN + 1], hq[BQNH + 1], pq[BQNPT + 1], sl[BQN + 1], su[BQN + 1], d[BQN + 1], gnew[BQN + 1];
  for (int k = 1; k <= BQNPT; ++k) pq[k] = pq_m[k];
  for (int i = 1; i <= BQNH; ++i) hq[i] = hq_m[i];
  for (int i = 1; i <= BQN; ++i) {
    xopt[i] = xopt_m[i];
    sl[i] = sl_m[i];
    su[i] = su_m[i];
  }
#define BQ_D_AT(i) bq_get(d, i)
#else  // (experiment builds) every array in LDS
  const BQ_AS double *const xopt = xopt_m, *const hq = hq_m, *const pq = pq_m, *const sl = sl_m, *const su = su_m;
  BQ_AS double *const d = d_m, *const gnew = gnew_m;
#define BQ_D_AT(i) d[i]
#endif
  double xbdi[BQN + 1], s[BQN + 1], hs[BQN + 1], hred[BQN + 1];
  int iterc = 0, nact = 0, itermax = 0, itcsav = 0, iact = 0, isav = 0, iu = 0;
  double delsq, qred, crvmin, beta = 0, stepsq = 0, gredsq = 0, resid, ds, shs = 0, temp, blen = 0,
         stplen = 0, xsum, sdec, ggsav = 0, dredsq = 0, dredg = 0, sredg = 0, angbd = 0, tempa, tempb,
         ssq, xsav = 0, dhs = 0, dhd = 0, redmax, redsav, angt = 0, sth, rednew, rdprev = 0,
         rdnext = 0, cth;
  for (int i = 1; i <= BQN; ++i) {
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
  delsq = delta * delta;
  qred = zero;
  crvmin = onemin;
L20:
  beta = zero;
L30:
  stepsq = zero;
  for (int i = 1; i <= BQN; ++i) {
    if (xbdi[i] != zero) s[i] = zero;
    else if (beta == zero) s[i] = -gnew[i];
    else s[i] = beta * s[i] - gnew[i];
    stepsq += s[i] * s[i];
  }
  if (stepsq == zero) goto L190;
  if (beta == zero) {
    gredsq = stepsq;
    itermax = iterc + BQN - nact;
  }
  if (gredsq * delsq <= qred * 1e-4 * qred) goto L190;
  goto L210;
L50:
  resid = delsq;
  ds = zero;
  shs = zero;
  for (int i = 1; i <= BQN; ++i) {
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
  for (int i = 1; i <= BQN; ++i) {
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
    for (int i = 1; i <= BQN; ++i) {
      gnew[i] += stplen * hs[i];
      if (xbdi[i] == zero) gredsq += gnew[i] * gnew[i];
      d[i] += stplen * s[i];
    }
    sdec = bq_max(stplen * (ggsav - half * stplen * shs), zero);
    qred += sdec;
  }
  if (iact > 0) {
    ++nact;
    bq_set(xbdi, iact, bq_get(s, iact) < zero ? onemin : one);
    {
      const double di = BQ_D_AT(iact);
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
  if (nact >= BQN - 1) goto L190;
  dredsq = zero;
  dredg = zero;
  gredsq = zero;
  for (int i = 1; i <= BQN; ++i) {
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
  for (int i = 1; i <= BQN; ++i) {
    if (xbdi[i] == zero) s[i] = (dredg * d[i] - dredsq * gnew[i]) / temp;
    else s[i] = zero;
  }
  sredg = -temp;
  angbd = one;
  iact = 0;
  for (int i = 1; i <= BQN; ++i) {
    if (xbdi[i] == zero) {
      tempa = xopt[i] + d[i] - sl[i];
      tempb = su[i] - xopt[i] - d[i];
      if (tempa <= zero) {
        ++nact;
        xbdi[i] = onemin;
        goto L100;
      } else if (tempb <= zero) {
        ++nact;
        xbdi[i] = one;
        goto L100;
      }
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
  goto L210;
L150:
  shs = zero;
  dhs = zero;
  dhd = zero;
  for (int i = 1; i <= BQN; ++i) {
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
  {
    // Powell's search over iu angles (about 20 per optimizer step on the refine's objective).  The
    // angles' reductions are independent of each other, so they are evaluated BQ_UNR at a time --
    // their f64 divisions overlap instead of running one dependent chain per angle -- and then
    // scanned in order, exactly as the sequential loop compares them; angt keeps the last angle's
    // value, as after the loop.  Same operations on the same values: the results are unchanged.
    constexpr int BQ_UNR = 4;
    int i = 1;
    for (; i + BQ_UNR - 1 <= iu; i += BQ_UNR) {
      double ra[BQ_UNR], rr[BQ_UNR];
      for (int u = 0; u < BQ_UNR; ++u) {
        const double at = angbd * (double)(i + u) / (double)iu;
        const double st = (at + at) / (one + at * at);
        const double tp = shs + at * (at * dhd - dhs - dhs);
        ra[u] = at;
        rr[u] = st * (at * dredg - sredg - half * st * tp);
      }
      for (int u = 0; u < BQ_UNR; ++u) {
        rednew = rr[u];
        if (rednew > redmax) {
          redmax = rednew;
          isav = i + u;
          rdprev = redsav;
        } else if (i + u == isav + 1) {
          rdnext = rednew;
        }
        redsav = rednew;
      }
      angt = ra[BQ_UNR - 1];
    }
    for (; i <= iu; ++i) {
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
  for (int i = 1; i <= BQN; ++i) {
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
    bq_set(xbdi, iact, xsav);
    goto L100;
  }
  if (sdec > qred * .01) goto L120;
L190: {
    double dsq = zero;
    for (int i = 1; i <= BQN; ++i) {
      double xn = bq_max(bq_min(xopt[i] + d[i], su[i]), sl[i]);
      if (xbdi[i] == onemin) xn = sl[i];
      if (xbdi[i] == one) xn = su[i];
      xnew[i] = xn;
      d[i] = xn - xopt[i];
      dsq += d[i] * d[i];
    }
    for (int i = 1; i <= BQN; ++i) {
      d_m[i] = d[i];
      gnew_m[i] = gnew[i];
    }
    *dsq_out = dsq;
    *crvmin_out = crvmin;
    return;
  }
L210: {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(BQ_TRSBOX_LDS)
    // xpt is read here only: re-read it per product instead of letting the compiler hoist its 21
    // loads out of the iterations (with them in registers the routine spills)
    __asm__ volatile("" ::: "memory");
#endif
    int ih = 0;
    for (int j = 1; j <= BQN; ++j) {
      hs[j] = zero;
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) hs[j] += hq[ih] * s[i];
        hs[i] += hq[ih] * s[j];
      }
    }
    for (int k = 1; k <= BQNPT; ++k) {
      if (pq[k] != zero) {
        temp = zero;
        for (int j = 1; j <= BQN; ++j) temp += xpt[k][j] * s[j];
        temp *= pq[k];
        for (int i = 1; i <= BQN; ++i) hs[i] += temp * xpt[k][i];
      }
    }
    if (crvmin != zero) goto L50;
    if (iterc > itcsav) goto L150;
    for (int i = 1; i <= BQN; ++i) hred[i] = hs[i];
    goto L120;
  }
}

#undef BQ_D_AT

// ---------------------------------------------------------------- ALTMOV
BQ_NI void bq_altmov(const BQ_AS double (*BQ_RS xpt)[BQN], const BQ_AS double* BQ_RS xopt, const BQ_AS double (*BQ_RS bmat)[BQN],
                     const BQ_AS double (*BQ_RS zmat)[BQNPTM], const BQ_AS double* BQ_RS sl, const BQ_AS double* BQ_RS su, int kopt,
                     int knew, double adelt, BQ_AS double* BQ_RS xnew, BQ_AS double* BQ_RS xalt, BQ_AS double* BQ_RS alpha,
                     BQ_AS double* BQ_RS cauchy) {
  const double half = 0.5, one = 1.0, zero = 0.0;
  const double cnst = one + sqrt(2.0);
  double glag[BQN + 1], hcol[BQNPT + 1], w[2 * BQN + 1];
  double ha, temp, presav, dderiv, distsq, subd, slbd, sumin, diff, step = 0, vlag, tempd, tempa,
      tempb, predsq, stpsav = 0, bigstp, wfixsq, ggfree, wsqsav, gw, curv, scale, csave = 0;
  int ilbd, iubd, isbd, ksav = 0, ibdsav = 0, iflag;
  for (int k = 1; k <= BQNPT; ++k) hcol[k] = zero;
  for (int j = 1; j <= BQNPTM; ++j) {
    temp = zmat[knew][j];
    for (int k = 1; k <= BQNPT; ++k) hcol[k] += temp * zmat[k][j];
  }
  *alpha = bq_get(hcol, knew);
  ha = half * *alpha;
  for (int i = 1; i <= BQN; ++i) glag[i] = bmat[knew][i];
  for (int k = 1; k <= BQNPT; ++k) {
    temp = zero;
    for (int j = 1; j <= BQN; ++j) temp += xpt[k][j] * xopt[j];
    temp = hcol[k] * temp;
    for (int i = 1; i <= BQN; ++i) glag[i] += temp * xpt[k][i];
  }
  presav = zero;
  for (int k = 1; k <= BQNPT; ++k) {
    if (k == kopt) continue;
    dderiv = zero;
    distsq = zero;
    for (int i = 1; i <= BQN; ++i) {
      temp = xpt[k][i] - xopt[i];
      dderiv += glag[i] * temp;
      distsq += temp * temp;
    }
    subd = adelt / sqrt(distsq);
    slbd = -subd;
    ilbd = 0;
    iubd = 0;
    sumin = bq_min(one, subd);
    for (int i = 1; i <= BQN; ++i) {
      temp = xpt[k][i] - xopt[i];
      if (temp > zero) {
        if (slbd * temp < sl[i] - xopt[i]) {
          slbd = (sl[i] - xopt[i]) / temp;
          ilbd = -i;
        }
        if (subd * temp > su[i] - xopt[i]) {
          subd = bq_max(sumin, (su[i] - xopt[i]) / temp);
          iubd = i;
        }
      } else if (temp < zero) {
        if (slbd * temp > su[i] - xopt[i]) {
          slbd = (su[i] - xopt[i]) / temp;
          ilbd = i;
        }
        if (subd * temp < sl[i] - xopt[i]) {
          subd = bq_max(sumin, (sl[i] - xopt[i]) / temp);
          iubd = -i;
        }
      }
    }
    if (k == knew) {
      diff = dderiv - one;
      step = slbd;
      vlag = slbd * (dderiv - slbd * diff);
      isbd = ilbd;
      temp = subd * (dderiv - subd * diff);
      if (fabs(temp) > fabs(vlag)) {
        step = subd;
        vlag = temp;
        isbd = iubd;
      }
      tempd = half * dderiv;
      tempa = tempd - diff * slbd;
      tempb = tempd - diff * subd;
      if (tempa * tempb < zero) {
        temp = tempd * tempd / diff;
        if (fabs(temp) > fabs(vlag)) {
          step = tempd / diff;
          vlag = temp;
          isbd = 0;
        }
      }
    } else {
      step = slbd;
      vlag = slbd * (one - slbd);
      isbd = ilbd;
      temp = subd * (one - subd);
      if (fabs(temp) > fabs(vlag)) {
        step = subd;
        vlag = temp;
        isbd = iubd;
      }
      if (subd > half) {
        if (fabs(vlag) < .25) {
          step = half;
          vlag = .25;
          isbd = 0;
        }
      }
      vlag *= dderiv;
    }
    temp = step * (one - step) * distsq;
    predsq = vlag * vlag * (vlag * vlag + ha * temp * temp);
    if (predsq > presav) {
      presav = predsq;
      ksav = k;
      stpsav = step;
      ibdsav = isbd;
    }
  }
  for (int i = 1; i <= BQN; ++i) {
    temp = xopt[i] + stpsav * (xpt[ksav][i] - xopt[i]);
    xnew[i] = bq_max(sl[i], bq_min(su[i], temp));
  }
  if (ibdsav < 0) xnew[-ibdsav] = sl[-ibdsav];
  if (ibdsav > 0) xnew[ibdsav] = su[ibdsav];
  bigstp = adelt + adelt;
  iflag = 0;
L100:
  wfixsq = zero;
  ggfree = zero;
  for (int i = 1; i <= BQN; ++i) {
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
    return;
  }
L120:
  temp = adelt * adelt - wfixsq;
  if (temp > zero) {
    wsqsav = wfixsq;
    step = sqrt(temp / ggfree);
    ggfree = zero;
    for (int i = 1; i <= BQN; ++i) {
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
  for (int i = 1; i <= BQN; ++i) {
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
  curv = zero;
  for (int k = 1; k <= BQNPT; ++k) {
    temp = zero;
    for (int j = 1; j <= BQN; ++j) temp += xpt[k][j] * w[j];
    curv += hcol[k] * temp * temp;
  }
  if (iflag == 1) curv = -curv;
  if (curv > -gw && curv < -cnst * gw) {
    scale = -gw / curv;
    for (int i = 1; i <= BQN; ++i) {
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
    for (int i = 1; i <= BQN; ++i) {
      glag[i] = -glag[i];
      w[BQN + i] = xalt[i];
    }
    csave = *cauchy;
    iflag = 1;
    goto L100;
  }
  if (csave > *cauchy) {
    for (int i = 1; i <= BQN; ++i) xalt[i] = w[BQN + i];
    *cauchy = csave;
  }
}

// ---------------------------------------------------------------- UPDATE
BQ_NI void bq_update(BQ_AS double (*BQ_RS bmat)[BQN], BQ_AS double (*BQ_RS zmat)[BQNPTM], BQ_AS double* BQ_RS vlag, double beta,
                     double denom, int knew, BQ_AS double* BQ_RS w) {
  const double one = 1.0, zero = 0.0;
  double ztest = zero, temp, tempa, tempb, alpha, tau;
  for (int k = 1; k <= BQNPT; ++k)
    for (int j = 1; j <= BQNPTM; ++j) ztest = bq_max(ztest, fabs(zmat[k][j]));
  ztest *= 1e-20;
  for (int j = 2; j <= BQNPTM; ++j) {
    if (fabs(zmat[knew][j]) > ztest) {
      const double d1 = zmat[knew][1], d2 = zmat[knew][j];
      temp = sqrt(d1 * d1 + d2 * d2);
      tempa = zmat[knew][1] / temp;
      tempb = zmat[knew][j] / temp;
      for (int i = 1; i <= BQNPT; ++i) {
        temp = tempa * zmat[i][1] + tempb * zmat[i][j];
        zmat[i][j] = tempa * zmat[i][j] - tempb * zmat[i][1];
        zmat[i][1] = temp;
      }
    }
    zmat[knew][j] = zero;
  }
  for (int i = 1; i <= BQNPT; ++i) w[i] = zmat[knew][1] * zmat[i][1];
  alpha = w[knew];
  tau = vlag[knew];
  vlag[knew] -= one;
  temp = sqrt(denom);
  tempb = zmat[knew][1] / temp;
  tempa = tau / temp;
  for (int i = 1; i <= BQNPT; ++i) zmat[i][1] = tempa * zmat[i][1] - tempb * vlag[i];
  for (int j = 1; j <= BQN; ++j) {
    const int jp = BQNPT + j;
    w[jp] = bmat[knew][j];
    tempa = (alpha * vlag[jp] - tau * w[jp]) / denom;
    tempb = (-beta * w[jp] - tau * vlag[jp]) / denom;
    for (int i = 1; i <= jp; ++i) {
      bmat[i][j] = bmat[i][j] + tempa * vlag[i] + tempb * w[i];
      if (i > BQNPT) bmat[jp][i - BQNPT] = bmat[i][j];
    }
  }
}

// NLopt 2.6.1 nlopt_set_default_initial_step for one coordinate.
BQ_HD double bq_default_step(double x, double lb, double ub) {
  double step = HUGE_VAL;
  if (!isinf(ub) && !isinf(lb) && (ub - lb) * 0.25 < step && ub > lb) step = (ub - lb) * 0.25;
  if (!isinf(ub) && ub - x < step && ub > x) step = (ub - x) * 0.75;
  if (!isinf(lb) && x - lb < step && x > lb) step = (x - lb) * 0.75;
  if (isinf(step)) {
    if (!isinf(ub) && fabs(ub - x) < fabs(step)) step = (ub - x) * 1.1;
    if (!isinf(lb) && fabs(x - lb) < fabs(step)) step = (x - lb) * 1.1;
  }
  if (isinf(step) || step == 0.0 || fabs(step) < 2.2250738585072014e-308) step = x;
  if (isinf(step) || step == 0.0) step = 1;
  return step;
}

// Initialise: the nlopt_optimize -> bobyqa() wrapper up to the call of BOBYQB.
// Returns 0 (then call bq_step with any f) or a negative NLopt error code.
BQ_HD int bq_begin(BQ_AS BqState& st, const double* x0, const double* lb, const double* ub,
                   double xtol_rel, int maxeval) {
  BQ_ALIASES(st);
  double dxs[BQN];
  for (int i = 0; i < BQN; ++i) dxs[i] = bq_default_step(x0[i], lb[i], ub[i]);
  for (int i = 0; i < BQN; ++i) st.s[i] = 1.0;
  {
    int i = 1;
    for (; i < BQN && dxs[i] == dxs[i - 1]; ++i) {
    }
    if (i < BQN)
      for (i = 1; i < BQN; ++i) st.s[i] = dxs[i] / dxs[0];
  }
  for (int i = 0; i < BQN; ++i) {
    x[i + 1] = x0[i] / st.s[i];
    xl[i + 1] = lb[i] / st.s[i];
    xu[i + 1] = ub[i] / st.s[i];
  }
  st.rhobeg = fabs(dxs[0] / st.s[0]);
  st.rhoend = xtol_rel * st.rhobeg;
  st.maxeval = maxeval;
  st.nevals = 0;
  st.rc = BQR_SUCCESS;
  st.resume = 0;
  st.minf = 0;
  for (int j = 1; j <= BQN; ++j) {
    const double temp = xu[j] - xl[j];
    if (temp < st.rhobeg + st.rhobeg) {
      st.rc = BQR_INVALID_ARGS;
      for (int i = 0; i < BQN; ++i) st.xout[i] = x0[i];
      st.resume = -1;
      return BQR_INVALID_ARGS;
    }
    sl[j] = xl[j] - x[j];
    su[j] = xu[j] - x[j];
    if (sl[j] >= -st.rhobeg) {
      if (sl[j] >= 0.0) {
        x[j] = xl[j];
        sl[j] = 0.0;
        su[j] = temp;
      } else {
        x[j] = xl[j] + st.rhobeg;
        sl[j] = -st.rhobeg;
        su[j] = bq_max(xu[j] - x[j], st.rhobeg);
      }
    } else if (su[j] <= st.rhobeg) {
      if (su[j] <= 0.0) {
        x[j] = xu[j];
        sl[j] = -temp;
        su[j] = 0.0;
      } else {
        x[j] = xu[j] - st.rhobeg;
        sl[j] = bq_min(xl[j] - x[j], -st.rhobeg);
        su[j] = st.rhobeg;
      }
    }
  }
  return 0;
}

// Request an evaluation at the rescaled point p (1-based): nlopt's rescale_fun unscales it.
#define BQ_CALFUN(P, LABEL_ID)                                             \
  do {                                                                     \
    for (int i_ = 0; i_ < BQN; ++i_) st.xeval[i_] = (P)[i_ + 1] * st.s[i_]; \
    st.nevals++;                                                           \
    st.resume = LABEL_ID;                                                  \
    return BQ_NEED_F;                                                      \
  } while (0)

// Advance the optimizer.  fin is the objective value requested by the previous call (ignored
// on the first call).  Returns BQ_NEED_F with st.xeval set, or BQ_DONE with st.rc/st.xout.
BQ_NI int bq_step_impl(BQ_AS BqState& st, double fin);
BQ_HD int bq_step(BQ_AS BqState& st, double fin) {
  BQ_PT(t_all);
  const int r = bq_step_impl(st, fin);
  BQ_PA(3, t_all);
  return r;
}
BQ_NI int bq_step_impl(BQ_AS BqState& st, double fin) {
  BQ_ALIASES(st);
  const double half = 0.5, one = 1.0, ten = 10.0, tenth = 0.1, two = 2.0, zero = 0.0;
  double temp, sum, suma, sumb, bsum, dx, delsq, scaden, biglsq, hdiag, den, errbig, frhosq,
      bdtol, bdtest, curv, fracsq, sumpq, sumz, sumw, densav, pqold, gqsq, gisq, dist;
  int ih, ksav;
  switch (st.resume) {
    case 0: goto PSTART;
    case 1: goto PRESUME;
    case 2: goto L360R;
    case 3: goto R260R;
    default: return BQ_DONE;
  }
PSTART: {
    for (int j = 1; j <= BQN; ++j) {
      xbase[j] = x[j];
      for (int k = 1; k <= BQNPT; ++k) xpt[k][j] = zero;
      for (int i = 1; i <= BQNDIM; ++i) bmat[i][j] = zero;
    }
    for (int i = 1; i <= BQNH; ++i) hq[i] = zero;
    for (int k = 1; k <= BQNPT; ++k) {
      pq[k] = zero;
      for (int j = 1; j <= BQNPTM; ++j) zmat[k][j] = zero;
    }
    st.nf = 0;
    st.kopt = 1;
  PLOOP:
    st.nfm = st.nf;
    st.nfx = st.nf - BQN;
    ++st.nf;
    if (st.nfm <= 2 * BQN) {
      if (st.nfm >= 1 && st.nfm <= BQN) {
        st.stepa = st.rhobeg;
        if (su[st.nfm] == zero) st.stepa = -st.stepa;
        xpt[st.nf][st.nfm] = st.stepa;
      } else if (st.nfm > BQN) {
        st.stepa = xpt[st.nf - BQN][st.nfx];
        st.stepb = -st.rhobeg;
        if (sl[st.nfx] == zero) st.stepb = bq_min(two * st.rhobeg, su[st.nfx]);
        if (su[st.nfx] == zero) st.stepb = bq_max(-two * st.rhobeg, sl[st.nfx]);
        xpt[st.nf][st.nfx] = st.stepb;
      }
    }
    for (int j = 1; j <= BQN; ++j) {
      x[j] = bq_min(bq_max(xl[j], xbase[j] + xpt[st.nf][j]), xu[j]);
      if (xpt[st.nf][j] == sl[j]) x[j] = xl[j];
      if (xpt[st.nf][j] == su[j]) x[j] = xu[j];
    }
    BQ_CALFUN(x, 1);
  }
PRESUME: {
    const double rhosq = st.rhobeg * st.rhobeg;
    const int nf = st.nf, nfm = st.nfm, nfx = st.nfx;
    st.f = fin;
    fval[nf] = st.f;
    if (nf == 1) {
      st.fbeg = st.f;
      st.kopt = 1;
    } else if (st.f < fval[st.kopt]) {
      st.kopt = nf;
    }
    if (nf <= 2 * BQN + 1) {
      if (nf >= 2 && nf <= BQN + 1) {
        gopt[nfm] = (st.f - st.fbeg) / st.stepa;
        if (BQNPT < nf + BQN) {
          bmat[1][nfm] = -one / st.stepa;
          bmat[nf][nfm] = one / st.stepa;
          bmat[BQNPT + nfm][nfm] = -half * rhosq;
        }
      } else if (nf >= BQN + 2) {
        ih = nfx * (nfx + 1) / 2;
        temp = (st.f - st.fbeg) / st.stepb;
        st.diff = st.stepb - st.stepa;
        hq[ih] = two * (temp - gopt[nfx]) / st.diff;
        gopt[nfx] = (gopt[nfx] * st.stepb - temp * st.stepa) / st.diff;
        if (st.stepa * st.stepb < zero) {
          if (st.f < fval[nf - BQN]) {
            fval[nf] = fval[nf - BQN];
            fval[nf - BQN] = st.f;
            if (st.kopt == nf) st.kopt = nf - BQN;
            xpt[nf - BQN][nfx] = st.stepb;
            xpt[nf][nfx] = st.stepa;
          }
        }
        bmat[1][nfx] = -(st.stepa + st.stepb) / (st.stepa * st.stepb);
        bmat[nf][nfx] = -half / xpt[nf - BQN][nfx];
        bmat[nf - BQN][nfx] = -bmat[1][nfx] - bmat[nf][nfx];
        zmat[1][nfx] = sqrt(two) / (st.stepa * st.stepb);
        zmat[nf][nfx] = sqrt(half) / rhosq;
        zmat[nf - BQN][nfx] = -zmat[1][nfx] - zmat[nf][nfx];
      }
    }
    if (st.maxeval > 0 && st.nevals >= st.maxeval) {
      st.rc = BQR_MAXEVAL;
    } else if (st.nf < BQNPT) {
      goto PLOOP;
    }
  }
  st.xoptsq = zero;
  for (int i = 1; i <= BQN; ++i) {
    xopt[i] = xpt[st.kopt][i];
    st.xoptsq += xopt[i] * xopt[i];
  }
  st.fsave = fval[1];
  if (st.rc != BQR_SUCCESS) goto L720;
  st.kbase = 1;
  st.rho = st.rhobeg;
  st.delta = st.rho;
  st.nresc = st.nf;
  st.ntrits = 0;
  st.diffa = zero;
  st.diffb = zero;
  st.diffc = zero;
  st.ratio = zero;
  st.itest = 0;
  st.nfsav = st.nf;
  st.knew = 0;
L20:
  if (st.kopt != st.kbase) {
    ih = 0;
    for (int j = 1; j <= BQN; ++j) {
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) gopt[j] += hq[ih] * xopt[i];
        gopt[i] += hq[ih] * xopt[j];
      }
    }
    if (st.nf > BQNPT) {
      for (int k = 1; k <= BQNPT; ++k) {
        temp = zero;
        for (int j = 1; j <= BQN; ++j) temp += xpt[k][j] * xopt[j];
        temp = pq[k] * temp;
        for (int i = 1; i <= BQN; ++i) gopt[i] += temp * xpt[k][i];
      }
    }
  }
L60:
  {
  BQ_PT(t_trs);
  bq_trsbox(xpt, xopt, gopt, hq, pq, sl, su, st.delta, xnew, d, gnew,
            &st.dsq, &st.crvmin);
  BQ_PA(0, t_trs);
  }
  st.dnorm = bq_min(st.delta, sqrt(st.dsq));
  if (st.dnorm < half * st.rho) {
    st.ntrits = -1;
    temp = ten * st.rho;
    st.distsq = temp * temp;
    if (st.nf <= st.nfsav + 2) goto L650;
    errbig = bq_max(bq_max(st.diffa, st.diffb), st.diffc);
    frhosq = st.rho * .125 * st.rho;
    if (st.crvmin > zero && errbig > frhosq * st.crvmin) goto L650;
    bdtol = errbig / st.rho;
    for (int j = 1; j <= BQN; ++j) {
      bdtest = bdtol;
      if (xnew[j] == sl[j]) bdtest = gnew[j];
      if (xnew[j] == su[j]) bdtest = -gnew[j];
      if (bdtest < bdtol) {
        curv = hq[(j + j * j) / 2];
        for (int k = 1; k <= BQNPT; ++k) curv += pq[k] * (xpt[k][j] * xpt[k][j]);
        bdtest += half * curv * st.rho;
        if (bdtest < bdtol) goto L650;
      }
    }
    goto L680;
  }
  ++st.ntrits;
L90:
  if (st.dsq <= st.xoptsq * .001) {
    fracsq = st.xoptsq * .25;
    sumpq = zero;
    for (int k = 1; k <= BQNPT; ++k) {
      sumpq += pq[k];
      sum = -half * st.xoptsq;
      for (int i = 1; i <= BQN; ++i) sum += xpt[k][i] * xopt[i];
      w[BQNPT + k] = sum;
      temp = fracsq - half * sum;
      for (int i = 1; i <= BQN; ++i) {
        w[i] = bmat[k][i];
        vlag[i] = sum * xpt[k][i] + temp * xopt[i];
        const int ip = BQNPT + i;
        for (int j = 1; j <= i; ++j)
          bmat[ip][j] = bmat[ip][j] + w[i] * vlag[j] + vlag[i] * w[j];
      }
    }
    for (int jj = 1; jj <= BQNPTM; ++jj) {
      sumz = zero;
      sumw = zero;
      for (int k = 1; k <= BQNPT; ++k) {
        sumz += zmat[k][jj];
        vlag[k] = w[BQNPT + k] * zmat[k][jj];
        sumw += vlag[k];
      }
      for (int j = 1; j <= BQN; ++j) {
        sum = (fracsq * sumz - half * sumw) * xopt[j];
        for (int k = 1; k <= BQNPT; ++k) sum += vlag[k] * xpt[k][j];
        w[j] = sum;
        for (int k = 1; k <= BQNPT; ++k) bmat[k][j] += sum * zmat[k][jj];
      }
      for (int i = 1; i <= BQN; ++i) {
        const int ip = i + BQNPT;
        temp = w[i];
        for (int j = 1; j <= i; ++j) bmat[ip][j] += temp * w[j];
      }
    }
    ih = 0;
    for (int j = 1; j <= BQN; ++j) {
      w[j] = -half * sumpq * xopt[j];
      for (int k = 1; k <= BQNPT; ++k) {
        w[j] += pq[k] * xpt[k][j];
        xpt[k][j] -= xopt[j];
      }
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] = hq[ih] + w[i] * xopt[j] + xopt[i] * w[j];
        bmat[BQNPT + i][j] = bmat[BQNPT + j][i];
      }
    }
    for (int i = 1; i <= BQN; ++i) {
      xbase[i] += xopt[i];
      xnew[i] -= xopt[i];
      sl[i] -= xopt[i];
      su[i] -= xopt[i];
      xopt[i] = zero;
    }
    st.xoptsq = zero;
  }
  if (st.ntrits == 0) goto L210;
  goto L230;

L190:  // ---- RESCUE
#if defined(BQ_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
  if ((int)__lane_id() == (int)__builtin_ctzll(__ballot(1))) atomicAdd(&bq_prof[4], 1ull);
#endif
  st.nfsav = st.nf;
  st.kbase = st.kopt;
  {
    const double sfrac = half / (double)BQNP;
    double winc = zero, bet2 = 0, den2 = 0, dsqmin, vlmxsq;
    int nrem, kold, kn, ip, iq, iw;
    sumpq = zero;
    for (int k = 1; k <= BQNPT; ++k) {
      st.distsq = zero;
      for (int j = 1; j <= BQN; ++j) {
        xpt[k][j] -= xopt[j];
        st.distsq += xpt[k][j] * xpt[k][j];
      }
      sumpq += pq[k];
      w[BQNDIM + k] = st.distsq;
      winc = bq_max(winc, st.distsq);
      for (int j = 1; j <= BQNPTM; ++j) zmat[k][j] = zero;
    }
    ih = 0;
    for (int j = 1; j <= BQN; ++j) {
      w[j] = half * sumpq * xopt[j];
      for (int k = 1; k <= BQNPT; ++k) w[j] += pq[k] * xpt[k][j];
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] = hq[ih] + w[i] * xopt[j] + w[j] * xopt[i];
      }
    }
    for (int j = 1; j <= BQN; ++j) {
      xbase[j] += xopt[j];
      sl[j] -= xopt[j];
      su[j] -= xopt[j];
      xopt[j] = zero;
      ptsaux[1][j] = bq_min(st.delta, su[j]);
      ptsaux[2][j] = bq_max(-st.delta, sl[j]);
      if (ptsaux[1][j] + ptsaux[2][j] < zero) {
        temp = ptsaux[1][j];
        ptsaux[1][j] = ptsaux[2][j];
        ptsaux[2][j] = temp;
      }
      if (fabs(ptsaux[2][j]) < half * fabs(ptsaux[1][j])) ptsaux[2][j] = half * ptsaux[1][j];
      for (int i = 1; i <= BQNDIM; ++i) bmat[i][j] = zero;
    }
    st.rs_fbase = fval[st.kopt];
    ptsid[1] = sfrac;
    for (int j = 1; j <= BQN; ++j) {
      const int jp = j + 1, jpn = jp + BQN;
      ptsid[jp] = (double)j + sfrac;
      if (jpn <= BQNPT) {
        ptsid[jpn] = (double)j / (double)BQNP + sfrac;
        temp = one / (ptsaux[1][j] - ptsaux[2][j]);
        bmat[jp][j] = -temp + one / ptsaux[1][j];
        bmat[jpn][j] = temp + one / ptsaux[2][j];
        bmat[1][j] = -bmat[jp][j] - bmat[jpn][j];
        zmat[1][j] = sqrt(2.) / fabs(ptsaux[1][j] * ptsaux[2][j]);
        zmat[jp][j] = zmat[1][j] * ptsaux[2][j] * temp;
        zmat[jpn][j] = -zmat[1][j] * ptsaux[1][j] * temp;
      } else {
        bmat[1][j] = -one / ptsaux[1][j];
        bmat[jp][j] = one / ptsaux[1][j];
        bmat[j + BQNPT][j] = -half * (ptsaux[1][j] * ptsaux[1][j]);
      }
    }
    nrem = BQNPT;
    kold = 1;
    kn = st.kopt;
  R80:
    for (int j = 1; j <= BQN; ++j) {
      temp = bmat[kold][j];
      bmat[kold][j] = bmat[kn][j];
      bmat[kn][j] = temp;
    }
    for (int j = 1; j <= BQNPTM; ++j) {
      temp = zmat[kold][j];
      zmat[kold][j] = zmat[kn][j];
      zmat[kn][j] = temp;
    }
    ptsid[kold] = ptsid[kn];
    ptsid[kn] = zero;
    w[BQNDIM + kn] = zero;
    --nrem;
    if (kn != st.kopt) {
      temp = vlag[kold];
      vlag[kold] = vlag[kn];
      vlag[kn] = temp;
      bq_update(bmat, zmat, vlag, bet2, den2, kn, w);
      if (nrem == 0) goto R350;
      for (int k = 1; k <= BQNPT; ++k) w[BQNDIM + k] = fabs(w[BQNDIM + k]);
    }
  R120:
    dsqmin = zero;
    for (int k = 1; k <= BQNPT; ++k) {
      if (w[BQNDIM + k] > zero) {
        if (dsqmin == zero || w[BQNDIM + k] < dsqmin) {
          kn = k;
          dsqmin = w[BQNDIM + k];
        }
      }
    }
    if (dsqmin == zero) goto R260;
    for (int j = 1; j <= BQN; ++j) w[BQNPT + j] = xpt[kn][j];
    for (int k = 1; k <= BQNPT; ++k) {
      sum = zero;
      if (k == st.kopt) {
      } else if (ptsid[k] == zero) {
        for (int j = 1; j <= BQN; ++j) sum += w[BQNPT + j] * xpt[k][j];
      } else {
        ip = (int)ptsid[k];
        if (ip > 0) sum = w[BQNPT + ip] * ptsaux[1][ip];
        iq = (int)((double)BQNP * ptsid[k] - (double)(ip * BQNP));
        if (iq > 0) {
          iw = 1;
          if (ip == 0) iw = 2;
          sum += w[BQNPT + iq] * ptsaux[iw][iq];
        }
      }
      w[k] = half * sum * sum;
    }
    for (int k = 1; k <= BQNPT; ++k) {
      sum = zero;
      for (int j = 1; j <= BQN; ++j) sum += bmat[k][j] * w[BQNPT + j];
      vlag[k] = sum;
    }
    bet2 = zero;
    for (int j = 1; j <= BQNPTM; ++j) {
      sum = zero;
      for (int k = 1; k <= BQNPT; ++k) sum += zmat[k][j] * w[k];
      bet2 -= sum * sum;
      for (int k = 1; k <= BQNPT; ++k) vlag[k] += sum * zmat[k][j];
    }
    bsum = zero;
    st.distsq = zero;
    for (int j = 1; j <= BQN; ++j) {
      sum = zero;
      for (int k = 1; k <= BQNPT; ++k) sum += bmat[k][j] * w[k];
      const int jp = j + BQNPT;
      bsum += sum * w[jp];
      for (int ipp = BQNPT + 1; ipp <= BQNDIM; ++ipp) sum += bmat[ipp][j] * w[ipp];
      bsum += sum * w[jp];
      vlag[jp] = sum;
      st.distsq += xpt[kn][j] * xpt[kn][j];
    }
    bet2 = half * st.distsq * st.distsq + bet2 - bsum;
    vlag[st.kopt] += one;
    den2 = zero;
    vlmxsq = zero;
    for (int k = 1; k <= BQNPT; ++k) {
      if (ptsid[k] != zero) {
        hdiag = zero;
        for (int j = 1; j <= BQNPTM; ++j) hdiag += zmat[k][j] * zmat[k][j];
        den = bet2 * hdiag + vlag[k] * vlag[k];
        if (den > den2) {
          kold = k;
          den2 = den;
        }
      }
      vlmxsq = bq_max(vlmxsq, vlag[k] * vlag[k]);
    }
    if (den2 <= vlmxsq * .01) {
      w[BQNDIM + kn] = -w[BQNDIM + kn] - winc;
      goto R120;
    }
    goto R80;
  }
R260:
  st.kpt = 1;
R260LOOP:
  if (st.kpt > BQNPT) goto R350;
  if (ptsid[st.kpt] == zero) {
    ++st.kpt;
    goto R260LOOP;
  }
  if (st.maxeval > 0 && st.nevals >= st.maxeval) {
    st.nf = -1;
    goto R350;
  }
  {
    const int kpt = st.kpt;
    ih = 0;
    for (int j = 1; j <= BQN; ++j) {
      w[j] = xpt[kpt][j];
      xpt[kpt][j] = zero;
      temp = pq[kpt] * w[j];
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] += temp * w[i];
      }
    }
    pq[kpt] = zero;
    st.rs_ip = (int)ptsid[kpt];
    st.rs_iq = (int)((double)BQNP * ptsid[kpt] - (double)(st.rs_ip * BQNP));
    const int ip = st.rs_ip, iq = st.rs_iq;
    int ihp = 0, ihq;
    if (ip > 0) {
      st.rs_xp = ptsaux[1][ip];
      xpt[kpt][ip] = st.rs_xp;
    }
    if (iq > 0) {
      st.rs_xq = ptsaux[1][iq];
      if (ip == 0) st.rs_xq = ptsaux[2][iq];
      xpt[kpt][iq] = st.rs_xq;
    }
    st.rs_vq = st.rs_fbase;
    if (ip > 0) {
      ihp = (ip + ip * ip) / 2;
      st.rs_vq += st.rs_xp * (gopt[ip] + half * st.rs_xp * hq[ihp]);
    }
    if (iq > 0) {
      ihq = (iq + iq * iq) / 2;
      st.rs_vq += st.rs_xq * (gopt[iq] + half * st.rs_xq * hq[ihq]);
      if (ip > 0) {
        const int iw = (ihp > ihq ? ihp : ihq) - (ip > iq ? ip - iq : iq - ip);
        st.rs_vq += st.rs_xp * st.rs_xq * hq[iw];
      }
    }
    for (int k = 1; k <= BQNPT; ++k) {
      temp = zero;
      if (ip > 0) temp += st.rs_xp * xpt[k][ip];
      if (iq > 0) temp += st.rs_xq * xpt[k][iq];
      st.rs_vq += half * pq[k] * temp * temp;
    }
    for (int i = 1; i <= BQN; ++i) {
      w[i] = bq_min(bq_max(xl[i], xbase[i] + xpt[kpt][i]), xu[i]);
      if (xpt[kpt][i] == sl[i]) w[i] = xl[i];
      if (xpt[kpt][i] == su[i]) w[i] = xu[i];
    }
    ++st.nf;
    BQ_CALFUN(w, 3);
  }
R260R: {
    const int kpt = st.kpt, ip0 = st.rs_ip, iq0 = st.rs_iq;
    (void)ip0; (void)iq0;
    st.f = fin;
    fval[kpt] = st.f;
    if (st.f < fval[st.kopt]) st.kopt = kpt;
    st.diff = st.f - st.rs_vq;
    for (int i = 1; i <= BQN; ++i) gopt[i] += st.diff * bmat[kpt][i];
    for (int k = 1; k <= BQNPT; ++k) {
      sum = zero;
      for (int j = 1; j <= BQNPTM; ++j) sum += zmat[k][j] * zmat[kpt][j];
      temp = st.diff * sum;
      if (ptsid[k] == zero) {
        pq[k] += temp;
      } else {
        const int ip = (int)ptsid[k];
        const int iq = (int)((double)BQNP * ptsid[k] - (double)(ip * BQNP));
        const int ihq = (iq * iq + iq) / 2;
        if (ip == 0) {
          hq[ihq] += temp * (ptsaux[2][iq] * ptsaux[2][iq]);
        } else {
          const int ihp = (ip * ip + ip) / 2;
          hq[ihp] += temp * (ptsaux[1][ip] * ptsaux[1][ip]);
          if (iq > 0) {
            hq[ihq] += temp * (ptsaux[1][iq] * ptsaux[1][iq]);
            const int iw = (ihp > ihq ? ihp : ihq) - (iq > ip ? iq - ip : ip - iq);
            hq[iw] += temp * ptsaux[1][ip] * ptsaux[1][iq];
          }
        }
      }
    }
    ptsid[kpt] = zero;
    ++st.kpt;
    goto R260LOOP;
  }
R350:
  st.xoptsq = zero;
  if (st.kopt != st.kbase) {
    for (int i = 1; i <= BQN; ++i) {
      xopt[i] = xpt[st.kopt][i];
      st.xoptsq += xopt[i] * xopt[i];
    }
  }
  if (st.nf < 0) {
    st.nf = st.maxeval;
    st.rc = BQR_MAXEVAL;
    goto L720;
  }
  st.nresc = st.nf;
  if (st.nfsav < st.nf) {
    st.nfsav = st.nf;
    goto L20;
  }
  if (st.ntrits > 0) goto L60;
L210:
  {
  BQ_PT(t_alt);
  bq_altmov(xpt, xopt, bmat, zmat, sl, su, st.kopt, st.knew, st.adelt, xnew,
            xalt, &st.alpha, &st.cauchy);
  BQ_PA(1, t_alt);
  }
  for (int i = 1; i <= BQN; ++i) d[i] = xnew[i] - xopt[i];
L230:
  for (int k = 1; k <= BQNPT; ++k) {
    suma = zero;
    sumb = zero;
    sum = zero;
    for (int j = 1; j <= BQN; ++j) {
      suma += xpt[k][j] * d[j];
      sumb += xpt[k][j] * xopt[j];
      sum += bmat[k][j] * d[j];
    }
    w[k] = suma * (half * suma + sumb);
    vlag[k] = sum;
    w[BQNPT + k] = suma;
  }
  st.beta = zero;
  for (int jj = 1; jj <= BQNPTM; ++jj) {
    sum = zero;
    for (int k = 1; k <= BQNPT; ++k) sum += zmat[k][jj] * w[k];
    st.beta -= sum * sum;
    for (int k = 1; k <= BQNPT; ++k) vlag[k] += sum * zmat[k][jj];
  }
  st.dsq = zero;
  bsum = zero;
  dx = zero;
  for (int j = 1; j <= BQN; ++j) {
    st.dsq += d[j] * d[j];
    sum = zero;
    for (int k = 1; k <= BQNPT; ++k) sum += w[k] * bmat[k][j];
    bsum += sum * d[j];
    const int jp = BQNPT + j;
    for (int i = 1; i <= BQN; ++i) sum += bmat[jp][i] * d[i];
    vlag[jp] = sum;
    bsum += sum * d[j];
    dx += d[j] * xopt[j];
  }
  st.beta = dx * dx + st.dsq * (st.xoptsq + dx + dx + half * st.dsq) + st.beta - bsum;
  vlag[st.kopt] += one;
  if (st.ntrits == 0) {
    st.denom = vlag[st.knew] * vlag[st.knew] + st.alpha * st.beta;
    if (st.denom < st.cauchy && st.cauchy > zero) {
      for (int i = 1; i <= BQN; ++i) {
        xnew[i] = xalt[i];
        d[i] = xnew[i] - xopt[i];
      }
      st.cauchy = zero;
      goto L230;
    }
    if (st.denom <= half * (vlag[st.knew] * vlag[st.knew])) {
      if (st.nf > st.nresc) goto L190;
      st.rc = BQR_ROUNDOFF;
      goto L720;
    }
  } else {
    delsq = st.delta * st.delta;
    scaden = zero;
    biglsq = zero;
    st.knew = 0;
    for (int k = 1; k <= BQNPT; ++k) {
      if (k == st.kopt) continue;
      hdiag = zero;
      for (int jj = 1; jj <= BQNPTM; ++jj) hdiag += zmat[k][jj] * zmat[k][jj];
      den = st.beta * hdiag + vlag[k] * vlag[k];
      st.distsq = zero;
      for (int j = 1; j <= BQN; ++j) {
        temp = xpt[k][j] - xopt[j];
        st.distsq += temp * temp;
      }
      temp = st.distsq / delsq;
      temp = bq_max(one, temp * temp);
      if (temp * den > scaden) {
        scaden = temp * den;
        st.knew = k;
        st.denom = den;
      }
      biglsq = bq_max(biglsq, temp * (vlag[k] * vlag[k]));
    }
    if (scaden <= half * biglsq) {
      if (st.nf > st.nresc) goto L190;
      st.rc = BQR_ROUNDOFF;
      goto L720;
    }
  }
L360:
  for (int i = 1; i <= BQN; ++i) {
    x[i] = bq_min(bq_max(xl[i], xbase[i] + xnew[i]), xu[i]);
    if (xnew[i] == sl[i]) x[i] = xl[i];
    if (xnew[i] == su[i]) x[i] = xu[i];
  }
  if (st.maxeval > 0 && st.nevals >= st.maxeval) {
    st.rc = BQR_MAXEVAL;
    goto L720;
  }
  ++st.nf;
  BQ_CALFUN(x, 2);
L360R:
  st.f = fin;
  if (st.ntrits == -1) {
    st.fsave = st.f;
    st.rc = BQR_XTOL;
    if (st.fsave < fval[st.kopt]) {
      st.minf = st.f;
      for (int i = 0; i < BQN; ++i) st.xout[i] = x[i + 1] * st.s[i];
      st.resume = -1;
      return BQ_DONE;
    }
    goto L720;
  }
  st.fopt = fval[st.kopt];
  st.vquad = zero;
  ih = 0;
  for (int j = 1; j <= BQN; ++j) {
    st.vquad += d[j] * gopt[j];
    for (int i = 1; i <= j; ++i) {
      ++ih;
      temp = d[i] * d[j];
      if (i == j) temp = half * temp;
      st.vquad += hq[ih] * temp;
    }
  }
  for (int k = 1; k <= BQNPT; ++k) {
    temp = w[BQNPT + k];
    st.vquad += half * pq[k] * (temp * temp);
  }
  st.diff = st.f - st.fopt - st.vquad;
  st.diffc = st.diffb;
  st.diffb = st.diffa;
  st.diffa = fabs(st.diff);
  if (st.dnorm > st.rho) st.nfsav = st.nf;
  if (st.ntrits > 0) {
    if (st.vquad >= zero) {
      st.rc = BQR_ROUNDOFF;
      goto L720;
    }
    st.ratio = (st.f - st.fopt) / st.vquad;
    if (st.ratio <= tenth) st.delta = bq_min(half * st.delta, st.dnorm);
    else if (st.ratio <= .7) st.delta = bq_max(half * st.delta, st.dnorm);
    else st.delta = bq_max(half * st.delta, st.dnorm + st.dnorm);
    if (st.delta <= st.rho * 1.5) st.delta = st.rho;
    if (st.f < st.fopt) {
      ksav = st.knew;
      densav = st.denom;
      delsq = st.delta * st.delta;
      scaden = zero;
      biglsq = zero;
      st.knew = 0;
      for (int k = 1; k <= BQNPT; ++k) {
        hdiag = zero;
        for (int jj = 1; jj <= BQNPTM; ++jj) hdiag += zmat[k][jj] * zmat[k][jj];
        den = st.beta * hdiag + vlag[k] * vlag[k];
        st.distsq = zero;
        for (int j = 1; j <= BQN; ++j) {
          temp = xpt[k][j] - xnew[j];
          st.distsq += temp * temp;
        }
        temp = st.distsq / delsq;
        temp = bq_max(one, temp * temp);
        if (temp * den > scaden) {
          scaden = temp * den;
          st.knew = k;
          st.denom = den;
        }
        biglsq = bq_max(biglsq, temp * (vlag[k] * vlag[k]));
      }
      if (scaden <= half * biglsq) {
        st.knew = ksav;
        st.denom = densav;
      }
    }
  }
  {
  BQ_PT(t_upd);
  bq_update(bmat, zmat, vlag, st.beta, st.denom, st.knew, w);
  BQ_PA(2, t_upd);
  }
  ih = 0;
  pqold = pq[st.knew];
  pq[st.knew] = zero;
  for (int i = 1; i <= BQN; ++i) {
    temp = pqold * xpt[st.knew][i];
    for (int j = 1; j <= i; ++j) {
      ++ih;
      hq[ih] += temp * xpt[st.knew][j];
    }
  }
  for (int jj = 1; jj <= BQNPTM; ++jj) {
    temp = st.diff * zmat[st.knew][jj];
    for (int k = 1; k <= BQNPT; ++k) pq[k] += temp * zmat[k][jj];
  }
  fval[st.knew] = st.f;
  for (int i = 1; i <= BQN; ++i) {
    xpt[st.knew][i] = xnew[i];
    w[i] = bmat[st.knew][i];
  }
  for (int k = 1; k <= BQNPT; ++k) {
    suma = zero;
    for (int jj = 1; jj <= BQNPTM; ++jj) suma += zmat[st.knew][jj] * zmat[k][jj];
    sumb = zero;
    for (int j = 1; j <= BQN; ++j) sumb += xpt[k][j] * xopt[j];
    temp = suma * sumb;
    for (int i = 1; i <= BQN; ++i) w[i] += temp * xpt[k][i];
  }
  for (int i = 1; i <= BQN; ++i) gopt[i] += st.diff * w[i];
  if (st.f < st.fopt) {
    st.kopt = st.knew;
    st.xoptsq = zero;
    ih = 0;
    for (int j = 1; j <= BQN; ++j) {
      xopt[j] = xnew[j];
      st.xoptsq += xopt[j] * xopt[j];
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) gopt[j] += hq[ih] * d[i];
        gopt[i] += hq[ih] * d[j];
      }
    }
    for (int k = 1; k <= BQNPT; ++k) {
      temp = zero;
      for (int j = 1; j <= BQN; ++j) temp += xpt[k][j] * d[j];
      temp = pq[k] * temp;
      for (int i = 1; i <= BQN; ++i) gopt[i] += temp * xpt[k][i];
    }
  }
  if (st.ntrits > 0) {
    for (int k = 1; k <= BQNPT; ++k) {
      vlag[k] = fval[k] - fval[st.kopt];
      w[k] = zero;
    }
    for (int j = 1; j <= BQNPTM; ++j) {
      sum = zero;
      for (int k = 1; k <= BQNPT; ++k) sum += zmat[k][j] * vlag[k];
      for (int k = 1; k <= BQNPT; ++k) w[k] += sum * zmat[k][j];
    }
    for (int k = 1; k <= BQNPT; ++k) {
      sum = zero;
      for (int j = 1; j <= BQN; ++j) sum += xpt[k][j] * xopt[j];
      w[k + BQNPT] = w[k];
      w[k] = sum * w[k];
    }
    gqsq = zero;
    gisq = zero;
    for (int i = 1; i <= BQN; ++i) {
      sum = zero;
      for (int k = 1; k <= BQNPT; ++k) sum = sum + bmat[k][i] * vlag[k] + xpt[k][i] * w[k];
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
      vlag[BQNPT + i] = sum;
    }
    ++st.itest;
    if (gqsq < ten * gisq) st.itest = 0;
    if (st.itest >= 3) {
      const int imax = BQNPT > BQNH ? BQNPT : BQNH;
      for (int i = 1; i <= imax; ++i) {
        if (i <= BQN) gopt[i] = vlag[BQNPT + i];
        if (i <= BQNPT) pq[i] = w[BQNPT + i];
        if (i <= BQNH) hq[i] = zero;
        st.itest = 0;
      }
    }
  }
  if (st.ntrits == 0) goto L60;
  if (st.f <= st.fopt + tenth * st.vquad) goto L60;
  {
    const double t1 = two * st.delta, t2 = ten * st.rho;
    st.distsq = bq_max(t1 * t1, t2 * t2);
  }
L650:
  st.knew = 0;
  for (int k = 1; k <= BQNPT; ++k) {
    sum = zero;
    for (int j = 1; j <= BQN; ++j) {
      temp = xpt[k][j] - xopt[j];
      sum += temp * temp;
    }
    if (sum > st.distsq) {
      st.knew = k;
      st.distsq = sum;
    }
  }
  if (st.knew > 0) {
    dist = sqrt(st.distsq);
    if (st.ntrits == -1) {
      st.delta = bq_min(tenth * st.delta, half * dist);
      if (st.delta <= st.rho * 1.5) st.delta = st.rho;
    }
    st.ntrits = 0;
    st.adelt = bq_max(bq_min(tenth * dist, st.delta), st.rho);
    st.dsq = st.adelt * st.adelt;
    goto L90;
  }
  if (st.ntrits == -1) goto L680;
  if (st.ratio > zero) goto L60;
  if (bq_max(st.delta, st.dnorm) > st.rho) goto L60;
L680:
  if (st.rho > st.rhoend) {
    st.delta = half * st.rho;
    st.ratio = st.rho / st.rhoend;
    if (st.ratio <= 16.) st.rho = st.rhoend;
    else if (st.ratio <= 250.) st.rho = sqrt(st.ratio) * st.rhoend;
    else st.rho = tenth * st.rho;
    st.delta = bq_max(st.delta, st.rho);
    st.ntrits = 0;
    st.nfsav = st.nf;
    goto L60;
  }
  if (st.ntrits == -1) goto L360;
  st.rc = BQR_XTOL;
L720:
  if (fval[st.kopt] <= st.fsave) {
    for (int i = 1; i <= BQN; ++i) {
      x[i] = bq_min(bq_max(xl[i], xbase[i] + xopt[i]), xu[i]);
      if (xopt[i] == sl[i]) x[i] = xl[i];
      if (xopt[i] == su[i]) x[i] = xu[i];
    }
    st.f = fval[st.kopt];
  }
  st.minf = st.f;
  for (int i = 0; i < BQN; ++i) st.xout[i] = x[i + 1] * st.s[i];
  st.resume = -1;
  return BQ_DONE;
}

#undef BQ_CALFUN

}  // namespace pmvsdev
