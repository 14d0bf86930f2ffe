// oracle/bobyqa_oracle.h -- TEST INFRASTRUCTURE ONLY (oracle). Never linked into the product.
//
// CPU restatement of the optimiser the reference calls in COptim::refinePatchBFGS
// (reference source/pmvs/optim.cpp:615-647): NLopt v2.6.1 (lib/CMakeLists.txt:22, a
// configure-time git clone that is ABSENT from /root/reference and from this image)
// algorithm LN_BOBYQA with n = 3.  The arithmetic below restates
//   * M.J.D. Powell, "The BOBYQA algorithm for bound constrained optimization without
//     derivatives", DAMTP 2009/NA06 (subroutines BOBYQB, PRELIM, TRSBOX, ALTMOV, UPDATE,
//     RESCUE), in Powell's operation order, with
//   * the NLopt 2.6.1 driver semantics the reference relies on: npt = 2n+1, the default
//     initial-step heuristic (nlopt_set_default_initial_step), per-dimension rescaling so the
//     initial steps are equal (nlopt_compute_rescaling), rhobeg = dx[0]/s[0],
//     rhoend = xtol_rel*rhobeg, maxeval checked before every evaluation, and the result codes
//     (XTOL_REACHED on normal termination; MAXEVAL_REACHED; ROUNDOFF_LIMITED on
//     denominator cancellation or a trust-region step that fails to reduce the model).
// Parity of the optimiser trajectory against NLopt itself is UNPINNED (NLopt is absent);
// the product's device BOBYQA (cmvs-pmvs_amd/csrc/bobyqa_dev.h) is checked against THIS file.
#pragma once
#include <cmath>
#include <functional>

namespace oracle {

enum BqResult {
  BQ_SUCCESS = 1, BQ_STOPVAL = 2, BQ_FTOL = 3, BQ_XTOL = 4, BQ_MAXEVAL = 5,
  BQ_FAILURE = -1, BQ_INVALID_ARGS = -2, BQ_ROUNDOFF = -4
};

// Objective in the caller's (unscaled) coordinates.
typedef std::function<double(const double* x)> BqFunc;

namespace bq {
constexpr int N = 3;
constexpr int NPT = 2 * N + 1;   // NLopt passes npt = 2n+1
constexpr int NP = N + 1;
constexpr int NPTM = NPT - NP;
constexpr int NDIM = NPT + N;
constexpr int NH = N * NP / 2;

// NLopt's C translation uses MIN2/MAX2 macros: ((a) <= (b) ? (a) : (b)), ((a) >= (b) ? (a) : (b)).
static inline double dmin(double a, double b) { return (a <= b) ? a : b; }
static inline double dmax(double a, double b) { return (a >= b) ? a : b; }

// ---------------------------------------------------------------- TRSBOX
static void trsbox(const double xpt[NPT + 1][N + 1], const double* xopt, const double* gopt,
                   const double* hq, const double* pq, const double* sl, const double* su,
                   double delta, double* xnew, double* d, double* gnew, double* xbdi,
                   double* s, double* hs, double* hred, double* dsq_out, double* crvmin_out) {
  const double half = 0.5, one = 1.0, onemin = -1.0, zero = 0.0;
  int iterc = 0, nact = 0, itermax = 0, itcsav = 0, iact = 0, isav = 0, iu = 0;
  double sqstp = zero, ggsav = 0, delsq, qred, crvmin, beta = 0, stepsq = 0, gredsq = 0, resid, ds, shs = 0,
         temp, blen = 0, stplen = 0, xsum, sdec, dredsq = 0, dredg = 0, sredg = 0, angbd = 0,
         tempa, tempb, ratio, ssq, xsav = 0, dhs = 0, dhd = 0, redmax, redsav, angt = 0, sth,
         rednew, rdprev = 0, rdnext = 0, cth;
  (void)sqstp; (void)ratio;
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
  delsq = delta * delta;
  qred = zero;
  crvmin = onemin;
L20:
  beta = zero;
L30:
  stepsq = zero;
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] != zero) {
      s[i] = zero;
    } else if (beta == zero) {
      s[i] = -gnew[i];
    } else {
      s[i] = beta * s[i] - gnew[i];
    }
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
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] == zero) {
      resid -= d[i] * d[i];
      ds += s[i] * d[i];
      shs += s[i] * hs[i];
    }
  }
  if (resid <= zero) goto L90;
  temp = std::sqrt(stepsq * resid + ds * ds);
  if (ds < zero) {
    blen = (temp - ds) / stepsq;
  } else {
    blen = resid / (temp + ds);
  }
  stplen = blen;
  if (shs > zero) stplen = dmin(blen, gredsq / shs);
  iact = 0;
  for (int i = 1; i <= N; ++i) {
    if (s[i] != zero) {
      xsum = xopt[i] + d[i];
      if (s[i] > zero) {
        temp = (su[i] - xsum) / s[i];
      } else {
        temp = (sl[i] - xsum) / s[i];
      }
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
      crvmin = dmin(crvmin, temp);
      if (crvmin == onemin) crvmin = temp;
    }
    ggsav = gredsq;
    gredsq = zero;
    for (int i = 1; i <= N; ++i) {
      gnew[i] += stplen * hs[i];
      if (xbdi[i] == zero) gredsq += gnew[i] * gnew[i];
      d[i] += stplen * s[i];
    }
    sdec = dmax(stplen * (ggsav - half * stplen * shs), zero);
    qred += sdec;
  }
  if (iact > 0) {
    ++nact;
    xbdi[iact] = one;
    if (s[iact] < zero) xbdi[iact] = onemin;
    delsq -= d[iact] * d[iact];
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
  temp = std::sqrt(temp);
  for (int i = 1; i <= N; ++i) {
    if (xbdi[i] == zero) {
      s[i] = (dredg * d[i] - dredsq * gnew[i]) / temp;
    } else {
      s[i] = zero;
    }
  }
  sredg = -temp;
  angbd = one;
  iact = 0;
  for (int i = 1; i <= N; ++i) {
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
        temp = std::sqrt(temp) - s[i];
        if (angbd * temp > tempa) {
          angbd = tempa / temp;
          iact = i;
          xsav = onemin;
        }
      }
      temp = su[i] - xopt[i];
      temp = ssq - temp * temp;
      if (temp > zero) {
        temp = std::sqrt(temp) + s[i];
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
    xbdi[iact] = xsav;
    goto L100;
  }
  if (sdec > qred * .01) goto L120;
L190:
  *dsq_out = zero;
  for (int i = 1; i <= N; ++i) {
    xnew[i] = dmax(dmin(xopt[i] + d[i], su[i]), sl[i]);
    if (xbdi[i] == onemin) xnew[i] = sl[i];
    if (xbdi[i] == one) xnew[i] = su[i];
    d[i] = xnew[i] - xopt[i];
    *dsq_out += d[i] * d[i];
  }
  *crvmin_out = crvmin;
  return;
L210: {
    int ih = 0;
    for (int j = 1; j <= N; ++j) {
      hs[j] = zero;
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) hs[j] += hq[ih] * s[i];
        hs[i] += hq[ih] * s[j];
      }
    }
    for (int k = 1; k <= NPT; ++k) {
      if (pq[k] != zero) {
        temp = zero;
        for (int j = 1; j <= N; ++j) temp += xpt[k][j] * s[j];
        temp *= pq[k];
        for (int i = 1; i <= N; ++i) hs[i] += temp * xpt[k][i];
      }
    }
    if (crvmin != zero) goto L50;
    if (iterc > itcsav) goto L150;
    for (int i = 1; i <= N; ++i) hred[i] = hs[i];
    goto L120;
  }
}

// ---------------------------------------------------------------- ALTMOV
static void altmov(const double xpt[NPT + 1][N + 1], const double* xopt,
                   const double bmat[NDIM + 1][N + 1], const double zmat[NPT + 1][NPTM + 1],
                   const double* sl, const double* su, int kopt, int knew, double adelt,
                   double* xnew, double* xalt, double* alpha, double* cauchy, double* glag,
                   double* hcol, double* w) {
  const double half = 0.5, one = 1.0, zero = 0.0;
  const double cnst = one + std::sqrt(2.0);
  double ha, temp, presav, dderiv, distsq, subd, slbd, sumin, diff, step = 0, vlag, tempd, tempa,
      tempb, predsq, stpsav = 0, bigstp, wfixsq, ggfree, wsqsav, gw, curv, scale, csave = 0;
  int ilbd, iubd, isbd, ksav = 0, ibdsav = 0, iflag;
  for (int k = 1; k <= NPT; ++k) hcol[k] = zero;
  for (int j = 1; j <= NPTM; ++j) {
    temp = zmat[knew][j];
    for (int k = 1; k <= NPT; ++k) hcol[k] += temp * zmat[k][j];
  }
  *alpha = hcol[knew];
  ha = half * *alpha;
  for (int i = 1; i <= N; ++i) glag[i] = bmat[knew][i];
  for (int k = 1; k <= NPT; ++k) {
    temp = zero;
    for (int j = 1; j <= N; ++j) temp += xpt[k][j] * xopt[j];
    temp = hcol[k] * temp;
    for (int i = 1; i <= N; ++i) glag[i] += temp * xpt[k][i];
  }
  presav = zero;
  for (int k = 1; k <= NPT; ++k) {
    if (k == kopt) continue;
    dderiv = zero;
    distsq = zero;
    for (int i = 1; i <= N; ++i) {
      temp = xpt[k][i] - xopt[i];
      dderiv += glag[i] * temp;
      distsq += temp * temp;
    }
    subd = adelt / std::sqrt(distsq);
    slbd = -subd;
    ilbd = 0;
    iubd = 0;
    sumin = dmin(one, subd);
    for (int i = 1; i <= N; ++i) {
      temp = xpt[k][i] - xopt[i];
      if (temp > zero) {
        if (slbd * temp < sl[i] - xopt[i]) {
          slbd = (sl[i] - xopt[i]) / temp;
          ilbd = -i;
        }
        if (subd * temp > su[i] - xopt[i]) {
          subd = dmax(sumin, (su[i] - xopt[i]) / temp);
          iubd = i;
        }
      } else if (temp < zero) {
        if (slbd * temp > su[i] - xopt[i]) {
          slbd = (su[i] - xopt[i]) / temp;
          ilbd = i;
        }
        if (subd * temp < sl[i] - xopt[i]) {
          subd = dmax(sumin, (sl[i] - xopt[i]) / temp);
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
      if (std::fabs(temp) > std::fabs(vlag)) {
        step = subd;
        vlag = temp;
        isbd = iubd;
      }
      tempd = half * dderiv;
      tempa = tempd - diff * slbd;
      tempb = tempd - diff * subd;
      if (tempa * tempb < zero) {
        temp = tempd * tempd / diff;
        if (std::fabs(temp) > std::fabs(vlag)) {
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
      if (std::fabs(temp) > std::fabs(vlag)) {
        step = subd;
        vlag = temp;
        isbd = iubd;
      }
      if (subd > half) {
        if (std::fabs(vlag) < .25) {
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
  for (int i = 1; i <= N; ++i) {
    temp = xopt[i] + stpsav * (xpt[ksav][i] - xopt[i]);
    xnew[i] = dmax(sl[i], dmin(su[i], temp));
  }
  if (ibdsav < 0) xnew[-ibdsav] = sl[-ibdsav];
  if (ibdsav > 0) xnew[ibdsav] = su[ibdsav];
  bigstp = adelt + adelt;
  iflag = 0;
L100:
  wfixsq = zero;
  ggfree = zero;
  for (int i = 1; i <= N; ++i) {
    w[i] = zero;
    tempa = dmin(xopt[i] - sl[i], glag[i]);
    tempb = dmax(xopt[i] - su[i], glag[i]);
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
    step = std::sqrt(temp / ggfree);
    ggfree = zero;
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
  for (int i = 1; i <= N; ++i) {
    if (w[i] == bigstp) {
      w[i] = -step * glag[i];
      xalt[i] = dmax(sl[i], dmin(su[i], xopt[i] + w[i]));
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
  for (int k = 1; k <= NPT; ++k) {
    temp = zero;
    for (int j = 1; j <= N; ++j) temp += xpt[k][j] * w[j];
    curv += hcol[k] * temp * temp;
  }
  if (iflag == 1) curv = -curv;
  if (curv > -gw && curv < -cnst * gw) {
    scale = -gw / curv;
    for (int i = 1; i <= N; ++i) {
      temp = xopt[i] + scale * w[i];
      xalt[i] = dmax(sl[i], dmin(su[i], temp));
    }
    temp = half * gw * scale;
    *cauchy = temp * temp;
  } else {
    temp = gw + half * curv;
    *cauchy = temp * temp;
  }
  if (iflag == 0) {
    for (int i = 1; i <= N; ++i) {
      glag[i] = -glag[i];
      w[N + i] = xalt[i];
    }
    csave = *cauchy;
    iflag = 1;
    goto L100;
  }
  if (csave > *cauchy) {
    for (int i = 1; i <= N; ++i) xalt[i] = w[N + i];
    *cauchy = csave;
  }
}

// ---------------------------------------------------------------- UPDATE
static void update(double bmat[NDIM + 1][N + 1], double zmat[NPT + 1][NPTM + 1], double* vlag,
                   double beta, double denom, int knew, double* w) {
  const double one = 1.0, zero = 0.0;
  double ztest = zero, temp, tempa, tempb, alpha, tau;
  for (int k = 1; k <= NPT; ++k)
    for (int j = 1; j <= NPTM; ++j) ztest = dmax(ztest, std::fabs(zmat[k][j]));
  ztest *= 1e-20;
  for (int j = 2; j <= NPTM; ++j) {
    if (std::fabs(zmat[knew][j]) > ztest) {
      double d1 = zmat[knew][1], d2 = zmat[knew][j];
      temp = std::sqrt(d1 * d1 + d2 * d2);
      tempa = zmat[knew][1] / temp;
      tempb = zmat[knew][j] / temp;
      for (int i = 1; i <= NPT; ++i) {
        temp = tempa * zmat[i][1] + tempb * zmat[i][j];
        zmat[i][j] = tempa * zmat[i][j] - tempb * zmat[i][1];
        zmat[i][1] = temp;
      }
    }
    zmat[knew][j] = zero;
  }
  for (int i = 1; i <= NPT; ++i) w[i] = zmat[knew][1] * zmat[i][1];
  alpha = w[knew];
  tau = vlag[knew];
  vlag[knew] -= one;
  temp = std::sqrt(denom);
  tempb = zmat[knew][1] / temp;
  tempa = tau / temp;
  for (int i = 1; i <= NPT; ++i) zmat[i][1] = tempa * zmat[i][1] - tempb * vlag[i];
  for (int j = 1; j <= N; ++j) {
    int jp = NPT + j;
    w[jp] = bmat[knew][j];
    tempa = (alpha * vlag[jp] - tau * w[jp]) / denom;
    tempb = (-beta * w[jp] - tau * vlag[jp]) / denom;
    for (int i = 1; i <= jp; ++i) {
      bmat[i][j] = bmat[i][j] + tempa * vlag[i] + tempb * w[i];
      if (i > NPT) bmat[jp][i - NPT] = bmat[i][j];
    }
  }
}

struct Stop {
  int nevals = 0;
  int maxeval = 0;
};

// ---------------------------------------------------------------- BOBYQB (+PRELIM, RESCUE)
// x, xl, xu are 1-based, in the RESCALED space; calfun receives rescaled x.
static BqResult bobyqb(double* x, const double* xl, const double* xu, double rhobeg,
                       double rhoend, Stop& stop, double* minf,
                       const std::function<double(const double*)>& calfun, double* sl,
                       double* su) {
  const double half = 0.5, one = 1.0, ten = 10.0, tenth = 0.1, two = 2.0, zero = 0.0;
  double xbase[N + 1], xpt[NPT + 1][N + 1], fval[NPT + 1], xopt[N + 1], gopt[N + 1], hq[NH + 1],
      pq[NPT + 1], bmat[NDIM + 1][N + 1], zmat[NPT + 1][NPTM + 1], xnew[N + 1], xalt[N + 1],
      d[N + 1], vlag[NDIM + 1], w[NDIM + NPT + 1];
  double gnew[N + 1], xbdi[N + 1], sv[N + 1], hs[N + 1], hred[N + 1];  // TRSBOX work (W(1..N)=GNEW)
  double glag[N + 1], hcol[NPT + 1], wa[2 * N + 1];                    // ALTMOV work
  double ptsaux[3][N + 1], ptsid[NPT + 1];                              // RESCUE work
  BqResult rc = BQ_SUCCESS;
  int nf = 0, kopt = 1, kbase, nresc, ntrits, itest, nfsav, knew = 0, ksav, ih;
  double f = 0, fbeg = 0, fsave, xoptsq, rho, delta, diffa, diffb, diffc = 0, dnorm, distsq,
         errbig, frhosq, bdtol, bdtest, curv, fracsq, sumpq, sum, temp, sumz, sumw, dsq = 0,
         crvmin = 0, adelt = 0, alpha = 0, cauchy = 0, suma, sumb, beta = 0, bsum, dx, denom = 0,
         delsq, scaden, biglsq, hdiag, den, fopt, vquad, diff = 0, ratio = 0, densav, pqold,
         gqsq, gisq, dist;
  double stepa = 0, stepb = 0;

  // ---- PRELIM (Powell's subroutine, inlined because it calls CALFUN)
  {
    const double rhosq = rhobeg * rhobeg;
    const double recip = one / rhosq;
    (void)recip;
    for (int j = 1; j <= N; ++j) {
      xbase[j] = x[j];
      for (int k = 1; k <= NPT; ++k) xpt[k][j] = zero;
      for (int i = 1; i <= NDIM; ++i) bmat[i][j] = zero;
    }
    for (int i = 1; i <= NH; ++i) hq[i] = zero;
    for (int k = 1; k <= NPT; ++k) {
      pq[k] = zero;
      for (int j = 1; j <= NPTM; ++j) zmat[k][j] = zero;
    }
    nf = 0;
    for (;;) {
      int nfm = nf, nfx = nf - N;
      ++nf;
      if (nfm <= 2 * N) {
        if (nfm >= 1 && nfm <= N) {
          stepa = rhobeg;
          if (su[nfm] == zero) stepa = -stepa;
          xpt[nf][nfm] = stepa;
        } else if (nfm > N) {
          stepa = xpt[nf - N][nfx];
          stepb = -rhobeg;
          if (sl[nfx] == zero) stepb = dmin(two * rhobeg, su[nfx]);
          if (su[nfx] == zero) stepb = dmax(-two * rhobeg, sl[nfx]);
          xpt[nf][nfx] = stepb;
        }
      }  // npt = 2n+1: the off-diagonal branch of PRELIM is never reached
      for (int j = 1; j <= N; ++j) {
        x[j] = dmin(dmax(xl[j], xbase[j] + xpt[nf][j]), xu[j]);
        if (xpt[nf][j] == sl[j]) x[j] = xl[j];
        if (xpt[nf][j] == su[j]) x[j] = xu[j];
      }
      stop.nevals++;
      f = calfun(x);
      fval[nf] = f;
      if (nf == 1) {
        fbeg = f;
        kopt = 1;
      } else if (f < fval[kopt]) {
        kopt = nf;
      }
      if (nf <= 2 * N + 1) {
        if (nf >= 2 && nf <= N + 1) {
          gopt[nfm] = (f - fbeg) / stepa;
          if (NPT < nf + N) {
            bmat[1][nfm] = -one / stepa;
            bmat[nf][nfm] = one / stepa;
            bmat[NPT + nfm][nfm] = -half * rhosq;
          }
        } else if (nf >= N + 2) {
          ih = nfx * (nfx + 1) / 2;
          temp = (f - fbeg) / stepb;
          diff = stepb - stepa;
          hq[ih] = two * (temp - gopt[nfx]) / diff;
          gopt[nfx] = (gopt[nfx] * stepb - temp * stepa) / diff;
          if (stepa * stepb < zero) {
            if (f < fval[nf - N]) {
              fval[nf] = fval[nf - N];
              fval[nf - N] = f;
              if (kopt == nf) kopt = nf - N;
              xpt[nf - N][nfx] = stepb;
              xpt[nf][nfx] = stepa;
            }
          }
          bmat[1][nfx] = -(stepa + stepb) / (stepa * stepb);
          bmat[nf][nfx] = -half / xpt[nf - N][nfx];
          bmat[nf - N][nfx] = -bmat[1][nfx] - bmat[nf][nfx];
          zmat[1][nfx] = std::sqrt(two) / (stepa * stepb);
          zmat[nf][nfx] = std::sqrt(half) / rhosq;
          zmat[nf - N][nfx] = -zmat[1][nfx] - zmat[nf][nfx];
        }
      }
      if (stop.maxeval > 0 && stop.nevals >= stop.maxeval) {
        rc = BQ_MAXEVAL;
        break;
      }
      if (!(nf < NPT)) break;
    }
  }
  xoptsq = zero;
  for (int i = 1; i <= N; ++i) {
    xopt[i] = xpt[kopt][i];
    xoptsq += xopt[i] * xopt[i];
  }
  fsave = fval[1];
  if (rc != BQ_SUCCESS) goto L720;
  kbase = 1;
  rho = rhobeg;
  delta = rho;
  nresc = nf;
  ntrits = 0;
  diffa = zero;
  diffb = zero;
  itest = 0;
  nfsav = nf;
L20:
  if (kopt != kbase) {
    ih = 0;
    for (int j = 1; j <= N; ++j) {
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) gopt[j] += hq[ih] * xopt[i];
        gopt[i] += hq[ih] * xopt[j];
      }
    }
    if (nf > NPT) {
      for (int k = 1; k <= NPT; ++k) {
        temp = zero;
        for (int j = 1; j <= N; ++j) temp += xpt[k][j] * xopt[j];
        temp = pq[k] * temp;
        for (int i = 1; i <= N; ++i) gopt[i] += temp * xpt[k][i];
      }
    }
  }
L60:
  trsbox(xpt, xopt, gopt, hq, pq, sl, su, delta, xnew, d, gnew, xbdi, sv, hs, hred, &dsq, &crvmin);
  dnorm = dmin(delta, std::sqrt(dsq));
  if (dnorm < half * rho) {
    ntrits = -1;
    temp = ten * rho;
    distsq = temp * temp;
    if (nf <= nfsav + 2) goto L650;
    errbig = dmax(dmax(diffa, diffb), diffc);
    frhosq = rho * .125 * rho;
    if (crvmin > zero && errbig > frhosq * crvmin) goto L650;
    bdtol = errbig / rho;
    for (int j = 1; j <= N; ++j) {
      bdtest = bdtol;
      if (xnew[j] == sl[j]) bdtest = gnew[j];   // W(J) == GNEW(J) left by TRSBOX
      if (xnew[j] == su[j]) bdtest = -gnew[j];
      if (bdtest < bdtol) {
        curv = hq[(j + j * j) / 2];
        for (int k = 1; k <= NPT; ++k) curv += pq[k] * (xpt[k][j] * xpt[k][j]);
        bdtest += half * curv * rho;
        if (bdtest < bdtol) goto L650;
      }
    }
    goto L680;
  }
  ++ntrits;
L90:
  if (dsq <= xoptsq * .001) {
    fracsq = xoptsq * .25;
    sumpq = zero;
    for (int k = 1; k <= NPT; ++k) {
      sumpq += pq[k];
      sum = -half * xoptsq;
      for (int i = 1; i <= N; ++i) sum += xpt[k][i] * xopt[i];
      w[NPT + k] = sum;
      temp = fracsq - half * sum;
      for (int i = 1; i <= N; ++i) {
        w[i] = bmat[k][i];
        vlag[i] = sum * xpt[k][i] + temp * xopt[i];
        int ip = NPT + i;
        for (int j = 1; j <= i; ++j) bmat[ip][j] = bmat[ip][j] + w[i] * vlag[j] + vlag[i] * w[j];
      }
    }
    for (int jj = 1; jj <= NPTM; ++jj) {
      sumz = zero;
      sumw = zero;
      for (int k = 1; k <= NPT; ++k) {
        sumz += zmat[k][jj];
        vlag[k] = w[NPT + k] * zmat[k][jj];
        sumw += vlag[k];
      }
      for (int j = 1; j <= N; ++j) {
        sum = (fracsq * sumz - half * sumw) * xopt[j];
        for (int k = 1; k <= NPT; ++k) sum += vlag[k] * xpt[k][j];
        w[j] = sum;
        for (int k = 1; k <= NPT; ++k) bmat[k][j] += sum * zmat[k][jj];
      }
      for (int i = 1; i <= N; ++i) {
        int ip = i + NPT;
        temp = w[i];
        for (int j = 1; j <= i; ++j) bmat[ip][j] += temp * w[j];
      }
    }
    ih = 0;
    for (int j = 1; j <= N; ++j) {
      w[j] = -half * sumpq * xopt[j];
      for (int k = 1; k <= NPT; ++k) {
        w[j] += pq[k] * xpt[k][j];
        xpt[k][j] -= xopt[j];
      }
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] = hq[ih] + w[i] * xopt[j] + xopt[i] * w[j];
        bmat[NPT + i][j] = bmat[NPT + j][i];
      }
    }
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

L190:  // ---- RESCUE (Powell's subroutine, inlined because it calls CALFUN)
  nfsav = nf;
  kbase = kopt;
  {
    const double sfrac = half / (double)NP;
    double winc = zero, fbase, vq, xp = 0, xq = 0, bet2 = 0, den2 = 0, dsqmin, vlmxsq;
    int nrem, kold, kn, ip, iq, iw, ihp = 0, ihq;
    sumpq = zero;
    for (int k = 1; k <= NPT; ++k) {
      distsq = zero;
      for (int j = 1; j <= N; ++j) {
        xpt[k][j] -= xopt[j];
        distsq += xpt[k][j] * xpt[k][j];
      }
      sumpq += pq[k];
      w[NDIM + k] = distsq;
      winc = dmax(winc, distsq);
      for (int j = 1; j <= NPTM; ++j) zmat[k][j] = zero;
    }
    ih = 0;
    for (int j = 1; j <= N; ++j) {
      w[j] = half * sumpq * xopt[j];
      for (int k = 1; k <= NPT; ++k) w[j] += pq[k] * xpt[k][j];
      for (int i = 1; i <= j; ++i) {
        ++ih;
        hq[ih] = hq[ih] + w[i] * xopt[j] + w[j] * xopt[i];
      }
    }
    for (int j = 1; j <= N; ++j) {
      xbase[j] += xopt[j];
      sl[j] -= xopt[j];
      su[j] -= xopt[j];
      xopt[j] = zero;
      ptsaux[1][j] = dmin(delta, su[j]);
      ptsaux[2][j] = dmax(-delta, sl[j]);
      if (ptsaux[1][j] + ptsaux[2][j] < zero) {
        temp = ptsaux[1][j];
        ptsaux[1][j] = ptsaux[2][j];
        ptsaux[2][j] = temp;
      }
      if (std::fabs(ptsaux[2][j]) < half * std::fabs(ptsaux[1][j])) ptsaux[2][j] = half * ptsaux[1][j];
      for (int i = 1; i <= NDIM; ++i) bmat[i][j] = zero;
    }
    fbase = fval[kopt];
    ptsid[1] = sfrac;
    for (int j = 1; j <= N; ++j) {
      int jp = j + 1, jpn = jp + N;
      ptsid[jp] = (double)j + sfrac;
      if (jpn <= NPT) {
        ptsid[jpn] = (double)j / (double)NP + sfrac;
        temp = one / (ptsaux[1][j] - ptsaux[2][j]);
        bmat[jp][j] = -temp + one / ptsaux[1][j];
        bmat[jpn][j] = temp + one / ptsaux[2][j];
        bmat[1][j] = -bmat[jp][j] - bmat[jpn][j];
        zmat[1][j] = std::sqrt(2.) / std::fabs(ptsaux[1][j] * ptsaux[2][j]);
        zmat[jp][j] = zmat[1][j] * ptsaux[2][j] * temp;
        zmat[jpn][j] = -zmat[1][j] * ptsaux[1][j] * temp;
      } else {
        bmat[1][j] = -one / ptsaux[1][j];
        bmat[jp][j] = one / ptsaux[1][j];
        bmat[j + NPT][j] = -half * (ptsaux[1][j] * ptsaux[1][j]);
      }
    }
    // NPT >= N+NP is false for npt = 2n+1: no further identifiers.
    nrem = NPT;
    kold = 1;
    kn = kopt;
  R80:
    for (int j = 1; j <= N; ++j) {
      temp = bmat[kold][j];
      bmat[kold][j] = bmat[kn][j];
      bmat[kn][j] = temp;
    }
    for (int j = 1; j <= NPTM; ++j) {
      temp = zmat[kold][j];
      zmat[kold][j] = zmat[kn][j];
      zmat[kn][j] = temp;
    }
    ptsid[kold] = ptsid[kn];
    ptsid[kn] = zero;
    w[NDIM + kn] = zero;
    --nrem;
    if (kn != kopt) {
      temp = vlag[kold];
      vlag[kold] = vlag[kn];
      vlag[kn] = temp;
      update(bmat, zmat, vlag, bet2, den2, kn, w);
      if (nrem == 0) goto R350;
      for (int k = 1; k <= NPT; ++k) w[NDIM + k] = std::fabs(w[NDIM + k]);
    }
  R120:
    dsqmin = zero;
    for (int k = 1; k <= NPT; ++k) {
      if (w[NDIM + k] > zero) {
        if (dsqmin == zero || w[NDIM + k] < dsqmin) {
          kn = k;
          dsqmin = w[NDIM + k];
        }
      }
    }
    if (dsqmin == zero) goto R260;
    for (int j = 1; j <= N; ++j) w[NPT + j] = xpt[kn][j];
    for (int k = 1; k <= NPT; ++k) {
      sum = zero;
      if (k == kopt) {
      } else if (ptsid[k] == zero) {
        for (int j = 1; j <= N; ++j) sum += w[NPT + j] * xpt[k][j];
      } else {
        ip = (int)ptsid[k];
        if (ip > 0) sum = w[NPT + ip] * ptsaux[1][ip];
        iq = (int)((double)NP * ptsid[k] - (double)(ip * NP));
        if (iq > 0) {
          iw = 1;
          if (ip == 0) iw = 2;
          sum += w[NPT + iq] * ptsaux[iw][iq];
        }
      }
      w[k] = half * sum * sum;
    }
    for (int k = 1; k <= NPT; ++k) {
      sum = zero;
      for (int j = 1; j <= N; ++j) sum += bmat[k][j] * w[NPT + j];
      vlag[k] = sum;
    }
    bet2 = zero;
    for (int j = 1; j <= NPTM; ++j) {
      sum = zero;
      for (int k = 1; k <= NPT; ++k) sum += zmat[k][j] * w[k];
      bet2 -= sum * sum;
      for (int k = 1; k <= NPT; ++k) vlag[k] += sum * zmat[k][j];
    }
    bsum = zero;
    distsq = zero;
    for (int j = 1; j <= N; ++j) {
      sum = zero;
      for (int k = 1; k <= NPT; ++k) sum += bmat[k][j] * w[k];
      int jp = j + NPT;
      bsum += sum * w[jp];
      for (int ipp = NPT + 1; ipp <= NDIM; ++ipp) sum += bmat[ipp][j] * w[ipp];
      bsum += sum * w[jp];
      vlag[jp] = sum;
      distsq += xpt[kn][j] * xpt[kn][j];
    }
    bet2 = half * distsq * distsq + bet2 - bsum;
    vlag[kopt] += one;
    den2 = zero;
    vlmxsq = zero;
    for (int k = 1; k <= NPT; ++k) {
      if (ptsid[k] != zero) {
        hdiag = zero;
        for (int j = 1; j <= NPTM; ++j) hdiag += zmat[k][j] * zmat[k][j];
        den = bet2 * hdiag + vlag[k] * vlag[k];
        if (den > den2) {
          kold = k;
          den2 = den;
        }
      }
      vlmxsq = dmax(vlmxsq, vlag[k] * vlag[k]);
    }
    if (den2 <= vlmxsq * .01) {
      w[NDIM + kn] = -w[NDIM + kn] - winc;
      goto R120;
    }
    goto R80;
  R260:
    for (int kpt = 1; kpt <= NPT; ++kpt) {
      if (ptsid[kpt] == zero) continue;
      if (stop.maxeval > 0 && stop.nevals >= stop.maxeval) {
        nf = -1;
        goto R350;
      }
      ih = 0;
      for (int j = 1; j <= N; ++j) {
        w[j] = xpt[kpt][j];
        xpt[kpt][j] = zero;
        temp = pq[kpt] * w[j];
        for (int i = 1; i <= j; ++i) {
          ++ih;
          hq[ih] += temp * w[i];
        }
      }
      pq[kpt] = zero;
      ip = (int)ptsid[kpt];
      iq = (int)((double)NP * ptsid[kpt] - (double)(ip * NP));
      if (ip > 0) {
        xp = ptsaux[1][ip];
        xpt[kpt][ip] = xp;
      }
      if (iq > 0) {
        xq = ptsaux[1][iq];
        if (ip == 0) xq = ptsaux[2][iq];
        xpt[kpt][iq] = xq;
      }
      vq = fbase;
      if (ip > 0) {
        ihp = (ip + ip * ip) / 2;
        vq += xp * (gopt[ip] + half * xp * hq[ihp]);
      }
      if (iq > 0) {
        ihq = (iq + iq * iq) / 2;
        vq += xq * (gopt[iq] + half * xq * hq[ihq]);
        if (ip > 0) {
          iw = (ihp > ihq ? ihp : ihq) - std::abs(ip - iq);
          vq += xp * xq * hq[iw];
        }
      }
      for (int k = 1; k <= NPT; ++k) {
        temp = zero;
        if (ip > 0) temp += xp * xpt[k][ip];
        if (iq > 0) temp += xq * xpt[k][iq];
        vq += half * pq[k] * temp * temp;
      }
      for (int i = 1; i <= N; ++i) {
        w[i] = dmin(dmax(xl[i], xbase[i] + xpt[kpt][i]), xu[i]);
        if (xpt[kpt][i] == sl[i]) w[i] = xl[i];
        if (xpt[kpt][i] == su[i]) w[i] = xu[i];
      }
      ++nf;
      stop.nevals++;
      f = calfun(w);
      fval[kpt] = f;
      if (f < fval[kopt]) kopt = kpt;
      diff = f - vq;
      for (int i = 1; i <= N; ++i) gopt[i] += diff * bmat[kpt][i];
      for (int k = 1; k <= NPT; ++k) {
        sum = zero;
        for (int j = 1; j <= NPTM; ++j) sum += zmat[k][j] * zmat[kpt][j];
        temp = diff * sum;
        if (ptsid[k] == zero) {
          pq[k] += temp;
        } else {
          ip = (int)ptsid[k];
          iq = (int)((double)NP * ptsid[k] - (double)(ip * NP));
          ihq = (iq * iq + iq) / 2;
          if (ip == 0) {
            hq[ihq] += temp * (ptsaux[2][iq] * ptsaux[2][iq]);
          } else {
            ihp = (ip * ip + ip) / 2;
            hq[ihp] += temp * (ptsaux[1][ip] * ptsaux[1][ip]);
            if (iq > 0) {
              hq[ihq] += temp * (ptsaux[1][iq] * ptsaux[1][iq]);
              iw = (ihp > ihq ? ihp : ihq) - std::abs(iq - ip);
              hq[iw] += temp * ptsaux[1][ip] * ptsaux[1][iq];
            }
          }
        }
      }
      ptsid[kpt] = zero;
    }
  R350:;
  }
  xoptsq = zero;
  if (kopt != kbase) {
    for (int i = 1; i <= N; ++i) {
      xopt[i] = xpt[kopt][i];
      xoptsq += xopt[i] * xopt[i];
    }
  }
  if (nf < 0) {
    nf = stop.maxeval;
    rc = BQ_MAXEVAL;
    goto L720;
  }
  nresc = nf;
  if (nfsav < nf) {
    nfsav = nf;
    goto L20;
  }
  if (ntrits > 0) goto L60;
L210:
  altmov(xpt, xopt, bmat, zmat, sl, su, kopt, knew, adelt, xnew, xalt, &alpha, &cauchy, glag, hcol,
         wa);
  for (int i = 1; i <= N; ++i) d[i] = xnew[i] - xopt[i];
L230:
  for (int k = 1; k <= NPT; ++k) {
    suma = zero;
    sumb = zero;
    sum = zero;
    for (int j = 1; j <= N; ++j) {
      suma += xpt[k][j] * d[j];
      sumb += xpt[k][j] * xopt[j];
      sum += bmat[k][j] * d[j];
    }
    w[k] = suma * (half * suma + sumb);
    vlag[k] = sum;
    w[NPT + k] = suma;
  }
  beta = zero;
  for (int jj = 1; jj <= NPTM; ++jj) {
    sum = zero;
    for (int k = 1; k <= NPT; ++k) sum += zmat[k][jj] * w[k];
    beta -= sum * sum;
    for (int k = 1; k <= NPT; ++k) vlag[k] += sum * zmat[k][jj];
  }
  dsq = zero;
  bsum = zero;
  dx = zero;
  for (int j = 1; j <= N; ++j) {
    dsq += d[j] * d[j];
    sum = zero;
    for (int k = 1; k <= NPT; ++k) sum += w[k] * bmat[k][j];
    bsum += sum * d[j];
    int jp = NPT + j;
    for (int i = 1; i <= N; ++i) sum += bmat[jp][i] * d[i];
    vlag[jp] = sum;
    bsum += sum * d[j];
    dx += d[j] * xopt[j];
  }
  beta = dx * dx + dsq * (xoptsq + dx + dx + half * dsq) + beta - bsum;
  vlag[kopt] += one;
  if (ntrits == 0) {
    denom = vlag[knew] * vlag[knew] + alpha * beta;
    if (denom < cauchy && cauchy > zero) {
      for (int i = 1; i <= N; ++i) {
        xnew[i] = xalt[i];
        d[i] = xnew[i] - xopt[i];
      }
      cauchy = zero;
      goto L230;
    }
    if (denom <= half * (vlag[knew] * vlag[knew])) {
      if (nf > nresc) goto L190;
      rc = BQ_ROUNDOFF;
      goto L720;
    }
  } else {
    delsq = delta * delta;
    scaden = zero;
    biglsq = zero;
    knew = 0;
    for (int k = 1; k <= NPT; ++k) {
      if (k == kopt) continue;
      hdiag = zero;
      for (int jj = 1; jj <= NPTM; ++jj) hdiag += zmat[k][jj] * zmat[k][jj];
      den = beta * hdiag + vlag[k] * vlag[k];
      distsq = zero;
      for (int j = 1; j <= N; ++j) {
        temp = xpt[k][j] - xopt[j];
        distsq += temp * temp;
      }
      temp = distsq / delsq;
      temp = dmax(one, temp * temp);
      if (temp * den > scaden) {
        scaden = temp * den;
        knew = k;
        denom = den;
      }
      biglsq = dmax(biglsq, temp * (vlag[k] * vlag[k]));
    }
    if (scaden <= half * biglsq) {
      if (nf > nresc) goto L190;
      rc = BQ_ROUNDOFF;
      goto L720;
    }
  }
L360:
  for (int i = 1; i <= N; ++i) {
    x[i] = dmin(dmax(xl[i], xbase[i] + xnew[i]), xu[i]);
    if (xnew[i] == sl[i]) x[i] = xl[i];
    if (xnew[i] == su[i]) x[i] = xu[i];
  }
  if (stop.maxeval > 0 && stop.nevals >= stop.maxeval) {
    rc = BQ_MAXEVAL;
    goto L720;
  }
  ++nf;
  stop.nevals++;
  f = calfun(x);
  if (ntrits == -1) {
    fsave = f;
    rc = BQ_XTOL;
    if (fsave < fval[kopt]) {
      *minf = f;
      return rc;
    }
    goto L720;
  }
  fopt = fval[kopt];
  vquad = zero;
  ih = 0;
  for (int j = 1; j <= N; ++j) {
    vquad += d[j] * gopt[j];
    for (int i = 1; i <= j; ++i) {
      ++ih;
      temp = d[i] * d[j];
      if (i == j) temp = half * temp;
      vquad += hq[ih] * temp;
    }
  }
  for (int k = 1; k <= NPT; ++k) {
    temp = w[NPT + k];
    vquad += half * pq[k] * (temp * temp);
  }
  diff = f - fopt - vquad;
  diffc = diffb;
  diffb = diffa;
  diffa = std::fabs(diff);
  if (dnorm > rho) nfsav = nf;
  if (ntrits > 0) {
    if (vquad >= zero) {
      rc = BQ_ROUNDOFF;
      goto L720;
    }
    ratio = (f - fopt) / vquad;
    if (ratio <= tenth) {
      delta = dmin(half * delta, dnorm);
    } else if (ratio <= .7) {
      delta = dmax(half * delta, dnorm);
    } else {
      delta = dmax(half * delta, dnorm + dnorm);
    }
    if (delta <= rho * 1.5) delta = rho;
    if (f < fopt) {
      ksav = knew;
      densav = denom;
      delsq = delta * delta;
      scaden = zero;
      biglsq = zero;
      knew = 0;
      for (int k = 1; k <= NPT; ++k) {
        hdiag = zero;
        for (int jj = 1; jj <= NPTM; ++jj) hdiag += zmat[k][jj] * zmat[k][jj];
        den = beta * hdiag + vlag[k] * vlag[k];
        distsq = zero;
        for (int j = 1; j <= N; ++j) {
          temp = xpt[k][j] - xnew[j];
          distsq += temp * temp;
        }
        temp = distsq / delsq;
        temp = dmax(one, temp * temp);
        if (temp * den > scaden) {
          scaden = temp * den;
          knew = k;
          denom = den;
        }
        biglsq = dmax(biglsq, temp * (vlag[k] * vlag[k]));
      }
      if (scaden <= half * biglsq) {
        knew = ksav;
        denom = densav;
      }
    }
  }
  update(bmat, zmat, vlag, beta, denom, knew, w);
  ih = 0;
  pqold = pq[knew];
  pq[knew] = zero;
  for (int i = 1; i <= N; ++i) {
    temp = pqold * xpt[knew][i];
    for (int j = 1; j <= i; ++j) {
      ++ih;
      hq[ih] += temp * xpt[knew][j];
    }
  }
  for (int jj = 1; jj <= NPTM; ++jj) {
    temp = diff * zmat[knew][jj];
    for (int k = 1; k <= NPT; ++k) pq[k] += temp * zmat[k][jj];
  }
  fval[knew] = f;
  for (int i = 1; i <= N; ++i) {
    xpt[knew][i] = xnew[i];
    w[i] = bmat[knew][i];
  }
  for (int k = 1; k <= NPT; ++k) {
    suma = zero;
    for (int jj = 1; jj <= NPTM; ++jj) suma += zmat[knew][jj] * zmat[k][jj];
    sumb = zero;
    for (int j = 1; j <= N; ++j) sumb += xpt[k][j] * xopt[j];
    temp = suma * sumb;
    for (int i = 1; i <= N; ++i) w[i] += temp * xpt[k][i];
  }
  for (int i = 1; i <= N; ++i) gopt[i] += diff * w[i];
  if (f < fopt) {
    kopt = knew;
    xoptsq = zero;
    ih = 0;
    for (int j = 1; j <= N; ++j) {
      xopt[j] = xnew[j];
      xoptsq += xopt[j] * xopt[j];
      for (int i = 1; i <= j; ++i) {
        ++ih;
        if (i < j) gopt[j] += hq[ih] * d[i];
        gopt[i] += hq[ih] * d[j];
      }
    }
    for (int k = 1; k <= NPT; ++k) {
      temp = zero;
      for (int j = 1; j <= N; ++j) temp += xpt[k][j] * d[j];
      temp = pq[k] * temp;
      for (int i = 1; i <= N; ++i) gopt[i] += temp * xpt[k][i];
    }
  }
  if (ntrits > 0) {
    for (int k = 1; k <= NPT; ++k) {
      vlag[k] = fval[k] - fval[kopt];
      w[k] = zero;
    }
    for (int j = 1; j <= NPTM; ++j) {
      sum = zero;
      for (int k = 1; k <= NPT; ++k) sum += zmat[k][j] * vlag[k];
      for (int k = 1; k <= NPT; ++k) w[k] += sum * zmat[k][j];
    }
    for (int k = 1; k <= NPT; ++k) {
      sum = zero;
      for (int j = 1; j <= N; ++j) sum += xpt[k][j] * xopt[j];
      w[k + NPT] = w[k];
      w[k] = sum * w[k];
    }
    gqsq = zero;
    gisq = zero;
    for (int i = 1; i <= N; ++i) {
      sum = zero;
      for (int k = 1; k <= NPT; ++k) sum = sum + bmat[k][i] * vlag[k] + xpt[k][i] * w[k];
      if (xopt[i] == sl[i]) {
        temp = dmin(zero, gopt[i]);
        gqsq += temp * temp;
        temp = dmin(zero, sum);
        gisq += temp * temp;
      } else if (xopt[i] == su[i]) {
        temp = dmax(zero, gopt[i]);
        gqsq += temp * temp;
        temp = dmax(zero, sum);
        gisq += temp * temp;
      } else {
        gqsq += gopt[i] * gopt[i];
        gisq += sum * sum;
      }
      vlag[NPT + i] = sum;
    }
    ++itest;
    if (gqsq < ten * gisq) itest = 0;
    if (itest >= 3) {
      const int imax = NPT > NH ? NPT : NH;
      for (int i = 1; i <= imax; ++i) {
        if (i <= N) gopt[i] = vlag[NPT + i];
        if (i <= NPT) pq[i] = w[NPT + i];
        if (i <= NH) hq[i] = zero;
        itest = 0;
      }
    }
  }
  if (ntrits == 0) goto L60;
  if (f <= fopt + tenth * vquad) goto L60;
  {
    double t1 = two * delta, t2 = ten * rho;
    distsq = dmax(t1 * t1, t2 * t2);
  }
L650:
  knew = 0;
  for (int k = 1; k <= NPT; ++k) {
    sum = zero;
    for (int j = 1; j <= N; ++j) {
      temp = xpt[k][j] - xopt[j];
      sum += temp * temp;
    }
    if (sum > distsq) {
      knew = k;
      distsq = sum;
    }
  }
  if (knew > 0) {
    dist = std::sqrt(distsq);
    if (ntrits == -1) {
      delta = dmin(tenth * delta, half * dist);
      if (delta <= rho * 1.5) delta = rho;
    }
    ntrits = 0;
    adelt = dmax(dmin(tenth * dist, delta), rho);
    dsq = adelt * adelt;
    goto L90;
  }
  if (ntrits == -1) goto L680;
  if (ratio > zero) goto L60;
  if (dmax(delta, dnorm) > rho) goto L60;
L680:
  if (rho > rhoend) {
    delta = half * rho;
    ratio = rho / rhoend;
    if (ratio <= 16.) {
      rho = rhoend;
    } else if (ratio <= 250.) {
      rho = std::sqrt(ratio) * rhoend;
    } else {
      rho = tenth * rho;
    }
    delta = dmax(delta, rho);
    ntrits = 0;
    nfsav = nf;
    goto L60;
  }
  // NLopt: after the optional final Newton step (L360 with ntrits == -1) the result is XTOL.
  if (ntrits == -1) goto L360;
  rc = BQ_XTOL;
L720:
  if (fval[kopt] <= fsave) {
    for (int i = 1; i <= N; ++i) {
      x[i] = dmin(dmax(xl[i], xbase[i] + xopt[i]), xu[i]);
      if (xopt[i] == sl[i]) x[i] = xl[i];
      if (xopt[i] == su[i]) x[i] = xu[i];
    }
    f = fval[kopt];
  }
  *minf = f;
  return rc;
}
}  // namespace bq

// NLopt 2.6.1 nlopt_set_default_initial_step (options.c) for one coordinate.
static inline double bq_default_step(double x, double lb, double ub) {
  double step = HUGE_VAL;
  if (!std::isinf(ub) && !std::isinf(lb) && (ub - lb) * 0.25 < step && ub > lb) step = (ub - lb) * 0.25;
  if (!std::isinf(ub) && ub - x < step && ub > x) step = (ub - x) * 0.75;
  if (!std::isinf(lb) && x - lb < step && x > lb) step = (x - lb) * 0.75;
  if (std::isinf(step)) {
    if (!std::isinf(ub) && std::fabs(ub - x) < std::fabs(step)) step = (ub - x) * 1.1;
    if (!std::isinf(lb) && std::fabs(x - lb) < std::fabs(step)) step = (x - lb) * 1.1;
  }
  if (std::isinf(step) || step == 0.0 || std::fabs(step) < 2.2250738585072014e-308) step = x;
  if (std::isinf(step) || step == 0.0) step = 1;
  return step;
}

// nlopt::opt(LN_BOBYQA, 3) with set_xtol_rel(xtol_rel), set_maxeval(maxeval), bounds lb/ub,
// optimize(x, minf).  x (0-based, 3 entries) must already be inside the bounds
// (the reference clamps it, optim.cpp:629-634).  Returns the NLopt result code; x is the
// unscaled final point (NLopt writes it back even on MAXEVAL).  *nevals = evaluations used.
static inline BqResult bobyqa_minimize(double* x, const double* lb, const double* ub,
                                       double xtol_rel, int maxeval, const BqFunc& f,
                                       double* minf, int* nevals) {
  using namespace bq;
  double dxs[N], s[N];
  for (int i = 0; i < N; ++i) dxs[i] = bq_default_step(x[i], lb[i], ub[i]);
  // nlopt_compute_rescaling
  for (int i = 0; i < N; ++i) s[i] = 1.0;
  {
    int i = 1;
    for (; i < N && dxs[i] == dxs[i - 1]; ++i) {}
    if (i < N)
      for (i = 1; i < N; ++i) s[i] = dxs[i] / dxs[0];
  }
  double xs[N + 1], xl[N + 1], xu[N + 1], sl[N + 1], su[N + 1];
  for (int i = 0; i < N; ++i) {
    xs[i + 1] = x[i] / s[i];
    xl[i + 1] = lb[i] / s[i];
    xu[i + 1] = ub[i] / s[i];
  }
  const double rhobeg = std::fabs(dxs[0] / s[0]);
  const double rhoend = xtol_rel * rhobeg;  // xtol_abs = 0
  for (int j = 1; j <= N; ++j) {
    const double temp = xu[j] - xl[j];
    if (temp < rhobeg + rhobeg) {
      *nevals = 0;
      return BQ_INVALID_ARGS;
    }
    sl[j] = xl[j] - xs[j];
    su[j] = xu[j] - xs[j];
    if (sl[j] >= -rhobeg) {
      if (sl[j] >= 0.0) {
        xs[j] = xl[j];
        sl[j] = 0.0;
        su[j] = temp;
      } else {
        xs[j] = xl[j] + rhobeg;
        sl[j] = -rhobeg;
        su[j] = bq::dmax(xu[j] - xs[j], rhobeg);
      }
    } else if (su[j] <= rhobeg) {
      if (su[j] <= 0.0) {
        xs[j] = xu[j];
        sl[j] = -temp;
        su[j] = 0.0;
      } else {
        xs[j] = xu[j] - rhobeg;
        sl[j] = bq::dmin(xl[j] - xs[j], -rhobeg);
        su[j] = rhobeg;
      }
    }
  }
  Stop stop;
  stop.maxeval = maxeval;
  auto calfun = [&](const double* xsc) {
    double xu_[N];
    for (int i = 0; i < N; ++i) xu_[i] = xsc[i + 1] * s[i];  // nlopt_unscale
    return f(xu_);
  };
  BqResult rc = bobyqb(xs, xl, xu, rhobeg, rhoend, stop, minf, calfun, sl, su);
  for (int i = 0; i < N; ++i) x[i] = xs[i + 1] * s[i];
  *nevals = stop.nevals;
  return rc;
}

}  // namespace oracle
