// tests/csrc/bq_host.cpp -- host build of the DEVICE reverse-communication BOBYQA
// (cmvs-pmvs_amd/csrc/bobyqa_dev.h) so its trajectories can be compared with the callback
// oracle (oracle/bobyqa_oracle.h) on the CPU.  Same objectives as oracle_bobyqa_test (bq_objectives.h).
#include <math.h>
#include "bobyqa_dev.h"
#include "bq_objectives.h"

using namespace pmvsdev;

static double objective(int kind, const double* v) { return bq_objective(kind, v); }

extern "C" int bq_host_run(int kind, const double* x0, int maxeval, double* xout, double* fout, double* frec,
                           int maxrec, int* nrec) {
  BqState st;
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999}, ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  double x[3] = {x0[0], x0[1], x0[2]};
  bq_begin(st, x, lb, ub, 1e-7, maxeval);
  double f = 0.0;
  int cnt = 0;
  while (bq_step(st, f) == BQ_NEED_F) {
    f = objective(kind, st.xeval);
    if (cnt < maxrec) frec[cnt] = f;
    cnt++;
  }
  for (int i = 0; i < 3; ++i) xout[i] = st.xout[i];
  *fout = st.minf;
  *nrec = cnt;
  return st.rc;
}
