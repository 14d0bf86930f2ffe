// tests/csrc/bql_host.cpp -- host build of the LANE-DISTRIBUTED BOBYQA (cmvs-pmvs_amd/csrc/bobyqa_lane.h:
// a wavefront emulated by 64-element arrays) with the objectives of bq_host.cpp, so that its
// trajectories can be compared with bobyqa_dev.h's evaluation for evaluation (tests/test_bobyqa_host.py).
#include <math.h>
#include "bobyqa_lane.h"
#include "bq_objectives.h"

using namespace pmvsdev;

#if defined(BQL_COUNT)
long long pmvsdev::bql::bql_hits[16];
extern "C" const long long* bql_host_hits() { return pmvsdev::bql::bql_hits; }
#endif

extern "C" int bql_host_run(int kind, const double* x0, int maxeval, double* xout, double* fout, double* frec,
                            int maxrec, int* nrec) {
  const double lb[3] = {-HUGE_VAL, -23.99999, -23.99999}, ub[3] = {HUGE_VAL, 23.99999, 23.99999};
  int cnt = 0;
  auto f = [&](const double* xe) {
    const double v = bq_objective(kind, xe);
    if (cnt < maxrec) frec[cnt] = v;
    cnt++;
    return v;
  };
  int nev = 0;
  bql::BqlU U;
  bql::BqlProf prof;
  const int rc = bql::bobyqa(U, f, x0, lb, ub, 1e-7, maxeval, xout, fout, &nev, prof);
  *nrec = cnt;
  return rc;
}
