// tests/csrc/bq_objectives.h -- objectives of the BOBYQA host tests (bq_host.cpp: bobyqa_dev.h's state
// machine; bql_host.cpp: bobyqa_lane.h's lane-distributed form).  Kinds 0-2 are oracle_bobyqa_test's
// (oracle/pmvs_oracle.cpp); 3-5 are rough on purpose -- hash noise, a quantised staircase and a
// plateau at 2.0 like the refine objective's invalid-texture value -- so that trajectories take the
// trust region's rare branches (RESCUE, the roundoff exits, ALTMOV's Cauchy step).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline double bq_noise(const double* v, int salt) {
  uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)salt;
  for (int i = 0; i < 3; ++i) {
    uint64_t b;
    memcpy(&b, &v[i], 8);
    h ^= b + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
  }
  return (double)(h >> 11) * (1.0 / 9007199254740992.0) - 0.5;
}

static inline double bq_objective(int kind, const double* v) {
  if (kind == 0) return (v[0] - 1.5) * (v[0] - 1.5) + 2 * (v[1] - 3) * (v[1] - 3) + 0.5 * (v[2] + 2) * (v[2] + 2) + 0.1 * v[0] * v[1];
  if (kind == 1) {
    const double a = 1 - v[0], b = v[1] - v[0] * v[0], c = v[2] - v[1] * v[1];
    return a * a + 100 * b * b + 100 * c * c;
  }
  if (kind == 2) return (v[0] - 1) * (v[0] - 1) + (v[1] - 40) * (v[1] - 40) + (v[2] + 50) * (v[2] + 50);
  const double q = 0.3 * (v[0] - 0.7) * (v[0] - 0.7) + 0.01 * (v[1] - 5) * (v[1] - 5) + 0.02 * (v[2] + 3) * (v[2] + 3);
  if (kind == 3) return q + 1e-3 * bq_noise(v, 3);
  if (kind == 4) return floor(q * 64.0) / 64.0;
  if (kind == 6) return 1e10 * v[0] * v[0] + (v[1] - 1) * (v[1] - 1) + 1e-10 * v[2] * v[2];
  if (kind == 7) return fabs(v[0] - 0.3) + 2.0 * fabs(v[1] + 1.0) + 0.5 * fabs(v[2] - 2.0);
  if (kind == 8) return bq_noise(v, 8);
  if (kind == 9) return floor(v[0] * 3.0) + floor(v[1] * 0.5) * floor(v[2] * 0.5) + 1e-9 * q;
  // kind 5: 2.0 outside a ball (the refine objective's "too few valid textures"), rough inside
  const double r2 = v[0] * v[0] + 0.01 * v[1] * v[1] + 0.01 * v[2] * v[2];
  if (r2 > 4.0) return 2.0;
  return 1.0 - exp(-q) + 0.05 * bq_noise(v, 5);
}
