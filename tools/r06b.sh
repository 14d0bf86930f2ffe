#!/bin/bash
# lane form: optimizer-step / objective split per round (LANE_PROFILE build) and waves-per-SIMD
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
for w in 2 1; do
  PMVS_LANE_WPS=$w PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_laneprof.so timeout -k 10 300 python -u tools/refine_sizes.py 300000 2000,10000 > $O/prof_w$w.jsonl 2> $O/prof_w$w.err || { echo FAIL; tail $O/prof_w$w.err; exit 1; }
  cat $O/prof_w$w.jsonl
done
