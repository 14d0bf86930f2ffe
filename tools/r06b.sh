#!/bin/bash
# lane form: optimizer-step / objective split per round (LANE_PROFILE builds), evaluation inlined
# (laneprof) or out of line (lanecall), and waves per SIMD
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
for v in laneprof:2 lanecall:2 laneprof:1; do
  lib=${v%%:*}; w=${v##*:}
  PMVS_LANE_WPS=$w PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_$lib.so timeout -k 10 300 python -u tools/refine_sizes.py 300000 2000,10000 > $O/${lib}_w$w.jsonl 2> $O/${lib}_w$w.err || { echo FAIL; tail $O/${lib}_w$w.err; exit 1; }
  cat $O/${lib}_w$w.jsonl
done
