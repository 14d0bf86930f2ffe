#!/bin/bash
# lane form after the DPP / swizzle / readlane hand-offs: parity, small-batch timing and round profile
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
  -k "refine_configs and (300000 or 300004 or 300008)" > $O/parity.log 2>&1 || { echo PARITY_FAIL; tail -30 $O/parity.log; exit 1; }
tail -5 $O/parity.log
timeout -k 10 300 python -u tools/refine_sizes.py 300000 2000,5000,7000,10000 > $O/sizes.jsonl 2> $O/sizes.err || { echo SIZES_FAIL; tail $O/sizes.err; exit 1; }
cat $O/sizes.jsonl | cut -c1-200
PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_laneprof.so timeout -k 10 300 python -u tools/refine_sizes.py 300000 2000 > $O/prof.jsonl 2> $O/prof.err || { echo PROF_FAIL; tail $O/prof.err; exit 1; }
python3 -c "
import json
for l in open('$O/prof.jsonl'):
    d=json.loads(l); p=d['prof']; r=d['rounds']
    print(d['n'], d['refine_ms'], 'step_cyc/round %.0f eval_cyc/round %.0f' % (p[0]/r, p[1]/r))"
