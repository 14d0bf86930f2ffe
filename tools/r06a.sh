#!/bin/bash
# round 6: lane-form refine kernel -- parity of its layouts against the oracle, then small-batch timing
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
  -k "refine_configs and (300000 or 300004 or 300008 or 132042)" > $O/parity.log 2>&1 || { echo PARITY_FAIL; tail -30 $O/parity.log; exit 1; }
tail -8 $O/parity.log
timeout -k 10 300 python -u tools/small_chains.py 300000,132042 2500 > $O/small.jsonl 2> $O/small.err || { echo SMALL_FAIL; tail $O/small.err; exit 1; }
cat $O/small.jsonl
timeout -k 10 400 python -u tools/refine_sizes.py 300000,132042,226014 2000,5000,10000,20000,40000 > $O/sizes.jsonl 2> $O/sizes.err || { echo SIZES_FAIL; tail $O/sizes.err; exit 1; }
cat $O/sizes.jsonl
