#!/bin/bash
# phase times of the C5 unit test, and the C3 full-size tests' durations (GPU-suite budget)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06k; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_c5.py tests/test_gpu_c3_full.py -m gpu -x -v -s --timeout 500 --timeout-method thread --durations=0 > $O/pytest.log 2>&1; rc=$?
grep -E "^\[c5|passed|failed|PASSED|FAILED|s call|s setup" $O/pytest.log | head -30; exit $rc
