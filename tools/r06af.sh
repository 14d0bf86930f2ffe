#!/bin/bash
# the opt-in long GPU cases (PMVS_LONG_TESTS=1) on the final tree: the 8K C5 two-cluster exchange and
# the long schedule-gap cases
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06af; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && PMVS_LONG_TESTS=1 timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_c5_exchange.py tests/test_gpu_loop_scale.py -k "c5_two_clusters_two_iterations or schedule_gap" -m gpu -v -s --timeout 1050 --timeout-method thread --durations=5 > $O/long_tests.txt 2>&1; rc=$?
grep -E "C5 cluster|PASS|FAIL|passed|failed|s call" $O/long_tests.txt | cut -c1-300
exit $rc
