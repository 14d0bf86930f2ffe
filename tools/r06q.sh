#!/bin/bash
# the 1920x1080 C5-shaped two-cluster exchange test, then the CPU oracle over the whole iteration-1
# expansion and a full filter pass (tools/cpu_full_iteration.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06q; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_c5_exchange.py::test_c5_shaped_two_clusters_exchange_small" -m gpu -x -v -s --timeout 280 --timeout-method thread --durations=3 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
grep -E "C5 cluster|passed|failed|s call" $O/pytest.log | cut -c1-400
timeout -k 10 850 python3 -u tools/cpu_full_iteration.py > $O/cpu_full.jsonl 2> $O/cpu_full.err || { echo CPU_FULL_FAIL; tail $O/cpu_full.err; exit 1; }
tail -1 $O/cpu_full.jsonl
