#!/bin/bash
# re-entry check of the round-6 tree: the 3840x2160 (level 1) C5-shaped exchange test, smoke(), then
# the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06t; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 320 python3 -u -m pytest "tests/test_gpu_c5_exchange.py::test_c5_shaped_two_clusters_exchange_small" -m gpu -x -v -s --timeout 300 --timeout-method thread --durations=3 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
grep -E "C5 cluster|passed|failed|s call" $O/pytest.log | cut -c1-400
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
