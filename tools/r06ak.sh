#!/bin/bash
# final tree: the whole GPU suite, smoke(), then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ak; mkdir -p $O
cd $R && timeout -k 10 850 python3 -u -m pytest tests/ -m gpu -x -v --timeout 400 --timeout-method thread --durations=10 > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" >> $O/gpu_tests.txt 2>&1 || { echo SMOKE_FAIL; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 250 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
