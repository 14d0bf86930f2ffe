#!/bin/bash
# tools/gpu_r03j.sh <tag> -- expansion / loop GPU tests, the expansion phase profile of one C3 step,
# and the bench line (each step under its own limit, chained with &&)
set -o pipefail
TAG=${1:-r03j}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python3 -u -m pytest $R/tests/test_gpu_expand.py $R/tests/test_gpu_loop_scale.py $R/tests/test_gpu_filter.py $R/tests/test_gpu_dist.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
PMVS_EXPAND_PROFILE=1 timeout -k 10 300 python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/phase.json 2> $O/phase.err && \
timeout -k 10 500 python3 -u $R/bench.py --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; exit $rc
