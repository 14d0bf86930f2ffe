#!/bin/bash
# tools/gpu_r03q.sh <tag> -- filter / expansion / loop / seed GPU tests, the refine launch tails of one
# C3 step (PMVS_REFINE_TAIL=1), and the bench line (each step under its own limit, chained with &&)
set -o pipefail
TAG=${1:-r03q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 800 python3 -u -m pytest $R/tests/test_gpu_filter.py $R/tests/test_gpu_expand.py $R/tests/test_gpu_loop_scale.py $R/tests/test_gpu_poison.py $R/tests/test_gpu_seed.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
PMVS_REFINE_TAIL=1 timeout -k 10 300 python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/tail.json 2> $O/tail.err && \
timeout -k 10 500 python3 -u $R/bench.py --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; exit $rc
