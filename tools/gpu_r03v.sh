#!/bin/bash
# tools/gpu_r03v.sh <tag> [tests] -- filter/expansion/loop GPU tests, a kernel-trace profile of one
# bench step, and the bench line (each step under its own limit, chained with &&)
set -o pipefail
TAG=${1:-r03v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
TESTS=${2:-"test_gpu_filter.py test_gpu_expand.py test_gpu_loop_scale.py test_gpu_cluster.py test_gpu_poison.py"}
T=""; for t in $TESTS; do T="$T $R/tests/$t"; done
timeout -k 10 600 python3 -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1 && \
timeout -k 10 500 python3 -u $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; exit $rc
