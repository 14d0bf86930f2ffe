#!/bin/bash
# tools/gpu_r03x.sh <tag> -- the sharded-expansion / distributed / RCCL GPU tests and the
# filter/expansion parity tests (each step under its own limit)
set -o pipefail
TAG=${1:-r03x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_expand.py $R/tests/test_gpu_dist.py $R/tests/test_gpu_rccl.py $R/tests/test_gpu_cluster.py $R/tests/test_gpu_filter.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
