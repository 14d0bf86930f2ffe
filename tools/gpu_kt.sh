#!/bin/bash
# tools/gpu_kt.sh <tag> -- rocprofv3 kernel-trace stats of one C3 bench step (no PMC)
set -o pipefail
TAG=${1:-kt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
