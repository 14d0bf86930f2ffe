#!/bin/bash
# tools/gpu_phase.sh <tag> -- host wall time per expansion phase (PMVS_EXPAND_PROFILE=1, synchronising
# at phase ends) for one C3 loop step
set -o pipefail
TAG=${1:-phase}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PMVS_EXPAND_PROFILE=1 timeout -k 10 400 python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; exit $rc
