#!/bin/bash
# tools/gpu_r03p.sh <tag> -- the refine launch tails of one C3 step (PMVS_REFINE_TAIL=1), then the
# profiling passes of tools/gpu_round.sh prof (kernel-trace stats; FETCH_SIZE / WRITE_SIZE in
# separate --pmc runs for the C3 loop and the C2 batch)
set -o pipefail
TAG=${1:-r03p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PMVS_REFINE_TAIL=1 timeout -k 10 300 python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/tail.json 2> $O/tail.err && \
bash $R/tools/gpu_round.sh prof $TAG
rc=$?; echo "rc=$rc"; exit $rc
