#!/bin/bash
# tools/gpu_round.sh -- one gpurun call: parity tests, smoke, bench, rocprofv3 kernel stats and
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs, kernel-trace only).
# Every GPU step has its own time limit; steps are chained with &&.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest $R/tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python3 $R/bench.py "$@" > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/pmc_write.log 2>&1
rc=$?
echo "gpu_round rc=$rc"
exit $rc
