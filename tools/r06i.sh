#!/bin/bash
# the whole GPU suite + smoke() on the round-6 tree, then a kernel trace of one untimed-warmup C3 step
# reduced to the GPU's idle gaps (tools/ktgaps.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06i; mkdir -p $O
bash $R/tools/gpu_round.sh suite r06i || { echo SUITE_FAIL; grep -E "FAILED|ERROR|passed|failed" $O/pytest_all.log | tail -20; exit 1; }
grep -E "passed|failed" $O/pytest_all.log | tail -2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1 || { echo KT_FAIL; tail $O/kt.log; exit 1; }
python3 $R/tools/ktgaps.py $O/kt > $O/gaps.json && python3 $R/tools/ktsum.py $O/kt > $O/kt_summary.json && rm -rf $O/kt && head -c 2500 $O/gaps.json
