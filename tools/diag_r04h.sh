#!/bin/bash
# tools/diag_r04h.sh -- round-4 checks: filter/expand GPU tests (neighbour re-walks, commit tail), C4/C5,
# the commit-tail sweep and a one-iteration kernel trace of the bench
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04h; mkdir -p $O; cd $R
ok() { local rc=$1; [ $rc -le 1 ]; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_filter.py tests/test_gpu_expand.py -m gpu -v --timeout 250 --timeout-method thread --durations=0 > $O/pytest_fe.log 2>&1; ok $? || exit 3
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_c4_c5.py -m gpu -v --timeout 650 --timeout-method thread --durations=0 -s > $O/pytest_c4c5.log 2>&1; ok $? || exit 4
bash tools/sweep_quad.sh r04h PMVS_COMMIT_TAIL "0 256 1024" > $O/sweep_tail.txt 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline > $O/prof.log 2>&1
