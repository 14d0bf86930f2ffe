#!/bin/bash
# tools/diag_r04q.sh -- expansion / filter / parity GPU tests, the default bench line and a kernel
# trace of one C3 step (round 4, batched texture grabs)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04q; mkdir -p $O; cd $R
ok() { local rc=$1; [ $rc -le 1 ]; }
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_filter.py tests/test_gpu_parity.py tests/test_gpu_parity_matrix.py tests/test_gpu_seed.py tests/test_gpu_golden.py -m gpu -v --timeout 250 --timeout-method thread --durations=0 > $O/pytest.log 2>&1; ok $? || exit 3
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 4
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1
