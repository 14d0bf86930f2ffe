#!/bin/bash
# tools/diag_r04k.sh -- the C5 test alone (allocation failures traced), then smoke() and the default
# bench line
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04k; mkdir -p $O; cd $R
ok() { local rc=$1; [ $rc -le 1 ]; }
PMVS_TRACE_ERRORS=1 timeout -k 10 420 python3 -u -m pytest tests/test_gpu_c5.py -m gpu -v --timeout 400 --timeout-method thread -s > $O/pytest_c5.log 2>&1; ok $? || exit 3
timeout -k 10 200 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err
