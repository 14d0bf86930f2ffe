#!/bin/bash
# tools/diag_r04j.sh -- the whole GPU suite as the round end runs it (durations), allocation
# failures traced (PMVS_TRACE_ERRORS)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04j; mkdir -p $O; cd $R
PMVS_TRACE_ERRORS=1 timeout -k 10 1080 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=0 > $O/pytest_all.log 2>&1
