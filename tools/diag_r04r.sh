#!/bin/bash
# tools/diag_r04r.sh -- the whole GPU suite (durations) and smoke(), as the round end runs them
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04r; mkdir -p $O; cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=0 > $O/pytest_all.log 2>&1
rc=$?
[ $rc -le 1 ] && timeout -k 10 200 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
exit $rc
