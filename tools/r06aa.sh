#!/bin/bash
# the whole GPU suite on the current tree (as the driver runs it), then smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r06aa}; mkdir -p $O
cd $R && timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 > $O/gpu_tests.txt 2>&1; rc=$?
tail -25 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" >> $O/gpu_tests.txt 2>&1 || { echo SMOKE_FAIL; exit 1; }
tail -1 $O/gpu_tests.txt
