#!/bin/bash
# row-slot neighbour walks (PMVS_NB_ROWS=1, product) against cell slots (libpmvs_amd_cells.so):
# the filter / expansion parity tests on the product, then C3 steps of both libraries (sweep_walks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06u; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_filter.py tests/test_gpu_expand.py tests/test_gpu_parity_matrix.py \
  "tests/test_gpu_c3_full.py::test_c3_4k_filter_pass_matches_oracle" tests/test_gpu_loop_scale.py -k "not plain_1080p and not schedule_gap" \
  -m gpu -x -q --timeout 200 --timeout-method thread --durations=5 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
STEPS=2 WARMUP=1 bash tools/sweep_walks.sh r06u "main cells main cells" || exit 1
