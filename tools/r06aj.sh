#!/bin/bash
# the delta-chain pool as one {item, next} array: parity (refine,
# golden, parity-matrix counters, expansion, loops), then C3 steps against the previous library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06aj; mkdir -p $O
cd $R && timeout -k 10 500 python3 -u -m pytest tests/test_gpu_filter.py tests/test_gpu_parity_matrix.py tests/test_gpu_expand.py "tests/test_gpu_c3_full.py::test_c3_full_size_step_and_first_waves_match_oracle" \
  tests/test_gpu_seed.py tests/test_gpu_loop_scale.py -k "not plain_1080p and not schedule_gap" \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
STEPS=2 WARMUP=1 bash tools/sweep_walks.sh r06aj "main prev main prev" || exit 1
