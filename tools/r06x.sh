#!/bin/bash
# interleaved delta-chain cursors in the walks: parity, the walk-phase split (nbprof build), then C3
# steps of the product against the previous commit's filter TU (libpmvs_amd_prev.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06x; mkdir -p $O
cd $R && timeout -k 10 450 python3 -u -m pytest tests/test_gpu_filter.py tests/test_gpu_expand.py tests/test_gpu_parity_matrix.py \
  "tests/test_gpu_c3_full.py::test_c3_4k_filter_pass_matches_oracle" tests/test_gpu_loop_scale.py -k "not plain_1080p and not schedule_gap" \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
PMVS_AMD_LIB=$R/cmvs-pmvs_amd/libpmvs_amd_nbprof.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline \
  > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
grep nb_prof $O/bench.err
STEPS=2 WARMUP=1 bash tools/sweep_walks.sh r06x "main prev main prev" || exit 1
