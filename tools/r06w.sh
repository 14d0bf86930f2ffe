#!/bin/bash
# walk-phase cycle split (libpmvs_amd_nbprof.so, -DNB_PROFILE): one C3 step, the nb_prof lines per
# filter pass and expansion
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06w; mkdir -p $O
cd $R && PMVS_AMD_LIB=$R/cmvs-pmvs_amd/libpmvs_amd_nbprof.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline \
  > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
grep nb_prof $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], [round(i['filter_ms']) for i in d['iterations']], d['checks']['model_hash'][:12])"
# the one-pass radius + unit sum in the walks' setup (product) against the previous library
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_filter.py tests/test_gpu_expand.py tests/test_gpu_parity_matrix.py \
  "tests/test_gpu_c3_full.py::test_c3_4k_filter_pass_matches_oracle" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
STEPS=2 WARMUP=1 bash tools/sweep_walks.sh r06w "main prev main prev" || exit 1
