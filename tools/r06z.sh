#!/bin/bash
# filterSmallGroups label sweeps: all-vertex pointer jump every PMVS_LAB_JUMP-th sweep (1 = rounds 4-6)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z; mkdir -p $O
cd $R
for J in 1 2 4 8 1 4; do
  PMVS_LAB_JUMP=$J timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --no-c2 --no-cpu-baseline > $O/j$J.json 2> $O/j$J.err || exit 1
  echo "jump $J $(python3 -c "import json; d=json.load(open('$O/j$J.json')); it=d['iterations']; print(d['ms_per_step'], [round(i['filter_ms']) for i in it], d['checks']['model_hash'][:12])")"
done
PMVS_LAB_JUMP=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_filter.py "tests/test_gpu_c3_full.py::test_c3_4k_filter_pass_matches_oracle" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
