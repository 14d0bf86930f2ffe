#!/bin/bash
# postProcess fused into the lane-form refine kernel: parity tests, then the C3 bench with it on and off
# (PMVS_LANE_POST), and a kernel trace of one step with it on (idle gaps and per-form durations)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06j; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_matrix.py tests/test_gpu_expand.py tests/test_gpu_loop_hash.py tests/test_gpu_golden.py "tests/test_gpu_c3_full.py::test_c3_full_size_step_and_first_waves_match_oracle" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for P in 1 0 1; do
  PMVS_LANE_POST=$P timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c2 > $O/b$P.out 2> $O/b$P.err || { echo "B${P}_FAIL"; tail $O/b$P.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$P.out').read().strip().splitlines()[-1]); print('post fused', $P, d['ms_per_step'], d['value'], d['checks']['model_hash'][:8], d['stage_s_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1 || { echo KT_FAIL; tail $O/kt.log; exit 1; }
python3 $R/tools/ktgaps.py $O/kt > $O/gaps.json && python3 $R/tools/ktsum.py $O/kt > $O/kt_summary.json && rm -rf $O/kt && head -c 3000 $O/gaps.json
