#!/bin/bash
# commit: early rejection of candidates whose checkCounts already fails -- parity tests, the rounds
# per commit (PMVS_COMMIT_TRACE), one traced C3 step (commit kernels) and the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06l; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_loop_hash.py tests/test_gpu_parity_matrix.py tests/test_gpu_loop_scale.py tests/test_gpu_cluster.py tests/test_gpu_c5.py -m gpu -x -q --durations=8 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
grep -E 's call|passed|failed' $O/pytest.log | tail -10
PMVS_COMMIT_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/ctrace.out 2> $O/ctrace.err || { echo CT_FAIL; tail $O/ctrace.err; exit 1; }
python3 - $O <<'PY'
import re, statistics, sys, json
rows = []
for l in open(sys.argv[1] + "/ctrace.err"):
    m = re.match(r"\[commit\] nk=(\d+) nlive=(\d+) na=(\d+):(.*)", l)
    if m: rows.append(list(map(int, m.group(4).split())))
print("commits", len(rows), "rounds mean", round(statistics.mean(len(r) for r in rows), 2), "max", max(len(r) for r in rows))
b = json.loads(open(sys.argv[1] + "/ctrace.out").read().strip().splitlines()[-1]); print("hash", b["checks"]["model_hash"][:8])
PY
timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c2 > $O/b.out 2> $O/b.err || { echo B_FAIL; tail $O/b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/b.out').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['checks']['model_hash'][:8], d['stage_s_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1 || { echo KT_FAIL; tail $O/kt.log; exit 1; }
python3 $R/tools/ktgaps.py $O/kt > $O/gaps.json && python3 $R/tools/ktsum.py $O/kt > $O/kt_summary.json && rm -rf $O/kt
python3 -c "
import json; k=json.load(open('$O/kt_summary.json'))['kernels']; cm={n:v for n,v in k.items() if n.startswith('cm_')}
print('commit kernels ms', round(sum(v[0] for v in cm.values()),1), 'launches', sum(v[1] for v in cm.values())); print(cm)"
