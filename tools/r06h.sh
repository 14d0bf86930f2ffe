#!/bin/bash
# commit rounds: grid rounds to the end (PMVS_COMMIT_GRID_ROUNDS=0) against the one-workgroup tail after
# 1 / 2 grid rounds; one traced C3 bench (warmup + 1 step) each, model hash and commit kernels printed
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for G in ${GS:-2 1 0}; do
  PMVS_COMMIT_GRID_ROUNDS=$G timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$G -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/b$G.out 2> $O/b$G.err || { echo "B${G}_FAIL"; tail $O/b$G.err; exit 1; }
  python3 $R/tools/ktsum.py $O/kt$G > $O/kt${G}_summary.json && rm -rf $O/kt$G || exit 1
  python3 - $O $G <<'PY' || exit 1
import json, sys
o, g = sys.argv[1], sys.argv[2]
b = json.loads(open(f"{o}/b{g}.out").read().strip().splitlines()[-1])
k = json.load(open(f"{o}/kt{g}_summary.json"))
cm = {n: v for n, v in k["kernels"].items() if n.startswith("cm_")}
tot = sum(v[0] for v in cm.values()); nl = sum(v[1] for v in cm.values())
print(g, b["ms_per_step"], b["value"], b["checks"]["model_hash"][:8], "span", k["span_ms"], "commit kernels ms", round(tot, 1), "launches", nl)
print("  ", {n: v for n, v in cm.items()})
PY
done
cd $R && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_loop_hash.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
