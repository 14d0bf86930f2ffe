#!/bin/bash
# tools/sweep_quad.sh -- C3 one-iteration filter time vs resident quad_lane_kernel wavefronts per CU
# (PMVS_QUAD_WAVES_PER_CU; 0 = one lane per job, uncapped grid).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_quad}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in 0 2 4 8; do
  PMVS_QUAD_WAVES_PER_CU=$w timeout -k 10 240 python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline \
    > $O/w$w.json 2> $O/w$w.err || exit 1
  echo "quad waves/CU $w $(python3 -c "import json; d=json.load(open('$O/w$w.json')); i=d['iterations'][0]; print(d['ms_per_step'], i['filter_ms'], d['checks']['model_hash'])")"
done
echo sweep done
