#!/bin/bash
# tools/sweep_loop.sh -- C3 loop schedule sweep: expansion wave (parents per chunk) x min_candidates.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_loop}; mkdir -p $O
for cfg in ${CFGS:-32768:65536 32768:131072 65536:262144}; do
  w=${cfg%%:*}; m=${cfg##*:}
  timeout -k 10 200 env PMVS_GRID_WAVES_PER_CU=${GPC:-8} python3 $R/bench.py --steps 1 --warmup 1 --no-c2 --no-cpu-baseline --wave $w --min-candidates $m \
    > $O/loop_${w}_${m}_g${GPC:-8}.json 2> $O/loop_${w}_${m}_g${GPC:-8}.err || exit 1
  echo "$w $m $(python3 -c "import json; d=json.load(open('$O/loop_${w}_${m}_g${GPC:-8}.json')); print(d['value'], d['ms_per_step'], d['model_patches'], d['stage_s_per_step'], [(i['waves'], i['candidates'], i['added']) for i in d['iterations']])")"
done
echo sweep done
