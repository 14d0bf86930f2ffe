#!/bin/bash
# tools/sweep.sh -- refine-kernel tuning sweep (TSLOTS x waves per CU) on the GPU box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep}; mkdir -p $O
for ts in ${TS:-1608 1616 3208 3216 4808}; do for w in ${WPC:-2 3 4 8}; do
  PMVS_REFINE_CONFIG=$ts PMVS_REFINE_WAVES_PER_CU=$w timeout -k 10 120 python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/b_${ts}_${w}.json 2>/dev/null || exit 1
done; done
echo sweep done
