#!/bin/bash
# tools/sweep_c2.sh -- refine-kernel tuning sweep on the C2 batch (bench.py --only-c2):
# PMVS_REFINE_CONFIG (texture slots * 100 + chains per wavefront) x refine wavefronts per CU.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_c2}; mkdir -p $O
for ts in ${TS:-1608 1604 804}; do for w in ${WPC:-4 8 12}; do
  PMVS_REFINE_CONFIG=$ts PMVS_REFINE_WAVES_PER_CU=$w timeout -k 10 120 python3 $R/bench.py --only-c2 > $O/c2_${ts}_${w}.json 2>$O/c2_${ts}_${w}.err || exit 1
  echo "$ts $w $(python3 -c "import json,sys; d=json.load(open('$O/c2_${ts}_${w}.json'))['refine_c2']; print(d['value'], d['roofline']['kernel_ms_avg'])")"
done; done
echo sweep done
