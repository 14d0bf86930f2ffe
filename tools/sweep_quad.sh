#!/bin/bash
# tools/sweep_quad.sh OUT VAR "V1 V2 ..." -- C3 one-iteration filter time and model hash vs one
# quad-fit setting, e.g.
#   tools/sweep_quad.sh r04f PMVS_QUAD_LDS_ROWS "0 64 96 128 160"   (0 = every fit one lane per job)
#   tools/sweep_quad.sh r02z PMVS_QUAD_WAVES_PER_CU "0 2 4 8"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_quad}; mkdir -p $O
VAR=${2:-PMVS_QUAD_LDS_ROWS}
cd /tmp && export TMPDIR=/tmp
for w in ${3:-0 96}; do
  env $VAR=$w timeout -k 10 240 python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline \
    > $O/$VAR.$w.json 2> $O/$VAR.$w.err || exit 1
  echo "$VAR $w $(python3 -c "import json; d=json.load(open('$O/$VAR.$w.json')); i=d['iterations'][0]; print(d['ms_per_step'], i['filter_ms'], d['checks']['model_hash'])")"
done
echo sweep done
