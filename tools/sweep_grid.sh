#!/bin/bash
# tools/sweep_grid.sh -- C3 one-iteration loop time vs persistent single-wave workgroups per CU
# (PMVS_GRID_WAVES_PER_CU: pre/post, organizer and filter kernels; neighbour walks use twice it).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_grid}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in 8 12 16 4; do
  PMVS_GRID_WAVES_PER_CU=$g timeout -k 10 240 python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline \
    > $O/g$g.json 2> $O/g$g.err || exit 1
  echo "gpc $g $(python3 -c "import json; d=json.load(open('$O/g$g.json')); i=d['iterations'][0]; print(d['ms_per_step'], i['expand_ms'], i['filter_ms'], d['checks']['model_hash'])")"
done
echo sweep done
