#!/bin/bash
# tools/sweep_walks.sh OUT "lib1 lib2 ..." -- one C3 step (3 iterations) per library variant of the
# filter TU (make variant VARTU=pmvs_filter VAR=... VARFLAGS="-DPMVS_NB_CAP=..."; "main" = product):
# step time, filter and expansion time, model hash.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_walks}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for lib in ${2:-main}; do
  i=$((i+1))
  L=$R/cmvs-pmvs_amd/libpmvs_amd_$lib.so
  [ "$lib" = main ] && L=$R/cmvs-pmvs_amd/libpmvs_amd.so
  PMVS_AMD_LIB=$L timeout -k 10 240 python3 $R/bench.py --steps ${STEPS:-1} --warmup ${WARMUP:-0} --no-c2 --no-cpu-baseline \
    > $O/$lib.$i.json 2> $O/$lib.$i.err || exit 1
  echo "$lib $(python3 -c "import json; d=json.load(open('$O/$lib.$i.json')); it=d['iterations']; print(d['ms_per_step'], [round(i['filter_ms']) for i in it], [round(i.get('expand_ms',0)) for i in it], d['checks']['model_hash'][:12])")"
done
echo sweep done
