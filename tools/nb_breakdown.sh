#!/bin/bash
# tools/nb_breakdown.sh -- neighbor_kernel (filterNeighbor) cost split on C3, one loop iteration:
# the product library vs timing-only variants built with
#   make -C cmvs-pmvs_amd variant VAR=nbsort|nblls|nbboth VARTU=pmvs_filter VARFLAGS=-DNBX_SKIP_SORT|-DNBX_SKIP_LLS|both
# Only the first filter pass sees identical input across variants (the skips change what it keeps).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-nb_breakdown}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in main nbsort nblls nbboth; do
  L=$R/cmvs-pmvs_amd/libpmvs_amd_$v.so
  [ "$v" = main ] && L=$R/cmvs-pmvs_amd/libpmvs_amd.so
  PMVS_AMD_LIB=$L timeout -k 10 240 python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline \
    > $O/$v.json 2> $O/$v.err || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('$O/$v.json')); print(d['iterations'][0]['filter_ms'], d['ms_per_step'])")"
done
echo breakdown done
