#!/bin/bash
# tools/eb_breakdown.sh -- findEmptyBlocks (empty_blocks_kernel) cost split on C3: kernel traces of one
# loop iteration with the product library and timing-only variants built with
#   make -C cmvs-pmvs_amd variant VAR=ebsort|ebbin|ebwalk VARTU=pmvs_filter VARFLAGS=-DNBX_SKIP_SORT|-DEBX_SKIP_BIN|-DEBX_SKIP_WALK
# Only the first wave sees identical input across variants (the skips change the candidates):
# python3 tools/eb_breakdown.py <out dir> compares the launches before the first prepare_kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-eb_breakdown}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in main ebsort ebbin ebwalk; do
  L=$R/cmvs-pmvs_amd/libpmvs_amd_$v.so
  [ "$v" = main ] && L=$R/cmvs-pmvs_amd/libpmvs_amd.so
  PMVS_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit 1
done
echo breakdown done
