#!/bin/bash
# tools/sweep_variants.sh -- C2 refine throughput of kernel-TU variants (make variant VAR=...) x
# refine configs x wavefronts per CU:  SPECS="lib:config:wpc ..." bash tools/sweep_variants.sh tag
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep_var}; mkdir -p $O
for spec in $SPECS; do
  IFS=: read lib ts w <<< "$spec"
  L=$R/cmvs-pmvs_amd/libpmvs_amd${lib:+_$lib}.so
  [ "$lib" = main ] && L=$R/cmvs-pmvs_amd/libpmvs_amd.so
  PMVS_AMD_LIB=$L PMVS_REFINE_CONFIG=$ts PMVS_REFINE_WAVES_PER_CU=$w timeout -k 10 150 python3 $R/bench.py --only-c2 > $O/c2_${lib}_${ts}_${w}.json 2>$O/c2_${lib}_${ts}_${w}.err || exit 1
  echo "$lib $ts $w $(python3 -c "import json,sys; d=json.load(open('$O/c2_${lib}_${ts}_${w}.json'))['refine_c2']; print(d['value'], d['roofline']['kernel_ms_avg'])")"
done
echo sweep done
