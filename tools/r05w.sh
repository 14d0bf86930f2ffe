# round 5: texture loops' bounded unroll (pre / post / setRefImage without spills), their residency
# variants (PMVS_PREPOST_WPE 3 / 4), frontier label sweeps, findEmptyBlocks breakdown.  Traces are
# summarised on the box (tools/ktsum.py) and the raw CSVs removed (gpurun_out returns <= 64 MiB).
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filter.py tests/test_gpu_expand.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
(cd /tmp && export TMPDIR=/tmp && for v in main wpe3 wpe4 ebsort ebbin ebwalk; do
   L=$R/cmvs-pmvs_amd/libpmvs_amd_$v.so; [ "$v" = main ] && L=$R/cmvs-pmvs_amd/libpmvs_amd.so
   IT=3; case $v in eb*) IT=1;; esac
   PMVS_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 1 --warmup 1 --iterations $IT --no-cpu-baseline --no-c2 > $R/$O/kt_$v.log 2>&1 || exit 1
   python3 $R/tools/ktsum.py $R/$O/kt_$v > $R/$O/kt_$v.json && rm -rf $R/$O/kt_$v || exit 1
 done)
echo "rc=$?"
