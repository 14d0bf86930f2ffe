set -o pipefail
O=$(pwd)/gpurun_out/r05q; mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/ht -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/ht.log 2>&1
rc=$?
cd $O/ht && python3 $R/tools/api_gaps.py . > $O/api_summary.txt 2>&1
find $O/ht -name "*hip_api_trace.csv" -delete
find $O/ht -name "*kernel_trace.csv" -size +30M -delete
exit $rc
