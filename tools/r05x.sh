# round 5: lane-group list kernels (first_cell one atomic per wave), vis_rows 4 targets per thread,
# pre / post at 3 waves per SIMD; depth maps 1 vs 4 targets per thread: tests, bench, traced steps
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filter.py tests/test_gpu_expand.py tests/test_gpu_dist.py tests/test_gpu_cluster.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
(cd /tmp && export TMPDIR=/tmp && for d in 1 4; do
   PMVS_DM_TARGETS=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt$d -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $R/$O/kt$d.log 2>&1 || exit 1
   python3 $R/tools/ktsum.py $R/$O/kt$d > $R/$O/kt$d.json && rm -rf $R/$O/kt$d || exit 1
 done)
echo "rc=$?"
