# round 5: cooperative label fixpoint + cooperative commit rounds (tests, bench, trace), findEmptyBlocks breakdown
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_filter.py tests/test_gpu_cluster.py tests/test_gpu_dist.py tests/test_gpu_c3_full.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $R/$O/kt.log 2>&1) && \
bash tools/eb_breakdown.sh r05v/eb && python3 tools/eb_breakdown.py gpurun_out/r05v/eb > $O/eb_summary.txt
echo "rc=$?"
