# round 5: findEmptyBlocks' unbounded re-walk, setRefImage in collect order, label sweeps' plain flag
# reads: tests, bench, a traced step (summarised), then the opt-in C5 exchange test with error tracing
set -o pipefail
O=gpurun_out/r05aa; mkdir -p $O
R=$(pwd)
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_filter.py tests/test_gpu_c3_full.py tests/test_gpu_parity_matrix.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $R/$O/kt.log 2>&1) && \
python3 tools/ktsum.py $O/kt > $O/kt.json && rm -rf $O/kt && \
PMVS_LONG_TESTS=1 PMVS_TRACE_ERRORS=1 timeout -k 10 700 python3 -u -m pytest tests/test_gpu_c5_exchange.py -m gpu -x -v -s --timeout 680 --timeout-method thread > $O/c5x.log 2>&1
echo "rc=$?"
