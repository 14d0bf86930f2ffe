# round 5: lean loop mode (pass buffers released before a cluster exchange): the cluster / C4 tests in
# lean mode (bit-exact against the oracle), then the opt-in C5 exchange test
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMVS_LOOP_LEAN=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_c4.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/lean_tests.log 2>&1 && \
PMVS_LONG_TESTS=1 PMVS_TRACE_ERRORS=1 timeout -k 10 750 python3 -u -m pytest tests/test_gpu_c5_exchange.py -m gpu -x -v -s --timeout 740 --timeout-method thread > $O/c5x.log 2>&1
echo "rc=$?"
