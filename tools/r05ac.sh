# round 5: the expansion's error codes (capacity overflow vs device memory) and the opt-in C5 exchange
# test at pyramid level 1 in lean mode
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_expand.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/expand.log 2>&1 && \
PMVS_LONG_TESTS=1 PMVS_TRACE_ERRORS=1 timeout -k 10 750 python3 -u -m pytest tests/test_gpu_c5_exchange.py -m gpu -x -v -s --timeout 740 --timeout-method thread > $O/c5x.log 2>&1
echo "rc=$?"
