# round 5, final tree: the opt-in long GPU cases (PMVS_LONG_TESTS=1)
set -o pipefail
O=gpurun_out/r05ah; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMVS_LONG_TESTS=1 timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_c5_exchange.py tests/test_gpu_loop_scale.py -k "exchange or hard" -m gpu -v -s --timeout 700 --timeout-method thread > $O/long.log 2>&1
echo "rc=$?"
