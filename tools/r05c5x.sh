# round 5: the 50-view 720p two-process shard test, then the opt-in C5 exchange test
set -o pipefail
O=gpurun_out/r05c5x; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dist.py -k ring50 -m gpu -x -v -s --timeout 380 --timeout-method thread > $O/dist.log 2>&1 && \
PMVS_LONG_TESTS=1 timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_c5_exchange.py -m gpu -x -v -s --timeout 1000 --timeout-method thread > $O/c5x.log 2>&1
echo "rc=$?"
