set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_dist.py tests/test_gpu_cluster.py tests/test_gpu_loop_hash.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py --no-c2 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_loop_scale.py -m gpu -x -v --timeout 300 --timeout-method thread -k plain_1080p > $O/tests_scale.log 2>&1
echo "rc=$?"
