set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_loop_hash.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "hash or refine_batch or c2" > $O/tests.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "rc=$?"
