set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 240 python3 -u tools/bq_lanes.py 3 1 > $O/bq_lanes.jsonl 2>&1 && \
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 400 python3 -u tools/refine_sizes.py 1206,202032,202040,203024,204016 2000,10000,40000,80000 > $O/sizes.jsonl 2> $O/sizes.err
echo "rc=$?"
