set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bobyqa.py -m gpu -x -v --timeout 200 --timeout-method thread -k "configs or refine_batch or c2 or bobyqa" > $O/parity.log 2>&1 && \
timeout -k 10 200 python3 -u tools/bq_lanes.py 3 > $O/bq_lanes.jsonl 2>&1 && \
timeout -k 10 400 python3 -u tools/refine_sizes.py 1206,132042,226014,246014,228010 2000,10000,80000 > $O/sizes.jsonl 2> $O/sizes.err
echo "rc=$?"
