# round 5 final measurement: the cell-bit sorts validated (expansion / filter / C3 / sharding tests),
# smoke + the default bench line, then the kernel-trace stats and HBM PMC passes (gpu_round.sh prof)
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_filter.py tests/test_gpu_c3_full.py tests/test_gpu_dist.py tests/test_gpu_cluster.py tests/test_gpu_parity_matrix.py tests/test_gpu_loop_hash.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
bash tools/gpu_round.sh bench r05z && bash tools/gpu_round.sh prof r05z
echo "rc=$?"
