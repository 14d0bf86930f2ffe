# round 5, last kernel changes (commit rounds over the undecided list, used bits by lane groups):
# expansion / filter / C3 / sharding tests, smoke + the default bench line, a traced step (summarised)
set -o pipefail
O=gpurun_out/r05ae; mkdir -p $O
R=$(pwd)
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_filter.py tests/test_gpu_c3_full.py tests/test_gpu_dist.py tests/test_gpu_cluster.py tests/test_gpu_parity_matrix.py tests/test_gpu_loop_hash.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
bash tools/gpu_round.sh bench r05ae && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $R/$O/kt.log 2>&1) && \
python3 tools/ktsum.py $O/kt > $O/kt.json && rm -rf $O/kt
echo "rc=$?"
