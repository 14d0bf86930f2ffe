set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_filter.py $R/tests/test_gpu_expand.py $R/tests/test_gpu_loop_scale.py $R/tests/test_gpu_cluster.py $R/tests/test_gpu_poison.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 500 python3 -u $R/bench.py --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; exit $rc
