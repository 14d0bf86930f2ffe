# round 5: addPatch's depth-map updates skip cells a stale read shows cannot change: expansion tests,
# the C3 bench (hash), a traced step (summarised)
set -o pipefail
O=gpurun_out/r05ak; mkdir -p $O
R=$(pwd)
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_expand.py tests/test_gpu_c3_full.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $R/$O/kt.log 2>&1) && \
python3 tools/ktsum.py $O/kt > $O/kt.json && rm -rf $O/kt
echo "rc=$?"
