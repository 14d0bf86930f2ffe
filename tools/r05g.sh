set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
B="python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c2"
timeout -k 10 300 $B > $O/bench_1206.json 2> $O/bench_1206.err && \
PMVS_REFINE_LARGE_CONFIG=228010 timeout -k 10 300 $B > $O/bench_L228010.json 2> $O/bench_L228010.err && \
PMVS_REFINE_LARGE_CONFIG=226014 timeout -k 10 300 $B > $O/bench_L226014.json 2> $O/bench_L226014.err && \
PMVS_REFINE_CONFIG=228010 timeout -k 10 300 $B > $O/bench_A228010.json 2> $O/bench_A228010.err && \
PMVS_REFINE_CONFIG=226014 timeout -k 10 300 $B > $O/bench_A226014.json 2> $O/bench_A226014.err
echo "rc=$?"
