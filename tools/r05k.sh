set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
B="python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c2"
timeout -k 10 300 $B > $O/bench_def.json 2> $O/bench_def.err && \
PMVS_REFINE_SMALL_CONFIG=248010 timeout -k 10 300 $B > $O/bench_S248010.json 2> $O/bench_S248010.err && \
PMVS_REFINE_SMALL_CONFIG=226014 timeout -k 10 300 $B > $O/bench_S226014.json 2> $O/bench_S226014.err && \
PMVS_REFINE_SMALL_CONFIG=228010 timeout -k 10 300 $B > $O/bench_S228010.json 2> $O/bench_S228010.err && \
PMVS_REFINE_SMALL_CONFIG=248010 PMVS_REFINE_LARGE_CONFIG=227012 timeout -k 10 300 $B > $O/bench_S248010_L227012.json 2> $O/bench_S248010_L227012.err
echo "rc=$?"
