#!/bin/bash
# end-of-round record on the final tree: the default bench line, the refine launches' tails
# (PMVS_REFINE_TAIL=1), and a rocprofv3 kernel-trace --stats of the same bench command shape
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ac; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-900
PMVS_REFINE_TAIL=1 timeout -k 10 240 python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline > $O/tail.json 2> $O/tail.err || { tail $O/tail.err; exit 1; }
grep "refine tail" $O/tail.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { echo KT_FAIL; tail $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/kt
head -4 $O/kernel_stats.csv | cut -c1-200
