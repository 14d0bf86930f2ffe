#!/bin/bash
# kernel trace of the current tree (one C3 warmup + one step), summarised by tools/ktsum.py / ktgaps.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06y; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1 || { echo KT_FAIL; tail $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 $R/tools/ktsum.py $O/kt > $O/kt_summary.json || exit 1
python3 $R/tools/ktgaps.py $O/kt > $O/kt_gaps.txt 2>&1 || true
rm -rf $O/kt
python3 -c "import json; d=json.load(open('$O/kt_summary.json')); print(d['span_ms'], d['busy_ms']); [print(k, v) for k, v in list(d['kernels'].items())[:32]]"
