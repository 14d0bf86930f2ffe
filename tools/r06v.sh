#!/bin/bash
# the CPU oracle over the whole iteration-1 expansion and a full filter pass (tools/cpu_full_iteration.py):
# the measured CPU rates beside the bench's extrapolated cpu_baseline (round-5 advisor)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06v; mkdir -p $O
( while true; do sleep 50; echo "alive $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd $R && timeout -k 10 1000 python3 -u tools/cpu_full_iteration.py > $O/cpu_full.jsonl 2> $O/cpu_full.err || { echo CPU_FULL_FAIL; tail $O/cpu_full.err; exit 1; }
cat $O/cpu_full.jsonl
