#!/bin/bash
# commit rounds trace, lane optimizer phase split (LANE_PROFILE build) and a kernel trace of one C3 step on the new defaults
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g; mkdir -p $O
PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_laneprof.so timeout -k 10 300 python -u tools/refine_sizes.py 300000 2000 > $O/prof.jsonl 2> $O/prof.err || { echo PROF_FAIL; tail $O/prof.err; exit 1; }
python3 -c "
import json
for l in open('$O/prof.jsonl'):
    d=json.loads(l); p=d['prof']; r=d['rounds']
    print(d['n'], d['refine_ms'], 'per round: step %.0f eval %.0f | trsbox %.0f altmov %.0f update %.0f' % (p[0]/r, p[1]/r, p[3]/r, p[4]/r, p[5]/r))"
PMVS_COMMIT_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/ctrace.out 2> $O/ctrace.err || { echo CT_FAIL; tail $O/ctrace.err; exit 1; }
grep -c '^\[commit\]' $O/ctrace.err
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1 || { echo KT_FAIL; tail $O/kt.log; exit 1; }
python3 $R/tools/ktsum.py $O/kt > $O/kt_summary.json && rm -rf $O/kt && python3 -c "import json; d=json.load(open('$O/kt_summary.json')); print(d['span_ms'], d['busy_ms']); [print(k, v) for k, v in list(d['kernels'].items())[:30]]"
