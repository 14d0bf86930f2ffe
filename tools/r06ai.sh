#!/bin/bash
# walk kernels' counters on one C3 iteration: L2 hit/miss, and the SQ issue / wait / instruction mix
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ai; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc -o run -- python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-cpu-baseline --no-c2 > $O/tcc.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d $O/sq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --iterations 1 --no-cpu-baseline --no-c2 > $O/sq.log 2>&1 || { echo PMC_FAIL; tail $O/tcc.log $O/sq.log; exit 1; }
python3 $R/tools/pmc_summary.py $O/tcc > $O/tcc.json && python3 $R/tools/pmc_summary.py $O/sq > $O/sq.json && rm -rf $O/tcc $O/sq
python3 -c "
import json
for f in ('tcc','sq'):
    d=json.load(open('$O/'+f+'.json'))
    ks = d.get('kernels', d)
    for k,v in ks.items():
        if any(x in k for x in ('neighbor_kernel<1024','empty_blocks_kernel<1024','refine_split','depth_map','filter_refimage','post_kernel','pre_kernel')): print(f, k[:50], v)
"
