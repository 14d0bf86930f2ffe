#!/bin/bash
# lane-form refine kernel: SQ counters over one 2000-candidate launch (refine_sizes.py), one pass each,
# plus the device's counter list (to find the instruction-cache counters)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="$R/tools/refine_sizes.py 300000 2000"
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
grep -io "SQC[A-Z_]*ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $O/counters.txt | sort -u > $O/icache_counters.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_SMEM \
  --output-format csv -d $O/sq_a -o run -- python3 $W > $O/sq_a.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  --output-format csv -d $O/sq_b -o run -- python3 $W > $O/sq_b.log 2>&1 && \
python3 $R/tools/pmc_summary.py $O/sq_a > $O/sq_a.json && python3 $R/tools/pmc_summary.py $O/sq_b > $O/sq_b.json && \
rm -rf $O/sq_a $O/sq_b
rc=$?
cat $O/icache_counters.txt
python3 - <<PY
import json
for p in ("sq_a", "sq_b"):
    d = json.load(open("$O/" + p + ".json"))
    for k, v in d.items():
        if "refine_lane" in k:
            print(p, k, json.dumps(v))
PY
exit $rc
