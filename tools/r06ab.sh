#!/bin/bash
# the refine launches' tails on the C3 loop (PMVS_REFINE_TAIL=1): span and drained-queue tail per form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ab; mkdir -p $O
cd $R && PMVS_REFINE_TAIL=1 timeout -k 10 240 python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline > $O/tail.json 2> $O/tail.err || { tail $O/tail.err; exit 1; }
grep "refine tail" $O/tail.err
