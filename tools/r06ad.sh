#!/bin/bash
# per-job preProcess outputs and evaluation counts of the first four large refine batches (PMVS_DUMP_JOBS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ad; mkdir -p $O
cd $R && PMVS_DUMP_JOBS=$O/jobs.bin timeout -k 10 240 python3 bench.py --steps 1 --warmup 0 --iterations 1 --no-c2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
ls -la $O/jobs.bin
