#!/bin/bash
# tools/gpu_round.sh -- GPU steps of one round, each under its own time limit, chained with &&.
#   bash tools/gpu_round.sh test <tag>      pytest -m gpu, smoke(), the default bench line
#   bash tools/gpu_round.sh tests <tag>     pytest -m gpu alone;  bench <tag>: smoke() + the bench line
#   bash tools/gpu_round.sh prof <tag>      rocprofv3 kernel-trace stats of the bench, and the
#                                           HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in
#                                           separate runs, kernel-trace only) for the C3 loop and
#                                           the C2 refine batch
#   bash tools/gpu_round.sh loop <tag>      filter / expansion / loop / sharding GPU tests, the
#                                           expansion phase profile (PMVS_EXPAND_PROFILE=1) and the
#                                           refine launch tails (PMVS_REFINE_TAIL=1) of one C3 step,
#                                           and the bench line
#   bash tools/gpu_round.sh kt <tag>        rocprofv3 kernel-trace stats of one C3 step only
#   bash tools/gpu_round.sh suite <tag>     the whole GPU suite with durations, then smoke() (round 4)
#   bash tools/gpu_round.sh check <tag>     expansion / filter / parity / seed / golden GPU tests, the
#                                           default bench line and a kernel trace of one C3 step
#   bash tools/gpu_round.sh c5 <tag>        the C5 test alone, allocation failures traced
#                                           (PMVS_TRACE_ERRORS)
#   bash tools/gpu_round.sh sq <tag>        three SQ counter passes (issue, waits, instruction mix, active
#                                           lanes per VALU instruction) over one C3 iteration, one run each
set -o pipefail
WHAT=${1:-test}; TAG=${2:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
# a line every 50 s under gpurun_out: a long single test or the bench's setup is not taken for a hang
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$WHAT" = test ]; then
  timeout -k 10 700 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
  timeout -k 10 400 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.err
elif [ "$WHAT" = tests ]; then  # the GPU suite alone (no -x: every failure is listed)
  timeout -k 10 1100 python3 -u -m pytest $R/tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
elif [ "$WHAT" = bench ]; then  # smoke() and the default bench line
  timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
  timeout -k 10 500 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.err
elif [ "$WHAT" = loop ]; then
  T=""; for t in test_gpu_filter.py test_gpu_expand.py test_gpu_loop_scale.py test_gpu_dist.py test_gpu_poison.py; do T="$T $R/tests/$t"; done
  timeout -k 10 800 python3 -u -m pytest $T -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
  PMVS_EXPAND_PROFILE=1 timeout -k 10 300 python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/phase.json 2> $O/phase.err && \
  PMVS_REFINE_TAIL=1 timeout -k 10 300 python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/tail.json 2> $O/tail.err && \
  timeout -k 10 500 python3 -u $R/bench.py --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err
elif [ "$WHAT" = suite ]; then
  timeout -k 10 1000 python3 -u -m pytest $R/tests -m gpu -v --timeout 600 --timeout-method thread --durations=0 > $O/pytest_all.log 2>&1
  rc=$?
  [ $rc -le 1 ] && timeout -k 10 200 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  [ $rc -eq 0 ]
elif [ "$WHAT" = check ]; then
  T=""; for t in test_gpu_expand.py test_gpu_filter.py test_gpu_parity.py test_gpu_parity_matrix.py test_gpu_seed.py test_gpu_golden.py; do T="$T $R/tests/$t"; done
  timeout -k 10 420 python3 -u -m pytest $T -m gpu -v --timeout 250 --timeout-method thread --durations=0 > $O/pytest.log 2>&1
  rc=$?
  [ $rc -le 1 ] && timeout -k 10 500 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1 && \
  [ $rc -eq 0 ]
elif [ "$WHAT" = c5 ]; then
  PMVS_TRACE_ERRORS=1 timeout -k 10 420 python3 -u -m pytest $R/tests/test_gpu_c5.py -m gpu -v --timeout 400 --timeout-method thread -s > $O/pytest_c5.log 2>&1
elif [ "$WHAT" = sq ]; then
  B="$R/bench.py --steps 1 --warmup 0 --iterations 1 --no-cpu-baseline --no-c2"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY \
    --output-format csv -d $O/sq_a -o run -- python3 $B > $O/sq_a.log 2>&1 && \
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE \
    --output-format csv -d $O/sq_b -o run -- python3 $B > $O/sq_b.log 2>&1 && \
  timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES \
    --output-format csv -d $O/sq_c -o run -- python3 $B > $O/sq_c.log 2>&1 && \
  python3 $R/tools/pmc_summary.py $O/sq_a > $O/sq_a.json && python3 $R/tools/pmc_summary.py $O/sq_b > $O/sq_b.json && \
  python3 $R/tools/pmc_summary.py $O/sq_c > $O/sq_c.json && \
  rm -rf $O/sq_a $O/sq_b $O/sq_c  # per-dispatch CSVs: far above what gpurun copies back
elif [ "$WHAT" = kt ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c2 > $O/kt.log 2>&1
else
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/pmc_fetch.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/pmc_write.log 2>&1 && \
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2/pmc_fetch -o run -- python3 $R/bench.py --only-c2 > $O/c2_pmc_fetch.log 2>&1 && \
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2/pmc_write -o run -- python3 $R/bench.py --only-c2 > $O/c2_pmc_write.log 2>&1
fi
rc=$?
echo "gpu_round $WHAT rc=$rc"
exit $rc
