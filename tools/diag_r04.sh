#!/bin/bash
# tools/diag_r04.sh -- round-4 diagnostics on one GPU box: the expansion's phase profile with the
# refine round-trip share (PMVS_EXPAND_PROFILE), the refine kernel's phase split at small and large
# batch sizes (-DBQ_PROFILE build), and refine time per batch size and layout on the C3 scene
# (product layouts; the scratch-state variant, make variant VAR=bqp VARFLAGS=-DBQ_PRIVATE; one wavefront
# per SIMD with TRSBOX's restrict hoisting (VAR=reg1) or the inlined optimizer (VAR=inl1)).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04c}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PMVS_EXPAND_PROFILE=1 timeout -k 10 300 python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/phase.json 2> $O/phase.err && \
PMVS_AMD_LIB=$R/cmvs-pmvs_amd/libpmvs_amd_prof.so PMVS_REFINE_CONFIG=1206 timeout -k 10 200 python3 -u $R/tools/refine_phases.py 1000 5000 20000 100000 > $O/phases_1206.jsonl 2> $O/phases.err && \
timeout -k 10 300 python3 -u $R/tools/refine_sizes.py 1206,132042 2000,5000,10000,20000,40000,80000,120000 > $O/sizes_main.jsonl 2> $O/sizes.err && \
PMVS_AMD_LIB=$R/cmvs-pmvs_amd/libpmvs_amd_bqp.so timeout -k 10 300 python3 -u $R/tools/refine_sizes.py 2448,2432,1232 10000,20000,40000,80000,120000 > $O/sizes_bqp.jsonl 2>> $O/sizes.err && \
for v in reg1 inl1; do PMVS_AMD_LIB=$R/cmvs-pmvs_amd/libpmvs_amd_$v.so timeout -k 10 300 python3 -u $R/tools/refine_sizes.py 164011,164041,1206 1000,2000,5000,10000,80000 > $O/sizes_$v.jsonl 2>> $O/sizes.err || exit 1; done
rc=$?
echo "diag rc=$rc"
exit $rc
