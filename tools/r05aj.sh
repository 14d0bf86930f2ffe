# round 5: env-knob A/B on the C3 loop: the small/large refine split point, the depth maps' targets
# per thread (defaults: PMVS_REFINE_SMALL_N=10000, PMVS_DM_TARGETS=4)
set -o pipefail
O=gpurun_out/r05aj; mkdir -p $O
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-c2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['checks']['model_hash'][:8])" >> $O/summary.txt
}
run default PMVS_X=0 && run small5k PMVS_REFINE_SMALL_N=5000 && run small20k PMVS_REFINE_SMALL_N=20000 && \
run dm8 PMVS_DM_TARGETS=8 && run default2 PMVS_X=0
rc=$?
cat $O/summary.txt
exit $rc
