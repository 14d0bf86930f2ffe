# round 5: the large refine launches' lanes per texture (LP 2 / 3 / 4) on the C3 loop
set -o pipefail
O=gpurun_out/r05ai; mkdir -p $O
for c in 226014 236014 246014 226014; do
  PMVS_REFINE_LARGE_CONFIG=$c timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-c2 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print($c, d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['kernel'], d['checks']['model_hash'][:8])" >> $O/summary.txt || exit 1
done
cat $O/summary.txt
