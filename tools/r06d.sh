#!/bin/bash
# C3 loop A/B: the small refine batches on the workgroup form (default) or the lane form, split point
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
B="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c2"
( while true; do sleep 50; echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in base:132042:10000 lane10k:300000:10000 lane7k:300000:7000 lane5k:300000:5000; do
  IFS=: read tag cfg n <<< "$v"
  PMVS_REFINE_SMALL_CONFIG=$cfg PMVS_REFINE_SMALL_N=$n timeout -k 10 400 $B > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; m=r['small_batches']
print('$tag', d['value'], d['ms_per_step'], d['checks']['model_digest'], 'large', r['launches'], r['kernel_ms_avg'], 'small', m['launches'], m['kernel_ms_avg'], round(m['launches'] * m['kernel_ms_avg'] / d['steps'], 1), 'ms/step')"
done
