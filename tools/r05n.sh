set -o pipefail
O=$(pwd)/gpurun_out/r05n; mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/ht -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-c2 > $O/ht.log 2>&1
rc=$?
cd $O/ht && python3 - <<'PY' > $O/api_summary.txt
import csv, glob, re
f = glob.glob('**/*hip_api_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print(len(rows), 'api rows; columns:', list(rows[0].keys()))
big = []
for r in rows:
    d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    if d > 500000: big.append((int(r['Start_Timestamp']), d, r['Function']))
big.sort()
t0 = big[0][0] if big else 0
for s, d, fn in big: print(f"{(s - t0)/1e6:10.1f} ms  {d/1e6:8.2f} ms  {fn}")
PY
find $O/ht -name "*hip_api_trace.csv" -delete
find $O/ht -name "*kernel_trace.csv" -size +20M -delete
exit $rc
