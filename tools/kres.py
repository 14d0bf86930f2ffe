"""Kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin):
name, VGPRs, AGPRs, scratch bytes/lane, occupancy (waves/SIMD), LDS bytes.
    hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [name-regex]"""
import re
import subprocess
import sys

rx = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = re.sub(r"\(.*", "", n)
    if rx and not rx.search(n):
        continue
    print(f"{n[:58]:58s} v{r.get('VGPRs', '?'):>4s} a{r.get('AGPRs', '?'):>4s} scr{r.get('ScratchSize [bytes/lane]', '?'):>5s} "
          f"occ{r.get('Occupancy [waves/SIMD]', '?'):>3s} lds{r.get('LDS Size [bytes/block]', '?'):>7s}")
