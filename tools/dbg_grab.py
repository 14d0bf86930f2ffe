import sys, os, numpy as np
sys.path.insert(0, 'cmvs-pmvs_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import pmvs_amd as P, pyoracle as O
from conftest import small_scene
inp, p = small_scene(8, 480, 360, level=1)
g = P.Scene(inp); o = O.OracleScene(inp)
cands = P.synth_candidates(p, inp.projections, 300, seed=11)
q = np.zeros(len(cands) * 3, P.TEX_QUERY_DTYPE)
k = 0
for c in cands:
    ref = int(c["images"][0]); px, py = o.paxes(ref, c["coord"], c["normal"])
    for view in (ref, int(c["images"][1]), (ref + 3) % 8):
        q[k]["coord"] = c["coord"]; q[k]["pxaxis"] = px; q[k]["pyaxis"] = py; q[k]["normal"] = c["normal"]
        q[k]["view"] = view; q[k]["normalize"] = k % 2; k += 1
tg, vg = g.grab_tex(q); to, vo = o.grab_tex(q)
np.savez('gpurun_out/dbg_grab.npz', q=q, tg=tg, vg=vg, to=to, vo=vo)
d = tg.view(np.uint32) != to.view(np.uint32)
print('mismatch elems', d.sum(), 'rows', d.any(1).sum(), 'raw rows', d[q['normalize']==0].any(1).sum(), 'norm rows', d[q['normalize']==1].any(1).sum())
