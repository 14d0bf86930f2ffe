"""Diagnostic: optimizer sub-step wave time in the refine kernel (libpmvs_amd_prof.so, built with
-DBQ_PROFILE).  Run: PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_prof.so python3 tools/bq_profile.py"""
import ctypes as C, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import pmvs_amd as P
lib = P.load_library()
lib.pmvs_debug_bq_prof.argtypes = [C.c_void_p]
buf = np.zeros(8, np.uint64)
inp, p = P.synth_scene(8, 1920, 1080, level=1, supersample=2, nthreads=16)
s = P.Scene(inp)
c = P.synth_candidates(p, inp.projections, 100000, seed=0x5EED)
s.refine_batch(c)
lib.pmvs_debug_bq_prof(buf.ctypes.data)
out, st = s.refine_batch(c)
lib.pmvs_debug_bq_prof(buf.ctypes.data)
names = ["trsbox", "altmov", "update", "bq_step_total", "rescue_entries"]
print(json.dumps({"refine_ms": st["refine_ms"], "step_cycles(wave)": st["prof"][1],
                  "bq": {n: int(v) for n, v in zip(names, buf[:5])}}))
rng = np.random.default_rng(0)
x0 = np.zeros((131072, 3)); x0[:, 1:] = rng.uniform(-20, 20, (131072, 2))
for mode in (0, 2, 4):
    for kind in (0, 1):
        lib.pmvs_debug_bq_prof(buf.ctypes.data)
        o, ms = P.selftest_bobyqa(kind, x0, mode=mode, maxeval=200)
        lib.pmvs_debug_bq_prof(buf.ctypes.data)
        print(json.dumps({"mode": mode, "kind": kind, "ms": round(ms, 2), "steps": int(o[:, 4].sum()),
                          "bq": {n: int(v) for n, v in zip(names, buf[:5])}}))
