"""Time the full expand/filter loop (CFindMatch::run after seeds, pmvs_run_loop) on the GPU.

usage: python tools/loop_probe.py VIEWS WIDTH HEIGHT LEVEL SEEDS [WAVE] [native|py] [MIN_CANDIDATES]
Prints one line per stage (flushed) so a long run shows progress."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import pmvs_amd as P  # noqa: E402

V, W, H, L, S = (int(a) for a in sys.argv[1:6])
wave = int(sys.argv[6]) if len(sys.argv) > 6 else 4096
native = (sys.argv[7] if len(sys.argv) > 7 else "native") == "native"
minc = int(sys.argv[8]) if len(sys.argv) > 8 else 0
t0 = time.time()
inp, p = P.synth_scene(V, W, H, level=L, supersample=2, nthreads=16)
print(f"synth {time.time() - t0:.1f}s", flush=True)
g = P.Scene(inp)
cands = P.synth_candidates(p, inp.projections, S, seed=11)
r, st = g.refine_batch(cands)
seeds = P.patches_from_refined(r)
print(f"seeds {len(seeds)}/{S} kernel {st['kernel_ms']:.1f}ms", flush=True)
for rep in range(2):
    t0 = time.time()
    model, log = g.run_loop(seeds, inp.threshold, wave=wave, native=native, min_candidates=minc)
    tl = time.time() - t0
    for it in log:
        print(f"  iter depth {it['depth']} patches {it['patches']} expand {it['expand']}", flush=True)
        print(f"     filter {it['filter']}", flush=True)
    added = sum(it["expand"]["added"] for it in log)
    refined = sum(it["expand"]["refined"] for it in log)
    evals = sum(it["expand"]["evals"] for it in log)
    rms = sum(it["expand"]["refine_ms"] for it in log)
    print(f"loop rep {rep}: {tl:.2f}s final {len(model)} added {added} ({added / tl:.0f}/s) refined {refined} "
          f"evals {evals} ({evals / tl / 1e6:.1f} M/s) refine_kernel {rms / 1e3:.2f}s", flush=True)
g.close()
