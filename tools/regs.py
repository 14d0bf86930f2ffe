"""Resource usage per function/kernel from a device assembly file (hipcc --cuda-device-only -S):
resolves the `.set <sym>.num_vgpr, max(...)` expressions so callers show their callees' peaks.
    python tools/regs.py file.s [name-regex]
"""
import re
import subprocess
import sys


def parse(path):
    sets = {}
    pat = re.compile(r"^\s*\.set\s+(\S+)\.(num_vgpr|num_agpr|private_seg_size),\s*(.+)$")
    for line in open(path):
        m = pat.match(line)
        if m:
            sets[(m.group(1), m.group(2))] = m.group(3).strip()
    return sets


def value(sets, sym, field, memo):
    key = (sym, field)
    if key in memo:
        return memo[key]
    expr = sets.get(key, "0")
    refs = re.findall(r"(\.?L?_Z\w+|\.L\w+)\.(num_vgpr|num_agpr|private_seg_size)", expr)
    e = expr
    for name, fld in refs:
        e = e.replace(f"{name}.{fld}", str(value(sets, name, fld, memo)))
    e = e.replace("max(", "max((").replace(")", "),)") if False else e
    v = eval(e, {"max": lambda *a: max(a)})
    memo[key] = v
    return v


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return out[: len(names)]
    except OSError:
        return names


def main():
    sets = parse(sys.argv[1])
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    memo = {}
    syms = sorted({s for s, _ in sets})
    names = demangle([s.lstrip(".L").lstrip("_") and (s[2:] if s.startswith(".L") else s) for s in syms])
    for s, n in zip(syms, names):
        short = n.split("(")[0]
        if rx and not rx.search(short):
            continue
        v = value(sets, s, "num_vgpr", memo)
        a = value(sets, s, "num_agpr", memo)
        p = value(sets, s, "private_seg_size", memo)
        print(f"{short[:70]:70s} vgpr {v:4d} agpr {a:4d} scratch {p:5d}")


if __name__ == "__main__":
    main()
