"""Which kernels differ between two gfx950 assembly files (per-function
bodies, register names included).  Not product code:
python tools/isa_funcdiff.py a.s b.s"""
import re
import sys


def funcs(path):
    out, cur, name = {}, None, None
    for l in open(path):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            name, cur = m.group(1), []
            continue
        if name and l.startswith(".Lfunc_end"):
            out[name] = cur
            name = None
            continue
        if name is not None:
            cur.append(l)
    return out


a, b = funcs(sys.argv[1]), funcs(sys.argv[2])
for n in sorted(set(a) | set(b)):
    if a.get(n) != b.get(n):
        la, lb = len(a.get(n, [])), len(b.get(n, []))
        print(f"{n[:110]}  {la} -> {lb} lines")
