"""Approximate VGPR pressure over a kernel's assembly (linear order, ignores
loop back-edges).  Usage: vgpr_pressure.py file.s kernel_prefix [context]
Prints the peak live count and the code around it."""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
ctx = int(sys.argv[3]) if len(sys.argv) > 3 else 15
start = next(i for i, l in enumerate(src) if l.startswith(name))
end = start
while not src[end].strip().startswith("s_endpgm"):
    end += 1
lines = src[start:end]

reg_re = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs(text):
    out = []
    for m in reg_re.finditer(text):
        if m.group(1):
            out.append(int(m.group(1)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


first_def, last_use = {}, {}
for i, l in enumerate(lines):
    t = l.split(";")[0].strip()
    if not t or t.endswith(":") or t.startswith("."):
        continue
    parts = t.split(None, 1)
    if len(parts) < 2:
        continue
    op, args = parts
    ops = [a.strip() for a in args.split(",")]
    stores = op.startswith(("global_store", "ds_write", "scratch_store", "buffer_store", "flat_store")) or \
        op.startswith(("v_cmp", "s_", "v_readfirstlane", "v_readlane"))
    dsts = [] if stores else regs(ops[0])
    srcs = regs(",".join(ops if stores else ops[1:]))
    for r in srcs:
        last_use[r] = i
        first_def.setdefault(r, i)
    for r in dsts:
        first_def.setdefault(r, i)
        last_use.setdefault(r, i)
        last_use[r] = max(last_use[r], i)

n = len(lines)
delta = [0] * (n + 2)
for r, d in first_def.items():
    u = last_use.get(r, d)
    delta[d] += 1
    delta[u + 1] -= 1
live, peak, at = 0, 0, 0
for i in range(n):
    live += delta[i]
    if live > peak:
        peak, at = live, i
print("peak approx live VGPRs", peak, "at line", at)
livers = sorted(r for r, d in first_def.items() if d <= at <= last_use.get(r, d))
print("live:", livers)
for l in lines[max(0, at - ctx):at + ctx]:
    print(l)
