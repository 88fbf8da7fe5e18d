"""VGPR pressure of one kernel in a hipcc -S assembly file: backward liveness
over the basic-block CFG, then the peak point and the code around it.
Usage: vgpr_pressure.py file.s kernel_prefix [context_lines] [top_n_peaks]"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
ctx = int(sys.argv[3]) if len(sys.argv) > 3 else 12
topn = int(sys.argv[4]) if len(sys.argv) > 4 else 1
start = next(i for i, l in enumerate(src) if l.startswith(name))
end = start
while not src[end].strip().startswith("s_endpgm"):
    end += 1
lines = src[start:end + 1]

reg_re = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in reg_re.finditer(text):
        if m.group(1):
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


NO_DST = ("global_store", "ds_write", "scratch_store", "buffer_store", "flat_store", "s_", "v_cmp", "v_cmpx",
          "v_readfirstlane", "v_readlane", "ds_swizzle_nop")
insts = []  # (line_idx, op, defs, uses, label, targets, falls)
for i, l in enumerate(lines):
    t = l.split(";")[0].strip()
    if not t:
        continue
    if t.endswith(":"):
        insts.append((i, "LABEL", set(), set(), t[:-1], [], True))
        continue
    if t.startswith("."):
        continue
    parts = t.split(None, 1)
    op = parts[0]
    args = parts[1] if len(parts) > 1 else ""
    ops = [a.strip() for a in args.split(",")]
    if op.startswith(NO_DST) and not op.startswith("s_") or op.startswith("s_"):
        defs, uses = set(), regs(args)
    else:
        defs, uses = regs(ops[0]) if ops else set(), regs(",".join(ops[1:]))
        if op.startswith(("v_writelane", "v_mac", "v_fmac")) or "_dpp" in op:
            uses |= defs
    targets, falls = [], True
    if op.startswith("s_cbranch") or op == "s_branch":
        targets = [ops[0]]
        falls = op != "s_branch"
    if op == "s_endpgm":
        falls = False
    insts.append((i, op, defs, uses, None, targets, falls))

# basic blocks
blocks, cur = [], []
label_block = {}
for ins in insts:
    if ins[1] == "LABEL":
        if cur:
            blocks.append(cur)
        cur = []
        label_block[ins[4]] = len(blocks)
        continue
    cur.append(ins)
    if ins[5] or not ins[6]:
        blocks.append(cur)
        cur = []
if cur:
    blocks.append(cur)
succ = []
for b, blk in enumerate(blocks):
    s = []
    last = blk[-1] if blk else None
    if last is not None:
        s += [label_block[t] for t in last[5] if t in label_block]
        if last[6] and b + 1 < len(blocks):
            s.append(b + 1)
    elif b + 1 < len(blocks):
        s.append(b + 1)
    succ.append(s)
live_in = [set() for _ in blocks]
changed = True
while changed:
    changed = False
    for b in range(len(blocks) - 1, -1, -1):
        out = set()
        for s in succ[b]:
            out |= live_in[s]
        live = set(out)
        for ins in reversed(blocks[b]):
            live -= ins[2]
            live |= ins[3]
        if live != live_in[b]:
            live_in[b] = live
            changed = True
points = []
for b, blk in enumerate(blocks):
    live = set()
    for s in succ[b]:
        live |= live_in[s]
    for ins in reversed(blk):
        points.append((len(live | ins[2]), ins[0], sorted(live | ins[2])))
        live -= ins[2]
        live |= ins[3]
points.sort(key=lambda p: -p[0])
for n, at, live in points[:topn]:
    print(f"peak live VGPRs {n} at line {at}: {live}")
    for l in lines[max(0, at - ctx):at + 3]:
        print("   ", l)

if len(sys.argv) > 5 and sys.argv[5] == "defs":
    n, at, live = points[0]
    # last definition of each live register before the peak (linear scan)
    lastdef = {}
    for ins in insts:
        if ins[0] >= at:
            break
        for r in ins[2]:
            lastdef[r] = ins[0]
    for r in live:
        d = lastdef.get(r)
        print(f"v{r}: line {d}: {lines[d].strip() if d is not None else '?'}")
