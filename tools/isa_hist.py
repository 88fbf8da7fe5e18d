"""Instruction histogram of one kernel in a device assembly file (hipcc -S
--cuda-device-only).  Usage: isa_hist.py FILE.s SUBSTRING_OF_MANGLED_NAME [N]"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
start = end = None
for i, l in enumerate(lines):
    if start is None and re.match(r"^_Z\S*:", l) and pat in l.split(":")[0]:
        start, name = i, l.split(":")[0]
    elif start is not None and l.startswith(".Lfunc_end"):
        end = i
        break
c = collections.Counter()
for l in lines[start:end]:
    t = l.strip().split()
    if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
        c[t[0]] += 1
print(name, "static instructions:", sum(c.values()))
for k, v in c.most_common(top):
    print(f"  {k:32s} {v}")
for l in lines[end:end + 80]:
    if any(x in l for x in ("NumVgprs", "ScratchSize", "Occupancy", "NumAgprs", "spill")):
        print(" ", l.strip())
