"""Static instruction mix of one kernel in a device .s file:
python tools/isa_mix.py file.s kernel_substring"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and pat in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
cnt = collections.Counter()
for l in lines[start:end]:
    t = l.strip()
    if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
        continue
    op = t.split()[0]
    cnt[op] += 1
tot = sum(cnt.values())
v = sum(c for o, c in cnt.items() if o.startswith("v_"))
print(f"{lines[start][:70]} total {tot} valu {v}")
for o, c in cnt.most_common(40):
    print(f"  {o:32s} {c}")
