"""Per-kernel register / spill summary of one HIP source file (gfx950):
python tools/res_usage.py csrc/kernels_fast.hip [extra hipcc flags]."""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
       "-Wno-unused-function", "-c", src, "-o", "/tmp/res_usage.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = re.sub(r"_ZN2np12_GLOBAL__N_1\d+", "", r["name"])[:60]
    print(f"{n:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>4} vspill={r.get('VGPRs Spill','?'):>4} "
          f"sspill={r.get('SGPRs Spill','?'):>4} scratch={r.get('ScratchSize [bytes/lane]','?'):>4} occ={r.get('Occupancy [waves/SIMD]','?')}")
