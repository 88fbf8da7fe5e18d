"""Summarise a round's rocprofv3 outputs (tools/profile_round.sh) into
profiles/<tag>_pmc_summary.json: per-bench-step HBM traffic of the codec kernels
(FETCH_SIZE and WRITE_SIZE from separate passes, corrected by the calibration
microbenchmark for 8-byte lanes), SQ utilisation counters, and the kernel-trace
averages.  Usage: python tools/pmc_summary.py r01"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)

# The bench's "reconstruct" span is the prefix-locator launch plus both fast
# reconstruct instances (prefixes of <= 2 and of 4 segments); their per-launch
# traffic and durations add up.  Each instance is also reported on its own.
KINDS = {"encode": ("k_encode_fast", "k_encode_multi", "k_encode_big", "k_encode_res"),
         "reconstruct": ("k_reconstruct_fast", "k_prefix_locator", "k_reconstruct_big", "k_big_records", "k_payload_status",
                         "k_reconstruct_res"),
         "locator": ("k_error_locator",), "calib_read8": ("read8",), "calib_copy8": ("copy8",)}
# bench steps per profiled command (tools/profile_round.sh): PMC passes run
# 1 warmup + 3 timed steps, the kernel-trace pass 3 + 10; per-step values are
# the sums over every dispatch of a kind divided by these
PMC_STEPS, STATS_STEPS = 4, 13


def instance(name):
    """Kernel instance (template arguments kept, parameter list dropped)."""
    for pats in KINDS.values():
        for pat in pats:
            i = name.find(pat + "(")
            if i < 0:
                i = name.find(pat + "<")
            if i >= 0:
                return name[i:].split("(")[0]
    return None


def kind(inst):
    for k, pats in KINDS.items():
        if any(inst == p or inst.startswith(p + "<") for p in pats):
            return k
    return None


def newest(pattern):
    """Latest file of a pass (gpurun merges every call's outputs into gpurun_out/)."""
    f = sorted(glob.glob(pattern), key=os.path.getmtime)
    return f[-1:] if f else []


def counters(pass_name):
    """{instance: {counter: [per-launch values]}}"""
    f = newest(os.path.join(src, pass_name, "*", "*_counter_collection.csv"))
    agg = defaultdict(lambda: defaultdict(list))
    if not f:
        return agg
    for r in csv.DictReader(open(f[0])):
        i = instance(r["Kernel_Name"])
        if i:
            agg[i][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def by_kind(c, k, name, steps=PMC_STEPS):
    """Per-step value of counter `name` for kind k: the sum over every dispatch
    of its instances, divided by the steps of the profiled run."""
    vals = [sum(v[name]) for i, v in c.items() if kind(i) == k and v.get(name)]
    return sum(vals) / steps if vals else None


def mean(v):
    return sum(v) / len(v) if v else None


out = {"tag": tag, "kernels": {}}
fetch, write = counters("fetch"), counters("write")
cf, cw = counters("calib_fetch"), counters("calib_write")
GIB = 1 << 30
# calibration: read8 reads exactly 1 GiB per dispatch; copy8 reads 1 GiB and writes 1 GiB
f_read8 = by_kind(cf, "calib_read8", "FETCH_SIZE", 1)
w_copy8 = by_kind(cw, "calib_copy8", "WRITE_SIZE", 1)
if f_read8:  # per dispatch of the calibration kernels
    f_read8 /= len(next(v["FETCH_SIZE"] for i, v in cf.items() if kind(i) == "calib_read8"))
if w_copy8:
    w_copy8 /= len(next(v["WRITE_SIZE"] for i, v in cw.items() if kind(i) == "calib_copy8"))
if not f_read8 or not w_copy8:  # every pass measures its own correction (tools/profile_round.sh)
    sys.exit(f"pmc_summary: no calibration counters under {src}/calib_fetch or calib_write")
# FETCH_SIZE / WRITE_SIZE are reported in KB (1024 B) by rocprofv3
fetch_factor = GIB / (f_read8 * 1024) if f_read8 else None
write_factor = GIB / (w_copy8 * 1024) if w_copy8 else None
out["calibration"] = {"read8_FETCH_SIZE_KB": f_read8, "copy8_WRITE_SIZE_KB": w_copy8,
                      "fetch_factor": fetch_factor, "write_factor": write_factor,
                      "note": "factor = known bytes / (counter * 1024) for 8-byte-per-lane coalesced access, "
                              "1 GiB buffers (beyond the 256 MiB Infinity Cache)"}
for k in ("encode", "reconstruct", "locator"):
    fs, ws = by_kind(fetch, k, "FETCH_SIZE"), by_kind(write, k, "WRITE_SIZE")
    if fs is None or ws is None:
        continue
    rd = fs * 1024 * (fetch_factor or 1.0)
    wr = ws * 1024 * (write_factor or 1.0)
    out["kernels"][k] = {"FETCH_SIZE_KB": fs, "WRITE_SIZE_KB": ws, "read_bytes": rd, "write_bytes": wr,
                         "traffic_bytes": rd + wr}
out["instances"] = {}
for pname in ("sq", "sq2", "fetch", "write"):
    c = counters(pname)
    for i, cs in c.items():
        if kind(i) and not kind(i).startswith("calib"):
            for name, vals in cs.items():
                out["instances"].setdefault(i, {})[name] = mean(vals)
# kernel-trace averages
st = newest(os.path.join(src, "stats", "*", "*_kernel_stats.csv"))
if st:
    for r in csv.DictReader(open(st[0])):
        i = instance(r["Name"])
        if i and kind(i) and not kind(i).startswith("calib"):
            out["instances"].setdefault(i, {})["avg_ns"] = float(r["AverageNs"])
            out["instances"][i]["calls"] = int(r["Calls"])
            k = out["kernels"].setdefault(kind(i), {})
            # per bench step: every dispatch of the kind in one step
            k["ns_per_step"] = k.get("ns_per_step", 0.0) + float(r["TotalDurationNs"]) / STATS_STEPS
    shutil.copy(st[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
for i, v in out["instances"].items():
    if "SQ_INSTS_VALU" in v and v.get("SQ_WAVES"):
        v["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / v["SQ_WAVES"]
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1, sort_keys=True))
