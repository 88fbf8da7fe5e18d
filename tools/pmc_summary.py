"""Summarise a round's rocprofv3 outputs (tools/profile_round.sh) into
profiles/<tag>_pmc_summary.json: per-launch HBM traffic of the codec kernels
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

KERNELS = {"encode": "k_encode_fast", "reconstruct": "k_reconstruct_fast", "locator": "k_error_locator",
           "encode_big": "k_encode_big", "reconstruct_big": "k_reconstruct_big",
           "calib_read8": "read8", "calib_copy8": "copy8"}


def kind(name):
    for k, pat in KERNELS.items():
        if pat + "(" in name or pat + "<" in name:
            return k
    return None


def newest(pattern):
    """Latest file of a pass (gpurun merges every call's outputs into gpurun_out/)."""
    f = sorted(glob.glob(pattern), key=os.path.getmtime)
    return f[-1:] if f else []


def counters(pass_name):
    f = newest(os.path.join(src, pass_name, "*", "*_counter_collection.csv"))
    agg = defaultdict(lambda: defaultdict(list))
    if not f:
        return agg
    for r in csv.DictReader(open(f[0])):
        k = kind(r["Kernel_Name"])
        if k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def mean(v):
    return sum(v) / len(v) if v else None


out = {"tag": tag, "kernels": {}}
fetch, write = counters("fetch"), counters("write")
cf, cw = counters("calib_fetch"), counters("calib_write")
GIB = 1 << 30
# calibration: read8 reads exactly 1 GiB per dispatch; copy8 reads 1 GiB and writes 1 GiB
f_read8 = mean(cf["calib_read8"].get("FETCH_SIZE", []))
w_copy8 = mean(cw["calib_copy8"].get("WRITE_SIZE", []))
# FETCH_SIZE / WRITE_SIZE are reported in KB (1024 B) by rocprofv3
fetch_factor = GIB / (f_read8 * 1024) if f_read8 else None
write_factor = GIB / (w_copy8 * 1024) if w_copy8 else None
out["calibration"] = {"read8_FETCH_SIZE_KB": f_read8, "copy8_WRITE_SIZE_KB": w_copy8,
                      "fetch_factor": fetch_factor, "write_factor": write_factor,
                      "note": "factor = known bytes / (counter * 1024) for 8-byte-per-lane coalesced access, "
                              "1 GiB buffers (beyond the 256 MiB Infinity Cache)"}
for k in ("encode", "reconstruct", "locator", "encode_big", "reconstruct_big"):
    fs, ws = mean(fetch[k].get("FETCH_SIZE", [])), mean(write[k].get("WRITE_SIZE", []))
    if fs is None or ws is None:
        continue
    rd = fs * 1024 * (fetch_factor or 1.0)
    wr = ws * 1024 * (write_factor or 1.0)
    out["kernels"][k] = {"FETCH_SIZE_KB": fs, "WRITE_SIZE_KB": ws, "read_bytes": rd, "write_bytes": wr,
                         "traffic_bytes": rd + wr}
for pname in ("sq", "sq2"):
    c = counters(pname)
    for k in ("encode", "reconstruct", "locator", "encode_big", "reconstruct_big"):
        for name, vals in c[k].items():
            out["kernels"].setdefault(k, {})[name] = mean(vals)
# kernel-trace averages
st = newest(os.path.join(src, "stats", "*", "*_kernel_stats.csv"))
if st:
    for r in csv.DictReader(open(st[0])):
        k = kind(r["Name"])
        if k:
            out["kernels"].setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            out["kernels"][k]["calls"] = int(r["Calls"])
    shutil.copy(st[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
for k, v in out["kernels"].items():
    if "SQ_INSTS_VALU" in v and "SQ_WAVES" in v:
        v["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / v["SQ_WAVES"]
    if "SQ_ACTIVE_INST_VALU" in v and "SQ_BUSY_CYCLES" in v:
        # SQ_ACTIVE_INST_VALU counts quad-cycles summed over SIMDs; busy cycles summed over SEs (32)
        pass
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1, sort_keys=True))
