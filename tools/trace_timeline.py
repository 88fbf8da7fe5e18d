"""Timeline of the last host-pipeline call in a rocprofv3 --kernel-trace
--memory-copy-trace CSV pair: kernels and copies sorted by start, relative
times in µs.  Usage: trace_timeline.py DIR_PREFIX [MARKER_KERNEL] [N_MARKERS] [ROWS]"""
import csv
import sys

pre = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_copy_rows"
nm = int(sys.argv[3]) if len(sys.argv) > 3 else 22
rows = int(sys.argv[4]) if len(sys.argv) > 4 else 80
ev = []
for r in csv.DictReader(open(pre + "_kernel_trace.csv")):
    n = r["Kernel_Name"]
    n = n[n.find("k_"):].split("(")[0] if "k_" in n else n[:28]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + n, "q" + r["Queue_Id"], r["Grid_Size_X"]))
for r in csv.DictReader(open(pre + "_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r["Direction"][12:], "s" + r["Stream_Id"], ""))
ev.sort()
g = [e for e in ev if marker in e[2]]
t_last = g[-nm][0] - 1000
sel = [e for e in ev if e[0] >= t_last]
t0 = sel[0][0]
for e in sel[:rows]:
    print(f"{(e[0]-t0)/1e3:9.1f} {(e[1]-t0)/1e3:9.1f} {(e[1]-e[0])/1e3:8.1f} {e[2]:40s} {e[3]} {e[4]}")
print("span", (max(e[1] for e in sel) - t0) / 1e3)
