"""Average duration of a kernel's executed launches from a rocprofv3 kernel trace
(launches that early-exited on the device-side flags, below `min_us`, are
listed separately): the figure bench.py's HIP-event average must agree with.

    python scripts/kernel_avg.py <run_kernel_trace.csv> [kernel=k_ba_solve] [min_us=10]
"""
import csv
import json
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_ba_solve"
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(path))
     if r["Kernel_Name"].replace("void ", "").startswith(("vg::" + name + "(", "vg::" + name + "<"))]
ex = [x for x in d if x >= min_us]
out = {"kernel": name, "launches": len(d), "executed": len(ex),
       "executed_avg_us": round(sum(ex) / max(1, len(ex)), 3),
       "early_exit": len(d) - len(ex), "all_avg_us": round(sum(d) / max(1, len(d)), 3)}
print(json.dumps(out))
