"""Per-kernel duration and L2 (TCC) hit rate of multi_pmc.py runs, one column
per run directory (each holding a --pmc TCC_HIT_sum TCC_MISS_sum pass with
--kernel-trace), kernels ranked by total time in the first run.

    python3 scripts/multi_pmc_summary.py gpurun_out/mpmc_B4 gpurun_out/mpmc_B8
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    k = defaultdict(lambda: {"n": 0, "dur": 0.0, "hit": 0.0, "miss": 0.0})
    seen = {}
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].replace("vg::", "")
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        key = (name, did)
        if key not in seen:
            seen[key] = True
            k[name]["n"] += 1
            if "End_Timestamp" in r and r["End_Timestamp"]:
                k[name]["dur"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c = r["Counter_Name"]
        if c.startswith("TCC_HIT"):
            k[name]["hit"] += float(r["Counter_Value"])
        elif c.startswith("TCC_MISS"):
            k[name]["miss"] += float(r["Counter_Value"])
    return k


def main(dirs):
    runs = [load(d) for d in dirs]
    base = runs[0]
    names = sorted(base, key=lambda n: -base[n]["dur"])[:25]
    out = {"runs": dirs, "kernels": {}}
    for n in names:
        row = {}
        for d, r in zip(dirs, runs):
            v = r.get(n)
            if not v or not v["n"]:
                continue
            tot = v["hit"] + v["miss"]
            row[d] = {"launches": v["n"], "mean_us": round(v["dur"] / v["n"], 2) if v["dur"] else None,
                      "tcc_hit_rate": round(v["hit"] / tot, 4) if tot else None,
                      "tcc_req_per_launch": round(tot / v["n"])}
        out["kernels"][n] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
