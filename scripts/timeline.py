"""Print one scan's GPU timeline (kernels + memory copies) from a rocprofv3 csv trace.

    python scripts/timeline.py gpurun_out/<dir>/prof [scan_index]
"""
import csv
import os
import sys


def load(d):
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:58]))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "memcpy " + r.get("Direction", "")))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else -3
    ev = load(d)
    idx = [i for i, e in enumerate(ev) if e[2].endswith("k_ds_keys")]
    a, b = idx[k - 1], idx[k]
    t0 = ev[a][0]
    prev = t0
    busy = 0
    for s, e, n in ev[a:b]:
        print("%8.1f gap%7.1f dur%7.1f %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, n))
        prev = max(prev, e)
        busy += e - s
    print("scan span %.1f us, busy %.1f us, events %d" % ((ev[b][0] - t0) / 1e3, busy / 1e3, b - a))


if __name__ == "__main__":
    main()
