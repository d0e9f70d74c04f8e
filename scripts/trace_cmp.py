"""Per-kernel median / total duration of two rocprofv3 kernel traces side by side.

    python scripts/trace_cmp.py <a/run_kernel_trace.csv> <b/run_kernel_trace.csv> [top=45]
"""
import collections
import csv
import sys


def stats(p):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].split("(")[0].replace("vg::", "")
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return d


a, b = stats(sys.argv[1]), stats(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
med = lambda v: sorted(v)[len(v) // 2] if v else 0.0
for k in sorted(set(a) | set(b), key=lambda k: -sum(b.get(k, [0])))[:top]:
    fa, fb = a.get(k, []), b.get(k, [])
    print("%-28s a n=%5d med %6.1f tot %8.0f | b n=%5d med %6.1f tot %8.0f" % (k, len(fa), med(fa), sum(fa), len(fb), med(fb), sum(fb)))
