"""Per-kernel share of summed kernel time (a proxy for block time when many
queues overlap) over the second half of a rocprofv3 kernel trace.

    python scripts/kernel_share.py run_kernel_trace.csv [top]
"""
import csv
import sys
from collections import defaultdict

rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
        for r in csv.DictReader(open(sys.argv[1]))]
rows.sort()
t0, t1 = rows[0][0], max(r[1] for r in rows)
rows = [r for r in rows if r[0] >= t0 + (t1 - t0) // 2]
tot, cnt = defaultdict(int), defaultdict(int)
for s, e, k in rows:
    tot[k] += e - s
    cnt[k] += 1
all_ns = sum(tot.values())
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print("%6.2f%%  %8.1f us avg  %6d  %s" % (100.0 * v / all_ns, v / cnt[k] / 1e3, cnt[k], k))
