"""GPU busy fraction of a rocprofv3 kernel trace over a time window: the union
of all kernels' [start, end) intervals across queues, and per-queue counts.

    python scripts/busy_union.py run_kernel_trace.csv [skip_fraction]
"""
import csv
import sys
from collections import Counter

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]))
              for r in csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
t0, t1 = rows[0][0], max(r[1] for r in rows)
ts = t0 + (t1 - t0) * skip
rows = [r for r in rows if r[0] >= ts]
busy, cur_s, cur_e = 0, None, None
for s, e, q in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = max(r[1] for r in rows) - rows[0][0]
# concurrency: average number of kernels in flight
ev = sorted([(s, 1) for s, e, q in rows] + [(e, -1) for s, e, q in rows])
inflight, last, acc = 0, ev[0][0], 0
for t, d in ev:
    acc += inflight * (t - last)
    inflight += d
    last = t
print("kernels %d  span %.1f ms  busy(union) %.1f%%  mean in flight %.2f  queues %d" % (
    len(rows), span / 1e6, 100.0 * busy / span, acc / span, len(Counter(q for _, _, q in rows))))
