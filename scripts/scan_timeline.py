"""One steady-state scan's kernel timeline from a rocprofv3 kernel trace, and
the scan-to-scan spans (scans start at their first k_iekf launch).

    python scripts/scan_timeline.py gpurun_out/trace_<tag>/run_kernel_trace.csv [scan_from_end]
"""
import csv
import re
import sys


def short(n):
    if "rocprim" in n or "hipcub" in n:
        k = re.findall(r"detail::(\w+)", n)
        return "rocprim." + (k[1] if len(k) > 1 else (k[0] if k else "x"))
    m = re.match(r"(?:void )?(?:vg::)?([\w:<>]+)", n)
    return m.group(1) if m else n


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Queue_Id"]))
                  for r in csv.DictReader(open(path)))
    iekf = [i for i, r in enumerate(rows) if r[2].split("<")[0] in ("k_iekf", "k_iekf_all")]
    scans, last = [], -1e18
    for i in iekf:
        if rows[i][0] - last > 300000:
            scans.append(i)
        last = rows[i][0]
    a, b = scans[-back], scans[-back + 1]
    t0 = rows[a][0]
    lo = a
    while lo > 0 and rows[lo - 1][0] > rows[scans[-back - 1]][0] and rows[lo - 1][3] != rows[a][3]:
        lo -= 1
    prev_end = {}
    for s, e, n, q in rows[lo:b + 1]:
        gap = (s - prev_end[q]) / 1e3 if q in prev_end else 0.0
        prev_end[q] = e
        print("%8.1f %7.1f  gap %6.1f  q%d %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, q, n))
    spans = [(rows[y][0] - rows[x][0]) / 1e3 for x, y in zip(scans[:-1], scans[1:])]
    tail = spans[-12:]
    print("scan spans us", [round(x) for x in tail], "median %.0f" % sorted(tail)[len(tail) // 2])


if __name__ == "__main__":
    main()
