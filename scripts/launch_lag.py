"""When the host launched a kernel against when it ran, from a rocprofv3
kernel trace + HIP runtime API trace of the same run (scripts/gpu_hiptrace.sh).

    python scripts/launch_lag.py gpurun_out/htrace_<tag> [kernel-substring ...]

For the last 8 steady-state scans (scans start at their first k_iekf) prints,
per named kernel (default: k_scan_prop, k_hds_args, k_ba_init), its launch
call's host start, the kernel's start and end, relative to the scan's first
k_iekf, and the previous scan's k_margi_leaf end. Graph launches: a kernel
inside a replayed graph is matched to its hipGraphLaunch by correlation id.
"""
import csv
import glob
import os
import sys

from scan_timeline import short


def main():
    d = sys.argv[1]
    names = sys.argv[2:] or ["k_scan_prop", "k_hds_args", "k_ba_init", "k_iekf"]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    api = {}
    for r in csv.DictReader(open(ht)):
        api[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   int(r["Correlation_Id"])) for r in csv.DictReader(open(kt)))
    iekf = [i for i, r in enumerate(rows) if r[2].split("<")[0] == "k_iekf"]
    scans, last = [], -1e18
    for i in iekf:
        if rows[i][0] - last > 300000:
            scans.append(i)
        last = rows[i][0]
    for a, b in zip(scans[-9:-1], scans[-8:]):
        t0 = rows[b][0]
        lo = a
        out = []
        for s, e, n, c in rows[a:b + 4]:
            if n.startswith("k_margi_leaf") and s < t0:
                out.append("margi_leaf end %.1f" % ((e - t0) / 1e3))
        for s, e, n, c in rows[max(a - 400, 0):b + 40]:
            if any(n.startswith(x) for x in names) and abs(s - t0) < 800000:
                h = api.get(c)
                hs = (h[0] - t0) / 1e3 if h else float("nan")
                out.append("%s: launch %.1f (%s) start %.1f end %.1f" % (n, hs, h[2] if h else "?", (s - t0) / 1e3,
                                                                        (e - t0) / 1e3))
        print("scan @%d:" % b)
        for o in out:
            print("   ", o)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
