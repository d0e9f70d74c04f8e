"""Host/device timeline of one steady-state scan from a rocprofv3 kernel +
HIP runtime trace (scripts/gpu_apitrace.sh): every HIP API call of the scan
with its host duration, and for launches the kernel it produced and how long
the device waited for it (device-idle gap before that kernel).

    python scripts/api_timeline.py gpurun_out/api_<tag> [scan_from_end]
"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from scan_timeline import short  # noqa: E402


def main():
    d = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    at = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    kern = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   int(r["Correlation_Id"])) for r in csv.DictReader(open(kt)))
    by_corr = {}
    for k in kern:  # a graph launch's kernels share its correlation id: keep the first
        by_corr.setdefault(k[3], k)
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], int(r["Correlation_Id"]))
                 for r in csv.DictReader(open(at)))
    # scans open with k_scan_begin
    starts = [k[0] for k in kern if k[2] == "k_scan_begin"]
    t0, t1 = starts[-back], starts[-back + 1]
    # device busy intervals, to find the idle gap before each kernel
    prev_end = {}
    last = 0
    for s, e, n, c in kern:
        prev_end[c] = last
        last = max(last, e)
    # the API calls issued while this scan's kernels run: from the API call
    # that launched k_scan_begin to the one that launched the next scan's
    first = next(a for a in api if a[3] in by_corr and by_corr[a[3]][0] == t0)
    nxt = next(a for a in api if a[3] in by_corr and by_corr[a[3]][0] == t1)
    tot = {}
    print("%9s %8s  %-28s %-28s %9s %8s" % ("host_us", "dur_us", "api", "kernel", "dev_us", "idle_us"))
    for s, e, f, c in api:
        if s < first[0] or s >= nxt[0]:
            continue
        tot[f] = tot.get(f, 0.0) + (e - s) / 1e3
        k = by_corr.get(c)
        if k:
            idle = max(0.0, (k[0] - prev_end[c]) / 1e3)
            print("%9.1f %8.1f  %-28s %-28s %9.1f %8.1f" % ((s - first[0]) / 1e3, (e - s) / 1e3, f[:28], k[2][:28],
                                                         (k[0] - t0) / 1e3, idle))
        elif (e - s) > 2000:
            print("%9.1f %8.1f  %-28s" % ((s - first[0]) / 1e3, (e - s) / 1e3, f[:28]))
    print("host time per API in this scan (us):")
    for f, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
        print("  %-32s %8.1f" % (f, v))
    print("scan span on the device: %.1f us" % ((t1 - t0) / 1e3))


if __name__ == "__main__":
    main()
