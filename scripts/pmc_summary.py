"""Per-launch HBM traffic of the roofline kernels from two rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir>/fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir>/write -o run -- python3 bench.py ...
    python scripts/pmc_summary.py <dir> profiles/r01/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. On gfx950 FETCH_SIZE reports half
the bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM), so
it is doubled. Launches that early-exited on the device-side LM / IEKF flags
(a few KiB) are excluded: only dispatches above `min_kib` count.
"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = {"vg::k_ba_solve": 16.0, "vg::k_iekf": 256.0}  # name -> min KiB of an executed launch


def load(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]].append(float(r["Counter_Value"]))
    return d


def main(src, dst):
    fetch = load(src + "/fetch/run_counter_collection.csv")
    write = load(src + "/write/run_counter_collection.csv")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH x2 (gfx950)", "kernels": {}}
    for k, mn in KERNELS.items():
        f = [v for v in fetch.get(k, []) if v > mn]
        w = write.get(k, [])
        w = sorted(w)[len(w) - len(f):] if len(w) >= len(f) else w  # the executed launches write the most
        if not f:
            continue
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / max(len(w), 1)
        out["kernels"][k.split("::")[-1]] = {"launches": len(f), "fetch_bytes": round(fb), "write_bytes": round(wb),
                                             "traffic_bytes": round(fb + wb), "fetch_raw_bytes": round(fb / 2.0)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
