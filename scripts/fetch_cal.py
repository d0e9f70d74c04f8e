"""FETCH_SIZE / WRITE_SIZE calibration summary (scripts/micro/fetch_cal.hip).

    python scripts/fetch_cal.py <dir> <bytes.csv> <out.json>

<dir>/fetch/run_counter_collection.csv and <dir>/write/... are the two
rocprofv3 --pmc passes over the micro binary, <bytes.csv> its stdout (the
algorithmic bytes per kernel). Reports, per access shape, the counter bytes
(KiB x 1024, averaged over the repetitions) divided by the algorithmic bytes:
the factor to divide a kernel's counter by, shape by shape.
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0].replace("void ", "").strip()].append(float(r["Counter_Value"]))
    return d


def main(src, bytes_csv, dst):
    known = {r["kernel"]: (int(r["read_bytes"]), int(r["write_bytes"])) for r in csv.DictReader(open(bytes_csv))}
    fetch = load(src + "/fetch/run_counter_collection.csv")
    write = load(src + "/write/run_counter_collection.csv")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (KiB), separate passes over scripts/micro/fetch_cal.hip;"
                     " ratio = counter bytes / algorithmic bytes (no correction applied)", "shapes": {}}
    for k, (rb, wb) in known.items():
        v = fetch.get(k, [])
        if rb and v:
            f = 1024.0 * sum(v) / len(v)
            out["shapes"][k] = {"read_bytes": rb, "fetch_bytes": round(f), "fetch_ratio": round(f / rb, 4)}
    for k, (rb, wb) in known.items():
        v = write.get(k, [])
        if wb and v:
            w = 1024.0 * sum(v) / len(v)
            out["shapes"].setdefault(k, {}).update(write_bytes=wb, counter_bytes=round(w), write_ratio=round(w / wb, 4))
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
