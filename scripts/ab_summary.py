"""Summarise one same-box A/B (scripts/ab_env.sh): gpurun_out/ab_<tag><round>.json -> one JSON.

usage: python3 scripts/ab_summary.py BUILD NOTE > profiles/r04/ab_<tag>.json
"""
import glob
import json
import os
import re
import sys


def main():
    build, note = sys.argv[1], sys.argv[2]
    runs = {}
    for f in sorted(glob.glob("gpurun_out/ab_*.json")):
        m = re.match(r"ab_(.+?)(\d)\.json$", os.path.basename(f))
        if not m:
            continue
        try:
            d = json.load(open(f))
        except (json.JSONDecodeError, OSError):
            continue
        runs.setdefault(m.group(1), []).append(d["value"])
    mean = {k: round(sum(v) / len(v), 1) for k, v in runs.items()}
    base = mean.get("A")
    rel = {k: round(v / base - 1.0, 4) for k, v in mean.items()} if base else {}
    print(json.dumps({"build": build, "note": note, "scans_per_s": runs, "mean": mean, "vs_A": rel}, indent=1))


if __name__ == "__main__":
    main()
