"""HBM traffic of the roofline kernels against their algorithmic bytes, over
the same launches.

    python3 scripts/pmc_summary.py <dir> profiles/<round>/pmc_traffic.json [first_scan]

<dir>/fetch and <dir>/write each hold one rocprofv3 pass (--pmc FETCH_SIZE,
resp. WRITE_SIZE, --kernel-trace, csv) of scripts/pmc_run.py and that run's
scans.json (the per-scan counters of SURVEY 8(d)'s byte model); <dir>/scans_pk.json
is a run of its own with the per-stage profiling (P_k per IEKF iteration), the
same scans (checked). Every counter
row is one kernel dispatch; in dispatch order the rows are paired with the
scan (and IEKF / LM iteration) they belong to:
  * k_iekf: 4 launches per scan, iteration it executed iff it < iekf_iters;
    algorithmic bytes 16 N_raw + 224 P_k (P_k: that iteration's distinct plane
    records, fp64 PlaneRec as the gate reads them);
  * the recut's level kernels (k_rc_level0 + max_layer x k_rc_level), per scan:
    V_slide (80 W + 80);
  * k_ba_hess, executed launches (Hessian passes; the second LM iteration's
    rides in k_ba_resid_hess): F (80 W + 176);
  * k_ba_solve, executed launches (no byte model: the LM step's flops).
Counters are KiB per dispatch. `traffic` follows MI355X_MICROARCH.md: FETCH x2
(on gfx950 FETCH_SIZE reports half the bytes of a 16 B/lane streaming read)
+ WRITE. FETCH at the per-shape ratios of profiles/<round>/fetch_calibration.json
(k_iekf's own access shapes, measured on micro-kernels of known bytes) is
reported beside it as `fetch_calibrated`. Only scans >= first_scan (default
12, the bench's warm-up) count, so the ratios describe the bench's timed scans
and do not depend on how many the bench times. The per-scan P_k of those
scans is kept (`per_scan`): the bench prices its own timed scans with them.
"""
import bisect
import csv
import glob
import json
import math
import os
import sys
from collections import defaultdict

PLANE_B = 224.0


def hess_chunk(W):
    """factors per k_ba_hess chunk (ba.hip hess_fs, kHessThreads = 512)"""
    return 2 * (256 // W) if 2 * (256 // W) <= 64 and 2 * (256 // W) <= 512 // W else min(512 // W, 64)


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def load(path):
    rows = defaultdict(list)  # kernel -> [(dispatch_id, KiB)]
    for r in csv.DictReader(open(path)):
        rows[short(r["Kernel_Name"])].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    for k in rows:
        rows[k].sort()
    return {k: [v for _, v in rows[k]] for k in rows}, {k: [i for i, _ in rows[k]] for k in rows}


def calibration(repo):
    files = sorted(glob.glob(os.path.join(repo, "profiles", "*", "fetch_calibration.json")))
    if not files:
        return None
    d = {k: v["fetch_ratio"] for k, v in json.load(open(files[-1]))["shapes"].items() if "fetch_ratio" in v}
    d["_file"] = os.path.relpath(files[-1], repo)
    return d


def summarise(pass_dir, counter):
    scans = json.load(open(os.path.join(pass_dir, "scans.json")))
    rows, ids = load(glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)[0])
    return scans, rows, ids


def main(src, dst, first):
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    meta, fetch, fid = summarise(os.path.join(src, "fetch"), "FETCH_SIZE")
    meta_w, write, _ = summarise(os.path.join(src, "write"), "WRITE_SIZE")
    S = meta["scans"]
    for other in (meta_w["scans"], json.load(open(os.path.join(src, "scans_pk.json")))["scans"]):
        assert [(s["n_raw"], s["n_ds"], s["iekf_iters"], s["n_factors"], s["ba_iters"]) for s in S] == \
            [(s["n_raw"], s["n_ds"], s["iekf_iters"], s["n_factors"], s["ba_iters"]) for s in other], \
            "the runs stepped different scans"
    pk = json.load(open(os.path.join(src, "scans_pk.json")))["scans"]  # P_k from the per-stage run
    for s, q in zip(S, pk):
        s["iekf_planes"] = q["iekf_planes"]
    W = meta["win_size"]
    L = meta["max_layer"]
    ns = len(S)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes of scripts/pmc_run.py; traffic = "
                     "FETCH x2 (gfx950) + WRITE; algorithmic bytes from the same run's per-scan counters",
           "workload": meta["workload"], "seq": meta["seq"], "scans_counted": [first, ns], "kernels": {}}
    cal = calibration(repo)

    def entry(unit, pairs, alg_note):
        """pairs: [(fetch KiB, write KiB, algorithmic bytes)] of the counted launches"""
        n = len(pairs)
        f = sum(p[0] for p in pairs) * 1024.0 / n
        w = sum(p[1] for p in pairs) * 1024.0 / n
        a = sum(p[2] for p in pairs) / n
        e = {"unit": unit, "count": n, "alg_bytes": round(a), "fetch_raw_bytes": round(f), "fetch_bytes": round(2 * f),
             "write_bytes": round(w), "traffic_bytes": round(2 * f + w),
             "traffic_ratio": round((2 * f + w) / a, 4) if a > 0 else None, "alg_model": alg_note}
        return e

    # k_iekf: 4 dispatches per scan
    fi, wi = fetch.get("k_iekf", []), write.get("k_iekf", [])
    assert len(fi) == 4 * ns and len(wi) == 4 * ns, ("k_iekf dispatches", len(fi), len(wi), ns)
    pairs, n_soa, n_rec = [], 0.0, 0.0
    for s in range(first, ns):
        st = S[s]
        for it in range(st["iekf_iters"]):
            d = 4 * s + it
            a = 16.0 * st["n_raw"] + PLANE_B * st["iekf_planes"][it]
            pairs.append((fi[d], wi[d], a))
            n_soa += 16.0 * st["n_raw"]
            n_rec += PLANE_B * st["iekf_planes"][it]
    e = entry("launch (executed IEKF iteration)", pairs, "16 N_raw + 224 P_k per iteration")
    if cal:
        exp = (cal["k_soa4"] * n_soa + cal["k_rec224"] * n_rec) / len(pairs)
        e["fetch_calibrated"] = {"expected_fetch_raw": round(exp), "measured_fetch_raw": e["fetch_raw_bytes"],
                                 "ratio": round(e["fetch_raw_bytes"] / exp, 4),
                                 "shape_ratios": {"soa4": cal["k_soa4"], "rec224": cal["k_rec224"]},
                                 "source": cal["_file"]}
    out["kernels"]["k_iekf"] = e
    # the recut's level kernels, per scan
    f0, w0 = fetch.get("k_rc_level0", []), write.get("k_rc_level0", [])
    f1, w1 = fetch.get("k_rc_level", []), write.get("k_rc_level", [])
    assert len(f0) == ns and len(f1) == L * ns, ("recut dispatches", len(f0), len(f1), ns)
    pairs = []
    for s in range(first, ns):
        fs = f0[s] + sum(f1[L * s:L * s + L])
        ws = w0[s] + sum(w1[L * s:L * s + L])
        pairs.append((fs, ws, S[s]["n_slide"] * (80.0 * W + 80.0)))
    out["kernels"]["recut_levels"] = entry("scan (k_rc_level0 + %d x k_rc_level)" % L, pairs,
                                           "V_slide (80 W + 80) per scan")
    # k_ba_hess: executed launches, each paired with its scan by dispatch order
    # (a scan's launches follow its four k_iekf dispatches). A scan has at most
    # ba_hess of them: the second LM iteration's pass rides in k_ba_resid_hess
    fh, wh = fetch.get("k_ba_hess", []), write.get("k_ba_hess", [])
    starts = fid["k_iekf"][0::4]
    ex = [i for i, v in enumerate(fh) if v > 64.0]  # an early exit fetches a few KiB
    per = [0] * ns
    pairs = []
    for d in ex:
        s = bisect.bisect_right(starts, fid["k_ba_hess"][d]) - 1
        per[s] += 1
        if s >= first:
            pairs.append((fh[d], wh[d], S[s]["n_factors"] * (80.0 * W + 176.0)))
    assert all(0 <= s and per[s] <= S[s]["ba_hess"] for s in range(ns)), ("k_ba_hess launches per scan", per)
    e = entry("launch (executed Hessian pass)", pairs, "F (80 W + 176) per pass")
    if cal and "k_fachess" in cal:  # the pass's own read shape (scripts/micro/fetch_cal.hip k_fachess)
        exp = cal["k_fachess"] * e["alg_bytes"]
        e["fetch_calibrated"] = {"expected_fetch_raw": round(exp), "measured_fetch_raw": e["fetch_raw_bytes"],
                                 "ratio": round(e["fetch_raw_bytes"] / exp, 4),
                                 "shape_ratios": {"fachess": cal["k_fachess"]}, "source": cal["_file"]}
    # its own stores: the chunk partials (1,891 packed entries at W = 10) + the
    # IMU blocks (931 doubles each); WRITE_SIZE also counts the write-back of
    # earlier kernels' dirty lines evicted under the pass (the PMC run is
    # serialised: k_ba_init's factor copies and the recut's records)
    nl = 6 * W * (6 * W + 1) // 2 + 6 * W + 1
    own = [math.ceil(S[s]["n_factors"] / hess_chunk(W)) * nl * 8.0 + (W - 1) * 931 * 8.0
           for s in range(first, ns) for _ in range(per[s])]
    if own:
        e["own_store_bytes"] = round(sum(own) / len(own))
    out["kernels"]["k_ba_hess"] = e
    # k_ba_solve: executed launches (traffic only)
    fs_, ws_ = fetch.get("k_ba_solve", []), write.get("k_ba_solve", [])
    ex = [i for i, v in enumerate(fs_) if v > 16.0]
    if ex:
        n = len(ex)
        f = sum(fs_[i] for i in ex) * 1024.0 / n
        w = sum(ws_[i] for i in ex if i < len(ws_)) * 1024.0 / n
        out["kernels"]["k_ba_solve"] = {"unit": "launch (executed LM step)", "count": n, "fetch_raw_bytes": round(f),
                                        "fetch_bytes": round(2 * f), "write_bytes": round(w),
                                        "traffic_bytes": round(2 * f + w)}
    out["per_scan"] = {"first": first, "P_k": [s["iekf_planes"][:s["iekf_iters"]] for s in S],
                       "n_raw": [s["n_raw"] for s in S]}
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_scan"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 12)
