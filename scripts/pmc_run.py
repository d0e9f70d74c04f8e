"""The workload of a PMC (hardware counter) pass, with its own per-scan log.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D/fetch -o run -- \
        python3 scripts/pmc_run.py --out D/fetch/scans.json
    (the same with WRITE_SIZE into D/write), then
    python3 scripts/pmc_summary.py D profiles/<round>/pmc_traffic.json

Runs the bench's metric workload (synthetic 64-line, mid360.yaml, sequence 0,
the same scans bench.py times: warm-up 12, then its timed scans) through one
context; with --stages (a run of its own, outside the counter passes) the
per-stage profiling is on for every scan, so that the stats log carries, per
scan, every counter of SURVEY 8(d)'s byte model, including P_k (distinct plane
records each IEKF iteration read). The pipeline is deterministic, so the
counter passes (without --stages) run the same scans. pmc_summary.py pairs each
counter row (one per kernel dispatch) with the scan and iteration it belongs
to, so the algorithmic bytes and the measured counters cover the same
launches. Under rocprofv3 --pmc the library runs with event waits
(ROCPROF_COUNTER_COLLECTION, vg_create): kernels are serialised there.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--lidar", default="64line")
    ap.add_argument("--config", default="mid360")
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--scans", type=int, default=56, help="scans stepped (bench default: 12 warm-up + 40 timed)")
    ap.add_argument("--stages", action="store_true",
                    help="per-stage profiling on every scan: the log carries P_k (the k_iekf_planes pass and its "
                         "per-point leaf writes ride along, so a counter pass runs without it)")
    args = ap.parse_args()
    import synth
    import vgconfig
    p = vgconfig.load(args.config)
    g = p["General"]
    seq = synth.Sequence(args.lidar, args.seq, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    host = []
    for k in range(args.scans):
        xyz, inten, b, e = seq.scan(k)
        host.append((xyz, inten, b, e, seq.imu(k)))
        if k % 8 == 7:
            print("[pmc_run] generated %d scans" % (k + 1), file=sys.stderr, flush=True)
    import torch

    import vgpu
    dev = torch.device("cuda", 0)
    scans = []
    for xyz, inten, b, e, _ in host:
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e))
    ctx = vgpu.Context(vgconfig.to_c(p), device=0, max_points=max(s[1] for s in scans) + 16)
    ctx.seed(seq.gt_state(0))
    torch.cuda.synchronize(dev)
    if args.stages:
        ctx.profile(True, stages=True)  # P_k of every IEKF iteration (k_iekf_planes)
    for k, (t, n, b, e) in enumerate(scans):
        ctx.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, host[k][4])
        if k % 8 == 7:
            print("[pmc_run] stepped %d scans" % (k + 1), file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    stats = ctx.stats_log()
    if args.stages:
        ctx.profile(False)
    ctx.close()
    out = {"workload": "synthetic-%s@%s.yaml" % (args.lidar, args.config), "lidar": args.lidar, "config": args.config,
           "seq": args.seq, "win_size": p["LocalBA"]["win_size"], "max_layer": p["LocalBA"]["max_layer"],
           "scans": stats}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(out, open(args.out, "w"))
    print("[pmc_run] %d scans -> %s" % (len(stats), args.out), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
