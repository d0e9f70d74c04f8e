"""Benchmark: scans/s of the full per-scan LIO hot path (downsample + voxel-map
correspondence + IEKF + map maintenance + LM solve) on synthetic LiDAR-inertial
sequences, MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--lidar 64line] [--config mid360]

N > 1 is launched by torch.distributed.run: one process per GPU, each running an
independent sequence (replica mode, "scaling": "weak" — the path has no
cross-sequence exchange). Timed region: K scans after W warm-up scans (the
window must fill before BA/margi run), bracketed by barrier + synchronize;
max over ranks. Inputs are resident in HBM before timing starts.

Rank 0 at N = 1 also times the CPU restatement (oracle, test infrastructure) on
a bounded sample of the same sequence: the cpu_baseline object.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))

import numpy as np  # noqa: E402

METRIC = "scans/sec (downsample+kNN+LM solve), 64-line LiDAR, 1/2/4/8 MI355X; ATE vs CPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--lidar", default="64line")
    ap.add_argument("--config", default="mid360")
    ap.add_argument("--cpu-scans", type=int, default=24, help="oracle sample: scans timed after its own warm-up")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--stage-scans", type=int, default=8, help="untimed profiled scans for the stage breakdown")
    ap.add_argument("--target-steps", type=int, default=20,
                    help="N=1 only: scans timed on the north star's target workload (synthetic 128-line "
                         "/ 200 k rays), reported beside the metric; 0 skips it")
    ap.add_argument("--mode", choices=["replica", "tile"], default="replica",
                    help="replica: an independent sequence per GPU (weak scaling); tile: ONE sequence with its "
                         "voxel map sharded by spatial tile over the GPUs, RCCL all-reduce of the normal "
                         "equations (strong scaling)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import synth
    import vgconfig
    import vgpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    p = vgconfig.load(args.config)
    g = p["General"]
    tile = args.mode == "tile" and world > 1
    seq = synth.Sequence(args.lidar, args.seq + (0 if tile else rank), blind=g["blind"], ext_R=g["extrinsic_rota"],
                         ext_t=g["extrinsic_tran"])
    total = args.warmup + args.steps
    scans, imus = [], []
    for k in range(total + args.stage_scans):
        xyz, inten, b, e = seq.scan(k)
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e))
        imus.append(seq.imu(k))
    npts = int(np.mean([s[1] for s in scans[args.warmup:total]]))
    ctx = vgpu.Context(vgconfig.to_c(p), device=local, max_points=max(s[1] for s in scans) + 16)
    if tile:  # one RCCL communicator inside the library, id from rank 0
        obj = [vgpu.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx.shard_rccl(rank, world, obj[0])
    ctx.seed(seq.gt_state(0))
    torch.cuda.synchronize(dev)

    def run(k):
        t, n, b, e = scans[k]
        ctx.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imus[k])

    for k in range(args.warmup):
        run(k)
    # k_ba_solve launch events on every 4th scan's LM run: each event record
    # leaves a few-us gap in the stream
    ctx.profile(True, every=4)
    stats = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    nlog0 = len(ctx.stats_log())
    t0 = time.perf_counter()
    for k in range(args.warmup, total):
        run(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    stats = ctx.stats_log()[nlog0:]  # completes the last scan's bookkeeping (outside the timed region)
    prof = ctx.profile_read()
    value, dt = aggregate(dt, args.steps, world, dev)
    if tile:  # every rank worked on the same scans
        value /= world
    # per-stage breakdown: a separate, untimed profiled pass over further scans
    # of the same sequence (stage events cost ~6 % of a step)
    stage_ms = {}
    stage_prof = {}
    stage_stats = []
    extra = min(args.stage_scans, len(scans) - total)
    if extra > 0:
        ctx.profile(True, stages=True)
        nlog1 = len(ctx.stats_log())
        for k in range(total, total + extra):
            run(k)
        torch.cuda.synchronize(dev)
        stage_prof = ctx.profile_read()
        stage_stats = ctx.stats_log()[nlog1:]
        stage_ms = {k: round(v["ms"] / extra, 4) for k, v in stage_prof.items() if not k.startswith("host_")}
        ctx.profile(False)

    # roofline of the dominant kernel by device time, k_ba_solve (the LM
    # step's 15W x 15W LDL^T solve, one workgroup, fp64 MFMA trailing
    # updates): algorithmic flops per launch = n^3/3 (LDL^T) + 2 n^2 (the two
    # triangular solves), n = 15 * win_size - 15 (the gauge frame's 15
    # unknowns are decoupled and not factored); peak = MI355X fp64 matrix
    # 78.6 TFLOP/s (AMD spec). Launch time: HIP events around each executed
    # k_ba_solve on the context stream over the timed region.
    W = p["LocalBA"]["win_size"]
    n_sys = 15 * W - 15
    flops = n_sys ** 3 / 3.0 + 2.0 * n_sys ** 2
    sol = prof["ba_solve"]
    s_launch = sol["launches"]
    s_avg = sol["ms"] * 1e-3 / max(s_launch, 1)
    s_ach = flops / s_avg / 1e12 if s_avg > 0 else 0.0
    host_ms = {k[5:]: round(v["ms"] / args.steps, 4) for k, v in prof.items() if k.startswith("host_")}
    roof = {"kernel": "k_ba_solve", "bound": "mfma", "achieved": round(s_ach, 5), "peak": 78.6, "unit": "TFLOP/s",
            "frac": round(s_ach / 78.6, 7), "traffic": None, "avg_launch_us": round(s_avg * 1e6, 3),
            "launches": s_launch, "flops_per_launch": int(flops), "stage_ms_per_scan": stage_ms}
    # secondary: the IEKF point loop k_iekf (HBM-bound gather): 16 B per raw
    # point (fp32 xyz + cached leaf id read) + 4 B per matched point (cached
    # leaf write); plane/node records are cache-resident and not counted. In
    # the timed region the IEKF replays as one hipGraph, so its per-launch
    # events come from the per-stage pass (direct launches, same scans' kind)
    iek = stage_prof.get("iekf", {"ms": 0.0, "launches": 0})
    n_launch = iek["launches"]
    pts = sum(s["n_raw"] * s["iekf_iters"] for s in stage_stats)
    matched = sum(sum(s["iekf_matches"][: s["iekf_iters"]]) for s in stage_stats)
    bytes_tot = 16.0 * pts + 4.0 * matched
    avg_s = iek["ms"] * 1e-3 / max(n_launch, 1)
    achieved = (bytes_tot / max(n_launch, 1)) / avg_s / 1e9 if avg_s > 0 else 0.0
    roof_iekf = {"kernel": "k_iekf", "bound": "hbm", "achieved": round(achieved, 2), "peak": 8000.0, "unit": "GB/s",
                 "frac": round(achieved / 8000.0, 5), "traffic": None, "avg_launch_us": round(avg_s * 1e6, 3),
                 "launches": n_launch}

    # whole-scan algorithmic bytes over the timed scans, a LOWER
    # bound: the per-scan counters do not give the distinct plane records
    # read per IEKF iteration (P_k) or the leaves an insert touches (V_ins),
    # so those terms are left out, and the Hessian passes count once per LM run
    W = p["LocalBA"]["win_size"]
    b_scan = 0.0
    for st in stats:
        b_scan += 16.0 * st["n_raw"] + 16.0 * st["n_ds"]  # read xyz+t, write centroid+count
        b_scan += st["iekf_iters"] * 16.0 * st["n_raw"]  # body xyz + cached leaf per IEKF iteration
        b_scan += 12.0 * st["n_ds"]  # insert
        b_scan += st["n_slide"] * (W * 80.0 + 80.0)  # recut
        b_scan += (1 + st["ba_iters"]) * st["n_factors"] * (W * 80.0 + 176.0)  # BA Hessian + residual passes
    b_scan /= max(len(stats), 1)
    scan_gbps = b_scan / (dt / args.steps) / 1e9 if dt > 0 else 0.0
    roof_scan = {"bound": "hbm", "achieved": round(scan_gbps, 2), "peak": 8000.0, "unit": "GB/s",
                 "frac": round(scan_gbps / 8000.0, 6), "bytes_per_scan": int(b_scan),
                 "note": "SURVEY 8(d) algorithmic bytes per scan / ms_per_step; lower bound (P_k, V_ins omitted)"}

    pmc = pmc_traffic()
    if "k_ba_solve" in pmc:
        roof["traffic"] = pmc["k_ba_solve"]["traffic_bytes"]
        roof["traffic_source"] = pmc["_file"]
    if "k_iekf" in pmc:
        roof_iekf["traffic"] = pmc["k_iekf"]["traffic_bytes"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, p, seq)
    target = None
    if world == 1 and args.target_steps > 0 and args.lidar != "128line":
        target = target_workload(args, p, dev)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "scans/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 4), "higher_is_better": True,
            "scaling": "strong" if tile else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "synthetic-%s@%s.yaml" % (args.lidar, args.config), "lidar": args.lidar,
                       "points_per_scan": npts, "downsampled_per_scan": int(np.mean([s["n_ds"] for s in stats])),
                       "factors_per_scan": int(np.mean([s["n_factors"] for s in stats])),
                       "parallelism": ("tile-sharded x%d" if tile else "replica x%d") % world},
            "roofline": roof, "roofline_k_iekf": roof_iekf, "roofline_scan": roof_scan, "host_ms_per_scan": host_ms,
            "cpu_baseline": cpu, "target_128line": target,
        }
        print(json.dumps(line))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def target_workload(args, p, dev):
    """The north star's target workload (synthetic 128-line clouds, 200,064
    rays) on one GPU, same pipeline and protocol as the metric, fewer scans:
    reported beside the metric, never as `value`."""
    import torch

    import synth
    import vgconfig
    import vgpu
    g = p["General"]
    seq = synth.Sequence("128line", args.seq, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    warm, steps = args.warmup, args.target_steps
    scans, imus = [], []
    for k in range(warm + steps):
        xyz, inten, b, e = seq.scan(k)
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e))
        imus.append(seq.imu(k))
    ctx = vgpu.Context(vgconfig.to_c(p), device=dev.index or 0, max_points=max(s[1] for s in scans) + 16)
    ctx.seed(seq.gt_state(0))

    def run(k):
        t, n, b, e = scans[k]
        ctx.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imus[k])

    for k in range(warm):
        run(k)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        run(k)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    st = ctx.stats_log()[warm:]
    ctx.close()
    return {"workload": "synthetic-128line@%s.yaml" % args.config, "value": round(steps / dt, 3), "unit": "scans/s",
            "ms_per_step": round(dt * 1e3 / steps, 4), "steps": steps, "warmup": warm,
            "points_per_scan": int(np.mean([s[1] for s in scans[warm:]])),
            "downsampled_per_scan": int(np.mean([x["n_ds"] for x in st])) if st else None,
            "factors_per_scan": int(np.mean([x["n_factors"] for x in st])) if st else None}


def pmc_traffic():
    """HBM bytes per launch from the newest committed PMC summary
    (profiles/<round>/pmc_traffic.json, scripts/pmc_summary.py): rocprofv3
    FETCH_SIZE (x2 on gfx950) + WRITE_SIZE, separate passes."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_traffic.json")))
    if not files:
        return {}
    d = json.load(open(files[-1]))["kernels"]
    d["_file"] = os.path.relpath(files[-1], REPO)
    return d


def aggregate(dt, steps, world, dev):
    """Whole-job scans/s from per-rank wall times: max over ranks (RCCL on GPU,
    gloo on CPU), every rank processed `steps` scans of its own sequence."""
    if world > 1:
        import torch
        import torch.distributed as dist
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return world * steps / dt, dt


def cpu_baseline(args, p, seq):
    """Time the CPU restatement (oracle) on a bounded sample of the same sequence."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: the baseline leg only
    import vgconfig

    oracle.build()
    pl = oracle.Pipeline(vgconfig.to_c(p, use_threads=1, vnc_prep=1))
    pl.seed(seq.gt_state(0))
    warm = min(args.warmup, 12)
    times = []
    for k in range(warm + args.cpu_scans):
        xyz, it, b, e = seq.scan(k)
        tm = pl.step(xyz, it, b, e, seq.imu(k))
        if k >= warm:
            times.append(tm[6])
    tot = float(np.sum(times))
    return {"value": round(len(times) / tot, 3), "unit": "scans/s", "cores": 5, "kind": "port",
            "sample": "%d scans after %d warm-up scans of the same synthetic %s sequence, %s.yaml; "
                      "IEKF single-threaded, map/BA 5 std::threads as the reference; median %.1f ms/scan"
                      % (len(times), warm, args.lidar, args.config, 1e3 * float(np.median(times)))}


if __name__ == "__main__":
    main()
