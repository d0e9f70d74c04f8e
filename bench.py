"""Benchmark: scans/s of the full per-scan LIO hot path (downsample + voxel-map
correspondence + IEKF + map maintenance + LM solve) on synthetic LiDAR-inertial
sequences, MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--lidar 64line] [--config mid360]

N > 1 is launched by torch.distributed.run: one process per GPU, each running an
independent sequence (replica mode, "scaling": "weak" — the path has no
cross-sequence exchange). Timed region: K scans after W warm-up scans, bracketed
by barrier + synchronize; max over ranks. The warm-up is raised to at least
win_size + 2 whatever the command line says: the LM and margi run only once the
window is full, so every timed scan is a steady-state scan. Inputs are resident
in HBM before timing starts (vg_step_dev); the host-input rate (vg_step, H2D
copy inside) is reported beside it.

Rank 0 at N = 1 also times the CPU restatement (oracle, test infrastructure) on
a bounded sample of the same sequence (5 worker threads as the reference, and
1 thread): the cpu_baseline object, and the GPU trajectory's ATE against it.
"""
import argparse
import json
import multiprocessing as mproc
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))

import numpy as np  # noqa: E402

METRIC = "scans/sec (downsample+kNN+LM solve), 64-line LiDAR, 1/2/4/8 MI355X; ATE vs CPU"
# one plane record as the correspondence gate reads it: SURVEY 8(d) prices it
# at 112 B (fp32 c, n, radius, 21 sym plane_var); bit-faithful gating reads the
# reference's fp64 record (PlaneRec, 224 B), so the byte model uses that
PLANE_B = 224.0
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md)
FP64_MFMA_TFLOPS = 78.6  # MI355X dense fp64 matrix peak (AMD spec)
FP64_TFLOPS = 78.6       # MI355X fp64 vector peak (AMD spec; k_ba_hess is mostly VALU)


class _StdoutToStderr:
    """fd 1 -> stderr for a block: RCCL prints its version banner on stdout when
    it initialises, which must not precede the bench's one JSON line"""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *a):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--lidar", default="64line")
    ap.add_argument("--config", default="mid360")
    ap.add_argument("--cpu-warmup", type=int, default=20, help="oracle warm-up scans (BASELINE.md: 20)")
    ap.add_argument("--cpu-scans", type=int, default=200,
                    help="oracle sample: timed scans after its warm-up (BASELINE.md: >= 200)")
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
    ap.add_argument("--workers", type=int, default=0,
                    help="scan-generation processes (0: min(16, cpus); 1 under a profiler)")
    ap.add_argument("--no-h2d", action="store_true", help="skip the host-input (vg_step) rate")
    ap.add_argument("--no-tile1", action="store_true", help="skip the one-GPU sharded-path leg")
    ap.add_argument("--max-nodes", type=int, default=0, help="context capacity: octree nodes (0: product default)")
    ap.add_argument("--max-fix", type=int, default=0, help="context capacity: point_fix points (0: default)")
    ap.add_argument("--hash-log2", type=int, default=0, help="context capacity: root hash slots, log2 (0: default)")
    ap.add_argument("--multi", default="2,4,8,16",
                    help="multi-sequence mode (vg_multi_*): B values to time at N=1 (empty: skip); each B runs "
                         "in one child process started before this one touches the GPU, warmed up, then released; "
                         "B distinct sequences")
    ap.add_argument("--multi-1m", default="1,2,4,8",
                    help="BASELINE config 5 (synthetic 1M-ray scans, batched): B values of the multi-sequence "
                         "mode on the 1M workload at N=1 (empty: skip)")
    ap.add_argument("--multi-1m-steps", type=int, default=10, help="timed scans per sequence of the 1M leg")
    ap.add_argument("--multi-active", type=int, default=0,
                    help="at most this many sequences on the device at once (vg_multi_set_active; 0: no cap)")
    ap.add_argument("--multi-child", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--multi-scans", default="", help=argparse.SUPPRESS)
    ap.add_argument("--multi-max-points", type=int, default=0, help=argparse.SUPPRESS)
    return ap.parse_args()


T_START = time.perf_counter()


def beat(msg):
    """One stderr line per bench leg, so that a stalled run names its leg."""
    print("[bench %7.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


def under_profiler():
    """rocprofv3 hands its configuration to the preloaded tool library through
    ROCPROF_* variables; a fork()ed pool inside such a process can deadlock on
    the tool's threads, so scans are then generated in-process."""
    return any(k.startswith("ROCPROF_") for k in os.environ)


# ---- synthetic scans, generated before the GPU is touched (a process pool;
# the ray caster is numpy and ~0.4 s per 64-line scan)
def _gen(job):
    import synth
    lidar, seq_id, blind, ext_R, ext_t, k = job
    seq = synth.Sequence(lidar, seq_id, blind=blind, ext_R=ext_R, ext_t=ext_t)
    xyz, inten, b, e = seq.scan(k)
    return xyz, inten, b, e, seq.imu(k)


def gen_scans(lidar, seq_id, general, n, workers):
    jobs = [(lidar, seq_id, general["blind"], general["extrinsic_rota"], general["extrinsic_tran"], k)
            for k in range(n)]
    if workers <= 1 or n <= 2 or under_profiler():
        return [_gen(j) for j in jobs]
    with mproc.get_context("fork").Pool(min(workers, n)) as pool:
        return pool.map(_gen, jobs, chunksize=1)


CAP = {}  # context capacities (--max-nodes / --max-fix / --hash-log2; 0 = the product's defaults)


def main():
    args = parse()
    CAP.update(max_nodes=args.max_nodes, max_fix_points=args.max_fix, hash_log2=args.hash_log2)
    # recorded in the line: the headline leg runs with the environment's value
    # (HIP's default is 4 hardware queues per process); only the multi-sequence
    # children raise it (multi_children)
    hwq = os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)")
    import synth
    import vgconfig

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    tile = args.mode == "tile" and world > 1
    p = vgconfig.load(args.config)
    g = p["General"]
    W = p["LocalBA"]["win_size"]
    warmup = max(args.warmup, W + 2)
    total = warmup + args.steps
    if args.multi_child:
        return multi_child(args, p, g, warmup, total)
    cpu_on = rank == 0 and world == 1 and not args.no_cpu
    n_need = max(total + args.stage_scans, args.cpu_warmup + args.cpu_scans if cpu_on else 0)
    workers = args.workers or min(16, os.cpu_count() or 8)
    if world > 1:
        workers = max(1, workers // world)
    seq_id = args.seq + (0 if tile else rank)
    beat("generating %d %s scans (workers %d%s)" % (n_need, args.lidar, workers,
                                                   ", in-process: profiler" if under_profiler() else ""))
    host_scans = gen_scans(args.lidar, seq_id, g, n_need, workers)
    tgt_scans = {}
    if world == 1 and args.target_steps > 0 and args.lidar != "128line":
        for cfg in ("mid360", "robosense"):
            beat("generating the 128-line target scans (%s)" % cfg)
            gg = vgconfig.load(cfg)["General"]
            tgt_scans[cfg] = gen_scans("128line", args.seq, gg, warmup + args.target_steps + TARGET_STAGE,
                                       workers)

    multi, multi_1m, scans_1m = None, None, None
    if world == 1 and args.multi:
        multi = multi_children(args, args.lidar, args.multi, warmup, args.steps, workers,
                               first=host_scans[:total])
    if world == 1 and args.multi_1m:
        keep = []  # sequence 0 of the leg, plus TARGET_STAGE scans: its single-context roofline (workload_roofline)
        multi_1m = multi_children(args, "1M", args.multi_1m, warmup, args.multi_1m_steps, workers, keep=keep)
        scans_1m = keep[0] if keep else None

    import torch
    import torch.distributed as dist

    import vgpu
    # VG_BENCH_REHEARSE=1 (replica mode only): the N > 1 flow on a box with
    # fewer GPUs than ranks — every rank on GPU local % count, gloo instead of
    # RCCL for the barriers and the max over ranks (scripts/gpu_rehearse.sh);
    # never part of a reported line
    rehearse = world > 1 and os.environ.get("VG_BENCH_REHEARSE") == "1" and not tile
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        with _StdoutToStderr():  # (RCCL's banner)
            if rehearse:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist.barrier()
    dev = torch.device("cuda", local)
    seq = synth.Sequence(args.lidar, seq_id, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])

    beat("uploading scans, creating the context")
    scans = []
    for xyz, inten, b, e, _ in host_scans:
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e))
    imus = [h[4] for h in host_scans]
    npts = int(np.mean([s[1] for s in scans[warmup:total]]))
    ctx = vgpu.Context(vgconfig.to_c(p), device=local, max_points=max(s[1] for s in scans) + 16, **CAP)
    # same-build A/B experiments only: VG_BENCH_DEBUG="key=value,..." sets test knobs (vgx_debug) on the
    # metric leg's context; the line records them
    dbg = os.environ.get("VG_BENCH_DEBUG", "")
    for kv in filter(None, dbg.split(",")):
        k, v = kv.split("=")
        ctx.debug(int(k), int(v))
    if tile:  # one RCCL communicator inside the library, id from rank 0
        with _StdoutToStderr():
            obj = [vgpu.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.shard_rccl(rank, world, obj[0])
    ctx.seed(seq.gt_state(0))
    torch.cuda.synchronize(dev)

    # the per-scan arguments converted before the timed region: each step is
    # one call with resident pointers, as a C++ caller's would be
    prepped = [ctx.prep_step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e,
                                 imus[k]) for k, (t, n, b, e) in enumerate(scans)]

    def run(k):
        if os.environ.get("VG_BENCH_UNPREPPED"):  # A/B knob: per-step argument conversion in the timed region
            t, n, b, e = scans[k]
            ctx.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imus[k])
            return
        ctx.step_prepped(prepped[k])

    beat("metric leg: %d warm-up + %d timed scans" % (warmup, args.steps))
    for k in range(warmup):
        run(k)
    # k_ba_solve launch events on every 4th scan's LM run: each event record
    # leaves a few-us gap in the stream
    # host stage timers + the in-kernel clocks of k_iekf / k_ba_solve (no
    # events in the stream: every graph replays as it does untimed)
    ctx.profile(True, clock=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    nlog0 = len(ctx.stats_log())
    t0 = time.perf_counter()
    for k in range(warmup, total):
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
    # of the same sequence (stage events cost ~6 % of a step); it also counts
    # the distinct plane records each IEKF iteration reads (P_k)
    stage_ms, stage_prof, stage_stats = {}, {}, []
    extra = min(args.stage_scans, len(scans) - total)
    if extra > 0:
        beat("per-stage pass: %d scans" % extra)
        ctx.profile(True, stages=True)
        nlog1 = len(ctx.stats_log())
        for k in range(total, total + extra):
            run(k)
        torch.cuda.synchronize(dev)
        stage_prof = ctx.profile_read()
        stage_stats = ctx.stats_log()[nlog1:]
        stage_ms = {k: round(v["ms"] / extra, 4) for k, v in stage_prof.items()
                    if not k.startswith("host_") and not k.endswith("_clock")}
        ctx.profile(False)
    # the rest of the CPU baseline's sample, untimed: the ATE is taken over the
    # same scans as the CPU timing (>= 200 after a 20-scan warm-up)
    for k in range(total + max(extra, 0), len(scans)):
        run(k)
    traj_gpu = ctx.trajectory()
    ctx.close()
    host_ms = {k[5:]: round(v["ms"] / args.steps, 4) for k, v in prof.items() if k.startswith("host_")}

    # P_k of the timed scans themselves, from the committed PMC pass over the
    # same scans (scripts/pmc_run.py: same workload, sequence and warm-up; the
    # pipeline is deterministic, so a scan's P_k is the same in every run)
    pmc = pmc_traffic()
    pk_scans = pmc_pk(pmc, "synthetic-%s@%s.yaml" % (args.lidar, args.config), seq_id, warmup, total, stats)
    # ---- headline roofline: the whole scan against HBM -------
    roof = scan_roofline(stats, stage_stats, W, dt / args.steps, pk_scans)
    # ---- per-kernel rooflines ----------------------------------------------
    # Kernel-only launch times from the in-kernel clocks (vg_profile bit 2:
    # the device's constant-rate wall clock read inside the kernel, executed
    # launches of the timed region, graph replays as untimed; rocprofv3's
    # kernel average of the same command is the cross-check, profiles/).
    # k_ba_solve (the LM step's 15W x 15W LDL^T, one workgroup, fp64 MFMA
    # trailing updates): algorithmic flops per launch = n^3/3 + 2 n^2 with
    # n = 15 W - 15 (the gauge frame is not factored)
    n_sys = 15 * W - 15
    flops = n_sys ** 3 / 3.0 + 2.0 * n_sys ** 2
    sol = prof["k_ba_solve_clock"]
    s_avg = sol["ms"] * 1e-3 / max(sol["launches"], 1)
    s_ach = flops / s_avg / 1e12 if s_avg > 0 else 0.0
    roof_solve = {"kernel": "k_ba_solve", "bound": "mfma", "achieved": round(s_ach, 5), "peak": FP64_MFMA_TFLOPS,
                  "unit": "TFLOP/s", "frac": round(s_ach / FP64_MFMA_TFLOPS, 7), "traffic": None,
                  "avg_launch_us": round(s_avg * 1e6, 3), "launches": sol["launches"], "flops_per_launch": int(flops),
                  "timing": "in-kernel clock (wall_clock64), executed launches of the timed region"}
    # k_iekf (hot loop #1, HBM-bound gather): 16 B per raw point (fp32 xyz +
    # cached leaf) + PLANE_B per distinct plane record (P_k) per launch. The
    # timed scans' own point counts, iteration counts and P_k (from the PMC
    # pass over the same scans; else the per-stage pass's mean)
    iek = prof["k_iekf_clock"]
    n_launch = iek["launches"]
    it_n = sum(s["iekf_iters"] for s in stage_stats)
    p_mean = sum(sum(s["iekf_planes"][: s["iekf_iters"]]) for s in stage_stats) / it_n if it_n else 0.0
    it_t = sum(s["iekf_iters"] for s in stats)
    if pk_scans:
        bytes_tot = sum(s["iekf_iters"] * 16.0 * s["n_raw"] + PLANE_B * sum(pk[: s["iekf_iters"]])
                        for s, pk in zip(stats, pk_scans))
        p_mean = sum(sum(pk[: s["iekf_iters"]]) for s, pk in zip(stats, pk_scans)) / max(it_t, 1)
    else:
        bytes_tot = sum(s["iekf_iters"] * 16.0 * s["n_raw"] for s in stats) + PLANE_B * p_mean * it_t
    avg_s = iek["ms"] * 1e-3 / max(n_launch, 1)
    bpl = bytes_tot / max(it_t, 1)
    achieved = bpl / avg_s / 1e9 if avg_s > 0 else 0.0
    ev = stage_prof.get("iekf", {"ms": 0.0, "launches": 0})
    roof_iekf = {"kernel": "k_iekf", "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                 "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": None,
                 "avg_launch_us": round(avg_s * 1e6, 3), "launches": n_launch, "iterations_executed": it_t,
                 "bytes_per_launch": int(bpl), "P_k_mean": round(p_mean, 1),
                 "timing": "in-kernel clock (wall_clock64: first workgroup start -> last workgroup end), executed "
                           "launches of the timed region",
                 "P_k_source": "PMC pass over the same scans (%s)" % pmc.get("_file") if pk_scans else
                               "per-stage pass mean",
                 "event_interval_us": round(ev["ms"] * 1e3 / ev["launches"], 3) if ev["launches"] else None}
    # the recut's level kernels (k_rc_level0 + max_layer x k_rc_level), one
    # span per scan: SURVEY 8(d)'s recut bytes V_slide (80 W + 80) per scan
    rck = prof["k_rc_clock"]
    rc_s = rck["ms"] * 1e-3 / max(rck["launches"], 1)
    rc_b = sum(s["n_slide"] * (80.0 * W + 80.0) for s in stats) / max(len(stats), 1)
    rc_a = rc_b / rc_s / 1e9 if rc_s > 0 else 0.0
    roof_rc = {"kernel": "k_rc_level0 + %d x k_rc_level (the recut's levels, one span per scan)" % p["LocalBA"]["max_layer"],
               "bound": "hbm", "achieved": round(rc_a, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
               "frac": round(rc_a / HBM_PEAK_GBPS, 6), "traffic": None, "avg_span_us": round(rc_s * 1e6, 3),
               "spans": rck["launches"], "bytes_per_scan": int(rc_b),
               "timing": "in-kernel clock: k_rc_level0's first workgroup start -> the last level kernel's last "
                         "workgroup end, timed scans"}
    # k_ba_hess (the LM's LiDAR + IMU Hessian pass): SURVEY 8(d)'s BA bytes
    # F (80 W + 176) per pass; fp64 flops per pass from the kernel's operations
    # (hess_flops: counted per (factor, frame) lane, off-diagonal X^T S X,
    # the ordered reduction and the IMU factor blocks)
    hk = prof["k_ba_hess_clock"]
    h_s = hk["ms"] * 1e-3 / max(hk["launches"], 1)
    nh = sum(s["ba_hess"] for s in stats)
    h_b = sum(s["ba_hess"] * s["n_factors"] * (80.0 * W + 176.0) for s in stats) / max(nh, 1)
    h_f = sum(s["ba_hess"] * hess_flops(W, s["n_factors"]) for s in stats) / max(nh, 1)
    h_a = h_b / h_s / 1e9 if h_s > 0 else 0.0
    h_t = h_f / h_s / 1e12 if h_s > 0 else 0.0
    roof_hess = {"kernel": "k_ba_hess", "bound": "hbm", "achieved": round(h_a, 2), "peak": HBM_PEAK_GBPS,
                 "unit": "GB/s", "frac": round(h_a / HBM_PEAK_GBPS, 6), "traffic": None,
                 "avg_launch_us": round(h_s * 1e6, 3), "launches": hk["launches"], "bytes_per_launch": int(h_b),
                 "fp64": {"flops_per_launch": int(h_f), "achieved_tflops": round(h_t, 4), "peak_tflops": FP64_TFLOPS,
                          "frac": round(h_t / FP64_TFLOPS, 6)},
                 "timing": "in-kernel clock (first workgroup start -> last workgroup end), executed launches of the "
                           "timed region"}
    # traffic: FETCH x2 + WRITE per unit (MI355X_MICROARCH.md), and its ratio
    # to the algorithmic bytes, both over the same launches of the PMC pass
    # (scripts/pmc_summary.py; a fixed set of scans, so the same whatever
    # --steps this run times)
    for r, key in ((roof_solve, "k_ba_solve"), (roof_iekf, "k_iekf"), (roof_rc, "recut_levels"),
                   (roof_hess, "k_ba_hess")):
        e = pmc.get(key)
        if not e:
            continue
        r["traffic"] = e["traffic_bytes"]
        r["traffic_source"] = pmc["_file"]
        if e.get("traffic_ratio") is not None:
            r["traffic_ratio"] = e["traffic_ratio"]
            r["traffic_unit"] = e["unit"]
            r["traffic_alg_bytes"] = e["alg_bytes"]
        if "fetch_calibrated" in e:
            r["fetch_calibrated"] = dict(e["fetch_calibrated"], note="measured FETCH_SIZE bytes (no x2) / the FETCH "
                                         "the algorithmic bytes produce at the calibrated per-shape ratios, same "
                                         "launches of the PMC pass")
        if "own_store_bytes" in e:  # k_ba_hess: its own stores; WRITE_SIZE adds evicted dirty lines
            r["own_store_bytes"] = e["own_store_bytes"]
    roof["stage_ms_per_scan"] = stage_ms

    # the legs after the metric's: a leg that fails records its error in the
    # line (which still prints, with the metric) and the exit status reports it
    leg_errors = {}

    def leg(name, fn):
        try:
            return fn()
        except Exception as ex:  # noqa: BLE001
            leg_errors[name] = "%s: %s" % (type(ex).__name__, str(ex)[-300:])
            beat("%s failed: %s" % (name, leg_errors[name]))
            return {"error": leg_errors[name]}

    h2d = None
    if world == 1 and not args.no_h2d:
        beat("host-input leg")
        h2d = leg("host_input", lambda: host_input_rate(p, seq, host_scans, imus, warmup, args.steps, dev))
    tile1 = None
    if world == 1 and not args.no_tile1:
        beat("sharded-path leg on one GPU")
        tile1 = leg("tile_path_1gpu", lambda: tile_path_rate(p, seq, scans, imus, warmup, args.steps, dev, value))
    cpu, ate_cpu = None, None
    if cpu_on:
        beat("CPU baseline: %d + %d scans, 5 threads then 1" % (args.cpu_warmup, args.cpu_scans))
        res = leg("cpu_baseline", lambda: cpu_baseline(args, p, seq, host_scans))
        if isinstance(res, dict):
            cpu = res
        else:
            cpu, traj_cpu = res
            lo, hi = args.cpu_warmup, min(traj_cpu.shape[0], traj_gpu.shape[0])
            if hi > lo:
                d = np.linalg.norm(traj_cpu[lo:hi, 10:13] - traj_gpu[lo:hi, 10:13], axis=1)
                ate_cpu = {"ate_m": float("%.3e" % np.sqrt(np.mean(d ** 2))), "max_m": float("%.3e" % d.max()),
                           "scans": hi - lo, "first_scan": lo,
                           "reference": "CPU restatement, 5 threads, the CPU baseline's own scans",
                           "tolerance_m": 0.01}
    targets = {}
    for cfg, sc in tgt_scans.items():
        beat("128-line target workload (%s)" % cfg)
        targets[cfg] = leg("target_128line." + cfg, lambda: target_workload(args, cfg, sc, warmup, dev))
    w1 = None
    if multi_1m and scans_1m:
        beat("1M workload: single-context roofline")
        w1 = leg("multi_sequence_1M.single_context",
                 lambda: target_workload(args, args.config, scans_1m, warmup, dev, lidar="1M"))
    if w1 and "error" not in w1:
        multi_1m["bytes_per_scan"] = w1["bytes_per_scan"]
        multi_1m["counters_mean"] = w1["counters_mean"]
        multi_1m["single_context"] = {k: w1[k] for k in ("value", "ms_per_step", "steps", "achieved", "frac")}
        multi_1m["roofline_frac_by_B"] = {B: round(v * w1["bytes_per_scan"] / (HBM_PEAK_GBPS * 1e9), 6)
                                          for B, v in multi_1m["by_B"].items()}
        multi_1m["roofline_note"] = ("SURVEY 8(d) algorithmic bytes per 1M-ray scan (sequence 0 of the leg, one "
                                     "context, its own counters) x by_B / 8 TB/s")

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "scans/s", "n_gpus": world, "steps": args.steps,
            "warmup": warmup, "warmup_requested": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong" if tile else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "synthetic-%s@%s.yaml" % (args.lidar, args.config), "lidar": args.lidar,
                       "rays_per_scan": int(synth.LIDARS[args.lidar][0] * synth.LIDARS[args.lidar][1]),
                       "points_per_scan": npts, "downsampled_per_scan": int(np.mean([s["n_ds"] for s in stats])),
                       "nodes_used_end": int(stats[-1]["nodes_used"]), "fix_used_end": int(stats[-1]["fix_used"]),
                       "factors_per_scan": int(np.mean([s["n_factors"] for s in stats])),
                       "lm_iters_per_scan": round(float(np.mean([s["ba_iters"] for s in stats])), 2),
                       "parallelism": ("tile-sharded x%d" if tile else "replica x%d") % world,
                       "vnc_prep": "skipped on the GPU: matchVoxelMap always returns 0, so the scan-plane prep "
                                   "(voxel_map.cpp:169-200, octree.cpp:628-684, odometry.cpp:22-61) never changes "
                                   "the output (SURVEY A8); the CPU baseline pays it"},
            "roofline": roof, "roofline_k_ba_solve": roof_solve, "roofline_k_iekf": roof_iekf,
            "roofline_k_rc_level": roof_rc, "roofline_k_ba_hess": roof_hess,
            "host_ms_per_scan": host_ms, "host_input": h2d, "tile_path_1gpu": tile1, "cpu_baseline": cpu,
            "ate_vs_cpu": ate_cpu,
            "target_128line": targets or None, "multi_sequence": multi_roofline(multi, roof),
            "multi_sequence_1M": multi_1m, "env": {"GPU_MAX_HW_QUEUES": hwq, "VG_BENCH_DEBUG": dbg or None},
            **({"rehearsal": "VG_BENCH_REHEARSE: %d ranks on %d GPU(s) over gloo, not a measurement"
                % (world, torch.cuda.device_count())} if rehearse else {}),
        }
        print(json.dumps(line), flush=True)
        # a multi-sequence child that crashed is a defect, not a data point: the
        # line above keeps what was measured (failed_by_B names the B), the exit
        # status reports the failure
        failed = {k: v.get("failed_by_B") for k, v in (("64line", multi), ("1M", multi_1m)) if v and v.get("failed_by_B")}
        if failed:
            print("bench: multi-sequence children failed: %s" % json.dumps(failed), file=sys.stderr, flush=True)
        if leg_errors:
            print("bench: legs failed: %s" % json.dumps(leg_errors), file=sys.stderr, flush=True)
        if failed or leg_errors:
            sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


def scan_roofline(stats, stage_stats, W, t_scan, pk_scans=None):
    """Whole-scan algorithmic bytes per timed scan / its wall time:
    B = 16 N_raw + 16 N_ds + sum_k (12 N_raw + 4 N_raw + PLANE_B P_k) + 12 N_ds
        + 2 V_ins 440 + V_slide (80 W + 80) + (I_H + I_R) F (80 W + 176).
    Every counter is the timed scan's own (I_H = Hessian passes, I_R = LM
    iterations), except P_k, which is counted only in the per-stage pass
    (distinct plane records per IEKF iteration) and enters as that pass's mean
    per executed iteration."""
    it_n = sum(s["iekf_iters"] for s in stage_stats)
    p_mean = sum(sum(s["iekf_planes"][: s["iekf_iters"]]) for s in stage_stats) / it_n if it_n else 0.0
    if pk_scans:  # the timed scans' own P_k (PMC pass over the same scans)
        it_t = sum(s["iekf_iters"] for s in stats)
        p_mean = sum(sum(pk[: s["iekf_iters"]]) for s, pk in zip(stats, pk_scans)) / max(it_t, 1)
    b = 0.0
    for q, s in enumerate(stats):
        b += 16.0 * s["n_raw"] + 16.0 * s["n_ds"]
        if pk_scans:
            b += s["iekf_iters"] * 16.0 * s["n_raw"] + PLANE_B * sum(pk_scans[q][: s["iekf_iters"]])
        else:
            b += s["iekf_iters"] * (16.0 * s["n_raw"] + PLANE_B * p_mean)
        b += 12.0 * s["n_ds"] + 2.0 * s["v_ins"] * 440.0
        b += s["n_slide"] * (W * 80.0 + 80.0)
        b += (s["ba_hess"] + s["ba_iters"]) * s["n_factors"] * (W * 80.0 + 176.0)
    b /= max(len(stats), 1)
    gbps = b / t_scan / 1e9 if t_scan > 0 else 0.0
    mean = lambda k: round(float(np.mean([s[k] for s in stats])), 1)  # noqa: E731
    return {"kernel": "whole scan (every kernel of the per-scan path)", "bound": "hbm", "achieved": round(gbps, 2),
            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(gbps / HBM_PEAK_GBPS, 6), "traffic": None,
            "bytes_per_scan": int(b), "scan_us": round(t_scan * 1e6, 2),
            "counters_mean": {"N_raw": mean("n_raw"), "N_ds": mean("n_ds"), "K": mean("iekf_iters"),
                              "P_k": round(p_mean, 1), "V_ins": mean("v_ins"), "V_slide": mean("n_slide"),
                              "F": mean("n_factors"), "I_H": mean("ba_hess"), "I_R": mean("ba_iters")},
            "note": "SURVEY 8(d) algorithmic bytes per scan / ms_per_step, plane records at %d B (fp64, as the "
                    "gate reads them; SURVEY prices 112 B fp32); P_k %s" % (
                        PLANE_B, "of each timed scan (PMC pass over the same scans)" if pk_scans else
                        "from the per-stage pass")}


def multi_roofline(multi, roof):
    """The whole-scan HBM fraction of each multi-sequence rate (the same scans,
    so the same SURVEY 8(d) algorithmic bytes per scan as the metric's)."""
    if not multi or not roof or not roof.get("bytes_per_scan"):
        return multi
    multi["roofline_frac_by_B"] = {B: round(v * roof["bytes_per_scan"] / (roof["peak"] * 1e9), 6)
                                   for B, v in multi["by_B"].items()}
    return multi


def multi_children(args, lidar, Bs, warmup, steps, workers, first=None, keep=None):
    """A multi-sequence leg (vg_multi_*), one child process per B, started
    before this process initialises the GPU: HIP keeps every hardware queue a
    process has created, and once a process holds more queues than the
    sequences need, sequences end up sharing queues (measured: the same B = 4
    run at 1,100 or 3,300 scans/s depending on the streams created before it).
    Every context runs a distinct synthetic sequence (seed args.seq + b; no two
    contexts read the same scan). GPU_MAX_HW_QUEUES (children only): 16, a
    hardware queue per stream. Past four sequences the library runs them on
    four shared streams (vg_multi_create; more busy hardware queues are
    time-sliced by the GPU).
    """
    import subprocess
    import tempfile

    import vgconfig
    g = vgconfig.load(args.config)["General"]
    Bs = [int(b) for b in Bs.split(",")]
    total = warmup + steps
    paths = []
    out = {"lidar": lidar, "unit": "scans/s", "steps": steps, "warmup": warmup,
           "workers": "B <= 4: one native thread + one stream per sequence; B > 4: four streams, one thread "
                      "each, stepping its sequences (b % 4) one scan each in turn (vg_multi_create)",
           "inputs": "B distinct sequences",
           "wait_policy": "spin",
           "process": "one process per B, released after its warm-up%s; rate = B x steps / (release -> end)"
                      % (", at most %d sequences on the device at once (vg_multi_set_active)" % args.multi_active
                         if args.multi_active > 0 else ""),
           "env": {"GPU_MAX_HW_QUEUES": "16"},
           "by_B": {}}
    npmax = 0
    try:
        for b in range(max(Bs)):
            beat("multi-sequence %s: generating sequence %d of %d" % (lidar, b + 1, max(Bs)))
            sc = first if (b == 0 and first is not None) else gen_scans(
                lidar, args.seq + b, g, total + (TARGET_STAGE if b == 0 and keep is not None else 0), workers)
            if b == 0 and keep is not None:
                keep.append(sc)
            fd, path = tempfile.mkstemp(suffix=".npz", prefix="vg_multi_")
            os.close(fd)
            arrs = {}
            for k, (xyz, inten, tb, te, imu) in enumerate(sc[:total]):
                arrs["x%d" % k], arrs["i%d" % k], arrs["m%d" % k] = xyz, inten, imu
                arrs["t%d" % k] = np.array([tb, te])
                npmax = max(npmax, xyz.shape[0])
            np.savez(path, **arrs)
            paths.append(path)
            del sc, arrs
        hwq = os.environ.get("VG_MULTI_HWQ", "16")  # experiments only; the line records what ran
        out["env"]["GPU_MAX_HW_QUEUES"] = hwq
        env = dict(os.environ, GPU_MAX_HW_QUEUES=hwq)
        wait = os.environ.get("VG_MULTI_WAIT", "")  # experiments: "spin_us,sleep_us" (the line records it)
        if wait:
            out["wait_policy"] = "spin %s us, then sleep %s us" % tuple(wait.split(","))
        for B in Bs:
            # a child that fails (or crashes) costs this B its number, not the line
            runs = []
            try:
                beat("multi-sequence %s: B = %d" % (lidar, B))
                # the child warms up, reports READY and waits; the parent then
                # releases it and times the job from GO to its end.
                # ONE process per B. Past ~4 busy hardware queues the GPU
                # time-slices them (profiles/r04/multi_pmc_r04g.json: same L2 hit
                # rates, a ~47 us floor per kernel at B = 8); past four
                # sequences the library therefore shares four streams among
                # them (B = 8: 3,837 scans/s against 2,970 over eight streams
                # sharing four hardware queues, profiles/r06/multi_streams_r06.txt)
                P = 1
                benv = env
                out.setdefault("hw_queues_by_B", {})[str(B)] = int(benv["GPU_MAX_HW_QUEUES"])
                ms = os.environ.get("VG_MULTI_STREAMS")
                G = int(ms) if ms is not None else (4 if B > 4 else 0)
                out.setdefault("streams_by_B", {})[str(B)] = G if 0 < G < B else B
                sizes = [B // P + (1 if q < B % P else 0) for q in range(P)]
                runs, first_seq = [], 0
                for q in range(P):
                    cmd = [sys.executable, os.path.abspath(__file__), "--multi-child", str(sizes[q]),
                           "--multi-scans", ",".join(paths[first_seq:first_seq + sizes[q]]),
                           "--multi-max-points", str(npmax + 16),
                           "--lidar", lidar, "--config", args.config, "--steps", str(steps), "--warmup", str(args.warmup),
                           "--max-nodes", str(args.max_nodes), "--max-fix", str(args.max_fix),
                           "--hash-log2", str(args.hash_log2), "--multi-active", str(args.multi_active)]
                    first_seq += sizes[q]
                    runs.append(subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=benv))
                for r in runs:  # every child warmed up and idle
                    line = r.stdout.readline()
                    if line.strip() != "READY":
                        for x in runs:
                            x.kill()
                        raise RuntimeError("multi-sequence child B=%d: %r" % (B, line[-500:]))
                t0 = time.perf_counter()
                for r in runs:
                    r.stdin.write("GO\n")
                    r.stdin.flush()
                res = []
                for r in runs:
                    res.append(json.loads(r.stdout.readline()))
                wall = time.perf_counter() - t0
                for r in runs:
                    r.stdin.close()
                    r.wait(timeout=60)
                    if r.returncode != 0:
                        raise RuntimeError("multi-sequence child B=%d failed (%d)" % (B, r.returncode))
                out["by_B"][str(B)] = round(B * steps / wall, 1)
                out.setdefault("processes_by_B", {})[str(B)] = P
                out.setdefault("points_per_scan", res[0]["points_per_scan"])
            except Exception as ex:  # noqa: BLE001
                for r in runs:
                    if r.poll() is None:
                        r.kill()
                out.setdefault("failed_by_B", {})[str(B)] = str(ex)[-300:]
                beat("multi-sequence %s: B = %d failed: %s" % (lidar, B, str(ex)[-200:]))
    finally:
        for path in paths:
            os.unlink(path)
    return out


def multi_child(args, p, g, warmup, total):
    """One B of a multi-sequence leg: B contexts on one GPU, one native worker
    thread each, context b stepping its own sequence's resident scans; whole-job
    scans/s over the timed scans after the warm-up."""
    import torch

    import synth
    import vgconfig
    import vgpu
    B = args.multi_child
    dev = torch.device("cuda", 0)
    data = []
    for path in args.multi_scans.split(",")[:B]:
        z = np.load(path)
        sc = []
        for k in range(total):
            xyz, inten = z["x%d" % k], z["i%d" % k]
            t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
            tb, te = z["t%d" % k]
            sc.append((t, xyz.shape[0], float(tb), float(te), z["m%d" % k]))
        data.append(sc)
    seq = synth.Sequence(args.lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    ctxs = [vgpu.Context(vgconfig.to_c(p), device=0, max_points=args.multi_max_points, **CAP) for _ in range(B)]
    for c in ctxs:
        c.seed(seq.gt_state(0))  # every synthetic sequence follows the same trajectory (synth.Trajectory)
    wait = os.environ.get("VG_MULTI_WAIT", "")
    mv = vgpu.Multi(ctxs, *([int(v) for v in wait.split(",")] if wait else [0, 0]))
    if 0 < args.multi_active < B:
        mv.set_active(args.multi_active)

    def step(k):
        scans = []
        for d in data:
            t, n, tb, te, imu = d[k]
            scans.append((t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), 0, n, tb, te, imu))
        mv.step_dev(scans)

    for k in range(warmup):
        step(k)
    mv.sync()
    torch.cuda.synchronize(dev)
    print("READY", flush=True)  # the parent releases every child of this B at once
    if sys.stdin.readline().strip() != "GO":
        return 1
    t0 = time.perf_counter()
    for k in range(warmup, total):
        step(k)
    mv.sync()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    npts = int(np.mean([d[k][1] for d in data for k in range(warmup, total)]))
    print(json.dumps({"B": B, "scans_per_s": round(B * (total - warmup) / dt, 1), "points_per_scan": npts}), flush=True)
    mv.close()
    for c in ctxs:
        c.close()
    return 0


def tile_path_rate(p, seq, scans, imus, warmup, steps, dev, unsharded):
    """The spatial-tile sharded code path (BASELINE config 4) on ONE GPU: a
    one-rank RCCL communicator (vgx_debug 30), so every exchange point runs its
    collective (ncclAllReduce on the context stream, the guarded frames) and
    the scan takes the sharded launches (no scan graph, no IEKF/margi overlap).
    Against the unsharded metric leg on the same scans: the sharded path's own
    cost per scan, no peer traffic (RCCL over xGMI is unmeasured here)."""
    import torch

    import vgconfig
    import vgpu
    n = min(warmup + steps, len(scans))
    ctx = vgpu.Context(vgconfig.to_c(p), device=dev.index or 0, max_points=max(s[1] for s in scans) + 16, **CAP)
    ctx.debug(30, 1)
    for kv in filter(None, os.environ.get("VG_TILE_DEBUG", "").split(",")):  # same-build A/Bs of this leg only
        k_, v_ = kv.split("=")
        ctx.debug(int(k_), int(v_))
    with _StdoutToStderr():  # (RCCL's banner)
        ctx.shard_rccl(0, 1, vgpu.rccl_unique_id())
    ctx.seed(seq.gt_state(0))
    prepped = [ctx.prep_step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), m, b, e, imus[k])
               for k, (t, m, b, e) in enumerate(scans[:n])]
    for k in range(warmup):
        ctx.step_prepped(prepped[k])
    ctx.stats_log()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(warmup, n):
        ctx.step_prepped(prepped[k])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ctx.stats_log()
    ctx.close()
    k = n - warmup
    v = k / dt
    return {"value": round(v, 3), "unit": "scans/s", "ms_per_step": round(dt * 1e3 / k, 4), "steps": k,
            "overhead_ms_per_scan": round(dt * 1e3 / k - 1e3 / unsharded, 4),
            "note": "the tile-sharded path (config 4) with a one-rank RCCL communicator (vgx_debug 30): every "
                    "exchange runs ncclAllReduce on the stream, direct launches, no peer traffic; overhead vs the "
                    "unsharded metric leg on the same scans",
            "debug": os.environ.get("VG_TILE_DEBUG") or None}


def host_input_rate(p, seq, host_scans, imus, warmup, steps, dev):
    """The same protocol through vg_step with host buffers (the scan's H2D copy
    inside the timed region, as a src/pipeline caller would pay it)."""
    import torch

    import vgconfig
    import vgpu
    n = min(warmup + steps, len(host_scans))
    ctx = vgpu.Context(vgconfig.to_c(p), device=dev.index or 0, max_points=max(h[0].shape[0] for h in host_scans) + 16,
                       **CAP)
    ctx.seed(seq.gt_state(0))
    xs = [np.ascontiguousarray(h[0]) for h in host_scans[:n]]
    its = [np.ascontiguousarray(h[1]) for h in host_scans[:n]]
    for k in range(warmup):
        ctx.step(xs[k], its[k], host_scans[k][2], host_scans[k][3], imus[k])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(warmup, n):
        ctx.step(xs[k], its[k], host_scans[k][2], host_scans[k][3], imus[k])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ctx.stats_log()
    ctx.close()
    k = n - warmup
    return {"value": round(k / dt, 3), "unit": "scans/s", "ms_per_step": round(dt * 1e3 / k, 4), "steps": k,
            "note": "vg_step: host xyz (AoS) + intensity inside the timed region: one copy into a pinned "
                    "in-flight slot, DMA to HBM and AoS->SoA unpack on the device ahead of the scan's kernels"}


TARGET_STAGE = 4  # per-stage scans after the target workload's timed ones (P_k for its roofline)


def target_workload(args, cfg, host, warm, dev, lidar="128line"):
    """The north star's target workload (synthetic 128-line clouds, 200,064
    rays) on one GPU, same pipeline and protocol as the metric, fewer scans:
    reported beside the metric, never as `value`. Its whole-scan roofline uses
    the same SURVEY 8(d) byte model (scan_roofline) with this workload's own
    counters; P_k comes from TARGET_STAGE untimed per-stage scans after it."""
    import torch

    import synth
    import vgconfig
    import vgpu
    p = vgconfig.load(cfg)
    g = p["General"]
    W = p["LocalBA"]["win_size"]
    seq = synth.Sequence(lidar, args.seq, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    steps = len(host) - warm - TARGET_STAGE
    scans = []
    for xyz, inten, b, e, _ in host:
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e))
    ctx = vgpu.Context(vgconfig.to_c(p), device=dev.index or 0, max_points=max(s[1] for s in scans) + 16, **CAP)
    ctx.seed(seq.gt_state(0))

    def run(k):
        t, n, b, e = scans[k]
        ctx.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, host[k][4])

    for k in range(warm):
        run(k)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        run(k)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    st = ctx.stats_log()[warm:]
    ctx.profile(True, stages=True)
    for k in range(warm + steps, len(scans)):
        run(k)
    torch.cuda.synchronize(dev)
    stage_st = ctx.stats_log()[warm + steps:]
    ctx.profile(False)
    ctx.close()
    roof = scan_roofline(st, stage_st, W, dt / steps)
    return {"workload": "synthetic-%s@%s.yaml" % (lidar, cfg), "value": round(steps / dt, 3), "unit": "scans/s",
            "ms_per_step": round(dt * 1e3 / steps, 4), "steps": steps, "warmup": warm,
            "rays_per_scan": int(synth.LIDARS[lidar][0] * synth.LIDARS[lidar][1]),
            "points_per_scan": int(np.mean([s[1] for s in scans[warm:warm + steps]])),
            "downsampled_per_scan": int(np.mean([x["n_ds"] for x in st])) if st else None,
            "factors_per_scan": int(np.mean([x["n_factors"] for x in st])) if st else None,
            "lm": bool(p["General"]["if_BA"]),
            "bytes_per_scan": roof["bytes_per_scan"], "achieved": roof["achieved"], "peak": roof["peak"],
            "unit_roofline": roof["unit"], "frac": roof["frac"], "counters_mean": roof["counters_mean"]}


def pmc_traffic():
    """HBM bytes per unit from the newest committed PMC summary
    (profiles/<round>/pmc_traffic.json, scripts/pmc_summary.py): rocprofv3
    FETCH_SIZE (x2 on gfx950) + WRITE_SIZE, separate passes, paired with the
    algorithmic bytes of the same launches."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_traffic.json")))
    if not files:
        return {}
    f = json.load(open(files[-1]))
    d = dict(f["kernels"])
    d["_file"] = os.path.relpath(files[-1], REPO)
    d["_meta"] = {k: f.get(k) for k in ("workload", "seq", "per_scan")}
    return d


def pmc_pk(pmc, workload, seq_id, first, end, stats):
    """The per-iteration P_k of scans [first, end) of this workload from the
    PMC pass's log, when that pass ran the same workload and sequence and its
    point counts agree with this run's (the same scans); else None."""
    m = pmc.get("_meta") or {}
    ps = m.get("per_scan")
    if not ps or m.get("workload") != workload or m.get("seq") != seq_id or len(ps["P_k"]) < end:
        return None
    if [s["n_raw"] for s in stats] != ps["n_raw"][first:end]:
        return None
    return ps["P_k"][first:end]


def hess_flops(W, F):
    """fp64 flops of one k_ba_hess pass over F factors, counted from the
    kernel's operations: per (factor, frame) lane
    factor_frame's ~972 (A_uk, the diagonal block A^T umumT A + corrections,
    the gradient, the three rank-1 rows) + 54 accumulating it; per factor the
    lower off-diagonal blocks as three rank-1 terms, 3 (18 W^2 - 18 W) x 2,
    plus their S scaling 18 W and the ordered row reduction 27 W; per IMU
    factor J^T C (450 x 29), J^T C J (900 x 29), J^T C r and r^T C r."""
    per_factor = W * 1026 + 6 * (18 * W * W - 18 * W) + 18 * W + 27 * W
    imu = (W - 1) * (450 * 29 + 900 * 29 + 30 * 29 + 15 * 29 + 29)
    return F * per_factor + imu


def aggregate(dt, steps, world, dev):
    """Whole-job scans/s from per-rank wall times: max over ranks (RCCL on GPU,
    gloo on CPU), every rank processed `steps` scans of its own sequence."""
    if world > 1:
        import torch
        import torch.distributed as dist
        on_cpu = dist.get_backend() == "gloo"  # (the rehearsal)
        tt = torch.tensor([dt], device="cpu" if on_cpu else dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return world * steps / dt, dt


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, p, seq, host_scans):
    """Time the CPU restatement (oracle) on a bounded sample of the same
    sequence: 5 std::threads for the map/BA fan-outs as the reference
    (thread_num, optimizers.cpp:184), IEKF single-threaded, the dead VNC prep
    included (the reference pays it); and the same with one thread. Per scan
    steady_clock; median and p90 over the scans after the warm-up."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: the baseline leg only
    import vgconfig

    oracle.build()
    warm, n = args.cpu_warmup, args.cpu_warmup + args.cpu_scans
    out, traj5 = {}, None
    for threads in (5, 1):
        pl = oracle.Pipeline(vgconfig.to_c(p, use_threads=1 if threads > 1 else 0, vnc_prep=1))
        pl.seed(seq.gt_state(0))
        tms, stages = [], []
        for k in range(n):
            xyz, it, b, e, imu = host_scans[k]
            tm = pl.step(xyz, it, b, e, imu)
            if k >= warm:
                tms.append(tm[6])
                stages.append(tm[:6])
        if threads == 5:
            traj5 = pl.trajectory()
        pl.close()
        tms = np.array(tms)
        st = np.median(np.array(stages), axis=0) * 1e3
        out[threads] = {"value": round(len(tms) / float(np.sum(tms)), 3), "median_ms": round(1e3 * np.median(tms), 2),
                        "p90_ms": round(1e3 * np.percentile(tms, 90), 2),
                        "stage_median_ms": {k: round(float(v), 2) for k, v in zip(
                            ("prep_downsample", "iekf", "insert", "recut", "ba", "margi"), st)}}
    r = out[5]
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return ({"value": r["value"], "unit": "scans/s", "cores": 5, "kind": "port",
             "sample": "%d scans after %d warm-up scans of the same synthetic %s sequence, %s.yaml; IEKF "
                       "single-threaded, map/BA fan-outs on 5 std::threads as the reference, VNC prep included"
                       % (n - warm, warm, args.lidar, args.config),
             "median_ms": r["median_ms"], "p90_ms": r["p90_ms"], "stage_median_ms": r["stage_median_ms"],
             "one_thread": dict(out[1], cores=1), "cpu_model": cpu_model(), "nproc": os.cpu_count(),
             "cpus_available": avail}, traj5)


if __name__ == "__main__":
    main()
