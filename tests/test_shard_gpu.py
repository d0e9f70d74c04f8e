"""Spatial-tile sharding of one sequence (include/vina_gpu.h vg_shard_*), two
ranks on the one GPU of the test box with the host-callback transport over
torch.distributed gloo (RCCL needs one GPU per rank; the bench's tile mode uses
RCCL). Every rank must produce the unsharded trajectory (the state is
replicated; only the fp summation order of the all-reduced sums differs), and
the per-rank map counts must add up to the unsharded ones (each root voxel
lives on exactly one rank)."""
import os
import socket

import numpy as np
import pytest

import synth
import vgconfig
import vgpu

pytestmark = pytest.mark.gpu
CAP = {"16line": dict(max_points=120_000, max_nodes=600_000, max_fix_points=2_000_000, hash_log2=20),
       "128line": dict(max_points=220_000, max_nodes=1_500_000, max_fix_points=6_000_000, hash_log2=21)}
TIGHT_M = 1e-9  # per-scan position bound, sharded vs unsharded (observed ~3e-15 m)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cfgname, lidar, nscan, rank, world, q, port):
    import torch
    import torch.distributed as dist
    tag = rank if world > 1 else "single"
    try:
        p = vgconfig.load(cfgname)
        g = p["General"]
        seq = synth.Sequence(lidar, 2, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
        ctx = vgpu.Context(vgconfig.to_c(p), **CAP[lidar])
        if world > 1:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            dist.init_process_group("gloo", rank=rank, world_size=world)

            log = os.environ.get("VG_AR_LOG")
            seqn = [0]

            def allreduce(arr):
                pre = hash(arr.tobytes()) if log else 0
                dist.all_reduce(torch.from_numpy(arr))
                if log:  # debugging aid: every exchange of this rank, in order (input / result digests)
                    with open("%s.%d" % (log, rank), "a") as f:
                        f.write("%d %d %s %x %x\n" % (seqn[0], arr.size, arr.dtype, pre & 0xffffffff,
                                                     hash(arr.tobytes()) & 0xffffffff))
                seqn[0] += 1

            ctx.shard_host(rank, world, allreduce)
        ctx.seed(seq.gt_state(0))
        for k in range(nscan):
            xyz, it, b, e = seq.scan(k)
            ctx.step(xyz, it, b, e, seq.imu(k))
        q.put((tag, ctx.trajectory(), ctx.stats_log()))
        ctx.close()
        if world > 1:
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((tag, "error", traceback.format_exc()))


# (config, lidar, scans): the 16-line cases cover the LM (mid360) and the dense
# map (HILTI); robosense 128-line is BASELINE configs[3]'s tile-sharded workload
@pytest.mark.parametrize("cfgname,lidar,nscan", [("mid360", "16line", 16), ("HILTI", "16line", 16),
                                                 ("robosense", "128line", 14)])
def test_two_shards_match_one(cfgname, lidar, nscan):
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _port()
    procs = [ctxm.Process(target=_run, args=(cfgname, lidar, nscan, r, 2, q, port)) for r in range(2)]
    for pr in procs:
        pr.start()
    _run(cfgname, lidar, nscan, 0, 1, q, port)  # the unsharded run, in this process
    res = {}
    for _ in range(3):
        tag, tr, st = q.get(timeout=300)
        assert not isinstance(tr, str), st
        res[tag] = (tr, st)
    for pr in procs:
        pr.join(timeout=60)
    (t1, s1), (ta, sa), (tb, sb) = res["single"], res[0], res[1]
    assert len(s1) == len(sa) == len(sb) == nscan
    for k, (a, b, c) in enumerate(zip(sa, sb, s1)):
        print(k, "roots", a["roots_new"], b["roots_new"], c["roots_new"], "slide", a["n_slide"], b["n_slide"],
              c["n_slide"], "factors", a["n_factors"], b["n_factors"], c["n_factors"])
        assert a["roots_new"] + b["roots_new"] == c["roots_new"], k
        assert a["n_slide"] + b["n_slide"] == c["n_slide"], k
        assert a["n_factors"] + b["n_factors"] == c["n_factors"], k
        assert a["iekf_iters"] == b["iekf_iters"] == c["iekf_iters"], k
        assert a["ba_iters"] == b["ba_iters"] == c["ba_iters"], k
        # the match count is part of the all-reduced normal equations: global on every rank
        assert a["iekf_matches"] == b["iekf_matches"] == c["iekf_matches"], k
    # per-rank work: each rank's IEKF transforms and matches only the points of
    # its tiles plus a 0.1 m band, not the whole scan (map.hip k_keep_*). The
    # synthetic box's floor lies on the z = 0 tile face, so its points (a third
    # of the scan, +-2 cm of range noise) are near-boundary for both ranks:
    # observed 0.82 + 0.55 (mid360, 8 m tiles) and 0.64 + 0.57 (1 m voxels,
    # 16 m tiles) of the unsharded count
    for k, (a, b, c) in enumerate(zip(sa, sb, s1)):
        print(k, "IEKF points per iteration / n_raw: %.3f %.3f (iterations %d)"
              % (a["iekf_points"] / a["iekf_iters"] / c["n_raw"], b["iekf_points"] / b["iekf_iters"] / c["n_raw"],
                 c["iekf_iters"]))
    pa, pb, pc = (sum(s["iekf_points"] for s in x) for x in (sa, sb, s1))
    print("IEKF points over %d scans: rank 0 %d (%.2f), rank 1 %d (%.2f), unsharded %d"
          % (nscan, pa, pa / pc, pb, pb / pc, pc))
    assert pc == sum(s["n_raw"] * s["iekf_iters"] for s in s1)
    assert pa < 0.9 * pc and pb < 0.9 * pc and pa + pb < 1.45 * pc
    assert np.array_equal(ta, tb), "the ranks' trajectories must agree bit for bit"
    err = synth.ate(t1, ta)
    dpos = np.linalg.norm(t1[:, 10:13] - ta[:, 10:13], axis=1).max()
    drot = np.abs(t1[:, 1:10] - ta[:, 1:10]).max()
    print("ATE sharded vs unsharded: %.3e m, max dpos %.3e m, max dR %.3e" % (err, dpos, drot))
    assert dpos < TIGHT_M and drot < TIGHT_M


def _run_desync(rank, world, q, port):
    """Rank 1's exchange counter is advanced by one before the first scan: its
    exchanges carry another guard value than rank 0's (shard.hip), so both
    ranks must get VG_E_STATE ("out of step") at their first exchange instead
    of pairing different exchanges."""
    import torch
    import torch.distributed as dist
    try:
        p = vgconfig.load("mid360")
        g = p["General"]
        seq = synth.Sequence("16line", 2, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
        ctx = vgpu.Context(vgconfig.to_c(p), **CAP["16line"])
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ctx.shard_host(rank, world, lambda arr: dist.all_reduce(torch.from_numpy(arr)))
        if rank == 1:
            ctx.debug(12, 1)
        ctx.seed(seq.gt_state(0))
        msg = "no error"
        for k in range(4):
            xyz, it, b, e = seq.scan(k)
            try:
                ctx.step(xyz, it, b, e, seq.imu(k))
                ctx.stats_log()
            except vgpu.VgError as ex:
                msg = "scan %d: %s" % (k, ex)
                break
        q.put((rank, msg))
        ctx.close()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "exception: " + traceback.format_exc()))


def test_desynchronised_rank_gets_an_error():
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _port()
    procs = [ctxm.Process(target=_run_desync, args=(r, 2, q, port)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for pr in procs:
        pr.join(timeout=60)
    for r in (0, 1):
        assert "out of step" in res[r] and "(-5)" in res[r], res[r]


def test_one_rank_rccl_sharded_path_matches_unsharded():
    """The sharded code path on one GPU (vgx_debug 30: a one-rank RCCL
    communicator, the bench's `tile_path_1gpu` leg): every exchange point runs
    ncclAllReduce in its guarded frame, the scans take the sharded launches;
    every counter equals the unsharded run's and the trajectory is within the
    sharded tolerance (the sharded sums are ordered per shard)."""
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("16line", 2, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    out = []
    for force in (False, True):
        ctx = vgpu.Context(vgconfig.to_c(p), **CAP["16line"])
        if force:
            ctx.debug(30, 1)
            ctx.shard_rccl(0, 1, vgpu.rccl_unique_id())
        ctx.seed(seq.gt_state(0))
        for k in range(16):
            xyz, it, b, e = seq.scan(k)
            ctx.step(xyz, it, b, e, seq.imu(k))
        out.append((ctx.trajectory(), ctx.stats_log()))
        ctx.close()
    (t0, s0), (t1, s1) = out
    keys = ("n_raw", "n_ds", "iekf_iters", "iekf_matches", "roots_new", "n_slide", "n_factors", "ba_iters",
            "plane_updates", "fix_full")
    for k, (a, b) in enumerate(zip(s0, s1)):
        for key in keys:
            assert a[key] == b[key], (k, key, a[key], b[key])
    assert np.abs(t0[:, 10:13] - t1[:, 10:13]).max() < TIGHT_M and np.abs(t0[:, 1:10] - t1[:, 1:10]).max() < TIGHT_M
