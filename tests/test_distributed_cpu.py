"""bench.py's multi-process path on CPU: world_size-2 gloo, max-over-ranks
timing and the whole-job aggregate (replica mode, weak scaling)."""
import os
import socket

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dt = 1.0 + rank  # rank 1 is the slow one
    steps = 10
    v, dmax = bench.aggregate(dt, steps, world, torch.device("cpu"))
    q.put((rank, v, dmax))
    dist.destroy_process_group()


def test_two_rank_aggregate():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    for rank, v, dmax in res:
        assert dmax == 2.0
        assert abs(v - 2 * 10 / 2.0) < 1e-12


def _shard_worker(rank, world, port, q, cfgname, nscan):
    import torch
    import torch.distributed as dist
    import oracle
    import synth
    import vgconfig
    tag = rank if world > 1 else "single"
    p = vgconfig.load(cfgname)
    g = p["General"]
    seq = synth.Sequence("16line", 3, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        orc.shard(rank, world, lambda arr: dist.all_reduce(torch.from_numpy(arr)))
    orc.seed(seq.gt_state(0))
    stats = []
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        orc.step(xyz, it, b, e, seq.imu(k))
        stats.append(orc.stats())
    q.put((tag, orc.trajectory(), stats))
    if world > 1:
        dist.destroy_process_group()


def test_tile_sharded_oracle_matches_unsharded():
    """The spatial-tile partition of SURVEY §8(e) on the CPU restatement, two
    gloo ranks: each rank keeps only its tiles' root voxels and the normal
    equations / LM Hessian / residual / quirk counts are all-reduced; every rank
    must reproduce the unsharded trajectory, and the per-rank map counts must
    add up to the unsharded ones (each root voxel lives on exactly one rank)."""
    import numpy as np
    import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nscan = 13
    ps = [ctx.Process(target=_shard_worker, args=(r, 2, port, q, "mid360", nscan)) for r in range(2)]
    for p in ps:
        p.start()
    _shard_worker(0, 1, port, q, "mid360", nscan)
    res = {}
    for _ in range(3):
        tag, tr, st = q.get(timeout=300)
        res[tag] = (tr, st)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    (t1, s1), (ta, sa), (tb, sb) = res["single"], res[0], res[1]
    for k, (a, b, c) in enumerate(zip(sa, sb, s1)):
        assert a["roots_new"] + b["roots_new"] == c["roots_new"], k
        assert a["n_slide"] + b["n_slide"] == c["n_slide"], k
        assert a["n_factors"] + b["n_factors"] == c["n_factors"], k
        assert a["iekf_iters"] == b["iekf_iters"] == c["iekf_iters"], k
        assert a["iekf_matches"] == b["iekf_matches"] == c["iekf_matches"], k
        assert a["ba_iters"] == b["ba_iters"] == c["ba_iters"], k
        assert min(a["roots_new"], b["roots_new"]) > 0 or c["roots_new"] < 4, k  # both ranks hold map
    assert np.array_equal(ta, tb)
    assert synth.ate(t1, ta) < 1e-6
