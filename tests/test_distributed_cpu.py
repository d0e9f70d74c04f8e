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
