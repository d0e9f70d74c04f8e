"""Throughput of B independent sequences on ONE GPU (diagnostic): B contexts,
each driven by its own host thread (ctypes releases the GIL, so the stage calls
run concurrently in C), each with its own HIP streams.

    GPU_MAX_HW_QUEUES=16 python scripts/batch_probe.py [lidar] [B ...]
"""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import vgconfig  # noqa: E402


def main():
    lidar = sys.argv[1] if len(sys.argv) > 1 else "64line"
    Bs = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8, 16]
    p = vgconfig.load("mid360")
    g = p["General"]
    warm, steps = 12, 30
    nseq = max(Bs)
    # one scan set shared by every sequence (the sequences differ only in seed
    # otherwise; the throughput does not depend on it)
    host = bench.gen_scans(lidar, 0, g, warm + steps, 16)
    import torch

    import synth
    import vgpu
    dev = torch.device("cuda", 0)
    seq = synth.Sequence(lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    scans = []
    for xyz, inten, b, e, imu in host:
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e, imu))
    npmax = max(s[1] for s in scans) + 16
    _ = nseq
    for B in Bs:
        use = [vgpu.Context(vgconfig.to_c(p), device=0, max_points=npmax, max_nodes=1_000_000,
                            max_fix_points=3_000_000, hash_log2=20) for _ in range(B)]
        for c in use:
            c.seed(seq.gt_state(0))

        def drive(c, ks, barrier=None):
            if barrier is not None:
                barrier.wait()
            for k in ks:
                t, n, b, e, imu = scans[k]
                c.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imu)

        th = [threading.Thread(target=drive, args=(c, range(warm))) for c in use]
        [x.start() for x in th]
        [x.join() for x in th]
        for c in use:
            c.stats_log()
        torch.cuda.synchronize(dev)
        bar = threading.Barrier(B + 1)
        th = [threading.Thread(target=drive, args=(c, range(warm, warm + steps), bar)) for c in use]
        [x.start() for x in th]
        bar.wait()
        t0 = time.perf_counter()
        [x.join() for x in th]
        for c in use:
            c.stats_log()  # completes every enqueued scan
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        trajs = [c.trajectory() for c in use]
        same = all(np.array_equal(trajs[0], t) for t in trajs[1:])
        print(json.dumps({"lidar": lidar, "B": B, "scans_per_s": round(B * steps / dt, 1),
                          "ms_per_round": round(dt * 1e3 / steps, 3), "identical": same,
                          "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
        for c in use:
            c.close()


if __name__ == "__main__":
    main()
