"""Multi-sequence mode throughput (vg_multi_*): B contexts stepped together,
one native worker thread each, for a few wait policies.

    python scripts/multi_probe.py [lidar] [spin_us,sleep_us ...] -- B ...
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import vgconfig  # noqa: E402


def main():
    argv = sys.argv[1:]
    lidar = argv.pop(0) if argv and argv[0] != "--" and "," not in argv[0] else "64line"
    pols, Bs = [], []
    cur = pols
    for a in argv:
        if a == "--":
            cur = Bs
            continue
        cur.append(a)
    pols = [tuple(int(v) for v in x.split(",")) for x in pols] or [(0, 0), (20, 20)]
    Bs = [int(b) for b in Bs] or [1, 2, 4, 8, 16]
    p = vgconfig.load("mid360")
    g = p["General"]
    warm, steps = 12, 30
    host = bench.gen_scans(lidar, 0, g, warm + steps, int(os.environ.get("MP_WORKERS", "16")))
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
    for spin, sleep in pols:
        for B in Bs:
            ctxs = [vgpu.Context(vgconfig.to_c(p), device=0, max_points=npmax, max_nodes=1_000_000,
                                 max_fix_points=3_000_000, hash_log2=20) for _ in range(B)]
            for c in ctxs:
                c.seed(seq.gt_state(0))
                for key, env in ((7, "MP_OVERLAP"), (8, "MP_SPEC")):  # vgx_debug knobs, 0 = off
                    if os.environ.get(env) is not None:
                        vgpu.lib().vgx_debug(c.h, key, int(os.environ[env]))
            mv = vgpu.Multi(ctxs, spin, sleep)

            def step(k):
                t, n, b, e, imu = scans[k]
                mv.step_dev([(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), 0, n, b, e, imu)] * B)

            for k in range(warm):
                step(k)
            mv.sync()
            t0 = time.perf_counter()
            for k in range(warm, warm + steps):
                step(k)
            mv.sync()
            dt = time.perf_counter() - t0
            trajs = [c.trajectory() for c in ctxs]
            same = all(np.array_equal(trajs[0], tr) for tr in trajs[1:])
            print(json.dumps({"lidar": lidar, "B": B, "spin_us": spin, "sleep_us": sleep,
                              "scans_per_s": round(B * steps / dt, 1), "ms_per_round": round(dt * 1e3 / steps, 3),
                              "identical": same, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                              "overlap": os.environ.get("MP_OVERLAP", "1"), "spec": os.environ.get("MP_SPEC", "1")}),
                  flush=True)
            mv.close()
            for c in ctxs:
                c.close()


if __name__ == "__main__":
    main()
