"""B sequences stepped together in ONE process (vg_multi_*), for PMC passes
that compare B = 4 and B = 8 (the multi-sequence regression past B = 4):

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d <dir> -o run -- python3 scripts/multi_pmc.py 4
    python3 scripts/multi_pmc_summary.py <dir4> <dir8> ...

Scans are generated in-process (no fork under the profiler); the rate is
printed as one JSON line.
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
    B = int(sys.argv[1])
    lidar = sys.argv[2] if len(sys.argv) > 2 else "64line"  # argv[3]: vg_multi_set_active cap (0: none)
    p = vgconfig.load("mid360")
    g = p["General"]
    warm, steps = 12, 16
    host = [bench.gen_scans(lidar, b, g, warm + steps, 1) for b in range(B)]
    import torch

    import synth
    import vgpu
    dev = torch.device("cuda", 0)
    seq = synth.Sequence(lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    data = []
    for hs in host:
        sc = []
        for xyz, inten, b, e, imu in hs:
            t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
            sc.append((t, xyz.shape[0], b, e, imu))
        data.append(sc)
    npmax = max(s[1] for sc in data for s in sc) + 16
    ctxs = [vgpu.Context(vgconfig.to_c(p), device=0, max_points=npmax) for _ in range(B)]
    for c in ctxs:
        c.seed(seq.gt_state(0))
    mv = vgpu.Multi(ctxs, 0, 0)
    cap = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if cap:
        mv.set_active(cap)  # at most `cap` sequences on the device at once

    def step(k):
        mv.step_dev([(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), 0, n, b, e, imu)
                     for (t, n, b, e, imu) in (d[k] for d in data)])

    for k in range(warm):
        step(k)
    mv.sync()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        step(k)
    mv.sync()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    print(json.dumps({"B": B, "active_cap": cap, "scans_per_s": round(B * steps / dt, 1)}), flush=True)
    mv.close()
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
