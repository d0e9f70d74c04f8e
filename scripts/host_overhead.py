"""Host-side overhead per scan: per-step stats() call and the ctypes step call."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vgconfig  # noqa: E402
import vgpu  # noqa: E402


def main():
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("64line", 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    dev = torch.device("cuda", 0)
    scans, imus = [], []
    for k in range(72):
        xyz, it, b, e = seq.scan(k)
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, it[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e))
        imus.append(seq.imu(k))
    for mode in ("stats", "nostats"):
        ctx = vgpu.Context(vgconfig.to_c(p), device=0, max_points=max(s[1] for s in scans) + 16)
        ctx.seed(seq.gt_state(0))
        host = []
        for k in range(72):
            t, n, b, e = scans[k]
            if k == 32:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            a = time.perf_counter()
            ctx.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imus[k])
            if mode == "stats":
                ctx.stats()
            host.append(time.perf_counter() - a)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(mode, "ms/step %.4f" % (dt * 1e3 / 40))
        ctx.close()
    # bare ctypes call cost
    ctx = vgpu.Context(vgconfig.to_c(p), device=0)
    a = time.perf_counter()
    for _ in range(1000):
        ctx.stats()
    print("stats() us %.2f" % ((time.perf_counter() - a) * 1e3))
    ctx.close()


if __name__ == "__main__":
    main()
