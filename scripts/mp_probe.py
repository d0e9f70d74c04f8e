"""Throughput of B independent sequences on ONE GPU as B processes
(diagnostic): each process runs its own context; every process starts its timed
region at the same wall-clock instant.

    python scripts/mp_probe.py B [lidar] [steps]
"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
sys.path.insert(0, REPO)


def worker(t_start, lidar, steps, seq_id):
    import numpy as np

    import bench
    import synth
    import vgconfig
    p = vgconfig.load("mid360")
    g = p["General"]
    warm = 12
    host = bench.gen_scans(lidar, seq_id, g, warm + steps, 1)
    import torch

    import vgpu
    dev = torch.device("cuda", 0)
    seq = synth.Sequence(lidar, seq_id, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    scans = []
    for xyz, inten, b, e, imu in host:
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, inten[None]], 0))).to(dev)
        scans.append((t, xyz.shape[0], b, e, imu))
    c = vgpu.Context(vgconfig.to_c(p), device=0, max_points=max(s[1] for s in scans) + 16, max_nodes=1_000_000,
                     max_fix_points=3_000_000, hash_log2=20)
    c.seed(seq.gt_state(0))

    def run(k):
        t, n, b, e, imu = scans[k]
        c.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imu)

    for k in range(warm):
        run(k)
    c.stats_log()
    torch.cuda.synchronize(dev)
    while time.time() < t_start:
        time.sleep(0.001)
    t0 = time.time()
    for k in range(warm, warm + steps):
        run(k)
    c.stats_log()
    torch.cuda.synchronize(dev)
    t1 = time.time()
    print(json.dumps({"t0": t0, "t1": t1, "steps": steps}), flush=True)
    c.close()


def main():
    if sys.argv[1] == "worker":
        worker(float(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
        return
    B = int(sys.argv[1])
    lidar = sys.argv[2] if len(sys.argv) > 2 else "64line"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    t_start = time.time() + 25 + 1.5 * B
    procs = [subprocess.Popen([sys.executable, __file__, "worker", str(t_start), lidar, str(steps), str(b)],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL) for b in range(B)]
    res = []
    for pr in procs:
        out, _ = pr.communicate(timeout=300)
        res.append(json.loads(out.decode().strip().splitlines()[-1]))
    t0 = min(r["t0"] for r in res)
    t1 = max(r["t1"] for r in res)
    late = max(r["t0"] for r in res) - t0
    print(json.dumps({"lidar": lidar, "B_processes": B, "scans_per_s": round(B * steps / (t1 - t0), 1),
                      "per_process": [round(steps / (r["t1"] - r["t0"]), 1) for r in res],
                      "start_skew_s": round(late, 3)}), flush=True)


if __name__ == "__main__":
    main()
