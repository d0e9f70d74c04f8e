"""GPU-vs-oracle pipeline parity probe over the BASELINE configs (diagnostic, not a test):
per config, the first scan where any integer counter differs and the max pose difference.

    python scripts/parity_probe.py [cfg:lidar:nscan ...] > gpurun_out/parity.jsonl
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (test infrastructure: the checker)
import synth  # noqa: E402
import vgconfig  # noqa: E402
import vgpu  # noqa: E402

KEYS = ("n_raw", "n_ds", "iekf_iters", "iekf_matches", "roots_new", "n_slide", "n_factors", "ba_iters")
DEFAULT = ["mid360:64line:30", "robosense:128line:12", "HILTI:64line:15", "mid360:128line:12", "mid360:1M:4"]


def probe(cfgname, lidar, nscan):
    p = vgconfig.load(cfgname)
    g = p["General"]
    seq = synth.Sequence(lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    gpu = vgpu.Context(vgconfig.to_c(p), max_points=1_100_000, max_nodes=2_000_000, max_fix_points=8_000_000,
                       hash_log2=22)
    s0 = seq.gt_state(0)
    orc.seed(s0)
    gpu.seed(s0)
    first_diff, rows = None, []
    t_o = t_g = 0.0
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        imu = seq.imu(k)
        t0 = time.perf_counter()
        orc.step(xyz, it, b, e, imu)
        t1 = time.perf_counter()
        gpu.step(xyz, it, b, e, imu)
        sg = gpu.stats()
        t2 = time.perf_counter()
        t_o += t1 - t0
        t_g += t2 - t1
        so = orc.stats()
        d = [key for key in KEYS if so[key] != sg[key]]
        if d and first_diff is None:
            first_diff = {"scan": k, "keys": d, "oracle": {x: so[x] for x in d}, "gpu": {x: sg[x] for x in d}}
        rows.append({x: sg[x] for x in KEYS})
    to, tg = orc.trajectory(), gpu.trajectory()
    dp = np.linalg.norm(to[:, 10:13] - tg[:, 10:13], axis=1)
    dR = np.abs(to[:, 1:10] - tg[:, 1:10]).max(axis=1)
    out = {"config": cfgname, "lidar": lidar, "nscan": nscan, "first_diff": first_diff, "ate": synth.ate(to, tg),
           "max_dpos": float(dp.max()), "max_dR": float(dR.max()), "dpos": [float("%.3e" % x) for x in dp],
           "oracle_s": round(t_o, 2), "gpu_s": round(t_g, 2), "counters": rows}
    gpu.close()
    orc.close()
    return out


def main():
    specs = sys.argv[1:] or DEFAULT
    for s in specs:
        c, l, n = s.split(":")
        print(json.dumps(probe(c, l, int(n))), flush=True)


if __name__ == "__main__":
    main()
