"""Micro-benchmark of the A1 downsample kernel chain on device-resident scans."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
import numpy as np  # noqa: E402
import synth  # noqa: E402
import vgconfig  # noqa: E402
import vgpu  # noqa: E402

lidar = sys.argv[1] if len(sys.argv) > 1 else "64line"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ctx = vgpu.Context(vgconfig.to_c(vgconfig.load("mid360")))
seq = synth.Sequence(lidar, seq_id=0, blind=3.0)
xyz, inten, _, _ = seq.scan(3)
for i in range(5):
    out = ctx.downsample(xyz, inten, 0.1)
t = time.time()
for i in range(reps):
    out = ctx.downsample(xyz, inten, 0.1)
dt = (time.time() - t) / reps
print("n_raw", xyz.shape[0], "n_ds", out.shape[0], "host-inclusive ms/call %.3f" % (dt * 1e3))
