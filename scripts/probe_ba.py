"""Phase clocks of the probed kernels (instrumented build, `make -C vina-slam_amd probe`).

    VINA_GPU_LIB=vina-slam_amd/lib_probe/libvina_gpu.so python scripts/probe_ba.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VINA_GPU_LIB", os.path.join(REPO, "vina-slam_amd", "lib_probe", "libvina_gpu.so"))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
import numpy as np  # noqa: E402

import synth  # noqa: E402
import vgconfig  # noqa: E402
import vgpu  # noqa: E402

PHASES = {3: "load || inv(0)", 10: "wave0: L, tile, y", 11: "wave0: inv(K+1)", 6: "barrier wait",
          5: "w(NB-1)", 7: "backward solve", 8: "trial/q1"}
EXTRA = {12: "(slowest trailing wave's jobs, summed over phases)"}


def main(nscan=40, lidar="64line"):
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence(lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    ctx = vgpu.Context(vgconfig.to_c(p), device=0)
    ctx.seed(seq.gt_state(0))
    L = vgpu.lib()
    buf = (ctypes.c_ulonglong * 64)()
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        ctx.step(xyz, it, b, e, seq.imu(k))
        if k == 11:
            L.vg_probe_read(buf, 64)  # clear the warm-up
            L.vg_probe_read_map(buf, 64)
    L.vg_probe_read(buf, 64)
    calls = max(buf[63], 1)
    print("k_ba_solve real calls:", buf[63])
    tot = 0.0
    for k, name in PHASES.items():
        us = buf[k] * 0.01 / calls
        tot += us
        print("  %-16s %8.2f us/call" % (name, us))
    print("  %-16s %8.2f us/call" % ("total", tot))
    for k, name in EXTRA.items():
        print("  %8.2f us/call %s" % (buf[k] * 0.01 / calls, name))
    L.vg_probe_read_map(buf, 64)
    na = max(buf[62], 1)
    print("k_rc_apply calls:", buf[62])
    for k, name in {16: "sort subs+events", 17: "child alloc", 18: "keys", 19: "bitonic", 20: "push", 21: "finish"}.items():
        print("  %-16s %8.2f us/call" % (name, buf[k] * 0.01 / na))
    ctx.close()




def iekf(nscan=40, lidar="64line"):
    """Phase clocks of the IEKF update run by the last k_iekf workgroup."""
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence(lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    ctx = vgpu.Context(vgconfig.to_c(p), device=0)
    ctx.seed(seq.gt_state(0))
    L = vgpu.lib()
    buf = (ctypes.c_ulonglong * 64)()
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        ctx.step(xyz, it, b, e, seq.imu(k))
        ctx.stats()
        if k == 11:
            L.vg_probe_read_map(buf, 64)
    L.vg_probe_read_map(buf, 64)
    n, nf = max(buf[61], 1), max(buf[60], 1)
    print("iekf updates:", buf[61], "final:", buf[60])
    for k, name in {24: "reduce partials", 25: "K6 (6x6 solve)", 26: "G6/vec/sol", 27: "plus/conv"}.items():
        print("  %-16s %8.2f us/call" % (name, buf[k] * 0.01 / n))
    for k, name in {28: "cov update", 29: "eig3/final"}.items():
        print("  %-16s %8.2f us/final" % (name, buf[k] * 0.01 / nf))
    ni = max(buf[59], 1)
    print("k_iekf block 0, thread 0:", buf[59], "launches")
    for k, name in {30: "point loop", 31: "block reduction"}.items():
        print("  %-16s %8.2f us/launch" % (name, buf[k] * 0.01 / ni))
    nb = max(buf[47], 1)
    print("k_margi_leaf: %d working blocks, leaves (max) %d" % (buf[47], buf[50]))
    print("  %-16s %8.2f us" % ("mean block span", buf[46] * 0.01 / nb))
    print("  %-16s %8.2f us" % ("max block span", buf[45] * 0.01))


if __name__ == "__main__":
    iekf() if "iekf" in sys.argv else main()
