"""Phase clocks of the IEKF iteration (k_iekf point loop + k_iekf_update),
instrumented build:

    VINA_GPU_LIB=vina-slam_amd/lib_probe/libvina_gpu.so python scripts/probe_iekf.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VINA_GPU_LIB", os.path.join(REPO, "vina-slam_amd", "lib_probe", "libvina_gpu.so"))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))

import synth  # noqa: E402
import vgconfig  # noqa: E402
import vgpu  # noqa: E402

UPD = {23: "ordered sum of the block partials", 24: "iteration bookkeeping", 25: "6x6 wave solve (K6)",
       26: "G6, x_prop - x_curr, sol", 27: "x_curr update + convergence", 28: "covariance update (final)",
       29: "trajectory / done (final)"}
PTS = {30: "point loop (block 0)", 31: "block reduction (block 0)"}


def main(nscan=30):
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("64line", 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    ctx = vgpu.Context(vgconfig.to_c(p), device=0)
    ctx.seed(seq.gt_state(0))
    L = vgpu.lib()
    buf = (ctypes.c_ulonglong * 64)()
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        ctx.step(xyz, it, b, e, seq.imu(k))
        if k == 11:
            ctx.stats_log()
            L.vg_probe_read_map(buf, 64)  # clear the warm-up
    ctx.stats_log()
    L.vg_probe_read_map(buf, 64)
    calls, fin, kcalls = max(buf[61], 1), max(buf[60], 1), max(buf[59], 1)
    print("k_iekf_update calls: %d (finishing %d); k_iekf calls: %d" % (buf[61], buf[60], buf[59]))
    for k, name in UPD.items():
        n = fin if k >= 28 else calls
        print("  %-36s %8.2f us/call" % (name, buf[k] / n / 100.0))  # 100 MHz wall clock
    for k, name in PTS.items():
        print("  %-36s %8.2f us/call" % (name, buf[k] / kcalls / 100.0))
    ctx.close()


if __name__ == "__main__":
    main()
