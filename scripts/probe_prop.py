"""Phase clocks of k_scan_prop (device IMU propagation), instrumented build:

    VINA_GPU_LIB=vina-slam_amd/lib_probe/libvina_gpu.so python scripts/probe_prop.py
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

PHASES = {1: "arguments -> LDS", 2: "per-pair Exp / F00", 7: "wait for the margi head's flag",
          3: "rotation chain (lane 0)", 4: "F60/F612/noise + cov load", 5: "cov sandwich chain",
          6: "opening (x_prop, flags)"}


def main(nscan=30):
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("64line", 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    ctx = vgpu.Context(vgconfig.to_c(p), device=0)
    ctx.debug(13, 1)
    ctx.seed(seq.gt_state(0))
    L = vgpu.lib()
    buf = (ctypes.c_ulonglong * 64)()
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        ctx.step(xyz, it, b, e, seq.imu(k))
        if k == 11:
            ctx.stats_log()
            L.vg_probe_read_state(buf, 64)  # clear the warm-up
    ctx.stats_log()
    L.vg_probe_read_state(buf, 64)
    calls = max(buf[63], 1)
    khz = ctypes.c_int(0)
    print("k_scan_prop calls:", buf[63])
    for k, name in PHASES.items():
        print("  %-28s %8.2f us/call" % (name, buf[k] / calls / 100.0))  # 100 MHz wall clock
    ctx.close()


if __name__ == "__main__":
    main()
