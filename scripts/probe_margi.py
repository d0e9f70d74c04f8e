"""Per-leaf phase clocks of k_margi_leaf (the margi's leaf pass, on the scan
chain), instrumented build:

    VINA_GPU_LIB=vina-slam_amd/lib_probe/libvina_gpu.so python scripts/probe_margi.py
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

PH = {51: "header, run, own cluster", 52: "frame clusters, merge, eigen", 54: "plane update",
      55: "point_fix carve + stores"}


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
    nl = max(buf[56], 1)
    print("k_margi_leaf: %d live leaves (%d with a factor) over %d scans; longest leaf %.2f us; "
          "longest block %.2f us" % (buf[56], buf[58], nscan - 12, buf[57] / 100.0, buf[45] / 100.0))
    for k, name in PH.items():
        print("  %-32s %8.2f us/leaf" % (name, buf[k] / nl / 100.0))  # 100 MHz wall clock
    ctx.close()


if __name__ == "__main__":
    main()
