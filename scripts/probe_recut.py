"""Phase clocks of the fused recut level kernel (k_rc_level, workgroup 0),
instrumented build:

    VINA_GPU_LIB=vina-slam_amd/lib_probe/libvina_gpu.so python scripts/probe_recut.py
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

PH = {1: "sort of the subdividing leaves", 2: "child counts + prefix", 3: "push loop (wave 0)",
      4: "visit tail (wave 0)"}


def main(nscan=40):
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
    for lev, pb in ((0, 0), (1, 8), (2, 32)):
        n = max(buf[pb], 1)
        print("level %d: %d calls, nsub %.1f, children %.1f, other nodes %.1f" %
              (lev, buf[pb], buf[pb + 5] / n, buf[pb + 6] / n, buf[pb + 7] / n))
        for k, name in PH.items():
            print("  %-32s %8.2f us/call" % (name, buf[pb + k] / n / 100.0))  # 100 MHz wall clock
    n = max(buf[40], 1)
    print("pushes by workgroup 0 wave 0: %d, events %.1f/push" % (buf[40], buf[41] / n))
    for k, name in ((42, "prologue (fix count, runs, s_pre)"), (43, "batch loads + records"), (44, "serial sums")):
        print("  %-32s %8.2f us/push" % (name, buf[k] / n / 100.0))
    print("children by workgroup 0 wave 0 (all levels): %d, of which subdividing %d" % (buf[40], buf[53]))
    for k, name in ((48, "parent lookup + child init"), (49, "push"), (51, "visit + append"),
                    (52, "window split (rc_win_leaf)")):
        print("  %-32s %8.2f us/child" % (name, buf[k] / n / 100.0))
    n = max(buf[18], 1)
    print("window splits (rc_win_leaf, every wave): %d, %.1f us each, longest %.2f us; points %.1f each, "
          "most %d" % (buf[18], buf[17] / n / 100.0, buf[16] / 100.0, buf[20] / n, buf[19]))
    ctx.close()


if __name__ == "__main__":
    main()
