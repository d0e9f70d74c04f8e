"""The LM's first Hessian pass, entry by entry: the device's k_ba_hess /
k_ba_hfinal output (the 6W x 6W LiDAR Hessian from the MFMA X^T S X tiles and
the per-frame diagonal blocks, gradient, residual) and the IMU factor blocks
against the oracle's divide_thread pass (LidarFactor::acc_evaluate2 summed over
the factors, factors.cpp:22-126; IMU_PRE::give_evaluate,
imu_preintegration.cpp:97-163) at the same window state. W = 10 (mid360) and
W = 11 (the largest window the LDS-resident solve holds: 15W <= 176).

Tolerances, relative to the block's largest entry: Hessian blocks 1e-11
(observed <= 3e-13); gradients and residuals 1e-9 (observed <= 4e-11: they are
sums of nearly cancelling terms — J^T C r with a small r — so the summation
order, chunk partials vs thread partitions, shows more)."""
import numpy as np
import pytest

import oracle
import synth
import vgconfig
import vgpu

pytestmark = pytest.mark.gpu
REL_H = 1e-11
REL_G = 1e-9


def _blocks(v, W):
    L = 6 * W
    H = v[: L * L].reshape(L, L)
    g = v[L * L: L * L + L]
    r = v[L * L + L]
    imu = v[L * L + L + 1:].reshape(W - 1, 931)
    return H, g, r, imu


def _rel(a, b):
    s = max(np.abs(a).max(), np.abs(b).max(), 1e-300)
    return float(np.abs(a - b).max() / s)


@pytest.mark.parametrize("win", [10, 11])
def test_first_hessian_pass_matches_oracle(oracle_lib, win):
    p = vgconfig.load("mid360")
    p["LocalBA"]["win_size"] = win
    g = p["General"]
    seq = synth.Sequence("16line", 5, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    gpu = vgpu.Context(vgconfig.to_c(p), max_points=100_000, max_nodes=500_000, max_fix_points=2_000_000,
                       hash_log2=20)
    s0 = seq.gt_state(0)
    orc.seed(s0)
    gpu.seed(s0)
    checked = 0
    for k in range(win + 4):
        capture = k in (win - 1, win + 3)  # the first LM run (window just full) and a later one
        if capture:
            orc.capture_arm()
            gpu.capture_arm()
        xyz, it, b, e = seq.scan(k)
        imu = seq.imu(k)
        orc.step(xyz, it, b, e, imu)
        gpu.step(xyz, it, b, e, imu)
        so, sg = orc.stats(), gpu.stats()
        assert (so["n_factors"], so["ba_iters"]) == (sg["n_factors"], sg["ba_iters"]), k
        if not capture:
            continue
        vo, vg = orc.capture_get(), gpu.capture_get()
        L = 6 * win
        assert vo.size == vg.size == L * L + L + 1 + (win - 1) * 931
        Ho, go, ro, io = _blocks(vo, win)
        Hg, gg, rg, ig = _blocks(vg, win)
        assert np.abs(Ho).max() > 0 and so["n_factors"] > 0
        errs = {"H": _rel(Ho, Hg), "g": _rel(go, gg), "r": abs(ro - rg) / abs(ro)}
        for q in range(win - 1):
            errs["imu%d_jtj" % q] = _rel(io[q, :900], ig[q, :900])
            errs["imu%d_gg" % q] = _rel(io[q, 900:930], ig[q, 900:930])
            errs["imu%d_r" % q] = abs(io[q, 930] - ig[q, 930]) / max(abs(io[q, 930]), 1e-300)
        print("scan", k, "factors", sg["n_factors"], {a: "%.1e" % v for a, v in errs.items() if v > 1e-15})
        assert max(v for a, v in errs.items() if a == "H" or a.endswith("jtj")) < REL_H, errs
        assert max(errs.values()) < REL_G, errs
        # the Hessian is symmetric and its off-diagonal frame blocks are populated (MFMA tiles)
        assert np.abs(Hg[6:12, 0:6]).max() > 0
        checked += 1
    assert checked == 2
    gpu.close()
    orc.close()
