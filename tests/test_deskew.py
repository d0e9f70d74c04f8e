"""SURVEY row f1 — IMUEKF::motion_blur's per-point deskew (imu_ekf.cpp:114-144).

CPU: the oracle's restatement moves every raw point (fired at its own time,
expressed in the LiDAR frame of that instant) into the LiDAR frame at the scan
end; with the state propagated from the true pose by the (noisy) IMU, the
deskewed points must land where the true sensor motion puts them.
GPU (marked): the device deskew inside the pipeline reproduces the oracle's
pipeline on the same raw scans (integer counters exact, trajectory)."""
import numpy as np
import pytest

import synth
import vgconfig


def _world(seq, t, pts):
    R, p = seq.traj.rot(t), seq.traj.pos(t)
    return (pts @ seq.ext_R.T + seq.ext_t) @ R.T + p


def test_oracle_deskew_recovers_sensor_motion(oracle_lib):
    import oracle
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("tiny", 7, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    k = 5
    s0 = seq.gt_state(k - 1)
    # a first step only sets the scan-end time (no propagation on the first scan)
    xyz, it, b, e = seq.scan(k - 1)
    orc2 = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    orc2.seed(s0)
    orc2.step(xyz, it, b, e, seq.imu(k - 1))
    raw, inten, times, beg, end = seq.scan_raw(k)
    assert np.all(np.diff(times) >= 0)
    out, npose = orc2.deskew_only(raw, times, beg, end, seq.imu(k))
    assert npose > 10
    # true world position of every raw point vs where the deskewed point says it is
    ts = beg + times.astype(np.float64)
    w_true = np.stack([_world(seq, t, q[None])[0] for t, q in zip(ts[::37], raw[::37].astype(np.float64))])
    w_desk = _world(seq, end, out[::37].astype(np.float64))
    w_none = _world(seq, end, raw[::37].astype(np.float64))
    err = np.linalg.norm(w_true - w_desk, axis=1)
    err0 = np.linalg.norm(w_true - w_none, axis=1)
    print("deskew error median %.4f max %.4f m; uncompensated median %.4f m" % (np.median(err), err.max(),
                                                                                 np.median(err0)))
    assert np.median(err0) > 0.05          # the sweep really moves
    assert np.median(err) < 0.005
    assert err.max() < 0.03
    assert np.array_equal(out[times <= 0], raw[times <= 0])


@pytest.mark.gpu
@pytest.mark.parametrize("cfgname", ["mid360", "HILTI"])
def test_pipeline_deskew_matches_oracle(oracle_lib, cfgname):
    import oracle
    import vgpu
    p = vgconfig.load(cfgname)
    g = p["General"]
    seq = synth.Sequence("16line", 8, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    gpu = vgpu.Context(vgconfig.to_c(p), max_points=120_000, max_nodes=600_000, max_fix_points=2_000_000,
                       hash_log2=20)
    s0 = seq.gt_state(0)
    orc.seed(s0)
    gpu.seed(s0)
    so, sg = [], []
    for k in range(14):
        raw, inten, times, beg, end = seq.scan_raw(k)
        imu = seq.imu(k)
        orc.step_deskew(raw, inten, times, beg, end, imu)
        gpu.step_deskew(raw, inten, times, beg, end, imu)
        so.append(orc.stats())
    sg = gpu.stats_log()
    for k, (a, b) in enumerate(zip(so, sg)):
        assert a["n_ds"] == b["n_ds"], (k, a, b)
        assert a["roots_new"] == b["roots_new"], (k, a, b)
        assert a["n_slide"] == b["n_slide"], (k, a, b)
    err = synth.ate(orc.trajectory(), gpu.trajectory())
    print("ATE gpu vs oracle (deskewed raw scans): %.3e m" % err)
    assert err < 0.01
