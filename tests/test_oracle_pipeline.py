"""The oracle's full per-scan loop is deterministic (reproduces the committed
golden trajectory bit for bit), tracks ground truth, and its worker threads do
not change results (the reference partitions never change a value)."""
import os

import numpy as np

import oracle
import synth
import vgconfig

GOLD = os.path.join(os.path.dirname(__file__), "golden", "trajectory_16line_mid360.npz")


def _run(use_threads, n=14, seq_id=2):
    p = vgconfig.load("mid360")
    c = vgconfig.to_c(p, use_threads=use_threads, vnc_prep=0)
    g = p["General"]
    seq = synth.Sequence("16line", seq_id=seq_id, blind=g["blind"], ext_R=g["extrinsic_rota"],
                         ext_t=g["extrinsic_tran"])
    pl = oracle.Pipeline(c)
    pl.seed(seq.gt_state(0))
    for k in range(n):
        xyz, it, b, e = seq.scan(k)
        pl.step(xyz, it, b, e, seq.imu(k))
    return seq, pl


def test_golden_trajectory(oracle_lib):
    seq, pl = _run(0)
    d = np.load(GOLD)
    assert np.array_equal(pl.trajectory(), d["traj"])
    assert np.array_equal(pl.window_states(), d["window"])


def test_threads_do_not_change_results(oracle_lib):
    _, a = _run(0, n=12)
    _, b = _run(1, n=12)
    assert np.array_equal(a.trajectory(), b.trajectory())


def test_tracks_ground_truth(oracle_lib):
    seq, pl = _run(0)
    tr = pl.trajectory()
    gt = np.array([seq.gt_pose(k)[1] for k in range(tr.shape[0])])
    err = np.linalg.norm(tr[:, 10:13] - gt, axis=1)
    assert err.max() < 0.05, err
