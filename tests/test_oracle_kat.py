"""Independent pins of the oracle's restatement: the
reference ships no tests or fixtures, so the restated Jacobians, gradients and
Hessians are checked against central finite differences of the restated
residuals, and the IEKF against a known pose. CPU only (test infrastructure).

* p2p Jacobian (odometry.cpp:136-142) vs FD of r = n.(R Exp(d) pnt + p + dp - c);
* LidarFactor (factors.cpp:22-158): JacT vs FD of lambda_min over the
  right-perturbed window poses; the analytic Hessian vs the symmetrised FD of
  JacT (the FD of a manifold gradient is asymmetric by -1/2 hat(g) on the
  rotation blocks, which the reference's `- 0.5 hat(jjt)` term accounts for);
* IMU_PRE::give_evaluate (imu_preintegration.cpp:97-163): [joca | jocb] vs FD
  of the 15-residual over both states' boxplus increments (the first state's
  bias increments also move the preintegration's dbg / dba, as update_state,
  imu_preintegration.cpp:239-246, does);
* IEKF known-pose recovery: a pose error injected after the window is full is
  pulled back to ground truth by one LioStateEstimation (odometry.cpp:64-255).
"""
import numpy as np
from scipy.spatial.transform import Rotation as Rot

import oracle
import synth
import vgconfig


def expm(w):
    return Rot.from_rotvec(w).as_matrix()


def test_p2p_jacobian_fd(oracle_lib):
    rng = np.random.default_rng(7)
    for _ in range(20):
        R = expm(rng.normal(0, 1, 3))
        p = rng.normal(0, 5, 3)
        pnt = rng.normal(0, 10, 3)
        n = rng.normal(0, 1, 3)
        n /= np.linalg.norm(n)
        c = R @ pnt + p + rng.normal(0, 0.05, 3)
        r0, j = oracle.kat_p2p(R, p, pnt, n, c)
        assert abs(r0 - n @ (R @ pnt + p - c)) < 1e-12
        h = 1e-6
        jfd = np.zeros(6)
        for k in range(6):
            e = np.zeros(3)
            e[k % 3] = h
            if k < 3:
                a = oracle.kat_p2p(R @ expm(e), p, pnt, n, c)[0]
                b = oracle.kat_p2p(R @ expm(-e), p, pnt, n, c)[0]
            else:
                a = oracle.kat_p2p(R, p + e, pnt, n, c)[0]
                b = oracle.kat_p2p(R, p - e, pnt, n, c)[0]
            jfd[k] = (a - b) / (2 * h)
        assert np.abs(j - jfd).max() < 1e-6 * max(1.0, np.abs(j).max()), (j, jfd)


def _plane_voxel(rng, W):
    """W frames observing one noisy plane (local clusters), a fixed cluster,
    and slightly perturbed window poses."""
    n = np.array([-0.3, 0.1, 1.0])

    def pts(k):
        xy = rng.uniform(-1, 1, (k, 2))
        return np.c_[xy, 0.3 * xy[:, 0] - 0.1 * xy[:, 1] + 2] + rng.normal(0, 0.01, (k, 3))

    clus, poses = [], []
    for i in range(W):
        R, p = expm(rng.normal(0, 0.3, 3)), rng.normal(0, 1, 3)
        pl = (pts(25 + 3 * i) - p) @ R  # R^T (pw - p)
        clus.append(np.r_[(pl.T @ pl).ravel(), pl.sum(0), len(pl)])
        poses.append((R @ expm(rng.normal(0, 0.01, 3)), p + rng.normal(0, 0.01, 3)))
    fp = pts(20)
    fix = np.r_[(fp.T @ fp).ravel(), fp.sum(0), len(fp)]
    _ = n
    return np.array(clus), fix, poses


def _pack(ps):
    return np.array([np.r_[R.ravel(), p] for R, p in ps])


def _boxplus(ps, i, k, s):
    q = list(ps)
    R, p = q[i]
    e = np.zeros(3)
    e[k % 3] = s
    q[i] = (R @ expm(e), p) if k < 3 else (R, p + e)
    return q


def test_lidar_factor_gradient_hessian_fd(oracle_lib):
    rng = np.random.default_rng(3)
    for W in (3, 10):
        clus, fix, ps = _plane_voxel(rng, W)
        lam, J, H = oracle.kat_lidar_factor(clus, fix, _pack(ps))
        assert lam > 0 and np.abs(H - H.T).max() < 1e-12 * np.abs(H).max()
        jfd = np.zeros(6 * W)
        hfd = np.zeros((6 * W, 6 * W))
        for i in range(W):
            for k in range(6):
                a = oracle.kat_lidar_factor(clus, fix, _pack(_boxplus(ps, i, k, 1e-6)), False)
                b = oracle.kat_lidar_factor(clus, fix, _pack(_boxplus(ps, i, k, -1e-6)), False)
                jfd[6 * i + k] = (a[0] - b[0]) / 2e-6
                a = oracle.kat_lidar_factor(clus, fix, _pack(_boxplus(ps, i, k, 1e-5)), False)
                b = oracle.kat_lidar_factor(clus, fix, _pack(_boxplus(ps, i, k, -1e-5)), False)
                hfd[:, 6 * i + k] = (a[1] - b[1]) / 2e-5
        assert np.abs(J - jfd).max() < 1e-6 * np.abs(J).max(), np.abs(J - jfd).max()
        hs = 0.5 * (hfd + hfd.T)
        assert np.abs(H - hs).max() < 1e-7 * np.abs(H).max(), np.abs(H - hs).max()


def test_imu_factor_jacobian_fd(oracle_lib):
    seq = synth.Sequence("tiny", 0)
    rng = np.random.default_rng(0)
    noise = [0.01, 2.0, 1e-4, 1e-4]
    for k in (2, 5):
        imu = seq.imu(k + 1)

        def st(s):
            x = np.zeros(24)
            x[:9], x[9:12], x[12:15] = s[1:10], s[10:13], s[13:16]
            x[15:18] = rng.normal(0, 1e-3, 3)
            x[18:21] = rng.normal(0, 1e-2, 3)
            x[21:24] = s[22:25]
            return x

        x1, x2 = st(seq.gt_state(k)), st(seq.gt_state(k + 1))
        b0 = np.r_[x1[15:18], x1[18:21]]
        db = rng.normal(0, 1e-3, 6)
        cost, rr, J = oracle.kat_imu(imu, b0, db, x1, x2, noise)
        assert cost > 0 and np.abs(rr).max() < 0.1

        def plus(x, kk, s):
            y = x.copy()
            if kk < 3:
                e = np.zeros(3)
                e[kk] = s
                y[:9] = (x[:9].reshape(3, 3) @ expm(e)).ravel()
            else:
                y[9 + kk - 3] += s
            return y

        h = 1e-6
        jfd = np.zeros((15, 30))
        for f in range(2):
            for kk in range(15):
                def ev(s):
                    a = plus(x1, kk, s) if f == 0 else x1
                    b = plus(x2, kk, s) if f == 1 else x2
                    d = db.copy()
                    if f == 0 and kk >= 9:
                        d[kk - 9] += s
                    return oracle.kat_imu(imu, b0, d, a, b, noise)[1]
                jfd[:, 15 * f + kk] = (ev(h) - ev(-h)) / (2 * h)
        # 1e-5: the reference's Log (acos of (tr - 1) / 2) resolves a ~1e-3 rad
        # residual to ~1e-7 under a 1e-6 step
        assert np.abs(J - jfd).max() < 1e-5 * np.abs(J).max(), np.abs(J - jfd).max()


def test_iekf_recovers_known_pose(oracle_lib):
    """After the window is full, x_curr is knocked off ground truth by 4 cm /
    0.4 deg; the next scan's IEKF (odometry.cpp:64-255) pulls the pose back to
    ground truth (the synthetic scans are rendered from it)."""
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("16line", seq_id=6, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    pl = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    pl.seed(seq.gt_state(0))
    K = 13
    for k in range(K):
        xyz, it, b, e = seq.scan(k)
        pl.step(xyz, it, b, e, seq.imu(k))
    s = pl.state()
    s[1:10] = (s[1:10].reshape(3, 3) @ expm(np.deg2rad([0.4, -0.3, 0.2]))).ravel()
    s[10:13] += [0.04, -0.03, 0.02]
    pl.seed(s)
    xyz, it, b, e = seq.scan(K)
    pl.step(xyz, it, b, e, seq.imu(K))
    st = pl.stats()
    assert st["iekf_matches"][0] > 1000
    tr = pl.trajectory()
    Rg, pg = seq.gt_pose(K)
    perr = np.linalg.norm(tr[K, 10:13] - pg)
    rerr = np.linalg.norm(Rot.from_matrix(Rg.T @ tr[K, 1:10].reshape(3, 3)).as_rotvec())
    assert perr < 0.01 and np.rad2deg(rerr) < 0.1, (perr, np.rad2deg(rerr), st)
