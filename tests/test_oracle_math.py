"""Pin the oracle's dependency-free linear algebra (stand-ins for Eigen) with
numpy/scipy known answers. CPU only."""
import numpy as np
import pytest

import oracle


def _sym(rng, n, scale=1.0):
    A = rng.normal(size=(n, n)) * scale
    return 0.5 * (A + A.T)


def test_eig3_matches_numpy(oracle_lib):
    rng = np.random.default_rng(1)
    for k in range(200):
        A = _sym(rng, 3, 10.0 ** rng.uniform(-4, 2))
        if k % 3 == 0:  # plane-like covariance: one tiny eigenvalue (octree.cpp:362)
            U, _ = np.linalg.qr(rng.normal(size=(3, 3)))
            A = U @ np.diag([1e-6, 0.04, 0.2]) @ U.T
        w, V = oracle.eig3(A)
        wn = np.linalg.eigvalsh(A)
        assert np.all(np.diff(w) >= 0), "ascending order (SelfAdjointEigenSolver)"
        assert np.allclose(w, wn, rtol=0, atol=1e-13 * max(1.0, np.abs(wn).max()))
        assert np.allclose(A @ V, V * w, atol=1e-12 * max(1.0, np.abs(wn).max()))
        assert np.allclose(V.T @ V, np.eye(3), atol=1e-13)


def test_inverse15_matches_numpy(oracle_lib):
    rng = np.random.default_rng(2)
    for _ in range(20):
        M = rng.normal(size=(15, 15))
        A = M @ M.T + 1e-3 * np.eye(15)
        assert np.allclose(oracle.inverse15(A), np.linalg.inv(A), rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("n", [15, 60, 150])
def test_ldlt_matches_numpy(oracle_lib, n):
    rng = np.random.default_rng(n)
    M = rng.normal(size=(n, n))
    A = M @ M.T + 1e-2 * np.eye(n)
    A[:15, :] = 0
    A[:, :15] = 0
    A[:15, :15] = np.eye(15)  # the LM gauge block, optimizers.cpp:460-462
    b = rng.normal(size=n)
    x = oracle.ldlt_solve(A, b)
    assert np.allclose(x, np.linalg.solve(A, b), rtol=1e-8, atol=1e-10)


def test_so3_identities(oracle_lib):
    import ctypes
    L = oracle.lib()
    rng = np.random.default_rng(3)
    for _ in range(50):
        w = rng.normal(size=3)
        w = w / np.linalg.norm(w) * rng.uniform(1e-6, 3.0)
        R, lg, J, Ji = (np.zeros(9), np.zeros(3), np.zeros(9), np.zeros(9))
        L.orc_so3(oracle._d(w), oracle._d(R), oracle._d(lg), oracle._d(J), oracle._d(Ji))
        R = R.reshape(3, 3)
        assert np.allclose(R.T @ R, np.eye(3), atol=1e-13)
        assert np.allclose(lg, w, atol=1e-9)  # Log(Exp(w)) = w for |w| < pi
        # jr_inv(Exp(w)) is the inverse of jr(w) (math.hpp:57-88)
        assert np.allclose(Ji.reshape(3, 3) @ J.reshape(3, 3), np.eye(3), atol=1e-9)
