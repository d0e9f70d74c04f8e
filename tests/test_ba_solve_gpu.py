"""k_ba_solve (the LM step's LDL^T solve, optimizers.cpp:466) on given
symmetric systems against numpy's LU solve (vgx_ba_solve: the kernel as an LM
iteration launches it, identity pivot order).

Systems: D (M M^T + lam I) D with D a diagonal scaling over six decades (the
spread of a real LM system's rotation / position / velocity / bias unknowns),
and a symmetric indefinite, diagonally dominant one (the LiDAR Hessian of an
eigenvalue cost is not positive definite in general). Sizes: 15W - 15 for
W = 2 (one 16 x 16 tile, 15 real rows), 3, 5, 10 (the bench window) and 11
(the largest the LDS tile store holds).

Tolerance: relative to the solution's norm in the scaled unknowns D x, 1e-10
(LDL^T without pivoting is invariant under the symmetric scaling, so both
solvers see the conditioning of M M^T + lam I, ~1e2-1e3 here; observed
~1e-14)."""
import numpy as np
import pytest

import vgconfig
import vgpu

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _ctx(win):
    p = vgconfig.load("mid360")
    p["LocalBA"]["win_size"] = win
    return vgpu.Context(vgconfig.to_c(p), max_points=20_000, max_nodes=100_000, max_fix_points=200_000,
                        hash_log2=16)


def _spd(m, rng):
    M = rng.standard_normal((m, m))
    A = M @ M.T + m * np.eye(m)
    d = 10.0 ** rng.uniform(-2, 4, m)
    return d, (A * d[:, None]) * d[None, :]


def _indef(m, rng):
    M = rng.standard_normal((m, m))
    A = 0.5 * (M + M.T)
    A[np.diag_indices(m)] = rng.choice([-1.0, 1.0], m) * (4 * m + rng.uniform(0, m, m))
    d = 10.0 ** rng.uniform(-1, 3, m)
    return d, (A * d[:, None]) * d[None, :]


@pytest.mark.parametrize("win", [2, 3, 5, 10, 11])
@pytest.mark.parametrize("kind", ["spd", "indefinite"])
def test_ba_solve_matches_numpy(win, kind):
    m = 15 * win - 15
    rng = np.random.default_rng(1000 * win + (kind == "spd"))
    ctx = _ctx(win)
    try:
        for _ in range(3):
            d, A = (_spd if kind == "spd" else _indef)(m, rng)
            b = rng.standard_normal(m) * d
            x = ctx.ba_solve(A, b)
            ref = np.linalg.solve(A, b)
            err = np.abs(d * (x - ref)).max() / np.abs(d * ref).max()
            assert np.all(np.isfinite(x)) and err < TOL, (win, kind, err)
    finally:
        ctx.close()
