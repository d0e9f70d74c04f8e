"""Voxel-key rule and the VOXEL_LOC hash: known answers. CPU only."""
import numpy as np

import oracle


def key_py(x, size):
    """point_utils.hpp:16-23 / voxel_map.cpp:57-65 restated with numpy float32."""
    out = []
    for c in x:
        l = np.float32(np.float64(c) / size)
        if l < 0:
            l = np.float32(l - np.float32(1.0))
        out.append(int(l))  # C++ (int64_t) truncates toward zero
    return out


def test_truncation_not_floor(oracle_lib):
    # exact negative multiple maps one voxel LOWER than floor (-0.5/0.5 = -1 -> -2)
    k = oracle.voxel_keys(np.array([[-0.5, 0.5, -0.25]]), 0.5)[0]
    assert list(k) == [-2, 1, -1]
    assert list(k) == key_py([-0.5, 0.5, -0.25], 0.5)


def test_float_rounding_boundary(oracle_lib):
    # 2.9999999 m / 1.0 rounds to 3.0f -> key 3 although the point lies in voxel 2
    k = oracle.voxel_keys(np.array([[2.99999999, -1e-9, 0.0]]), 1.0)[0]
    assert list(k) == [3, -1, 0]


def test_random_keys_match_python(oracle_lib):
    rng = np.random.default_rng(7)
    P = rng.uniform(-200, 200, size=(3000, 3))
    P[:100] = np.round(P[:100] * 2) / 2  # exact multiples of 0.5
    for size in (0.5, 1.0, 0.1, 0.05):
        k = oracle.voxel_keys(P, size)
        ref = np.array([key_py(p, size) for p in P])
        assert np.array_equal(k, ref)


def test_hash_known_answers(oracle_lib):
    L = oracle.lib()
    M = 2 ** 64
    for (x, y, z) in [(0, 0, 0), (1, 2, 3), (-1, -2, -3), (123456, -98765, 4321)]:
        h = ((((z % M) * 1000033) % M % 100000000000 + (y % M)) % M * 1000033) % M % 100000000000
        h = (h + (x % M)) % M
        assert L.orc_voxel_hash(x, y, z) == h


def test_keys_golden(oracle_lib):
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "voxel_keys.npz"))
    for s in ("0.05", "0.1", "0.5", "1.0"):
        assert np.array_equal(oracle.voxel_keys(d["pts"], float(s)), d["k" + s])
