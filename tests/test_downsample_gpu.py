"""A1 parity: the HIP downsample (vg_downsample) against the oracle's
down_sampling_voxel (point_utils.hpp:7-44). Bit-exact as a set: keys, float
means, first-point intensity, counts."""
import numpy as np
import pytest

import oracle
import synth
import vgconfig
import vgpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = vgpu.Context(vgconfig.to_c(vgconfig.load("mid360")), max_points=400_000)
    yield c
    c.close()


def _canon(a):
    a = np.asarray(a, dtype=np.float32)
    order = np.lexsort(tuple(a[:, j] for j in range(4, -1, -1)))
    return a[order]


def _check(ctx, xyz, inten, size):
    g = ctx.downsample(xyz, inten, size)
    o = oracle.downsample(xyz, inten, size)
    assert g.shape == o.shape
    # GPU emits ascending key order; compare as sets, bit for bit
    assert np.array_equal(_canon(g).view(np.uint32), _canon(o).view(np.uint32))
    return g


@pytest.mark.parametrize("lidar,size", [("tiny", 0.1), ("64line", 0.1), ("64line", 0.05), ("128line", 0.1)])
def test_downsample_synthetic_bit_exact(ctx, oracle_lib, lidar, size):
    seq = synth.Sequence(lidar, seq_id=3, blind=1.0)
    xyz, inten, _, _ = seq.scan(5)
    g = _check(ctx, xyz, inten, size)
    assert g.shape[0] > 1000


def test_downsample_edge_cases(ctx, oracle_lib):
    rng = np.random.default_rng(5)
    # exact negative multiples, zeros, duplicates, huge clusters in one voxel
    xyz = np.array([[-0.5, -0.5, -0.5], [0, 0, 0], [0, 0, 0], [-0.1, 0.1, -1e-9], [0.1, -0.1, 1e-9]], np.float32)
    _check(ctx, xyz, np.arange(5, dtype=np.float32), 0.1)
    blob = (rng.normal(0, 0.01, (5000, 3)) + 3.05).astype(np.float32)
    g = _check(ctx, blob, np.zeros(5000, np.float32), 0.1)
    assert g[:, 4].sum() == 5000
    one = np.array([[1.0, 2.0, 3.0]], np.float32)
    _check(ctx, one, np.ones(1, np.float32), 0.1)


def test_downsample_empty_and_noop(ctx):
    assert ctx.downsample(np.zeros((0, 3), np.float32), np.zeros(0, np.float32), 0.1).shape[0] == 0
    xyz = np.ones((4, 3), np.float32)
    assert ctx.downsample(xyz, np.zeros(4, np.float32), 0.0005).shape[0] == 4


def test_downsample_range_error(ctx):
    xyz = np.array([[1e6, 0, 0]], np.float32)  # key 1e7 > 2^20: reported, not wrapped
    with pytest.raises(vgpu.VgError):
        ctx.downsample(xyz, np.zeros(1, np.float32), 0.1)


def test_downsample_golden(ctx):
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "downsample_tiny.npz"))
    g = ctx.downsample(d["xyz"], d["inten"], float(d["size"]))
    assert np.array_equal(_canon(g).view(np.uint32), _canon(d["out"]).view(np.uint32))


def _first_occurrence_order(xyz, size):
    """The hashed path's documented output order: voxels by their first point index."""
    loc = (np.asarray(xyz, np.float32).astype(np.float64) / size).astype(np.float32)
    loc = np.where(loc < 0, (loc.astype(np.float64) - 1.0).astype(np.float32), loc)
    keys = [tuple(k) for k in loc.astype(np.int64)]
    seen, order = set(), []
    for k in keys:
        if k not in seen:
            seen.add(k)
            order.append(k)
    return order


@pytest.mark.parametrize("case", ["scan", "dense", "giant", "ring_wrap"])
def test_hashed_downsample_bit_exact(ctx, oracle_lib, case):
    """The per-scan pipeline's hashed downsample (ds_enqueue_hashed: no sort,
    the voxel count on the device) = the oracle's down_sampling_voxel bit for
    bit as a set, emitted in first-occurrence order — including dense voxels
    (> 32 points: the workgroup bitmap path) with index ranges wider than one
    bitmap window."""
    rng = np.random.default_rng(7)
    size = 0.1
    if case == "scan":
        seq = synth.Sequence("64line", seq_id=3, blind=1.0)
        xyz, inten, _, _ = seq.scan(5)
    elif case == "dense":  # many voxels of 40-400 points
        c = rng.uniform(-5, 5, (300, 3))
        xyz = (c[rng.integers(0, 300, 60_000)] + rng.normal(0, 0.01, (60_000, 3))).astype(np.float32)
        inten = rng.uniform(0, 100, 60_000).astype(np.float32)
    elif case == "giant":  # one voxel holding 50 k points
        xyz = (rng.normal(0, 0.005, (50_000, 3)) + 3.05).astype(np.float32)
        inten = np.arange(50_000, dtype=np.float32)
    else:  # one voxel's points at both ends of a 300 k-point sweep (index range > one bitmap window)
        bg = rng.uniform(-50, 50, (300_000, 3)).astype(np.float32)
        bg[:100] = (rng.normal(0, 0.005, (100, 3)) + 7.05).astype(np.float32)
        bg[-100:] = (rng.normal(0, 0.005, (100, 3)) + 7.05).astype(np.float32)
        xyz, inten = bg, rng.uniform(0, 1, 300_000).astype(np.float32)
    g = ctx.downsample_hashed(xyz, inten, size)
    o = oracle.downsample(xyz, inten, size)
    assert g.shape == o.shape
    assert np.array_equal(_canon(g).view(np.uint32), _canon(o).view(np.uint32))
    if case != "scan":
        order = _first_occurrence_order(xyz, size)
        loc = (g[:, :3].astype(np.float64) / size).astype(np.float32)
        got = [tuple(k) for k in np.where(loc < 0, (loc.astype(np.float64) - 1.0).astype(np.float32),
                                          loc).astype(np.int64)]
        assert got == order


@pytest.mark.parametrize("case,size,halves", [("scan", 0.1, False), ("dense", 1.0, True), ("giant", 0.5, True),
                                              ("clusters", 0.5, True), ("1m", 2.0, True)])
def test_fallback_pass_matches_oracle(oracle_lib, case, size, halves):
    """down_sampling_voxel's /2 fallback below 2000 voxels (local_mapping.cpp:
    399-403) on the device: one workgroup redoes the pass at size / 2 when the
    first kept fewer than 2000 voxels (k_hds_fallback), bit for bit the oracle's
    set and the first-occurrence order; otherwise the first pass stands."""
    import oracle
    import vgpu
    rng = np.random.default_rng(9)
    p = vgconfig.load("mid360")
    ctx = vgpu.Context(vgconfig.to_c(p), max_points=1_100_000 if case == "1m" else 400_000, max_nodes=100_000,
                       max_fix_points=100_000, hash_log2=16)
    if case == "1m":  # a 1M-ray scan at 2 m: ~400 voxels, then ~1.5 k dense ones at 1 m (k_hds_big behind the pass)
        xyz, inten, _, _ = synth.Sequence("1M", seq_id=2, blind=3.0).scan(4)
    elif case == "scan":
        g_ = p["General"]
        seq = synth.Sequence("64line", 1, blind=g_["blind"], ext_R=g_["extrinsic_rota"], ext_t=g_["extrinsic_tran"])
        xyz, inten, _, _ = seq.scan(3)
    elif case == "dense":  # ~300 voxels at 1 m, dense ones (> 16 points) at 0.5 m
        c = rng.uniform(-5, 5, (300, 3))
        xyz = (c[rng.integers(0, 300, 60_000)] + rng.normal(0, 0.01, (60_000, 3))).astype(np.float32)
        inten = rng.uniform(0, 100, 60_000).astype(np.float32)
    elif case == "giant":  # one voxel of 50 k points, ~1 at 0.25 m too
        xyz = (rng.normal(0, 0.005, (50_000, 3)) + 3.05).astype(np.float32)
        inten = np.arange(50_000, dtype=np.float32)
    else:  # 1200 clusters at 0.5 m voxel centres: < 2000 voxels at 0.5 m, many more at 0.25 m (step 2 over
        # 30 tiles of 1024 points)
        c = (np.floor(rng.uniform(-40, 40, (1200, 3)) / 0.5) + 0.5) * 0.5
        xyz = (c[rng.integers(0, 1200, 30_000)] + rng.normal(0, 0.04, (30_000, 3))).astype(np.float32)
        inten = rng.uniform(0, 1, 30_000).astype(np.float32)
    first = oracle.downsample(xyz, inten, size)
    assert (first.shape[0] < 2000) == halves
    used = size / 2 if halves else size
    g = ctx.downsample_hashed(xyz, inten, size, fallback=True)
    o = oracle.downsample(xyz, inten, used)
    assert g.shape == o.shape
    assert np.array_equal(_canon(g).view(np.uint32), _canon(o).view(np.uint32))
    order = _first_occurrence_order(xyz, used)
    loc = (g[:, :3].astype(np.float64) / used).astype(np.float32)
    got = [tuple(k) for k in np.where(loc < 0, (loc.astype(np.float64) - 1.0).astype(np.float32),
                                      loc).astype(np.int64)]
    assert got == order
    ctx.close()


def test_hashed_downsample_1m_scan(oracle_lib):
    """BASELINE config 5's scan (synthetic 1M rays, ~750 k points after the
    blind filter): at 0.1 m about 13 k voxels hold 17-200 points (the
    wave-per-voxel path, k_hds_mid) — bit for bit the oracle's set."""
    seq = synth.Sequence("1M", seq_id=2, blind=3.0)
    xyz, inten, _, _ = seq.scan(4)
    c = vgpu.Context(vgconfig.to_c(vgconfig.load("mid360")), max_points=xyz.shape[0] + 16, max_nodes=100_000,
                     max_fix_points=100_000, hash_log2=16)
    try:
        g = c.downsample_hashed(xyz, inten, 0.1)
    finally:
        c.close()
    o = oracle.downsample(xyz, inten, 0.1)
    assert g.shape == o.shape and g.shape[0] > 50_000
    assert (o[:, 4] > 16).sum() > 5000
    assert np.array_equal(_canon(g).view(np.uint32), _canon(o).view(np.uint32))
