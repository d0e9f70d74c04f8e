"""The IEKF's memo of an unmatched point's leaf (k_iekf, an extension: the
reference re-descends from the hash every iteration, odometry.cpp:124-132,
voxel_map.cpp:241-266) must name the leaf the reference's descent reaches.
The descent is strict on centre planes (octant(): w > centre goes up,
octree.cpp:586), OctoTree::inside (octree.cpp:732-737) is inclusive on both
faces. So the memo is tested against the descent's own region (dbox), not the
inclusive box: a point that moves exactly onto an internal node's centre plane
between iterations must leave the upper sibling it was memoised in.

The probe (vgx_memo_probe) takes every internal node of a map built by the
pipeline, puts points exactly on its three centre planes, memoises each with
the leaf of the same point one ulp above / below the plane, and compares the
memo's verdict with a fresh hash + descent (the reference's path)."""
import pytest

import synth
import vgconfig
import vgpu

pytestmark = pytest.mark.gpu


def test_memo_matches_descent_on_centre_planes():
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("64line", 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    ctx = vgpu.Context(vgconfig.to_c(p), max_points=200_000, max_nodes=1_000_000, max_fix_points=4_000_000,
                       hash_log2=20)
    try:
        ctx.seed(seq.gt_state(0))
        for k in range(14):  # past the window fill: recut subdivisions (internal nodes at layers 0-2)
            xyz, it, b, e = seq.scan(k)
            ctx.step(xyz, it, b, e, seq.imu(k))
        samples, bad_inclusive, bad_region, split = ctx.memo_probe()
    finally:
        ctx.close()
    assert samples > 1000 and split > 100, (samples, split)
    assert bad_region == 0, (bad_region, samples)
    # sensitivity: the inclusive box would keep points on the plane in the upper sibling
    assert bad_inclusive > 0, (bad_inclusive, samples)
