"""The map's lifetime: the idle branch's journey release
(local_mapping.cpp:317-344: roots whose jour stamp is >= 700 m behind are
erased with their subtrees, octree.cpp:597-608) and the device's reclaim of
erased nodes and abandoned point_fix blocks (vg_release_far, lifetime.hip).

* release vs the oracle's restatement (oracle/pipeline.cpp release_far) on the
  same sequence, the release distance as a config key (release_dis) so that it
  fires within a few hundred scans of the synthetic box: every release's
  erased roots / nodes and the census after it agree exactly, and so do the
  per-scan counters and poses of the scans that follow (they match against the
  map that is left);
* compaction is invisible: a context compacted every few scans steps exactly
  (bit for bit) as one that never is — node ids keep their order;
* a long run at a small node / point_fix capacity that ends in VG_E_CAPACITY
  without the release completes with it.
"""
import numpy as np
import pytest

import oracle
import synth
import vgconfig
import vgpu
from test_pipeline_gpu import COUNTERS, TIGHT_M, check_pair

pytestmark = pytest.mark.gpu


def _pair(release_dis, seq_id, max_nodes, max_fix, cfgname="mid360", lidar="16line"):
    p = vgconfig.load(cfgname)
    g = p["General"]
    seq = synth.Sequence(lidar, seq_id, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0, release_dis=release_dis))
    gpu = vgpu.Context(vgconfig.to_c(p, release_dis=release_dis), max_points=100_000, max_nodes=max_nodes,
                       max_fix_points=max_fix, hash_log2=18)
    orc.seed(seq.gt_state(0))
    gpu.seed(seq.gt_state(0))
    return seq, orc, gpu


def check_scan(k, a, b):
    """Every integer counter of scan k, at that scan (the first divergence is named)."""
    for key in COUNTERS:
        assert a[key] == b[key], (k, key, a[key], b[key])


def check_roots(k, ro, rg):
    """The oracle's surf_map against the device map, root by root (vgx_roots /
    orc_roots): the same root keys, each with the same slide membership,
    isexist, subtree node count and point_fix points, and its jour stamp
    within the pose tolerance."""
    assert ro.keys() == rg.keys(), (k, sorted(set(ro) ^ set(rg))[:8])
    bad = [(key, ro[key], rg[key]) for key in ro
           if ro[key][1:] != rg[key][1:] or abs(ro[key][0] - rg[key][0]) > TIGHT_M]
    assert not bad, (k, len(bad), bad[:8])


def test_release_matches_oracle(oracle_lib):
    """release_dis = 4 m on the 16-line box sequence (~1.3 m of jour per 10
    scans): the release fires every tenth scan from ~scan 40 on and erases
    roots; both sides agree on every release and on every scan after it, and
    the two maps agree root by root after every scan."""
    seq, orc, gpu = _pair(4, 7, 400_000, 2_000_000)
    so, sg, rel = [], [], []
    fired = 0
    for k in range(160):
        xyz, it, b, e = seq.scan(k)
        imu = seq.imu(k)
        orc.step(xyz, it, b, e, imu)
        gpu.step(xyz, it, b, e, imu)
        so.append(orc.stats())
        sg.append(gpu.stats())
        check_scan(k, so[-1], sg[-1])
        check_roots(k, orc.roots(), gpu.roots())
        ro, rg = orc.release_far(), gpu.release_far()
        rel.append((k, ro, rg))
        assert ro[0] == rg[0], (k, ro, rg)  # roots erased (-1: none pending)
        assert ro[2] == rg[2], (k, ro, rg)  # roots left
        fired += ro[0] > 0
    for k, ro, rg in rel:
        if ro[0] >= 0:
            print("scan %d: oracle %s device %s" % (k, ro, rg))
    assert fired >= 3
    assert orc.jour() > 4 * 3 and np.abs(orc.path()[:, 13] - gpu.path()[:, 13]).max() < 1e-9
    check_pair(so, sg, orc.trajectory(), gpu.trajectory(), orc.window_states(), gpu.window_states())
    # the tree shapes and point_fix contents agree as well
    for k, ro, rg in rel:
        assert ro[1] == rg[1] and ro[3] == rg[3] and ro[4] == rg[4], (k, ro, rg)
    gpu.close()
    orc.close()


def test_compaction_is_invisible(oracle_lib):
    """Two contexts on one sequence, no release (release_dis 1e6): B compacts
    its pool and arena every 7 scans (flags bit 0). Trajectory, window states
    and per-scan counters bit-identical; B's pool and arena shrink."""
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("16line", 3, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    A = vgpu.Context(vgconfig.to_c(p, release_dis=1_000_000), max_points=100_000, max_nodes=400_000,
                     max_fix_points=2_000_000, hash_log2=18)
    B = vgpu.Context(vgconfig.to_c(p, release_dis=1_000_000), max_points=100_000, max_nodes=400_000,
                     max_fix_points=2_000_000, hash_log2=18)
    A.seed(seq.gt_state(0))
    B.seed(seq.gt_state(0))
    shrink = []
    for k in range(60):
        xyz, it, b, e = seq.scan(k)
        A.step(xyz, it, b, e, seq.imu(k))
        B.step(xyz, it, b, e, seq.imu(k))
        if k % 7 == 6:
            sa, r = A.stats(), B.release_far(compact=True)
            assert r[0] in (-1, 0)
            shrink.append((sa["nodes_used"], r[3], sa["fix_used"], r[5], r[4]))
    la, lb = A.stats_log(), B.stats_log()
    for k, (a, b) in enumerate(zip(la, lb)):
        for key in COUNTERS:
            assert a[key] == b[key], (k, key)
    assert np.array_equal(A.trajectory(), B.trajectory())
    assert np.array_equal(A.window_states(), B.window_states())
    assert np.array_equal(A.path(), B.path())
    print("nodes / compacted, point_fix used / compacted, held:", shrink)
    assert all(n1 <= n0 and f1 <= f0 for n0, n1, f0, f1, _ in shrink)
    assert any(f1 < f0 for _, _, f0, f1, _ in shrink)  # abandoned point_fix blocks were reclaimed
    A.close()
    B.close()


def _det_run(seq, n, release_dis):
    """One lone context over n scans with vg_release_far after every scan:
    the per-scan record (counters, release output, a digest of the whole root
    map with the jour stamps bit for bit)."""
    p = vgconfig.load("mid360")
    gpu = vgpu.Context(vgconfig.to_c(p, release_dis=release_dis), max_points=100_000, max_nodes=400_000,
                       max_fix_points=8_000_000, hash_log2=18)
    gpu.seed(seq.gt_state(0))
    rec = []
    for k in range(n):
        xyz, it, b, e = seq.scan(k)
        gpu.step(xyz, it, b, e, seq.imu(k))
        roots = gpu.roots()
        digest = hash(tuple(sorted((key, np.float64(v[0]).tobytes(), v[1:]) for key, v in roots.items())))
        rec.append((gpu.stats(), gpu.release_far(), digest))
    out = (rec, gpu.trajectory(), gpu.window_states(), gpu.path())
    gpu.close()
    return out


def test_release_runs_are_bit_identical():
    """Run-to-run determinism of the device path with the release (VERDICT r05
    #1: a release count differed on one box only): two lone contexts, one
    after the other, step the same 240 scans with vg_release_far after every
    scan. Every scan's counters, release output and root map (keys, jour
    stamps bit for bit, slide / isexist flags, subtree counts), and the final
    trajectory, window and path are identical."""
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("16line", 5, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    a = _det_run(seq, 240, 3)
    b = _det_run(seq, 240, 3)
    for k, (ra, rb) in enumerate(zip(a[0], b[0])):
        assert ra[0] == rb[0], (k, "counters", ra[0], rb[0])
        assert ra[1] == rb[1], (k, "release", ra[1], rb[1])
        assert ra[2] == rb[2], (k, "root map")
    for x, y in zip(a[1:], b[1:]):
        assert np.array_equal(x, y)
    assert sum(r[1][0] > 0 for r in a[0]) >= 10  # the release fired


def _gpu_run(seq, release_dis, n, max_nodes, max_fix, release):
    p = vgconfig.load("mid360")
    gpu = vgpu.Context(vgconfig.to_c(p, release_dis=release_dis), max_points=100_000, max_nodes=max_nodes,
                       max_fix_points=max_fix, hash_log2=18)
    gpu.seed(seq.gt_state(0))
    peak, err = [0, 0], None
    try:
        for k in range(n):
            xyz, it, b, e = seq.scan(k)
            gpu.step(xyz, it, b, e, seq.imu(k))
            s = gpu.stats()
            peak = [max(peak[0], s["nodes_used"]), max(peak[1], s["fix_used"])]
            if release:
                gpu.release_far()
    except vgpu.VgError as ex:
        err = (k, str(ex))
    out = (peak, err, None if err else gpu.trajectory())
    gpu.close()
    return out


def test_small_capacity_completes_with_release(oracle_lib):
    """The long box run (240 scans) with vg_release_far after every scan
    (release_dis 3 m) against the oracle doing the same releases: counters
    exact, poses tight. Then with the point_fix arena between the peak with
    the release and the peak without it: without the release the run ends in
    VG_E_CAPACITY (point_fix arena full); with it, it completes with the same
    trajectory, bit for bit."""
    N, RD, NODES, BIG = 240, 3, 400_000, 8_000_000
    seq, orc, gpu = _pair(RD, 5, NODES, BIG)
    so, sg = [], []
    for k in range(N):
        xyz, it, b, e = seq.scan(k)
        imu = seq.imu(k)
        orc.step(xyz, it, b, e, imu)
        gpu.step(xyz, it, b, e, imu)
        so.append(orc.stats())
        sg.append(gpu.stats())
        check_scan(k, so[-1], sg[-1])
        ro_map = orc.roots()
        check_roots(k, ro_map, gpu.roots())
        ro, rg = orc.release_far(), gpu.release_far()
        if ro[0] != rg[0] or ro[2] != rg[2]:  # name the roots the two sides treat differently
            jour = orc.jour()
            near = sorted((jour - v[0], key, v) for key, v in ro_map.items() if not v[1] & 1)
            print("jour %.17g; roots nearest the threshold:" % jour,
                  [x for x in near if abs(x[0] - RD) < 0.05][:8])
        assert ro[0] == rg[0] and ro[2] == rg[2], (k, ro, rg)
    check_pair(so, sg, orc.trajectory(), gpu.trajectory(), orc.window_states(), gpu.window_states())
    ref = gpu.trajectory()
    gpu.close()
    orc.close()
    peak_all, err, _ = _gpu_run(seq, RD, N, NODES, BIG, False)
    peak_rel, err2, _ = _gpu_run(seq, RD, N, NODES, BIG, True)
    assert err is None and err2 is None, (err, err2)
    print("peak nodes / point_fix: without the release %s, with it %s" % (peak_all, peak_rel))
    assert peak_all[1] > 1.3 * peak_rel[1]
    cap = (peak_all[1] + peak_rel[1]) // 2
    _, err, _ = _gpu_run(seq, RD, N, NODES, cap, False)
    assert err is not None and "(-3)" in err[1], err
    _, err2, tr = _gpu_run(seq, RD, N, NODES, cap, True)
    assert err2 is None, err2
    print("max_fix_points %d: without the release VG_E_CAPACITY at scan %d (%s); with it all %d scans"
          % (cap, err[0], err[1], N))
    assert np.array_equal(tr, ref)
