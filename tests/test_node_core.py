"""SURVEY §8 rows f3/f4 — the ROS-free node core (include/vina_node_core.hpp)
and its event-log replay (vina-slam_amd/examples/vg_node_replay.cpp).

CPU: the TUM row of save_pose_tum (io.cpp:67-77: t, p, Eigen::Quaterniond(R)
as x y z w, std::fixed with 9 decimals) from the header's quat_from_R /
tum_line, against scipy's rotation-to-quaternion on both of Eigen's branches
(trace > 0, and the largest-diagonal one near 180 degrees).

GPU (marked): a synthetic 16-line sequence recorded as the node would receive
it — Livox CustomMsg records (offset_time ns, x, y, z, reflectivity) and IMU
samples in arrival order — runs through NodeCore (vg_decode_scan at arrival,
sync_packages, vg_step_deskew per package); its TUM file must equal the CPU
restatement driven by the same events (oracle decode + the Python statement of
sync_packages + the oracle's deskewing step): every row, same count, poses to
1e-9 m. Parity is against the oracle restatement (the reference cannot be built
here)."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIVOX = np.dtype([("t", "<u4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("tag", "u1"),
                  ("line", "u1"), ("pad", "u1")])

_QUAT_SRC = r"""
#include <cstdio>
#include "vina_node_core.hpp"
int main() {
  double R[9], t, p[3];
  while (scanf("%lf %lf %lf %lf", &t, p, p + 1, p + 2) == 4) {
    for (int i = 0; i < 9; i++) if (scanf("%lf", R + i) != 1) return 1;
    vina_gpu::PoseStamped s;
    s.t = t;
    for (int i = 0; i < 9; i++) s.R[i] = R[i];
    for (int i = 0; i < 3; i++) s.p[i] = p[i];
    vina_gpu::quat_from_R(s.R, s.q);
    fputs(vina_gpu::tum_line(s).c_str(), stdout);
  }
  return 0;
}
"""


def test_tum_rows_match_eigen_quaternion(tmp_path):
    from scipy.spatial.transform import Rotation
    src = tmp_path / "q.cpp"
    src.write_text(_QUAT_SRC)
    exe = tmp_path / "q"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    rng = np.random.default_rng(3)
    rots = list(Rotation.random(40, random_state=5))
    for ax in np.eye(3):  # near 180 degrees: Eigen's largest-diagonal branches
        rots.append(Rotation.from_rotvec(ax * (np.pi - 1e-3)))
    lines, want = [], []
    for k, r in enumerate(rots):
        R = r.as_matrix()
        t, p = 1700000000.0 + 0.1 * k, rng.normal(size=3) * 10
        lines.append(" ".join("%.17g" % v for v in [t, *p, *R.ravel()]))
        q = r.as_quat()  # x y z w
        want.append((t, p, q))
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    rows = out.stdout.strip().splitlines()
    assert len(rows) == len(want)
    for row, (t, p, q) in zip(rows, want):
        f = row.split(" ")
        assert len(f) == 8 and all(len(x.split(".")[1]) == 9 for x in f)
        assert float(f[0]) == float("%.9f" % t)
        assert np.allclose([float(x) for x in f[1:4]], p, atol=1e-9)
        got = np.array([float(x) for x in f[4:]])
        assert np.allclose(got, q, atol=2e-9) or np.allclose(got, -q, atol=2e-9)
        assert abs(np.linalg.norm(got) - 1) < 1e-8


def _fmt(blind):
    return dict(kind=0, stride=LIVOX.itemsize, off_x=LIVOX.fields["x"][1], off_y=LIVOX.fields["y"][1],
                off_z=LIVOX.fields["z"][1], off_intensity=LIVOX.fields["r"][1], off_time=LIVOX.fields["t"][1],
                point_filter_num=1, blind=blind, omega_l=3610.0, time_base=0.0)


def _events(seq, nscan):
    """(kind, payload) in arrival order: IMU samples at their stamps, scan k's
    message at the end of its sweep (after the samples stamped <= then)."""
    imu = {}
    for k in range(nscan + 2):
        for row in seq.imu(k):
            imu[int(round(row[0] * 1e9))] = row
    ev = [(r[0], 0, ("imu", r)) for r in imu.values()]
    for k in range(nscan):
        raw, inten, times, beg, end = seq.scan_raw(k)
        a = np.zeros(raw.shape[0], LIVOX)
        a["x"], a["y"], a["z"] = raw[:, 0], raw[:, 1], raw[:, 2]
        a["r"] = np.clip(inten, 0, 255).astype(np.uint8)
        a["t"] = np.round(times.astype(np.float64) * 1e9).astype(np.uint32)
        ev.append((end, 1, ("scan", beg, a)))
    ev.sort(key=lambda e: (e[0], e[1]))
    return [e[2] for e in ev]


def _write_log(path, cfg, fmt, seed, events):
    import struct

    import vgpu
    with open(path, "wb") as f:
        f.write(b"VGEVENT1")
        f.write(bytes(cfg))
        f.write(bytes(vgpu.LidarFormat(**fmt)))
        f.write(struct.pack("<ii", 0, 1))
        f.write(np.ascontiguousarray(seed, dtype="<f8").tobytes())
        for e in events:
            if e[0] == "imu":
                f.write(struct.pack("<i", 0) + np.ascontiguousarray(e[1], dtype="<f8").tobytes())
            else:
                f.write(struct.pack("<idii", 1, e[1], e[2].size, LIVOX.itemsize) + e[2].tobytes())
        f.write(struct.pack("<i", -1))


def _oracle_tum(p, fmt, seed, events, extra=None):
    """The same events through the CPU restatement: decode at arrival, the
    Python statement of sync_packages (tests/test_decode.py), one deskewing
    step per package."""
    import oracle
    import vgconfig
    from test_decode import _ref_sync
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    orc.seed(seed)
    dec, sync_ev = {}, []
    for e in events:
        if e[0] == "imu":
            sync_ev.append(("imu", np.asarray(e[1])))
        else:
            sid = len(dec)
            d = oracle.decode_scan(e[2].tobytes(), fmt)
            dec[sid] = d
            sync_ev.append(("scan", sid, e[1], float(d[-1, 4]) if len(d) else 0.0))
    pk = _ref_sync(sync_ev, 0)
    for sid, beg, end, imu in pk:
        d = dec[sid]
        orc.step_deskew(d[:, :3].copy(), d[:, 3].copy(), d[:, 4].copy(), beg, end, imu)
    if extra is not None:
        extra.update(path=orc.path(), cmap=orc.local_map(), cmap_all=orc.local_map(all_points=True))
    return orc.trajectory(), len(pk)


@pytest.mark.gpu
def test_node_core_event_log_matches_oracle(oracle_lib, tmp_path):
    import synth
    import vgconfig
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("16line", 12, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    events = _events(seq, 16)
    fmt = _fmt(g["blind"])
    seed = seq.gt_state(0)
    log, tum = tmp_path / "ev.bin", tmp_path / "out.tum"
    pth, cmap = tmp_path / "path.txt", tmp_path / "cmap.bin"
    _write_log(log, vgconfig.to_c(p), fmt, seed, events)
    exe = os.path.join(REPO, "vina-slam_amd", "bin", "vg_node_replay")
    r = subprocess.run([exe, str(log), str(tum), "0", str(pth), str(cmap)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    print(r.stdout.strip())
    rows = np.array([[float(x) for x in ln.split()] for ln in tum.read_text().splitlines()])
    extra = {}
    ref, npk = _oracle_tum(p, fmt, seed, events, extra)
    assert npk >= 14 and rows.shape == (ref.shape[0], 8), (rows.shape, ref.shape, npk)
    assert np.array_equal(rows[:, 0], [float("%.9f" % t) for t in ref[:, 0]])
    err = np.linalg.norm(rows[:, 1:4] - ref[:, 10:13], axis=1)
    print("node core vs oracle: max position difference %.3e m over %d poses" % (err.max(), len(err)))
    assert err.max() < 1e-8  # TUM rows carry 9 decimals
    import json
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["stepped"] == npk and summary["last_scan_world_points"] > 1000
    check_path_and_cmap(np.loadtxt(pth), np.fromfile(cmap, dtype=np.float32).reshape(-1, 4), extra, 1e-8)


def check_path_and_cmap(path, cmap, ref, tol):
    """pub_localmap's outputs against the oracle's (publishers.cpp:99-131):
    the path rows (t exact, positions — BA re-writes included — within tol,
    jour), and the /map_cmap cloud: the same size ceil(n / 3), every device
    point one of the oracle's pvec_buf[0] points at x_buf[0] (the device takes
    every third point in its own downsample order)."""
    rp = ref["path"]
    assert path.shape[0] == rp.shape[0], (path.shape, rp.shape)
    assert np.array_equal(np.round(path[:, 0], 9), np.round(rp[:, 0], 9))
    assert np.abs(path[:, 1:4] - rp[:, 10:13]).max() < tol
    assert np.abs(path[:, 4] - rp[:, 13]).max() < 1e-6
    allp = ref["cmap_all"]
    assert cmap.shape == ref["cmap"].shape and cmap.shape[0] == (allp.shape[0] + 2) // 3 > 100
    from scipy.spatial import cKDTree
    d, j = cKDTree(allp[:, :3].astype(np.float64)).query(cmap[:, :3].astype(np.float64))
    assert d.max() < 1e-4, d.max()
    assert np.array_equal(cmap[:, 3], allp[j, 3])  # intensity of the voxel's first point
    assert len(np.unique(j)) == cmap.shape[0]
