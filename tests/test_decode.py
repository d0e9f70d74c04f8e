"""SURVEY §8(f) row f3 — sensor decoders (lidar_pointcloud_decoder.cpp:21-240)
and pcl_handler's scan preparation (lidar_decoder.cpp:7-43).

Synthetic little-endian records in each sensor's point layout (the
reference's point structs; livox_ros_driver2's CustomPoint as its published
message definition: offset_time u32, x, y, z f32, reflectivity, tag, line u8).
CPU: the oracle's restatement against a numpy statement of the same rules
(point_filter_num stride, blind on the squared range — x, y only for
RoboSense — per-format time, ascending time, the tail beyond 0.11 s dropped,
two dummy points when nothing is left). GPU (marked): vg_decode_scan = oracle
bit for bit (fields and the time sequence; records of equal time — absolute
f64 stamps quantise — compare as sets, std::sort leaving their order
unspecified)."""
import numpy as np
import pytest

FORMATS = {
    # kind, numpy record layout, field offsets
    "livox": (0, np.dtype([("t", "<u4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("tag", "u1"),
                           ("line", "u1"), ("pad", "u1")])),
    "velodyne": (1, np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("t", "<f4"), ("ring", "<u2"),
                              ("pad", "<u2")])),
    "ouster": (2, np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "<f4"), ("t", "<u4"),
                            ("refl", "<u2"), ("ring", "u1"), ("pad", "u1"), ("range", "<u4")])),
    "hesai": (3, np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "<f4"), ("t", "<f8"), ("ring", "<u2"),
                           ("pad", "V6")])),
    "robosense": (4, np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "<f4"), ("ring", "<u2"),
                               ("pad", "V6"), ("t", "<f8")])),
    "tartanair": (5, np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4")])),
}
T_BASE = 1700000000.25


def _records(name, n, seed, yaw_mode=False):
    kind, dt = FORMATS[name]
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=dt)
    az = np.linspace(0, 2 * np.pi, n, endpoint=False) + 0.3
    if yaw_mode:  # a clockwise sweep (yaw falls with time) through the +-180 deg wrap
        az = 2.5 - np.linspace(0, 2 * np.pi * 0.95, n)
    rr = rng.uniform(0.2, 30.0, n).astype(np.float32)
    a["x"], a["y"] = (rr * np.cos(az)).astype(np.float32), (rr * np.sin(az)).astype(np.float32)
    a["z"] = rng.uniform(-2, 2, n).astype(np.float32)
    tsec = np.sort(rng.uniform(0.0, 0.115, n)) + rng.uniform(0, 1e-7, n)  # distinct, a tail past 0.11 s
    rng.shuffle(tsec[: n // 3])  # records not in time order
    if "r" in dt.names:
        a["r"] = rng.uniform(0, 255, n).astype(a["r"].dtype)
    if name == "livox":
        a["t"] = (tsec * 1e9).astype(np.uint32)
    elif name == "velodyne":
        a["t"] = tsec.astype(np.float32) if not yaw_mode else 0.0
    elif name == "ouster":
        a["t"] = (tsec * 1e9).astype(np.uint32)
    elif name == "hesai":
        a["t"] = T_BASE + tsec
        a["t"][0] = T_BASE  # the first record carries the base stamp
    elif name == "robosense":
        a["t"] = T_BASE + tsec
    fmt = dict(kind=kind, stride=dt.itemsize, off_x=dt.fields["x"][1], off_y=dt.fields["y"][1],
               off_z=dt.fields["z"][1], off_intensity=dt.fields["r"][1] if "r" in dt.names else -1,
               off_time=dt.fields["t"][1] if "t" in dt.names else -1, point_filter_num=3, blind=0.5,
               omega_l=3610.0, time_base=T_BASE)
    return a, fmt


def _rows(a):
    return a[np.lexsort(a.T[::-1])]


def _numpy_decode(a, fmt):
    n = a.size
    x, y, z = a["x"], a["y"], a["z"]
    keep = (np.arange(n) % fmt["point_filter_num"]) == 0
    b2 = fmt["blind"] ** 2
    d = (x * x + y * y) if fmt["kind"] == 4 else (x * x + y * y) + z * z  # float32 arithmetic
    keep &= d.astype(np.float64) > b2
    k = fmt["kind"]
    if k == 0:
        t = (a["t"].astype(np.float64) * 1e-9).astype(np.float32)
        inten = a["r"].astype(np.float32)
    elif k == 1:
        t = a["t"].astype(np.float32)
        inten = np.zeros(n, np.float32)
    elif k == 2:
        t = (a["t"].astype(np.float64) / 1e9).astype(np.float32)
        inten = a["r"]
    elif k == 3:
        t = (a["t"] - a["t"][0]).astype(np.float32)
        inten = a["r"]
    elif k == 4:
        t = (a["t"] - fmt["time_base"]).astype(np.float32)
        inten = a["r"]
    else:
        t = np.zeros(n, np.float32)
        inten = np.zeros(n, np.float32)
        keep = np.ones(n, bool)
    out = np.stack([x, y, z, inten, t], 1)[keep]
    out = out[np.argsort(out[:, 4], kind="stable")]
    return out[out[:, 4].astype(np.float64) <= 0.11]


@pytest.mark.parametrize("name", list(FORMATS))
def test_oracle_decoders_match_numpy(oracle_lib, name):
    import oracle
    a, fmt = _records(name, 3000, 17)
    got = oracle.decode_scan(a.tobytes(), fmt)
    ref = _numpy_decode(a, fmt)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    if name == "tartanair":  # every time is 0: std::sort leaves the order unspecified
        got, ref = _rows(got), _rows(ref)
    assert np.array_equal(got, ref)
    assert np.all(np.diff(got[:, 4]) >= 0) and got[-1, 4] <= 0.11


def test_oracle_velodyne_yaw_times_and_empty_scan(oracle_lib):
    import oracle
    a, fmt = _records("velodyne", 2000, 3, yaw_mode=True)
    got = oracle.decode_scan(a.tobytes(), fmt)
    assert got.shape[0] > 100
    assert np.all(got[:, 4] >= 0) and np.all(got[:, 4] < 0.1)  # velodyne_handler 133-135
    a["x"] = a["y"] = a["z"] = 0.01  # everything inside blind: the two dummy points
    got = oracle.decode_scan(a.tobytes(), fmt)
    assert got.shape == (2, 5) and list(got[:, 4]) == [0.0, np.float32(0.09)]


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(FORMATS) + ["velodyne-yaw"])
def test_gpu_decode_matches_oracle(oracle_lib, name):
    import oracle
    import vgconfig
    import vgpu
    yaw = name == "velodyne-yaw"
    a, fmt = _records("velodyne" if yaw else name, 20000, 29, yaw_mode=yaw)
    ref = oracle.decode_scan(a.tobytes(), fmt)
    ctx = vgpu.Context(vgconfig.to_c(vgconfig.load("mid360")), max_points=60_000, max_nodes=100_000,
                       max_fix_points=200_000, hash_log2=16)
    xyz, inten, tm = ctx.decode_scan(a.tobytes(), fmt)
    got = np.concatenate([xyz, inten[:, None], tm[:, None]], 1)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    # the time sequence is identical; records of equal time (absolute f64
    # stamps near 1.7e9 s quantise to 0.24 us) may sit in either order
    assert np.array_equal(got[:, 4], ref[:, 4])
    assert np.array_equal(_rows(got), _rows(ref))
    ctx.close()


def _ref_sync(events, point_notime):
    """sync_packages (src/sensor/sync.cpp:18-96) restated in Python over an event
    stream; returns the packages in order and whether the IMU stream ran dry."""
    scans, imu, out = [], [], []
    st = dict(ready=False, last_pcl=-1.0, imu_last=-1.0, cur=None, beg=0.0, end=0.0)

    def step():
        if not st["ready"]:
            if not scans:
                return False
            sid, hb, last = scans.pop(0)
            st["cur"], st["beg"], st["end"] = sid, hb, hb + last
            if point_notime:
                if st["last_pcl"] < 0:
                    st["last_pcl"] = st["beg"]
                    return False
                st["end"] = st["beg"]
                st["beg"] = st["last_pcl"]
                st["last_pcl"] = st["end"]
            st["ready"] = True
        if st["imu_last"] <= st["end"]:
            return False
        taken = []
        t = imu[0][0]
        while imu and t < st["end"]:
            t = imu[0][0]
            if t > st["end"]:
                break
            taken.append(imu.pop(0))
        st["ready"] = False
        if not imu:
            raise RuntimeError("dry")
        if len(taken) > 4:
            out.append((st["cur"], st["beg"], st["end"], np.array(taken)))
        return True

    for ev in events:
        if ev[0] == "scan":
            scans.append(ev[1:])
        else:
            imu.append(ev[1])
            st["imu_last"] = ev[1][0]
        while step():
            pass
    return out


@pytest.mark.parametrize("point_notime", [0, 1])
def test_sync_packages_match_reference_rules(point_notime):
    import vgpu
    rng = np.random.default_rng(point_notime + 4)
    events, t_imu = [], 0.0
    for k in range(30):
        hb = 0.1 * k + rng.uniform(0, 0.002)
        last = 0.0995 if k % 7 else 0.02  # a short scan gets too few IMU samples
        while t_imu < hb + 0.12:
            t_imu += 0.005 + rng.uniform(-1e-4, 1e-4)
            events.append(("imu", np.array([t_imu, *rng.normal(size=6)])))
        events.insert(len(events) - rng.integers(0, 10), ("scan", k, hb, last))
    ref = _ref_sync(events, point_notime)
    s = vgpu.Sync(point_notime)
    got = []
    for ev in events:
        if ev[0] == "scan":
            s.push_scan(ev[2], ev[3], ev[1])
        else:
            s.push_imu(ev[1])
        while True:
            p = s.pop()
            if p is None:
                break
            if p != "dropped":
                got.append(p)
    s.close()
    assert len(got) == len(ref) and len(ref) > 10
    for (a, b, c, d), (e, f, g, h) in zip(got, ref):
        assert a == e and b == f and c == g and np.array_equal(d, h)
