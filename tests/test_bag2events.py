"""SURVEY §8 row f3 — the offline rosbag2 -> event-log converter
(vina-slam_amd/py/bag2events.py) and, on the GPU, the whole replay chain
bag -> event log -> vg_node_replay (the node core) -> TUM against the oracle.

The bags are written here with a CDR encoder stated independently of the
converter's reader, from the ROS 2 message definitions (XCDR1 little-endian:
encapsulation 00 01 00 00, natural alignment from the payload start; strings
as u32 length incl. NUL; sequences as u32 count + elements):
sensor_msgs/msg/Imu, sensor_msgs/msg/PointCloud2 (+ PointField) and
livox_ros_driver2/msg/CustomMsg (+ CustomPoint), in rosbag2's sqlite3 schema
(topics / messages tables). No bag from the reference is available (it ships
none), so the fixtures are synthetic."""
import os
import sqlite3
import struct
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class CdrW:
    def __init__(self):
        self.b = bytearray()

    def al(self, n):
        self.b += b"\0" * ((-len(self.b)) % n)

    def put(self, fmt, v):
        n = struct.calcsize("<" + fmt)
        self.al(n)
        self.b += struct.pack("<" + fmt, v)

    def string(self, s):
        e = s.encode() + b"\0"
        self.put("I", len(e))
        self.b += e

    def header(self, t, frame="livox_frame"):
        sec = int(np.floor(t))
        self.put("i", sec)
        self.put("I", int(round((t - sec) * 1e9)))
        self.string(frame)

    def payload(self):
        return b"\x00\x01\x00\x00" + bytes(self.b)


def cdr_imu(row):
    w = CdrW()
    w.header(row[0], "imu_link")
    for v in [0.0, 0.0, 0.0, 1.0] + [0.0] * 9:  # orientation, its covariance
        w.put("d", v)
    for v in list(row[1:4]) + [0.0] * 9 + list(row[4:7]) + [0.0] * 9:
        w.put("d", v)
    return w.payload()


def cdr_livox(stamp, rec):
    w = CdrW()
    w.header(stamp)
    w.put("Q", int(stamp * 1e9))  # timebase
    w.put("I", rec.size)          # point_num
    w.put("B", 0)                 # lidar_id
    for _ in range(3):
        w.put("B", 0)             # rsvd
    w.put("I", rec.size)
    for p in rec:
        w.put("I", int(p["t"]))
        for k in "xyz":
            w.put("f", float(p[k]))
        w.put("B", int(p["r"]))
        w.put("B", int(p["tag"]))
        w.put("B", int(p["line"]))
    return w.payload()


def cdr_pointcloud2(stamp, fields, step, data, n):
    w = CdrW()
    w.header(stamp, "velodyne")
    w.put("I", 1)
    w.put("I", n)
    w.put("I", len(fields))
    for name, off, dtype in fields:
        w.string(name)
        w.put("I", off)
        w.put("B", dtype)
        w.put("I", 1)
    w.put("B", 0)  # is_bigendian
    w.put("I", step)
    w.put("I", step * n)
    w.put("I", len(data))
    w.b += data
    w.put("B", 1)  # is_dense
    return w.payload()


def write_bag(path, msgs):
    """msgs: (topic, type, recv time s, payload) in any order."""
    db = sqlite3.connect(path)
    db.execute("CREATE TABLE topics(id INTEGER PRIMARY KEY, name TEXT NOT NULL, type TEXT NOT NULL, "
               "serialization_format TEXT NOT NULL, offered_qos_profiles TEXT NOT NULL)")
    db.execute("CREATE TABLE messages(id INTEGER PRIMARY KEY, topic_id INTEGER NOT NULL, "
               "timestamp INTEGER NOT NULL, data BLOB NOT NULL)")
    ids = {}
    for topic, typ, _, _ in msgs:
        if topic not in ids:
            ids[topic] = len(ids) + 1
            db.execute("INSERT INTO topics VALUES (?, ?, ?, 'cdr', '')", (ids[topic], topic, typ))
    for topic, _, t, data in msgs:
        db.execute("INSERT INTO messages(topic_id, timestamp, data) VALUES (?, ?, ?)",
                   (ids[topic], int(round(t * 1e9)), data))
    db.commit()
    db.close()


def _sequence_bag(tmp_path, nscan=16):
    import synth
    import vgconfig
    from test_node_core import _events
    p = vgconfig.load("mid360")
    g = p["General"]
    seq = synth.Sequence("16line", 12, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    events = _events(seq, nscan)
    msgs, t_last = [], 0.0
    for e in events:
        if e[0] == "imu":
            t_last = e[1][0]
            msgs.append(("/livox/imu", "sensor_msgs/msg/Imu", t_last, cdr_imu(e[1])))
        else:  # arrives after the IMU samples up to the sweep's end
            msgs.append(("/livox/lidar", "livox_ros_driver2/msg/CustomMsg", t_last + 1e-6, cdr_livox(e[1], e[2])))
    msgs.append(("/other", "std_msgs/msg/String", 0.5, b"\x00\x01\x00\x00\x01\x00\x00\x00\x00"))
    bag = tmp_path / "seq.db3"
    write_bag(bag, msgs)
    return p, seq, events, bag


def test_cdr_reader_round_trips():
    import bag2events as b2e
    row = np.array([12.25, 0.1, -0.2, 0.3, 9.7, -0.1, 0.05])
    got = b2e.parse_imu(cdr_imu(row))
    assert np.allclose(got, row, rtol=0, atol=1e-9) and np.array_equal(got[1:], row[1:])
    rec = np.zeros(5, b2e.LIVOX_REC)
    rec["t"], rec["x"], rec["y"], rec["z"] = np.arange(5) * 1000, 1.5, -2.5, np.arange(5),
    rec["r"], rec["tag"], rec["line"] = 7, 16, 3
    t, back = b2e.parse_livox(cdr_livox(3.5, rec))
    assert t == 3.5 and back.tobytes() == rec.tobytes()
    vel = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("intensity", "<f4"), ("ring", "<u2"), ("pad", "<u2"),
                    ("time", "<f4")])
    a = np.zeros(7, vel)
    a["x"], a["time"] = np.arange(7), np.linspace(0, 0.09, 7)
    fields = [(n, vel.fields[n][1], 7) for n in ("x", "y", "z", "intensity", "time")]
    t, fl, step, n, data = b2e.parse_pointcloud2(cdr_pointcloud2(4.0, fields, vel.itemsize, a.tobytes(), 7))
    assert t == 4.0 and step == vel.itemsize and n == 7 and data == a.tobytes()
    assert fl == {n: o for n, o, _ in fields}
    p = {"General": {"blind": 0.5, "point_filter_num": 2}}
    f = b2e.lidar_format(p, 1, fl, step)
    assert (f.kind, f.stride, f.off_time, f.off_intensity, f.point_filter_num) == (1, step, vel.fields["time"][1],
                                                                                  vel.fields["intensity"][1], 2)


def test_converter_keeps_messages_in_recording_order(tmp_path):
    import bag2events as b2e
    p, seq, events, bag = _sequence_bag(tmp_path)
    out = tmp_path / "ev.bin"
    n_imu, n_lid = b2e.convert(str(bag), str(out), "mid360", seed=seq.gt_state(0))
    assert n_lid == sum(e[0] == "scan" for e in events) and n_imu == len(events) - n_lid
    cfg, fmt, notime, seed, ev = b2e.read_events(str(out))
    assert np.array_equal(seed, seq.gt_state(0)) and fmt.kind == 0 and fmt.stride == 20 and notime == 0
    assert len(ev) == len(events)
    for a, b in zip(ev, events):
        assert a[0] == b[0]
        if a[0] == "imu":
            assert abs(a[1][0] - b[1][0]) < 1e-9 and np.array_equal(a[1][1:], b[1][1:])
        else:
            assert abs(a[1] - b[1]) < 1e-9 and a[2] == b[2].size and a[4] == b[2].tobytes()


@pytest.mark.gpu
def test_bag_replay_matches_oracle(oracle_lib, tmp_path):
    """bag -> event log -> vg_node_replay (GPU) = the oracle on the same events."""
    import bag2events as b2e
    from test_node_core import LIVOX, _oracle_tum
    p, seq, _, bag = _sequence_bag(tmp_path)
    log, tum = tmp_path / "ev.bin", tmp_path / "out.tum"
    b2e.convert(str(bag), str(log), "mid360", seed=seq.gt_state(0))
    _, fmt, _, seed, ev = b2e.read_events(str(log))
    exe = os.path.join(REPO, "vina-slam_amd", "bin", "vg_node_replay")
    r = subprocess.run([exe, str(log), str(tum)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = np.array([[float(x) for x in ln.split()] for ln in tum.read_text().splitlines()])
    events = [e if e[0] == "imu" else ("scan", e[1], np.frombuffer(e[4], LIVOX)) for e in ev]
    fd = {k: getattr(fmt, k) for k, _ in fmt._fields_}
    ref, npk = _oracle_tum(p, fd, seed, events)
    assert npk >= 14 and rows.shape == (ref.shape[0], 8)
    err = np.linalg.norm(rows[:, 1:4] - ref[:, 10:13], axis=1)
    print("bag replay vs oracle: max position difference %.3e m over %d poses" % (err.max(), len(err)))
    assert err.max() < 1e-8
