"""rosbag2 (sqlite3 storage, CDR serialization) -> the event log of
vg_node_replay ("an offline rosbag2 -> flat-binary
converter").

The reference subscribes to an IMU topic (sensor_msgs/msg/Imu) and a LiDAR
topic (livox_ros_driver2/msg/CustomMsg for lidar_type 0, else
sensor_msgs/msg/PointCloud2; node.cpp:144-170). This tool reads those two
topics of a bag in recording order — the order the node's callbacks would see
— and writes, per message, an event the node core replays
(include/vina_node_core.hpp): an IMU sample (stamp, angular velocity, linear
acceleration) or a LiDAR message (header stamp + its records). Livox points
are repacked into the decoder's 20-byte CustomPoint record (offset_time u32,
x, y, z f32, reflectivity, tag, line u8, pad); PointCloud2 data is copied as
is with its point_step and field offsets (taken from the first message).

Only what a bag holds is read: the sqlite3 tables `topics` (id, name, type,
serialization_format) and `messages` (topic_id, timestamp, data) of a
rosbag2 .db3 file, and XCDR1 little-endian payloads (4-byte encapsulation
header, natural alignment relative to the payload start). Bags recorded in
the MCAP storage format are not read (no MCAP reader in this image).

    python bag2events.py <bag.db3 or bag dir> <out.bin> --config mid360 [--lidar-topic T] [--imu-topic T]
"""
import argparse
import glob
import os
import sqlite3
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

IMU_TYPE = "sensor_msgs/msg/Imu"
PC2_TYPE = "sensor_msgs/msg/PointCloud2"
LIVOX_TYPE = "livox_ros_driver2/msg/CustomMsg"
LIVOX_REC = np.dtype([("t", "<u4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("tag", "u1"),
                      ("line", "u1"), ("pad", "u1")])
# the per-format time field of a PointCloud2 (lidar_pointcloud_decoder.hpp point structs)
TIME_FIELD = {1: "time", 2: "t", 3: "timestamp", 4: "timestamp"}


class Cdr:
    """XCDR1 little-endian reader (ROS 2's default serialization)."""

    def __init__(self, buf):
        if len(buf) < 4 or buf[1] != 1:
            raise ValueError("not a little-endian CDR payload (encapsulation %r)" % bytes(buf[:4]))
        self.b = memoryview(buf)[4:]
        self.o = 0

    def _al(self, n):
        self.o += (-self.o) % n

    def prim(self, fmt, size):
        self._al(size)
        v = struct.unpack_from("<" + fmt, self.b, self.o)[0]
        self.o += size
        return v

    def u8(self):
        return self.prim("B", 1)

    def u32(self):
        return self.prim("I", 4)

    def i32(self):
        return self.prim("i", 4)

    def u64(self):
        return self.prim("Q", 8)

    def f64(self):
        return self.prim("d", 8)

    def f64s(self, n):
        self._al(8)
        v = np.frombuffer(self.b, dtype="<f8", count=n, offset=self.o).copy()
        self.o += 8 * n
        return v

    def string(self):
        n = self.u32()
        s = bytes(self.b[self.o:self.o + n - 1]).decode() if n else ""
        self.o += n
        return s

    def header(self):
        sec, nsec = self.i32(), self.u32()
        self.string()  # frame_id
        return sec + nsec * 1e-9


def parse_imu(buf):
    """sensor_msgs/msg/Imu -> [t, gyr 3, acc 3]"""
    c = Cdr(buf)
    t = c.header()
    c.f64s(4 + 9)  # orientation, orientation_covariance
    gyr = c.f64s(3)
    c.f64s(9)
    acc = c.f64s(3)
    return np.array([t, *gyr, *acc])


def parse_pointcloud2(buf):
    """sensor_msgs/msg/PointCloud2 -> (stamp, {field: offset}, point_step, n, data bytes)"""
    c = Cdr(buf)
    t = c.header()
    h, w = c.u32(), c.u32()
    fields = {}
    for _ in range(c.u32()):
        name = c.string()
        off = c.u32()
        c.u8()   # datatype
        c.u32()  # count
        fields[name] = off
    if c.u8():
        raise ValueError("big-endian PointCloud2 data")
    step = c.u32()
    c.u32()  # row_step
    n = c.u32()
    data = bytes(c.b[c.o:c.o + n])
    return t, fields, step, h * w, data


def parse_livox(buf):
    """livox_ros_driver2/msg/CustomMsg -> (stamp, packed 20-byte records)"""
    c = Cdr(buf)
    t = c.header()
    c.u64()  # timebase
    c.u32()  # point_num
    c.u8()   # lidar_id
    for _ in range(3):
        c.u8()  # rsvd
    n = c.u32()
    # CDR lays CustomPoint (u32, 3 x f32, 3 x u8) out at 4-byte alignment: the
    # sequence is n contiguous 20-byte records (the last one's pad byte may be
    # missing at the end of the payload), i.e. LIVOX_REC exactly
    raw = bytes(c.b[c.o:c.o + 20 * n])
    raw += b"\0" * (20 * n - len(raw))
    rec = np.frombuffer(raw, LIVOX_REC).copy()
    rec["pad"] = 0
    return t, rec


def _db3(path):
    if os.path.isdir(path):
        files = sorted(glob.glob(os.path.join(path, "*.db3")))
        if not files:
            raise FileNotFoundError("no .db3 file in %s (MCAP bags are not read)" % path)
        return files
    return [path]


def read_bag(path, lidar_topic=None, imu_topic=None):
    """Yield ("imu", sample) / ("pc2", parsed) / ("livox", parsed) in recording order."""
    for f in _db3(path):
        db = sqlite3.connect("file:%s?mode=ro" % f, uri=True)
        topics = {i: (n, t, s) for i, n, t, s in db.execute("SELECT id, name, type, serialization_format FROM topics")}
        want = {}
        for i, (n, t, s) in topics.items():
            if s != "cdr":
                continue
            if t == IMU_TYPE and imu_topic in (None, n):
                want[i] = "imu"
            elif t == PC2_TYPE and lidar_topic in (None, n):
                want[i] = "pc2"
            elif t == LIVOX_TYPE and lidar_topic in (None, n):
                want[i] = "livox"
        if want:
            q = "SELECT topic_id, data FROM messages WHERE topic_id IN (%s) ORDER BY timestamp, id" % ",".join(
                str(i) for i in want)
            for tid, data in db.execute(q):
                kind = want[tid]
                if kind == "imu":
                    yield "imu", parse_imu(data)
                elif kind == "pc2":
                    yield "pc2", parse_pointcloud2(data)
                else:
                    yield "livox", parse_livox(data)
        db.close()


def lidar_format(p, kind, fields=None, step=None):
    """vg_lidar_format for the config's General section (node.cpp:69-76)."""
    import vgpu
    g = p["General"]
    f = dict(kind=kind, stride=0, off_x=-1, off_y=-1, off_z=-1, off_intensity=-1, off_time=-1,
             point_filter_num=int(g.get("point_filter_num", 3)), blind=float(g["blind"]), omega_l=3610.0,
             time_base=0.0)
    if kind == 0:
        f.update(stride=LIVOX_REC.itemsize, off_time=0, off_x=4, off_y=8, off_z=12, off_intensity=16)
    else:
        f.update(stride=step, off_x=fields.get("x", -1), off_y=fields.get("y", -1), off_z=fields.get("z", -1),
                 off_intensity=fields.get("intensity", -1), off_time=fields.get(TIME_FIELD.get(kind), -1))
    return vgpu.LidarFormat(**f)


def convert(bag, out, config="mid360", lidar_topic=None, imu_topic=None, seed=None):
    """Write the event log; returns (imu samples, lidar messages)."""
    import vgconfig
    p = vgconfig.load(config)
    kind = int(p["General"].get("lidar_type", 0))
    cfg = vgconfig.to_c(p, cold_start=0 if seed is not None else 1, scale_gravity=0.0 if seed is None else 1.0)
    events, fmt = [], None
    for ev in read_bag(bag, lidar_topic, imu_topic):
        if ev[0] == "imu":
            events.append(struct.pack("<i", 0) + np.ascontiguousarray(ev[1], dtype="<f8").tobytes())
            continue
        if ev[0] == "livox":
            t, rec = ev[1]
            if fmt is None:
                fmt = lidar_format(p, 0)
            events.append(struct.pack("<idii", 1, t, rec.size, rec.itemsize) + rec.tobytes())
        else:
            t, fields, step, n, data = ev[1]
            if fmt is None:
                fmt = lidar_format(p, kind, fields, step)
            events.append(struct.pack("<idii", 1, t, n, step) + data[: n * step])
    if fmt is None:
        raise ValueError("no LiDAR messages found in %s" % bag)
    with open(out, "wb") as f:
        f.write(b"VGEVENT1")
        f.write(bytes(cfg))
        f.write(bytes(fmt))
        f.write(struct.pack("<ii", int(p["Odometry"].get("point_notime", 0)), 1 if seed is not None else 0))
        if seed is not None:
            f.write(np.ascontiguousarray(seed, dtype="<f8").tobytes())
        for e in events:
            f.write(e)
        f.write(struct.pack("<i", -1))
    n_imu = sum(1 for e in events if e[:4] == b"\0\0\0\0")
    return n_imu, len(events) - n_imu


def read_events(path):
    """The event log back: (vg_config bytes, vg_lidar_format, point_notime, seed or
    None, events) with events ("imu", (7,) array) / ("scan", stamp, n, stride, bytes)."""
    import vgconfig
    import vgpu
    with open(path, "rb") as f:
        b = f.read()
    if b[:8] != b"VGEVENT1":
        raise ValueError("not an event log")
    o = 8
    ncfg, nfmt = ctypes_size(vgconfig.CConfig), ctypes_size(vgpu.LidarFormat)
    cfg = b[o:o + ncfg]
    o += ncfg
    fmt = vgpu.LidarFormat.from_buffer_copy(b[o:o + nfmt])
    o += nfmt
    notime, has_seed = struct.unpack_from("<ii", b, o)
    o += 8
    seed = None
    if has_seed:
        seed = np.frombuffer(b, "<f8", 250, o).copy()
        o += 8 * 250
    ev = []
    while o < len(b):
        (k,) = struct.unpack_from("<i", b, o)
        o += 4
        if k < 0:
            break
        if k == 0:
            ev.append(("imu", np.frombuffer(b, "<f8", 7, o).copy()))
            o += 56
        else:
            t, n, stride = struct.unpack_from("<dii", b, o)
            o += 16
            ev.append(("scan", t, n, stride, b[o:o + n * stride]))
            o += n * stride
    return cfg, fmt, notime, seed, ev


def ctypes_size(t):
    import ctypes
    return ctypes.sizeof(t)


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("bag")
    ap.add_argument("out")
    ap.add_argument("--config", default="mid360")
    ap.add_argument("--lidar-topic")
    ap.add_argument("--imu-topic")
    a = ap.parse_args()
    n_imu, n_lid = convert(a.bag, a.out, a.config, a.lidar_topic, a.imu_topic)
    print("%s: %d IMU samples, %d LiDAR messages" % (a.out, n_imu, n_lid))


if __name__ == "__main__":
    main()
