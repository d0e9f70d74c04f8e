"""Deterministic synthetic LiDAR + IMU sequences (SURVEY §8(d) "Synthetic inputs").

Scene: a 40 x 20 x 6 m box plus 32 random planar panels (axis-aligned and
30-degree-oblique, 1-6 m), so most voxels are planar. A spinning LiDAR with L
rings (uniform elevation in [-25, +15] deg) and A azimuth steps is ray-cast from
a smooth Lissajous trajectory (~1.4 m/s, yaw rate <= ~20 deg/s). Range noise
N(0, range_sigma), bearing noise N(0, bearing_sigma_deg). Ranges are clipped to
[blind, 80] m (the decoder's blind filter, lidar_pointcloud_decoder.cpp).
IMU at 200 Hz from analytic derivatives plus white noise and constant biases.

Scans are emitted motion-compensated (all points of scan k in the LiDAR frame
at the scan-end pose t_k), i.e. what IMUEKF::motion_blur's deskew
(imu_ekf.cpp:114-144) hands to the hot path.

Seeds: numpy PCG64 seeded with 0x5EED0000 + seq_id.
"""
import numpy as np

SCAN_DT = 0.1
IMU_HZ = 200
IMU_PER_SCAN = int(round(SCAN_DT * IMU_HZ))
G = np.array([0.0, 0.0, -9.8])

LIDARS = {
    "64line": (64, 2048),     # 131,072 rays
    "128line": (128, 1563),   # 200,064 rays
    "1M": (128, 7813),        # 1,000,064 rays
    "16line": (16, 1800),     # VLP-16-like, 28,800 rays
    "tiny": (16, 512),        # 8,192 rays (fast unit tests)
}


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])


def _ry(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1.0, 0], [-s, 0, c]])


def _rx(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1.0, 0, 0], [0, c, -s], [0, s, c]])


def _log(R):
    tr = np.trace(R)
    th = 0.0 if tr > 3 - 1e-12 else np.arccos(np.clip(0.5 * (tr - 1), -1, 1))
    K = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return 0.5 * K if abs(th) < 1e-6 else 0.5 * th / np.sin(th) * K


class Trajectory:
    """Smooth Lissajous body trajectory inside the box."""

    def pos(self, t):
        return np.array([12.0 * np.sin(0.1 * t), 5.0 * np.sin(0.13 * t + 0.5), 1.5 + 0.3 * np.sin(0.2 * t)])

    def vel(self, t):
        return np.array([1.2 * np.cos(0.1 * t), 0.65 * np.cos(0.13 * t + 0.5), 0.06 * np.cos(0.2 * t)])

    def acc(self, t):
        return np.array([-0.12 * np.sin(0.1 * t), -0.0845 * np.sin(0.13 * t + 0.5), -0.012 * np.sin(0.2 * t)])

    def rot(self, t):
        yaw = 1.2 * np.sin(0.3 * t)
        pitch = 0.04 * np.sin(0.5 * t)
        roll = 0.05 * np.sin(0.7 * t)
        return _rz(yaw) @ _ry(pitch) @ _rx(roll)

    def omega_body(self, t, h=1e-5):
        return _log(self.rot(t - h).T @ self.rot(t + h)) / (2 * h)


class Scene:
    def __init__(self, rng):
        # box: x in [-20,20], y in [-10,10], z in [0,6]
        self.box_lo = np.array([-20.0, -10.0, 0.0])
        self.box_hi = np.array([20.0, 10.0, 6.0])
        P = []
        for i in range(32):
            c = rng.uniform(self.box_lo + [1, 1, 0.5], self.box_hi - [1, 1, 0.5])
            axis = rng.integers(0, 3)
            n = np.zeros(3)
            n[axis] = 1.0
            if rng.uniform() < 0.5:  # 30-degree oblique about a perpendicular axis
                other = (axis + 1 + rng.integers(0, 2)) % 3
                ang = np.deg2rad(30.0) * (1 if rng.uniform() < 0.5 else -1)
                k = np.zeros(3)
                k[3 - axis - other] = 1.0
                K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
                Rk = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
                n = Rk @ n
            a = np.cross(n, [0.0, 0.0, 1.0] if abs(n[2]) < 0.9 else [1.0, 0.0, 0.0])
            a /= np.linalg.norm(a)
            b = np.cross(n, a)
            ha, hb = rng.uniform(0.5, 3.0, size=2)
            P.append((c, n, a, b, ha, hb))
        self.panels = P

    def cast(self, o, d, max_range=80.0):
        """Ray-cast from origin o ((3,) or per ray (n,3)) along unit dirs d (n,3). Returns ranges (n,) and
        surface id."""
        n = d.shape[0]
        o2 = np.broadcast_to(o, d.shape)
        best = np.full(n, np.inf)
        sid = np.full(n, -1, dtype=np.int32)
        with np.errstate(divide="ignore", invalid="ignore"):
            for ax in range(3):
                for k, bound in enumerate((self.box_lo[ax], self.box_hi[ax])):
                    t = (bound - o2[:, ax]) / d[:, ax]
                    ok = (t > 1e-6) & (t < best)
                    best = np.where(ok, t, best)
                    sid = np.where(ok, 2 * ax + k, sid)
            for j, (c, nrm, a, b, ha, hb) in enumerate(self.panels):
                den = d @ nrm
                t = ((c[None, :] - o2) @ nrm) / den
                p = o2 + t[:, None] * d
                q = p - c[None, :]
                ok = (t > 1e-6) & (t < best) & (np.abs(q @ a) <= ha) & (np.abs(q @ b) <= hb)
                best = np.where(ok, t, best)
                sid = np.where(ok, 6 + j, sid)
        best[best > max_range] = np.inf
        return best, sid


class Sequence:
    """A synthetic LiDAR-inertial sequence. scan(k) covers (t_k - 0.1, t_k]."""

    def __init__(self, lidar="64line", seq_id=0, blind=3.0, ext_R=None, ext_t=None, range_sigma=0.02,
                 bearing_sigma_deg=0.05, gyr_sigma=0.002, acc_sigma=0.02, imu_in_g=False):
        self.L, self.A = LIDARS[lidar]
        self.seed = 0x5EED0000 + seq_id
        rng = np.random.default_rng(self.seed)
        self.scene = Scene(rng)
        self.traj = Trajectory()
        self.blind = blind
        self.ext_R = np.eye(3) if ext_R is None else np.asarray(ext_R, dtype=np.float64).reshape(3, 3)
        self.ext_t = np.zeros(3) if ext_t is None else np.asarray(ext_t, dtype=np.float64)
        self.range_sigma = range_sigma
        self.bearing_sigma = np.deg2rad(bearing_sigma_deg)
        self.gyr_sigma, self.acc_sigma = gyr_sigma, acc_sigma
        # accelerometer unit: m/s^2, or g (Livox Mid-360's IMU; the reference
        # then multiplies every sample by scale_gravity = 9.8, imu_ekf.cpp:182-185)
        self.acc_unit = 9.8 if imu_in_g else 1.0
        self.bg = rng.normal(0, 0.002, 3)
        self.ba = rng.normal(0, 0.02, 3)
        el = np.deg2rad(np.linspace(-25.0, 15.0, self.L))
        az = np.linspace(0, 2 * np.pi, self.A, endpoint=False)
        E, Az = np.meshgrid(el, az, indexing="xy")  # azimuth-major order (firing order)
        self.dirs = np.stack([np.cos(E) * np.cos(Az), np.cos(E) * np.sin(Az), np.sin(E)], -1).reshape(-1, 3)
        self.t0 = 0.0

    @staticmethod
    def t_end(k):
        return (IMU_PER_SCAN * (k + 1)) / float(IMU_HZ)

    def scan(self, k):
        """Returns xyz float32 (n,3) in the LiDAR frame, intensity float32 (n,), beg, end."""
        rng = np.random.default_rng((self.seed << 20) + k)
        te = self.t_end(k)
        R = self.traj.rot(te)
        p = self.traj.pos(te)
        o = R @ self.ext_t + p
        Rl = R @ self.ext_R
        dw = self.dirs @ Rl.T
        r, sid = self.scene.cast(o, dw)
        ok = np.isfinite(r) & (r >= self.blind)
        d = self.dirs[ok]
        r = r[ok] + rng.normal(0, self.range_sigma, ok.sum())
        # bearing noise: perturb in the tangent plane
        t1 = np.cross(d, np.array([0.0, 0.0, 1.0]))
        t1 /= np.maximum(np.linalg.norm(t1, axis=1, keepdims=True), 1e-9)
        t2 = np.cross(d, t1)
        e = rng.normal(0, self.bearing_sigma, (d.shape[0], 2))
        dn = d + e[:, :1] * t1 + e[:, 1:] * t2
        dn /= np.linalg.norm(dn, axis=1, keepdims=True)
        xyz = (dn * r[:, None]).astype(np.float32)
        inten = (sid[ok] % 97).astype(np.float32)
        return xyz, inten, te - 0.1, te

    def scan_raw(self, k):
        """The same sweep as it leaves the sensor: ray (a, ring) fires at
        beg + 0.1 (a + 1) / A from the pose of that instant and is expressed in the
        LiDAR frame of that instant (what IMUEKF::motion_blur deskews, SURVEY row
        f1). Returns xyz float32 (n,3), intensity, per-point time offset from beg
        (float32, ascending: azimuth-major firing order), beg, end."""
        rng = np.random.default_rng((self.seed << 20) + k)
        te = self.t_end(k)
        beg = te - 0.1
        na = self.A
        tr = 0.1 * (np.arange(na) + 1) / na
        Rs = np.stack([self.traj.rot(beg + t) for t in tr])                   # (A,3,3)
        ps = np.stack([self.traj.pos(beg + t) for t in tr])
        a_of = np.repeat(np.arange(na), self.L)                                 # ray -> azimuth index
        Rl = Rs @ self.ext_R                                                    # (A,3,3)
        o = (Rs @ self.ext_t) + ps                                              # (A,3)
        dw = np.einsum("nij,nj->ni", Rl[a_of], self.dirs)
        r, sid = self.scene.cast(o[a_of], dw)
        ok = np.isfinite(r) & (r >= self.blind)
        d = self.dirs[ok]
        r = r[ok] + rng.normal(0, self.range_sigma, ok.sum())
        t1 = np.cross(d, np.array([0.0, 0.0, 1.0]))
        t1 /= np.maximum(np.linalg.norm(t1, axis=1, keepdims=True), 1e-9)
        t2 = np.cross(d, t1)
        e = rng.normal(0, self.bearing_sigma, (d.shape[0], 2))
        dn = d + e[:, :1] * t1 + e[:, 1:] * t2
        dn /= np.linalg.norm(dn, axis=1, keepdims=True)
        xyz = (dn * r[:, None]).astype(np.float32)
        inten = (sid[ok] % 97).astype(np.float32)
        times = tr[a_of[ok]].astype(np.float32)
        return xyz, inten, times, beg, te

    def imu(self, k):
        """IMU samples (m,7) [t, gx,gy,gz, ax,ay,az] covering [t_{k-1}, t_k] (empty for k=0)."""
        if k == 0:
            return np.zeros((0, 7))
        rng = np.random.default_rng((self.seed << 21) + k)
        js = np.arange(IMU_PER_SCAN * k, IMU_PER_SCAN * (k + 1) + 1)
        out = np.zeros((len(js), 7))
        for i, j in enumerate(js):
            t = j / float(IMU_HZ)
            R = self.traj.rot(t)
            w = self.traj.omega_body(t)
            f = R.T @ (self.traj.acc(t) - G)
            # noise is a deterministic function of the sample index so that the
            # shared boundary sample of two scans is identical
            nr = np.random.default_rng((self.seed << 22) + j)
            out[i, 0] = t
            out[i, 1:4] = w + self.bg + nr.normal(0, self.gyr_sigma, 3)
            out[i, 4:7] = (f + self.ba + nr.normal(0, self.acc_sigma, 3)) / self.acc_unit
        return out

    def gt_state(self, k):
        """Ground-truth body state at t_k as the 250-double IMUST layout (biases zero, default cov)."""
        te = self.t_end(k)
        s = np.zeros(250)
        s[0] = te
        s[1:10] = self.traj.rot(te).reshape(-1)
        s[10:13] = self.traj.pos(te)
        s[13:16] = self.traj.vel(te)
        s[22:25] = G
        cov = np.eye(15) * 1e-4
        cov[9:, 9:] = np.eye(6) * 1e-5
        s[25:] = cov.reshape(-1)
        return s

    def gt_pose(self, k):
        te = self.t_end(k)
        return self.traj.rot(te), self.traj.pos(te)


def ate(traj_a, traj_b):
    """RMS position difference between two trajectories given as (n,13) [t,R9,p3] arrays."""
    a = np.asarray(traj_a)[:, 10:13]
    b = np.asarray(traj_b)[:, 10:13]
    return float(np.sqrt(np.mean(np.sum((a - b) ** 2, axis=1))))


def write_replay(path, seq, cconfig, nscan, seed_state=None):
    """Flat replay file read by vina-slam_amd/examples/vg_replay.cpp."""
    import ctypes
    import struct
    with open(path, "wb") as f:
        f.write(b"VGRPLAY1")
        f.write(struct.pack("<i", nscan))
        f.write(bytes(cconfig))
        st = seq.gt_state(0) if seed_state is None else seed_state
        f.write(np.ascontiguousarray(st, dtype="<f8").tobytes())
        for k in range(nscan):
            xyz, inten, b, e = seq.scan(k)
            imu = seq.imu(k)
            f.write(struct.pack("<ddii", b, e, xyz.shape[0], imu.shape[0]))
            xyzi = np.concatenate([xyz, inten[:, None]], 1).astype("<f4")
            f.write(xyzi.tobytes())
            f.write(np.ascontiguousarray(imu, dtype="<f8").tobytes())
    _ = ctypes


def read_tum(path):
    """TUM pose file (io.cpp:67-77): t x y z qx qy qz qw -> (n, 8)."""
    return np.loadtxt(path, ndmin=2)
