"""ctypes binding of the product C-ABI (include/vina_gpu.h, lib/libvina_gpu.so).

This is the Python face of the drop-in boundary used by tests/ and bench.py. It
loads ONLY the in-tree HIP library; there is no CPU fallback — if the library
or a GPU is missing every call raises.
"""
import ctypes
import os
import re
import subprocess

import numpy as np

from vgconfig import CConfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
LIB = os.environ.get("VINA_GPU_LIB") or os.path.join(PKG, "lib", "libvina_gpu.so")
HEADER = os.path.join(REPO, "include", "vina_gpu.h")
STATE_LEN = 250


class Capacity(ctypes.Structure):
    _fields_ = [("max_points_per_scan", ctypes.c_int), ("max_nodes", ctypes.c_int),
                ("max_fix_points", ctypes.c_int), ("hash_log2", ctypes.c_int)]


class LidarFormat(ctypes.Structure):
    """vg_lidar_format."""
    _fields_ = [("kind", ctypes.c_int), ("stride", ctypes.c_int), ("off_x", ctypes.c_int), ("off_y", ctypes.c_int),
                ("off_z", ctypes.c_int), ("off_intensity", ctypes.c_int), ("off_time", ctypes.c_int),
                ("point_filter_num", ctypes.c_int), ("blind", ctypes.c_double), ("omega_l", ctypes.c_double),
                ("time_base", ctypes.c_double)]


class ScanDev(ctypes.Structure):
    _fields_ = [("d_x", ctypes.c_void_p), ("d_y", ctypes.c_void_p), ("d_z", ctypes.c_void_p),
                ("d_intensity", ctypes.c_void_p), ("d_time", ctypes.c_void_p), ("n", ctypes.c_int),
                ("pcl_beg_time", ctypes.c_double), ("pcl_end_time", ctypes.c_double),
                ("imu", ctypes.POINTER(ctypes.c_double)), ("m", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("n_raw", ctypes.c_int), ("n_ds", ctypes.c_int), ("iekf_iters", ctypes.c_int),
                ("iekf_matches", ctypes.c_int * 4), ("roots_new", ctypes.c_int), ("n_slide", ctypes.c_int),
                ("n_factors", ctypes.c_int), ("ba_iters", ctypes.c_int), ("degenerate", ctypes.c_int),
                ("nodes_used", ctypes.c_int), ("fix_used", ctypes.c_int), ("plane_updates", ctypes.c_int),
                ("fix_full", ctypes.c_int), ("iekf_planes", ctypes.c_int * 4), ("v_ins", ctypes.c_int),
                ("ba_hess", ctypes.c_int), ("init_phase", ctypes.c_int), ("init_rounds", ctypes.c_int),
                ("init_valid", ctypes.c_int), ("iekf_points", ctypes.c_int)]


def _stats_dict(s):
    return {k: (list(getattr(s, k)) if k in ("iekf_matches", "iekf_planes") else getattr(s, k))
            for k, _ in Stats._fields_}


# vg_host_allreduce_fn: int (*)(void* buf, int count, int dtype, void* user)
HOST_ALLREDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)


def rccl_unique_id():
    buf = ctypes.create_string_buffer(128)
    r = lib().vg_rccl_unique_id(buf)
    if r != 0:
        raise VgError("vg_rccl_unique_id failed (%d)" % r)
    return buf.raw


def build(jobs=8):
    subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", PKG])


def header_symbols():
    """Every function the C-ABI header declares."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void\*?|const char\*|vg_\w+\*)\s+(vg_\w+)\s*\(", txt, re.M)))


_lib = None


def _torch_first():
    """PyTorch-ROCm carries its own HIP runtime beside /opt/rocm's (which the
    library links). Both share the process's device address space, but the
    one that opens the GPU second must not be torch's: its init then reports
    "No HIP GPUs are available". Callers hand torch device buffers to the
    library, so open torch's runtime first whenever torch is installed."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("libvina_gpu.so not built: run `make -C vina-slam_amd` (no CPU fallback exists)")
        _torch_first()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        dp = ctypes.POINTER(ctypes.c_double)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int)
        L.vg_create.argtypes = [ctypes.POINTER(CConfig), ctypes.POINTER(Capacity), ctypes.c_int, ctypes.POINTER(P)]
        L.vg_destroy.argtypes = [P]
        L.vg_last_error.argtypes = [P]
        L.vg_last_error.restype = ctypes.c_char_p
        L.vg_reset.argtypes = [P]
        L.vg_downsample.argtypes = [P, fp, fp, ctypes.c_int, ctypes.c_double, fp, ip]
        L.vg_downsample_close.argtypes = [P, fp, fp, ctypes.c_int, ctypes.c_double, fp, ip]
        L.vg_seed.argtypes = [P, dp]
        L.vg_lio_kdtree.argtypes = [P, fp, ctypes.c_int, dp, ip, ip]
        L.vg_kdmap_get.argtypes = [P, fp, ctypes.c_int, ip]
        L.vg_decode_scan.argtypes = [P, P, ctypes.c_int, ctypes.POINTER(LidarFormat), fp, fp, fp, ip]
        L.vg_sync_create.argtypes = [ctypes.c_int]
        L.vg_sync_create.restype = P
        L.vg_sync_destroy.argtypes = [P]
        L.vg_sync_push_scan.argtypes = [P, ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.vg_sync_push_imu.argtypes = [P, dp]
        L.vg_sync_pop.argtypes = [P, ip, dp, dp, dp, ctypes.c_int, ip, ip]
        L.vg_step.argtypes = [P, fp, fp, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp, ctypes.c_int]
        L.vg_step_dev.argtypes = [P, P, P, P, P, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp, ctypes.c_int]
        L.vg_step_deskew.argtypes = [P, fp, fp, fp, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp, ctypes.c_int]
        L.vg_step_deskew_dev.argtypes = [P, P, P, P, P, P, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp,
                                         ctypes.c_int]
        L.vg_get_state.argtypes = [P, dp]
        L.vg_get_stats.argtypes = [P, ctypes.POINTER(Stats)]
        L.vg_stats_log.argtypes = [P, ctypes.POINTER(Stats), ctypes.c_int, ip]
        L.vg_release_far.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
        L.vg_window_states.argtypes = [P, dp, ip]
        L.vg_trajectory.argtypes = [P, dp, ctypes.c_int, ip]
        L.vg_path.argtypes = [P, dp, ctypes.c_int, ip]
        L.vg_poll.argtypes = [P, ip, ip, ip]
        L.vg_poll_rows.argtypes = [P, dp, ctypes.c_int, ctypes.c_int, dp, ctypes.c_int]
        L.vg_local_map.argtypes = [P, fp, ctypes.c_int, ip]
        L.vg_set_publish.argtypes = [P, ctypes.c_int]
        L.vg_scan_load.argtypes = [P, fp, fp, ctypes.c_int]
        L.vg_scan_bind_dev.argtypes = [P, P, P, P, P, ctypes.c_int]
        L.vg_propagate.argtypes = [P, dp, ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.vg_downsample_scan.argtypes = [P, ip]
        L.vg_lio_state_estimation.argtypes = [P, ip]
        L.vg_window_push.argtypes = [P, dp, ctypes.c_int]
        L.vg_cut_voxel_multi.argtypes = [P]
        L.vg_multi_recut.argtypes = [P, ip]
        L.vg_damping_iter.argtypes = [P, ip]
        L.vg_multi_margi.argtypes = [P]
        L.vg_step_end.argtypes = [P]
        L.vg_win_count.argtypes = [P, ip]
        L.vg_profile.argtypes = [P, ctypes.c_int]
        L.vg_profile_read.argtypes = [P, ctypes.c_int, dp, ip]
        L.vg_rccl_unique_id.argtypes = [ctypes.c_char_p]
        L.vg_shard_rccl.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
        L.vg_shard_host.argtypes = [P, ctypes.c_int, ctypes.c_int, HOST_ALLREDUCE, P]
        L.vg_stream.argtypes = [P]
        L.vg_stream.restype = P
        L.vg_set_wait_policy.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.vg_multi_create.argtypes = [ctypes.POINTER(P), ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.vg_multi_create.restype = P
        L.vg_multi_step_dev.argtypes = [P, ctypes.POINTER(ScanDev)]
        L.vg_multi_sync.argtypes = [P]
        L.vg_multi_set_active.argtypes = [P, ctypes.c_int]
        L.vg_multi_destroy.argtypes = [P]
        L.vgx_debug.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.vgx_downsample_hashed.argtypes = [P, fp, fp, ctypes.c_int, ctypes.c_double, fp, ip]
        L.vgx_ba_capture.argtypes = [P, dp, ctypes.c_int, ip]
        if hasattr(L, "vgx_ba_solve"):  # absent from builds older than the test entry (A/B runs)
            L.vgx_ba_solve.argtypes = [P, dp, dp, dp]
        if hasattr(L, "vgx_memo_probe"):
            L.vgx_memo_probe.argtypes = [P, ip]
        if hasattr(L, "vgx_roots"):
            L.vgx_roots.argtypes = [P, ctypes.POINTER(ctypes.c_longlong), dp, ip, ip, ip, ctypes.c_int, ip]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _f(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class VgError(RuntimeError):
    pass


class Context:
    """One device-resident LIO sequence (vg_ctx)."""

    def __init__(self, cconfig, device=0, max_points=2_000_000, max_nodes=0, max_fix_points=0, hash_log2=0):
        self.h = ctypes.c_void_p()
        cap = Capacity(max_points, max_nodes, max_fix_points, hash_log2)
        r = lib().vg_create(ctypes.byref(cconfig), ctypes.byref(cap), device, ctypes.byref(self.h))
        if r != 0:
            raise VgError("vg_create failed (%d)" % r)
        self._fn_step = lib().vg_step_dev

    def _chk(self, r, what):
        if r != 0:
            raise VgError("%s failed (%d): %s" % (what, r, lib().vg_last_error(self.h).decode()))

    def close(self):
        if self.h:
            lib().vg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def downsample(self, xyz, inten, size):
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        inten = np.ascontiguousarray(inten, dtype=np.float32)
        out = np.zeros((max(xyz.shape[0], 1), 5), dtype=np.float32)
        n = ctypes.c_int(0)
        self._chk(lib().vg_downsample(self.h, _f(xyz), _f(inten), xyz.shape[0], size, _f(out), ctypes.byref(n)),
                  "vg_downsample")
        return out[: n.value]

    def downsample_hashed(self, xyz, inten, size, fallback=False):
        """The per-scan pipeline's downsample (test hook): (m,5) in first-occurrence order;
        fallback: with the /2 pass below 2000 voxels (local_mapping.cpp:399-403)."""
        if fallback:
            size = -size
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        inten = np.ascontiguousarray(inten, dtype=np.float32)
        out = np.zeros((max(xyz.shape[0], 1), 5), dtype=np.float32)
        n = ctypes.c_int(0)
        self._chk(lib().vgx_downsample_hashed(self.h, _f(xyz), _f(inten), xyz.shape[0], size, _f(out),
                                              ctypes.byref(n)), "vgx_downsample_hashed")
        return out[: n.value]

    def downsample_close(self, xyz, times, size):
        """down_sampling_close + the init's time sort: (m,4) [x,y,z,t]."""
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        t = None if times is None else np.ascontiguousarray(times, dtype=np.float32)
        out = np.zeros((max(xyz.shape[0], 1), 4), dtype=np.float32)
        n = ctypes.c_int(0)
        self._chk(lib().vg_downsample_close(self.h, _f(xyz), None if t is None else _f(t), xyz.shape[0], size,
                                            _f(out), ctypes.byref(n)), "vg_downsample_close")
        return out[: n.value]

    def seed(self, state):
        s = np.ascontiguousarray(state, dtype=np.float64)
        self._chk(lib().vg_seed(self.h, _d(s)), "vg_seed")

    def step(self, xyz, inten, beg, end, imu):
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        inten = np.ascontiguousarray(inten, dtype=np.float32)
        imu = np.ascontiguousarray(imu, dtype=np.float64).reshape(-1, 7)
        self._chk(lib().vg_step(self.h, _f(xyz), _f(inten), xyz.shape[0], beg, end, _d(imu), imu.shape[0]),
                  "vg_step")

    def step_deskew(self, xyz, inten, times, beg, end, imu):
        """One scan of raw (not motion-compensated) points with per-point times (row f1)."""
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        inten = np.ascontiguousarray(inten, dtype=np.float32)
        times = np.ascontiguousarray(times, dtype=np.float32)
        imu = np.ascontiguousarray(imu, dtype=np.float64)
        self._chk(lib().vg_step_deskew(self.h, _f(xyz), _f(inten), _f(times), xyz.shape[0], beg, end, _d(imu),
                                       imu.shape[0]), "vg_step_deskew")

    def step_deskew_dev(self, dx, dy, dz, di, dt, n, beg, end, imu):
        imu = np.ascontiguousarray(imu, dtype=np.float64)
        self._chk(lib().vg_step_deskew_dev(self.h, ctypes.c_void_p(dx), ctypes.c_void_p(dy), ctypes.c_void_p(dz),
                                           ctypes.c_void_p(di), ctypes.c_void_p(dt), n, beg, end, _d(imu),
                                           imu.shape[0]), "vg_step_deskew_dev")

    def step_dev(self, dx, dy, dz, di, n, beg, end, imu):
        imu = np.ascontiguousarray(imu, dtype=np.float64).reshape(-1, 7)
        self._chk(lib().vg_step_dev(self.h, ctypes.c_void_p(dx), ctypes.c_void_p(dy), ctypes.c_void_p(dz),
                                    ctypes.c_void_p(di), n, beg, end, _d(imu), imu.shape[0]), "vg_step_dev")

    def prep_step_dev(self, dx, dy, dz, di, n, beg, end, imu):
        """vg_step_dev's arguments converted once (a caller that holds its
        scans resident passes them straight on, as a C++ caller would)."""
        imu = np.ascontiguousarray(imu, dtype=np.float64).reshape(-1, 7)
        return (imu, (ctypes.c_void_p(dx), ctypes.c_void_p(dy), ctypes.c_void_p(dz), ctypes.c_void_p(di),
                      ctypes.c_int(n), ctypes.c_double(beg), ctypes.c_double(end), _d(imu), ctypes.c_int(imu.shape[0])))

    def step_prepped(self, p):
        r = self._fn_step(self.h, *p[1])
        if r != 0:
            self._chk(r, "vg_step_dev")

    def state(self):
        s = np.zeros(STATE_LEN)
        self._chk(lib().vg_get_state(self.h, _d(s)), "vg_get_state")
        return s

    def lio_kdtree(self, xyz, state):
        """SURVEY A14 (init-phase LIO against the kNN map): returns (state,
        valid correspondences or -1 when the scan only seeded the map, IEKF
        iterations). xyz: the scan downsampled at max(down_size, 0.5)."""
        xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        st = np.array(state, dtype=np.float64, copy=True)
        v = ctypes.c_int(0)
        it = ctypes.c_int(0)
        self._chk(lib().vg_lio_kdtree(self.h, _f(xyz), xyz.shape[0], _d(st), ctypes.byref(v), ctypes.byref(it)),
                  "vg_lio_kdtree")
        return st, v.value, it.value

    def decode_scan(self, records, fmt):
        """Sensor records -> time-ordered scan: (xyz (m, 3), intensity, time)."""
        buf = np.frombuffer(bytes(records), dtype=np.uint8)
        f = LidarFormat(**{k: fmt.get(k, 3610.0 if k == "omega_l" else 0.0) for k, _ in LidarFormat._fields_})
        n = buf.size // f.stride
        xyz = np.zeros((n + 2, 3), dtype=np.float32)
        it = np.zeros(n + 2, dtype=np.float32)
        tm = np.zeros(n + 2, dtype=np.float32)
        m = ctypes.c_int(0)
        self._chk(lib().vg_decode_scan(self.h, buf.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(f), _f(xyz),
                                       _f(it), _f(tm), ctypes.byref(m)), "vg_decode_scan")
        return xyz[: m.value], it[: m.value], tm[: m.value]

    def kdmap(self):
        n = ctypes.c_int(0)
        self._chk(lib().vg_kdmap_get(self.h, None, 0, ctypes.byref(n)), "vg_kdmap_get")
        out = np.zeros((max(n.value, 1), 3), dtype=np.float32)
        self._chk(lib().vg_kdmap_get(self.h, _f(out), n.value, ctypes.byref(n)), "vg_kdmap_get")
        return out[: n.value]

    def stats(self):
        s = Stats()
        self._chk(lib().vg_get_stats(self.h, ctypes.byref(s)), "vg_get_stats")
        return _stats_dict(s)

    def stats_log(self):
        """Counters of every completed scan (drains the stream once)."""
        n = ctypes.c_int(0)
        self._chk(lib().vg_stats_log(self.h, None, 0, ctypes.byref(n)), "vg_stats_log")
        arr = (Stats * max(n.value, 1))()
        self._chk(lib().vg_stats_log(self.h, arr, n.value, ctypes.byref(n)), "vg_stats_log")
        return [_stats_dict(s) for s in arr[: n.value]]

    def release_far(self, compact=False, census=True):
        """The idle branch's journey release + pool compaction (vg_release_far): [roots erased (-1: none
        pending), nodes erased, roots, nodes, point_fix points held, point_fix arena used]; census=False:
        the caller's idle-branch call (returns at once with -1s when no release is pending)."""
        out = (ctypes.c_longlong * 6)()
        self._chk(lib().vg_release_far(self.h, (1 if compact else 0) | (2 if census else 0), out), "vg_release_far")
        return list(out)

    def window_states(self):
        out = np.zeros((64, STATE_LEN))
        n = ctypes.c_int(0)
        self._chk(lib().vg_window_states(self.h, _d(out), ctypes.byref(n)), "vg_window_states")
        return out[: n.value]

    def trajectory(self):
        n = ctypes.c_int(0)
        self._chk(lib().vg_trajectory(self.h, None, 0, ctypes.byref(n)), "vg_trajectory")
        out = np.zeros((max(n.value, 1), 13))
        self._chk(lib().vg_trajectory(self.h, _d(out), n.value, ctypes.byref(n)), "vg_trajectory")
        return out[: n.value]

    def path(self):
        """pcl_path rows (vg_path): t, R(9), p(3), jour; the window's positions re-written after each BA."""
        n = ctypes.c_int(0)
        self._chk(lib().vg_path(self.h, None, 0, ctypes.byref(n)), "vg_path")
        out = np.zeros((max(n.value, 1), 14))
        self._chk(lib().vg_path(self.h, _d(out), n.value, ctypes.byref(n)), "vg_path")
        return out[: n.value]

    def poll(self):
        """Non-blocking (vg_poll): (scans complete, TUM rows, path rows) absorbed so far."""
        a, b, c = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        self._chk(lib().vg_poll(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "vg_poll")
        return a.value, b.value, c.value

    def set_publish(self, flags):
        self._chk(lib().vg_set_publish(self.h, flags), "vg_set_publish")

    def local_map(self):
        """/map_cmap of the last window BA (vg_local_map): (n, 4) float32 x, y, z, intensity."""
        n = ctypes.c_int(0)
        self._chk(lib().vg_local_map(self.h, None, 0, ctypes.byref(n)), "vg_local_map")
        out = np.zeros((max(n.value, 1), 4), dtype=np.float32)
        self._chk(lib().vg_local_map(self.h, _f(out), n.value, ctypes.byref(n)), "vg_local_map")
        return out[: n.value]

    # ---- stage-level API (reference call order, include/vina_gpu.h) ----
    def scan_load(self, xyz, inten):
        self._xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        self._inten = np.ascontiguousarray(inten, dtype=np.float32)
        self._chk(lib().vg_scan_load(self.h, _f(self._xyz), _f(self._inten), self._xyz.shape[0]), "vg_scan_load")

    def propagate(self, imu, beg, end):
        imu = np.ascontiguousarray(imu, dtype=np.float64).reshape(-1, 7)
        self._chk(lib().vg_propagate(self.h, _d(imu), imu.shape[0], beg, end), "vg_propagate")

    def _int_call(self, fn, name):
        v = ctypes.c_int(0)
        self._chk(fn(self.h, ctypes.byref(v)), name)
        return v.value

    def downsample_scan(self):
        return self._int_call(lib().vg_downsample_scan, "vg_downsample_scan")

    def lio_state_estimation(self):
        return self._int_call(lib().vg_lio_state_estimation, "vg_lio_state_estimation")

    def window_push(self, imu):
        imu = np.ascontiguousarray(imu, dtype=np.float64).reshape(-1, 7)
        self._chk(lib().vg_window_push(self.h, _d(imu), imu.shape[0]), "vg_window_push")

    def cut_voxel_multi(self):
        self._chk(lib().vg_cut_voxel_multi(self.h), "vg_cut_voxel_multi")

    def multi_recut(self):
        return self._int_call(lib().vg_multi_recut, "vg_multi_recut")

    def damping_iter(self):
        return self._int_call(lib().vg_damping_iter, "vg_damping_iter")

    def multi_margi(self):
        self._chk(lib().vg_multi_margi(self.h), "vg_multi_margi")

    def step_end(self):
        self._chk(lib().vg_step_end(self.h), "vg_step_end")

    def win_count(self):
        return self._int_call(lib().vg_win_count, "vg_win_count")

    PROFILE_STAGES = ["downsample", "iekf", "insert", "recut", "ba", "margi", "iekf_total", "ba_solve",
                      "host_propagate", "host_downsample", "host_iekf", "host_push", "host_insert", "host_recut",
                      "host_ba", "host_margi", "k_iekf_clock", "k_ba_solve_clock", "k_rc_clock", "k_ba_hess_clock"]

    def profile(self, on=True, stages=False, every=1, clock=False):
        """on: k_iekf / k_ba_solve launch events (the solve's on every `every`-th
        BA run) and host stage timers; stages: per-stage events as well; clock:
        the in-kernel clocks of k_iekf / k_ba_solve (kernel-only time, graphs
        kept; replaces the solve's events)."""
        flags = (1 if on else 0) | (2 if stages else 0) | (4 if clock else 0) | ((max(1, min(255, every)) & 0xff) << 8)
        self._chk(lib().vg_profile(self.h, flags), "vg_profile")

    def profile_read(self):
        out = {}
        for i, name in enumerate(self.PROFILE_STAGES):
            ms = ctypes.c_double(0)
            n = ctypes.c_int(0)
            self._chk(lib().vg_profile_read(self.h, i, ctypes.byref(ms), ctypes.byref(n)), "vg_profile_read")
            out[name] = {"ms": ms.value, "launches": n.value}
        return out

    def shard_rccl(self, rank, world, uid):
        """Spatial-tile sharding over `world` contexts, RCCL inside the library."""
        self._chk(lib().vg_shard_rccl(self.h, rank, world, uid), "vg_shard_rccl")

    def shard_host(self, rank, world, allreduce):
        """Spatial-tile sharding with a host all-reduce: allreduce(np.ndarray) sums
        the array in place across ranks (e.g. torch.distributed gloo)."""
        def cb(buf, count, dtype, user):
            try:
                ct = ctypes.c_double if dtype == 0 else ctypes.c_int32
                arr = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ct)), shape=(count,))
                allreduce(arr)
                return 0
            except Exception:  # noqa: BLE001 - reported to the library as a failed exchange
                import traceback
                traceback.print_exc()
                return 1
        self._cb = HOST_ALLREDUCE(cb)  # keep alive
        self._chk(lib().vg_shard_host(self.h, rank, world, self._cb, None), "vg_shard_host")

    def stream(self):
        return lib().vg_stream(self.h)

    # ---- test-only knobs (vgx_*, not part of include/vina_gpu.h)
    def debug(self, key, value):
        self._chk(lib().vgx_debug(self.h, key, value), "vgx_debug")

    def memo_probe(self):
        """The IEKF memo at internal nodes' centre planes (vgx_memo_probe):
        samples, mismatches of OctoTree::inside's box, mismatches of the descent
        region k_iekf uses, samples whose plane separates two leaves."""
        out = np.zeros(4, np.int32)
        self._chk(lib().vgx_memo_probe(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int))), "vgx_memo_probe")
        return [int(v) for v in out]

    def roots(self):
        """Every root voxel of the device map (vgx_roots): {(x, y, z): (jour stamp,
        flags 1 in slide | 2 isexist, subtree nodes, point_fix points)} — the
        shape of the oracle's Pipeline.roots()."""
        def call(key, jour, flags, nodes, nfix, cap):
            n = ctypes.c_int(0)
            self._chk(lib().vgx_roots(self.h, key, jour, flags, nodes, nfix, cap, ctypes.byref(n)), "vgx_roots")
            return n.value
        n = call(None, None, None, None, None, 0)
        key = np.zeros((max(n, 1), 3), dtype=np.int64)
        jour = np.zeros(max(n, 1))
        arr = [np.zeros(max(n, 1), dtype=np.int32) for _ in range(3)]
        ip = ctypes.POINTER(ctypes.c_int)
        m = call(key.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), _d(jour), *[a.ctypes.data_as(ip) for a in arr], n)
        assert m == n, (m, n)
        return {tuple(int(v) for v in key[i]): (float(jour[i]), int(arr[0][i]), int(arr[1][i]), int(arr[2][i]))
                for i in range(n)}

    def capture_arm(self):
        """Capture the next LM run's first Hessian pass (vgx_debug 5)."""
        self.debug(5, 1)

    def capture_get(self):
        n = ctypes.c_int(0)
        self._chk(lib().vgx_ba_capture(self.h, None, 0, ctypes.byref(n)), "vgx_ba_capture")
        out = np.zeros(max(n.value, 1))
        self._chk(lib().vgx_ba_capture(self.h, _d(out), n.value, ctypes.byref(n)), "vgx_ba_capture")
        return out[: n.value]

    def ba_solve(self, A, b):
        """k_ba_solve on a (15W-15)-unknown symmetric system in identity pivot order."""
        A = np.ascontiguousarray(A, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.zeros(b.shape[0])
        self._chk(lib().vgx_ba_solve(self.h, _d(A), _d(b), _d(x)), "vgx_ba_solve")
        return x


class Sync:
    """sync_packages (replay side): host packager of scans and IMU samples."""

    def __init__(self, point_notime=0):
        self.h = lib().vg_sync_create(point_notime)

    def close(self):
        if self.h:
            lib().vg_sync_destroy(self.h)
            self.h = None

    def push_scan(self, header_time, last_point_time, scan_id):
        lib().vg_sync_push_scan(self.h, header_time, last_point_time, scan_id)

    def push_imu(self, imu7):
        a = np.ascontiguousarray(imu7, dtype=np.float64)
        lib().vg_sync_push_imu(self.h, _d(a))

    def pop(self, cap=4096):
        """(scan_id, beg, end, imu (m, 7)), "dropped" (a scan with <= 4 IMU samples was
        consumed), or None (wait for data); VgError when the IMU stream ran dry."""
        sid, m, rd = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        b, e = ctypes.c_double(0), ctypes.c_double(0)
        out = np.zeros((cap, 7))
        r = lib().vg_sync_pop(self.h, ctypes.byref(sid), ctypes.byref(b), ctypes.byref(e), _d(out), cap,
                              ctypes.byref(m), ctypes.byref(rd))
        if r != 0:
            raise VgError("vg_sync_pop: IMU stream ran dry (%d)" % r)
        if rd.value < 0:
            return "dropped"
        return (sid.value, b.value, e.value, out[: m.value].copy()) if rd.value else None


class Multi:
    """Multi-sequence mode (vg_multi_*): B contexts stepped together, one
    native worker thread each."""

    def __init__(self, contexts, spin_us=20, sleep_us=20):
        self.contexts = list(contexts)
        arr = (ctypes.c_void_p * len(self.contexts))(*[c.h.value for c in self.contexts])
        self.h = lib().vg_multi_create(arr, len(self.contexts), spin_us, sleep_us)
        if not self.h:
            raise VgError("vg_multi_create failed")
        self._keep = []

    def step_dev(self, scans):
        """scans: per context (d_x, d_y, d_z, d_intensity, d_time or 0, n, beg, end, imu (m,7) float64)."""
        B = len(self.contexts)
        arr = (ScanDev * B)()
        keep = []
        for b, (x, y, z, i, t, n, beg, end, imu) in enumerate(scans):
            imu = np.ascontiguousarray(imu, dtype=np.float64).reshape(-1, 7)
            keep.append(imu)
            arr[b] = ScanDev(x, y, z, i, t or None, n, beg, end, _d(imu), imu.shape[0])
        r = lib().vg_multi_step_dev(self.h, arr)
        if r != 0:
            lib().vg_multi_sync(self.h)  # the workers are idle before their error strings are read
            raise VgError("vg_multi_step_dev failed (%d): %s" % (
                r, "; ".join(lib().vg_last_error(c.h).decode() for c in self.contexts)))

    def set_active(self, cap):
        """At most `cap` sequences on the device at once (vg_multi_set_active)."""
        r = lib().vg_multi_set_active(self.h, int(cap))
        if r != 0:
            raise VgError("vg_multi_set_active failed (%d)" % r)

    def sync(self):
        r = lib().vg_multi_sync(self.h)
        if r != 0:
            raise VgError("vg_multi_sync failed (%d)" % r)

    def close(self):
        if self.h:
            lib().vg_multi_destroy(self.h)
            self.h = None

