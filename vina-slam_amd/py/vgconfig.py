"""Hot-path parameter sets (the reference's ROS 2 YAML keys) -> C config structs.

Defaults follow src/platform/ros2/node.cpp:52-291 (declare_parameter defaults);
min_point is hard-coded {20,20,15,10} (node.cpp:219) and max_points = 100
(octree.cpp:70). plane_eigen_value_thre is passed as written in the YAML; both
the oracle and the product invert it internally (node.cpp:256-259).
"""
import ctypes
import os

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
CONFIG_DIR = os.path.join(os.path.dirname(HERE), "configs")

DEFAULTS = {
    "General": {"blind": 0.1, "extrinsic_tran": [0.0] * 3, "extrinsic_rota": [1, 0, 0, 0, 1, 0, 0, 0, 1], "if_BA": 0},
    "Odometry": {"cov_gyr": 0.1, "cov_acc": 0.1, "rdw_gyr": 1e-4, "rdw_acc": 1e-4, "down_size": 0.1,
                 "dept_err": 0.02, "beam_err": 0.05, "voxel_size": 1.0, "min_eigen_value": 0.0025},
    "LocalBA": {"win_size": 10, "max_layer": 2, "cov_gyr": 0.1, "cov_acc": 0.1, "rdw_gyr": 1e-4, "rdw_acc": 1e-4,
                "plane_eigen_value_thre": [1, 1, 1, 1], "imu_coef": 1e-4, "thread_num": 5},
}


class CConfig(ctypes.Structure):
    """Field-for-field the layout of both orc_config (oracle/vina_oracle.h) and
    vg_config (include/vina_gpu.h)."""
    _fields_ = [
        ("voxel_size", ctypes.c_double), ("down_size", ctypes.c_double), ("min_eigen_value", ctypes.c_double),
        ("plane_eigen_value_thre", ctypes.c_double * 4), ("min_point", ctypes.c_double * 4),
        ("dept_err", ctypes.c_double), ("beam_err", ctypes.c_double), ("imu_coef", ctypes.c_double),
        ("ba_cov_gyr", ctypes.c_double), ("ba_cov_acc", ctypes.c_double), ("ba_rdw_gyr", ctypes.c_double),
        ("ba_rdw_acc", ctypes.c_double),
        ("odo_cov_gyr", ctypes.c_double), ("odo_cov_acc", ctypes.c_double), ("odo_rdw_gyr", ctypes.c_double),
        ("odo_rdw_acc", ctypes.c_double),
        ("ext_R", ctypes.c_double * 9), ("ext_t", ctypes.c_double * 3),
        ("max_layer", ctypes.c_int), ("max_points", ctypes.c_int), ("win_size", ctypes.c_int),
        ("thread_num", ctypes.c_int), ("if_BA", ctypes.c_int), ("use_threads", ctypes.c_int),
        ("vnc_prep", ctypes.c_int), ("cold_start", ctypes.c_int), ("scale_gravity", ctypes.c_double),
        ("release_dis", ctypes.c_int), ("pad_r", ctypes.c_int),
    ]


def load(name_or_path):
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(CONFIG_DIR, name_or_path if name_or_path.endswith(".yaml") else name_or_path + ".yaml")
    with open(path) as f:
        y = yaml.safe_load(f) or {}
    out = {}
    for sec, d in DEFAULTS.items():
        out[sec] = dict(d)
        out[sec].update((y.get(sec) or {}))
    return out


def to_c(p, use_threads=1, vnc_prep=1, scale_gravity=1.0, cold_start=0, release_dis=0):
    g, o, b = p["General"], p["Odometry"], p["LocalBA"]
    c = CConfig()
    c.voxel_size = o["voxel_size"]
    c.down_size = o["down_size"]
    c.min_eigen_value = o["min_eigen_value"]
    for i in range(4):
        c.plane_eigen_value_thre[i] = b["plane_eigen_value_thre"][i]
        c.min_point[i] = (20, 20, 15, 10)[i]
    c.dept_err, c.beam_err = o["dept_err"], o["beam_err"]
    c.imu_coef = b["imu_coef"]
    c.ba_cov_gyr, c.ba_cov_acc, c.ba_rdw_gyr, c.ba_rdw_acc = b["cov_gyr"], b["cov_acc"], b["rdw_gyr"], b["rdw_acc"]
    c.odo_cov_gyr, c.odo_cov_acc, c.odo_rdw_gyr, c.odo_rdw_acc = o["cov_gyr"], o["cov_acc"], o["rdw_gyr"], o["rdw_acc"]
    for i in range(9):
        c.ext_R[i] = g["extrinsic_rota"][i]
    for i in range(3):
        c.ext_t[i] = g["extrinsic_tran"][i]
    c.max_layer = b["max_layer"]
    c.max_points = 100
    c.win_size = b["win_size"]
    c.thread_num = b["thread_num"]
    c.if_BA = int(g["if_BA"])
    c.use_threads = use_threads
    c.vnc_prep = vnc_prep
    c.scale_gravity = scale_gravity
    c.cold_start = cold_start
    c.release_dis = release_dis  # 0: the reference's 700 (local_mapping.cpp:324)
    return c
