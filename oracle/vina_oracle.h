/* ORACLE — test infrastructure only. C API of the CPU restatement of the
 * VINA-SLAM per-scan hot path, loaded by tests/ (ctypes), smoke() and the
 * bench.py cpu_baseline leg. The product library never includes this file.
 *
 * State vector layout used by orc_seed/orc_get_state (250 doubles):
 *   [0] t, [1..9] R row-major, [10..12] p, [13..15] v, [16..18] bg,
 *   [19..21] ba, [22..24] g, [25..249] cov 15x15 row-major
 * (the reference's IMUST, include/vina_slam/core/types.hpp:43-113). */
#pragma once
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_config {
  double voxel_size;              /* Odometry.voxel_size        node.cpp:192 */
  double down_size;               /* Odometry.down_size         node.cpp:183 */
  double min_eigen_value;         /* Odometry.min_eigen_value   node.cpp:198 */
  double plane_eigen_value_thre[4]; /* LocalBA.plane_eigen_value_thre, as in YAML (inverted internally) */
  double min_point[4];            /* hard-coded {20,20,15,10}   node.cpp:219 */
  double dept_err, beam_err;      /* Odometry.dept_err/beam_err node.cpp:186-190 */
  double imu_coef;                /* LocalBA.imu_coef           node.cpp:247 */
  double ba_cov_gyr, ba_cov_acc, ba_rdw_gyr, ba_rdw_acc; /* LocalBA.* node.cpp:228-238 */
  double odo_cov_gyr, odo_cov_acc, odo_rdw_gyr, odo_rdw_acc; /* Odometry.* node.cpp:171-181 */
  double ext_R[9], ext_t[3];      /* General.extrinsic_rota/tran node.cpp:78-82 */
  int max_layer;                  /* LocalBA.max_layer */
  int max_points;                 /* octree.cpp:70 (100) */
  int win_size;                   /* LocalBA.win_size */
  int thread_num;                 /* LocalBA.thread_num (semantic: partition/quirks) */
  int if_BA;                      /* General.if_BA (default 0) */
  int use_threads;                /* oracle only: spawn real std::threads */
  int vnc_prep;                   /* oracle only: run the dead VNC prep (cost fidelity) */
  int cold_start;                 /* 1: the reference's initialisation (IMU_init, kd-tree LIO, motion_init;
                                     SURVEY row f2) instead of a seeded state */
  double scale_gravity;           /* IMUEKF::scale_gravity = imupre_scale_gravity (imu_ekf.cpp:51,
                                     imu_preintegration.cpp:51); 0 is read as 1 */
  int release_dis;                /* journey release distance (local_mapping.cpp:324, 700 m); 0 is read as 700 */
  int pad_r;
} orc_config;

typedef struct orc_stats {
  int n_raw, n_ds, iekf_iters, iekf_matches[4];
  int roots_new, n_slide, n_factors, ba_iters, degenerate;
  int plane_updates, fix_full; /* margi branch counters (octree.cpp:441-446, 461-469) */
  int init_phase;   /* cold start: 0 steady state, 1 IMU_init consumed the scan, 2 init-window scan
                       (kd-tree LIO), 3 motion_init succeeded (the scan ran the window tail too),
                       4 motion_init failed (system_reset) */
  int init_rounds;  /* motion_init rounds run on this scan */
  int init_valid;   /* init-window scan: kd-tree LIO correspondences (-1 = map seeded) */
} orc_stats;

void orc_voxel_key_d(const double* xyz, int n, double size, int64_t* out);
size_t orc_voxel_hash(int64_t x, int64_t y, int64_t z);
int orc_downsample(const float* xyz, const float* inten, int n, double size, float* out_xyzic, int* n_out);
int orc_down_sampling_close(const float* xyz, const float* times, int n, double size, float* out_xyzt);
void orc_calc_body_var(const double* p, double range_inc, double degree_inc, double* pnt_out, double* var_out);
void orc_eig3(const double* A, double* w, double* V);
void orc_inverse15(const double* A, double* out);
void orc_ldlt_solve(const double* A, const double* b, int n, double* x);
void orc_so3(const double* w, double* R_out, double* log_out, double* jr_out, double* jrinv_out);

void* orc_create(const orc_config* c);
void orc_destroy(void* h);
void orc_seed(void* h, const double* state);
void orc_get_state(void* h, double* state);
int orc_step(void* h, const float* xyz, const float* inten, int n, double beg, double end, const double* imu, int m,
             double* timing);
void orc_get_stats(void* h, orc_stats* s);
/* The idle branch's journey release (local_mapping.cpp:317-344): out[0] roots
 * erased (-1: jour has not advanced since the last call), [1] nodes erased,
 * [2] roots, [3] nodes, [4] point_fix points after it. orc_jour: jour. */
void orc_release_far(void* h, long long* out);
double orc_jour(void* h);
/* test hook: every root voxel (key x/y/z, jour stamp, flags 1: in the slide map |
 * 2: isexist, subtree nodes, point_fix points); returns the root count */
int orc_roots(void* h, long long* key, double* jour, int* flags, int* nodes, int* nfix, int cap);
/* orc_step with IMUEKF::motion_blur's per-point deskew first (imu_ekf.cpp:114-144);
 * times: per-point offset from beg in seconds (the reference's curvature), ascending. */
int orc_step_deskew(void* h, const float* xyz, const float* inten, const float* times, int n, double beg, double end,
                    const double* imu, int m, double* timing);
/* propagation + deskew only, in place (returns the number of IMU poses) */
int orc_deskew_only(void* h, float* xyz, const float* times, int n, double beg, double end, const double* imu, int m);
/* Spatial-tile sharding of the restatement: this pipeline keeps
 * only the root voxels of tiles owned by `rank`; fn sums n doubles in place
 * over the ranks at every exchange point. Call before the first step. */
void orc_shard(void* h, int rank, int world, int (*fn)(double* buf, int n, void* user), void* user);
int orc_traj_len(void* h);
void orc_get_traj(void* h, double* out);
int orc_path_len(void* h);
void orc_get_path(void* h, double* out);
int orc_local_map(void* h, int all, float* out, int cap);
int orc_window_states(void* h, double* out);
/* test hook: the next LM run's first divide_thread pass (optimizers.cpp:181-245)
 * as [6W x 6W LiDAR Hessian summed over the factors (row-major), 6W gradient,
 * residual, then per IMU factor: J^T C J 30x30, J^T C r 30, r^T C r] */
void orc_capture_arm(void* h);
/* known-answer hooks (oracle/kat.cpp): the restatement's p2p Jacobian, one
 * LidarFactor voxel and one IMU_PRE factor on caller-given inputs */
void orc_kat_p2p(const double* R9, const double* p3, const double* pnt3, const double* n3, const double* c3,
                 double* r, double* j6);
void orc_kat_lidar_factor(int W, const double* clu, const double* fix, const double* poses, double* res,
                          double* jac, double* hess);
double orc_kat_imu(const double* imu, int m, const double* bias0, const double* dbias, const double* x1,
                   const double* x2, const double* noise, double sg, double* rr, double* joc);
int orc_capture_get(void* h, double* out, int cap);

/* VINA_SLAM::lio_state_estimation_kdtree (odometry.cpp:267-439) on
 * the context's x_curr and its initialisation map; valid = -1 when the scan
 * only seeded the map (< 100 points). Helpers: the ColPivHouseholderQR solve
 * and the exact kNN it restates. */
int orc_lio_kdtree(void* h, const float* xyz, int n, int* valid, int* iters);
int orc_kdmap_size(void* h);
void orc_kdmap_get(void* h, float* xyz);
void orc_qr_solve(const double* A, int m, const double* b, double* x);
int orc_knn(const float* pts, int np, const float* q, int k, int* idx, float* sq);

/* sensor decoders + pcl_handler (kind = LID_TYPE order); out5 =
 * x, y, z, intensity, time per point (capacity cap); returns the count */
int orc_decode_scan(const void* rec, int n, int kind, int stride, int off_x, int off_y, int off_z, int off_i,
                    int off_t, int filter_num, double blind, double omega_l, double time_base, float* out5, int cap);

#ifdef __cplusplus
}
#endif
