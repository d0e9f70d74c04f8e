/* vina_gpu.h — C-ABI of the MI355X-native VINA-SLAM per-scan LIO hot path.
 *
 * The reference (SheepYang666/VINA-SLAM) has no plugin/FFI layer: its hot path
 * is a plain C++ API called from the odometry thread. Each entry point below
 * replaces one of those calls (reference file:line cited); a C++ caller shaped
 * like src/pipeline/local_mapping.cpp binds them directly.
 *
 * Conventions
 *  - Every function returns int: 0 = ok, < 0 = error (VG_E_*); vg_last_error()
 *    gives text. Nothing calls exit() (the reference does: octree.cpp:407,
 *    optimizers.cpp:70).
 *  - Pointers without a _dev suffix are caller-owned HOST buffers; *_dev entry
 *    points take device pointers already resident in HBM.
 *  - Calls are synchronous with respect to the host unless stated; work inside
 *    is ordered on the context's HIP stream.
 *  - State vector (250 doubles), the reference's IMUST (types.hpp:43-113):
 *      [0] t, [1..9] R row-major, [10..12] p, [13..15] v, [16..18] bg,
 *      [19..21] ba, [22..24] g, [25..249] cov 15x15 row-major.
 *  - IMU samples: m rows of 7 doubles [t, gx, gy, gz, ax, ay, az]
 *    (sensor_msgs::Imu subset, m/s^2 and rad/s).
 *  - A context runs on three HIP streams and hands work between them through
 *    device flags that kernels poll, which needs kernels of different streams
 *    to run concurrently. Where they may not, the context uses event waits
 *    instead: serialised-kernel runs (AMD_SERIALIZE_KERNEL, VG_SERIAL_KERNELS=1,
 *    or rocprofv3 --pmc, detected at vg_create), and several live contexts on
 *    one device in one process (their streams would share the device's
 *    hardware queues; use vg_multi_* for several sequences). A hand-off that
 *    still times out (~1 s) fails the scan with VG_E_STATE; device errors are
 *    sticky: every later call returns them until vg_reset.
 */
#ifndef VINA_GPU_H
#define VINA_GPU_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define VG_OK 0
#define VG_E_ARG (-1)
#define VG_E_HIP (-2)
#define VG_E_CAPACITY (-3)
#define VG_E_RANGE (-4)
#define VG_E_STATE (-5)

#define VG_STATE_LEN 250

/* Hot-path parameters: the reference's ROS 2 keys (node.cpp:52-291). */
typedef struct vg_config {
  double voxel_size;                /* Odometry.voxel_size (node.cpp:192) */
  double down_size;                 /* Odometry.down_size (node.cpp:183) */
  double min_eigen_value;           /* Odometry.min_eigen_value (node.cpp:198) */
  double plane_eigen_value_thre[4]; /* LocalBA.plane_eigen_value_thre as written in YAML; inverted internally (node.cpp:256-259) */
  double min_point[4];              /* {20,20,15,10} (node.cpp:219) */
  double dept_err, beam_err;        /* Odometry.dept_err / beam_err (node.cpp:186-190) */
  double imu_coef;                  /* LocalBA.imu_coef (node.cpp:247) */
  double ba_cov_gyr, ba_cov_acc, ba_rdw_gyr, ba_rdw_acc;     /* LocalBA.* -> noiseMeas/noiseWalk (node.cpp:262-265) */
  double odo_cov_gyr, odo_cov_acc, odo_rdw_gyr, odo_rdw_acc; /* Odometry.* -> IMUEKF (node.cpp:211-214) */
  double ext_R[9], ext_t[3];        /* General.extrinsic_rota / extrinsic_tran (node.cpp:78-82, 217-218) */
  int max_layer;                    /* LocalBA.max_layer */
  int max_points;                   /* octree.cpp:70 (100) */
  int win_size;                     /* LocalBA.win_size */
  int thread_num;                   /* LocalBA.thread_num: only its semantic quirks (voxel_map.cpp:96-97, local_mapping.cpp:27,93) */
  int if_BA;                        /* General.if_BA (default 0, node.cpp:96) */
  int reserved0, reserved1;
  /* 1: cold start — the reference's initialisation (node.cpp:293-366, SURVEY
   * row f2) runs on the first scans: IMU_init (+ gravity scale), then per scan
   * the kd-tree LIO (A14) until the window is full, then motion_init (map
   * rounds with the gravity-optimising BA, align_gravity, gravity-norm and
   * degeneracy checks; failure -> system_reset); the steady state follows.
   * Scans given with per-point times (vg_step_deskew*) are deskewed as the
   * reference's; without, every point is at pcl_end_time. Only the whole-scan
   * entry points (vg_step*) may be used until vg_stats::init_phase reports 3.
   * 0: start from vg_seed's state on an empty map. */
  int cold_start;
  /* IMUEKF::scale_gravity / imupre_scale_gravity (ekf_imu.hpp:27,
   * imu_preintegration.cpp:3): every accelerometer sample is multiplied by it
   * in the propagation (imu_ekf.cpp:51) and the preintegration
   * (imu_preintegration.cpp:51). 1 for IMUs reporting m/s^2; the reference
   * sets G_m_s2 = 9.8 when the static mean |acc| < 2 (IMU in g, e.g. Livox
   * Mid-360; imu_ekf.cpp:182-185, node.cpp:309). vg_imu_init derives it the
   * same way. 0 is read as 1. */
  double scale_gravity;
  /* Journey release distance in metres (local_mapping.cpp:324: roots whose
   * jour stamp is >= 700 behind are erased, vg_release_far); 0 is read as 700. */
  int release_dis;
  int pad_r;
} vg_config;

/* Capacities of the device-resident map (HBM). Zero fields take defaults. */
typedef struct vg_capacity {
  int max_points_per_scan;   /* raw points per scan (default 2,000,000) */
  int max_nodes;             /* octree nodes (default 4,000,000) */
  int max_fix_points;        /* point_fix arena, points (default 16,000,000) */
  int hash_log2;             /* root voxel hash slots = 2^hash_log2 (default 23) */
} vg_capacity;

/* Per-scan counters (SURVEY §8(d) byte model inputs). */
typedef struct vg_stats {
  int n_raw, n_ds, iekf_iters, iekf_matches[4];
  int roots_new, n_slide, n_factors, ba_iters, degenerate;
  int nodes_used, fix_used;
  int plane_updates; /* margi: OctoTree::plane_update calls this scan (octree.cpp:441-446) */
  int fix_full;      /* margi: leaves past max_points, pcr_fix.N >= max_points (octree.cpp:461-469) */
  /* SURVEY 8(d) byte-model inputs: distinct plane records read per IEKF
   * iteration (P_k; counted in vg_profile's per-stage pass only, else 0),
   * leaves the insert touched (V_ins), LM Hessian passes (I_H) */
  int iekf_planes[4];
  int v_ins;
  int ba_hess;
  /* cold start (vg_config::cold_start): 0 steady state, 1 IMU_init consumed
   * the scan, 2 initialisation-window scan (kd-tree LIO), 3 motion_init
   * succeeded on this scan (which then ran the window tail too), 4 motion_init
   * failed (system_reset); motion_init rounds run on this scan; the kd-tree
   * LIO's valid correspondences (-1: the scan seeded the map) */
  int init_phase, init_rounds, init_valid;
  /* points the IEKF point loop processed, summed over the executed iterations
   * (sharded mode, world > 1: this rank's kept points, map.hip k_keep_*) */
  int iekf_points;
} vg_stats;

typedef struct vg_ctx vg_ctx;
typedef int (*vg_host_allreduce_fn)(void* buf, int count, int dtype, void* user);

/* Context lifecycle. Replaces the VINA_SLAM members surf_map, surf_map_slide,
 * sws, x_buf, pvec_buf, imu_pre_buf (node.hpp:34-70). device = HIP ordinal. */
int vg_create(const vg_config* cfg, const vg_capacity* cap, int device, vg_ctx** out);
int vg_destroy(vg_ctx* ctx);
const char* vg_last_error(const vg_ctx* ctx);
/* Drop the map and window; replaces VINA_SLAM::system_reset (node.cpp:368-408). */
int vg_reset(vg_ctx* ctx);

/* A1 — down_sampling_voxel (include/vina_slam/core/point_utils.hpp:7-44).
 * xyz: n x 3 floats (AoS), intensity: n floats (may be NULL).
 * out_xyzic: n x 5 floats [x, y, z, intensity(first point), count] in
 * ascending voxel-key order (the reference emits unordered_map order; the SET
 * is identical, bit-for-bit). Returns the voxel count in *n_out. */
int vg_downsample(vg_ctx* ctx, const float* xyz, const float* intensity, int n, double voxel_size,
                  float* out_xyzic, int* n_out);
/* f2 — down_sampling_close (include/vina_slam/core/point_utils.hpp:46-113) +
 * the time sort of VINA_SLAM::initialization (node.cpp:337-345): per voxel the
 * input point nearest the float mean of the voxel's points. time: n floats
 * (may be NULL: every point at time 0). out_xyzt: n x 4 floats [x, y, z, time]
 * sorted by time; equal times in ascending voxel-key order (the reference
 * std::sorts its unordered_map order, leaving their order unspecified).
 * Synchronous; drains the pipeline first (diagnostic / test entry point). */
int vg_downsample_close(vg_ctx* ctx, const float* xyz, const float* time, int n, double voxel_size, float* out_xyzt,
                        int* n_out);

/* Per-scan pipeline — the steady-state branch of
 * VINA_SLAM::thd_odometry_localmapping (local_mapping.cpp:389-547):
 * IMU propagation (imu_ekf.cpp:28-94) -> downsample (+ /2 fallback) ->
 * var_init -> IEKF (odometry.cpp:64-255) -> pvec_update -> cut_voxel_multi ->
 * multi_recut + tras_opt -> [win full] LI_BA damping_iter -> multi_margi -> slide.
 * vg_seed sets x_curr (the output of initialisation). */
int vg_seed(vg_ctx* ctx, const double* state);
int vg_step(vg_ctx* ctx, const float* xyz, const float* intensity, int n, double pcl_beg_time,
            double pcl_end_time, const double* imu, int m);
/* Same, with the scan already in HBM as SoA x/y/z/intensity device arrays. */
int vg_step_dev(vg_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, const float* d_intensity, int n,
                double pcl_beg_time, double pcl_end_time, const double* imu, int m);
/* vg_step / vg_step_dev return once the scan is ENQUEUED: the device runs it
 * asynchronously (the host waits only for device-side counts it needs, without
 * draining the stream). Every query below completes the outstanding work first.
 * vg_step / vg_step_deskew copy the caller's host arrays into one of two pinned
 * in-flight slots before returning (the caller may reuse them at once); the
 * H2D copy and the SoA unpack run on the device ahead of the scan's kernels.
 * vg_step_dev / vg_step_deskew_dev read the caller's device arrays while the
 * scan runs: keep them unchanged until a later query (vg_get_state, vg_get_stats, ...) returns. */
/* SURVEY row f1 — the same scan step with IMUEKF::motion_blur's per-point
 * deskew (imu_ekf.cpp:114-144) on the device first: `time` holds each point's
 * offset from pcl_beg_time in seconds (the reference's `curvature` field),
 * ascending (the reference's time-sorted cloud). The propagation records the
 * IMU poses; one lane per point moves it into the LiDAR frame at
 * pcl_end_time. Inputs as vg_step / vg_step_dev. */
int vg_step_deskew(vg_ctx* ctx, const float* xyz, const float* intensity, const float* time, int n,
                   double pcl_beg_time, double pcl_end_time, const double* imu, int m);
int vg_step_deskew_dev(vg_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, const float* d_intensity,
                       const float* d_time, int n, double pcl_beg_time, double pcl_end_time, const double* imu,
                       int m);
/* SURVEY row A14 — VINA_SLAM::lio_state_estimation_kdtree (odometry.cpp:267-439),
 * the initialisation-phase LIO (node.cpp:317). xyz: the scan downsampled at
 * max(down_size, 0.5), raw LiDAR frame, n x 3 floats (var_init applies the
 * extrinsic). state: 250 doubles (vg_get_state layout), updated in place.
 * While the context's init map holds fewer than 100 points the scan only seeds
 * it (*valid = -1, *iters = 0); otherwise up to 4 IEKF iterations against the
 * exact 5 nearest map points (device hashed grid in place of the kd-tree,
 * plane fit by column-pivoting Householder QR as colPivHouseholderQr), then the
 * registered scan is appended and the map re-downsampled at 0.5 m.
 * *valid: correspondences of the last iteration. vg_reset clears the map.
 * Synchronous; completes outstanding work first. */
int vg_lio_kdtree(vg_ctx* ctx, const float* xyz, int n, double* state, int* valid, int* iters);
/* the init map (float xyz, n x 3, key order of its last downsample): *n = its
 * size; up to cap points copied when xyz != NULL */
int vg_kdmap_get(vg_ctx* ctx, float* xyz, int cap, int* n);
/* SURVEY row f3 — sensor decode (LidarPointCloudDecoder, lidar_pointcloud_decoder.cpp:21-240)
 * and pcl_handler's scan preparation (lidar_decoder.cpp:7-43): per record the
 * xyz / intensity / per-point time of the sensor format, the point_filter_num
 * stride and blind test, then ascending time order and the tail beyond 0.11 s
 * dropped (an empty result becomes the reference's two dummy points).
 * records: n little-endian records of `stride` bytes; offsets are byte offsets
 * of the fields, -1 when absent. Field types per kind (the reference's point
 * structs): LIVOX x,y,z f32, reflectivity u8, offset_time u32 ns; VELODYNE
 * x,y,z,time f32 (a sweep without usable times takes the yaw-derived time,
 * omega_l deg/s, sequentially on the host as the reference does); OUSTER
 * x,y,z,intensity f32, t u32 ns; HESAI x,y,z,intensity f32, timestamp f64
 * (minus the first record's); ROBOSENSE x,y,z,intensity f32, timestamp f64
 * (minus time_base, the header stamp; blind on x,y only); TARTANAIR x,y,z f32
 * (no filter, time 0). blind in metres (squared as node.cpp:210 does).
 * Outputs (host, capacity n + 2): xyz n_out x 3, intensity, time (s). The
 * time sort is stable (std::sort's order among equal times is unspecified). */
enum { VG_LIVOX = 0, VG_VELODYNE = 1, VG_OUSTER = 2, VG_HESAI = 3, VG_ROBOSENSE = 4, VG_TARTANAIR = 5 };
typedef struct vg_lidar_format {
  int kind;
  int stride;
  int off_x, off_y, off_z, off_intensity, off_time;
  int point_filter_num;
  double blind;
  double omega_l;
  double time_base;
} vg_lidar_format;
int vg_decode_scan(vg_ctx* ctx, const void* records, int n, const vg_lidar_format* fmt, float* xyz, float* intensity,
                   float* time, int* n_out);
/* SURVEY row f3 (replay side) — sync_packages (src/sensor/sync.cpp:18-96) as a
 * host packager, no context: push scans (header time, the last point's time
 * offset after vg_decode_scan, an id) and IMU samples (t, gyr 3, acc 3) in
 * arrival order; vg_sync_pop sets *ready = 1 with one scan's window [beg, end]
 * and its IMU samples (stamped <= end; up to cap copied, *m = count) once an
 * IMU sample newer than end has arrived; *ready = 0: wait for more data;
 * *ready = -1: a scan was consumed and dropped (<= 4 samples, as the
 * reference), pop again. point_notime (Odometry.point_notime) windows scans by
 * consecutive header times. VG_E_STATE: the IMU queue ran dry (the reference
 * exits). */
typedef struct vg_sync vg_sync;
vg_sync* vg_sync_create(int point_notime);
void vg_sync_destroy(vg_sync* s);
int vg_sync_push_scan(vg_sync* s, double header_time, double last_point_time, int scan_id);
int vg_sync_push_imu(vg_sync* s, const double* imu7);
int vg_sync_pop(vg_sync* s, int* scan_id, double* beg, double* end, double* imu7, int cap, int* m, int* ready);
int vg_get_state(vg_ctx* ctx, double* state);
/* The last completed scan's downsampled cloud (body frame, after the deskew;
 * the map path's pl_down, local_mapping.cpp:396-406) as n x 3 floats, up to
 * cap copied, *n = its size: what pub_localtraj moves to the world and
 * publishes on /map_scan (publishers.cpp:65-97). Completes outstanding work. */
int vg_scan_points(vg_ctx* ctx, float* xyz, int cap, int* n);
int vg_get_stats(vg_ctx* ctx, vg_stats* out);
/* Per-scan counters of every completed scan since vg_create / vg_reset, in
 * order: copies min(n, cap) records, *n = total (out may be NULL to query). */
int vg_stats_log(vg_ctx* ctx, vg_stats* out, int cap, int* n);
/* The map's lifetime — the idle branch of thd_odometry_localmapping
 * (local_mapping.cpp:317-344), which the caller runs when it has no package
 * (sync_packages false): once jour has advanced (release_flag, :510-518),
 * every root voxel whose jour stamp is >= vg_config::release_dis (700 m)
 * behind is erased with its subtree (OctoTree::tras_ptr, octree.cpp:597-608).
 * The device then reclaims: erased nodes, point_fix blocks abandoned by
 * growth and the blocks of leaves past max_points (octree.cpp:467-468) are
 * compacted out of the node pool and the point_fix arena (order-preserving;
 * results are unchanged). flags bit 0: compact even without a release; bit
 * 1: report the census (out[2..5]) even without one. The pool is also
 * compacted when over half the arena is abandoned blocks. With flags 0 and no
 * release pending among the scans already published it returns at once (no
 * wait; out[] = -1), so a caller may call it whenever sync_packages comes back
 * empty; otherwise it completes outstanding work first. Between scans only.
 * out (6): [0] roots erased (-1: no release was pending), [1] nodes erased,
 * [2] roots, [3] nodes in the map after it, [4] point_fix points held,
 * [5] point_fix arena used.
 * A root still in surf_map_slide is never erased (the reference would keep a
 * dangling pointer in it; unreachable at 700 m). */
int vg_release_far(vg_ctx* ctx, int flags, long long* out);
/* Window states x_buf (win_count x 250 doubles); returns win_count via *n. */
int vg_window_states(vg_ctx* ctx, double* out, int* n);

/* ---- Stage-level API ------------------------------------------------------
 * The steps vg_step composes, one entry per reference call of the steady-state
 * loop (local_mapping.cpp:389-547), for a caller that keeps the reference's
 * loop shape. Order per scan:
 *   vg_scan_load | vg_scan_bind_dev        deskewed scan -> HBM
 *   vg_propagate                           IMUEKF::process state/cov part (imu_ekf.cpp:28-94)
 *   vg_downsample_scan                     down_sampling_voxel + /2 fallback (point_utils.hpp:7-44; local_mapping.cpp:396-403)
 *   vg_lio_state_estimation                VINA_SLAM::VNC_lio -> LioStateEstimation (odometry.cpp:64-255)
 *   vg_window_push                         x_buf / pvec_buf / IMU_PRE push (local_mapping.cpp:434-441)
 *   vg_cut_voxel_multi                     pvec_update + cut_voxel_multi (point_utils.cpp:54-65; voxel_map.cpp:47-135)
 *   vg_multi_recut                         VINA_SLAM::multi_recut + tras_opt (local_mapping.cpp:144-201)
 *   if win_count >= win_size:
 *     vg_damping_iter   (if if_BA)         LI_BA_Optimizer::damping_iter (optimizers.cpp:430-517)
 *     vg_multi_margi                       x_curr <- x_buf.back(), multi_margi, slide (local_mapping.cpp:499-546)
 *   vg_step_end                            per-scan counters (vg_get_stats)
 * Every call returns VG_E_STATE when issued out of order. */
int vg_scan_load(vg_ctx* ctx, const float* xyz, const float* intensity, int n);
int vg_scan_bind_dev(vg_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, const float* d_intensity,
                     int n);
int vg_propagate(vg_ctx* ctx, const double* imu, int m, double pcl_beg_time, double pcl_end_time);
int vg_downsample_scan(vg_ctx* ctx, int* n_ds);
int vg_lio_state_estimation(vg_ctx* ctx, int* degenerate);
int vg_window_push(vg_ctx* ctx, const double* imu, int m);
int vg_cut_voxel_multi(vg_ctx* ctx);
int vg_multi_recut(vg_ctx* ctx, int* n_factors);
int vg_damping_iter(vg_ctx* ctx, int* lm_iters);
int vg_multi_margi(vg_ctx* ctx);
int vg_step_end(vg_ctx* ctx);
int vg_win_count(vg_ctx* ctx, int* n);

/* The TUM pose file's rows (FileReaderWriter::save_pose_tum, io.cpp:67-77,
 * called at local_mapping.cpp:430): the pose right after the IEKF of every
 * steady-state scan — none for the initialisation's scans (cold start).
 * n rows of 13 doubles [t, R row-major 9, p 3]. Copies min(n, cap) rows;
 * *n = total rows. out may be NULL to query. Completes outstanding work. */
int vg_trajectory(vg_ctx* ctx, double* out, int cap, int* n);

/* pub_localtraj / pub_localmap's path (pcl_path, publishers.cpp:65-131): one
 * row per pub_localtraj call (every stepped scan, the initialisation's
 * included, node.cpp:325 / local_mapping.cpp:427), n rows of 14 doubles
 * [t, R row-major 9, p 3, jour]. After every window BA pub_localmap re-writes
 * the positions of the window's rows with the refined x_buf[i].p
 * (publishers.cpp:121-129, local_mapping.cpp:505); system_reset clears it
 * (node.cpp:403). Completes outstanding work. */
int vg_path(vg_ctx* ctx, double* out, int cap, int* n);

/* Non-blocking: absorb every enqueued scan whose device results are already
 * published (no stream drain, no wait), then report how many scans are
 * complete and how many rows vg_poll_rows can copy. A node publishes from
 * here instead of draining after every scan. Any out-pointer may be NULL. */
int vg_poll(vg_ctx* ctx, int* n_scans, int* n_traj, int* n_path);
/* The rows absorbed so far (after vg_poll; no wait): TUM rows from row
 * traj_from on (at most traj_cap), and the first path_cap path rows. */
int vg_poll_rows(vg_ctx* ctx, double* traj, int traj_from, int traj_cap, double* path, int path_cap);

/* /map_cmap (pub_localmap, publishers.cpp:102-119,130): every third point of
 * the oldest window frame's downsampled cloud at that frame's pose after the
 * BA, x y z intensity per point, computed on the device after each window BA
 * while enabled (vg_set_publish bit 0; off by default: no cost to the scan).
 * Points follow the device's downsample order (first occurrence, DESIGN.md
 * section 3), so "every third" selects from that order. Completes outstanding
 * work; *n = points of the last window BA (0 if none ran while enabled). */
int vg_local_map(vg_ctx* ctx, float* out_xyzi, int cap, int* n);
/* Optional per-scan outputs: bit 0 = the /map_cmap cloud (vg_local_map). */
int vg_set_publish(vg_ctx* ctx, int flags);

/* ---- Spatial-tile sharding (north_star: the voxel map shards by spatial tile
 * across the GPUs of one node, with an all-reduce of the normal equations).
 * One context per GPU runs the SAME sequence; each keeps only the root voxels
 * of its tiles (16^3 root voxels, owner = hash(tile) mod world) and sums only
 * its own points and factors. Per IEKF iteration the 34-value normal-equation
 * block is all-reduced, per LM iteration the 6W x 6W LiDAR Hessian + gradient
 * and the residual; three integer counts keep the reference's thread_num
 * quirks global. State and IMU factors are replicated, so every rank computes
 * the identical trajectory. Call once, before the first scan.
 *   vg_shard_rccl: RCCL communicator inside the library, collectives ordered on
 *                  the context stream (ncclAllReduce, no host synchronisation);
 *                  id128 from vg_rccl_unique_id on rank 0, broadcast by the caller.
 *   vg_shard_host: host callback fn(buf, count, dtype, user) summing `count`
 *                  elements of host memory in place across ranks (dtype 0 =
 *                  double, 1 = int32); the library stages through pinned memory
 *                  and synchronises the stream around each call (tests, CPU-
 *                  mediated transports). */
int vg_rccl_unique_id(void* id128);
int vg_shard_rccl(vg_ctx* ctx, int rank, int world, const void* id128);
int vg_shard_host(vg_ctx* ctx, int rank, int world, vg_host_allreduce_fn fn, void* user);

/* Stage timing with HIP events on the context stream (device time). stage:
 * 0 downsample, 1 IEKF point-loop kernel (k_iekf), 2 map insert, 3 recut +
 * factor extraction, 4 BA, 5 margi, 6 whole IEKF, 7 the LDL^T solve kernel
 * (k_ba_solve); 8..15 the HOST time of the stage calls (enqueue + waits):
 * propagate, downsample, IEKF, window push, insert, recut, BA, margi. `on`: 0 off, 1 the k_iekf and k_ba_solve launches only
 * (stages 1 and 7; cheap enough for a timed region), 3 every stage; bits 8-15
 * (n > 1) time k_ba_solve on every n-th BA run only; bit 2 (4): in-kernel
 * clocks of k_iekf and k_ba_solve (the device's constant-rate wall clock read
 * inside the kernels: kernel-only time of the executed launches, graph replays
 * included, no events in the stream), read as stages 16 (k_iekf), 17
 * (k_ba_solve), 18 (the recut's level kernels k_rc_level0 + k_rc_level, one
 * span per scan) and 19 (k_ba_hess), over the last <= 64 scans.
 * vg_profile resets the accumulators; vg_profile_read returns total ms and the
 * number of intervals. */
int vg_profile(vg_ctx* ctx, int on);
int vg_profile_read(vg_ctx* ctx, int stage, double* total_ms, int* count);

/* HIP stream the context enqueues on (hipStream_t as void*). */
void* vg_stream(vg_ctx* ctx);

/* How the host waits for device results: spin for spin_us, then poll every
 * sleep_us (sleep_us 0: spin only, the default and the lowest latency). Use
 * sleeping polls when several contexts run from their own threads. */
int vg_set_wait_policy(vg_ctx* ctx, int spin_us, int sleep_us);

/* Multi-sequence mode (BASELINE config 5): B independent sequences on one
 * GPU, each in its own context. vg_multi_create starts one native worker
 * thread per context (and sets their wait policy); vg_multi_step_dev queues
 * one scan per sequence (device-resident SoA, as vg_step_dev, or
 * vg_step_deskew_dev when d_time != NULL; the point buffers must stay valid
 * until vg_multi_sync, the IMU samples are copied) and returns — it blocks
 * only when a sequence has 4 scans queued; the workers run free, in order per
 * sequence. vg_multi_sync completes every queued scan. Each sequence's
 * results are exactly those of a lone context. vg_multi_step_dev queues all B
 * scans or none: after a worker's error it returns that status without
 * queuing (call vg_multi_sync before reading vg_last_error of the contexts).
 * With B > 1 the contexts run on one stream each while the multi object
 * exists; vg_multi_destroy gives each back its own stream, downsample stream
 * and the IEKF / margi overlap. Past four sequences they share four streams
 * (sequence b on stream b % 4, one worker thread per stream stepping its
 * sequences one scan each in turn): MI355X time-slices more than about four
 * busy hardware queues, and four shared streams keep B = 8 / 16 at B = 4's
 * rate. The environment variable VG_MULTI_STREAMS = G overrides
 * the count (G <= 0 or G >= B: one stream and one worker per sequence). */
typedef struct vg_scan_dev {
  const float *d_x, *d_y, *d_z, *d_intensity, *d_time;
  int n;
  double pcl_beg_time, pcl_end_time;
  const double* imu; /* host, m x 7 */
  int m;
} vg_scan_dev;
typedef struct vg_multi vg_multi;
vg_multi* vg_multi_create(vg_ctx** ctxs, int B, int spin_us, int sleep_us);
int vg_multi_step_dev(vg_multi* mv, const vg_scan_dev* scans);
/* At most `cap` sequences with device work in flight at once (0 or >= B: no
 * cap): sequence b runs in slot b % cap, one sequence per slot at a time, and
 * waits for its scan's device work before the slot passes on. Past about four
 * hardware queues per process the GPU time-slices them (every kernel >= ~47
 * us at B = 8, same L2 hit rates as B = 4), idle ones included, so pair the
 * cap with GPU_MAX_HW_QUEUES = cap (the B streams then share cap queues, slot
 * by slot). Between steps only (VG_E_STATE). */
int vg_multi_set_active(vg_multi* mv, int cap);
int vg_multi_sync(vg_multi* mv);
void vg_multi_destroy(vg_multi* mv);

#ifdef __cplusplus
}
#endif
#endif /* VINA_GPU_H */
