// vg_replay — C++ driver that keeps the reference's per-scan loop shape
// (VINA_SLAM::thd_odometry_localmapping, local_mapping.cpp:389-547) on top of
// the stage-level C-ABI, reading a flat replay file and writing the TUM pose
// file of FileReaderWriter::save_pose_tum (io.cpp:67-77).
//
// Replay format (little-endian):
//   "VGRPLAY1" | int32 n_scans | vg_config (sizeof) | double seed[250]
//   per scan: double beg, double end, int32 n, int32 m, float xyzi[4n], double imu[7m]
//
// usage: vg_replay <replay.bin> <out_tum.txt> [device]
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../include/vina_gpu.hpp"

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

// Eigen::Quaterniond(R) (the same trace/largest-diagonal branch Eigen uses)
static void quat(const double* R, double q[4]) {
  double t = R[0] + R[4] + R[8];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (R[7] - R[5]) * t;
    q[1] = (R[2] - R[6]) * t;
    q[2] = (R[3] - R[1]) * t;
  } else {
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[i * 4]) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (R[k * 3 + j] - R[j * 3 + k]) * t;
    q[j] = (R[j * 3 + i] + R[i * 3 + j]) * t;
    q[k] = (R[k * 3 + i] + R[i * 3 + k]) * t;
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s replay.bin out_tum.txt [device]\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror("replay");
    return 1;
  }
  char magic[8];
  int nscan = 0;
  vg_config cfg;
  double seed[VG_STATE_LEN];
  if (!rd(f, magic, 8) || memcmp(magic, "VGRPLAY1", 8) != 0 || !rd(f, &nscan, 4) || !rd(f, &cfg, sizeof(cfg)) ||
      !rd(f, seed, sizeof(seed))) {
    fprintf(stderr, "bad replay header\n");
    return 1;
  }
  FILE* out = fopen(argv[2], "w");
  if (!out) {
    perror("out");
    return 1;
  }
  try {
    vg_capacity cap = {0, 0, 0, 0};
    cap.max_points_per_scan = 400000;
    vina_gpu::LioCore lio(cfg, &cap, argc > 3 ? atoi(argv[3]) : 0);
    lio.seed(seed);
    std::vector<float> xyzi, xyz, inten;
    std::vector<double> imu;
    for (int s = 0; s < nscan; s++) {
      double beg, end;
      int n, m;
      if (!rd(f, &beg, 8) || !rd(f, &end, 8) || !rd(f, &n, 4) || !rd(f, &m, 4)) break;
      xyzi.resize((size_t)n * 4);
      imu.resize((size_t)m * 7);
      if (!rd(f, xyzi.data(), xyzi.size() * 4) || !rd(f, imu.data(), imu.size() * 8)) break;
      xyz.resize((size_t)n * 3);
      inten.resize(n);
      for (int i = 0; i < n; i++) {
        xyz[3 * i] = xyzi[4 * i];
        xyz[3 * i + 1] = xyzi[4 * i + 1];
        xyz[3 * i + 2] = xyzi[4 * i + 2];
        inten[i] = xyzi[4 * i + 3];
      }
      // ---- the steady-state branch, call for call ----
      lio.load_scan(xyz.data(), inten.data(), n);
      lio.odom_ekf_process(imu.data(), m, beg, end);
      lio.down_sampling_voxel();
      lio.VNC_lio();
      std::vector<double> x = lio.x_curr();  // save_pose_tum(x_curr), local_mapping.cpp:429-430
      double q[4];
      quat(&x[1], q);
      fprintf(out, "%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", x[0], x[10], x[11], x[12], q[0], q[1], q[2], q[3]);
      lio.push_window(imu.data(), m);
      lio.cut_voxel_multi();
      lio.multi_recut();
      if (lio.win_count() >= cfg.win_size) {
        if (cfg.if_BA == 1) lio.damping_iter();
        lio.multi_margi();
      }
      lio.end_scan();
    }
  } catch (const vina_gpu::Error& e) {
    fprintf(stderr, "vg_replay: %s (code %d)\n", e.what(), e.code);
    fclose(out);
    return 1;
  }
  fclose(out);
  fclose(f);
  return 0;
}
