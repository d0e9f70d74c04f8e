// vina_node_core.hpp — the ROS-free core of the reference's ROS 2 node
// (SURVEY §8 row f4), header-only on the C-ABI (vina_gpu.h):
//   imu_handler / the point-cloud handlers (src/platform/ros2/node.cpp:153-170)
//     -> NodeCore::imu / NodeCore::scan (pcl_handler's decode runs at arrival,
//        lidar_decoder.cpp:7-43, on the device through vg_decode_scan);
//   sync_packages (src/sensor/sync.cpp:18-96) + the odometry thread's per-scan
//     step (local_mapping.cpp:389-547, deskew included) -> NodeCore::spin;
//   ResultOutput::pub_localtraj (publishers.cpp:65-97): the pose after the IEKF
//     (the TF camera_init -> aft_mapped, pub_odom_func 42-63), the path point
//     and the scan moved to the world (/map_scan) -> path() / scan_world();
//   ResultOutput::pub_localmap (publishers.cpp:99-131, local_mapping.cpp:505):
//     the path's window rows re-written with the BA-refined positions (in
//     path()) and the /map_cmap cloud -> local_map();
//   FileReaderWriter::save_pose_tum (io.cpp:67-77) -> tum_rows() / tum_line /
//     write_tum (steady-state scans only, as the reference's file).
// Outputs are refreshed without draining the device pipeline (vg_poll): a
// scan's rows appear once its results are published; scan_world(),
// local_map() and write_tum() complete outstanding work first.
// A ROS 2 wrapper (vina-slam_amd/ros2/vina_node.cpp, built when rclcpp is
// found) only converts messages to these calls and these outputs to messages.
#pragma once
#include <cmath>
#include <cstdio>
#include <map>
#include <string>
#include <vector>
#include "vina_gpu.hpp"

namespace vina_gpu {

struct PoseStamped {
  double t;
  double R[9];  // row-major
  double p[3];
  double q[4];  // x, y, z, w
  double jour = 0;  // path points only: the journey (the PointType's curvature, publishers.cpp:88-92)
};

// Eigen::Quaterniond(const Matrix3d&): the trace branch, else the largest
// diagonal entry's branch
inline void quat_from_R(const double* R, double q[4]) {
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
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (R[k * 3 + j] - R[j * 3 + k]) * t;
    q[j] = (R[j * 3 + i] + R[i * 3 + j]) * t;
    q[k] = (R[k * 3 + i] + R[i * 3 + k]) * t;
  }
}

// one row of the TUM pose file: "t x y z qx qy qz qw", std::fixed, 9 decimals
inline std::string tum_line(const PoseStamped& s) {
  char b[320];
  snprintf(b, sizeof(b), "%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", s.t, s.p[0], s.p[1], s.p[2], s.q[0], s.q[1],
           s.q[2], s.q[3]);
  return b;
}

class NodeCore {
 public:
  // cfg.cold_start = 1 for a run from a bag (the node's initialization,
  // node.cpp:293-366); point_notime as the node's `point_notime` parameter
  NodeCore(const vg_config& cfg, const vg_capacity* cap, const vg_lidar_format& fmt, int point_notime = 0,
           int device = 0)
      : cfg_(cfg), fmt_(fmt), lio_(cfg, cap, device) {
    sync_ = vg_sync_create(point_notime);
    if (!sync_) throw Error(VG_E_ARG, "vg_sync_create");
  }
  ~NodeCore() { vg_sync_destroy(sync_); }
  NodeCore(const NodeCore&) = delete;
  NodeCore& operator=(const NodeCore&) = delete;

  // imu_handler: one sample (stamp, angular velocity, linear acceleration)
  void imu(double t, const double gyr[3], const double acc[3]) {
    const double s[7] = {t, gyr[0], gyr[1], gyr[2], acc[0], acc[1], acc[2]};
    check(vg_sync_push_imu(sync_, s), "vg_sync_push_imu");
  }

  // a point-cloud message: the sensor records and the header stamp; decoded
  // now, as pcl_handler does in the callback. fmt: this message's layout
  // (a PointCloud2's field offsets), else the constructor's
  void scan(double header_time, const void* records, int n, const vg_lidar_format* fmt = nullptr) {
    Scan& sc = scans_[next_id_];
    sc.xyz.resize((size_t)3 * (n + 2));
    sc.inten.resize(n + 2);
    sc.time.resize(n + 2);
    int m = 0;
    check(vg_decode_scan(lio_.raw(), records, n, fmt ? fmt : &fmt_, sc.xyz.data(), sc.inten.data(), sc.time.data(),
                         &m),
          "vg_decode_scan");
    sc.xyz.resize((size_t)3 * m);
    sc.inten.resize(m);
    sc.time.resize(m);
    const double last = m > 0 ? (double)sc.time[m - 1] : 0.0;
    check(vg_sync_push_scan(sync_, header_time, last, next_id_), "vg_sync_push_scan");
    next_id_++;
  }

  // sync_packages until it needs more data; one estimator step per package.
  // Returns the number of scans stepped.
  int spin() {
    int stepped = 0;
    std::vector<double> imu(7 * kImuCap);
    for (;;) {
      int id = -1, m = 0, ready = 0;
      double beg = 0, end = 0;
      check(vg_sync_pop(sync_, &id, &beg, &end, imu.data(), kImuCap, &m, &ready), "vg_sync_pop");
      if (ready == 0) {  // sync_packages came back empty: the idle branch (local_mapping.cpp:303-356)
        long long rel[6];
        check(vg_release_far(lio_.raw(), 0, rel), "vg_release_far");  // returns at once unless jour advanced
        break;
      }
      auto it = scans_.find(id);
      if (ready < 0) {  // too few IMU samples: the reference drops the scan
        if (it != scans_.end()) scans_.erase(it);
        continue;
      }
      if (it == scans_.end()) throw Error(VG_E_STATE, "sync_packages returned an unknown scan");
      Scan& sc = it->second;
      check(vg_step_deskew(lio_.raw(), sc.xyz.data(), sc.inten.data(), sc.time.data(), (int)sc.inten.size(), beg,
                           end, imu.data(), m),
            "vg_step_deskew");
      scans_.erase(it);
      stepped++;
    }
    poll();
    return stepped;
  }

  // Non-blocking refresh of the outputs from every scan whose results the
  // device has published (vg_poll); returns true when something changed.
  bool poll() {
    int ns = 0, nt = 0, np = 0;
    check(vg_poll(lio_.raw(), &ns, &nt, &np), "vg_poll");
    return take_rows(ns, nt, np);
  }
  // Blocking: complete every enqueued scan, then refresh (end of a run).
  void finish() {
    int nt = 0;
    check(vg_trajectory(lio_.raw(), nullptr, 0, &nt), "vg_trajectory");  // completes outstanding work
    poll();
  }

  // save_pose_tum's rows: the pose after the IEKF of every steady-state scan
  const std::vector<PoseStamped>& tum_rows() const { return tum_; }
  // pcl_path (pub_localtraj's points, the initialisation's scans included,
  // cleared by system_reset, the window's positions re-written by
  // pub_localmap after each BA); R is the pose's rotation after its IEKF
  const std::vector<PoseStamped>& path() const { return path_; }

  // /map_cmap (pub_localmap): switch the device-side cloud on (from the next
  // window BA on) and read the last one: x y z intensity per point
  void enable_local_map(bool on) { check(vg_set_publish(lio_.raw(), on ? 1 : 0), "vg_set_publish"); }
  std::vector<float> local_map() {
    int n = 0;
    check(vg_local_map(lio_.raw(), nullptr, 0, &n), "vg_local_map");
    std::vector<float> out((size_t)4 * n);
    if (n > 0) check(vg_local_map(lio_.raw(), out.data(), n, &n), "vg_local_map");
    return out;
  }

  // the last scan's downsampled points in the world (pwld of pvec_update,
  // local_mapping.cpp:425-427): R (ext_R q + ext_t) + p at the scan's pose
  std::vector<float> scan_world() {
    finish();
    int n = 0;
    check(vg_scan_points(lio_.raw(), nullptr, 0, &n), "vg_scan_points");
    std::vector<float> body((size_t)3 * n), out;
    if (n == 0 || path_.empty()) return out;
    check(vg_scan_points(lio_.raw(), body.data(), n, &n), "vg_scan_points");
    // the pose pvec_update used: right after the IEKF (the TUM row; a path
    // row's position may since have been re-written by pub_localmap)
    const PoseStamped& s = (!tum_.empty() && tum_.back().t == path_.back().t) ? tum_.back() : path_.back();
    const double* E = cfg_.ext_R;
    out.resize((size_t)3 * n);
    for (int i = 0; i < n; i++) {
      const double x = body[3 * i], y = body[3 * i + 1], z = body[3 * i + 2];
      double b[3];
      for (int r = 0; r < 3; r++) b[r] = E[3 * r] * x + E[3 * r + 1] * y + E[3 * r + 2] * z + cfg_.ext_t[r];
      for (int r = 0; r < 3; r++)
        out[3 * i + r] = (float)(s.R[3 * r] * b[0] + s.R[3 * r + 1] * b[1] + s.R[3 * r + 2] * b[2] + s.p[r]);
    }
    return out;
  }

  bool write_tum(const std::string& file) {
    finish();
    FILE* f = fopen(file.c_str(), "w");
    if (!f) return false;
    for (const PoseStamped& s : tum_) fputs(tum_line(s).c_str(), f);
    return fclose(f) == 0;
  }

  int init_phase() {
    vg_stats st;
    check(vg_get_stats(lio_.raw(), &st), "vg_get_stats");
    return st.init_phase;
  }
  LioCore& lio() { return lio_; }

 private:
  static constexpr int kImuCap = 4096;
  struct Scan {
    std::vector<float> xyz, inten, time;
  };
  void check(int r, const char* what) {
    if (r != VG_OK) throw Error(r, std::string(what) + ": " + vg_last_error(lio_.raw()));
  }
  static PoseStamped row_pose(const double* r) {
    PoseStamped s;
    s.t = r[0];
    for (int k = 0; k < 9; k++) s.R[k] = r[1 + k];
    for (int k = 0; k < 3; k++) s.p[k] = r[10 + k];
    quat_from_R(s.R, s.q);
    return s;
  }
  // TUM rows only grow; the path is re-read whenever more scans completed
  // (its window rows change after every BA, and a system_reset clears it)
  bool take_rows(int ns, int nt, int np) {
    if (ns == scans_done_ && nt == (int)tum_.size()) return false;
    scans_done_ = ns;
    const int nt_new = nt - (int)tum_.size();
    std::vector<double> t((size_t)13 * (nt_new > 0 ? nt_new : 0)), pth((size_t)14 * np);
    check(vg_poll_rows(lio_.raw(), t.data(), (int)tum_.size(), nt_new > 0 ? nt_new : 0, pth.data(), np),
          "vg_poll_rows");
    for (int i = 0; i < nt_new; i++) tum_.push_back(row_pose(&t[(size_t)13 * i]));
    path_.resize(np);
    for (int i = 0; i < np; i++) {
      path_[i] = row_pose(&pth[(size_t)14 * i]);
      path_[i].jour = pth[(size_t)14 * i + 13];
    }
    return true;
  }

  vg_config cfg_;
  vg_lidar_format fmt_;
  LioCore lio_;
  vg_sync* sync_ = nullptr;
  std::map<int, Scan> scans_;
  int next_id_ = 0;
  int scans_done_ = 0;
  std::vector<PoseStamped> tum_, path_;
};

}  // namespace vina_gpu
