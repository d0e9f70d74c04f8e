// vina_gpu.hpp — header-only C++ face of the C-ABI (vina_gpu.h) for a caller
// shaped like the reference's VINA_SLAM (include/vina_slam/platform/ros2/node.hpp:27-96).
// Method names follow the reference calls they replace so that
// thd_odometry_localmapping (local_mapping.cpp:387-547) keeps its structure;
// see INTEGRATION.md for the line-by-line mapping. Errors become exceptions
// (the reference calls exit(), octree.cpp:407, optimizers.cpp:70).
#pragma once
#include <stdexcept>
#include <string>
#include <vector>
#include "vina_gpu.h"

namespace vina_gpu {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

class LioCore {
 public:
  LioCore(const vg_config& cfg, const vg_capacity* cap = nullptr, int device = 0) {
    check(vg_create(&cfg, cap, device, &ctx_), "vg_create");
  }
  ~LioCore() { vg_destroy(ctx_); }
  LioCore(const LioCore&) = delete;
  LioCore& operator=(const LioCore&) = delete;

  // initialisation output (x_curr after Initialization::motion_init)
  void seed(const double* state250) { check(vg_seed(ctx_, state250), "vg_seed"); }
  // VINA_SLAM::system_reset (node.cpp:368-408)
  void system_reset() { check(vg_reset(ctx_), "vg_reset"); }

  // one scan (the whole steady-state branch, local_mapping.cpp:389-547)
  void process(const std::vector<float>& xyz, const std::vector<float>& intensity, double beg, double end,
               const std::vector<double>& imu7) {
    check(vg_step(ctx_, xyz.data(), intensity.empty() ? nullptr : intensity.data(), (int)(xyz.size() / 3), beg, end,
                  imu7.data(), (int)(imu7.size() / 7)),
          "vg_step");
  }
  // one raw sweep: IMUEKF::motion_blur's deskew (imu_ekf.cpp:114-144, row f1)
  // on the device, then the steady-state branch; time[i] = the point's offset
  // from beg in seconds (the reference's `curvature` field), ascending
  void process_raw(const std::vector<float>& xyz, const std::vector<float>& intensity, const std::vector<float>& time,
                   double beg, double end, const std::vector<double>& imu7) {
    check(vg_step_deskew(ctx_, xyz.data(), intensity.empty() ? nullptr : intensity.data(), time.data(),
                         (int)(xyz.size() / 3), beg, end, imu7.data(), (int)(imu7.size() / 7)),
          "vg_step_deskew");
  }

  // ---- the same, call by call (reference names) ----
  void load_scan(const float* xyz, const float* intensity, int n) { check(vg_scan_load(ctx_, xyz, intensity, n), "vg_scan_load"); }
  // odom_ekf.process(x_curr, *pcl_curr, imus)          local_mapping.cpp:389
  void odom_ekf_process(const double* imu7, int m, double beg, double end) {
    check(vg_propagate(ctx_, imu7, m, beg, end), "vg_propagate");
  }
  // down_sampling_voxel(pl_down, down_size) (+ /2)    local_mapping.cpp:396-403
  int down_sampling_voxel() {
    int n = 0;
    check(vg_downsample_scan(ctx_, &n), "vg_downsample_scan");
    return n;
  }
  // VNC_lio(no_ds_pptr)                                local_mapping.cpp:413
  bool VNC_lio() {
    int degenerate = 0;
    check(vg_lio_state_estimation(ctx_, &degenerate), "vg_lio_state_estimation");
    return degenerate == 0;
  }
  // x_buf.push_back / imu_pre_buf push_imu             local_mapping.cpp:434-441
  void push_window(const double* imu7, int m) { check(vg_window_push(ctx_, imu7, m), "vg_window_push"); }
  // cut_voxel_multi(surf_map, pvec_buf[..], ...)       local_mapping.cpp:448
  void cut_voxel_multi() { check(vg_cut_voxel_multi(ctx_), "vg_cut_voxel_multi"); }
  // multi_recut(surf_map_slide, win_count, x_buf, voxhess, ...)  local_mapping.cpp:451
  int multi_recut() {
    int nf = 0;
    check(vg_multi_recut(ctx_, &nf), "vg_multi_recut");
    return nf;
  }
  // LI_BA_Optimizer::damping_iter(x_buf, voxhess, imu_pre_buf, &hess)  local_mapping.cpp:496
  int damping_iter() {
    int it = 0;
    check(vg_damping_iter(ctx_, &it), "vg_damping_iter");
    return it;
  }
  // x_curr <- x_buf.back(); multi_margi(...); slide   local_mapping.cpp:499-546
  void multi_margi() { check(vg_multi_margi(ctx_), "vg_multi_margi"); }
  void end_scan() { check(vg_step_end(ctx_), "vg_step_end"); }
  int win_count() {
    int n = 0;
    check(vg_win_count(ctx_, &n), "vg_win_count");
    return n;
  }

  std::vector<double> x_curr() {
    std::vector<double> s(VG_STATE_LEN);
    check(vg_get_state(ctx_, s.data()), "vg_get_state");
    return s;
  }
  vg_stats stats() {
    vg_stats st;
    check(vg_get_stats(ctx_, &st), "vg_get_stats");
    return st;
  }
  vg_ctx* raw() { return ctx_; }

 private:
  void check(int r, const char* what) {
    if (r != VG_OK) throw Error(r, std::string(what) + ": " + vg_last_error(ctx_));
  }
  vg_ctx* ctx_ = nullptr;
};

}  // namespace vina_gpu
