// ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
// cpu_baseline leg). Never linked into or called by the product library.
//
// Restatement of the per-scan steady-state loop of VINA-SLAM:
//   IEKF  LioStateEstimation   src/pipeline/odometry.cpp:64-255
//   loop  thd_odometry_localmapping  src/pipeline/local_mapping.cpp:387-547
//   map   multi_recut / multi_margi  src/pipeline/local_mapping.cpp:17-84, 144-201
//   IMU   IMUEKF::motion_blur state/covariance propagation  src/estimation/imu_ekf.cpp:28-94
// plus a C API (orc_*) for ctypes-based tests and the CPU baseline.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include "map.hpp"
#include "vina_oracle.h"

#include "decode.hpp"
#include "kdlio.hpp"

namespace orc {

struct Pipeline {
  MapParams mpar;
  orc_config cfg;
  IMUST x_curr, extrin;
  SurfMap surf_map, surf_map_slide;
  std::vector<std::vector<SlideWindow*>> sws;
  std::vector<IMUST> x_buf;
  std::vector<PVecPtr> pvec_buf;
  std::vector<IMU_PRE*> imu_pre_buf;
  LidarFactor voxhess;
  int win_count = 0, win_base = 0;
  double jour = 0;
  bool release_flag = false;  // local_mapping.cpp:272: set when jour advanced (:510-518)
  V3 last_pos;
  double last_pcl_end_time = 0;
  bool first = true;
  // counters of the last step
  orc_stats st;
  std::vector<V3> pwld;
  std::vector<PointType> pl_tree;  // the initialisation map (odometry.cpp:269 pl_tree)

  // lio_state_estimation_kdtree — odometry.cpp:267-439. Returns
  // the valid correspondence count of the last iteration, or -1 when the map
  // held fewer than 100 points and the scan only seeded it (275-310).
  int lio_kdtree(PVec& pptr, int* iters_out) {
    *iters_out = 0;
    if (pptr.empty()) return -1;
    if (pl_tree.size() < 100) {
      for (pointVar pv : pptr) {
        pv.pnt = x_curr.R * pv.pnt + x_curr.p;
        PointType pp;
        pp.x = (float)pv.pnt[0];
        pp.y = (float)pv.pnt[1];
        pp.z = (float)pv.pnt[2];
        pl_tree.push_back(pp);
      }
      return -1;
    }
    const int num_max_iter = 4;
    IMUST x_prop = x_curr;
    const int psize = (int)pptr.size();
    bool EKF_stop_flg = false, flg_EKF_converged = false;
    M15 G, H_T_H;
    const M15 I_STATE = M15::Identity();
    int rematch_num = 0;
    M15 cov_inv = inverse(x_curr.cov);
    std::vector<double> ds(psize, -1);
    std::vector<V3> directs(psize);
    bool refind = true;
    int valid = 0;
    for (int iterCount = 0; iterCount < num_max_iter; iterCount++) {
      (*iters_out)++;
      M6 HTH;
      V6 HTz;
      valid = 0;
      for (int i = 0; i < psize; i++) {
        pointVar& pv = pptr[i];
        M3 phat = hat(pv.pnt);
        V3 wld = x_curr.R * pv.pnt + x_curr.p;
        if (refind) {
          int nearInd[kNMatch];
          float sqdis[kNMatch];
          knn_brute(pl_tree, (float)wld[0], (float)wld[1], (float)wld[2], kNMatch, nearInd, sqdis);
          double A[kNMatch * 3], b[kNMatch];
          for (int r = 0; r < kNMatch; r++) {
            const PointType& pp = pl_tree[nearInd[r]];
            A[r * 3 + 0] = pp.x;
            A[r * 3 + 1] = pp.y;
            A[r * 3 + 2] = pp.z;
            b[r] = -1.0;
          }
          double dir[3];
          colpiv_qr_solve(A, kNMatch, b, dir);
          bool check_flag = false;
          for (int r = 0; r < kNMatch; r++)
            if (std::fabs(((dir[0] * A[r * 3] + dir[1] * A[r * 3 + 1]) + dir[2] * A[r * 3 + 2]) + 1.0) > 0.1)
              check_flag = true;
          if (check_flag) {
            ds[i] = -1;
            continue;
          }
          const V3 direct = v3(dir[0], dir[1], dir[2]);
          const double d = 1.0 / norm(direct);
          ds[i] = d;
          directs[i] = direct * d;
        }
        if (ds[i] >= 0) {
          const double pd2 = dot(directs[i], wld) + ds[i];
          V6 jac_s;
          jac_s.setBlock(0, 0, (phat * x_curr.R.T()) * directs[i]);
          jac_s.setBlock(3, 0, directs[i]);
          HTH += jac_s * jac_s.T();
          HTz += jac_s * (-pd2);
          valid++;
        }
      }
      H_T_H.setBlock(0, 0, HTH);
      M15 kin = H_T_H;
      for (int r = 0; r < 15; r++)
        for (int c = 0; c < 15; c++) kin(r, c) = H_T_H(r, c) + cov_inv(r, c) / 1000;  // odometry.cpp:393
      M15 K_1 = inverse(kin);
      Mat<15, 6> K6 = K_1.block<15, 6>(0, 0);
      G.setBlock(0, 0, K6 * HTH);
      V15 vec = x_prop.minus(x_curr);
      V15 solution = K6 * HTz + vec - G.block<15, 6>(0, 0) * vec.block<6, 1>(0, 0);
      x_curr += solution;
      const V3 rot_add = solution.block<3, 1>(0, 0), tra_add = solution.block<3, 1>(3, 0);
      refind = false;
      if ((norm(rot_add) * 57.3 < 0.01) && (norm(tra_add) * 100 < 0.015)) {
        refind = true;
        flg_EKF_converged = true;
        rematch_num++;
      }
      if (iterCount == num_max_iter - 2 && !flg_EKF_converged) refind = true;
      if (rematch_num >= 2 || (iterCount == num_max_iter - 1)) {
        x_curr.cov = (I_STATE - G) * x_curr.cov;
        EKF_stop_flg = true;
      }
      if (EKF_stop_flg) break;
    }
    for (pointVar pv : pptr) {
      pv.pnt = x_curr.R * pv.pnt + x_curr.p;
      PointType ap;
      ap.x = (float)pv.pnt[0];
      ap.y = (float)pv.pnt[1];
      ap.z = (float)pv.pnt[2];
      pl_tree.push_back(ap);
    }
    down_sampling_voxel(pl_tree, 0.5, true);
    return valid;
  }

  explicit Pipeline(const orc_config& c) : voxhess(c.win_size) {
    cfg = c;
    motion_init_flag = c.cold_start != 0;
    mpar.voxel_size = c.voxel_size;
    mpar.max_layer = c.max_layer;
    mpar.max_points = c.max_points;
    mpar.min_eigen_value = c.min_eigen_value;
    for (int i = 0; i < 4; i++) {
      mpar.min_point[i] = c.min_point[i];
      mpar.plane_eigen_value_thre[i] = 1.0 / c.plane_eigen_value_thre[i];  // node.cpp:256-259
    }
    mpar.mp.resize(c.win_size);
    for (int i = 0; i < c.win_size; i++) mpar.mp[i] = i;
    mpar.imu_coef = c.imu_coef;
    mpar.imupre_scale_gravity = c.scale_gravity > 0 ? c.scale_gravity : 1.0;  // node.cpp:309
    mpar.noiseMeas.setZero();
    mpar.noiseWalk.setZero();
    for (int i = 0; i < 3; i++) {  // node.cpp:262-265
      mpar.noiseMeas(i, i) = c.ba_cov_gyr;
      mpar.noiseMeas(3 + i, 3 + i) = c.ba_cov_acc;
      mpar.noiseWalk(i, i) = c.ba_rdw_gyr;
      mpar.noiseWalk(3 + i, 3 + i) = c.ba_rdw_acc;
    }
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) extrin.R(i, j) = c.ext_R[3 * i + j];
      extrin.p[i] = c.ext_t[i];
    }
    sws.resize(c.thread_num);
    memset(&st, 0, sizeof(st));
  }
  ~Pipeline() {
    std::vector<OctoTree*> octos;
    for (auto& kv : surf_map) {
      kv.second->tras_ptr(octos);
      kv.second->clear_slwd(sws[0]);
      delete kv.second;
    }
    for (OctoTree* o : octos) delete o;
    for (auto& v : sws)
      for (SlideWindow* s : v) delete s;
    for (IMU_PRE* p : imu_pre_buf) delete p;
  }

  // IMUEKF::motion_blur state/covariance part — imu_ekf.cpp:28-94. The deskew
  // (imu_ekf.cpp:114-144) is out of scope: callers hand in
  // motion-compensated scans.
  // IMUEKF::imu_poses (ekf_imu.hpp): per processed IMU segment the offset of
  // its start from pcl_beg_time, R, p, v, bias-corrected angular velocity and
  // world acceleration (stored in the IMUST fields R, p, v, bg, ba as the
  // reference does, imu_ekf.cpp:64)
  struct ImuPose {
    double t;
    M3 R;
    V3 p, v, w, a;
  };
  std::vector<ImuPose> imu_poses;

  void propagate(const std::vector<ImuSample>& imus, double pcl_beg, double pcl_end) {
    IMUST& xc = x_curr;
    imu_poses.clear();
    V3 acc_imu, angvel_avr, acc_avr, vel_imu = xc.v, pos_imu = xc.p;
    M3 R_imu = xc.R;
    double dt = 0;
    for (size_t k = 0; k + 1 < imus.size(); k++) {
      const ImuSample& head = imus[k];
      const ImuSample& tail = imus[k + 1];
      if (head.t < last_pcl_end_time) continue;
      for (int j = 0; j < 3; j++) {
        angvel_avr[j] = 0.5 * (head.gyr[j] + tail.gyr[j]);
        acc_avr[j] = 0.5 * (head.acc[j] + tail.acc[j]);
      }
      angvel_avr -= xc.bg;
      acc_avr = acc_avr * mpar.imupre_scale_gravity - xc.ba;  // imu_ekf.cpp:51 (scale_gravity)
      acc_imu = R_imu * acc_avr + xc.g;
      double cur_time = head.t;
      if (cur_time < last_pcl_end_time) cur_time = last_pcl_end_time;
      dt = tail.t - cur_time;
      imu_poses.push_back({cur_time - pcl_beg, R_imu, pos_imu, vel_imu, angvel_avr, acc_imu});  // imu_ekf.cpp:64
      M3 acc_avr_skew = hat(acc_avr);
      M3 Exp_f = Exp(angvel_avr, dt);
      M15 F = M15::Identity(), cw;
      F.setBlock(0, 0, Exp(angvel_avr, -dt));
      F.setBlock(0, 9, M3::Identity() * -dt);
      F.setBlock(3, 6, M3::Identity() * dt);
      F.setBlock(6, 0, (R_imu * acc_avr_skew) * -dt);
      F.setBlock(6, 12, R_imu * -dt);
      for (int j = 0; j < 3; j++) {
        cw(j, j) = cfg.odo_cov_gyr * dt * dt;
        cw(9 + j, 9 + j) = cfg.odo_rdw_gyr * dt * dt;
        cw(12 + j, 12 + j) = cfg.odo_rdw_acc * dt * dt;
      }
      M3 ca;
      for (int j = 0; j < 3; j++) ca(j, j) = cfg.odo_cov_acc;
      cw.setBlock(6, 6, ((R_imu * ca) * R_imu.T()) * (dt * dt));
      xc.cov = (F * xc.cov) * F.T() + cw;
      pos_imu = pos_imu + vel_imu * dt + acc_imu * (0.5 * dt * dt);
      vel_imu = vel_imu + acc_imu * dt;
      R_imu = R_imu * Exp_f;
    }
    if (!imus.empty()) {
      double imu_end_time = imus.back().t;
      double note = pcl_end > imu_end_time ? 1.0 : -1.0;
      dt = note * (pcl_end - imu_end_time);
      xc.v = vel_imu + acc_imu * (note * dt);
      xc.R = R_imu * Exp(angvel_avr * note, dt);
      xc.p = pos_imu + vel_imu * (note * dt) + acc_imu * (note * 0.5 * dt * dt);
    }
    xc.t = pcl_end;
    last_pcl_end_time = pcl_end;
  }

  // IMUEKF::motion_blur's per-point deskew (imu_ekf.cpp:114-144) on a cloud
  // sorted by time (`curvature` = offset from pcl_beg_time, seconds): walking
  // segments and points backwards, every point later than a segment's start
  // is moved into the LiDAR frame at pcl_end_time. Faithful to the loop,
  // including its tail: once the first point has been compensated the inner
  // loop breaks, and each earlier segment whose start precedes that point's
  // time compensates it again.
  void deskew(float* xyz, const float* times, int n) {
    if (n <= 0 || imu_poses.empty()) return;
    const IMUST& xc = x_curr;
    const M3& Lr = extrin.R;  // Lid_rot_to_IMU / Lid_offset_to_IMU
    const V3& Lo = extrin.p;
    int it = n - 1;
    for (int i = (int)imu_poses.size() - 1; i >= 0; i--) {
      const ImuPose& h = imu_poses[i];
      for (; times[it] > h.t; it--) {
        const double dt = times[it] - h.t;
        const M3 R_i = h.R * Exp(h.w, dt);
        const V3 T_ei = h.p + h.v * dt + h.a * 0.5 * dt * dt - xc.p;
        const V3 P_i = v3((double)xyz[3 * it], (double)xyz[3 * it + 1], (double)xyz[3 * it + 2]);
        const V3 Pc = Lr.T() * (xc.R.T() * (R_i * (Lr * P_i + Lo) + T_ei) - Lo);
        for (int j = 0; j < 3; j++) xyz[3 * it + j] = (float)Pc[j];
        if (it == 0) break;
      }
    }
  }

  // ---- VNC scan-plane prep + VNC residual loop: odometry.cpp:22-61, 84-96,
  // 150-190. Never contributes (matchVoxelMap always returns 0, SURVEY
  // finding 3) but costs time in the reference, so the CPU baseline pays it.
  struct ScanPlaneInfo { V3 c, n; double quality, sigma_n; };
  static void collectScanPlanes(OctoTree* node, std::vector<ScanPlaneInfo>& out) {
    if (node == nullptr) return;
    if (node->octo_state == 0) {
      if (node->plane.is_plane && node->eig_value[1] > 1e-12 && node->eig_value[0] / node->eig_value[1] <= 0.12) {
        double l0 = node->eig_value[0], l1 = node->eig_value[1], l2 = node->eig_value[2];
        double ls = l0 + l1 + l2 + 1e-10;
        double q = 1.0 - l0 / ls;
        if (q > 0.5) {
          double nn = norm(node->plane.normal);
          if (nn >= 1e-12) out.push_back({node->plane.center, node->plane.normal / nn, q, std::sqrt(std::max(0.0, l0 / ls))});
        }
      }
    } else
      for (int i = 0; i < 8; i++)
        if (node->leaves[i]) collectScanPlanes(node->leaves[i], out);
  }

  // LioStateEstimation — odometry.cpp:64-255
  bool LioStateEstimation(PVec& pv, bool use_vnc) {
    IMUST x_prop = x_curr;
    const int num_max_iter = use_vnc ? 4 : 20;
    bool flg_conv = false;
    M15 G, H_T_H;
    const M15 I_STATE = M15::Identity();
    int rematch_num = 0;
    int psize = (int)pv.size();
    std::vector<OctoTree*> octos(psize, nullptr);
    M3 nnt;
    M15 cov_inv = inverse(x_curr.cov);
    SurfMap scan_voxels;
    std::vector<ScanPlaneInfo> scan_planes;
    if (use_vnc && cfg.vnc_prep) {
      PVec body = pv;
      generate_voxel(&mpar, scan_voxels, body, mpar.voxel_size);
      for (auto& kv : scan_voxels) kv.second->fitScanPlane();
      for (auto& kv : scan_voxels) collectScanPlanes(kv.second, scan_planes);
    }
    int iters = 0;
    for (int iterCount = 0; iterCount < num_max_iter; iterCount++) {
      iters++;
      M6 HTH;
      V6 HTz;
      M3 rot_var = x_curr.cov.block<3, 3>(0, 0);
      M3 tsl_var = x_curr.cov.block<3, 3>(3, 3);
      int match_num = 0;
      nnt.setZero();
      for (int i = 0; i < psize; i++) {
        pointVar& p = pv[i];
        M3 phat = hat(p.pnt);
        M3 var_world = (x_curr.R * p.var) * x_curr.R.T() + (phat * rot_var) * phat.T() + tsl_var;
        V3 wld = x_curr.R * p.pnt + x_curr.p;
        double sigma_d = 0;
        Plane* pla = nullptr;
        int flag = 0;
        if (octos[i] != nullptr && octos[i]->inside(wld)) {
          double max_prob = 0;
          flag = octos[i]->match(wld, pla, max_prob, var_world, sigma_d, octos[i]);
        } else {
          flag = match(&mpar, surf_map, wld, pla, var_world, sigma_d, octos[i]);
        }
        if (flag) {
          Plane& pp = *pla;
          double R_inv = 1.0 / (0.0005 + sigma_d);
          double resi;
          V6 jac;
          p2p_residual_jacobian(x_curr.R, p.pnt, wld, pp.normal, pp.center, resi, jac);
          HTH += (jac * R_inv) * jac.T();
          HTz -= jac * (R_inv * resi);
          nnt += outer(pp.normal, pp.normal);
          match_num++;
        }
      }
      if (use_vnc && cfg.vnc_prep) {
        M3 var_dummy = M3::Identity() * 0.01;
        for (const ScanPlaneInfo& sp : scan_planes) {
          V3 cw = x_curr.R * sp.c + x_curr.p;
          Plane* mpl = nullptr;
          double sv = 0;
          OctoTree* oct = nullptr;
          int found = matchVoxelMap(&mpar, surf_map, cw, mpl, var_dummy, sv, oct);
          if (!found || mpl == nullptr) continue;
          // unreachable (finding 3): the VNC residual would be added here
        }
      }
      if (mpar.shard_world > 1) {  // all-reduce the 34-value normal equations
        double buf[34];
        int k = 0;
        for (int r = 0; r < 6; r++)
          for (int c = r; c < 6; c++) buf[k++] = HTH(r, c);
        for (int r = 0; r < 6; r++) buf[k++] = HTz[r];
        for (int r = 0; r < 3; r++)
          for (int c = r; c < 3; c++) buf[k++] = nnt(r, c);
        buf[k++] = match_num;
        shard_sum(&mpar, buf, 34);
        k = 0;
        for (int r = 0; r < 6; r++)
          for (int c = r; c < 6; c++, k++) HTH(r, c) = HTH(c, r) = buf[k];
        for (int r = 0; r < 6; r++) HTz[r] = buf[k++];
        for (int r = 0; r < 3; r++)
          for (int c = r; c < 3; c++, k++) nnt(r, c) = nnt(c, r) = buf[k];
        match_num = (int)buf[k];
      }
      st.iekf_matches[iterCount < 4 ? iterCount : 3] = match_num;
      H_T_H.setBlock(0, 0, HTH);
      M15 K_1 = inverse(H_T_H + cov_inv);
      Mat<15, 6> K6 = K_1.block<15, 6>(0, 0);
      G.setBlock(0, 0, K6 * HTH);
      V15 vec = x_prop.minus(x_curr);
      V15 solution = K6 * HTz + vec - G.block<15, 6>(0, 0) * vec.block<6, 1>(0, 0);
      x_curr += solution;
      V3 rot_add = solution.block<3, 1>(0, 0), tra_add = solution.block<3, 1>(3, 0);
      bool stop = false;
      flg_conv = (norm(rot_add) * 57.3 < 0.01) && (norm(tra_add) * 100 < 0.015);
      if (flg_conv || ((rematch_num == 0) && (iterCount == num_max_iter - 2))) rematch_num++;
      if (rematch_num >= 2 || (iterCount == num_max_iter - 1)) {
        x_curr.cov = (I_STATE - G) * x_curr.cov;
        stop = true;
      }
      if (stop) break;
    }
    st.iekf_iters = iters;
    for (auto& kv : scan_voxels) {
      kv.second->delete_ptr();
      delete kv.second;
    }
    V3 ev;
    M3 evec;
    eig3(nnt, ev, evec);
    return !(ev[0] < 14);
  }

  // multi_recut(L,N) — local_mapping.cpp:144-201 (NormalFactor extraction at
  // line 199 feeds nothing on the live path, SURVEY finding 4, and is omitted)
  void multi_recut() {
    int thd_num = cfg.thread_num;
    std::vector<std::vector<OctoTree*>> octss(thd_num);
    int g_size = (int)surf_map_slide.size();
    if (shard_count(&mpar, g_size) < thd_num) return;  // over all shards (sharded mode)
    double part = 1.0 * g_size / thd_num;
    int cnt = 0;
    for (auto& kv : surf_map_slide) {
      octss[cnt].push_back(kv.second);
      if (octss[cnt].size() >= part && cnt < thd_num - 1) cnt++;
    }
    auto fn = [this](std::vector<OctoTree*>* oct, std::vector<SlideWindow*>* sw) {
      for (OctoTree* oc : *oct) oc->recut(win_count, x_buf, *sw);
    };
    std::vector<std::thread> th;
    for (int i = 1; i < thd_num; i++) {
      if (cfg.use_threads)
        th.emplace_back(fn, &octss[i], &sws[i]);
      else
        fn(&octss[i], &sws[i]);
    }
    fn(&octss[0], &sws[0]);
    for (auto& t : th) t.join();
    for (size_t i = 1; i < sws.size(); i++) {
      sws[0].insert(sws[0].end(), sws[i].begin(), sws[i].end());
      sws[i].clear();
    }
    for (auto& kv : surf_map_slide) kv.second->tras_opt(voxhess);
  }

  // multi_margi — local_mapping.cpp:17-84
  void multi_margi() {
    int thd_num = cfg.thread_num;
    std::vector<std::vector<OctoTree*>> octs(thd_num);
    int g_size = (int)surf_map_slide.size();
    if (shard_count(&mpar, g_size) < thd_num) return;  // over all shards (sharded mode)
    double part = 1.0 * g_size / thd_num;
    int cnt = 0;
    for (auto& kv : surf_map_slide) {
      kv.second->jour = jour;
      octs[cnt].push_back(kv.second);
      if (octs[cnt].size() >= part && cnt < thd_num - 1) cnt++;
    }
    auto fn = [this](std::vector<OctoTree*>* oct) {
      std::vector<IMUST> xxs = x_buf;
      for (OctoTree* oc : *oct) oc->margi(win_count, 1, xxs, voxhess);
    };
    std::vector<std::thread> th;
    for (int i = 1; i < thd_num; i++) {
      if (cfg.use_threads)
        th.emplace_back(fn, &octs[i]);
      else
        fn(&octs[i]);
    }
    fn(&octs[0]);
    for (auto& t : th) t.join();
    for (auto it = surf_map_slide.begin(); it != surf_map_slide.end();) {
      if (it->second->isexist)
        ++it;
      else {
        it->second->clear_slwd(sws[0]);
        it = surf_map_slide.erase(it);
      }
    }
  }

  // The idle branch's journey release (local_mapping.cpp:317-344), taken when
  // the caller has no package (sync_packages false): once jour has advanced
  // (release_flag), every root voxel whose jour stamp is >= release_dis (700,
  // :324) behind is erased with its subtree (OctoTree::tras_ptr,
  // octree.cpp:597-608; the deletes run at once here). The reference's int
  // truncation of jour - root.jour is kept. A root still in surf_map_slide is
  // kept: the reference would leave a dangling pointer there (unreachable at
  // 700 m: slide roots are stamped at every margi). out: [0] roots erased
  // (-1: no release pending), [1] nodes erased, then the census after it:
  // [2] roots, [3] nodes, [4] point_fix points held.
  static long long subtree_nodes(OctoTree* o) {
    std::vector<OctoTree*> v;
    o->tras_ptr(v);
    return 1 + (long long)v.size();
  }
  void census(long long* out) {
    long long nodes = 0, fix = 0;
    for (auto& kv : surf_map) {
      std::vector<OctoTree*> v;
      kv.second->tras_ptr(v);
      v.push_back(kv.second);
      nodes += (long long)v.size();
      for (OctoTree* o : v) fix += (long long)o->point_fix.size();
    }
    out[2] = (long long)surf_map.size();
    out[3] = nodes;
    out[4] = fix;
  }
  void release_far(long long* out) {
    out[0] = -1;
    out[1] = 0;
    if (release_flag) {
      release_flag = false;
      const int thr = cfg.release_dis > 0 ? cfg.release_dis : 700;
      out[0] = 0;
      for (auto it = surf_map.begin(); it != surf_map.end();) {
        const int dis = jour - it->second->jour;
        if (dis < thr || surf_map_slide.find(it->first) != surf_map_slide.end()) {
          ++it;
          continue;
        }
        std::vector<OctoTree*> octos;
        it->second->tras_ptr(octos);
        octos.push_back(it->second);
        out[0]++;
        out[1] += (long long)octos.size();
        it->second->clear_slwd(sws[0]);
        for (OctoTree* o : octos) delete o;
        it = surf_map.erase(it);
      }
    }
    census(out);
  }

  // local_mapping.cpp:489-546: with a full window, LI_BA damping_iter, x_curr.R/p
  // from the window's last frame, multi_margi, jour, the mp ring and the slide
  template <class TP>
  void window_tail(TP* t5, TP* t6) {
    using clk = std::chrono::steady_clock;
    if (cfg.if_BA == 1) {
      LI_BA_Optimizer opt;
      opt.mpar = &mpar;
      opt.use_threads = cfg.use_threads != 0;
      st.ba_iters = opt.damping_iter(x_buf, voxhess, imu_pre_buf);
    }
    x_curr.R = x_buf[win_count - 1].R;
    x_curr.p = x_buf[win_count - 1].p;
    pub_localmap();
    *t5 = clk::now();
    mpar.cnt_plane_update = 0;
    mpar.cnt_fix_full = 0;
    multi_margi();
    st.plane_updates = mpar.cnt_plane_update;
    st.fix_full = mpar.cnt_fix_full;
    *t6 = clk::now();
    const int mgsize = 1;
    if ((win_base + win_count) % 10 == 0) {
      double spat = norm(x_curr.p - last_pos);
      if (spat > 0.5) {
        jour += spat;
        last_pos = x_curr.p;
        release_flag = true;  // local_mapping.cpp:517
      }
    }
    for (int i = 0; i < cfg.win_size; i++) {
      mpar.mp[i] += mgsize;
      if (mpar.mp[i] >= cfg.win_size) mpar.mp[i] -= cfg.win_size;
    }
    for (int i = mgsize; i < win_count; i++) {
      x_buf[i - mgsize] = x_buf[i];
      std::swap(pvec_buf[i - mgsize], pvec_buf[i]);
    }
    for (int i = win_count - mgsize; i < win_count; i++) {
      x_buf.pop_back();
      pvec_buf.pop_back();
      delete imu_pre_buf.front();
      imu_pre_buf.erase(imu_pre_buf.begin());
    }
    win_base += mgsize;
    win_count -= mgsize;
  }

#include "init.inc"

  // One scan of thd_odometry_localmapping's steady-state branch,
  // local_mapping.cpp:389-547 (initialisation, SURVEY row f2, is replaced by a
  // seeded state and an empty map).
  int step(const float* xyz_in, const float* inten, int n, double beg, double end, const std::vector<ImuSample>& imus,
           double* timing, const float* times = nullptr) {
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    memset(&st, 0, sizeof(st));
    imu_poses.clear();
    if (motion_init_flag) {  // local_mapping.cpp:362-386: the initialisation branch
      const int r = initialization(imus, xyz_in, inten, times, n, beg, end);
      st.init_phase = init_phase;
      if (r != 1) {
        if (r == -1) system_reset(imus);
        if (timing) timing[6] = std::chrono::duration<double>(clk::now() - t0).count();
        return 0;
      }
      motion_init_flag = false;  // init success: the same scan continues into the window tail
      st.n_factors = (int)voxhess.plvec_voxels.size();
      st.roots_new = (int)surf_map.size();
      auto t5 = clk::now(), t6 = t5;
      if (win_count >= cfg.win_size) window_tail(&t5, &t6);
      st.n_slide = (int)surf_map_slide.size();
      if (timing) timing[6] = std::chrono::duration<double>(clk::now() - t0).count();
      return 0;
    }
    if (!first) propagate(imus, beg, end);
    else { x_curr.t = end; last_pcl_end_time = end; }
    std::vector<float> xyz_d;
    const float* xyz = xyz_in;
    if (times) {  // odom_ekf.process -> motion_blur deskew (local_mapping.cpp:389, imu_ekf.cpp:114-144)
      xyz_d.assign(xyz_in, xyz_in + 3 * (size_t)n);
      deskew(xyz_d.data(), times, n);
      xyz = xyz_d.data();
    }
    std::vector<PointType> pcl(n);
    for (int i = 0; i < n; i++) {
      pcl[i].x = xyz[3 * i];
      pcl[i].y = xyz[3 * i + 1];
      pcl[i].z = xyz[3 * i + 2];
      pcl[i].intensity = inten ? inten[i] : 0.f;
      pcl[i].curvature = (float)(end - beg);
    }
    std::vector<PointType> pl_down = pcl;
    down_sampling_voxel(pl_down, cfg.down_size);
    if (pl_down.size() < 2000) {
      pl_down = pcl;
      down_sampling_voxel(pl_down, cfg.down_size / 2);
    }
    st.n_raw = n;
    st.n_ds = (int)pl_down.size();
    PVecPtr pptr(new PVec);
    var_init(extrin, pl_down, *pptr, cfg.dept_err, cfg.beam_err);
    PVec no_ds;
    var_init(extrin, pcl, no_ds, cfg.dept_err, cfg.beam_err);
    auto t1 = clk::now();
    bool nondegen = LioStateEstimation(no_ds, true);
    st.degenerate = nondegen ? 0 : 1;
    auto t2 = clk::now();
    pwld.clear();
    pvec_update(*pptr, x_curr, pwld);
    path_push(jour);
    traj_push();
    win_count++;
    x_buf.push_back(x_curr);
    pvec_buf.push_back(pptr);
    if (win_count > 1) {
      imu_pre_buf.push_back(new IMU_PRE(&mpar, x_buf[win_count - 2].bg, x_buf[win_count - 2].ba));
      imu_pre_buf[win_count - 2]->push_imu(imus);
    }
    voxhess.clear();
    voxhess.win_size = cfg.win_size;
    size_t before = surf_map.size();
    cut_voxel_multi(&mpar, surf_map, *pvec_buf[win_count - 1], win_count - 1, surf_map_slide, cfg.win_size, pwld, sws,
                    cfg.use_threads != 0);
    st.roots_new = (int)(surf_map.size() - before);
    auto t3 = clk::now();
    multi_recut();
    st.n_factors = (int)voxhess.plvec_voxels.size();
    auto t4 = clk::now();
    auto t5 = t4, t6 = t4;
    if (win_count >= cfg.win_size) window_tail(&t5, &t6);
    first = false;
    st.n_slide = (int)surf_map_slide.size();
    auto t7 = clk::now();
    if (timing) {
      auto d = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
      timing[0] = d(t0, t1);  // propagate + downsample + var_init
      timing[1] = d(t1, t2);  // IEKF
      timing[2] = d(t2, t3);  // pvec_update + insert
      timing[3] = d(t3, t4);  // recut + factor extraction
      timing[4] = d(t4, t5);  // BA
      timing[5] = d(t5, t6);  // margi
      timing[6] = d(t0, t7);  // total
    }
    return 0;
  }

  // save_pose_tum (io.cpp:67-77, local_mapping.cpp:430): steady-state scans
  // only, per row t, R(9), p(3)
  std::vector<double> traj;
  void traj_push() {
    traj.push_back(x_curr.t);
    for (int i = 0; i < 9; i++) traj.push_back(x_curr.R[i]);
    for (int i = 0; i < 3; i++) traj.push_back(x_curr.p[i]);
  }
  // pcl_path of pub_localtraj (publishers.cpp:65-97): per row t, R(9), p(3),
  // jour (the path point's curvature); the initialisation's scans included
  // (node.cpp:325, jour 0), cleared by system_reset (node.cpp:403)
  std::vector<double> path;
  void path_push(double j) {
    path.push_back(x_curr.t);
    for (int i = 0; i < 9; i++) path.push_back(x_curr.R[i]);
    for (int i = 0; i < 3; i++) path.push_back(x_curr.p[i]);
    path.push_back(j);
  }
  // pub_localmap (publishers.cpp:99-131, local_mapping.cpp:505, mgsize = 1):
  // /map_cmap = every third point of pvec_buf[0] at x_buf[0]; the path rows
  // [win_base, win_base + win_count) take x_buf[i].p. cmap_all keeps every
  // point of pvec_buf[0] (the test compares sets: the device's point order
  // differs)
  std::vector<float> cmap, cmap_all;
  void pub_localmap() {
    cmap.clear();
    cmap_all.clear();
    const PVec& pv0 = *pvec_buf[0];
    for (size_t j = 0; j < pv0.size(); j++) {
      const V3 w = x_buf[0].R * pv0[j].pnt + x_buf[0].p;
      const float f[4] = {(float)w[0], (float)w[1], (float)w[2], pv0[j].intensity};
      cmap_all.insert(cmap_all.end(), f, f + 4);
      if (j % 3 == 0) cmap.insert(cmap.end(), f, f + 4);
    }
    for (int i = 0; i < win_count; i++) {
      const size_t r = (size_t)(i + win_base) * 14;
      if (r + 14 > path.size()) break;
      for (int k = 0; k < 3; k++) path[r + 10 + k] = x_buf[i].p[k];
    }
  }
};

}  // namespace orc

using namespace orc;

// ------------------------------------------------------------------ C API
static void state_to(const IMUST& x, double* o) {
  o[0] = x.t;
  for (int i = 0; i < 9; i++) o[1 + i] = x.R[i];
  for (int i = 0; i < 3; i++) {
    o[10 + i] = x.p[i];
    o[13 + i] = x.v[i];
    o[16 + i] = x.bg[i];
    o[19 + i] = x.ba[i];
    o[22 + i] = x.g[i];
  }
  for (int i = 0; i < 225; i++) o[25 + i] = x.cov[i];
}
static void state_from(IMUST& x, const double* o) {
  x.t = o[0];
  for (int i = 0; i < 9; i++) x.R[i] = o[1 + i];
  for (int i = 0; i < 3; i++) {
    x.p[i] = o[10 + i];
    x.v[i] = o[13 + i];
    x.bg[i] = o[16 + i];
    x.ba[i] = o[19 + i];
    x.g[i] = o[22 + i];
  }
  for (int i = 0; i < 225; i++) x.cov[i] = o[25 + i];
}

extern "C" {

void orc_voxel_key_d(const double* xyz, int n, double size, int64_t* out) {
  for (int i = 0; i < n; i++) {
    V3 w = v3(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    VOXEL_LOC k = voxel_key(w, size);
    out[3 * i] = k.x;
    out[3 * i + 1] = k.y;
    out[3 * i + 2] = k.z;
  }
}

size_t orc_voxel_hash(int64_t x, int64_t y, int64_t z) { return VoxHash()(VOXEL_LOC(x, y, z)); }

// down_sampling_close + the stable time sort of initialization (node.cpp:337-345)
int orc_down_sampling_close(const float* xyz, const float* times, int n, double size, float* out_xyzt) {
  std::vector<PointType> pl(n);
  for (int i = 0; i < n; i++) {
    pl[i].x = xyz[3 * i];
    pl[i].y = xyz[3 * i + 1];
    pl[i].z = xyz[3 * i + 2];
    pl[i].curvature = times ? times[i] : 0.f;
  }
  Pipeline::down_sampling_close(pl, size);
  std::stable_sort(pl.begin(), pl.end(), [](const PointType& a, const PointType& b) { return a.curvature < b.curvature; });
  for (size_t i = 0; i < pl.size(); i++) {
    out_xyzt[4 * i] = pl[i].x;
    out_xyzt[4 * i + 1] = pl[i].y;
    out_xyzt[4 * i + 2] = pl[i].z;
    out_xyzt[4 * i + 3] = pl[i].curvature;
  }
  return (int)pl.size();
}

int orc_downsample(const float* xyz, const float* inten, int n, double size, float* out_xyzic, int* n_out) {
  std::vector<PointType> pl(n);
  for (int i = 0; i < n; i++) {
    pl[i].x = xyz[3 * i];
    pl[i].y = xyz[3 * i + 1];
    pl[i].z = xyz[3 * i + 2];
    pl[i].intensity = inten ? inten[i] : 0.f;
    pl[i].curvature = 0.05f;
  }
  down_sampling_voxel(pl, size);
  for (size_t i = 0; i < pl.size(); i++) {
    out_xyzic[5 * i] = pl[i].x;
    out_xyzic[5 * i + 1] = pl[i].y;
    out_xyzic[5 * i + 2] = pl[i].z;
    out_xyzic[5 * i + 3] = pl[i].intensity;
    out_xyzic[5 * i + 4] = pl[i].curvature;
  }
  *n_out = (int)pl.size();
  return 0;
}

void orc_calc_body_var(const double* p, double range_inc, double degree_inc, double* pnt_out, double* var_out) {
  V3 pb = v3(p[0], p[1], p[2]);
  M3 var;
  calcBodyVar(pb, (float)range_inc, (float)degree_inc, var);
  for (int i = 0; i < 3; i++) pnt_out[i] = pb[i];
  for (int i = 0; i < 9; i++) var_out[i] = var[i];
}

void orc_eig3(const double* A, double* w, double* V) {
  M3 m;
  for (int i = 0; i < 9; i++) m[i] = A[i];
  V3 ev;
  M3 vec;
  eig3(m, ev, vec);
  for (int i = 0; i < 3; i++) w[i] = ev[i];
  for (int i = 0; i < 9; i++) V[i] = vec[i];
}

void orc_inverse15(const double* A, double* out) {
  M15 m;
  for (int i = 0; i < 225; i++) m[i] = A[i];
  M15 o = inverse(m);
  for (int i = 0; i < 225; i++) out[i] = o[i];
}

void orc_ldlt_solve(const double* A, const double* b, int n, double* x) {
  MatX m(n, n);
  for (int i = 0; i < n * n; i++) m.d[i] = A[i];
  std::vector<double> bb(b, b + n);
  std::vector<double> xx = ldlt_solve(m, bb);
  for (int i = 0; i < n; i++) x[i] = xx[i];
}

void orc_so3(const double* w, double* R_out, double* log_out, double* jr_out, double* jrinv_out) {
  V3 a = v3(w[0], w[1], w[2]);
  M3 R = Exp(a);
  V3 l = Log(R);
  M3 j = jr(a);
  M3 ji = jr_inv(R);
  for (int i = 0; i < 9; i++) {
    R_out[i] = R[i];
    jr_out[i] = j[i];
    jrinv_out[i] = ji[i];
  }
  for (int i = 0; i < 3; i++) log_out[i] = l[i];
}

void* orc_create(const orc_config* c) { return new Pipeline(*c); }
void orc_destroy(void* h) { delete (Pipeline*)h; }
void orc_seed(void* h, const double* state) {
  Pipeline* p = (Pipeline*)h;
  state_from(p->x_curr, state);
}
void orc_get_state(void* h, double* state) { state_to(((Pipeline*)h)->x_curr, state); }
int orc_step(void* h, const float* xyz, const float* inten, int n, double beg, double end, const double* imu, int m,
             double* timing) {
  std::vector<ImuSample> imus(m);
  for (int i = 0; i < m; i++) {
    imus[i].t = imu[7 * i];
    imus[i].gyr = v3(imu[7 * i + 1], imu[7 * i + 2], imu[7 * i + 3]);
    imus[i].acc = v3(imu[7 * i + 4], imu[7 * i + 5], imu[7 * i + 6]);
  }
  return ((Pipeline*)h)->step(xyz, inten, n, beg, end, imus, timing);
}
int orc_step_deskew(void* h, const float* xyz, const float* inten, const float* times, int n, double beg, double end,
                    const double* imu, int m, double* timing) {
  std::vector<ImuSample> imus(m);
  for (int i = 0; i < m; i++) {
    imus[i].t = imu[7 * i];
    imus[i].gyr = v3(imu[7 * i + 1], imu[7 * i + 2], imu[7 * i + 3]);
    imus[i].acc = v3(imu[7 * i + 4], imu[7 * i + 5], imu[7 * i + 6]);
  }
  return ((Pipeline*)h)->step(xyz, inten, n, beg, end, imus, timing, times);
}
int orc_deskew_only(void* h, float* xyz, const float* times, int n, double beg, double end, const double* imu, int m) {
  Pipeline* P = (Pipeline*)h;
  std::vector<ImuSample> imus(m);
  for (int i = 0; i < m; i++) {
    imus[i].t = imu[7 * i];
    imus[i].gyr = v3(imu[7 * i + 1], imu[7 * i + 2], imu[7 * i + 3]);
    imus[i].acc = v3(imu[7 * i + 4], imu[7 * i + 5], imu[7 * i + 6]);
  }
  P->propagate(imus, beg, end);
  P->deskew(xyz, times, n);
  return (int)P->imu_poses.size();
}
void orc_get_stats(void* h, orc_stats* s) { *s = ((Pipeline*)h)->st; }
void orc_release_far(void* h, long long* out) { ((Pipeline*)h)->release_far(out); }
// test hook: every root voxel of surf_map (any order) — key x/y/z, its jour
// stamp, flags (1: in surf_map_slide, 2: isexist), subtree nodes and
// point_fix points; returns the root count (rows past cap are not written)
int orc_roots(void* h, long long* key, double* jour, int* flags, int* nodes, int* nfix, int cap) {
  Pipeline* P = (Pipeline*)h;
  int n = 0;
  for (auto& kv : P->surf_map) {
    if (n < cap) {
      std::vector<OctoTree*> v;
      kv.second->tras_ptr(v);
      v.push_back(kv.second);
      long long f = 0;
      for (OctoTree* o : v) f += (long long)o->point_fix.size();
      key[3 * n] = kv.first.x;
      key[3 * n + 1] = kv.first.y;
      key[3 * n + 2] = kv.first.z;
      jour[n] = kv.second->jour;
      flags[n] = (P->surf_map_slide.find(kv.first) != P->surf_map_slide.end() ? 1 : 0) |
                 (kv.second->isexist ? 2 : 0);
      nodes[n] = (int)v.size();
      nfix[n] = (int)f;
    }
    n++;
  }
  return n;
}
double orc_jour(void* h) { return ((Pipeline*)h)->jour; }
// one lio_state_estimation_kdtree call on the scan downsampled at
// max(down_size, 0.5) (raw LiDAR frame; var_init applies the extrinsic),
// with the context's x_curr (orc_seed / orc_get_state) as the state
int orc_lio_kdtree(void* h, const float* xyz, int n, int* valid, int* iters) {
  Pipeline* P = (Pipeline*)h;
  std::vector<PointType> pl(n);
  for (int i = 0; i < n; i++) {
    pl[i].x = xyz[3 * i];
    pl[i].y = xyz[3 * i + 1];
    pl[i].z = xyz[3 * i + 2];
  }
  PVec pv;
  var_init(P->extrin, pl, pv, P->cfg.dept_err, P->cfg.beam_err);
  *valid = P->lio_kdtree(pv, iters);
  return 0;
}
int orc_kdmap_size(void* h) { return (int)((Pipeline*)h)->pl_tree.size(); }
void orc_kdmap_get(void* h, float* xyz) {
  const std::vector<PointType>& t = ((Pipeline*)h)->pl_tree;
  for (size_t i = 0; i < t.size(); i++) {
    xyz[3 * i] = t[i].x;
    xyz[3 * i + 1] = t[i].y;
    xyz[3 * i + 2] = t[i].z;
  }
}
void orc_qr_solve(const double* A, int m, const double* b, double* x) { colpiv_qr_solve(A, m, b, x); }
int orc_knn(const float* pts, int np, const float* q, int k, int* idx, float* sq) {
  std::vector<PointType> v(np);
  for (int i = 0; i < np; i++) {
    v[i].x = pts[3 * i];
    v[i].y = pts[3 * i + 1];
    v[i].z = pts[3 * i + 2];
  }
  return knn_brute(v, q[0], q[1], q[2], k, idx, sq);
}
void orc_shard(void* h, int rank, int world, int (*fn)(double*, int, void*), void* user) {
  Pipeline* P = (Pipeline*)h;
  P->mpar.shard_rank = rank;
  P->mpar.shard_world = world;
  P->mpar.allreduce = fn;
  P->mpar.ar_user = user;
}
int orc_traj_len(void* h) { return (int)((Pipeline*)h)->traj.size() / 13; }
int orc_path_len(void* h) { return (int)((Pipeline*)h)->path.size() / 14; }
void orc_get_path(void* h, double* out) {
  Pipeline* p = (Pipeline*)h;
  memcpy(out, p->path.data(), p->path.size() * sizeof(double));
}
int orc_local_map(void* h, int all, float* out, int cap) {
  const std::vector<float>& c = all ? ((Pipeline*)h)->cmap_all : ((Pipeline*)h)->cmap;
  const int n = (int)c.size() / 4;
  if (out) memcpy(out, c.data(), (size_t)(n < cap ? n : cap) * 4 * sizeof(float));
  return n;
}
void orc_get_traj(void* h, double* out) {
  Pipeline* p = (Pipeline*)h;
  memcpy(out, p->traj.data(), p->traj.size() * sizeof(double));
}
int orc_window_states(void* h, double* out) {
  Pipeline* p = (Pipeline*)h;
  for (size_t i = 0; i < p->x_buf.size(); i++) state_to(p->x_buf[i], out + 250 * i);
  return (int)p->x_buf.size();
}
void orc_capture_arm(void* h) {
  Pipeline* p = (Pipeline*)h;
  p->mpar.capture = 1;
  p->mpar.captured.clear();
}
int orc_capture_get(void* h, double* out, int cap) {
  const std::vector<double>& c = ((Pipeline*)h)->mpar.captured;
  if (out) memcpy(out, c.data(), (c.size() < (size_t)cap ? c.size() : (size_t)cap) * sizeof(double));
  return (int)c.size();
}

// decoders + pcl_handler over little-endian records
int orc_decode_scan(const void* rec, int n, int kind, int stride, int off_x, int off_y, int off_z, int off_i,
                    int off_t, int filter_num, double blind, double omega_l, double time_base, float* out5,
                    int cap) {
  DecFormat f{kind, stride, off_x, off_y, off_z, off_i, off_t, filter_num, blind, omega_l, time_base};
  std::vector<DecPoint> v = decode_records((const unsigned char*)rec, n, f);
  const int m = (int)v.size() < cap ? (int)v.size() : cap;
  for (int j = 0; j < m; j++) {
    out5[5 * j] = v[j].x;
    out5[5 * j + 1] = v[j].y;
    out5[5 * j + 2] = v[j].z;
    out5[5 * j + 3] = v[j].intensity;
    out5[5 * j + 4] = v[j].curvature;
  }
  return (int)v.size();
}

}  // extern "C"
