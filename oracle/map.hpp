// ORACLE — test infrastructure only. Never linked into the product library.
//
// CPU restatement of the VINA-SLAM adaptive voxel/octree map, the LiDAR BA
// factor, IMU preintegration and the LiDAR-inertial LM optimizer:
//   include/vina_slam/mapping/{octree,plane,slide_window,factors}.hpp,
//   src/mapping/{octree,voxel_map,factors,optimizers}.cpp,
//   include/vina_slam/preintegration.hpp, src/estimation/imu_preintegration.cpp.
// The reference's process-wide globals (octree.cpp:67-75, optimizers.cpp:8,
// imu_preintegration.cpp:3-5) live in one MapParams object per pipeline.
#pragma once
#include <atomic>
#include <mutex>
#include <vector>
#include "core.hpp"

namespace orc {

struct MapParams {
  double voxel_size = 1.0;      // octree.cpp:71
  int max_layer = 2;            // octree.cpp:69
  int max_points = 100;         // octree.cpp:70
  double min_eigen_value = 0.0025;
  double min_point[4] = {20, 20, 15, 10};            // node.cpp:219
  double plane_eigen_value_thre[4] = {1, 1, 1, 1};   // already inverted (node.cpp:256-259)
  std::vector<int> mp;                               // octree.cpp:75 (window ring index)
  double imu_coef = 1e-4;                            // optimizers.cpp:8
  double imupre_scale_gravity = 1.0;                 // imu_preintegration.cpp:3
  M6 noiseMeas, noiseWalk;                           // imu_preintegration.cpp:4-5
  // spatial-tile sharding; world 1 = the reference itself
  int shard_rank = 0, shard_world = 1;
  int (*allreduce)(double* buf, int n, void* user) = nullptr;  // in-place sum over ranks
  void* ar_user = nullptr;
  // per-scan branch counters of OctoTree::margi (observability for the parity
  // tests; the reference keeps none): plane_update calls (octree.cpp:441-446)
  // and leaves past max_points (octree.cpp:461-469)
  std::atomic<int> cnt_plane_update{0}, cnt_fix_full{0};
  // test hook (orc_capture_*): the next LM run's first divide_thread pass
  int capture = 0;  // 1 armed, 2 captured
  std::vector<double> captured;
};

// owner rank of the 16^3-root-voxel tile of a root key (the product's
// tile_owner, vina-slam_amd/csrc/vg_dev.h, on the same packed key)
inline int tile_owner(const VOXEL_LOC& k, int world) {
  const uint64_t off = 1ull << 20;
  const uint64_t tx = (((uint64_t)(k.x + (int64_t)off)) >> 4) & 0x1ffff;
  const uint64_t ty = (((uint64_t)(k.y + (int64_t)off)) >> 4) & 0x1ffff;
  const uint64_t tz = (((uint64_t)(k.z + (int64_t)off)) >> 4) & 0x1ffff;
  uint64_t h = (tx * 0x9E3779B97F4A7C15ull) ^ (ty * 0xC2B2AE3D27D4EB4Full) ^ (tz * 0x165667B19E3779F9ull);
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 29;
  return (int)(h % (uint64_t)world);
}
inline bool shard_owns(const MapParams* m, const VOXEL_LOC& k) {
  return m->shard_world <= 1 || tile_owner(k, m->shard_world) == m->shard_rank;
}
// sum over the ranks (no-op unsharded); counts travel as doubles (exact)
inline void shard_sum(const MapParams* m, double* buf, int n) {
  if (m->shard_world > 1 && m->allreduce) m->allreduce(buf, n, m->ar_user);
}
inline int shard_count(const MapParams* m, int local) {
  double v = local;
  shard_sum(m, &v, 1);
  return (int)v;
}

// Plane — plane.hpp:5-24
struct Plane {
  V3 center, normal;
  M6 plane_var;
  float radius = 0;
  bool is_plane = false;
};

// Point-to-plane residual and Jacobian of LioStateEstimation's point loop
// (odometry.cpp:136-142): r = n.(w - c), j = [hat(pnt) R^T n ; n] for the
// right-perturbed pose (R Exp(dtheta), p + dp)
inline void p2p_residual_jacobian(const M3& R, const V3& pnt, const V3& wld, const V3& normal, const V3& center,
                                  double& resi, V6& jac) {
  resi = dot(normal, wld - center);
  jac.setBlock(0, 0, (hat(pnt) * R.T()) * normal);
  jac.setBlock(3, 0, normal);
}

// Bf_var — octree.cpp:83-92
inline void Bf_var(const pointVar& pv, M9& bcov, const V3& vec) {
  Mat<6, 3> Bi;
  Bi(0, 0) = 2 * vec[0];
  Bi(1, 0) = vec[1]; Bi(1, 1) = vec[0];
  Bi(2, 0) = vec[2]; Bi(2, 2) = vec[0];
  Bi(3, 1) = 2 * vec[1];
  Bi(4, 1) = vec[2]; Bi(4, 2) = vec[1];
  Bi(5, 2) = 2 * vec[2];
  Mat<6, 3> Biup = Bi * pv.var;
  bcov.setBlock(0, 0, Biup * Bi.T());
  bcov.setBlock(0, 6, Biup);
  bcov.setBlock(6, 0, Biup.T());
  bcov.setBlock(6, 6, pv.var);
}

// SlideWindow — slide_window.hpp:6-20, octree.cpp:114-140
struct SlideWindow {
  std::vector<PVec> points;
  std::vector<PointCluster> pcrs_local;
  explicit SlideWindow(int w) { pcrs_local.resize(w); points.resize(w); }
  void resize(int w) {
    if ((int)points.size() != w) { points.resize(w); pcrs_local.resize(w); }
  }
  void clear() {
    for (size_t i = 0; i < points.size(); i++) { points[i].clear(); pcrs_local[i].clear(); }
  }
};

// LidarFactor — factors.hpp:10-36, factors.cpp:7-168
struct LidarFactor {
  std::vector<PointCluster> sig_vecs;
  std::vector<std::vector<PointCluster>> plvec_voxels;
  std::vector<double> coeffs;
  std::vector<V3> eig_values;
  std::vector<M3> eig_vectors;
  std::vector<PointCluster> pcr_adds;
  int win_size;
  explicit LidarFactor(int w) : win_size(w) {}
  void push_voxel(std::vector<PointCluster>& vec_orig, PointCluster& fix, double coe, V3& eig_value,
                  M3& eig_vector, PointCluster& pcr_add);
  void acc_evaluate2(const std::vector<IMUST>& xs, int head, int end, MatX& Hess, std::vector<double>& JacT,
                     double& residual) const;
  void evaluate_only_residual(const std::vector<IMUST>& xs, int head, int end, double& residual);
  void clear();
};

// OctoTree — octree.hpp:21-97
struct OctoTree {
  MapParams* mpar;
  SlideWindow* sw = nullptr;
  PointCluster pcr_add;
  M9 cov_add;
  PointCluster pcr_fix;
  PVec point_fix;
  int layer, octo_state, wdsize;
  OctoTree* leaves[8];
  double voxel_center[3] = {0, 0, 0};
  double jour = 0;
  float quater_length = 0;
  Plane plane;
  bool isexist = false;
  V3 eig_value;
  M3 eig_vector;
  int last_num = 0, opt_state = -1;
  std::mutex mVox;

  OctoTree(MapParams* m, int l, int w);
  void push(int ord, const pointVar& pv, const V3& pw, std::vector<SlideWindow*>& sws);
  void push_fix(pointVar& pv);
  void push_fix_novar(pointVar& pv);
  bool plane_judge(const V3& ev) const;
  void allocate(int ord, const pointVar& pv, const V3& pw, std::vector<SlideWindow*>& sws);
  void allocate_fix(pointVar& pv);
  void fix_divide(std::vector<SlideWindow*>& sws);
  void subdivide(int si, const IMUST& xx, std::vector<SlideWindow*>& sws);
  void plane_update();
  void recut(int win_count, const std::vector<IMUST>& x_buf, std::vector<SlideWindow*>& sws);
  void margi(int win_count, int mgsize, const std::vector<IMUST>& x_buf, const LidarFactor& vox_opt);
  void tras_opt(LidarFactor& vox_opt);
  int match(const V3& wld, Plane*& pla, double& max_prob, const M3& var_wld, double& sigma_d, OctoTree*& oc);
  void tras_ptr(std::vector<OctoTree*>& out);
  void delete_ptr();
  bool fitScanPlane();
  bool inside(const V3& wld) const;
  void clear_slwd(std::vector<SlideWindow*>& sws);
  OctoTree* make_child(int leafnum, const int xyz[3]);
};

using SurfMap = VoxMap<OctoTree*>;

// voxel_map.cpp
void cut_voxel_multi(MapParams* mpar, SurfMap& feat_map, PVec& pvec, int win_count, SurfMap& feat_tem_map,
                     int wdsize, std::vector<V3>& pwld, std::vector<std::vector<SlideWindow*>>& sws,
                     bool use_threads);
void generate_voxel(MapParams* mpar, SurfMap& feat_map, PVec& pvec, double voxel_size);
int match(MapParams* mpar, SurfMap& feat_map, const V3& wld, Plane*& pla, const M3& var_wld, double& sigma_d,
          OctoTree*& oc);
int matchVoxelMap(MapParams* mpar, SurfMap& feat_map, const V3& wld, Plane*& pla, const M3& var_wld,
                  double& sigma_d, OctoTree*& oc);

// IMU sample (sensor_msgs::Imu subset)
struct ImuSample {
  double t;
  V3 gyr, acc;
};

// IMU_PRE — preintegration.hpp:12-51, imu_preintegration.cpp:7-246
struct IMU_PRE {
  const MapParams* mpar;
  M3 R_delta;
  V3 p_delta, v_delta, bg, ba;
  M3 R_bg, p_bg, p_ba, v_bg, v_ba;
  double dtime = 0;
  M15 cov;
  V3 dbg, dba, dbg_buf, dba_buf;
  IMU_PRE(const MapParams* m, const V3& bg1, const V3& ba1);
  void push_imu(const std::vector<ImuSample>& buf);
  void add_imu(V3 gyr, V3 acc, double dt);
  double give_evaluate(const IMUST& st1, const IMUST& st2, Mat<30, 30>& jtj, Mat<30, 1>& gg, bool jac,
                       V15* rr_out = nullptr, Mat<15, 30>* joc_out = nullptr) const;
  // with the 3 gravity columns (imu_preintegration.cpp:165-237): jtj 33 x 33, gg 33
  double give_evaluate_g(const IMUST& st1, const IMUST& st2, Mat<33, 33>& jtj, Mat<33, 1>& gg, bool jac) const;
  void update_state(const V15& dxi);
};

// LI_BA_Optimizer — optimizers.hpp:27-57, optimizers.cpp:171-245, 340-376, 430-517
struct LI_BA_Optimizer {
  MapParams* mpar;
  int win_size = 0, jac_leng = 0, imu_leng = 0;
  bool use_threads = true;
  void hess_plus(MatX& Hess, std::vector<double>& JacT, const MatX& hs, const std::vector<double>& js);
  double divide_thread(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus, MatX& Hess,
                       std::vector<double>& JacT);
  double only_residual(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus);
  int damping_iter(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus);
};

// LI_BA_OptimizerGravity — optimizers.cpp:629-826 (initialisation only): the
// same LM with a shared gravity vector as 3 extra unknowns and only frame 0's
// rotation / position gauged
struct LI_BA_OptimizerGravity {
  MapParams* mpar;
  int win_size = 0, jac_leng = 0, imu_leng = 0;
  bool use_threads = true;
  void hess_plus(MatX& Hess, std::vector<double>& JacT, const MatX& hs, const std::vector<double>& js);
  double divide_thread(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus, MatX& Hess,
                       std::vector<double>& JacT);
  double only_residual(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus);
  void damping_iter(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus,
                    std::vector<double>& resis, int max_iter);
};

}  // namespace orc
