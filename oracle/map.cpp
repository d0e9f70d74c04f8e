// ORACLE — test infrastructure only. Never linked into the product library.
// Restatement of src/mapping/{octree,voxel_map,factors,optimizers}.cpp and
// src/estimation/imu_preintegration.cpp (file:line cited per function).
#include "map.hpp"
#include <cstdio>
#include <thread>

namespace orc {

// ---------------------------------------------------------------- OctoTree
// OctoTree::OctoTree — octree.cpp:144-149
OctoTree::OctoTree(MapParams* m, int l, int w) : mpar(m), layer(l), octo_state(0), wdsize(w) {
  for (int i = 0; i < 8; i++) leaves[i] = nullptr;
  cov_add.setZero();
}

OctoTree* OctoTree::make_child(int leafnum, const int xyz[3]) {
  if (leaves[leafnum] == nullptr) {
    OctoTree* c = new OctoTree(mpar, layer + 1, wdsize);
    c->voxel_center[0] = voxel_center[0] + (2 * xyz[0] - 1) * quater_length;
    c->voxel_center[1] = voxel_center[1] + (2 * xyz[1] - 1) * quater_length;
    c->voxel_center[2] = voxel_center[2] + (2 * xyz[2] - 1) * quater_length;
    c->quater_length = quater_length / 2;
    leaves[leafnum] = c;
  }
  return leaves[leafnum];
}

static inline int octant(const double* pt, const double* center, int xyz[3]) {
  for (int k = 0; k < 3; k++) xyz[k] = (pt[k] > center[k]) ? 1 : 0;
  return 4 * xyz[0] + 2 * xyz[1] + xyz[2];
}

// OctoTree::push — octree.cpp:151-177
void OctoTree::push(int ord, const pointVar& pv, const V3& pw, std::vector<SlideWindow*>& sws) {
  std::lock_guard<std::mutex> lk(mVox);
  if (sw == nullptr) {
    if (!sws.empty()) {
      sw = sws.back();
      sws.pop_back();
      sw->resize(wdsize);
    } else
      sw = new SlideWindow(wdsize);
  }
  if (!isexist) isexist = true;
  int mord = mpar->mp[ord];
  if (layer < mpar->max_layer) sw->points[mord].push_back(pv);
  sw->pcrs_local[mord].push(pv.pnt);
  pcr_add.push(pw);
  M9 Bi;
  Bf_var(pv, Bi, pw);
  cov_add += Bi;
}

// OctoTree::push_fix — octree.cpp:179-188
void OctoTree::push_fix(pointVar& pv) {
  if (layer < mpar->max_layer) point_fix.push_back(pv);
  pcr_fix.push(pv.pnt);
  pcr_add.push(pv.pnt);
  M9 Bi;
  Bf_var(pv, Bi, pv.pnt);
  cov_add += Bi;
}

// OctoTree::push_fix_novar — octree.cpp:190-196
void OctoTree::push_fix_novar(pointVar& pv) {
  if (layer < mpar->max_layer) point_fix.push_back(pv);
  pcr_fix.push(pv.pnt);
  pcr_add.push(pv.pnt);
}

// OctoTree::plane_judge — octree.cpp:198-201
bool OctoTree::plane_judge(const V3& ev) const {
  return ev[0] < mpar->min_eigen_value && (ev[0] / ev[2]) < mpar->plane_eigen_value_thre[layer];
}

// OctoTree::allocate — octree.cpp:203-228
void OctoTree::allocate(int ord, const pointVar& pv, const V3& pw, std::vector<SlideWindow*>& sws) {
  if (octo_state == 0) {
    push(ord, pv, pw, sws);
  } else {
    int xyz[3];
    int ln = octant(pw.d, voxel_center, xyz);
    make_child(ln, xyz)->allocate(ord, pv, pw, sws);
  }
}

// OctoTree::allocate_fix — octree.cpp:230-255
void OctoTree::allocate_fix(pointVar& pv) {
  if (octo_state == 0) {
    push_fix_novar(pv);
  } else if (layer < mpar->max_layer) {
    int xyz[3];
    int ln = octant(pv.pnt.d, voxel_center, xyz);
    make_child(ln, xyz)->allocate_fix(pv);
  }
}

// OctoTree::fix_divide — octree.cpp:257-277
void OctoTree::fix_divide(std::vector<SlideWindow*>&) {
  for (pointVar& pv : point_fix) {
    int xyz[3];
    int ln = octant(pv.pnt.d, voxel_center, xyz);
    make_child(ln, xyz)->push_fix(pv);
  }
}

// OctoTree::subdivide — octree.cpp:279-300
void OctoTree::subdivide(int si, const IMUST& xx, std::vector<SlideWindow*>& sws) {
  for (pointVar& pv : sw->points[mpar->mp[si]]) {
    V3 pw = xx.R * pv.pnt + xx.p;
    int xyz[3];
    int ln = octant(pw.d, voxel_center, xyz);
    make_child(ln, xyz)->push(si, pv, pw, sws);
  }
}

// OctoTree::plane_update — octree.cpp:302-333
void OctoTree::plane_update() {
  plane.center = pcr_add.v / (double)pcr_add.N;
  const int l = 0;
  V3 u[3] = {col(eig_vector, 0), col(eig_vector, 1), col(eig_vector, 2)};
  double nv = 1.0 / pcr_add.N;
  Mat<3, 9> u_c;
  for (int k = 0; k < 3; k++)
    if (k != l) {
      M3 ukl = outer(u[k], u[l]);
      Mat<1, 9> fkl;
      fkl[0] = ukl(0, 0);
      fkl[1] = ukl(1, 0) + ukl(0, 1);
      fkl[2] = ukl(2, 0) + ukl(0, 2);
      fkl[3] = ukl(1, 1);
      fkl[4] = ukl(1, 2) + ukl(2, 1);
      fkl[5] = ukl(2, 2);
      V3 t = (u[l] * dot(u[k], plane.center) + u[k] * dot(u[l], plane.center)) * -1.0;
      fkl[6] = t[0]; fkl[7] = t[1]; fkl[8] = t[2];
      u_c += (u[k] * (nv / (eig_value[l] - eig_value[k]))) * fkl;
    }
  Mat<3, 9> Jc = u_c * cov_add;
  plane.plane_var.setBlock(0, 0, Jc * u_c.T());
  M3 Jc_N = Jc.block<3, 3>(0, 6) * nv;
  plane.plane_var.setBlock(0, 3, Jc_N);
  plane.plane_var.setBlock(3, 0, Jc_N.T());
  plane.plane_var.setBlock(3, 3, cov_add.block<3, 3>(6, 6) * (nv * nv));
  plane.normal = u[0];
  plane.radius = eig_value[2];
}

// OctoTree::recut — octree.cpp:335-393 (normal_prev bookkeeping at 337-347 is
// VNC-only state and is omitted: it feeds nothing on the live path)
void OctoTree::recut(int win_count, const std::vector<IMUST>& x_buf, std::vector<SlideWindow*>& sws) {
  if (octo_state == 0) {
    if (layer >= 0) {
      opt_state = -1;
      if (pcr_add.N <= mpar->min_point[layer]) {
        plane.is_plane = false;
        return;
      }
      if (!isexist || sw == nullptr) return;
      eig3(pcr_add.cov(), eig_value, eig_vector);
      plane.is_plane = plane_judge(eig_value);
      if (plane.is_plane)
        return;
      else if (layer >= mpar->max_layer)
        return;
    }
    if (pcr_fix.N != 0) {
      fix_divide(sws);
      PVec().swap(point_fix);
    }
    for (int i = 0; i < win_count; i++) subdivide(i, x_buf[i], sws);
    sw->clear();
    sws.push_back(sw);
    sw = nullptr;
    octo_state = 1;
  }
  for (int i = 0; i < 8; i++)
    if (leaves[i] != nullptr) leaves[i]->recut(win_count, x_buf, sws);
}

// OctoTree::margi — octree.cpp:395-495
void OctoTree::margi(int win_count, int mgsize, const std::vector<IMUST>& x_buf, const LidarFactor& vox_opt) {
  if (octo_state == 0 && layer >= 0) {
    if (!isexist || sw == nullptr) return;
    std::lock_guard<std::mutex> lk(mVox);
    std::vector<PointCluster> pcrs_world(wdsize);
    if (opt_state >= int(vox_opt.pcr_adds.size())) {
      fprintf(stderr, "Error: opt_state: %d %zu\n", opt_state, vox_opt.pcr_adds.size());
      std::abort();
    }
    const std::vector<int>& mp = mpar->mp;
    if (opt_state >= 0) {
      pcr_add = vox_opt.pcr_adds[opt_state];
      eig_value = vox_opt.eig_values[opt_state];
      eig_vector = vox_opt.eig_vectors[opt_state];
      opt_state = -1;
      for (int i = 0; i < mgsize; i++)
        if (sw->pcrs_local[mp[i]].N != 0) pcrs_world[i].transform(sw->pcrs_local[mp[i]], x_buf[i]);
    } else {
      pcr_add = pcr_fix;
      for (int i = 0; i < win_count; i++)
        if (sw->pcrs_local[mp[i]].N != 0) {
          pcrs_world[i].transform(sw->pcrs_local[mp[i]], x_buf[i]);
          pcr_add += pcrs_world[i];
        }
      if (plane.is_plane) eig3(pcr_add.cov(), eig_value, eig_vector);
    }
    if (pcr_fix.N < mpar->max_points && plane.is_plane)
      if (pcr_add.N - last_num >= 5 || last_num <= 10) {
        plane_update();
        last_num = pcr_add.N;
        mpar->cnt_plane_update++;
      }
    if (pcr_fix.N >= mpar->max_points) mpar->cnt_fix_full++;
    if (pcr_fix.N < mpar->max_points) {
      for (int i = 0; i < mgsize; i++)
        if (pcrs_world[i].N != 0) {
          pcr_fix += pcrs_world[i];
          for (pointVar pv : sw->points[mp[i]]) {
            pv.pnt = x_buf[i].R * pv.pnt + x_buf[i].p;
            point_fix.push_back(pv);
          }
        }
    } else {
      for (int i = 0; i < mgsize; i++)
        if (pcrs_world[i].N != 0) pcr_add -= pcrs_world[i];
      if (!point_fix.empty()) PVec().swap(point_fix);
    }
    for (int i = 0; i < mgsize; i++)
      if (sw->pcrs_local[mp[i]].N != 0) {
        sw->pcrs_local[mp[i]].clear();
        sw->points[mp[i]].clear();
      }
    isexist = !(pcr_fix.N >= pcr_add.N);
  } else {
    isexist = false;
    for (int i = 0; i < 8; i++)
      if (leaves[i] != nullptr) {
        leaves[i]->margi(win_count, mgsize, x_buf, vox_opt);
        isexist = isexist || leaves[i]->isexist;
      }
  }
}

// OctoTree::tras_opt(LidarFactor&) — octree.cpp:498-521
void OctoTree::tras_opt(LidarFactor& vox_opt) {
  if (octo_state == 0) {
    if (layer >= 0 && isexist && plane.is_plane && sw != nullptr) {
      if (eig_value[0] / eig_value[1] > 0.12) return;
      double coe = 1;
      std::vector<PointCluster> pcrs(wdsize);
      for (int i = 0; i < wdsize; i++) pcrs[i] = sw->pcrs_local[mpar->mp[i]];
      opt_state = (int)vox_opt.plvec_voxels.size();
      vox_opt.push_voxel(pcrs, pcr_fix, coe, eig_value, eig_vector, pcr_add);
    }
  } else {
    for (int i = 0; i < 8; i++)
      if (leaves[i] != nullptr) leaves[i]->tras_opt(vox_opt);
  }
}

// OctoTree::match — octree.cpp:551-595 (max_prob is never written, as in the reference)
int OctoTree::match(const V3& wld, Plane*& pla, double& max_prob, const M3& var_wld, double& sigma_d,
                    OctoTree*& oc) {
  int flag = 0;
  if (octo_state == 0) {
    if (plane.is_plane) {
      float dis_to_plane = std::fabs(dot(plane.normal, wld - plane.center));
      float dis_to_center = squaredNorm(plane.center - wld);
      float range_dis = (dis_to_center - dis_to_plane * dis_to_plane);
      if (range_dis <= 3 * 3 * plane.radius) {
        Mat<1, 6> J;
        V3 d = wld - plane.center;
        J[0] = d[0]; J[1] = d[1]; J[2] = d[2];
        J[3] = -plane.normal[0]; J[4] = -plane.normal[1]; J[5] = -plane.normal[2];
        double sigma_l = (J * plane.plane_var * J.T())[0];
        sigma_l += dot(plane.normal, var_wld * plane.normal);
        if (dis_to_plane < 3 * std::sqrt(sigma_l)) {
          oc = this;
          sigma_d = sigma_l;
          pla = &plane;
          flag = 1;
        }
      }
    }
  } else {
    int xyz[3];
    int ln = octant(wld.d, voxel_center, xyz);
    if (leaves[ln] != nullptr) flag = leaves[ln]->match(wld, pla, max_prob, var_wld, sigma_d, oc);
  }
  return flag;
}

// OctoTree::tras_ptr — octree.cpp:597-608
void OctoTree::tras_ptr(std::vector<OctoTree*>& out) {
  if (octo_state == 1)
    for (int i = 0; i < 8; i++)
      if (leaves[i] != nullptr) {
        out.push_back(leaves[i]);
        leaves[i]->tras_ptr(out);
      }
}

// OctoTree::delete_ptr — octree.cpp:610-626
void OctoTree::delete_ptr() {
  for (int i = 0; i < 8; i++)
    if (leaves[i] != nullptr) {
      leaves[i]->delete_ptr();
      delete leaves[i];
      leaves[i] = nullptr;
    }
  if (sw != nullptr) {
    delete sw;
    sw = nullptr;
  }
}

// OctoTree::fitScanPlane — octree.cpp:628-684 (VNC scan-plane prep; output unused)
bool OctoTree::fitScanPlane() {
  plane.is_plane = false;
  isexist = (pcr_add.N != 0);
  if (octo_state == 1) {
    bool has = false;
    for (int i = 0; i < 8; i++)
      if (leaves[i] != nullptr) has = leaves[i]->fitScanPlane() || has;
    isexist = has;
    return has;
  }
  if (pcr_add.N < 3) return false;
  eig3(pcr_add.cov(), eig_value, eig_vector);
  plane.is_plane = plane_judge(eig_value);
  if (plane.is_plane) {
    plane.center = pcr_add.v / (double)pcr_add.N;
    plane.normal = col(eig_vector, 0);
    return true;
  }
  if (layer >= mpar->max_layer || pcr_add.N < 6 || point_fix.empty()) return false;
  octo_state = 1;
  for (pointVar& pv : point_fix) allocate_fix(pv);
  PVec().swap(point_fix);
  bool has = false;
  for (int i = 0; i < 8; i++)
    if (leaves[i] != nullptr) has = leaves[i]->fitScanPlane() || has;
  isexist = has;
  return has;
}

// OctoTree::inside — octree.cpp:732-737
bool OctoTree::inside(const V3& wld) const {
  double hl = quater_length * 2;
  return (wld[0] >= voxel_center[0] - hl && wld[0] <= voxel_center[0] + hl && wld[1] >= voxel_center[1] - hl &&
          wld[1] <= voxel_center[1] + hl && wld[2] >= voxel_center[2] - hl && wld[2] <= voxel_center[2] + hl);
}

// OctoTree::clear_slwd — octree.cpp:739-756
void OctoTree::clear_slwd(std::vector<SlideWindow*>& sws) {
  if (octo_state != 0)
    for (int i = 0; i < 8; i++)
      if (leaves[i] != nullptr) leaves[i]->clear_slwd(sws);
  if (sw != nullptr) {
    sw->clear();
    sws.push_back(sw);
    sw = nullptr;
  }
}

// ---------------------------------------------------------------- voxel_map.cpp
// cut_voxel_multi — voxel_map.cpp:47-135. Per-octree point lists keep point
// order; octrees are handed to threads in first-touch order (the reference
// iterates an unordered_map<OctoTree*,...> keyed by pointer value; the
// partition does not change any value because each octree is owned by exactly
// one thread).
void cut_voxel_multi(MapParams* mpar, SurfMap& feat_map, PVec& pvec, int win_count, SurfMap& feat_tem_map,
                     int wdsize, std::vector<V3>& pwld, std::vector<std::vector<SlideWindow*>>& sws,
                     bool use_threads) {
  std::vector<std::pair<OctoTree*, std::vector<int>>> octs;
  std::unordered_map<OctoTree*, int> slot;
  int plsize = (int)pvec.size();
  for (int i = 0; i < plsize; i++) {
    VOXEL_LOC position = voxel_key(pwld[i], mpar->voxel_size);
    if (!shard_owns(mpar, position)) continue;  // another shard's tile (sharded mode)
    auto iter = feat_map.find(position);
    OctoTree* ot = nullptr;
    if (iter != feat_map.end()) {
      iter->second->isexist = true;
      // reference: feat_tem_map.find(position) == feat_map.end() — libstdc++
      // end() iterators of both maps compare equal (null node), i.e. "absent".
      if (feat_tem_map.find(position) == feat_tem_map.end()) feat_tem_map[position] = iter->second;
      ot = iter->second;
    } else {
      ot = new OctoTree(mpar, 0, wdsize);
      ot->voxel_center[0] = (0.5 + position.x) * mpar->voxel_size;
      ot->voxel_center[1] = (0.5 + position.y) * mpar->voxel_size;
      ot->voxel_center[2] = (0.5 + position.z) * mpar->voxel_size;
      ot->quater_length = mpar->voxel_size / 4.0;
      feat_map[position] = ot;
      feat_tem_map[position] = ot;
    }
    auto s = slot.find(ot);
    if (s == slot.end()) {
      slot[ot] = (int)octs.size();
      octs.push_back({ot, {i}});
    } else
      octs[s->second].second.push_back(i);
  }
  int thd_num = (int)sws.size();
  int g_size = (int)octs.size();
  if (shard_count(mpar, g_size) < thd_num) return;  // voxel_map.cpp:96-97, over all shards
  double part = 1.0 * g_size / thd_num;
  int swsize = (int)sws[0].size() / thd_num;
  for (int i = 1; i < thd_num; i++) {
    sws[i].insert(sws[i].end(), sws[0].end() - swsize, sws[0].end());
    sws[0].erase(sws[0].end() - swsize, sws[0].end());
  }
  auto work = [&](int head, int tail, std::vector<SlideWindow*>& sw) {
    for (int j = head; j < tail; j++)
      for (int k : octs[j].second) octs[j].first->allocate(win_count, pvec[k], pwld[k], sw);
  };
  std::vector<std::thread> th;
  for (int i = 1; i < thd_num; i++) {
    int head = (int)(part * i), tail = (int)(part * (i + 1));
    if (use_threads)
      th.emplace_back(work, head, tail, std::ref(sws[i]));
    else
      work(head, tail, sws[i]);
  }
  work(0, (int)part, sws[0]);
  for (auto& t : th) t.join();
}

// generate_voxel — voxel_map.cpp:169-200 (VNC scan voxelisation, output unused)
void generate_voxel(MapParams* mpar, SurfMap& feat_map, PVec& pvec, double voxel_size) {
  for (pointVar& pv : pvec) {
    VOXEL_LOC position = voxel_key(pv.pnt, voxel_size);
    auto iter = feat_map.find(position);
    if (iter != feat_map.end()) {
      iter->second->allocate_fix(pv);
    } else {
      OctoTree* ot = new OctoTree(mpar, 0, 1);
      ot->push_fix_novar(pv);
      ot->voxel_center[0] = (0.5 + position.x) * voxel_size;
      ot->voxel_center[1] = (0.5 + position.y) * voxel_size;
      ot->voxel_center[2] = (0.5 + position.z) * voxel_size;
      ot->quater_length = voxel_size / 4.0;
      ot->isexist = true;
      feat_map[position] = ot;
    }
  }
}

// match — voxel_map.cpp:241-266
int match(MapParams* mpar, SurfMap& feat_map, const V3& wld, Plane*& pla, const M3& var_wld, double& sigma_d,
          OctoTree*& oc) {
  int flag = 0;
  VOXEL_LOC position = voxel_key(wld, mpar->voxel_size);
  auto iter = feat_map.find(position);
  if (iter != feat_map.end()) {
    double max_prob = 0;
    flag = iter->second->match(wld, pla, max_prob, var_wld, sigma_d, oc);
  }
  return flag;
}

// matchVoxelMap — voxel_map.cpp:268-313 (double key rule; always returns 0)
int matchVoxelMap(MapParams* mpar, SurfMap& feat_map, const V3& wld, Plane*& pla, const M3& var_wld,
                  double& sigma_d, OctoTree*& oc) {
  double loc[3];
  for (int j = 0; j < 3; j++) {
    loc[j] = wld[j] / mpar->voxel_size;
    if (loc[j] < 0) loc[j] -= 1.0;
  }
  VOXEL_LOC position((int64_t)loc[0], (int64_t)loc[1], (int64_t)loc[2]);
  double max_prob = 0;
  for (int ix = -1; ix <= 1; ix++)
    for (int iy = -1; iy <= 1; iy++)
      for (int iz = -1; iz <= 1; iz++) {
        VOXEL_LOC l(position.x + ix, position.y + iy, position.z + iz);
        auto iter = feat_map.find(l);
        if (iter != feat_map.end()) {
          Plane* pt = nullptr;
          double prob = 0, sig = 0;
          OctoTree* oct = nullptr;
          if (iter->second->match(wld, pt, prob, var_wld, sig, oct) > 0) {
            if (prob > max_prob) {
              max_prob = prob;
              pla = pt;
              sigma_d = sig;
              oc = oct;
            }
          }
        }
      }
  return (max_prob > 0) ? 1 : 0;
}

// ---------------------------------------------------------------- LidarFactor
// push_voxel — factors.cpp:11-20
void LidarFactor::push_voxel(std::vector<PointCluster>& vec_orig, PointCluster& fix, double coe, V3& eig_value,
                             M3& eig_vector, PointCluster& pcr_add) {
  plvec_voxels.push_back(vec_orig);
  sig_vecs.push_back(fix);
  coeffs.push_back(coe);
  eig_values.push_back(eig_value);
  eig_vectors.push_back(eig_vector);
  pcr_adds.push_back(pcr_add);
}

// acc_evaluate2 — factors.cpp:22-126
void LidarFactor::acc_evaluate2(const std::vector<IMUST>& xs, int head, int end, MatX& Hess,
                                std::vector<double>& JacT, double& residual) const {
  Hess.setZero();
  std::fill(JacT.begin(), JacT.end(), 0.0);
  residual = 0;
  const int kk = 0;
  std::vector<V3> viRiTuk(win_size);
  std::vector<M3> viRiTukukT(win_size);
  std::vector<Mat<3, 6>> Auk(win_size);
  const M3 I33 = M3::Identity();
  for (int a = head; a < end; a++) {
    const std::vector<PointCluster>& sig_orig = plvec_voxels[a];
    double coe = coeffs[a];
    V3 lmbd = eig_values[a];
    M3 U = eig_vectors[a];
    int NN = pcr_adds[a].N;
    V3 vBar = pcr_adds[a].v / (double)NN;
    V3 u[3] = {col(U, 0), col(U, 1), col(U, 2)};
    V3& uk = u[kk];
    M3 ukukT = outer(uk, uk);
    M3 umumT;
    for (int i = 0; i < 3; i++)
      if (i != kk) umumT += outer(u[i], u[i]) * (2.0 / (lmbd[kk] - lmbd[i]));
    for (int i = 0; i < win_size; i++) {
      if (sig_orig[i].N != 0) {
        M3 Pi = sig_orig[i].P;
        V3 vi = sig_orig[i].v;
        M3 Ri = xs[i].R;
        double ni = sig_orig[i].N;
        M3 vihat = hat(vi);
        V3 RiTuk = Ri.T() * uk;
        M3 RiTukhat = hat(RiTuk);
        V3 PiRiTuk = Pi * RiTuk;
        viRiTuk[i] = vihat * RiTuk;
        viRiTukukT[i] = outer(viRiTuk[i], uk);
        V3 ti_v = xs[i].p - vBar;
        double ukTti_v = dot(uk, ti_v);
        M3 combo1 = hat(PiRiTuk) + vihat * ukTti_v;
        V3 combo2 = Ri * vi + ti_v * ni;
        Auk[i].setBlock(0, 0, (Ri * Pi + outer(ti_v, vi)) * RiTukhat - Ri * combo1);
        Auk[i].setBlock(0, 3, outer(combo2, uk) + I33 * dot(combo2, uk));
        Auk[i] /= (double)NN;
        V6 jjt = Auk[i].T() * uk;
        for (int r = 0; r < 6; r++) JacT[6 * i + r] += coe * jjt[r];
        M3 HRt = viRiTukukT[i] * (2.0 / NN * (1.0 - ni / NN));
        M6 Hb = (Auk[i].T() * umumT) * Auk[i];
        Hb.addBlock(0, 0, ((combo1 - RiTukhat * Pi) * RiTukhat) * (2.0 / NN) -
                              outer(viRiTuk[i], viRiTuk[i]) * (2.0 / NN / NN) - hat(jjt.block<3, 1>(0, 0)) * 0.5);
        Hb.addBlock(0, 3, HRt);
        Hb.addBlock(3, 0, HRt.T());
        Hb.addBlock(3, 3, ukukT * (2.0 / NN * (ni - ni * ni / NN)));
        for (int r = 0; r < 6; r++)
          for (int c = 0; c < 6; c++) Hess(6 * i + r, 6 * i + c) += coe * Hb(r, c);
      }
    }
    for (int i = 0; i < win_size - 1; i++)
      if (sig_orig[i].N != 0) {
        double ni = sig_orig[i].N;
        for (int j = i + 1; j < win_size; j++)
          if (sig_orig[j].N != 0) {
            double nj = sig_orig[j].N;
            M6 Hb = (Auk[i].T() * umumT) * Auk[j];
            Hb.addBlock(0, 0, outer(viRiTuk[i], viRiTuk[j]) * (-2.0 / NN / NN));
            Hb.addBlock(0, 3, viRiTukukT[i] * (-2.0 * nj / NN / NN));
            Hb.addBlock(3, 0, viRiTukukT[j].T() * (-2.0 * ni / NN / NN));
            Hb.addBlock(3, 3, ukukT * (-2.0 * ni * nj / NN / NN));
            for (int r = 0; r < 6; r++)
              for (int c = 0; c < 6; c++) Hess(6 * i + r, 6 * j + c) += coe * Hb(r, c);
          }
      }
    residual += coe * lmbd[kk];
  }
  for (int i = 1; i < win_size; i++)
    for (int j = 0; j < i; j++)
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) Hess(6 * i + r, 6 * j + c) = Hess(6 * j + c, 6 * i + r);
}

// evaluate_only_residual — factors.cpp:128-158 (writes eig/pcr_add at the trial
// poses: the side effect margi consumes, octree.cpp:410-415)
void LidarFactor::evaluate_only_residual(const std::vector<IMUST>& xs, int head, int end, double& residual) {
  residual = 0;
  const int kk = 0;
  PointCluster pcr;
  for (int a = head; a < end; a++) {
    const std::vector<PointCluster>& sig_orig = plvec_voxels[a];
    PointCluster sig = sig_vecs[a];
    for (int i = 0; i < win_size; i++)
      if (sig_orig[i].N != 0) {
        pcr.transform(sig_orig[i], xs[i]);
        sig += pcr;
      }
    V3 vBar = sig.v / (double)sig.N;
    V3 lmbd;
    M3 U;
    eig3(sig.P / (double)sig.N - outer(vBar, vBar), lmbd, U);
    eig_values[a] = lmbd;
    eig_vectors[a] = U;
    pcr_adds[a] = sig;
    residual += coeffs[a] * lmbd[kk];
  }
}

void LidarFactor::clear() {
  sig_vecs.clear();
  plvec_voxels.clear();
  eig_values.clear();
  eig_vectors.clear();
  pcr_adds.clear();
  coeffs.clear();
}

// ---------------------------------------------------------------- IMU_PRE
// IMU_PRE::IMU_PRE — imu_preintegration.cpp:7-29
IMU_PRE::IMU_PRE(const MapParams* m, const V3& bg1, const V3& ba1) : mpar(m) {
  bg = bg1;
  ba = ba1;
  R_delta = M3::Identity();
  dtime = 0;
}

// push_imu — imu_preintegration.cpp:31-55
void IMU_PRE::push_imu(const std::vector<ImuSample>& buf) {
  for (size_t k = 1; k < buf.size(); k++) {
    const ImuSample& a = buf[k - 1];
    const ImuSample& b = buf[k];
    double dt = b.t - a.t;
    V3 gyr, acc;
    for (int j = 0; j < 3; j++) {
      gyr[j] = 0.5 * (a.gyr[j] + b.gyr[j]);
      acc[j] = 0.5 * (a.acc[j] + b.acc[j]);
    }
    gyr = gyr - bg;
    acc = acc * mpar->imupre_scale_gravity - ba;
    add_imu(gyr, acc, dt);
  }
}

// add_imu — imu_preintegration.cpp:57-95
void IMU_PRE::add_imu(V3 cur_gyr, V3 cur_acc, double dt) {
  dtime += dt;
  M3 rinc = Exp(cur_gyr, dt);
  M3 rj = jr(cur_gyr * dt);
  M3 rdt = R_delta * dt;
  M3 rdt2 = R_delta * (0.5 * dt * dt);
  M3 acc_skew = hat(cur_acc);
  p_ba = p_ba + v_ba * dt - rdt2;
  p_bg = p_bg + v_bg * dt - (rdt2 * acc_skew) * R_bg;
  v_ba = v_ba - rdt;
  v_bg = v_bg - (rdt * acc_skew) * R_bg;
  R_bg = rinc.T() * R_bg - rj * dt;
  M9 A = M9::Identity();
  Mat<9, 6> B;
  A.setBlock(0, 0, rinc.T());
  A.setBlock(3, 0, (rdt2 * acc_skew) * -1.0);
  A.setBlock(3, 6, M3::Identity() * dt);
  A.setBlock(6, 0, (rdt * acc_skew) * -1.0);
  B.setBlock(0, 0, rj * dt);
  B.setBlock(3, 3, rdt2);
  B.setBlock(6, 3, rdt);
  M9 c9 = cov.block<9, 9>(0, 0);
  cov.setBlock(0, 0, (A * c9) * A.T() + (B * mpar->noiseMeas) * B.T());
  cov.addBlock(9, 9, mpar->noiseWalk * dt);
  p_delta += v_delta * dt + rdt2 * cur_acc;
  v_delta += rdt * cur_acc;
  R_delta = R_delta * rinc;
}

// give_evaluate — imu_preintegration.cpp:97-163
double IMU_PRE::give_evaluate(const IMUST& st1, const IMUST& st2, Mat<30, 30>& jtj, Mat<30, 1>& gg,
                              bool jac, V15* rr_out, Mat<15, 30>* joc_out) const {
  M15 joca, jocb;
  V15 rr;
  M3 R_correct = R_delta * Exp(R_bg * dbg);
  V3 t_correct = p_delta + p_bg * dbg + p_ba * dba;
  V3 v_correct = v_delta + v_bg * dbg + v_ba * dba;
  M3 res_r = (R_correct.T() * st1.R.T()) * st2.R;
  V3 exp_v = st1.R.T() * (st2.v - st1.v - st1.g * dtime);
  V3 res_v = exp_v - v_correct;
  V3 exp_t = st1.R.T() * (st2.p - st1.p - st1.v * dtime - st1.g * (0.5 * dtime * dtime));
  V3 res_t = exp_t - t_correct;
  V3 res_bg = st2.bg - st1.bg;
  V3 res_ba = st2.ba - st1.ba;
  const double b_wei = 1;
  rr.setBlock(0, 0, Log(res_r));
  rr.setBlock(3, 0, res_t);
  rr.setBlock(6, 0, res_v);
  rr.setBlock(9, 0, res_bg * b_wei);
  rr.setBlock(12, 0, res_ba * b_wei);
  M15 cov_inv = inverse(cov);
  if (jac) {
    const M3 I33 = M3::Identity();
    M3 JR_inv = jr_inv(res_r);
    joca.setBlock(0, 0, ((JR_inv * st2.R.T()) * st1.R) * -1.0);
    jocb.setBlock(0, 0, JR_inv);
    joca.setBlock(0, 9, (((JR_inv * res_r.T()) * jr(R_bg * dbg)) * R_bg) * -1.0);
    joca.setBlock(3, 0, hat(exp_t));
    joca.setBlock(3, 3, st1.R.T() * -1.0);
    joca.setBlock(3, 6, st1.R.T() * -dtime);
    joca.setBlock(3, 9, p_bg * -1.0);
    joca.setBlock(3, 12, p_ba * -1.0);
    jocb.setBlock(3, 3, st1.R.T());
    joca.setBlock(6, 0, hat(exp_v));
    joca.setBlock(6, 6, st1.R.T() * -1.0);
    joca.setBlock(6, 9, v_bg * -1.0);
    joca.setBlock(6, 12, v_ba * -1.0);
    jocb.setBlock(6, 6, st1.R.T());
    joca.setBlock(9, 9, I33 * -b_wei);
    joca.setBlock(12, 12, I33 * -b_wei);
    jocb.setBlock(9, 9, I33 * b_wei);
    jocb.setBlock(12, 12, I33 * b_wei);
    Mat<15, 30> joc;
    joc.setBlock(0, 0, joca);
    joc.setBlock(0, 15, jocb);
    Mat<30, 15> jT = joc.T();
    jtj = (jT * cov_inv) * joc;
    gg = (jT * cov_inv) * rr;
    if (joc_out) *joc_out = joc;
  }
  if (rr_out) *rr_out = rr;
  return dot(rr, cov_inv * rr);
}

// give_evaluate_g — imu_preintegration.cpp:165-237: give_evaluate's residual
// plus the gravity Jacobian jocg (rows 3-8) of the shared gravity unknowns
double IMU_PRE::give_evaluate_g(const IMUST& st1, const IMUST& st2, Mat<33, 33>& jtj, Mat<33, 1>& gg,
                                bool jac) const {
  Mat<30, 30> j30;
  Mat<30, 1> g30;
  V15 rr;
  Mat<15, 30> joc;
  const double cost = give_evaluate(st1, st2, j30, g30, jac, &rr, &joc);
  if (jac) {
    Mat<15, 33> J;
    for (int r = 0; r < 15; r++)
      for (int c = 0; c < 30; c++) J(r, c) = joc(r, c);
    const double dt = dtime;
    J.setBlock(3, 30, st1.R.T() * (-0.5 * dt * dt));
    J.setBlock(6, 30, st1.R.T() * (-dt));
    const M15 cov_inv = inverse(cov);
    const Mat<33, 15> jT = J.T();
    jtj = (jT * cov_inv) * J;
    gg = (jT * cov_inv) * rr;
  }
  return cost;
}

// update_state — imu_preintegration.cpp:239-246
void IMU_PRE::update_state(const V15& dxi) {
  dbg_buf = dbg;
  dba_buf = dba;
  dbg += dxi.block<3, 1>(9, 0);
  dba += dxi.block<3, 1>(12, 0);
}

// ---------------------------------------------------------------- LI_BA_Optimizer
// hess_plus — optimizers.cpp:171-179
void LI_BA_Optimizer::hess_plus(MatX& Hess, std::vector<double>& JacT, const MatX& hs,
                                const std::vector<double>& js) {
  for (int i = 0; i < win_size; i++) {
    for (int r = 0; r < 6; r++) JacT[i * DIM + r] += js[i * 6 + r];
    for (int j = 0; j < win_size; j++)
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) Hess(i * DIM + r, j * DIM + c) += hs(i * 6 + r, j * 6 + c);
  }
}

// divide_thread — optimizers.cpp:181-245 (5 threads hard-coded, line 184)
double LI_BA_Optimizer::divide_thread(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus,
                                      MatX& Hess, std::vector<double>& JacT) {
  int thd_num = 5;
  double residual = 0;
  Hess.setZero();
  std::fill(JacT.begin(), JacT.end(), 0.0);
  std::vector<MatX> hessians(thd_num, MatX(jac_leng, jac_leng));
  std::vector<std::vector<double>> jacobins(thd_num, std::vector<double>(jac_leng, 0.0));
  std::vector<double> resis(thd_num, 0);
  int tthd_num = thd_num;
  int g_size = (int)vox.plvec_voxels.size();
  if (g_size < tthd_num) tthd_num = 1;
  double part = 1.0 * g_size / tthd_num;
  std::vector<std::thread> th;
  for (int i = 1; i < tthd_num; i++) {
    int head = (int)(part * i), tail = (int)(part * (i + 1));
    if (use_threads)
      th.emplace_back([&, i, head, tail]() { vox.acc_evaluate2(xs, head, tail, hessians[i], jacobins[i], resis[i]); });
    else
      vox.acc_evaluate2(xs, head, tail, hessians[i], jacobins[i], resis[i]);
  }
  Mat<30, 30> jtj;
  Mat<30, 1> gg;
  std::vector<double> cap_imu;
  for (int i = 0; i < win_size - 1; i++) {
    jtj.setZero();
    gg.setZero();
    const double ri = imus[i]->give_evaluate(xs[i], xs[i + 1], jtj, gg, true);
    residual += ri;
    if (mpar->capture == 1) {  // test hook: this IMU factor's blocks
      cap_imu.insert(cap_imu.end(), jtj.d, jtj.d + 900);
      cap_imu.insert(cap_imu.end(), gg.d, gg.d + 30);
      cap_imu.push_back(ri);
    }
    for (int r = 0; r < 2 * DIM; r++) {
      JacT[i * DIM + r] += gg[r];
      for (int c = 0; c < 2 * DIM; c++) Hess(i * DIM + r, i * DIM + c) += jtj(r, c);
    }
  }
  for (double& h : Hess.d) h *= mpar->imu_coef;
  for (double& j : JacT) j *= mpar->imu_coef;
  residual *= (mpar->imu_coef * 0.5);
  vox.acc_evaluate2(xs, 0, (int)part, hessians[0], jacobins[0], resis[0]);
  for (auto& t : th) t.join();
  if (mpar->capture == 1) {  // test hook: the LiDAR part summed over the thread partitions, then the IMU blocks
    std::vector<double>& c = mpar->captured;
    c.assign((size_t)jac_leng * jac_leng + jac_leng + 1, 0.0);
    for (int i = 0; i < tthd_num; i++) {
      for (size_t e = 0; e < (size_t)jac_leng * jac_leng; e++) c[e] += hessians[i].d[e];
      for (int e = 0; e < jac_leng; e++) c[(size_t)jac_leng * jac_leng + e] += jacobins[i][e];
      c.back() += resis[i];
    }
    c.insert(c.end(), cap_imu.begin(), cap_imu.end());
    mpar->capture = 2;
  }
  if (mpar->shard_world > 1) {  // this shard's LiDAR part, summed over the shards, then added
    std::vector<double> l((size_t)jac_leng * jac_leng + jac_leng + 1, 0.0);
    for (int i = 0; i < tthd_num; i++) {
      for (size_t e = 0; e < (size_t)jac_leng * jac_leng; e++) l[e] += hessians[i].d[e];
      for (int e = 0; e < jac_leng; e++) l[(size_t)jac_leng * jac_leng + e] += jacobins[i][e];
      l.back() += resis[i];
    }
    shard_sum(mpar, l.data(), (int)l.size());
    MatX hs(jac_leng, jac_leng);
    for (size_t e = 0; e < (size_t)jac_leng * jac_leng; e++) hs.d[e] = l[e];
    std::vector<double> js(l.begin() + (size_t)jac_leng * jac_leng, l.begin() + (size_t)jac_leng * jac_leng + jac_leng);
    hess_plus(Hess, JacT, hs, js);
    return residual + l.back();
  }
  for (int i = 0; i < tthd_num; i++) {
    hess_plus(Hess, JacT, hessians[i], jacobins[i]);
    residual += resis[i];
  }
  return residual;
}

// only_residual — optimizers.cpp:340-376
double LI_BA_Optimizer::only_residual(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus) {
  double residual1 = 0, residual2 = 0;
  Mat<30, 30> jtj;
  Mat<30, 1> gg;
  int thd_num = 5;
  std::vector<double> residuals(thd_num, 0);
  int g_size = (int)vox.plvec_voxels.size();
  if (g_size < thd_num) thd_num = 1;
  double part = 1.0 * g_size / thd_num;
  std::vector<std::thread> th;
  for (int i = 1; i < thd_num; i++) {
    int head = (int)(part * i), tail = (int)(part * (i + 1));
    if (use_threads)
      th.emplace_back([&, i, head, tail]() { vox.evaluate_only_residual(xs, head, tail, residuals[i]); });
    else
      vox.evaluate_only_residual(xs, head, tail, residuals[i]);
  }
  for (int i = 0; i < win_size - 1; i++) residual1 += imus[i]->give_evaluate(xs[i], xs[i + 1], jtj, gg, false);
  residual1 *= (mpar->imu_coef * 0.5);
  vox.evaluate_only_residual(xs, 0, (int)part, residuals[0]);
  for (auto& t : th) t.join();
  for (int i = 0; i < thd_num; i++) residual2 += residuals[i];
  shard_sum(mpar, &residual2, 1);  // sharded mode: the factor residual over all shards
  return residual1 + residual2;
}

// damping_iter (LiDAR + IMU overload) — optimizers.cpp:430-517. Returns the
// number of LM iterations run.
int LI_BA_Optimizer::damping_iter(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus) {
  win_size = vox.win_size;
  jac_leng = win_size * 6;
  imu_leng = win_size * DIM;
  double u = 0.01, v = 2;
  MatX Hess(imu_leng, imu_leng);
  std::vector<double> JacT(imu_leng, 0.0), D(imu_leng, 0.0);
  double residual1 = 0, residual2, q;
  bool is_calc_hess = true;
  std::vector<IMUST> xs_temp = xs;
  const int max_iter = 10;
  int it = 0;
  MatX Hcalc;
  std::vector<double> Jcalc;
  for (int i = 0; i < max_iter; i++) {
    it++;
    if (is_calc_hess) {
      residual1 = divide_thread(xs, vox, imus, Hess, JacT);
      Hcalc = Hess;
      Jcalc = JacT;
    } else {
      Hess = Hcalc;  // Eigen keeps the gauged Hess across rejected steps (same values)
      JacT = Jcalc;
    }
    for (int r = 0; r < DIM; r++)
      for (int c = 0; c < imu_leng; c++) {
        Hess(r, c) = 0;
        Hess(c, r) = 0;
      }
    for (int r = 0; r < DIM; r++) Hess(r, r) = 1;
    for (int r = 0; r < DIM; r++) JacT[r] = 0;
    for (int r = 0; r < imu_leng; r++) D[r] = Hess(r, r);
    MatX A = Hess;
    for (int r = 0; r < imu_leng; r++) A(r, r) += u * D[r];
    std::vector<double> mJ(imu_leng);
    for (int r = 0; r < imu_leng; r++) mJ[r] = -JacT[r];
    std::vector<double> dxi = ldlt_solve(A, mJ);
    for (int j = 0; j < win_size; j++) {
      V3 dr = v3(dxi[DIM * j], dxi[DIM * j + 1], dxi[DIM * j + 2]);
      xs_temp[j].R = xs[j].R * Exp(dr);
      for (int k = 0; k < 3; k++) {
        xs_temp[j].p[k] = xs[j].p[k] + dxi[DIM * j + 3 + k];
        xs_temp[j].v[k] = xs[j].v[k] + dxi[DIM * j + 6 + k];
        xs_temp[j].bg[k] = xs[j].bg[k] + dxi[DIM * j + 9 + k];
        xs_temp[j].ba[k] = xs[j].ba[k] + dxi[DIM * j + 12 + k];
      }
    }
    for (int j = 0; j < win_size - 1; j++) {
      V15 d;
      for (int k = 0; k < DIM; k++) d[k] = dxi[DIM * j + k];
      imus[j]->update_state(d);
    }
    double q1 = 0;  // 0.5 * dxi.dot(u * D * dxi - JacT)
    for (int r = 0; r < imu_leng; r++) q1 += dxi[r] * (u * D[r] * dxi[r] - JacT[r]);
    q1 *= 0.5;
    residual2 = only_residual(xs_temp, vox, imus);
    q = (residual1 - residual2);
    if (q > 0) {
      xs = xs_temp;
      double one_three = 1.0 / 3;
      q = q / q1;
      v = 2;
      q = 1 - std::pow(2 * q - 1, 3);
      u *= (q < one_three ? one_three : q);
      is_calc_hess = true;
    } else {
      u = u * v;
      v = 2 * v;
      is_calc_hess = false;
      for (int j = 0; j < win_size - 1; j++) {
        imus[j]->dbg = imus[j]->dbg_buf;
        imus[j]->dba = imus[j]->dba_buf;
      }
    }
    if (std::fabs((residual1 - residual2) / residual1) < 1e-6) break;
  }
  return it;
}

// ---------------------------------------------------------------- LI_BA_OptimizerGravity
// hess_plus — optimizers.cpp:629-638
void LI_BA_OptimizerGravity::hess_plus(MatX& Hess, std::vector<double>& JacT, const MatX& hs,
                                       const std::vector<double>& js) {
  for (int i = 0; i < win_size; i++) {
    for (int r = 0; r < 6; r++) JacT[i * DIM + r] += js[i * 6 + r];
    for (int j = 0; j < win_size; j++)
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) Hess(i * DIM + r, j * DIM + c) += hs(i * 6 + r, j * 6 + c);
  }
}

// divide_thread — optimizers.cpp:640-707
double LI_BA_OptimizerGravity::divide_thread(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus,
                                             MatX& Hess, std::vector<double>& JacT) {
  const int thd_num = 5;
  double residual = 0;
  Hess.setZero();
  std::fill(JacT.begin(), JacT.end(), 0.0);
  std::vector<MatX> hessians(thd_num, MatX(jac_leng, jac_leng));
  std::vector<std::vector<double>> jacobins(thd_num, std::vector<double>(jac_leng, 0.0));
  std::vector<double> resis(thd_num, 0);
  int tthd_num = thd_num;
  const int g_size = (int)vox.plvec_voxels.size();
  if (g_size < tthd_num) tthd_num = 1;
  const double part = 1.0 * g_size / tthd_num;
  std::vector<std::thread> th;
  for (int i = 1; i < tthd_num; i++) {
    const int head = (int)(part * i), tail = (int)(part * (i + 1));
    if (use_threads)
      th.emplace_back([&, i, head, tail]() { vox.acc_evaluate2(xs, head, tail, hessians[i], jacobins[i], resis[i]); });
    else
      vox.acc_evaluate2(xs, head, tail, hessians[i], jacobins[i], resis[i]);
  }
  const int g0 = imu_leng - 3;
  Mat<33, 33> jtj;
  Mat<33, 1> gg;
  for (int i = 0; i < win_size - 1; i++) {
    jtj.setZero();
    gg.setZero();
    residual += imus[i]->give_evaluate_g(xs[i], xs[i + 1], jtj, gg, true);
    for (int r = 0; r < 2 * DIM; r++) {
      for (int c = 0; c < 2 * DIM; c++) Hess(i * DIM + r, i * DIM + c) += jtj(r, c);
      for (int c = 0; c < 3; c++) Hess(i * DIM + r, g0 + c) += jtj(r, 2 * DIM + c);
    }
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 2 * DIM; c++) Hess(g0 + r, i * DIM + c) += jtj(2 * DIM + r, c);
      for (int c = 0; c < 3; c++) Hess(g0 + r, g0 + c) += jtj(2 * DIM + r, 2 * DIM + c);
    }
    for (int r = 0; r < 2 * DIM; r++) JacT[i * DIM + r] += gg[r];
    for (int r = 0; r < 3; r++) JacT[g0 + r] += gg[2 * DIM + r];
  }
  for (double& h : Hess.d) h *= mpar->imu_coef;
  for (double& j : JacT) j *= mpar->imu_coef;
  residual *= (mpar->imu_coef * 0.5);
  vox.acc_evaluate2(xs, 0, (int)part, hessians[0], jacobins[0], resis[0]);
  for (auto& t : th) t.join();
  for (int i = 0; i < tthd_num; i++) {
    hess_plus(Hess, JacT, hessians[i], jacobins[i]);
    residual += resis[i];
  }
  return residual;
}

// only_residual — optimizers.cpp:709-743
double LI_BA_OptimizerGravity::only_residual(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus) {
  double residual1 = 0, residual2 = 0;
  Mat<33, 33> jtj;
  Mat<33, 1> gg;
  int thd_num = 5;
  std::vector<double> residuals(thd_num, 0);
  const int g_size = (int)vox.plvec_voxels.size();
  if (g_size < thd_num) thd_num = 1;
  const double part = 1.0 * g_size / thd_num;
  std::vector<std::thread> th;
  for (int i = 1; i < thd_num; i++) {
    const int head = (int)(part * i), tail = (int)(part * (i + 1));
    if (use_threads)
      th.emplace_back([&, i, head, tail]() { vox.evaluate_only_residual(xs, head, tail, residuals[i]); });
    else
      vox.evaluate_only_residual(xs, head, tail, residuals[i]);
  }
  for (int i = 0; i < win_size - 1; i++) residual1 += imus[i]->give_evaluate_g(xs[i], xs[i + 1], jtj, gg, false);
  residual1 *= (mpar->imu_coef * 0.5);
  vox.evaluate_only_residual(xs, 0, (int)part, residuals[0]);
  for (auto& t : th) t.join();
  for (int i = 0; i < thd_num; i++) residual2 += residuals[i];
  return residual1 + residual2;
}

// damping_iter — optimizers.cpp:745-826. Faithful to its state handling:
// x_stats_temp is initialised once, so a rejected step's gravity increment
// stays in x_stats_temp[0].g for the next trial (line 775)
void LI_BA_OptimizerGravity::damping_iter(std::vector<IMUST>& xs, LidarFactor& vox, std::vector<IMU_PRE*>& imus,
                                          std::vector<double>& resis, int max_iter) {
  win_size = vox.win_size;
  jac_leng = win_size * 6;
  imu_leng = win_size * DIM + 3;
  double u = 0.01, v = 2;
  MatX Hess(imu_leng, imu_leng);
  std::vector<double> JacT(imu_leng, 0.0), D(imu_leng, 0.0);
  double residual1 = 0, residual2 = 0, q;
  bool is_calc_hess = true;
  std::vector<IMUST> xs_temp = xs;
  MatX Hcalc;
  std::vector<double> Jcalc;
  for (int i = 0; i < max_iter; i++) {
    if (is_calc_hess) {
      residual1 = divide_thread(xs, vox, imus, Hess, JacT);
      Hcalc = Hess;
      Jcalc = JacT;
    } else {
      Hess = Hcalc;  // the gauged rows below are rewritten identically
      JacT = Jcalc;
    }
    if (i == 0) resis.push_back(residual1);
    for (int r = 0; r < 6; r++)
      for (int c = 0; c < imu_leng; c++) {
        Hess(r, c) = 0;
        Hess(c, r) = 0;
      }
    for (int r = 0; r < 6; r++) Hess(r, r) = 1;
    for (int r = 0; r < 6; r++) JacT[r] = 0;
    for (int r = 0; r < imu_leng; r++) D[r] = Hess(r, r);
    MatX A = Hess;
    for (int r = 0; r < imu_leng; r++) A(r, r) += u * D[r];
    std::vector<double> mJ(imu_leng);
    for (int r = 0; r < imu_leng; r++) mJ[r] = -JacT[r];
    const std::vector<double> dxi = ldlt_solve(A, mJ);
    for (int k = 0; k < 3; k++) xs_temp[0].g[k] += dxi[imu_leng - 3 + k];
    for (int j = 0; j < win_size; j++) {
      xs_temp[j].R = xs[j].R * Exp(v3(dxi[DIM * j], dxi[DIM * j + 1], dxi[DIM * j + 2]));
      for (int k = 0; k < 3; k++) {
        xs_temp[j].p[k] = xs[j].p[k] + dxi[DIM * j + 3 + k];
        xs_temp[j].v[k] = xs[j].v[k] + dxi[DIM * j + 6 + k];
        xs_temp[j].bg[k] = xs[j].bg[k] + dxi[DIM * j + 9 + k];
        xs_temp[j].ba[k] = xs[j].ba[k] + dxi[DIM * j + 12 + k];
      }
      xs_temp[j].g = xs_temp[0].g;
    }
    for (int j = 0; j < win_size - 1; j++) {
      V15 d;
      for (int k = 0; k < DIM; k++) d[k] = dxi[DIM * j + k];
      imus[j]->update_state(d);
    }
    double q1 = 0;  // 0.5 * dxi.dot(u * D * dxi - JacT)
    for (int r = 0; r < imu_leng; r++) q1 += dxi[r] * (u * D[r] * dxi[r] - JacT[r]);
    q1 *= 0.5;
    residual2 = only_residual(xs_temp, vox, imus);
    q = residual1 - residual2;
    if (q > 0) {
      xs = xs_temp;
      const double one_three = 1.0 / 3;
      q = q / q1;
      v = 2;
      q = 1 - std::pow(2 * q - 1, 3);
      u *= (q < one_three ? one_three : q);
      is_calc_hess = true;
    } else {
      u = u * v;
      v = 2 * v;
      is_calc_hess = false;
      for (int j = 0; j < win_size - 1; j++) {
        imus[j]->dbg = imus[j]->dbg_buf;
        imus[j]->dba = imus[j]->dba_buf;
      }
    }
    if (std::fabs((residual1 - residual2) / residual1) < 1e-6) break;
  }
  resis.push_back(residual2);
}

}  // namespace orc
