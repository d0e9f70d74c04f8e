// ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
// cpu_baseline). Never linked into or called by the product library.
//
// CPU restatement of VINA-SLAM's core types and math
// (include/vina_slam/core/{types,math,constants,point_utils}.hpp,
//  src/core/point_utils.cpp). Dependency-free: Eigen/PCL are absent here.
#pragma once
#include <cstdint>
#include <cstddef>
#include <functional>
#include <memory>
#include <unordered_map>
#include <vector>
#include "la.hpp"

namespace orc {

constexpr int DIM = 15;          // constants.hpp:14
constexpr double G_m_s2 = 9.8;   // constants.hpp:12
constexpr size_t HASH_P = 1000033;        // constants.hpp:7
constexpr size_t MAX_N = 100000000000ULL;  // constants.hpp:8

// VOXEL_LOC — types.hpp:13-26
struct VOXEL_LOC {
  int64_t x, y, z;
  VOXEL_LOC(int64_t vx = 0, int64_t vy = 0, int64_t vz = 0) : x(vx), y(vy), z(vz) {}
  bool operator==(const VOXEL_LOC& o) const { return x == o.x && y == o.y && z == o.z; }
};
// hash<VOXEL_LOC> — types.hpp:28-41 (std::hash<int64_t> is the identity in libstdc++)
struct VoxHash {
  size_t operator()(const VOXEL_LOC& s) const {
    return ((((size_t)s.z * HASH_P) % MAX_N + (size_t)s.y) * HASH_P) % MAX_N + (size_t)s.x;
  }
};
template <class T>
using VoxMap = std::unordered_map<VOXEL_LOC, T, VoxHash>;

// The voxel-key rule: float(coord / size), minus 1 in float
// when negative, then truncation to int64. Division in double.
// point_utils.hpp:16-23 (float coords), voxel_map.cpp:57-65, 246-253 (double coords)
inline int64_t key_axis(double c, double size) {
  float l = (float)(c / size);
  if (l < 0) l -= 1;
  return (int64_t)l;
}
inline VOXEL_LOC voxel_key(const V3& w, double size) {
  return VOXEL_LOC(key_axis(w[0], size), key_axis(w[1], size), key_axis(w[2], size));
}

// math.hpp:50-55
inline M3 hat(const V3& v) {
  M3 m;
  m(0, 1) = -v[2]; m(0, 2) = v[1];
  m(1, 0) = v[2];  m(1, 2) = -v[0];
  m(2, 0) = -v[1]; m(2, 1) = v[0];
  return m;
}
// math.hpp:12-26
inline M3 Exp(const V3& ang) {
  double n = norm(ang);
  if (n >= 1e-9) {
    V3 r = ang / n;
    M3 K = hat(r);
    return M3::Identity() + K * std::sin(n) + (K * K) * (1.0 - std::cos(n));
  }
  return M3::Identity();
}
// math.hpp:28-41
inline M3 Exp(const V3& w, double dt) {
  double n = norm(w);
  if (n > 1e-7) {
    V3 r = w / n;
    M3 K = hat(r);
    double a = n * dt;
    return M3::Identity() + K * std::sin(a) + (K * K) * (1.0 - std::cos(a));
  }
  return M3::Identity();
}
// math.hpp:43-48
inline V3 Log(const M3& R) {
  double tr = R.trace();
  double theta = (tr > 3.0 - 1e-6) ? 0.0 : std::acos(0.5 * (tr - 1));
  V3 K = v3(R(2, 1) - R(1, 2), R(0, 2) - R(2, 0), R(1, 0) - R(0, 1));
  return (std::fabs(theta) < 0.001) ? (K * 0.5) : (K * (0.5 * theta / std::sin(theta)));
}
// math.hpp:57-71
inline M3 jr(V3 vec) {
  double ang = norm(vec);
  if (ang < 1e-9) return M3::Identity();
  vec /= ang;
  double ra = std::sin(ang) / ang;
  return M3::Identity() * ra + outer(vec, vec) * (1 - ra) - hat(vec) * ((1 - std::cos(ang)) / ang);
}
// Eigen::AngleAxisd(Matrix3d) via quaternion, as Eigen does (Quaternion from
// rotation matrix, then AngleAxis from quaternion).
inline void angle_axis(const M3& m, double& angle, V3& axis) {
  double q[4];  // x y z w
  double t = m.trace();
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m(2, 1) - m(1, 2)) * t;
    q[1] = (m(0, 2) - m(2, 0)) * t;
    q[2] = (m(1, 0) - m(0, 1)) * t;
  } else {
    int i = 0;
    if (m(1, 1) > m(0, 0)) i = 1;
    if (m(2, 2) > m(i, i)) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m(k, j) - m(j, k)) * t;
    q[j] = (m(j, i) + m(i, j)) * t;
    q[k] = (m(k, i) + m(i, k)) * t;
  }
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  if (n != 0.0) {
    angle = 2.0 * std::atan2(n, std::fabs(q[3]));
    if (q[3] < 0) n = -n;
    axis = v3(q[0] / n, q[1] / n, q[2] / n);
  } else {
    angle = 0.0;
    axis = v3(1, 0, 0);
  }
}
// math.hpp:73-88
inline M3 jr_inv(const M3& rotR) {
  double ang;
  V3 axi;
  angle_axis(rotR, ang, axi);
  if (ang < 1e-9) return M3::Identity();
  double ctt = ang / 2 / std::tan(ang / 2);
  return M3::Identity() * ctt + outer(axi, axi) * (1 - ctt) + hat(axi) * (ang / 2);
}

// IMUST — types.hpp:43-113
struct IMUST {
  double t = 0;
  M3 R = M3::Identity();
  V3 p, v, bg, ba, g;
  M15 cov;
  IMUST() { setZero(); }
  void setZero() {
    t = 0;
    R = M3::Identity();
    p.setZero(); v.setZero(); bg.setZero(); ba.setZero();
    g = v3(0, 0, -G_m_s2);
    cov = M15::Identity() * 0.0001;
    for (int i = 9; i < 15; i++) cov(i, i) = 0.00001;
  }
  IMUST& operator+=(const V15& ist) {
    R = R * Exp(ist.block<3, 1>(0, 0));
    p += ist.block<3, 1>(3, 0);
    v += ist.block<3, 1>(6, 0);
    bg += ist.block<3, 1>(9, 0);
    ba += ist.block<3, 1>(12, 0);
    return *this;
  }
  V15 minus(const IMUST& b) const {  // *this - b
    V15 a;
    a.setBlock(0, 0, Log(b.R.T() * R));
    a.setBlock(3, 0, p - b.p);
    a.setBlock(6, 0, v - b.v);
    a.setBlock(9, 0, bg - b.bg);
    a.setBlock(12, 0, ba - b.ba);
    return a;
  }
};

// PointCluster — types.hpp:115-175
struct PointCluster {
  M3 P;
  V3 v;
  int N = 0;
  void clear() { P.setZero(); v.setZero(); N = 0; }
  void push(const V3& vec) {
    N++;
    P += outer(vec, vec);
    v += vec;
  }
  M3 cov() const {
    V3 c = v / (double)N;
    return P / (double)N - outer(c, c);
  }
  PointCluster& operator+=(const PointCluster& s) { P += s.P; v += s.v; N += s.N; return *this; }
  PointCluster& operator-=(const PointCluster& s) { P -= s.P; v -= s.v; N -= s.N; return *this; }
  void transform(const PointCluster& s, const IMUST& st) {
    N = s.N;
    v = st.R * s.v + st.p * (double)N;
    M3 rp = outer(st.R * s.v, st.p);
    P = (st.R * s.P) * st.R.T() + rp + rp.T() + outer(st.p, st.p) * (double)N;
  }
};

// pointVar — types.hpp:177-182
struct pointVar {
  V3 pnt;
  M3 var;
  float intensity = 0;
};
using PVec = std::vector<pointVar>;
using PVecPtr = std::shared_ptr<PVec>;

// pcl::PointXYZINormal subset used on the path (x,y,z,intensity,curvature)
struct PointType {
  float x = 0, y = 0, z = 0, intensity = 0, curvature = 0;
  float data(int j) const { return j == 0 ? x : (j == 1 ? y : z); }
};

// down_sampling_voxel — point_utils.hpp:7-44. Output order = unordered_map
// iteration order (libstdc++, same hash), exactly as the reference; or, with
// key_order, ascending (x, y, z) voxel key (the device's order). The
// initialisation path uses key order: its kd map is re-downsampled after every
// scan, so the order of the points inside a voxel — which the reference leaves
// to the standard library's hash-table layout — sets the float means bit for
// bit, and only a fixed order makes the cold start reproducible.
inline void down_sampling_voxel(std::vector<PointType>& pl, double voxel_size, bool key_order = false) {
  if (voxel_size < 0.001) return;
  VoxMap<PointType> feat_map;
  float loc[3];
  for (PointType& pc : pl) {
    for (int j = 0; j < 3; j++) {
      loc[j] = pc.data(j) / voxel_size;
      if (loc[j] < 0) loc[j] -= 1.0;
    }
    VOXEL_LOC pos((int64_t)loc[0], (int64_t)loc[1], (int64_t)loc[2]);
    auto it = feat_map.find(pos);
    if (it == feat_map.end()) {
      PointType pp = pc;
      pp.curvature = 1;
      feat_map[pos] = pp;
    } else {
      PointType& pp = it->second;
      pp.x = (pp.x * pp.curvature + pc.x) / (pp.curvature + 1);
      pp.y = (pp.y * pp.curvature + pc.y) / (pp.curvature + 1);
      pp.z = (pp.z * pp.curvature + pc.z) / (pp.curvature + 1);
      pp.curvature += 1;
    }
  }
  pl.clear();
  if (!key_order) {
    for (auto& kv : feat_map) pl.push_back(kv.second);
    return;
  }
  std::vector<std::pair<VOXEL_LOC, PointType>> v(feat_map.begin(), feat_map.end());
  std::sort(v.begin(), v.end(), [](const std::pair<VOXEL_LOC, PointType>& a, const std::pair<VOXEL_LOC, PointType>& b) {
    if (a.first.x != b.first.x) return a.first.x < b.first.x;
    if (a.first.y != b.first.y) return a.first.y < b.first.y;
    return a.first.z < b.first.z;
  });
  for (auto& kv : v) pl.push_back(kv.second);
}

// calcBodyVar — point_utils.cpp:3-34
inline void calcBodyVar(V3& pb, const float range_inc, const float degree_inc, M3& var) {
  if (pb[2] == 0) pb[2] = 0.0001;
  float range = std::sqrt(pb[0] * pb[0] + pb[1] * pb[1] + pb[2] * pb[2]);
  float range_var = range_inc * range_inc;
  double s = std::sin(degree_inc * M_PI / 180.0);
  double dv = s * s;  // pow(sin(DEG2RAD(degree_inc)), 2)
  V3 direction = pb / norm(pb);
  M3 dhat = hat(direction);
  V3 b1 = v3(1, 1, -(direction[0] + direction[1]) / direction[2]);
  b1 = b1 / norm(b1);
  V3 b2 = cross(b1, direction);
  b2 = b2 / norm(b2);
  Mat<3, 2> Nm;
  Nm(0, 0) = b1[0]; Nm(0, 1) = b2[0];
  Nm(1, 0) = b1[1]; Nm(1, 1) = b2[1];
  Nm(2, 0) = b1[2]; Nm(2, 1) = b2[2];
  Mat<3, 2> A = (dhat * (double)range) * Nm;
  Mat<2, 2> D;
  D(0, 0) = dv; D(1, 1) = dv;
  var = outer(direction * (double)range_var, direction) + (A * D) * A.T();
}

// var_init — point_utils.cpp:36-52
inline void var_init(const IMUST& ext, const std::vector<PointType>& pl, PVec& out, double dept_err,
                     double beam_err) {
  int n = (int)pl.size();
  out.clear();
  out.resize(n);
  for (int i = 0; i < n; i++) {
    const PointType& ap = pl[i];
    pointVar& pv = out[i];
    pv.pnt = v3(ap.x, ap.y, ap.z);
    calcBodyVar(pv.pnt, (float)dept_err, (float)beam_err, pv.var);
    pv.pnt = ext.R * pv.pnt + ext.p;
    pv.var = (ext.R * pv.var) * ext.R.T();
    pv.intensity = ap.intensity;
  }
}

// pvec_update — point_utils.cpp:54-65
inline void pvec_update(PVec& pv, const IMUST& x, std::vector<V3>& pwld) {
  M3 rot_var = x.cov.block<3, 3>(0, 0);
  M3 tsl_var = x.cov.block<3, 3>(3, 3);
  for (pointVar& p : pv) {
    M3 phat = hat(p.pnt);
    p.var = (x.R * p.var) * x.R.T() + (phat * rot_var) * phat.T() + tsl_var;
    pwld.push_back(x.R * p.pnt + x.p);
  }
}

}  // namespace orc
