// ORACLE — test infrastructure only. Known-answer hooks:
// the restatement's point-to-plane Jacobian, LidarFactor gradient / Hessian /
// residual and IMU_PRE residual / Jacobian on caller-given inputs, so the
// tests can pin them against central finite differences (the reference ships
// no fixtures for them).
#include <cstring>
#include "map.hpp"
#include "vina_oracle.h"

using namespace orc;

static M3 m3_of(const double* a) {
  M3 m;
  for (int i = 0; i < 9; i++) m[i] = a[i];
  return m;
}
static V3 v3_of(const double* a) { return v3(a[0], a[1], a[2]); }
static PointCluster clu_of(const double* a) {  // P 9, v 3, N
  PointCluster c;
  for (int i = 0; i < 9; i++) c.P[i] = a[i];
  c.v = v3_of(a + 9);
  c.N = (int)a[12];
  return c;
}

extern "C" {

// odometry.cpp:136-142 at pose (R, p): residual and 6-vector Jacobian
void orc_kat_p2p(const double* R9, const double* p3, const double* pnt3, const double* n3, const double* c3,
                 double* r, double* j6) {
  const M3 R = m3_of(R9);
  const V3 pnt = v3_of(pnt3);
  const V3 wld = R * pnt + v3_of(p3);
  V6 jac;
  p2p_residual_jacobian(R, pnt, wld, v3_of(n3), v3_of(c3), *r, jac);
  for (int k = 0; k < 6; k++) j6[k] = jac[k];
}

// One LidarFactor voxel (factors.cpp:11-126): W local clusters (13 doubles
// each: P 9, v 3, N), the fixed cluster, window poses (12 each: R 9, p 3).
// The eigen system comes from the merged cluster at the given poses, as
// tras_opt hands it over after a recut / residual pass. Outputs lambda_min,
// JacT (6W) and the Hessian (6W x 6W, row-major). hess may be null.
void orc_kat_lidar_factor(int W, const double* clu, const double* fix, const double* poses, double* res,
                          double* jac, double* hess) {
  std::vector<IMUST> xs(W);
  for (int i = 0; i < W; i++) {
    xs[i].R = m3_of(poses + 12 * i);
    xs[i].p = v3_of(poses + 12 * i + 9);
  }
  std::vector<PointCluster> loc(W);
  PointCluster f = clu_of(fix), add = f;
  for (int i = 0; i < W; i++) {
    loc[i] = clu_of(clu + 13 * i);
    if (loc[i].N) {
      PointCluster t;
      t.transform(loc[i], xs[i]);
      add += t;
    }
  }
  V3 ev;
  M3 U;
  eig3(add.cov(), ev, U);
  LidarFactor lf(W);
  lf.push_voxel(loc, f, 1.0, ev, U, add);
  MatX H(6 * W, 6 * W);
  std::vector<double> J(6 * W, 0.0);
  lf.acc_evaluate2(xs, 0, 1, H, J, *res);
  memcpy(jac, J.data(), J.size() * sizeof(double));
  if (hess) memcpy(hess, H.d.data(), (size_t)36 * W * W * sizeof(double));
}

// IMU_PRE over samples imu (m x 7: t, gyr 3, acc 3) integrated at biases
// bias0 (bg 3, ba 3; push_imu / add_imu, imu_preintegration.cpp:31-95), with
// the bias deltas dbias (dbg 3, dba 3) of update_state, evaluated between two
// states (24 each: R 9, p 3, v 3, bg 3, ba 3, g 3): residual rr (15), the
// Jacobian [joca | jocb] (15 x 30, row-major) and r^T C^-1 r
// (give_evaluate, imu_preintegration.cpp:97-163). noise: cov_gyr, cov_acc,
// rdw_gyr, rdw_acc (noiseMeas / noiseWalk); sg: imupre_scale_gravity.
double orc_kat_imu(const double* imu, int m, const double* bias0, const double* dbias, const double* x1,
                   const double* x2, const double* noise, double sg, double* rr, double* joc) {
  MapParams mp;
  mp.imupre_scale_gravity = sg;
  mp.noiseMeas.setZero();
  mp.noiseWalk.setZero();
  for (int i = 0; i < 3; i++) {
    mp.noiseMeas(i, i) = noise[0];
    mp.noiseMeas(3 + i, 3 + i) = noise[1];
    mp.noiseWalk(i, i) = noise[2];
    mp.noiseWalk(3 + i, 3 + i) = noise[3];
  }
  IMU_PRE pre(&mp, v3_of(bias0), v3_of(bias0 + 3));
  std::vector<ImuSample> s(m);
  for (int i = 0; i < m; i++) {
    s[i].t = imu[7 * i];
    s[i].gyr = v3_of(imu + 7 * i + 1);
    s[i].acc = v3_of(imu + 7 * i + 4);
  }
  pre.push_imu(s);
  pre.dbg = v3_of(dbias);
  pre.dba = v3_of(dbias + 3);
  IMUST a, b;
  const double* xx[2] = {x1, x2};
  IMUST* st[2] = {&a, &b};
  for (int k = 0; k < 2; k++) {
    st[k]->R = m3_of(xx[k]);
    st[k]->p = v3_of(xx[k] + 9);
    st[k]->v = v3_of(xx[k] + 12);
    st[k]->bg = v3_of(xx[k] + 15);
    st[k]->ba = v3_of(xx[k] + 18);
    st[k]->g = v3_of(xx[k] + 21);
  }
  Mat<30, 30> jtj;
  Mat<30, 1> gg;
  V15 r;
  Mat<15, 30> J;
  const double cost = pre.give_evaluate(a, b, jtj, gg, true, &r, &J);
  for (int k = 0; k < 15; k++) rr[k] = r[k];
  memcpy(joc, J.d, sizeof(J.d));
  return cost;
}

}  // extern "C"
