// vg_imu.h — IMU_PRE::give_evaluate's residual and Jacobian
// (imu_preintegration.cpp:97-163) on a preintegration record, host and device:
// the BA kernels (ba.hip) and the initialisation's gravity LM (init.cpp,
// give_evaluate_g, imu_preintegration.cpp:165-237) evaluate the same code.
#pragma once
#include "vg_la.h"

namespace vg {

VG_HD M3 imu_m3(const double* a) {
  M3 m;
  for (int i = 0; i < 9; i++) m[i] = a[i];
  return m;
}
VG_HD V3 imu_v3(const double* a) { return v3(a[0], a[1], a[2]); }

// IMU record layout (doubles): R_delta 9, p_delta 3, v_delta 3, R_bg 9, p_bg 9,
// p_ba 9, v_bg 9, v_ba 9, dtime 1 (=61), pad to 64, cov_inv 225.
// bias state per factor: dbg 3, dba 3, dbg_buf 3, dba_buf 3.
VG_HD void imu_residual(const double* rec, const double* bias, const double* x1, const double* x2, double* rr,
                             double* joc /*15x30 or null*/) {
  const M3 Rd = imu_m3(rec), Rbg = imu_m3(rec + 15), pbg = imu_m3(rec + 24), pba = imu_m3(rec + 33),
           vbg = imu_m3(rec + 42), vba = imu_m3(rec + 51);
  const V3 pd = imu_v3(rec + 9), vd = imu_v3(rec + 12);
  const double dtime = rec[60];
  const V3 dbg = imu_v3(bias), dba = imu_v3(bias + 3);
  const M3 R1 = imu_m3(x1), R2 = imu_m3(x2);
  const V3 p1 = imu_v3(x1 + 9), p2 = imu_v3(x2 + 9), v1 = imu_v3(x1 + 12), v2 = imu_v3(x2 + 12);
  const V3 bg1 = imu_v3(x1 + 15), bg2 = imu_v3(x2 + 15), ba1 = imu_v3(x1 + 18), ba2 = imu_v3(x2 + 18);
  const V3 g1 = imu_v3(x1 + 21);
  M3 Rc = mul(Rd, Exp(mul(Rbg, dbg)));
  V3 tc = add(add(pd, mul(pbg, dbg)), mul(pba, dba));
  V3 vc = add(add(vd, mul(vbg, dbg)), mul(vba, dba));
  M3 res_r = mul(mul(tr(Rc), tr(R1)), R2);
  V3 exp_v = mul(tr(R1), sub(sub(v2, v1), scl(g1, dtime)));
  V3 res_v = sub(exp_v, vc);
  V3 exp_t = mul(tr(R1), sub(sub(sub(p2, p1), scl(v1, dtime)), scl(g1, 0.5 * dtime * dtime)));
  V3 res_t = sub(exp_t, tc);
  V3 lr = Log(res_r);
  for (int k = 0; k < 3; k++) {
    rr[k] = lr[k];
    rr[3 + k] = res_t[k];
    rr[6 + k] = res_v[k];
    rr[9 + k] = bg2[k] - bg1[k];
    rr[12 + k] = ba2[k] - ba1[k];
  }
  if (!joc) return;
  for (int k = 0; k < 450; k++) joc[k] = 0.0;
  auto put = [&](int r0, int c0, const M3& m) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) joc[(r0 + r) * 30 + c0 + c] = m(r, c);
  };
  const M3 JRi = jr_inv(res_r);
  const M3 R1t = tr(R1);
  put(0, 0, scl(mul(mul(JRi, tr(R2)), R1), -1.0));
  put(0, 15, JRi);
  put(0, 9, scl(mul(mul(mul(JRi, tr(res_r)), jr(mul(Rbg, dbg))), Rbg), -1.0));
  put(3, 0, hat(exp_t));
  put(3, 3, scl(R1t, -1.0));
  put(3, 6, scl(R1t, -dtime));
  put(3, 9, scl(pbg, -1.0));
  put(3, 12, scl(pba, -1.0));
  put(3, 18, R1t);
  put(6, 0, hat(exp_v));
  put(6, 6, scl(R1t, -1.0));
  put(6, 9, scl(vbg, -1.0));
  put(6, 12, scl(vba, -1.0));
  put(6, 21, R1t);
  put(9, 9, scl(M3::I(), -1.0));
  put(12, 12, scl(M3::I(), -1.0));
  put(9, 24, M3::I());
  put(12, 27, M3::I());
}

}  // namespace vg
