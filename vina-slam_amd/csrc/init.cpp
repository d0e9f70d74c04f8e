// init.cpp — the cold-start initialisation, host side.
//
// The reference initialises on the odometry thread (local_mapping.cpp:362-386):
//   IMUEKF::process / IMU_init             src/estimation/imu_ekf.cpp:147-201
//   VINA_SLAM::initialization              src/platform/ros2/node.cpp:293-366
//   Initialization::motion_init            src/pipeline/initialization.cpp:158-367
//   Initialization::motion_blur            initialization.cpp:64-156
//   Initialization::align_gravity          initialization.cpp:28-62
//   LI_BA_OptimizerGravity::damping_iter   src/mapping/optimizers.cpp:629-826
//   IMU_PRE::give_evaluate_g               src/estimation/imu_preintegration.cpp:165-237
//   VINA_SLAM::system_reset                node.cpp:368-408
// Placement: everything per point / per voxel / per factor runs on the device
// with the steady state's kernels — the deskew, the 0.5 m downsample and the
// kd-tree IEKF point passes (kdlio.hip), down_sampling_close (downsample.hip),
// motion_blur's per-point transform (state.hip k_blur_init), the map rebuild of
// every round (map.hip: the insert with precomputed body points, the recut with
// the initialisation thresholds) and the LiDAR factor Hessian / residual
// passes of the gravity LM (ba.hip). The host keeps what is O(IMU samples) or
// O(window): the IMU means, the IMU pose integration, the preintegration, the
// IMU factors with the gravity Jacobian, the (15W+3)-unknown LDLT of the 3 LM
// iterations per round, align_gravity and the accept / convergence rules.
// Initialisation runs once per sequence (about W + 3 scans); it is synchronous.
#include <algorithm>
#include <cmath>
#include <cstring>
#include "vg_host.h"
#include "vg_imu.h"

namespace vg {

constexpr int kMinInitNum = 30;  // IMUEKF::min_init_num (ekf_imu.hpp:18)
constexpr double kGms2 = 9.8;    // G_m_s2

struct InitState {
  bool active = true;          // motion_init_flag (local_mapping.cpp:362)
  bool init_flag = false;      // IMUEKF::init_flag
  int init_num = 0;            // IMUEKF::init_num
  V3 mean_acc = V3::Z(), mean_gyr = V3::Z();
  double scale_gravity = 1.0;  // IMUEKF::scale_gravity (ekf_imu.hpp:27)
  // the window being collected (initialization()'s statics, node.cpp:296-298)
  std::vector<double> beg_times;
  std::vector<std::vector<Imu>> vec_imus;
  std::vector<int> n_close;                 // close-downsampled points per window scan (device pool)
  std::vector<std::vector<float>> t_close;  // their times, ascending (host copy: the blur plan)
  // device buffers (allocated on the first scan)
  float4* pool = nullptr;  // win_size x cap: close-downsampled raw scans (x, y, z, t)
  int cap = 0;
  double* pnt = nullptr;   // one scan's motion-blurred body points (fp64), cap + kMaxBlurDup
  double* par = nullptr;   // blur parameters (frame pose, extrinsic, IMU poses)
  double* pose = nullptr;  // kXC pose / covariance block of the frame being inserted
  static constexpr int kMaxBlurDup = kDeskewBuf / 22 + 1;  // point 0 repeats once per later IMU pose
};

InitState* init_create(vg_ctx*) { return new InitState(); }
void init_destroy(InitState* I) {
  if (!I) return;
  if (I->pool) (void)hipFree(I->pool);
  if (I->pnt) (void)hipFree(I->pnt);
  if (I->par) (void)hipFree(I->par);
  if (I->pose) (void)hipFree(I->pose);
  delete I;
}
bool init_active(const HostPipe* P) { return P->init && P->init->active; }

static int init_dev(vg_ctx* ctx, InitState& I) {
  if (I.pool) return VG_OK;
  const int W = ctx->cfg.win_size;
  I.cap = ctx->cap.max_points_per_scan;
  VG_HIP(hipMalloc((void**)&I.pool, (size_t)W * I.cap * sizeof(float4)));
  VG_HIP(hipMalloc((void**)&I.pnt, ((size_t)I.cap + InitState::kMaxBlurDup) * 3 * sizeof(double)));
  VG_HIP(hipMalloc((void**)&I.par, kDeskewBuf * sizeof(double)));
  VG_HIP(hipMalloc((void**)&I.pose, 256 * sizeof(double)));
  return VG_OK;
}

// IMUEKF::IMU_init — imu_ekf.cpp:147-172 (running means)
static void imu_init(InitState& I, const std::vector<Imu>& imus) {
  for (const Imu& s : imus) {
    const V3 acc = v3(s.acc[0], s.acc[1], s.acc[2]), gyr = v3(s.gyr[0], s.gyr[1], s.gyr[2]);
    if (I.init_num != 0) {
      I.mean_acc = add(I.mean_acc, scl(sub(acc, I.mean_acc), 1.0 / (double)I.init_num));
      I.mean_gyr = add(I.mean_gyr, scl(sub(gyr, I.mean_gyr), 1.0 / (double)I.init_num));
    } else {
      I.mean_acc = acc;
      I.mean_gyr = gyr;
      I.init_num = 1;
    }
    I.init_num++;
  }
}

static void put_frame(const HX& x, double* o) {  // kXS layout: R, p, v, bg, ba, g
  memcpy(o, x.R.a, 72);
  memcpy(o + 9, x.p.a, 24);
  memcpy(o + 12, x.v.a, 24);
  memcpy(o + 15, x.bg.a, 24);
  memcpy(o + 18, x.ba.a, 24);
  memcpy(o + 21, x.g.a, 24);
}

// ---- Initialization::motion_blur (initialization.cpp:64-156): the IMU poses
// integrated backwards from the scan-end state xc with the biases of xl, in
// the deskew record layout (t offset, R, p, v, w, a); list order = descending
// start time
static void blur_poses(const HX& xc_in, const HX& xl, const std::vector<Imu>& imus, double beg, double sg,
                       std::vector<double>& rec) {
  HX xc = xc_in;
  xc.bg = xl.bg;
  xc.ba = xl.ba;
  V3 vel = xc.v, pos = xc.p, acc_imu, angvel, acc_avr;
  M3 R_imu = xc.R;
  rec.clear();
  for (int k = (int)imus.size() - 1; k >= 1; k--) {
    const Imu& head = imus[k - 1];
    const Imu& tail = imus[k];
    for (int j = 0; j < 3; j++) {
      angvel[j] = 0.5 * (head.gyr[j] + tail.gyr[j]);
      acc_avr[j] = 0.5 * (head.acc[j] + tail.acc[j]);
    }
    angvel = sub(angvel, xc.bg);
    acc_avr = sub(scl(acc_avr, sg), xc.ba);
    const double dt = head.t - tail.t;
    const M3 Exp_f = Exp(angvel, dt);
    acc_imu = add(mul(R_imu, acc_avr), xc.g);
    pos = add(add(pos, scl(vel, dt)), scl(acc_imu, 0.5 * dt * dt));
    vel = add(vel, scl(acc_imu, dt));
    R_imu = mul(R_imu, Exp_f);
    double r[22];
    r[0] = head.t - beg;
    memcpy(r + 1, R_imu.a, 72);
    memcpy(r + 10, pos.a, 24);
    memcpy(r + 13, vel.a, 24);
    memcpy(r + 16, angvel.a, 24);
    memcpy(r + 19, acc_imu.a, 24);
    rec.insert(rec.end(), r, r + 22);
  }
}

// the motion-blurred body points of window scan i, on the device (I.pnt);
// returns their count
static int blur_scan(vg_ctx* ctx, InitState& I, int i, const HX& xc, const HX& xl, double sg, int* nout) {
  std::vector<double> poses;
  blur_poses(xc, xl, I.vec_imus[i], I.beg_times[i], sg, poses);
  const int npose = (int)poses.size() / 22;
  const int n = I.n_close[i];
  const std::vector<float>& t = I.t_close[i];
  *nout = 0;
  if (n == 0 || npose == 0) return VG_OK;
  // the backward walk's plan: points after the last (earliest) pose start are
  // pushed, newest first; if that reaches point 0, it is pushed again with
  // each later pose
  const double t_last = poses[(size_t)(npose - 1) * 22];
  int j0 = 0;
  while (j0 < n && !((double)t[j0] > t_last)) j0++;
  int q0 = npose, dups = 0;
  if (j0 == 0) {
    q0 = 0;
    while (!(poses[(size_t)q0 * 22] < (double)t[0])) q0++;
    dups = npose - 1 - q0;
  }
  const int no = (n - j0) + dups;
  if (no > I.cap + InitState::kMaxBlurDup) {
    ctx->err = "motion_blur (init): point buffer too small";
    return VG_E_CAPACITY;
  }
  std::vector<double> par(24 + poses.size());
  memcpy(par.data(), xc.R.a, 72);
  memcpy(par.data() + 9, xc.p.a, 24);
  for (int k = 0; k < 9; k++) par[12 + k] = ctx->cfg.ext_R[k];
  for (int k = 0; k < 3; k++) par[21 + k] = ctx->cfg.ext_t[k];
  memcpy(par.data() + 24, poses.data(), poses.size() * sizeof(double));
  VG_TRY(state_blur_init(ctx, par.data(), npose, I.pool + (size_t)i * I.cap, n, j0, q0, no, I.par, I.pnt));
  *nout = no;
  return VG_OK;
}

// ---- the gravity LM (LI_BA_OptimizerGravity, optimizers.cpp:629-826)

// Eigen::LDLT<MatrixXd>(A).solve(b) on the lower triangle of A (n x n, row
// major): left-looking, so the pivot at step k is the largest |diagonal| of
// the ORIGINAL remaining rows (first on ties); zero pivots solve as 0
// (Eigen's pseudo-inverse of D). Same arithmetic order as the steady-state
// solve's reference (optimizers.cpp:466 vs 786).
static void ldlt_solve(std::vector<double> A, int n, const std::vector<double>& b, std::vector<double>& x) {
  auto a = [&](int i, int j) -> double& { return A[(size_t)i * n + j]; };
  std::vector<int> perm(n);
  std::vector<double> w(n);
  for (int k = 0; k < n; k++) {
    int p = k;
    double big = std::fabs(a(k, k));
    for (int i = k + 1; i < n; i++)
      if (std::fabs(a(i, i)) > big) {
        big = std::fabs(a(i, i));
        p = i;
      }
    perm[k] = p;
    if (p != k) {  // symmetric transposition of rows/columns k and p, lower triangle
      for (int j = 0; j < k; j++) std::swap(a(k, j), a(p, j));
      for (int i = p + 1; i < n; i++) std::swap(a(i, k), a(i, p));
      std::swap(a(k, k), a(p, p));
      for (int i = k + 1; i < p; i++) std::swap(a(i, k), a(p, i));
    }
    if (k > 0) {
      for (int j = 0; j < k; j++) w[j] = a(j, j) * a(k, j);
      double s = 0.0;
      for (int j = 0; j < k; j++) s += a(k, j) * w[j];
      a(k, k) -= s;
      for (int i = k + 1; i < n; i++) {
        double t = 0.0;
        for (int j = 0; j < k; j++) t += a(i, j) * w[j];
        a(i, k) -= t;
      }
    }
    const double d = a(k, k);
    if (k == 0 && d == 0.0) {
      for (int j = 0; j < n; j++) perm[j] = j;
      break;
    }
    if (d != 0.0)
      for (int i = k + 1; i < n; i++) a(i, k) /= d;
  }
  x = b;
  for (int k = 0; k < n; k++) std::swap(x[k], x[perm[k]]);
  for (int i = 0; i < n; i++) {
    double s = 0.0;
    for (int j = 0; j < i; j++) s += a(i, j) * x[j];
    x[i] -= s;
  }
  for (int i = 0; i < n; i++) x[i] = (std::fabs(a(i, i)) > 2.2250738585072014e-308) ? x[i] / a(i, i) : 0.0;
  for (int i = n - 1; i >= 0; i--) {
    double s = 0.0;
    for (int j = i + 1; j < n; j++) s += a(j, i) * x[j];
    x[i] -= s;
  }
  for (int k = n - 1; k >= 0; k--) std::swap(x[k], x[perm[k]]);
}

struct GravLM {
  vg_ctx* ctx;
  int W, L, n;
  const std::vector<std::vector<double>>& recs;  // IMU_PRE records of the window factors
  std::vector<double> bias;                      // per factor: dbg, dba, dbg_buf, dba_buf
  std::vector<int> ring;
  GravLM(vg_ctx* c, const std::vector<std::vector<double>>& r)
      : ctx(c), W(c->cfg.win_size), L(6 * c->cfg.win_size), n(15 * c->cfg.win_size + 3), recs(r),
        bias((size_t)(c->cfg.win_size - 1) * 12, 0.0), ring(c->cfg.win_size) {
    for (int i = 0; i < W; i++) ring[i] = i;
  }
  std::vector<double> frames(const std::vector<HX>& xs) const {
    std::vector<double> f((size_t)W * kXS);
    for (int i = 0; i < W; i++) put_frame(xs[i], &f[(size_t)i * kXS]);
    return f;
  }
  // give_evaluate_g (imu_preintegration.cpp:165-237): give_evaluate's residual
  // and 15x30 Jacobian (vg_imu.h) plus the gravity columns of rows 3-8
  double imu_g(int k, const double* f, double* jtj /*33x33*/, double* gg /*33*/) const {
    const double* rec = recs[k].data();
    double rr[15], joc[450];
    imu_residual(rec, &bias[(size_t)k * 12], f + (size_t)k * kXS, f + (size_t)(k + 1) * kXS, rr, jtj ? joc : nullptr);
    const double* C = rec + 64;  // cov_inv
    double cr[15];
    for (int r = 0; r < 15; r++) {
      double s = C[r * 15] * rr[0];
      for (int l = 1; l < 15; l++) s += C[r * 15 + l] * rr[l];
      cr[r] = s;
    }
    double cost = rr[0] * cr[0];
    for (int r = 1; r < 15; r++) cost += rr[r] * cr[r];
    if (!jtj) return cost;
    double J[15 * 33];
    for (int r = 0; r < 15; r++) {
      for (int c = 0; c < 30; c++) J[r * 33 + c] = joc[r * 30 + c];
      for (int c = 30; c < 33; c++) J[r * 33 + c] = 0.0;
    }
    const double dt = rec[60];
    const M3 R1t = tr(imu_m3(f + (size_t)k * kXS));
    const M3 Jp = scl(R1t, -0.5 * dt * dt), Jv = scl(R1t, -dt);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        J[(3 + r) * 33 + 30 + c] = Jp(r, c);
        J[(6 + r) * 33 + 30 + c] = Jv(r, c);
      }
    double P[33 * 15];  // J^T C
    for (int r = 0; r < 33; r++)
      for (int l = 0; l < 15; l++) {
        double s = J[0 * 33 + r] * C[0 * 15 + l];
        for (int q = 1; q < 15; q++) s += J[q * 33 + r] * C[q * 15 + l];
        P[r * 15 + l] = s;
      }
    for (int r = 0; r < 33; r++) {
      for (int c = 0; c < 33; c++) {
        double s = P[r * 15] * J[c];
        for (int l = 1; l < 15; l++) s += P[r * 15 + l] * J[l * 33 + c];
        jtj[r * 33 + c] = s;
      }
      double s = P[r * 15] * rr[0];
      for (int l = 1; l < 15; l++) s += P[r * 15 + l] * rr[l];
      gg[r] = s;
    }
    return cost;
  }
  // divide_thread (optimizers.cpp:640-707): IMU factors x imu_coef, then the
  // LiDAR factors' 6W x 6W blocks (device pass)
  int hessian(const std::vector<HX>& xs, std::vector<double>& H, std::vector<double>& g, double* res) {
    const std::vector<double> f = frames(xs);
    const double coef = ctx->cfg.imu_coef;
    std::fill(H.begin(), H.end(), 0.0);
    std::fill(g.begin(), g.end(), 0.0);
    double residual = 0.0;
    const int g0 = n - 3;
    std::vector<double> jtj(33 * 33), gg(33);
    for (int k = 0; k < W - 1; k++) {
      residual += imu_g(k, f.data(), jtj.data(), gg.data());
      for (int r = 0; r < 30; r++) {
        for (int c = 0; c < 30; c++) H[(size_t)(k * 15 + r) * n + k * 15 + c] += jtj[r * 33 + c];
        for (int c = 0; c < 3; c++) H[(size_t)(k * 15 + r) * n + g0 + c] += jtj[r * 33 + 30 + c];
      }
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 30; c++) H[(size_t)(g0 + r) * n + k * 15 + c] += jtj[(30 + r) * 33 + c];
        for (int c = 0; c < 3; c++) H[(size_t)(g0 + r) * n + g0 + c] += jtj[(30 + r) * 33 + 30 + c];
      }
      for (int r = 0; r < 30; r++) g[k * 15 + r] += gg[r];
      for (int r = 0; r < 3; r++) g[g0 + r] += gg[30 + r];
    }
    for (double& h : H) h *= coef;
    for (double& v : g) v *= coef;
    residual *= coef * 0.5;
    const int nl = L * (L + 1) / 2;
    std::vector<double> hl((size_t)nl + L + 1);
    VG_TRY(ba_lidar_pass(ctx, true, f.data(), ring.data(), hl.data()));
    for (int R = 0; R < L; R++) {
      const int Ri = (R / 6) * 15 + R % 6;
      for (int C = 0; C <= R; C++) {
        const int Ci = (C / 6) * 15 + C % 6;
        const double v = hl[(size_t)R * (R + 1) / 2 + C];
        H[(size_t)Ri * n + Ci] += v;
        if (Ri != Ci) H[(size_t)Ci * n + Ri] += v;
      }
      g[Ri] += hl[(size_t)nl + R];
    }
    *res = residual + hl[(size_t)nl + L];
    return VG_OK;
  }
  // only_residual (optimizers.cpp:709-743)
  int residual(const std::vector<HX>& xs, double* res) {
    const std::vector<double> f = frames(xs);
    double r1 = 0.0;
    for (int k = 0; k < W - 1; k++) r1 += imu_g(k, f.data(), nullptr, nullptr);
    r1 *= ctx->cfg.imu_coef * 0.5;
    double r2 = 0.0;
    VG_TRY(ba_lidar_pass(ctx, false, f.data(), ring.data(), &r2));
    *res = r1 + r2;
    return VG_OK;
  }
  // damping_iter (optimizers.cpp:745-826), including its state handling:
  // x_stats_temp is initialised once, so a rejected step's gravity increment
  // stays in x_stats_temp[0].g for the next trial (line 775)
  int damping_iter(std::vector<HX>& xs, double resis[2], int max_iter) {
    double u = 0.01, v = 2;
    std::vector<double> H((size_t)n * n), J(n), D(n), Hc, Jc, dxi, mJ(n);
    double residual1 = 0, residual2 = 0, q;
    bool calc = true;
    std::vector<HX> xt = xs;
    for (int i = 0; i < max_iter; i++) {
      if (calc) {
        VG_TRY(hessian(xs, H, J, &residual1));
        Hc = H;
        Jc = J;
      } else {
        H = Hc;
        J = Jc;
      }
      if (i == 0) resis[0] = residual1;
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < n; c++) H[(size_t)r * n + c] = H[(size_t)c * n + r] = 0.0;
      for (int r = 0; r < 6; r++) {
        H[(size_t)r * n + r] = 1.0;
        J[r] = 0.0;
      }
      for (int r = 0; r < n; r++) D[r] = H[(size_t)r * n + r];
      std::vector<double> A = H;
      for (int r = 0; r < n; r++) A[(size_t)r * n + r] += u * D[r];
      for (int r = 0; r < n; r++) mJ[r] = -J[r];
      ldlt_solve(A, n, mJ, dxi);
      for (int k = 0; k < 3; k++) xt[0].g[k] += dxi[n - 3 + k];
      for (int j = 0; j < W; j++) {
        xt[j].R = mul(xs[j].R, Exp(v3(dxi[15 * j], dxi[15 * j + 1], dxi[15 * j + 2])));
        for (int k = 0; k < 3; k++) {
          xt[j].p[k] = xs[j].p[k] + dxi[15 * j + 3 + k];
          xt[j].v[k] = xs[j].v[k] + dxi[15 * j + 6 + k];
          xt[j].bg[k] = xs[j].bg[k] + dxi[15 * j + 9 + k];
          xt[j].ba[k] = xs[j].ba[k] + dxi[15 * j + 12 + k];
        }
        xt[j].g = xt[0].g;
      }
      for (int j = 0; j < W - 1; j++) {  // IMU_PRE::update_state (imu_preintegration.cpp:239-246)
        double* b = &bias[(size_t)j * 12];
        for (int k = 0; k < 6; k++) b[6 + k] = b[k];
        for (int k = 0; k < 3; k++) {
          b[k] += dxi[15 * j + 9 + k];
          b[3 + k] += dxi[15 * j + 12 + k];
        }
      }
      double q1 = 0;
      for (int r = 0; r < n; r++) q1 += dxi[r] * (u * D[r] * dxi[r] - J[r]);
      q1 *= 0.5;
      VG_TRY(residual(xt, &residual2));
      q = residual1 - residual2;
      if (q > 0) {
        xs = xt;
        const double one_three = 1.0 / 3;
        q = q / q1;
        v = 2;
        q = 1 - std::pow(2 * q - 1, 3);
        u *= (q < one_three ? one_three : q);
        calc = true;
      } else {
        u = u * v;
        v = 2 * v;
        calc = false;
        for (int j = 0; j < W - 1; j++)
          for (int k = 0; k < 6; k++) bias[(size_t)j * 12 + k] = bias[(size_t)j * 12 + 6 + k];
      }
      if (std::fabs((residual1 - residual2) / residual1) < 1e-6) break;
    }
    resis[1] = residual2;
    return VG_OK;
  }
};

// Eigen::AngleAxisd(angle, axis).toRotationMatrix()
static M3 angle_axis(double angle, const V3& axis) {
  const V3 sa = scl(axis, std::sin(angle));
  const double c = std::cos(angle);
  const V3 ca = scl(axis, 1 - c);
  M3 m;
  double t = ca[0] * axis[1];
  m(0, 1) = t - sa[2];
  m(1, 0) = t + sa[2];
  t = ca[0] * axis[2];
  m(0, 2) = t + sa[1];
  m(2, 0) = t - sa[1];
  t = ca[1] * axis[2];
  m(1, 2) = t - sa[0];
  m(2, 1) = t + sa[0];
  for (int j = 0; j < 3; j++) m(j, j) = ca[j] * axis[j] + c;
  return m;
}

// Initialization::align_gravity — initialization.cpp:28-62
static void align_gravity(std::vector<HX>& xs) {
  V3 g0 = xs[0].g;
  const V3 n0 = scl(g0, 1.0 / norm3(g0));
  V3 n1 = v3(0, 0, 1);
  if (n0[2] < 0) n1[2] = -1;
  V3 rv = cross3(n0, n1);
  const double rn = norm3(rv);
  rv = scl(rv, 1.0 / rn);
  const M3 rot = angle_axis(std::asin(rn), rv);
  g0 = mul(rot, g0);
  const V3 p0 = xs[0].p;
  for (HX& x : xs) {
    x.p = add(mul(rot, sub(x.p, p0)), p0);
    x.R = mul(rot, x.R);
    x.v = mul(rot, x.v);
    x.g = g0;
  }
}

static std::vector<double> frame_block(const HX& x) {  // kXC: frame state + covariance
  std::vector<double> b(kXC);
  put_frame(x, b.data());
  memcpy(b.data() + kXS, x.cov.a, 225 * sizeof(double));
  return b;
}

// Initialization::motion_init — initialization.cpp:158-367. Returns
// converge_flag; *rounds: rounds run; *nf / *nroots: the last recut's factors
// and root voxels; nper: window points per slot.
static int motion_init(vg_ctx* ctx, HostPipe* P, InitState& I, int* rounds, int* nf_out, int* nroots,
                       std::vector<int>& nper) {
  const int W = ctx->cfg.win_size;
  const MP mp_orig = P->mpd;
  MP mp = mp_orig;
  mp.min_eig = 0.02;
  for (int k = 0; k < 4; k++) mp.thre[k] = 1.0 / 4;
  int converge_flag = 0;
  double converge_thre = 0.05;
  bool is_degrade = true;
  nper.assign(W, 0);
  std::vector<HX>& xb = P->x_buf;
  std::vector<std::vector<double>> recs(W - 1);
  for (int k = 0; k < W - 1; k++) recs[k] = P->imu_pre[k].rec;
  *rounds = 0;
  *nf_out = 0;
  for (int it = 0; it < 10; it++) {
    (*rounds)++;
    if (converge_flag == 1) mp = mp_orig;
    VG_TRY(map_reset(ctx));
    {  // the window poses the recut's window view reads (DState::xs)
      std::vector<double> xs((size_t)W * kXS);
      for (int i = 0; i < W; i++) put_frame(xb[i], &xs[(size_t)i * kXS]);
      VG_TRY(state_load(ctx, xs.data(), W, nullptr, nullptr, 0));
    }
    for (int i = 0; i < W; i++) {
      const int l = i == 0 ? 0 : i - 1;
      int no = 0;
      VG_TRY(blur_scan(ctx, I, i, xb[i], xb[l], P->sg, &no));
      const std::vector<double> blk = frame_block(xb[i]);
      VG_HIP(stream_wait(ctx));  // the previous insert has read I.pose
      VG_HIP(hipMemcpy(I.pose, blk.data(), kXC * sizeof(double), hipMemcpyHostToDevice));
      InsPre pre{I.pnt, I.pose, converge_flag == 1 ? 0 : 1};
      VG_TRY(map_insert(ctx, mp, i, no, 0, 0, nullptr, &pre));
      nper[i] = no;
      P->wp_n[i] = no;
    }
    WinArg wa;
    memset(&wa, 0, sizeof(wa));
    for (int i = 0; i < W; i++) {
      wa.mp[i] = i;
      wa.nper[i] = nper[i];
    }
    wa.win_count = W;
    int nf = 0;
    const int r = map_recut(ctx, mp, wa, 0, &nf);
    if (r == kNeedInsertReplay) {
      ctx->err = "initialisation: insert overflow during the map rebuild";
      return VG_E_CAPACITY;
    }
    VG_TRY(r);
    *nf_out = nf;
    VG_HIP(hipMemcpyAsync(ctx->h_pinned, ctx->map.counters, kCntN * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    VG_HIP(hipStreamSynchronize(ctx->stream));
    *nroots = ctx->h_pinned[kCntSlide];
    if (ctx->h_pinned[kCntErr]) {
      ctx->err = std::string("initialisation: device map error flags=") + std::to_string(ctx->h_pinned[kCntErr]);
      return VG_E_CAPACITY;
    }
    if (nf < 10) break;
    GravLM lm(ctx, recs);
    double resis[2] = {0, 0};
    VG_TRY(lm.damping_iter(xb, resis, 3));
    // fresh preintegrations at the new biases (initialization.cpp:283-289)
    P->imu_pre.clear();
    for (int i = 1; i < W; i++) {
      P->imu_pre.emplace_back(xb[i - 1].bg, xb[i - 1].ba);
      HImuPre& q = P->imu_pre.back();
      q.push_imu(I.vec_imus[i], P->noiseMeas, P->noiseWalk, P->sg);
      q.rec.resize(kBaImuRec);
      q.record(q.rec.data());
      recs[i - 1] = q.rec;
    }
    if (std::fabs(resis[0] - resis[1]) / resis[0] < converge_thre && it >= 2) {
      std::vector<double> nrm;
      VG_TRY(ba_factor_normals(ctx, nrm));
      M3 nnt = M3::Z();
      for (size_t a = 0; a < nrm.size() / 3; a++) {
        const V3 c0 = v3(nrm[a * 3], nrm[a * 3 + 1], nrm[a * 3 + 2]);
        nnt = add(nnt, outer3(c0, c0));
      }
      V3 ev;
      M3 U;
      eig3(nnt, ev, U);
      is_degrade = ev[0] < 15;
      converge_thre = 0.01;
      if (converge_flag == 0) {
        align_gravity(xb);
        converge_flag = 1;
        continue;
      }
      break;
    }
  }
  P->x_curr = xb[W - 1];
  const double gnm = norm3(P->x_curr.g);
  if (is_degrade) converge_flag = 0;
  if (gnm < 9.6 || gnm > 10.0) converge_flag = 0;
  I.beg_times.clear();
  I.vec_imus.clear();
  I.n_close.clear();
  I.t_close.clear();
  return converge_flag;
}

// VINA_SLAM::system_reset — node.cpp:368-408
static int system_reset(vg_ctx* ctx, HostPipe* P, InitState& I, const std::vector<Imu>& imus) {
  VG_TRY(map_reset(ctx));
  VG_TRY(kd_reset(ctx));
  P->x_curr = HX();
  P->x_curr.p = v3(0, 0, 30);
  I.mean_acc = V3::Z();
  I.init_num = 0;
  imu_init(I, imus);
  P->x_curr.g = scl(I.mean_acc, -P->sg);
  P->imu_pre.clear();
  P->x_buf.clear();
  for (int i = 0; i < ctx->cfg.win_size; i++) P->mp[i] = i;
  P->win_base = 0;
  P->win_count = 0;
  P->path.clear();  // pcl_path.clear() (node.cpp:403)
  return VG_OK;
}

static void log_scan(vg_ctx* ctx, HostPipe* P, const vg_stats& st) {
  ctx->stats = st;
  P->stats_log.push_back(st);
}

// One scan while motion_init_flag is set (local_mapping.cpp:362-386 ->
// VINA_SLAM::initialization, node.cpp:293-366). dt: per-point time offsets
// from beg (nullptr: every point at end - beg, no deskew).
int init_step(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, const float* dt, int n,
              double beg, double end, const double* imu, int m) {
  HostPipe* P = hp(ctx);
  InitState& I = *P->init;
  const vg_config& c = ctx->cfg;
  const int W = c.win_size;
  if (P->in_scan) {
    ctx->err = "cold start: a stage-level scan is open";
    return VG_E_STATE;
  }
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  VG_TRY(absorb(ctx, P, true));
  VG_TRY(init_dev(ctx, I));
  vg_stats st;
  memset(&st, 0, sizeof(st));
  st.init_phase = 1;
  const std::vector<Imu> imus = to_imus(imu, m);
  // IMUEKF::process (imu_ekf.cpp:174-201) until init_flag: IMU_init over the
  // scan's own samples (not the carried-over last one), the gravity scale
  if (!I.init_flag) {
    if (!imus.empty()) {  // sync_packages never hands over a scan without IMU samples
      std::vector<Imu> own = imus;
      if (own.front().t <= P->last_pcl_end_time && !P->first) own.erase(own.begin());
      imu_init(I, own);
      if (norm3(I.mean_acc) < 2) I.scale_gravity = kGms2;
      P->x_curr.g = scl(I.mean_acc, -I.scale_gravity);
      if (I.init_num > kMinInitNum) I.init_flag = true;
      P->first = false;
    }
    P->last_pcl_end_time = end;
    log_scan(ctx, P, st);
    return VG_OK;
  }
  st.init_phase = 2;
  P->sg = I.scale_gravity;  // mpar.imupre_scale_gravity (node.cpp:309, imu_ekf.cpp)
  propagate(ctx, P, imus, beg, end);
  const int slot = P->win_count;
  if (slot >= W) {
    ctx->err = "cold start: initialisation window overflow";
    return VG_E_STATE;
  }
  // down_sampling_close of the raw sweep (node.cpp:337-343), before the deskew
  // overwrites the staging buffers
  {
    float4* out = I.pool + (size_t)slot * I.cap;
    const float tconst = (float)(end - beg);
    int nc = 0;
    VG_TRY(ds_close(ctx, dx, dy, dz, dt, tconst, n, c.down_size, out, &nc));
    if (nc < 1000) VG_TRY(ds_close(ctx, dx, dy, dz, dt, tconst, n, c.down_size / 2, out, &nc));
    std::vector<float4> h(nc);  // ds_close has drained the stream
    if (nc > 0) VG_HIP(hipMemcpy(h.data(), out, (size_t)nc * sizeof(float4), hipMemcpyDeviceToHost));
    std::vector<float> t(nc);
    for (int k = 0; k < nc; k++) t[k] = h[k].w;
    I.n_close.push_back(nc);
    I.t_close.push_back(std::move(t));
  }
  // motion_blur's deskew (imu_ekf.cpp:114-144) of the sweep
  const float *sx = dx, *sy = dy, *sz = dz, *si = di;
  if (dt && n > 0) {
    const int npose = (int)P->poses.size() / 22;
    std::vector<double> par(24 + P->poses.size());
    memcpy(par.data(), P->x_curr.R.a, 72);
    memcpy(par.data() + 9, P->x_curr.p.a, 24);
    for (int k = 0; k < 9; k++) par[12 + k] = c.ext_R[k];
    for (int k = 0; k < 3; k++) par[21 + k] = c.ext_t[k];
    if (!P->poses.empty()) memcpy(par.data() + 24, P->poses.data(), P->poses.size() * sizeof(double));
    VG_TRY(state_deskew(ctx, par.data(), npose, dx, dy, dz, di, dt, n));
    sx = ctx->d_x;
    sy = ctx->d_y;
    sz = ctx->d_z;
    si = ctx->d_i;
  }
  // down_sampling_voxel at max(down_size, 0.5) + the kd-tree IEKF (A14)
  int n_ds = 0;
  VG_TRY(ds_run(ctx, sx, sy, sz, si, n, c.down_size >= 0.5 ? c.down_size : 0.5, &n_ds));
  int valid = -1, iters = 0;
  if (n_ds > 0) {
    hipStream_t s = ctx->stream;
    VG_HIP(hipMemcpyAsync(ctx->d_x, ctx->ds.ox, (size_t)n_ds * sizeof(float), hipMemcpyDeviceToDevice, s));
    VG_HIP(hipMemcpyAsync(ctx->d_y, ctx->ds.oy, (size_t)n_ds * sizeof(float), hipMemcpyDeviceToDevice, s));
    VG_HIP(hipMemcpyAsync(ctx->d_z, ctx->ds.oz, (size_t)n_ds * sizeof(float), hipMemcpyDeviceToDevice, s));
    VG_TRY(kd_lio(ctx, n_ds, P->x_curr, &valid, &iters));
  }
  st.iekf_iters = iters;
  st.n_raw = n;
  st.n_ds = n_ds;
  st.init_valid = valid;
  // pub_localtraj(pwld, 0, x_curr, 0, pcl_path) (node.cpp:325): a path point
  // with jour 0; no save_pose_tum row during the initialisation
  P->path.push_back(end);
  for (int k = 0; k < 9; k++) P->path.push_back(P->x_curr.R.a[k]);
  for (int k = 0; k < 3; k++) P->path.push_back(P->x_curr.p.a[k]);
  P->path.push_back(0.0);
  // x_buf / imu_pre_buf (node.cpp:321-330)
  P->win_count++;
  P->x_buf.push_back(P->x_curr);
  P->x_buf.back().t = end;
  if (P->win_count > 1) {
    const HX& xb = P->x_buf[P->win_count - 2];
    P->imu_pre.emplace_back(xb.bg, xb.ba);
    HImuPre& q = P->imu_pre.back();
    q.push_imu(imus, P->noiseMeas, P->noiseWalk, P->sg);
    q.rec.resize(kBaImuRec);
    q.record(q.rec.data());
  }
  I.beg_times.push_back(beg);
  I.vec_imus.push_back(imus);
  if (P->win_count < W) {
    log_scan(ctx, P, st);
    return VG_OK;
  }
  int rounds = 0, nf = 0, nroots = 0;
  std::vector<int> nper;
  const int ok = motion_init(ctx, P, I, &rounds, &nf, &nroots, nper);
  st.init_rounds = rounds;
  if (!ok) {
    st.init_phase = 4;
    VG_TRY(system_reset(ctx, P, I, imus));
    log_scan(ctx, P, st);
    return VG_OK;
  }
  // success: the device takes over the window (x_buf, x_curr, IMU records; the
  // map and the factors of the last round are already there) and the same
  // scan runs the window tail (local_mapping.cpp:489-546)
  st.init_phase = 3;
  st.n_factors = nf;
  st.roots_new = nroots;
  I.active = false;
  {
    std::vector<double> xs((size_t)W * kXS), recs((size_t)(W - 1) * kBaImuRec);
    for (int i = 0; i < W; i++) put_frame(P->x_buf[i], &xs[(size_t)i * kXS]);
    for (int k = 0; k < W - 1; k++) memcpy(&recs[(size_t)k * kBaImuRec], P->imu_pre[k].rec.data(), kBaImuRec * 8);
    const std::vector<double> xc = frame_block(P->x_curr);
    VG_TRY(state_load(ctx, xs.data(), W, xc.data(), recs.data(), W - 1));
  }
  for (int i = 0; i < W; i++) P->mp[i] = i;
  P->n_factors = nf;
  P->first = false;
  P->cur = Pend();
  P->cur.st = st;
  P->cur.t = end;
  P->cur.init_tail = true;
  P->in_scan = true;
  P->published = false;
  P->begin_pending = false;
  P->push_pending = false;
  P->ds_seq = 0;
  P->ds_n = -1;
  P->ins_slot = -1;
  P->prefix = false;
  P->rc_seq = 0;
  if (c.if_BA == 1) VG_TRY(stage_ba(ctx, nullptr, true));
  VG_TRY(stage_margi_slide(ctx));
  return stage_finish(ctx);
}

}  // namespace vg
