// ba.hip — sliding-window LiDAR-inertial LM.
//
// Replaces LI_BA_Optimizer::damping_iter (optimizers.cpp:430-517) with its
// divide_thread / only_residual / hess_plus (171-245, 340-376), the point-
// cluster factor LidarFactor::acc_evaluate2 / evaluate_only_residual
// (factors.cpp:22-158) and IMU_PRE::give_evaluate / update_state
// (imu_preintegration.cpp:97-163, 239-246).
//
// Per LM iteration, all device-resident, no host round trip:
//   k_ba_comp    one lane per (factor, frame): Auk (3x6), viRiTuk, the diagonal
//                6x6 block and the gradient piece                (fp64 VALU)
//   k_ba_hred    one workgroup per chunk of 16 factors staged in LDS: every
//                lane owns output entries of the 60x60 lower triangle + 60 + 1
//                and sums the chunk -> per-chunk partials (deterministic)
//   k_ba_hfinal  ordered sum of the chunk partials
//   k_ba_imu     one workgroup per IMU factor: residual, 15x30 Jacobian,
//                J^T C J (30x30) and J^T C r
//   k_ba_solve   one 1024-lane workgroup: assemble the 15W x 15W system
//                (IMU blocks x imu_coef + LiDAR 6x6 blocks), gauge frame 0,
//                Marquardt damping, LDL^T with diagonal pivoting in LDS
//                (lower triangle, 90 KB), the trial state and q1
//   k_ba_resid   one lane per factor: merge clusters at the trial poses, 3x3
//                eigen, write the trial eig/cluster (the side effect margi
//                consumes), chunk residual partials
//   k_ba_imures  IMU residuals at the trial state
//   k_ba_control LM accept/reject, Nielsen damping update, bias restore,
//                convergence flag (1 lane)
// Kernels early-exit on the device-side `done` / `calc_hess` flags, so the
// host enqueues all 10 iterations (optimizers.cpp:449) without syncing.
#include "vg_dev.h"

namespace vg {

constexpr int kMaxW = 16;
constexpr int kComp = 49;     // per (factor, frame): Auk 18, viRiTuk 3, ni 1, Hb lower 21, jjt 6
constexpr int kCompF = 24;    // per factor: umumT 9, ukukT 9, uk 3, NN, coe, lmbd0
constexpr int kFC = 16;       // factors per reduction chunk
constexpr int kImuRec = 64 + 225;  // preintegration record + cov_inv

struct BaState {             // device-resident LM state
  double u, v, res1, res2, q1;
  int calc_hess, done, iters, pad;
};

// x state per frame: R 9, p 3, v 3, bg 3, ba 3, g 3 = 24 doubles
constexpr int kX = 24;

__device__ __forceinline__ void factor_basics(const double* e, const Clu& pcr, double* f) {
  // f: umumT(9) ukukT(9) uk(3) NN lmbd0
  V3 u[3];
  for (int k = 0; k < 3; k++) u[k] = v3(e[3 + 0 * 3 + k], e[3 + 1 * 3 + k], e[3 + 2 * 3 + k]);
  M3 um;
  um.zero();
  for (int i = 1; i < 3; i++) {
    M3 o = outer3(u[i], u[i]);
    double c = 2.0 / (e[0] - e[i]);
    for (int t = 0; t < 9; t++) um[t] += o[t] * c;
  }
  M3 uu = outer3(u[0], u[0]);
  for (int t = 0; t < 9; t++) {
    f[t] = um[t];
    f[9 + t] = uu[t];
  }
  for (int t = 0; t < 3; t++) f[18 + t] = u[0][t];
  f[21] = (double)pcr.N;
  f[22] = 1.0;  // coe (octree.cpp:507)
  f[23] = e[0];
}

// acc_evaluate2 per (factor, frame) — factors.cpp:57-97
__global__ void __launch_bounds__(256) k_ba_comp(int nf, int W, const int* __restrict__ fac_node, const double* __restrict__ fac_eig,
                          const Clu* __restrict__ fac_pcr, const Clu* __restrict__ pcrs, const int* __restrict__ mpring,
                          const double* __restrict__ xs, double* __restrict__ comp, double* __restrict__ compf,
                          const BaState* __restrict__ st) {
  if (st->done || !st->calc_hess) return;
  const int total = nf * W;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int a = t / W, i = t % W;
    const double* e = &fac_eig[(size_t)a * 12];
    const Clu pa = fac_pcr[a];
    double f[kCompF];
    factor_basics(e, pa, f);
    if (i == 0)
      for (int k = 0; k < kCompF; k++) compf[(size_t)a * kCompF + k] = f[k];
    double* o = &comp[((size_t)a * W + i) * kComp];
    const Clu s = pcrs[(size_t)fac_node[a] * W + mpring[i]];
    if (s.N == 0) {
      for (int k = 0; k < kComp; k++) o[k] = 0.0;
      continue;
    }
    const double NN = f[21];
    M3 umumT, ukukT;
    for (int k = 0; k < 9; k++) {
      umumT[k] = f[k];
      ukukT[k] = f[9 + k];
    }
    const V3 uk = v3(f[18], f[19], f[20]);
    const V3 vBar = v3(pa.v[0] / NN, pa.v[1] / NN, pa.v[2] / NN);
    const M3 Pi = clu_Pm(s);
    const V3 vi = clu_v(s);
    const M3 Ri = ld_m3(&xs[(size_t)i * kX]);
    const double ni = (double)s.N;
    const M3 vihat = hat(vi);
    const V3 RiTuk = mul(tr(Ri), uk);
    const M3 RiTukhat = hat(RiTuk);
    const V3 PiRiTuk = mul(Pi, RiTuk);
    const V3 viRiTuk = mul(vihat, RiTuk);
    const V3 ti_v = sub(ld_v3(&xs[(size_t)i * kX + 9]), vBar);
    const double ukTti_v = dot3(uk, ti_v);
    const M3 combo1 = add(hat(PiRiTuk), scl(vihat, ukTti_v));
    const V3 combo2 = add(mul(Ri, vi), scl(ti_v, ni));
    M<3, 6> A;
    M3 A1 = sub(mul(add(mul(Ri, Pi), outer3(ti_v, vi)), RiTukhat), mul(Ri, combo1));
    M3 A2 = add(outer3(combo2, uk), scl(M3::I(), dot3(combo2, uk)));
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        A(r, c) = A1(r, c) / NN;
        A(r, 3 + c) = A2(r, c) / NN;
      }
    V6 jjt = mul(tr(A), uk);
    M3 HRt = scl(outer3(viRiTuk, uk), 2.0 / NN * (1.0 - ni / NN));
    M6 Hb = mul(mul(tr(A), umumT), A);
    M3 c00 = sub(sub(scl(mul(sub(combo1, mul(RiTukhat, Pi)), RiTukhat), 2.0 / NN),
                     scl(outer3(viRiTuk, viRiTuk), 2.0 / NN / NN)),
                 scl(hat(v3(jjt[0], jjt[1], jjt[2])), 0.5));
    M3 c11 = scl(ukukT, 2.0 / NN * (ni - ni * ni / NN));
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        Hb(r, c) += c00(r, c);
        Hb(r, 3 + c) += HRt(r, c);
        Hb(3 + r, c) += HRt(c, r);
        Hb(3 + r, 3 + c) += c11(r, c);
      }
    for (int k = 0; k < 18; k++) o[k] = A[k];
    for (int k = 0; k < 3; k++) o[18 + k] = viRiTuk[k];
    o[21] = ni;
    int q = 22;
    for (int r = 0; r < 6; r++)
      for (int c = 0; c <= r; c++) o[q++] = Hb(r, c);  // lower triangle
    for (int k = 0; k < 6; k++) o[43 + k] = jjt[k];
  }
}

// outputs: 1830 lower entries of the 6W x 6W LiDAR Hessian (row-major lower),
// then 6W gradient, then the residual
__device__ __forceinline__ int lower_idx(int r, int c) { return r * (r + 1) / 2 + c; }

__global__ void __launch_bounds__(256) k_ba_hred(int nf, int W, const double* __restrict__ comp,
                                                 const double* __restrict__ compf, double* __restrict__ part,
                                                 const BaState* __restrict__ st) {
  if (st->done || !st->calc_hess) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int a0 = blockIdx.x * kFC;
  const int na = min(kFC, nf - a0);
  const int per = W * kComp + kCompF;
  for (int t = threadIdx.x; t < na * per; t += blockDim.x) {
    int a = t / per, k = t % per;
    sm[t] = (k < W * kComp) ? comp[((size_t)(a0 + a) * W) * kComp + k] : compf[(size_t)(a0 + a) * kCompF + (k - W * kComp)];
  }
  __syncthreads();
  const int L = 6 * W;
  const int nl = L * (L + 1) / 2;
  const int nout = nl + L + 1;
  for (int e = threadIdx.x; e < nout; e += blockDim.x) {
    double acc = 0.0;
    if (e < nl) {
      int row = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      while (lower_idx(row + 1, 0) <= e) row++;
      while (lower_idx(row, 0) > e) row--;
      int col = e - lower_idx(row, 0);
      int bi = row / 6, r = row % 6, bj = col / 6, c = col % 6;
      for (int a = 0; a < na; a++) {
        const double* F = &sm[a * per + W * kComp];
        const double coe = F[22];
        if (bi == bj) {
          const double* o = &sm[a * per + bi * kComp];
          if (o[21] != 0.0) acc += coe * o[22 + lower_idx(r, c)];
        } else {
          // lower entry (6bi+r, 6bj+c) = upper block (i=bj, j=bi) entry (c, r)
          const double* oi = &sm[a * per + bj * kComp];
          const double* oj = &sm[a * per + bi * kComp];
          const double ni = oi[21], nj = oj[21];
          if (ni == 0.0 || nj == 0.0) continue;
          const double NN = F[21];
          // (Auk_i^T umumT Auk_j)(c, r)
          double tmp[3];
          for (int k = 0; k < 3; k++) tmp[k] = F[k * 3 + 0] * oj[0 * 6 + r] + F[k * 3 + 1] * oj[1 * 6 + r] + F[k * 3 + 2] * oj[2 * 6 + r];
          double hb = oi[0 * 6 + c] * tmp[0] + oi[1 * 6 + c] * tmp[1] + oi[2 * 6 + c] * tmp[2];
          const double* vi = &oi[18];
          const double* vj = &oj[18];
          const double* uk = &F[18];
          if (c < 3 && r < 3) hb += -2.0 / NN / NN * (vi[c] * vj[r]);
          else if (c < 3) hb += -2.0 * nj / NN / NN * (vi[c] * uk[r - 3]);
          else if (r < 3) hb += -2.0 * ni / NN / NN * (uk[c - 3] * vj[r]);
          else hb += -2.0 * ni * nj / NN / NN * (uk[c - 3] * uk[r - 3]);
          acc += coe * hb;
        }
      }
    } else if (e < nl + L) {
      int g = e - nl, bi = g / 6, r = g % 6;
      for (int a = 0; a < na; a++) {
        const double* o = &sm[a * per + bi * kComp];
        acc += sm[a * per + W * kComp + 22] * o[43 + r];
      }
    } else {
      for (int a = 0; a < na; a++) acc += sm[a * per + W * kComp + 22] * sm[a * per + W * kComp + 23];
    }
    part[(size_t)blockIdx.x * nout + e] = acc;
  }
}

// ordered sum of the chunk partials: 8 lanes per output split the chunks
// (stride 8), then a fixed 3-step shuffle tree (deterministic)
__global__ void __launch_bounds__(256) k_ba_hfinal(int nchunk, int nout, const double* __restrict__ part,
                                                   double* __restrict__ out, const BaState* __restrict__ st) {
  if (st->done || !st->calc_hess) return;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = gt >> 3, sub = gt & 7;
  double s = 0.0;
  if (e < nout)
    for (int b = sub; b < nchunk; b += 8) s += part[(size_t)b * nout + e];
  s += __shfl_down(s, 4, 8);
  s += __shfl_down(s, 2, 8);
  s += __shfl_down(s, 1, 8);
  if (e < nout && sub == 0) out[e] = s;
}

// IMU record layout (doubles): R_delta 9, p_delta 3, v_delta 3, R_bg 9, p_bg 9,
// p_ba 9, v_bg 9, v_ba 9, dtime 1 (=61), pad to 64, cov_inv 225.
// bias state per factor: dbg 3, dba 3, dbg_buf 3, dba_buf 3.
__device__ void imu_residual(const double* rec, const double* bias, const double* x1, const double* x2, double* rr,
                             double* joc /*15x30 or null*/) {
  const M3 Rd = ld_m3(rec), Rbg = ld_m3(rec + 15), pbg = ld_m3(rec + 24), pba = ld_m3(rec + 33),
           vbg = ld_m3(rec + 42), vba = ld_m3(rec + 51);
  const V3 pd = ld_v3(rec + 9), vd = ld_v3(rec + 12);
  const double dtime = rec[60];
  const V3 dbg = ld_v3(bias), dba = ld_v3(bias + 3);
  const M3 R1 = ld_m3(x1), R2 = ld_m3(x2);
  const V3 p1 = ld_v3(x1 + 9), p2 = ld_v3(x2 + 9), v1 = ld_v3(x1 + 12), v2 = ld_v3(x2 + 12);
  const V3 bg1 = ld_v3(x1 + 15), bg2 = ld_v3(x2 + 15), ba1 = ld_v3(x1 + 18), ba2 = ld_v3(x2 + 18);
  const V3 g1 = ld_v3(x1 + 21);
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

// give_evaluate with jac_enable at the current state; out per factor: jtj 900, gg 30, res 1
__global__ void __launch_bounds__(256) k_ba_imu(int nimu, const double* __restrict__ imurec,
                                                const double* __restrict__ bias, const double* __restrict__ xs,
                                                double* __restrict__ out, const BaState* __restrict__ st) {
  if (st->done || !st->calc_hess) return;
  const int k = blockIdx.x;
  if (k >= nimu) return;
  __shared__ double joc[450], rr[15], P[450], C[225];
  const double* rec = &imurec[(size_t)k * kImuRec];
  if (threadIdx.x == 0) imu_residual(rec, &bias[k * 12], &xs[(size_t)k * kX], &xs[(size_t)(k + 1) * kX], rr, joc);
  for (int t = threadIdx.x; t < 225; t += blockDim.x) C[t] = rec[64 + t];
  __syncthreads();
  // P = joc^T C (30 x 15)
  for (int t = threadIdx.x; t < 450; t += blockDim.x) {
    int r = t / 15, l = t % 15;
    double s = joc[0 * 30 + r] * C[0 * 15 + l];
    for (int q = 1; q < 15; q++) s += joc[q * 30 + r] * C[q * 15 + l];
    P[t] = s;
  }
  __syncthreads();
  double* o = &out[(size_t)k * 931];
  for (int t = threadIdx.x; t < 900; t += blockDim.x) {
    int r = t / 30, c = t % 30;
    double s = P[r * 15 + 0] * joc[0 * 30 + c];
    for (int l = 1; l < 15; l++) s += P[r * 15 + l] * joc[l * 30 + c];
    o[t] = s;
  }
  if (threadIdx.x < 30) {
    int r = threadIdx.x;
    double s = P[r * 15 + 0] * rr[0];
    for (int l = 1; l < 15; l++) s += P[r * 15 + l] * rr[l];
    o[900 + r] = s;
  }
  if (threadIdx.x == 0) {
    double cr[15];
    for (int r = 0; r < 15; r++) {
      double s = C[r * 15] * rr[0];
      for (int l = 1; l < 15; l++) s += C[r * 15 + l] * rr[l];
      cr[r] = s;
    }
    double s = rr[0] * cr[0];
    for (int r = 1; r < 15; r++) s += rr[r] * cr[r];
    o[930] = s;
  }
}

// IMU residuals only (give_evaluate(..., false)) at the trial state
__global__ void __launch_bounds__(256) k_ba_imures(int nimu, const double* __restrict__ imurec, const double* __restrict__ bias,
                            const double* __restrict__ xt, double* __restrict__ res, const BaState* __restrict__ st) {
  if (st->done) return;
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nimu) return;
  const double* rec = &imurec[(size_t)k * kImuRec];
  double rr[15];
  imu_residual(rec, &bias[k * 12], &xt[(size_t)k * kX], &xt[(size_t)(k + 1) * kX], rr, nullptr);
  double cr[15];
  for (int r = 0; r < 15; r++) {
    double s = rec[64 + r * 15] * rr[0];
    for (int l = 1; l < 15; l++) s += rec[64 + r * 15 + l] * rr[l];
    cr[r] = s;
  }
  double s = rr[0] * cr[0];
  for (int r = 1; r < 15; r++) s += rr[r] * cr[r];
  res[k] = s;
}

// packed lower storage of the n x n system
__device__ __forceinline__ int lo(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// assemble (or reload), gauge, damp, LDL^T-solve, trial state, IMU bias trial
__global__ void __launch_bounds__(1024) k_ba_solve(int W, int nimu, double imu_coef, const double* __restrict__ hl,
                                                   const double* __restrict__ imuout, double* __restrict__ Hcalc,
                                                   double* __restrict__ Jcalc, const double* __restrict__ xs,
                                                   double* __restrict__ xt, double* __restrict__ bias,
                                                   double* __restrict__ dxi_out, BaState* __restrict__ st) {
  if (st->done) return;
  extern __shared__ __attribute__((aligned(16))) double A[];
  const int n = 15 * W;
  const int nn = n * (n + 1) / 2;
  __shared__ double J[15 * kMaxW], D[15 * kMaxW], col[15 * kMaxW], y[15 * kMaxW];
  __shared__ int perm[15 * kMaxW];
  __shared__ int piv;
  const int tid = threadIdx.x, nt = blockDim.x;
  const bool calc = st->calc_hess != 0;
  const double u = st->u;
  if (calc) {
    for (int t = tid; t < nn; t += nt) A[t] = 0.0;
    for (int t = tid; t < n; t += nt) J[t] = 0.0;
    __syncthreads();
    // IMU blocks: rows/cols 15k .. 15k+29, accumulated in k order (divide_thread 215-222)
    for (int k = 0; k < nimu; k++) {
      const double* o = &imuout[(size_t)k * 931];
      for (int t = tid; t < 900; t += nt) {
        int r = t / 30, c = t % 30;
        if (r >= c) A[lo(15 * k + r, 15 * k + c)] += o[t];
      }
      for (int t = tid; t < 30; t += nt) J[15 * k + t] += o[900 + t];
      __syncthreads();
    }
    for (int t = tid; t < nn; t += nt) A[t] *= imu_coef;
    for (int t = tid; t < n; t += nt) J[t] *= imu_coef;
    __syncthreads();
    // hess_plus (optimizers.cpp:171-179): LiDAR 6x6 blocks into the rot/pos sub-blocks
    const int L = 6 * W;
    for (int t = tid; t < L * (L + 1) / 2; t += nt) {
      int row = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
      while ((row + 1) * (row + 2) / 2 <= t) row++;
      while (row * (row + 1) / 2 > t) row--;
      int colx = t - row * (row + 1) / 2;
      int R = (row / 6) * 15 + row % 6, C = (colx / 6) * 15 + colx % 6;
      A[lo(R, C)] += hl[t];
    }
    for (int t = tid; t < L; t += nt) J[(t / 6) * 15 + t % 6] += hl[L * (L + 1) / 2 + t];
    __syncthreads();
    for (int t = tid; t < nn; t += nt) Hcalc[t] = A[t];
    for (int t = tid; t < n; t += nt) Jcalc[t] = J[t];
  } else {
    for (int t = tid; t < nn; t += nt) A[t] = Hcalc[t];
    for (int t = tid; t < n; t += nt) J[t] = Jcalc[t];
  }
  __syncthreads();
  // gauge frame 0 (optimizers.cpp:460-463)
  for (int t = tid; t < 15 * n; t += nt) {
    int r = t / n, c = t % n;
    A[lo(r, c)] = (r == c) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int t = tid; t < n; t += nt) {
    if (t < 15) J[t] = 0.0;
    D[t] = A[lo(t, t)];
    perm[t] = t;
  }
  __syncthreads();
  for (int t = tid; t < n; t += nt) A[lo(t, t)] += u * D[t];
  __syncthreads();
  // LDL^T with diagonal pivoting (largest remaining |d|, first index on ties,
  // as Eigen::LDLT / the oracle): the pivot is swapped physically (symmetric
  // row+column swap in the packed lower triangle), so every step updates the
  // contiguous trailing triangle with a 32 x 32 lane tiling.
  const int tr_ = tid >> 5, tc_ = tid & 31;
  for (int k = 0; k < n; k++) {
    if (tid < 64) {
      double best = -1.0;
      int bi = n;
      for (int i = k + tid; i < n; i += 64) {
        double v = fabs(A[lo(i, i)]);
        if (v > best) {
          best = v;
          bi = i;
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        double ob = __shfl_down(best, off, 64);
        int oi = __shfl_down(bi, off, 64);
        if (ob > best || (ob == best && oi < bi)) {
          best = ob;
          bi = oi;
        }
      }
      if (tid == 0) piv = bi;
    }
    __syncthreads();
    const int p = piv;
    if (p != k) {
      for (int j = tid; j < n; j += nt) {
        if (j < k) {
          double t = A[lo(k, j)]; A[lo(k, j)] = A[lo(p, j)]; A[lo(p, j)] = t;
        } else if (j == k) {
          double t = A[lo(k, k)]; A[lo(k, k)] = A[lo(p, p)]; A[lo(p, p)] = t;
          int q = perm[k]; perm[k] = perm[p]; perm[p] = q;
        } else if (j < p) {
          double t = A[lo(j, k)]; A[lo(j, k)] = A[lo(p, j)]; A[lo(p, j)] = t;
        } else if (j > p) {
          double t = A[lo(j, k)]; A[lo(j, k)] = A[lo(j, p)]; A[lo(j, p)] = t;
        }
      }
      __syncthreads();
    }
    const double dk = A[lo(k, k)];
    for (int i = k + 1 + tid; i < n; i += nt) col[i] = A[lo(i, k)];
    __syncthreads();
    for (int i = k + 1 + tr_; i < n; i += 32) {
      const double lik = (dk != 0.0) ? col[i] / dk : 0.0;
      const int base = i * (i + 1) / 2;
      for (int j = k + 1 + tc_; j <= i; j += 32) A[base + j] -= lik * col[j];
      if (tc_ == 0) A[base + k] = lik;
    }
    __syncthreads();
  }
  // triangular solves on one wave, y held in registers (lane owns rows lane + 64 r)
  if (tid < 64) {
    double yv[3];
    for (int r = 0; r < 3; r++) {
      int i = tid + 64 * r;
      yv[r] = i < n ? -J[perm[i]] : 0.0;
    }
    for (int k = 0; k < n; k++) {  // L y = P(-J)
      const double yk = __shfl(yv[k >> 6], k & 63, 64);
      for (int r = 0; r < 3; r++) {
        int i = tid + 64 * r;
        if (i > k && i < n) yv[r] -= A[lo(i, k)] * yk;
      }
    }
    for (int r = 0; r < 3; r++) {
      int i = tid + 64 * r;
      if (i < n) {
        double d = A[lo(i, i)];
        yv[r] = (d != 0.0) ? yv[r] / d : 0.0;
      }
    }
    for (int k = n - 1; k >= 0; k--) {  // L^T x = y
      const double yk = __shfl(yv[k >> 6], k & 63, 64);
      for (int r = 0; r < 3; r++) {
        int i = tid + 64 * r;
        if (i < k) yv[r] -= A[lo(k, i)] * yk;
      }
    }
    for (int r = 0; r < 3; r++) {
      int i = tid + 64 * r;
      if (i < n) y[i] = yv[r];
    }
  }
  __syncthreads();
  for (int t = tid; t < n; t += nt) col[perm[t]] = y[t];
  __syncthreads();
  // trial states (optimizers.cpp:468-475) and IMU bias trial (477-478)
  if (tid < W) {
    const int j = tid;
    const double* x = &xs[(size_t)j * kX];
    double* o = &xt[(size_t)j * kX];
    M3 Rn = mul(ld_m3(x), Exp(v3(col[15 * j], col[15 * j + 1], col[15 * j + 2])));
    for (int t = 0; t < 9; t++) o[t] = Rn[t];
    for (int t = 0; t < 3; t++) {
      o[9 + t] = x[9 + t] + col[15 * j + 3 + t];
      o[12 + t] = x[12 + t] + col[15 * j + 6 + t];
      o[15 + t] = x[15 + t] + col[15 * j + 9 + t];
      o[18 + t] = x[18 + t] + col[15 * j + 12 + t];
      o[21 + t] = x[21 + t];
    }
    if (j < nimu) {
      double* b = &bias[j * 12];
      for (int t = 0; t < 3; t++) {
        b[6 + t] = b[t];
        b[9 + t] = b[3 + t];
        b[t] += col[15 * j + 9 + t];
        b[3 + t] += col[15 * j + 12 + t];
      }
    }
  }
  for (int t = tid; t < n; t += nt) dxi_out[t] = col[t];
  if (tid == 0) {
    double q1 = 0.0;
    for (int r = 0; r < n; r++) q1 += col[r] * (u * D[r] * col[r] - J[r]);
    st->q1 = 0.5 * q1;
  }
}

// evaluate_only_residual (factors.cpp:128-158) at the trial poses
__global__ void __launch_bounds__(256) k_ba_resid(int nf, int W, const int* __restrict__ fac_node,
                                                  const Clu* __restrict__ pcr_fix, const Clu* __restrict__ pcrs,
                                                  const int* __restrict__ mpring, const double* __restrict__ xt,
                                                  double* __restrict__ fac_eig, Clu* __restrict__ fac_pcr,
                                                  double* __restrict__ rpart, const BaState* __restrict__ st) {
  if (st->done) return;
  double acc = 0.0;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a < nf) {
    const int node = fac_node[a];
    Clu sig = pcr_fix[node];
    for (int i = 0; i < W; i++) {
      const Clu s = pcrs[(size_t)node * W + mpring[i]];
      if (s.N != 0) {
        Clu t = clu_transform(s, ld_m3(&xt[(size_t)i * kX]), ld_v3(&xt[(size_t)i * kX + 9]));
        clu_add(sig, t);
      }
    }
    V3 ev;
    M3 U;
    eig3(clu_cov(sig), ev, U);
    double* e = &fac_eig[(size_t)a * 12];
    for (int j = 0; j < 3; j++) e[j] = ev[j];
    for (int j = 0; j < 9; j++) e[3 + j] = U[j];
    fac_pcr[a] = sig;
    acc = 1.0 * ev[0];
  }
  __shared__ double red[4];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) rpart[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// LM bookkeeping (optimizers.cpp:480-515)
__global__ void __launch_bounds__(256) k_ba_control(int W, int nimu, int nrb, double imu_coef, const double* __restrict__ hl, int nl,
                             const double* __restrict__ imuout, const double* __restrict__ imures,
                             const double* __restrict__ rpart, double* __restrict__ xs,
                             const double* __restrict__ xt, double* __restrict__ bias, BaState* __restrict__ st) {
  __shared__ int accept;
  if (threadIdx.x == 0) {
    accept = -1;
    if (!st->done) {
      if (st->calc_hess) {  // residual1 of divide_thread at the current state
        double r = 0.0;
        for (int k = 0; k < nimu; k++) r += imuout[(size_t)k * 931 + 930];
        r *= imu_coef * 0.5;
        r += hl[nl];
        st->res1 = r;
      }
      double r1 = 0.0;
      for (int k = 0; k < nimu; k++) r1 += imures[k];
      r1 *= imu_coef * 0.5;
      double r2 = 0.0;
      for (int b = 0; b < nrb; b++) r2 += rpart[b];
      const double residual2 = r1 + r2;
      st->res2 = residual2;
      const double residual1 = st->res1;
      double q = residual1 - residual2;
      if (q > 0) {
        accept = 1;
        const double one_three = 1.0 / 3;
        q = q / st->q1;
        st->v = 2;
        q = 1 - pow(2 * q - 1, 3);
        st->u *= (q < one_three ? one_three : q);
        st->calc_hess = 1;
      } else {
        accept = 0;
        st->u = st->u * st->v;
        st->v = 2 * st->v;
        st->calc_hess = 0;
      }
      st->iters += 1;
      if (fabs((residual1 - residual2) / residual1) < 1e-6) st->done = 1;
    }
  }
  __syncthreads();
  if (accept == 1) {
    for (int t = threadIdx.x; t < W * kX; t += blockDim.x) xs[t] = xt[t];
  } else if (accept == 0) {
    for (int t = threadIdx.x; t < nimu * 6; t += blockDim.x) {
      int k = t / 6, j = t % 6;
      bias[k * 12 + j] = bias[k * 12 + 6 + j];
    }
  }
}

__global__ void __launch_bounds__(256) k_ba_init(BaState* st) {
  st->u = 0.01;
  st->v = 2;
  st->res1 = st->res2 = st->q1 = 0.0;
  st->calc_hess = 1;
  st->done = 0;
  st->iters = 0;
}

struct BaDev {
  double* comp;
  double* compf;
  double* part;
  double* hl;
  double* imurec;
  double* bias;
  double* imuout;
  double* imures;
  double* Hcalc;
  double* Jcalc;
  double* xs;
  double* xt;
  double* dxi;
  double* rpart;
  int* mpring;
  BaState* st;
};
static BaDev g_dummy;

int ba_alloc(vg_ctx* ctx) {
  BaBufs& b = ctx->ba;
  const int W = ctx->cfg.win_size;
  b.cap_f = ctx->cap.max_nodes / 8 > 262144 ? 262144 : (ctx->cap.max_nodes / 8 > 4096 ? ctx->cap.max_nodes / 8 : 4096);
  const int L = 6 * W, nout = L * (L + 1) / 2 + L + 1, n = 15 * W;
  bool good = true;
  good &= (b.fac_node = ctx->arena.take<int>(b.cap_f)) != nullptr;
  good &= (b.fac_eig = ctx->arena.take<double>((size_t)b.cap_f * 12)) != nullptr;
  good &= (b.fac_pcr = ctx->arena.take<Clu>(b.cap_f)) != nullptr;
  good &= (b.fac_comp = ctx->arena.take<double>((size_t)b.cap_f * (W * kComp + kCompF))) != nullptr;
  good &= (b.hpart = ctx->arena.take<double>((size_t)(b.cap_f / kFC + 1) * nout)) != nullptr;
  good &= (b.hout = ctx->arena.take<double>(nout + 16)) != nullptr;
  good &= (b.rpart = ctx->arena.take<double>(b.cap_f / 256 + 16)) != nullptr;
  good &= (b.xs = ctx->arena.take<double>(1024 + 2 * n * (n + 1) / 2 + 4 * n + 2 * kMaxW * kX + kMaxW * kImuRec +
                                          kMaxW * 12 + kMaxW * 931 + kMaxW + 64)) != nullptr;
  if (!good) {
    ctx->err = "arena exhausted (BA)";
    return VG_E_CAPACITY;
  }
  const int Wc = W > 12 ? 12 : W;
  VG_HIP(hipFuncSetAttribute((const void*)k_ba_solve, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (15 * Wc) * (15 * Wc + 1) / 2 * (int)sizeof(double)));
  VG_HIP(hipFuncSetAttribute((const void*)k_ba_hred, hipFuncAttributeMaxDynamicSharedMemorySize,
                             kFC * (W * kComp + kCompF) * (int)sizeof(double)));
  return VG_OK;
}

// carve the scratch block in BaBufs::xs; the first 1024 doubles are the WinD /
// counts staging area used by the map stages
static BaDev carve(vg_ctx* ctx) {
  BaBufs& b = ctx->ba;
  const int W = ctx->cfg.win_size;
  const int n = 15 * W, nn = n * (n + 1) / 2;
  double* p = b.xs + 1024;
  BaDev d;
  d.Hcalc = p;
  p += nn;
  d.Jcalc = p;
  p += n;
  d.dxi = p;
  p += n;
  d.xs = p;
  p += kMaxW * kX;
  d.xt = p;
  p += kMaxW * kX;
  d.imurec = p;
  p += kMaxW * kImuRec;
  d.bias = p;
  p += kMaxW * 12;
  d.imuout = p;
  p += kMaxW * 931;
  d.imures = p;
  p += kMaxW;
  d.st = (BaState*)p;
  p += 8;
  d.mpring = (int*)p;
  p += 16;
  d.comp = b.fac_comp;
  d.compf = b.fac_comp + (size_t)b.cap_f * W * kComp;
  d.part = b.hpart;
  d.hl = b.hout;
  d.rpart = b.rpart;
  return d;
}

// Run damping_iter on the device. xs_io: W x 24 doubles (R,p,v,bg,ba,g), in/out.
// imurec: (W-1) x kImuRec host records; bias_io: (W-1) x 12 (dbg, dba, bufs), in/out.
int ba_run(vg_ctx* ctx, int nf, const int* mp_ring, double* xs_io, const double* imurec, double* bias_io,
           int* iters) {
  const int W = ctx->cfg.win_size;
  if (W > 12) {
    ctx->err = "win_size > 12 unsupported by the BA kernels (LDS-resident 15W x 15W solve)";
    return VG_E_ARG;
  }
  hipStream_t s = ctx->stream;
  BaDev d = carve(ctx);
  const int nimu = W - 1;
  const int L = 6 * W, nl = L * (L + 1) / 2, nout = nl + L + 1;
  VG_HIP(hipMemcpyAsync(d.xs, xs_io, (size_t)W * kX * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.imurec, imurec, (size_t)nimu * kImuRec * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.bias, bias_io, (size_t)nimu * 12 * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.mpring, mp_ring, W * sizeof(int), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemsetAsync(d.hl, 0, nout * sizeof(double), s));
  k_ba_init<<<1, 1, 0, s>>>(d.st);
  const int nchunk = (nf + kFC - 1) / kFC;
  const int nrb = (nf + 255) / 256;
  const size_t hred_lds = (size_t)kFC * (W * kComp + kCompF) * sizeof(double);
  const size_t solve_lds = (size_t)(15 * W) * (15 * W + 1) / 2 * sizeof(double);
  for (int it = 0; it < 10; it++) {
    if (nf > 0) {
      k_ba_comp<<<grid_for((long)nf * W), kBlock, 0, s>>>(nf, W, ctx->ba.fac_node, ctx->ba.fac_eig, ctx->ba.fac_pcr,
                                                         ctx->map.pcrs, d.mpring, d.xs, d.comp, d.compf, d.st);
      k_ba_hred<<<nchunk, 256, hred_lds, s>>>(nf, W, d.comp, d.compf, d.part, d.st);
      k_ba_hfinal<<<(nout * 8 + 255) / 256, 256, 0, s>>>(nchunk, nout, d.part, d.hl, d.st);
    }
    if (nimu > 0) k_ba_imu<<<nimu, 256, 0, s>>>(nimu, d.imurec, d.bias, d.xs, d.imuout, d.st);
    k_ba_solve<<<1, 1024, solve_lds, s>>>(W, nimu, ctx->cfg.imu_coef, d.hl, d.imuout, d.Hcalc, d.Jcalc, d.xs, d.xt,
                                          d.bias, d.dxi, d.st);
    if (nf > 0)
      k_ba_resid<<<nrb, 256, 0, s>>>(nf, W, ctx->ba.fac_node, ctx->map.pcr_fix, ctx->map.pcrs, d.mpring, d.xt,
                                     ctx->ba.fac_eig, ctx->ba.fac_pcr, d.rpart, d.st);
    if (nimu > 0) k_ba_imures<<<1, 64, 0, s>>>(nimu, d.imurec, d.bias, d.xt, d.imures, d.st);
    k_ba_control<<<1, 256, 0, s>>>(W, nimu, nf > 0 ? nrb : 0, ctx->cfg.imu_coef, d.hl, nl + L, d.imuout, d.imures,
                                   d.rpart, d.xs, d.xt, d.bias, d.st);
  }
  VG_HIP(hipGetLastError());
  BaState hs;
  VG_HIP(hipMemcpyAsync(xs_io, d.xs, (size_t)W * kX * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(hipMemcpyAsync(bias_io, d.bias, (size_t)nimu * 12 * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(hipMemcpyAsync(&hs, d.st, sizeof(BaState), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  *iters = hs.iters;
  (void)g_dummy;
  return VG_OK;
}

}  // namespace vg
