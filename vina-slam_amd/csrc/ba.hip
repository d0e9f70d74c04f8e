// ba.hip — sliding-window LiDAR-inertial LM.
//
// Replaces LI_BA_Optimizer::damping_iter (optimizers.cpp:430-517) with its
// divide_thread / only_residual / hess_plus (171-245, 340-376), the point-
// cluster factor LidarFactor::acc_evaluate2 / evaluate_only_residual
// (factors.cpp:22-158) and IMU_PRE::give_evaluate / update_state
// (imu_preintegration.cpp:97-163, 239-246).
//
// Per LM iteration, all device-resident, no host round trip:
//   k_ba_hess    one 512-lane workgroup per chunk of min(512/W, 64) factors:
//                one lane per (factor, frame) evaluates Auk, the diagonal 6x6
//                block and the gradient piece (fp64 VALU); the off-diagonal
//                blocks, sums of rank-1 terms, are reduced as X^T S X on fp64
//                MFMA from LDS -> per-chunk partials (deterministic). The IMU
//                factors ride in the same launch (one workgroup each)
//   k_ba_hfinal  ordered sum of the chunk partials
//   k_ba_prep    assemble the 15W x 15W system (IMU blocks x imu_coef + LiDAR
//                6x6 blocks), gauge, Marquardt damping, pivoted tile image
//   k_ba_solve   one 1024-lane workgroup: blocked LDL^T of the pivoted
//                system in LDS (16x16 tiles, MFMA f64 trailing updates), the trial
//                state and q1
//   k_ba_resid   one lane per factor: merge clusters at the trial poses, 3x3
//                eigen, write the trial eig/cluster (the side effect margi
//                consumes), chunk residual partials
//   k_ba_imures  IMU residuals at the trial state
//   k_ba_control LM accept/reject, Nielsen damping update, bias restore,
//                convergence flag (1 lane)
// Kernels early-exit on the device-side `done` / `calc_hess` flags; the host
// enqueues two iterations at a time and reads `done` in between.
#include "vg_dev.h"

#include "vg_imu.h"  // imu_residual (host and device)

namespace vg {

constexpr int kMaxW = 16;
constexpr int kCompF = 24;    // per factor: umumT 9, ukukT 9, uk 3, NN, coe, lmbd0
constexpr int kImuRec = kBaImuRec;  // preintegration record + cov_inv

struct BaState {             // device-resident LM state
  double u, v, res1, res2, q1;
  int calc_hess, done, iters, seq;  // seq: the next LM publication number (k_ba_control)
  int nhess;                        // Hessian passes executed (I_H, SURVEY 8(d) byte model)
  int fin;                          // the run has finished (converged or 10 iterations): the margi tail's gate
  int skip, pad_[3];                // the recut needs the host (k_ba_init): the run is skipped, the gate stays shut
};
static_assert(sizeof(BaState) <= 16 * sizeof(double), "BaState is carved as 16 doubles");

typedef double v4d __attribute__((ext_vector_type(4)));

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

// IMU record k of DState's ring (pushed by k_push_state, slid by moving the head)
__device__ __forceinline__ const double* imu_rec(const double* imurec, int head, int k) {
  return &imurec[(size_t)((head + k) % kMaxWin) * kImuRec];
}
// give_evaluate with jac_enable at the current state; out per factor: jtj 900, gg 30, res 1
__device__ void imu_factor_block(int k, const double* __restrict__ imurec, int head, const double* __restrict__ bias,
                                 const double* __restrict__ xs, double* __restrict__ out) {
  __shared__ double joc[450], rr[15], P[450], C[225];
  const double* rec = imu_rec(imurec, head, k);
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
__device__ void imu_residual_lane(int k, const double* __restrict__ imurec, int head, const double* __restrict__ bias,
                                  const double* __restrict__ xt, double* __restrict__ res) {
  const double* rec = imu_rec(imurec, head, k);
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

// acc_evaluate2 per (factor, frame) — factors.cpp:57-97. Outputs the
// diagonal 6x6 block Hb (lower, 21), the gradient piece jjt (6) and the three
// 6-vectors whose outer products make every off-diagonal block:
//   Auk_i^T umumT Auk_j = sum_{m=1,2} c_m (Auk_i^T u_m)(Auk_j^T u_m)^T,
//       umumT = sum_m c_m u_m u_m^T, c_m = 2/(lambda_0 - lambda_m)
//   the correction terms (factors.cpp:80-86) = -(2/NN^2) h_i h_j^T,
//       h_i = [viRiTuk; n_i uk]
__device__ __forceinline__ void factor_frame(const double* e, const Clu& pa, const Clu& s, const double* x,
                                             double* hb, double* jjt_o, double* g1, double* g2, double* h) {
  double f[kCompF];
  factor_basics(e, pa, f);
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
  const M3 Ri = ld_m3(x);
  const double ni = (double)s.N;
  const M3 vihat = hat(vi);
  const V3 RiTuk = mul(tr(Ri), uk);
  const M3 RiTukhat = hat(RiTuk);
  const V3 PiRiTuk = mul(Pi, RiTuk);
  const V3 viRiTuk = mul(vihat, RiTuk);
  const V3 ti_v = sub(ld_v3(x + 9), vBar);
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
  // Hb = (A^T umumT) A + the corrections, only the lower triangle the output
  // keeps: every entry formed exactly as the full products form it (same
  // terms, same order), the upper 15 entries and their registers skipped
  // (the full 6x6 pushed k_ba_hess past 256 VGPRs: 50 spilled)
  M<6, 3> AtU = mul(tr(A), umumT);
  const double s2n = 2.0 / NN * (1.0 - ni / NN);  // HRt's scale
  const double c00s = 2.0 / NN, c00v = 2.0 / NN / NN;
  const double c11s = 2.0 / NN * (ni - ni * ni / NN);
  M3 L1;  // combo1 - RiTukhat Pi (c00's left factor, full: its rows meet RiTukhat's columns)
  {
    const M3 RP = mul(RiTukhat, Pi);
    for (int t = 0; t < 9; t++) L1[t] = combo1[t] - RP[t];
  }
  int q = 0;
  for (int r = 0; r < 6; r++)
    for (int c = 0; c <= r; c++) {
      double v = AtU(r, 0) * A(0, c);
      v += AtU(r, 1) * A(1, c);
      v += AtU(r, 2) * A(2, c);
      if (r < 3) {  // c00 = ((L1 RiTukhat) * 2/NN - (viRiTuk viRiTuk^T) * 2/NN/NN) - hat(jjt[0..3]) * 0.5
        double m = L1(r, 0) * RiTukhat(0, c);
        m += L1(r, 1) * RiTukhat(1, c);
        m += L1(r, 2) * RiTukhat(2, c);
        const V3 jt = v3(jjt[0], jjt[1], jjt[2]);
        const double hj = r == c ? 0.0 : (r == 1 ? (c == 0 ? jt[2] : 0.0) : (c == 0 ? -jt[1] : jt[0]));
        v += (m * c00s - (viRiTuk[r] * viRiTuk[c]) * c00v) - hj * 0.5;
      } else if (c < 3) {  // HRt(c, r - 3) (the lower off-diagonal block)
        v += (viRiTuk[c] * uk[r - 3]) * s2n;
      } else {
        v += ukukT(r - 3, c - 3) * c11s;
      }
      hb[q++] = v;
    }
  for (int k = 0; k < 6; k++) jjt_o[k] = jjt[k];
  const V3 u1 = v3(e[3 + 0 * 3 + 1], e[3 + 1 * 3 + 1], e[3 + 2 * 3 + 1]);
  const V3 u2 = v3(e[3 + 0 * 3 + 2], e[3 + 1 * 3 + 2], e[3 + 2 * 3 + 2]);
  for (int k = 0; k < 6; k++) {
    g1[k] = A(0, k) * u1[0] + A(1, k) * u1[1] + A(2, k) * u1[2];
    g2[k] = A(0, k) * u2[0] + A(1, k) * u2[1] + A(2, k) * u2[2];
  }
  for (int k = 0; k < 3; k++) {
    h[k] = viRiTuk[k];
    h[3 + k] = ni * uk[k];
  }
}

// outputs per chunk: 1830 lower entries of the 6W x 6W LiDAR Hessian
// (row-major lower), then 6W gradient, then the residual
__device__ __forceinline__ int lower_idx(int r, int c) { return r * (r + 1) / 2 + c; }

constexpr int kHessThreads = 512;  // 8 waves: a chunk's (factor, frame) lanes in one pass
constexpr int kHessGridMax = 256;  // k_ba_hess chunk workgroups (more chunks loop)
constexpr int kResidBlocks = 512;  // k_ba_resid workgroups (more chunks loop)
constexpr int kResidThreads = 256;  // k_ba_resid's workgroup (its chunking and residual order)
// factors per sub-chunk: two of k_ba_resid's chunks (256 / W factors) where
// that fits the lanes and the 64-row cap (W >= 8), so a Hessian chunk holds
// whole residual chunks (k_ba_resid_hess); else min(512 / W, 64)
__host__ __device__ constexpr int hess_fs(int W) {
  return 2 * (256 / W) <= 64 && 2 * (256 / W) <= kHessThreads / W ? 2 * (256 / W)
                                                                    : (kHessThreads / W < 64 ? kHessThreads / W : 64);
}
__host__ __device__ constexpr bool resid_hess_ok(int W) { return hess_fs(W) == 2 * (256 / W) && 256 / W <= 64; }
__host__ __device__ constexpr int hess_ks(int W) { return (3 * hess_fs(W) + 3) / 4 * 4; }  // GEMM K per sub-chunk
__host__ __device__ constexpr int hess_nt(int W) { return (6 * W + 15) / 16; }           // 16-wide output tiles
__host__ __device__ constexpr int hess_xs(int W) { return hess_nt(W) * 16 + 16; }        // X row stride (+16: rows k, k+1 in opposite LDS halves)
__host__ __device__ constexpr int hess_chunk(int W) { return hess_fs(W); }      // factors per workgroup (one sub-chunk)

// One workgroup per chunk of factors, no HBM intermediates: lane (f, i)
// evaluates factor f of the sub-chunk at frame i, keeps the coe-weighted
// diagonal block / gradient in registers and writes its three rank-1 rows to
// X (LDS); the off-diagonal blocks are then X^T S X on v_mfma_f64_16x16x4
// (one wave per lower 16x16 output tile, accumulators live across
// sub-chunks). Chunk partials go to `part` (summed by k_ba_hfinal).
// kSpec (k_ba_resid_hess): the pass at the LM's trial state, `xs` = the trial
// states. The chunk first does k_ba_resid's work for its factors —
// evaluate_only_residual: frame clusters moved to the trial poses, merged onto
// pcr_fix in frame order, 3x3 eigen, fac_eig / fac_pcr written — with
// k_ba_resid's operations, then evaluates the Hessian from those values (LDS)
// instead of fac_eig / fac_pcr. ev0[0] / ev0[1] take each lane's smallest
// eigenvalues for the two residual chunks the Hessian chunk holds.
template <bool kSpec = false>
__device__ __forceinline__ void hess_chunk_eval(int ch, int nf, int W, const int* __restrict__ fac_node,
                                                const double* __restrict__ fac_eig, const Clu* __restrict__ fac_pcr,
                                                const Clu* __restrict__ pcrs, const int* __restrict__ mpring,
                                                const double* __restrict__ xs, double* __restrict__ part,
                                                const Clu* __restrict__ pcr_fix = nullptr,
                                                double* __restrict__ eig_out = nullptr,
                                                Clu* __restrict__ pcr_out = nullptr, double* ev0 = nullptr,
                                                const double* __restrict__ eig_src = nullptr,
                                                const Clu* __restrict__ pcr_src = nullptr,
                                                NodeHdr* __restrict__ hdr = nullptr) {
  __syncthreads();  // the previous chunk's reduction has read the LDS
  extern __shared__ __attribute__((aligned(16))) double X[];
  __shared__ double S[kHessThreads];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int FS = hess_fs(W), KS = hess_ks(W), NT = hess_nt(W), XS = hess_xs(W);
  const int L = 6 * W, nl = L * (L + 1) / 2, nout = nl + L + 1;
  const int f = tid / W, i = tid % W;
  const bool active = f < FS;
  const int a_begin = ch * hess_chunk(W);
  const int a_end = min(nf, a_begin + hess_chunk(W));
  const int ntl = NT * (NT + 1) / 2;
  __shared__ double s_e[kSpec ? 64 : 1][12];  // kSpec: the chunk's eigen systems and merged clusters at the trial
  __shared__ Clu s_pa[kSpec ? 64 : 1];
  if constexpr (kSpec) {
    Clu* s_t = reinterpret_cast<Clu*>(X);  // the moved frame clusters (X is filled below)
    {
      const int a = a_begin + f;
      if (active && a < a_end) {
        const Clu src = pcrs[(size_t)fac_node[a] * W + mpring[i]];
        Clu t;
        if (src.N != 0) {
          t = clu_transform(src, ld_m3(&xs[(size_t)i * kX]), ld_v3(&xs[(size_t)i * kX + 9]));
        } else {
          clu_zero(t);
          t.N = 0;
        }
        s_t[tid] = t;
      }
    }
    __syncthreads();
    const int a2 = a_begin + tid;
    if (tid < FS && a2 < a_end) {
      Clu sig = pcr_fix[fac_node[a2]];
      for (int k = 0; k < W; k++) {
        const Clu& t = s_t[tid * W + k];
        if (t.N != 0) clu_add(sig, t);
      }
      V3 ev;
      M3 U;
      eig3(clu_cov(sig), ev, U);
      double* e = &eig_out[(size_t)a2 * 12];
      for (int j = 0; j < 3; j++) e[j] = s_e[tid][j] = ev[j];
      for (int j = 0; j < 9; j++) e[3 + j] = s_e[tid][3 + j] = U[j];
      pcr_out[a2] = sig;
      s_pa[tid] = sig;
      ev0[tid < FS / 2 ? 0 : 1] += 1.0 * ev[0];  // k_ba_resid's acc (lane tid mod FS/2 of its chunk)
    }
    __syncthreads();  // s_t is read: X may be cleared
  }
  // A chunk is one sub-chunk (hess_chunk == hess_fs): the lane's factor_frame
  // writes its diagonal block and gradient straight into hb / jj (0 + coe x,
  // the accumulation's value), so no second copy is live beside the call
  // (it was: 256 VGPRs and ~50 spilled, scratch traffic ~5x the kernel's bytes)
  for (int t = tid; t < KS * XS; t += kHessThreads) X[t] = 0.0;
  for (int t = tid; t < KS; t += kHessThreads) S[t] = 0.0;
  __syncthreads();
  double hb[21], jj[6], res = 0.0;
  {
    const int a = a_begin + f;
    bool got = false;
    if (active && a < a_end) {
      const int node = fac_node[a];
      // eig_src (k_ba_init_hess): tras_opt's bookkeeping in this pass, the
      // factor's eigen system and cluster read from the map and copied out
      const double* e = kSpec ? s_e[f] : (eig_src ? &eig_src[(size_t)node * 12] : &fac_eig[(size_t)a * 12]);
      const Clu pa = kSpec ? s_pa[f] : (eig_src ? pcr_src[node] : fac_pcr[a]);
      if (!kSpec && eig_src && i == 0) {
        for (int j = 0; j < 12; j++) eig_out[(size_t)a * 12 + j] = e[j];
        pcr_out[a] = pa;
        hdr[node].opt_state = a;
      }
      const double coe = 1.0;  // octree.cpp:507
      if (i == 0) {
        res = 0.0 + coe * e[0];
        const double NN = (double)pa.N;
        S[3 * f + 0] = coe * (2.0 / (e[0] - e[1]));
        S[3 * f + 1] = coe * (2.0 / (e[0] - e[2]));
        S[3 * f + 2] = -coe * (2.0 / NN / NN);
      }
      const Clu sc = pcrs[(size_t)node * W + mpring[i]];
      if (sc.N != 0) {
        double g1[6], g2[6], h[6];
        factor_frame(e, pa, sc, &xs[(size_t)i * kX], hb, jj, g1, g2, h);
        for (int k = 0; k < 21; k++) hb[k] = 0.0 + coe * hb[k];
        for (int k = 0; k < 6; k++) jj[k] = 0.0 + coe * jj[k];
        double* x0 = &X[(size_t)(3 * f) * XS + 6 * i];
        for (int k = 0; k < 6; k++) {
          x0[k] = g1[k];
          x0[XS + k] = g2[k];
          x0[2 * XS + k] = h[k];
        }
        got = true;
      }
    }
    if (!got) {
      for (int k = 0; k < 21; k++) hb[k] = 0.0;
      for (int k = 0; k < 6; k++) jj[k] = 0.0;
    }
  }
  __syncthreads();
  v4d acc[4];  // <= 15 lower tiles (W <= 11) over the 8 waves (<= 2 per wave; 4 slots)
  for (int q = wave, slot = 0; q < ntl; q += kHessThreads / 64, slot++) {
    int TI = 0;
    while ((TI + 1) * (TI + 2) / 2 <= q) TI++;
    const int TJ = q - TI * (TI + 1) / 2;
    const int cc = lane & 15, rq = lane >> 4;
    v4d c = v4d{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < KS; k0 += 4) {
      const int k = k0 + rq;
      const double av = S[k] * X[(size_t)k * XS + 16 * TI + cc];
      const double bv = X[(size_t)k * XS + 16 * TJ + cc];
      c = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c, 0, 0, 0);
    }
    acc[slot] = c;
  }
  __syncthreads();
  double* out = &part[(size_t)ch * nout];
  // off-diagonal blocks from the MFMA tiles (diagonal 6x6 blocks come from Hb)
  for (int q = wave, slot = 0; q < ntl; q += kHessThreads / 64, slot++) {
    int TI = 0;
    while ((TI + 1) * (TI + 2) / 2 <= q) TI++;
    const int TJ = q - TI * (TI + 1) / 2;
    const int cc = lane & 15, rq = lane >> 4;
    for (int g = 0; g < 4; g++) {
      const int row = 16 * TI + rq + 4 * g, colx = 16 * TJ + cc;
      if (row < L && colx <= row && row / 6 != colx / 6) out[lower_idx(row, colx)] = acc[slot][g];
    }
  }
  // per-frame diagonal blocks, gradient and residual: ordered sum over f
  double* R = X;
  if (active) {
    for (int k = 0; k < 21; k++) R[tid * 28 + k] = hb[k];
    for (int k = 0; k < 6; k++) R[tid * 28 + 21 + k] = jj[k];
    R[tid * 28 + 27] = res;
  }
  __syncthreads();
  for (int e = tid; e < W * 27 + 1; e += kHessThreads) {
    if (e == W * 27) {
      double sres = 0.0;
      for (int ff = 0; ff < FS; ff++) sres += R[(ff * W) * 28 + 27];
      out[nl + L] = sres;
      continue;
    }
    const int fi = e / 27, k = e % 27;
    double sv = 0.0;
    for (int ff = 0; ff < FS; ff++) sv += R[(ff * W + fi) * 28 + k];
    if (k < 21) {
      int r = 0;
      while ((r + 1) * (r + 2) / 2 <= k) r++;
      const int c = k - r * (r + 1) / 2;
      out[lower_idx(6 * fi + r, 6 * fi + c)] = sv;
    } else {
      out[nl + 6 * fi + (k - 21)] = sv;
    }
  }
}

// The factor count is read on the device (*nfp): workgroups [0, G) loop over
// the chunks (chunk c -> partial c, whatever G), G + k evaluates IMU factor k.
__device__ __forceinline__ void hess_body(const int* __restrict__ nfp, int W, const int* __restrict__ fac_node,
                                          const double* __restrict__ fac_eig, const Clu* __restrict__ fac_pcr,
                                          const Clu* __restrict__ pcrs, const int* __restrict__ mpring,
                                          const double* __restrict__ xs, double* __restrict__ part,
                                          const BaState* __restrict__ st, int G, int nimu,
                                          const double* __restrict__ imurec, const int* __restrict__ imu_head,
                                          const double* __restrict__ bias, double* __restrict__ imuout);
__global__ void __launch_bounds__(kHessThreads) k_ba_hess(const int* __restrict__ nfp, int W,
                                                          const int* __restrict__ fac_node,
                                                          const double* __restrict__ fac_eig,
                                                          const Clu* __restrict__ fac_pcr, const Clu* __restrict__ pcrs,
                                                          const int* __restrict__ mpring, const double* __restrict__ xs,
                                                          double* __restrict__ part, const BaState* __restrict__ st,
                                                          int G, int nimu, const double* __restrict__ imurec,
                                                          const int* __restrict__ imu_head,
                                                          const double* __restrict__ bias, double* __restrict__ imuout,
                                                          KClock* __restrict__ clk) {
  if (st->done || !st->calc_hess) return;
  // in-kernel clock (vg_profile bit 2): slot (scan, LM iteration), start by
  // workgroup 0, every workgroup's end (KClock h_*)
  const bool clk_on = clk && clk->on;
  const int clk_slot = clk_on ? (clk->scan * 8 + (st->iters < 7 ? st->iters : 7)) & (kClkHRing - 1) : 0;
  if (clk_on && blockIdx.x == 0 && threadIdx.x == 0) {
    clk->h_t0[clk_slot] = (unsigned long long)wall_clock64();
    clk->h_exec[clk_slot] = 1;
  }
  hess_body(nfp, W, fac_node, fac_eig, fac_pcr, pcrs, mpring, xs, part, st, G, nimu, imurec, imu_head, bias, imuout);
  if (clk_on && blockIdx.x < kClkHBlocks) {
    __syncthreads();
    if (threadIdx.x == 0) clk->h_tend[clk_slot][blockIdx.x] = (unsigned long long)wall_clock64();
  }
}
__device__ __forceinline__ void hess_body(const int* __restrict__ nfp, int W, const int* __restrict__ fac_node,
                                          const double* __restrict__ fac_eig, const Clu* __restrict__ fac_pcr,
                                          const Clu* __restrict__ pcrs, const int* __restrict__ mpring,
                                          const double* __restrict__ xs, double* __restrict__ part,
                                          const BaState* __restrict__ st, int G, int nimu,
                                          const double* __restrict__ imurec, const int* __restrict__ imu_head,
                                          const double* __restrict__ bias, double* __restrict__ imuout) {
  if ((int)blockIdx.x >= G) {  // IMU factors ride in the same launch (give_evaluate, jac_enable)
    const int k = blockIdx.x - G;
    if (k < nimu) imu_factor_block(k, imurec, *imu_head, bias, xs, imuout);
    return;
  }
  const int nf = *nfp;
  const int nchunk = (nf + hess_chunk(W) - 1) / hess_chunk(W);
  for (int ch = blockIdx.x; ch < nchunk; ch += G) hess_chunk_eval(ch, nf, W, fac_node, fac_eig, fac_pcr, pcrs, mpring, xs, part);
}

// ordered sum of the chunk partials: 8 lanes per output split the chunks
// (stride 8), then a fixed 3-step shuffle tree (deterministic)
// xa.frame (sharded): `out` is the exchange frame, closed here (nout = its payload)
__global__ void __launch_bounds__(256) k_ba_hfinal(const int* __restrict__ nfp, int chunk, int nout,
                                                   const double* __restrict__ part, double* __restrict__ out,
                                                   const BaState* __restrict__ st, XchgArg xa) {
  if (xa.frame && blockIdx.x == 0 && threadIdx.x == 0) xchg_close(xa.frame, xa.n, 3, xa.seq);
  if (st->done || !st->calc_hess) return;
  const int nchunk = (*nfp + chunk - 1) / chunk;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = gt >> 3, sub = gt & 7;
  double s = 0.0;
  if (e < nout) {  // chunks sub, sub + 8, ... in order; up to 32 loads issued per batch (one batch up to
                   // 256 chunks: one memory round trip), then added
    constexpr int kB = 32;
    for (int b = sub; b < nchunk; b += 8 * kB) {
      double v[kB];
#pragma unroll
      for (int k = 0; k < kB; k++) v[k] = b + 8 * k < nchunk ? part[(size_t)(b + 8 * k) * nout + e] : 0.0;
#pragma unroll
      for (int k = 0; k < kB; k++)
        if (b + 8 * k < nchunk) s += v[k];
    }
  }
  s += __shfl_down(s, 4, 8);
  s += __shfl_down(s, 2, 8);
  s += __shfl_down(s, 1, 8);
  if (e < nout && sub == 0) out[e] = s;
}

// packed lower storage of the n x n system (Hcalc)
__device__ __forceinline__ int lo(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// ---- LDS tile store of the permuted system: lower block triangle of 16x16
// fp64 tiles, tile (I,J) (I >= J) at I(I+1)/2 + J, element (r,c) at
// r*16 + (c ^ r): rows and columns of a tile both read conflict-free, which
// the MFMA operand loads (16 rows of one column per lane group) need.
constexpr int kTile = 16;
constexpr int kMaxNB = 11;  // 15W <= 176
__device__ __forceinline__ int tix(int I, int J) { return I * (I + 1) / 2 + J; }
__device__ __forceinline__ int tel(int r, int c) { return r * 16 + (c ^ r); }

__device__ __forceinline__ double bcast(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo32 = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi32 = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi32 << 32) | (unsigned int)lo32);
}


// broadcast lane qd of every quad (DPP quad_perm) — qd must fold to a constant
template <int Q>
__device__ __forceinline__ double quad_bcast_c(double v) {
  const long long b = __double_as_longlong(v);
  const int lo32 = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), Q * 0x55, 0xf, 0xf, false);
  const int hi32 = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), Q * 0x55, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi32 << 32) | (unsigned int)lo32);
}
__device__ __forceinline__ double quad_bcast(double v, int qd) {
  switch (qd) {
    case 0: return quad_bcast_c<0>(v);
    case 1: return quad_bcast_c<1>(v);
    case 2: return quad_bcast_c<2>(v);
    default: return quad_bcast_c<3>(v);
  }
}

// one assembled lower entry (R >= C) of the 15W x 15W system in the host
// loop's accumulation order (divide_thread 215-222: IMU factors k ascending,
// x imu_coef, then hess_plus 171-179 adds the LiDAR 6x6 blocks)
__device__ __forceinline__ double asm_entry(int R, int C, int nimu, double imu_coef, const double* hl,
                                            const double* imuout, int L) {
  const int bR = R / 15, bC = C / 15, rR = R % 15, rC = C % 15;
  double v = 0.0;
  for (int k = bR > 0 ? bR - 1 : 0; k <= bC && k < nimu; k++)
    v += imuout[(size_t)k * 931 + (R - 15 * k) * 30 + (C - 15 * k)];
  v *= imu_coef;
  if (rR < 6 && rC < 6) {
    const int lr = bR * 6 + rR, lc = bC * 6 + rC;
    v += hl[lr * (lr + 1) / 2 + lc];
  }
  return v;
}
__device__ __forceinline__ double asm_grad(int t, int nimu, double imu_coef, const double* hl, const double* imuout,
                                           int L) {
  const int b = t / 15, r = t % 15;
  double v = 0.0;
  if (b >= 1 && b - 1 < nimu) v += imuout[(size_t)(b - 1) * 931 + 900 + r + 15];
  if (b < nimu) v += imuout[(size_t)b * 931 + 900 + r];
  v *= imu_coef;
  if (r < 6) v += hl[L * (L + 1) / 2 + b * 6 + r];
  return v;
}

// Wide preparation of the permuted, gauged, damped system: one block per
// 16x16 tile of the lower block triangle. Every block ranks the damped
// diagonal (Eigen's LDLT is left-looking, so its pivot order is the
// descending order of |diag|, see the oracle's ldlt_solve) and writes its
// tile of P A P^T to the tile image; on Hessian iterations it also stores
// the assembled entries it visits (each lower entry exactly once) for the
// damping-only retries. Block 0 writes the permuted right-hand side.
// The gauge frame's 15 variables (optimizers.cpp:460-463: unit rows and
// columns, zero gradient) are decoupled from the rest, so wherever Eigen's
// pivot order puts them their elimination changes nothing and their solution
// is 0: they are left out of the factored system (n - 15 unknowns).
__global__ void __launch_bounds__(256) k_ba_prep(int W, int nimu, double imu_coef, const double* __restrict__ hl,
                                                 const double* __restrict__ imuout, double* __restrict__ Hcalc,
                                                 double* __restrict__ Jcalc, double* __restrict__ timg,
                                                 double* __restrict__ bvec, double* __restrict__ dvec,
                                                 double* __restrict__ jvec, int* __restrict__ ipg,
                                                 BaState* __restrict__ st, int structural, int xworld,
                                                 int* __restrict__ xerr) {
  if (st->done) return;
  // sharded: `hl` is the all-reduced exchange frame; a guard mismatch ends the
  // LM (error bit 32: the scan fails with VG_E_STATE)
  if (xworld > 0 && !xchg_ok(hl, 3 * W * (6 * W + 1) + 6 * W + 1 + 2, xworld)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      atomicOr(xerr, 32);
      st->done = 1;
    }
    return;
  }
  constexpr int kN = kMaxNB * kTile;
  __shared__ double Dv[kN], Jg[kN];
  __shared__ int ip[kN];
  const int n = 15 * W, L = 6 * W, m = n - 15, NB = (m + kTile - 1) / kTile, N = NB * kTile;
  const int tid = threadIdx.x, q = blockIdx.x;
  const bool calc = st->calc_hess != 0;
  const double u = st->u;
  for (int t = tid; t < n; t += blockDim.x)
    Dv[t] = t < 15 ? 1.0 : (calc ? asm_entry(t, t, nimu, imu_coef, hl, imuout, L) : Hcalc[lo(t, t)]);
  __syncthreads();
  for (int i = 15 + tid; i < n; i += blockDim.x) {
    if (structural) {  // v / bg / ba of frames 1..W-1 first (frame order), then their poses
      const int j = i / 15, v = i - 15 * j;
      ip[v >= 6 ? 9 * (j - 1) + (v - 6) : 9 * (W - 1) + 6 * (j - 1) + v] = i;
      continue;
    }
    // Eigen's order: rank of |D + u D| descending, index ascending on ties
    const unsigned long long ki = (unsigned long long)__double_as_longlong(fabs(Dv[i] + u * Dv[i]));
    int c = 0;
    for (int j = 15; j < n; j++) {
      const unsigned long long kj = (unsigned long long)__double_as_longlong(fabs(Dv[j] + u * Dv[j]));
      c += (kj > ki) || (kj == ki && j < i);
    }
    ip[c] = i;
  }
  __syncthreads();
  int TI = 0;
  while ((TI + 1) * (TI + 2) / 2 <= q) TI++;
  const int TJ = q - TI * (TI + 1) / 2;
  for (int e = tid; e < 256; e += blockDim.x) {
    const int r = e >> 4, c = e & 15, R = TI * 16 + r, C = TJ * 16 + c;
    double v;
    if (R >= m || C >= m) {
      v = (R == C) ? 1.0 : 0.0;
    } else {
      const int pr = ip[R], pc = ip[C], a = pr > pc ? pr : pc, bb = pr > pc ? pc : pr;
      const double raw = calc ? asm_entry(a, bb, nimu, imu_coef, hl, imuout, L) : Hcalc[lo(a, bb)];
      if (calc && R >= C) Hcalc[lo(a, bb)] = raw;
      v = (pr == pc) ? Dv[pr] + u * Dv[pr] : raw;
    }
    timg[(size_t)q * 256 + tel(r, c)] = v;
  }
  if (q == 0) {
    // residual1 of divide_thread at the current state (optimizers.cpp:454), on
    // a lane the gradient loop below leaves idle (n < 256)
    if (calc && tid == (int)blockDim.x - 1) {
      double r = 0.0;
      for (int k = 0; k < nimu; k++) r += imuout[(size_t)k * 931 + 930];
      r *= imu_coef * 0.5;
      r += hl[L * (L + 1) / 2 + L];
      st->res1 = r;
    }
    for (int t = tid; t < n; t += blockDim.x) {
      const double raw = calc ? asm_grad(t, nimu, imu_coef, hl, imuout, L) : Jcalc[t];
      if (calc) Jcalc[t] = raw;
      Jg[t] = t < 15 ? 0.0 : raw;
      dvec[t] = Dv[t];
      if (t < m) ipg[t] = ip[t];
    }
    __syncthreads();
    for (int t = tid; t < N; t += blockDim.x) bvec[t] = t < m ? -Jg[ip[t]] : 0.0;
    for (int t = tid; t < n; t += blockDim.x) jvec[t] = Jg[t];
  }
}

// 4x4 symmetric sweep in registers, pivots in index order: b -> -b^-1. A
// pivot with |d| <= DBL_MIN contributes nothing (Eigen's LDLT leaves such a
// column undivided and its solve takes D^+, so that unknown's share is 0).
__device__ __forceinline__ void sweep4(double (&b)[4][4]) {
#pragma unroll
  for (int p = 0; p < 4; p++) {
    const double d = b[p][p];
    double ip = __builtin_amdgcn_rcp(d);
    ip = fma(ip, fma(-d, ip, 1.0), ip);
    ip = fabs(d) > 2.2250738585072014e-308 ? ip : 0.0;
    double c[4];
#pragma unroll
    for (int i = 0; i < 4; i++) c[i] = b[i][p] * ip;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j <= i; j++)
        if (i != p && j != p) {
          b[i][j] = fma(-c[i], b[p][j], b[i][j]);
          b[j][i] = b[i][j];
        }
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i != p) b[i][p] = b[p][i] = c[i];
    b[p][p] = -ip;
  }
}
// v_i for a lane-varying i in [0, 4): flat selects (no divergent branches)
__device__ __forceinline__ double sel4(double v0, double v1, double v2, double v3, int i) {
  double r = v3;
  r = i == 2 ? v2 : r;
  r = i == 1 ? v1 : r;
  r = i == 0 ? v0 : r;
  return r;
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int C>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo32 = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), C, 0xf, 0xf, false);
  const int hi32 = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), C, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi32 << 32) | (unsigned int)lo32);
}
// sum over the 16 lanes of each row (lanes with equal lane >> 4): DPP
// quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror; every lane
// adds the same pairs, so all 16 hold the same bits
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  return v;
}
// sum over lanes l, l^16, l^32, l^48 (the four rows): gfx950's
// v_permlane16_swap / v_permlane32_swap, (even + odd) then (low + high)
__device__ __forceinline__ double xrow_sum(double v) {
  long long b = __double_as_longlong(v);
  auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  v = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
  b = __double_as_longlong(v);
  lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

// Block LDL^T solve of the prepared system P A P^T y = P b in one workgroup
// (the LDLT the reference runs at optimizers.cpp:466, pivot order from
// k_ba_prep: Eigen's, descending |diag|). 16 x 16 tiles, no further pivoting:
//   P A P^T = L D L^T with D = diag(S_KK) (the Schur-complement diagonal
//   tiles) and L_IK = S_IK S_KK^-1, so
//   forward  y_I -= L_IK y_K (rides along the trailing update),
//   diagonal w_K  = S_KK^-1 y_K,
//   backward x_K  = w_K - S_KK^-1 sum_{J>K} S_JK^T x_J.
// A diagonal tile is inverted in registers by one wave as a 4-column block
// sweep (Gauss-Jordan on the symmetric tile): each step inverts its 4 x 4
// pivot block (sweep4, redundantly per lane), exchanges one 16 x 4 panel
// through LDS and applies the rank-4 update with one v_mfma_f64_16x16x4; the
// pivot rows/columns are written directly (not as the difference of two
// rounded products). Tiles live in the D layout of that MFMA (lane (c, q)
// holds rows q + 4g of column c), which is also the layout a tile has after a
// trailing update, so the factor never leaves registers between the update
// and the inversion.
// Phase K (one workgroup barrier each): wave 0 computes -L_{K+1,K}^T, brings
// tile (K+1, K+1) and y_{K+1} up to date and inverts the tile (the critical
// chain); the twelve waves on the other three SIMDs take the rest of panel K's
// trailing update, row pieces of up to four tiles that each compute their
// row's -L_IK^T = S_KK^-1 S_IK^T once in registers (that transposed product
// is exactly the MFMA A-operand layout of the update), plus w_K. The backward
// substitution keeps acc_J in wave J's registers: one barrier per tile row.
// Rounding differs from Eigen's sequential recurrences (tolerance level).
__global__ void __launch_bounds__(1024) k_ba_solve(int W, int nimu, const double* __restrict__ timg,
                                                  const double* __restrict__ bvec, const double* __restrict__ dvec,
                                                  const double* __restrict__ jvec, const int* __restrict__ ipg,
                                                  const double* __restrict__ xs, double* __restrict__ xt,
                                                  double* __restrict__ bias, double* __restrict__ dxi_out,
                                                  BaState* __restrict__ st, KClock* __restrict__ clk) {
  if (st->done) return;
  const unsigned long long clk0 = wall_clock64();  // vg_profile bit 2 (KClock)
  extern __shared__ __attribute__((aligned(16))) double T[];
  constexpr int kN = kMaxNB * kTile;
  __shared__ double Jv[kN], Dv[kN], yv[kN], wv[kN], xv[kN], col[kN], sP[64], sG[64];
  __shared__ int ip[kN];
  const int n = 15 * W, m = n - 15;  // the gauge frame's unknowns are not factored (k_ba_prep)
  const int NB = (m + kTile - 1) / kTile, N = NB * kTile;
  const int ntile = NB * (NB + 1) / 2;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int cc = lane & 15, rq = lane >> 4;
  const double u = st->u;
#ifdef VG_PROBE
  __shared__ unsigned s_tmax;
  if (tid == 0) s_tmax = 0;
#endif
  VG_PROBE_BEGIN();

  // -S^-1 of a diagonal tile held in registers (D layout), on one wave
  auto diag = [&](v4d a) __attribute__((always_inline)) {
    const int cq = cc & 3, cb = cc >> 2;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      sP[rq * 16 + cc] = a[k];  // rows 4k..4k+3 of the tile
      wave_lds_sync();
      double b[4][4], p[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j < 4; j++) b[i][j] = sP[i * 16 + 4 * k + j];
        p[i] = sP[i * 16 + cc];  // A(4k+i, c) = A(c, 4k+i)
      }
      sweep4(b);  // -B^-1
      double bc[4];
#pragma unroll
      for (int j = 0; j < 4; j++) bc[j] = sel4(b[j][0], b[j][1], b[j][2], b[j][3], rq);  // -B^-1(j, q)
      double gq = 0.0;  // -G(c, q), G = A(:, K) B^-1
#pragma unroll
      for (int j = 0; j < 4; j++) gq = fma(p[j], bc[j], gq);
      const bool inK = cb == k;
      sG[cc * 4 + rq] = -gq;
      a = __builtin_amdgcn_mfma_f64_16x16x4f64(inK ? 0.0 : gq, inK ? 0.0 : a[k], a, 0, 0, 0);  // A_OO -= G A_KO
      wave_lds_sync();
      double go[4];
#pragma unroll
      for (int g = 0; g < 4; g++) go[g] = sG[(rq + 4 * g) * 4 + cq];
#pragma unroll
      for (int g = 0; g < 4; g++)
        if (g != k) a[g] = inK ? go[g] : a[g];  // A_OK <- G
      a[k] = inK ? sel4(bc[0], bc[1], bc[2], bc[3], cq) : -gq;  // A_KK <- -B^-1, A_KO <- B^-1 A_KO = G^T
    }
    return a;
  };
  // -L_IK^T = S_KK^-1 S_IK^T as (-S_KK^-1) S_IK^T: lane (c, q) reg g =
  // -L_IK(c, q + 4g). tv[ks] = (-S_KK^-1)(c, 4ks + q) (from the tile store, or
  // wave 0's registers: the inverse is symmetric, so its D-layout register g
  // is that A operand), sv[ks] = S_IK(c, 4ks + q). Two accumulation chains.
  auto mk_gt = [&](const v4d& tv, const v4d& sv) __attribute__((always_inline)) {
    const v4d z = v4d{0.0, 0.0, 0.0, 0.0};
    v4d g1 = __builtin_amdgcn_mfma_f64_16x16x4f64(tv[0], sv[0], z, 0, 0, 0);
    v4d g2 = __builtin_amdgcn_mfma_f64_16x16x4f64(tv[2], sv[2], z, 0, 0, 0);
    g1 = __builtin_amdgcn_mfma_f64_16x16x4f64(tv[1], sv[1], g1, 0, 0, 0);
    g2 = __builtin_amdgcn_mfma_f64_16x16x4f64(tv[3], sv[3], g2, 0, 0, 0);
    return g1 + g2;
  };
  // operand columns of a tile: lane (c, q) reg ks = tile(c, 4ks + q)
  auto ld_ops = [&](const double* t) __attribute__((always_inline)) {
    v4d o;
#pragma unroll
    for (int ks = 0; ks < 4; ks++) o[ks] = t[tel(cc, 4 * ks + rq)];
    return o;
  };
  // acc -= L_IK S_JK^T, sj = ld_ops(S_JK); two accumulation chains
  auto tile_upd = [&](v4d acc, const v4d& gt, const v4d& sj) __attribute__((always_inline)) {
    v4d a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(gt[2], sj[2], v4d{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(gt[0], sj[0], acc, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(gt[3], sj[3], a2, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(gt[1], sj[1], acc, 0, 0, 0);
    return acc + a2;
  };
  // y_I -= L_IK y_K
  auto y_upd = [&](const v4d& gt, int K, int I) __attribute__((always_inline)) {
    double s = 0.0;
#pragma unroll
    for (int g = 0; g < 4; g++) s = fma(gt[g], yv[16 * K + rq + 4 * g], s);
    s = xrow_sum(s);
    if (rq == 0) yv[16 * I + cc] += s;
  };
  // w_K = S_KK^-1 y_K (into wv, and into xv as well for the last tile row)
  auto w_job = [&](int K, bool last) __attribute__((always_inline)) {
    const double* Ti = &T[tix(K, K) * 256];
    const double yk = yv[16 * K + cc];
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const double s = -row16_sum(Ti[tel(rq + 4 * g, cc)] * yk);
      if (cc == 0) {
        wv[16 * K + rq + 4 * g] = s;
        if (last) xv[16 * K + rq + 4 * g] = s;
      }
    }
  };
  auto ld_tile = [&](const double* t) __attribute__((always_inline)) {
    v4d a;
#pragma unroll
    for (int g = 0; g < 4; g++) a[g] = t[tel(rq + 4 * g, cc)];
    return a;
  };
  auto st_tile = [&](double* t, const v4d& a) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 4; g++) t[tel(rq + 4 * g, cc)] = a[g];
  };
  // an all-zero tile (wave-uniform): its updates are exact no-ops and are
  // skipped. In the structural order (k_ba_prep) the v/bg/ba tiles far from the
  // diagonal are zero and stay zero (the IMU factors couple adjacent frames only)
  auto zero_tile = [&](const v4d& o) __attribute__((always_inline)) {
    const bool nz = o[0] != 0.0 || o[1] != 0.0 || o[2] != 0.0 || o[3] != 0.0;
    return __ballot(nz) == 0;
  };

  // wave 0 takes tile (0, 0) straight from the image and inverts it while the
  // other waves fill the tile store and the vectors
  v4d tinv;  // wave 0: -S_KK^-1 of the current panel, kept in registers
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);  // the critical chain issues first on its SIMD
    tinv = diag(ld_tile(timg));
    st_tile(T, tinv);
  } else {
    const double2* src = reinterpret_cast<const double2*>(timg);
    double2* dst = reinterpret_cast<double2*>(T);
    for (int t = 128 + tid - 64; t < ntile * 128; t += nt - 64) dst[t] = src[t];
    for (int t = tid - 64; t < N; t += nt - 64) yv[t] = bvec[t];
    for (int t = tid - 64; t < n; t += nt - 64) {
      Dv[t] = dvec[t];
      Jv[t] = jvec[t];
      if (t < m) ip[t] = ipg[t];
    }
  }
  __syncthreads();
  VG_PROBE_MARK(3);

  // -L_IK^T of a phase goes to tile (I, K) in the next phase, once no wave
  // reads S_IK any more (the backward substitution needs L, not S): at most
  // two rows per wave and phase (wave-uniform bookkeeping)
  v4d pg0, pg1;
  int pt0 = -1, pt1 = -1;
  auto flush = [&]() __attribute__((always_inline)) {
    if (pt0 >= 0) st_tile(&T[pt0 * 256], pg0);
    if (pt1 >= 0) st_tile(&T[pt1 * 256], pg1);
    pt0 = pt1 = -1;
  };
  auto pend = [&](const v4d& gt, int t) __attribute__((always_inline)) {
    if (pt0 < 0) {
      pg0 = gt;
      pt0 = t;
    } else {
      pg1 = gt;
      pt1 = t;
    }
  };
  for (int K = 0; K + 1 < NB; K++) {
    flush();
    if (wave == 0) {
      const v4d s1 = ld_ops(&T[tix(K + 1, K) * 256]);
      v4d a = ld_tile(&T[tix(K + 1, K + 1) * 256]);
      const v4d gt = mk_gt(tinv, s1);
      a = tile_upd(a, gt, s1);
      pend(gt, tix(K + 1, K));
      VG_PROBE_MARK(10);
      tinv = diag(a);
      st_tile(&T[tix(K + 1, K + 1) * 256], tinv);
      VG_PROBE_MARK(11);
    } else if (wave & 3) {
      // the twelve waves off wave 0's SIMD: job 0 = w_K and y_{K+1}, then row
      // pieces of up to four tiles (the three other waves on wave 0's SIMD
      // stay idle: as helpers they slowed the critical chain more than they
      // shortened the trailing update, phase clocks 34.1 -> 35.5 us)
#ifdef VG_PROBE
      const unsigned long long tj0 = wall_clock64();
#endif
      const int wk = wave - (wave >> 2) - 1;
      constexpr int nwk = 12;
      const v4d tv = ld_ops(&T[tix(K, K) * 256]);
      int q = 0;
      if (q++ == wk) {
        w_job(K, false);
        y_upd(mk_gt(tv, ld_ops(&T[tix(K + 1, K) * 256])), K, K + 1);
      }
      for (int I = K + 2; I < NB; I++)
        for (int J0 = K + 1; J0 <= I; J0 += 4) {
          if (q++ % nwk != wk) continue;
          const v4d sik = ld_ops(&T[tix(I, K) * 256]);
          if (zero_tile(sik)) continue;  // L_IK = 0: no update, no y update, the tile stays 0 (= -L_IK^T)
          const v4d gt = mk_gt(tv, sik);
          const int J1 = J0 + 4 < I + 1 ? J0 + 4 : I + 1;
          for (int J = J0; J < J1; J++) {
            const v4d sjk = ld_ops(&T[tix(J, K) * 256]);
            if (zero_tile(sjk)) continue;
            double* Tij = &T[tix(I, J) * 256];
            st_tile(Tij, tile_upd(ld_tile(Tij), gt, sjk));
          }
          if (J0 == K + 1) {
            y_upd(gt, K, I);
            pend(gt, tix(I, K));
          }
        }
#ifdef VG_PROBE
      if (lane == 0) atomicMax(&s_tmax, (unsigned)(wall_clock64() - tj0));
#endif
    }
    __syncthreads();
#ifdef VG_PROBE
    if (tid == 0) {
      atomicAdd(&g_probe[12], (unsigned long long)s_tmax);  // the slowest trailing wave's job time
      s_tmax = 0;
    }
#endif
    VG_PROBE_MARK(6);
  }
  flush();
  if (wave == 0) w_job(NB - 1, true);
  __syncthreads();
  VG_PROBE_MARK(5);

  // backward: x_J = w_J + sum_{I>J} (-L_IJ^T) x_I, tile (I, J) now holding
  // -L_IJ^T; wave J keeps its lane shares pa[g] of rows q + 4g and completes
  // x_J at step J+1 (one 16-lane DPP sum per row group)
  {
    double pa[4] = {0.0, 0.0, 0.0, 0.0};
    for (int I = NB - 1; I >= 1; I--) {
      if (wave < I) {
        const double* Lt = &T[tix(I, wave) * 256];
        const double xi = xv[16 * I + cc];
#pragma unroll
        for (int g = 0; g < 4; g++) pa[g] = fma(Lt[tel(rq + 4 * g, cc)], xi, pa[g]);
        if (wave == I - 1) {
#pragma unroll
          for (int g = 0; g < 4; g++) {
            const double t = row16_sum(pa[g]);
            if (cc == 0) xv[16 * (I - 1) + rq + 4 * g] = wv[16 * (I - 1) + rq + 4 * g] + t;
          }
        }
      }
      __syncthreads();
    }
  }
  VG_PROBE_MARK(7);
  for (int t = tid; t < n; t += nt) {
    if (t < m) col[ip[t]] = xv[t];
    else col[t - m] = 0.0;  // the gauge frame (t - m < 15)
  }
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
  if (wave == 1) {  // q1 on its own wave (the trial states run on wave 0): lane-strided sums, fixed xor tree
    double q1 = 0.0;
    for (int r = lane; r < n; r += 64) q1 += col[r] * (u * Dv[r] * col[r] - Jv[r]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) q1 += __shfl_xor(q1, off, 64);
    if (lane == 0) st->q1 = 0.5 * q1;
  }
  if (clk && clk->on) {
    __syncthreads();
    if (tid == 0) {
      clk->solve_ticks += (unsigned long long)wall_clock64() - clk0;
      clk->solve_n += 1;
    }
  }
  VG_PROBE_MARK(8);
#ifdef VG_PROBE
  if (tid == 0) atomicAdd(&g_probe[63], 1ull);
#endif
}

// LM bookkeeping (optimizers.cpp:480-515): k_ba_control, or
// k_ba_resid's IMU workgroup (CtlArg::err set, unsharded; resid_bookkeeping)
struct CtlArg {
  int W, nimu, nrb, nl;
  double imu_coef;
  const double* hl;
  const double* imuout;
  const double* imures;
  const double* rpart;
  double* xs;
  const double* xt;
  double* bias;
  BaState* st;
  Pub* pub;
  int* err;   // k_ba_resid runs the bookkeeping (nullptr: k_ba_control follows); error bit 64 on a stalled hand-off
  int xworld;  // sharded: rpart is the all-reduced exchange frame, its guard checked here (mismatch: bit 32 in xerr)
  int* xerr;
};
// `pre`: the lane's strided sum of the residual partials, already formed (k_ba_resid).
// The sums run over the first kResidThreads lanes whatever the workgroup size
// (k_ba_resid_hess's is 512), so the residual's order is k_ba_resid's.
__device__ __forceinline__ void ba_control_body(const CtlArg& c, const double* pre = nullptr) {
  __shared__ int accept;
  __shared__ double s_r[kResidThreads];
  const int nt = kResidThreads;
  {  // residual partials: lane-strided sums, then a fixed tree (deterministic)
    double part = 0.0;
    const bool ok = c.xworld <= 0 || xchg_ok(c.rpart, kShardSmall, c.xworld);  // (the frame's consumers read zeros)
    if (!ok && threadIdx.x == 0) atomicOr(c.xerr, 32);
    if (pre) part = *pre;
    else if (!c.st->done && ok) {  // a lane's loads in one batch, summed in the same order
      constexpr int kU = 4;
      for (int b0 = threadIdx.x; b0 < c.nrb; b0 += kU * nt) {
        double v[kU];
#pragma unroll
        for (int k = 0; k < kU; k++) v[k] = b0 + k * nt < c.nrb ? c.rpart[b0 + k * nt] : 0.0;
#pragma unroll
        for (int k = 0; k < kU; k++)
          if (b0 + k * nt < c.nrb) part += v[k];
      }
    }
    if ((int)threadIdx.x < nt) s_r[threadIdx.x] = part;
    __syncthreads();
    for (int w = nt >> 1; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) s_r[threadIdx.x] += s_r[threadIdx.x + w];
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    accept = -1;
    if (!c.st->done) {
      // (residual1 of divide_thread at the current state: k_ba_prep, on the Hessian iterations)
      if (c.st->calc_hess) c.st->nhess += 1;
      double r1 = 0.0;
      for (int k = 0; k < c.nimu; k++) r1 += c.imures[k];
      r1 *= c.imu_coef * 0.5;
      const double r2 = s_r[0];
      const double residual2 = r1 + r2;
      c.st->res2 = residual2;
      const double residual1 = c.st->res1;
      double q = residual1 - residual2;
      if (q > 0) {
        accept = 1;
        const double one_three = 1.0 / 3;
        q = q / c.st->q1;
        c.st->v = 2;
        q = 1 - pow(2 * q - 1, 3);
        c.st->u *= (q < one_three ? one_three : q);
        c.st->calc_hess = 1;
      } else {
        accept = 0;
        c.st->u = c.st->u * c.st->v;
        c.st->v = 2 * c.st->v;
        c.st->calc_hess = 0;
      }
      c.st->iters += 1;
      if (fabs((residual1 - residual2) / residual1) < 1e-6) c.st->done = 1;
    }
  }
  __syncthreads();
  if (accept == 1) {
    for (int t = threadIdx.x; t < c.W * kX; t += blockDim.x) c.xs[t] = c.xt[t];
  } else if (accept == 0) {
    for (int t = threadIdx.x; t < c.nimu * 6; t += blockDim.x) {
      int k = t / 6, j = t % 6;
      c.bias[k * 12 + j] = c.bias[k * 12 + 6 + j];
    }
  }
  if (threadIdx.x == 0) {  // LM flags -> host (read without draining the stream)
    c.st->fin = ((c.st->done || c.st->iters >= 10) && !c.st->skip) ? 1 : 0;
    const int seq = c.st->seq;  // one publication per launch, numbered on the device (graph replays)
    c.st->seq = seq + 1;
    // done and the iteration count in one word: the host reads them as one
    // (a queued-ahead iteration publishing between two separate reads could
    // pair one iteration's count with the next one's done, and sharded ranks
    // would then enqueue different iteration counts)
    pub_store(&c.pub->ba_word, c.st->iters * 2 + (c.st->done ? 1 : 0));
    pub_flag(&c.pub->seq_ba, seq);
  }
}
__global__ void __launch_bounds__(256) k_ba_control(CtlArg c) { ba_control_body(c); }

// The LM bookkeeping inside k_ba_resid, without a fence per workgroup (an
// agent-scope release writes back the XCD's L2): every residual slot starts
// as a sentinel NaN (k_ba_init, and the reader re-arms it), each workgroup
// stores its partial with one relaxed agent-scope 64-bit store, and the IMU
// workgroup (the last dispatched) polls the slots until none holds the
// sentinel, then runs k_ba_control's body on the values it read.
constexpr unsigned long long kRpartEmpty = 0x7ff4deadbeef0001ull;  // a NaN payload arithmetic never produces
__device__ __forceinline__ void rpart_put(double* slot, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(slot), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void resid_bookkeeping(const CtlArg& c) {
  __shared__ int s_late;
  if (threadIdx.x == 0) s_late = 0;
  __syncthreads();
  double part = 0.0;  // k_ba_control's lane-strided order: slots t, t + 256, ...
  for (int b = threadIdx.x; b < c.nrb && (int)threadIdx.x < kResidThreads; b += kResidThreads) {
    unsigned long long* p = reinterpret_cast<unsigned long long*>(const_cast<double*>(c.rpart) + b);
    unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int spin = 0; v == kRpartEmpty; spin++) {
      if (spin > (1 << 22)) {  // ~seconds: a workgroup never stored (should not happen)
        s_late = 1;
        v = 0ull;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(p, kRpartEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
    part += __longlong_as_double((long long)v);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_late) atomicOr(c.err, 64);
  ba_control_body(c, &part);
}

// evaluate_only_residual (factors.cpp:128-158) at the trial poses. A chunk of
// 256/W factors per workgroup step: lane (f, i) moves factor f's frame-i
// cluster to the trial pose (independent work, in parallel), then lane f merges
// them onto pcr_fix in frame order (the reference's order) and takes the 3x3
// eigen-decomposition. Workgroup b < nrb takes chunks b, b + nrb, ... of the
// device factor count *nfp; its residual partial goes to rpart[b].
__global__ void __launch_bounds__(256, 2) k_ba_resid(const int* __restrict__ nfp, int W, const int* __restrict__ fac_node,
                                                  const Clu* __restrict__ pcr_fix, const Clu* __restrict__ pcrs,
                                                  const int* __restrict__ mpring, const double* __restrict__ xt,
                                                  double* __restrict__ fac_eig, Clu* __restrict__ fac_pcr,
                                                  double* __restrict__ rpart, const BaState* st, int nrb,
                                                  int nimu, const double* __restrict__ imurec,
                                                  const int* __restrict__ imu_head,
                                                  const double* __restrict__ bias, double* __restrict__ imures,
                                                  CtlArg ctl) {
  if (st->done) {  // converged: the bookkeeping still publishes the flags
    if (ctl.err && (int)blockIdx.x == nrb) ba_control_body(ctl);
    return;
  }
  if ((int)blockIdx.x >= nrb) {  // IMU residuals at the trial state in the same launch
    if ((int)threadIdx.x < nimu) imu_residual_lane(threadIdx.x, imurec, *imu_head, bias, xt, imures);
    if (ctl.err) {
      __syncthreads();  // imures, read by thread 0 of this workgroup
      resid_bookkeeping(ctl);
    }
    return;
  }
  __shared__ Clu s_t[256];
  __shared__ double red[4];
  const int FS = 256 / W;
  const int f = threadIdx.x / W, i = threadIdx.x % W;
  const int nf = *nfp;
  const int nchunk = (nf + FS - 1) / FS;
  double acc = 0.0;
  for (int ch = blockIdx.x; ch < nchunk; ch += nrb) {
    const int a = ch * FS + f;
    if (f < FS && a < nf) {
      const Clu src = pcrs[(size_t)fac_node[a] * W + mpring[i]];
      Clu t;
      if (src.N != 0) {
        t = clu_transform(src, ld_m3(&xt[(size_t)i * kX]), ld_v3(&xt[(size_t)i * kX + 9]));
      } else {
        clu_zero(t);
        t.N = 0;
      }
      s_t[threadIdx.x] = t;
    }
    __syncthreads();
    const int a2 = ch * FS + (int)threadIdx.x;
    if ((int)threadIdx.x < FS && a2 < nf) {
      Clu sig = pcr_fix[fac_node[a2]];
      for (int k = 0; k < W; k++) {
        const Clu& t = s_t[threadIdx.x * W + k];
        if (t.N != 0) clu_add(sig, t);
      }
      V3 ev;
      M3 U;
      eig3(clu_cov(sig), ev, U);
      double* e = &fac_eig[(size_t)a2 * 12];
      for (int j = 0; j < 3; j++) e[j] = ev[j];
      for (int j = 0; j < 9; j++) e[3 + j] = U[j];
      fac_pcr[a2] = sig;
      acc += 1.0 * ev[0];
    }
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) rpart_put(&rpart[blockIdx.x], ((red[0] + red[1]) + red[2]) + red[3]);
}

// The first LM iteration's residual pass and, speculatively, the second
// iteration's Hessian pass at the same trial state, as one launch
// (vg_ctx::ba_resid_hess). An accepted step makes the trial the state
// (optimizers.cpp:480-492), so the second iteration's Hessian is the one of
// the trial poses: every chunk workgroup does k_ba_resid's work for its
// factors (hess_chunk_eval<true>) and goes straight on to their Hessian, so
// the second iteration needs no k_ba_hess launch. A rejected step leaves the
// Hessian unused (calc_hess = 0: k_ba_hfinal / k_ba_prep take the stored
// system). Layout: workgroups [0, kResidBlocks / 2) the Hessian chunks c, c +
// kResidBlocks / 2, ... (hess_fs = 2 x k_ba_resid's chunk: chunk c holds
// residual chunks 2c and 2c + 1, and this workgroup stores their residual
// partials exactly as k_ba_resid's workgroups 2c and 2c + 1 would); then the
// IMU residuals + the LM bookkeeping (resid_bookkeeping); then one workgroup
// per IMU factor's Hessian block (imu_factor_block at the trial). Results are
// bit-identical to k_ba_resid followed by k_ba_hess.
constexpr int kRhChunkWg = kResidBlocks / 2;
__global__ void __launch_bounds__(kHessThreads) k_ba_resid_hess(const int* __restrict__ nfp, int W,
                                                                const int* __restrict__ fac_node,
                                                                const Clu* __restrict__ pcr_fix,
                                                                const Clu* __restrict__ pcrs,
                                                                const int* __restrict__ mpring,
                                                                const double* __restrict__ xt,
                                                                double* __restrict__ fac_eig, Clu* __restrict__ fac_pcr,
                                                                double* __restrict__ part, double* __restrict__ rpart,
                                                                const BaState* st, int nimu,
                                                                const double* __restrict__ imurec,
                                                                const int* __restrict__ imu_head,
                                                                const double* __restrict__ bias,
                                                                double* __restrict__ imures, double* __restrict__ imuout,
                                                                CtlArg ctl) {
  const int G = kRhChunkWg;
  if (st->done) {  // converged: the bookkeeping still publishes the flags
    if (ctl.err && (int)blockIdx.x == G) ba_control_body(ctl);
    return;
  }
  if ((int)blockIdx.x == G) {  // IMU residuals at the trial state, then the bookkeeping (k_ba_resid's)
    if ((int)threadIdx.x < nimu) imu_residual_lane(threadIdx.x, imurec, *imu_head, bias, xt, imures);
    if (ctl.err) {  // (sharded: k_ba_rsum, the exchange and k_ba_control follow)
      __syncthreads();
      resid_bookkeeping(ctl);
    }
    return;
  }
  if ((int)blockIdx.x > G) {  // the IMU factors' Hessian blocks at the trial (k_ba_hess's IMU workgroups)
    const int k = blockIdx.x - G - 1;
    if (k < nimu) imu_factor_block(k, imurec, *imu_head, bias, xt, imuout);
    return;
  }
  const int nf = *nfp;
  const int nchunk = (nf + hess_chunk(W) - 1) / hess_chunk(W);
  double ev0[2] = {0.0, 0.0};
  for (int ch = blockIdx.x; ch < nchunk; ch += G)
    hess_chunk_eval<true>(ch, nf, W, fac_node, nullptr, nullptr, pcrs, mpring, xt, part, pcr_fix, fac_eig, fac_pcr,
                          ev0);
  // the residual partials of chunks 2c and 2c + 1 in k_ba_resid's form: lane l
  // of its wave 0 holds the chunk's factor l, the other waves hold zeros
  if (threadIdx.x < 64) {
    const int fr = 256 / W, lane = threadIdx.x;
    double r0 = ev0[0];
    double r1 = __shfl_down(ev0[1], fr, 64);
    if (lane >= fr) r1 = 0.0;
    for (int off = 32; off > 0; off >>= 1) r0 += __shfl_down(r0, off, 64);
    for (int off = 32; off > 0; off >>= 1) r1 += __shfl_down(r1, off, 64);
    double z = 0.0;  // waves 1-3 of k_ba_resid: an all-zero tree
    for (int off = 32; off > 0; off >>= 1) z += __shfl_down(z, off, 64);
    if (lane == 0) {
      rpart_put(&rpart[2 * blockIdx.x], ((r0 + z) + z) + z);
      rpart_put(&rpart[2 * blockIdx.x + 1], ((r1 + z) + z) + z);
    }
  }
}

// sharded mode: this shard's factor residual (ordered sum of the block
// partials) packed into the exchange frame (k_ba_control checks its guard)
// (the partials staged in LDS by every lane in one round of loads, then the
// same sequential sum on one lane)
__global__ void k_ba_rsum(int nrb, const double* __restrict__ rpart, const BaState* __restrict__ st, XchgArg xa) {
  __shared__ double sp[kResidBlocks];
  for (int i = threadIdx.x + 1; i < xa.n - 2; i += blockDim.x) xa.frame[i] = 0.0;
  const bool run = !st->done && nrb <= kResidBlocks;
  if (run) {
    constexpr int kU = kResidBlocks / 64;
    double v[kU];
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const int b = threadIdx.x + 64 * k;
      v[k] = b < nrb ? rpart[b] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const int b = threadIdx.x + 64 * k;
      if (b < nrb) sp[b] = v[k];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0.0;
    if (run)
      for (int b = 0; b < nrb; b++) r += sp[b];
    else if (!st->done)
      for (int b = 0; b < nrb; b++) r += rpart[b];
    xa.frame[0] = r;
    xchg_close(xa.frame, xa.n, 4, xa.seq);
  }
}

struct MpRing {
  int mp[kMaxW];
};
// LM state (optimizers.cpp:436-441), the reduced-Hessian accumulator, the ring.
// ph (the scan graph, pipeline.cpp): the per-scan numbers k_ins_prep copied
// from host-mapped memory into DState::ph — the LM's first flag number
// replaces seq0, and the recut-done flag the margi prefix waits for
// (vg_ctx::d_sync[3]) is raised here (the recut's kernels have ended)
// fin (an asynchronous recut, map_recut): tras_opt's factor bookkeeping
// (k_factor_finish_dev's work: opt_state = factor index, the factors' eigen
// and cluster copies) over the whole grid, beside the LM state in workgroup 0 —
// one launch fewer on the chain
__device__ __forceinline__ void ba_init_common(int gt, int gn, bool wg0, BaState* st, double* __restrict__ hl,
                                               double* __restrict__ hl_part, int nout, const MpRing& ring,
                                               int* __restrict__ mpring, int W, int status, int seq0,
                                               double* __restrict__ rpart, int nrb, const int* __restrict__ ph,
                                               unsigned* __restrict__ rc_flag);
__global__ void __launch_bounds__(256) k_ba_init(BaState* st, double* __restrict__ hl, double* __restrict__ hl_part,
                                                 int nout, MpRing ring, int* __restrict__ mpring, int W,
                                                 const int* __restrict__ rc_status, int seq0, double* __restrict__ rpart,
                                                 int nrb, const int* __restrict__ ph, unsigned* __restrict__ rc_flag,
                                                 int fin, DevMap m, const int* __restrict__ fac_node,
                                                 double* __restrict__ fac_eig, Clu* __restrict__ fac_pcr) {
  const int gt = blockIdx.x * blockDim.x + threadIdx.x, gn = gridDim.x * blockDim.x;
  const int status = rc_status ? *rc_status : 0;
  if (fin && !status) {
    const int nf = m.counters[kCntFactors];
    for (int a = gt; a < nf; a += gn) {
      const int node = fac_node[a];
      m.hdr[node].opt_state = a;
      for (int j = 0; j < 12; j++) fac_eig[(size_t)a * 12 + j] = m.eig[(size_t)node * 12 + j];
      fac_pcr[a] = m.pcr_add[node];
    }
  }
  ba_init_common(gt, gn, blockIdx.x == 0, st, hl, hl_part, nout, ring, mpring, W, status, seq0, rpart, nrb, ph,
                 rc_flag);
}
// k_ba_init's part after the factor bookkeeping: the residual slots armed, the
// Hessian accumulators cleared (grid-stride gt / gn), then (wg0) the ring and
// the LM state
__device__ __forceinline__ void ba_init_common(int gt, int gn, bool wg0, BaState* st, double* __restrict__ hl,
                                               double* __restrict__ hl_part, int nout, const MpRing& ring,
                                               int* __restrict__ mpring, int W, int status, int seq0,
                                               double* __restrict__ rpart, int nrb, const int* __restrict__ ph,
                                               unsigned* __restrict__ rc_flag) {
  for (int b = gt; b < nrb; b += gn)  // empty residual slots (resid_bookkeeping)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(rpart + b), kRpartEmpty, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  for (int t = gt; t < nout; t += gn) {
    hl[t] = 0.0;
    hl_part[t] = 0.0;
  }
  if (!wg0) return;
  if ((int)threadIdx.x < W) mpring[threadIdx.x] = ring.mp[threadIdx.x];
  if (threadIdx.x == 0) {
    const int skip = status ? 1 : 0;  // an asynchronous recut that needs the host: skip
    st->u = 0.01;
    st->v = 2;
    st->res1 = st->res2 = st->q1 = 0.0;
    st->calc_hess = 1;
    st->done = skip;
    st->skip = skip;
    st->iters = 0;
    st->nhess = 0;
    st->seq = ph ? ph[0] : seq0;
    st->fin = 0;
    if (ph) __hip_atomic_store(rc_flag, (unsigned)ph[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// k_ba_init + the first LM iteration's k_ba_hess as one launch (the scan
// graph, vg_ctx::ba_init_hess): workgroups [0, G) the Hessian chunks, which
// also do tras_opt's bookkeeping for their own factors when `fin` (each
// factor's eigen system and cluster read from the map, copied to fac_eig /
// fac_pcr, opt_state = factor index: k_ba_init's loop), with the ring from
// the arguments; then the IMU factors' blocks; the last workgroup does the
// rest of k_ba_init (ba_init_common). Nothing in the launch reads the LM state
// the last workgroup writes: the chunks decide on the recut status, the same
// test k_ba_init's skip is.
__global__ void __launch_bounds__(kHessThreads) k_ba_init_hess(
    const int* __restrict__ nfp, int W, const int* __restrict__ fac_node, double* __restrict__ fac_eig,
    Clu* __restrict__ fac_pcr, const Clu* __restrict__ pcrs, const double* __restrict__ xs, double* __restrict__ part,
    int G, int nimu, const double* __restrict__ imurec, const int* __restrict__ imu_head,
    const double* __restrict__ bias, double* __restrict__ imuout, KClock* __restrict__ clk, BaState* st,
    double* __restrict__ hl, double* __restrict__ hl_part, int nout, MpRing ring, int* __restrict__ mpring,
    const int* __restrict__ rc_status, double* __restrict__ rpart, int nrb, const int* __restrict__ ph,
    unsigned* __restrict__ rc_flag, int fin, DevMap m, int seq0) {
  const int status = rc_status ? *rc_status : 0;
  if ((int)blockIdx.x == G + nimu) {
    ba_init_common(threadIdx.x, blockDim.x, true, st, hl, hl_part, nout, ring, mpring, W, status, seq0, rpart, nrb, ph,
                   rc_flag);
    return;
  }
  if (status) return;  // the recut needs the host: the LM is skipped (k_ba_init's skip)
  if ((int)blockIdx.x >= G) {  // IMU factors (give_evaluate, jac_enable)
    imu_factor_block(blockIdx.x - G, imurec, *imu_head, bias, xs, imuout);
    return;
  }
  __shared__ int s_mp[kMaxW];
  if ((int)threadIdx.x < kMaxW) s_mp[threadIdx.x] = ring.mp[threadIdx.x];
  const bool clk_on = clk && clk->on;  // in-kernel clock (vg_profile bit 2): the LM's iteration 0 slot
  const int clk_slot = clk_on ? (clk->scan * 8) & (kClkHRing - 1) : 0;
  if (clk_on && blockIdx.x == 0 && threadIdx.x == 0) {
    clk->h_t0[clk_slot] = (unsigned long long)wall_clock64();
    clk->h_exec[clk_slot] = 1;
  }
  __syncthreads();  // s_mp
  const int nf = *nfp;
  const int nchunk = (nf + hess_chunk(W) - 1) / hess_chunk(W);
  for (int ch = blockIdx.x; ch < nchunk; ch += G)
    hess_chunk_eval<false>(ch, nf, W, fac_node, fac_eig, fac_pcr, pcrs, s_mp, xs, part, nullptr, fac_eig, fac_pcr,
                           nullptr, fin ? m.eig : nullptr, fin ? m.pcr_add : nullptr, fin ? m.hdr : nullptr);
  if (clk_on && blockIdx.x < kClkHBlocks) {
    __syncthreads();
    if (threadIdx.x == 0) clk->h_tend[clk_slot][blockIdx.x] = (unsigned long long)wall_clock64();
  }
}

struct BaDev {
  double* part;
  double* hl;
  double* imurec;
  double* bias;
  double* imuout;
  double* imures;
  double* Hcalc;
  double* timg;
  double* bvec;
  double* dvec;
  double* jvec;
  int* ipg;
  double* Jcalc;
  double* xs;
  double* xt;
  double* dxi;
  double* rpart;
  int* mpring;
  BaState* st;
};
static BaDev g_dummy;

// dynamic LDS of k_ba_hess: the X operand of a sub-chunk, reused as the
// per-lane (hb, jj, res) rows of the final reduction (512 x 28 doubles =
// 112 KB); with the static S[512] (4 KB) it must fit gfx950's 160 KB LDS,
// checked at context creation (ba_alloc) against the device limit
static size_t hess_lds_bytes(int W) {
  const size_t gemm = (size_t)hess_ks(W) * hess_xs(W), red = (size_t)kHessThreads * 28;
  return (gemm > red ? gemm : red) * sizeof(double);
}
static_assert((size_t)kHessThreads * 28 * sizeof(double) + kHessThreads * sizeof(double) <= 160 * 1024,
              "k_ba_hess reduction rows exceed gfx950 LDS");

static size_t solve_lds_bytes(int W) {
  const int NB = (15 * W - 15 + kTile - 1) / kTile;  // the gauge frame is not factored
  return (size_t)NB * (NB + 1) / 2 * 256 * sizeof(double);
}

int ba_alloc(vg_ctx* ctx) {
  BaBufs& b = ctx->ba;
  const int W = ctx->cfg.win_size;
  b.cap_f = ctx->cap.max_nodes / 8 > 262144 ? 262144 : (ctx->cap.max_nodes / 8 > 4096 ? ctx->cap.max_nodes / 8 : 4096);
  const int L = 6 * W, nout = L * (L + 1) / 2 + L + 1, n = 15 * W;
  bool good = true;
  good &= (b.fac_node = ctx->arena.take<int>(b.cap_f)) != nullptr;
  good &= (b.fac_eig = ctx->arena.take<double>((size_t)b.cap_f * 12)) != nullptr;
  good &= (b.fac_pcr = ctx->arena.take<Clu>(b.cap_f)) != nullptr;
  good &= (b.hpart = ctx->arena.take<double>((size_t)(b.cap_f / hess_chunk(W) + 1) * nout)) != nullptr;
  good &= (b.hout = ctx->arena.take<double>(nout + 16)) != nullptr;
  good &= (b.hout_part = ctx->arena.take<double>(nout + 16)) != nullptr;
  good &= (b.rpart = ctx->arena.take<double>(kResidBlocks + 16)) != nullptr;
  good &= (b.xs = ctx->arena.take<double>(1024 + 2 * n * (n + 1) / 2 + 4 * n + kMaxNB * (kMaxNB + 1) / 2 * 256 + 4 * kMaxNB * kTile + 2 * kMaxW * kX + kMaxW * kImuRec +
                                          kMaxW * 12 + kMaxW * 931 + kMaxW + 64)) != nullptr;
  if (!good) {
    ctx->err = "arena exhausted (BA)";
    return VG_E_CAPACITY;
  }
  if (W > kMaxW || 15 * W > kMaxNB * kTile) {
    ctx->err = "win_size > 11 unsupported by the BA solve (LDS-resident 15W x 15W tile store)";
    return VG_E_ARG;
  }
  {  // both LM kernels keep their working set in LDS: check the device limit up front
    int lds_max = 0;
    VG_HIP(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, ctx->device));
    const size_t hess_total = hess_lds_bytes(W) + kHessThreads * sizeof(double);
    if (lds_max > 0 && (hess_total > (size_t)lds_max || solve_lds_bytes(W) > (size_t)lds_max)) {
      ctx->err = "LM kernels need " + std::to_string(hess_total) + " / " + std::to_string(solve_lds_bytes(W)) +
                 " B of LDS per workgroup; the device allows " + std::to_string(lds_max);
      return VG_E_ARG;
    }
  }
  VG_HIP(hipFuncSetAttribute((const void*)k_ba_solve, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)solve_lds_bytes(W)));
  VG_HIP(hipFuncSetAttribute((const void*)k_ba_hess, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hess_lds_bytes(W)));
  VG_HIP(hipFuncSetAttribute((const void*)k_ba_resid_hess, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hess_lds_bytes(W)));
  VG_HIP(hipFuncSetAttribute((const void*)k_ba_init_hess, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hess_lds_bytes(W)));
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
  d.timg = p;
  p += kMaxNB * (kMaxNB + 1) / 2 * 256;
  d.bvec = p;
  p += kMaxNB * kTile;
  d.dvec = p;
  p += kMaxNB * kTile;
  d.jvec = p;
  p += kMaxNB * kTile;
  d.ipg = (int*)p;
  p += kMaxNB * kTile;
  d.Jcalc = p;
  p += n;
  d.dxi = p;
  p += n;
  d.xs = ctx->st->xs;  // window states live in the device state (state.hip)
  p += kMaxW * kX;
  d.xt = p;
  p += kMaxW * kX;
  d.imurec = ctx->st->imurec;
  p += kMaxW * kImuRec;
  d.bias = ctx->st->bias;
  p += kMaxW * 12;
  d.imuout = p;
  p += kMaxW * 931;
  d.imures = p;
  p += kMaxW;
  d.st = (BaState*)p;
  p += 16;
  d.mpring = (int*)p;
  p += 16;
  d.part = b.hpart;
  d.hl = b.hout;
  d.rpart = b.rpart;
  return d;
}

const int* ba_iters_dev(vg_ctx* ctx) { return &carve(ctx).st->iters; }
const int* ba_hess_dev(vg_ctx* ctx) { return &carve(ctx).st->nhess; }
const int* ba_gate_dev(vg_ctx* ctx) { return &carve(ctx).st->fin; }

// one LM iteration (optimizers.cpp:449-516); kernels early-exit on the
// device-side flags once converged. Every argument is fixed per context (the
// factor count, the flags and the publication number live on the device), so
// an unsharded run replays one captured graph per iteration; the sampled
// solve-timing runs launch directly (events around k_ba_solve).
// rh: 1 this iteration's residual pass is k_ba_resid_hess (it also forms the
// next iteration's Hessian at the trial), 2 this iteration's Hessian came
// from the previous iteration's k_ba_resid_hess (no k_ba_hess launch)
// ih (the scan graph, k == 0): k_ba_init_hess replaces k_ba_init + k_ba_hess
struct InitHessArg {
  MpRing ring;
  int fin;
  int seq0;  // > 0: the LM's first flag number (a direct launch); 0: DState::ph (the scan graph)
};
static void ba_iter_kernels(vg_ctx* ctx, int k, bool solve_ev, int& xerr, int rh = 0,
                            const InitHessArg* ih = nullptr) {
  const int W = ctx->cfg.win_size;
  hipStream_t s = ctx->stream;
  BaDev d = carve(ctx);
  const int nimu = W - 1;
  const int L = 6 * W, nl = L * (L + 1) / 2, nout = nl + L + 1;
  const bool shard_on = sharded(ctx);
  // factor count on the device (the recut's kCntFactors): fixed grids, so an
  // asynchronous recut needs no host round trip before the LM
  const int* nfp = ctx->map.counters + kCntFactors;
  const int G = std::min(kHessGridMax, ctx->ba.cap_f / hess_chunk(W) + 1);
  const int nrb = kResidBlocks;
  const size_t hess_lds = hess_lds_bytes(W);
  const size_t solve_lds = solve_lds_bytes(W);
  const int NBt = (15 * W - 15 + kTile - 1) / kTile, ntile = NBt * (NBt + 1) / 2;
  Shard& sh = ctx->shard;
  // sharded: the Hessian / gradient / residual frame and the trial residual's
  // frame are packed by k_ba_hfinal / k_ba_rsum and checked by k_ba_prep /
  // k_ba_control (no pack / unpack launches)
  const double* hlx = shard_on ? sh.d_frame : d.hl;  // the LiDAR system the assembly reads
  CtlArg ctl{W, nimu, shard_on ? 1 : nrb, nl + L, ctx->cfg.imu_coef, hlx, d.imuout, d.imures,
             shard_on ? sh.d_frame : d.rpart, d.xs, d.xt, d.bias, d.st, ctx->d_pub, nullptr,
             shard_on ? sh.world : 0, ctx->map.counters + kCntErr};
  CtlArg ctl_fused = ctl;  // unsharded: the bookkeeping rides in k_ba_resid's IMU workgroup
  if (!shard_on && ctx->ba_fuse_ctl) ctl_fused.err = ctx->map.counters + kCntErr;
  if (ih)
    k_ba_init_hess<<<G + nimu + 1, kHessThreads, hess_lds, s>>>(
        nfp, W, ctx->ba.fac_node, ctx->ba.fac_eig, ctx->ba.fac_pcr, ctx->map.pcrs, d.xs, d.part, G, nimu, d.imurec,
        &ctx->st->imu_head, d.bias, d.imuout, &ctx->st->clk, d.st, d.hl, ctx->ba.hout_part, nout, ih->ring, d.mpring,
        map_rc_status(ctx), d.rpart, kResidBlocks, ih->seq0 > 0 ? nullptr : ctx->st->ph,
        ih->seq0 > 0 ? nullptr : ctx->d_sync + 3, ih->fin, ctx->map, ih->seq0);
  else if (rh != 2)
    k_ba_hess<<<G + nimu, kHessThreads, hess_lds, s>>>(nfp, W, ctx->ba.fac_node, ctx->ba.fac_eig, ctx->ba.fac_pcr,
                                                      ctx->map.pcrs, d.mpring, d.xs, d.part, d.st, G, nimu, d.imurec,
                                                      &ctx->st->imu_head, d.bias, d.imuout, &ctx->st->clk);
  const XchgArg xh{shard_on ? sh.d_frame : nullptr, sh.d_seq, ctx->map.counters + kCntErr, sh.frame_n, sh.world};
  k_ba_hfinal<<<(nout * 8 + 255) / 256, 256, 0, s>>>(nfp, hess_chunk(W), nout, d.part, shard_on ? sh.d_frame : d.hl,
                                                       d.st, xh);
  // sharded: every shard's factors -> one LiDAR Hessian / gradient / residual
  if (shard_on && xerr == VG_OK) xerr = shard_exchange(ctx, sh.frame_n);
  if (k == 0 && ctx->dbg_capture == 1 && ctx->dbg_cap_buf) {  // test knob (vgx_debug 5): the first pass
    (void)hipMemcpyAsync(ctx->dbg_cap_buf, d.hl, nout * sizeof(double), hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(ctx->dbg_cap_buf + nout, d.imuout, (size_t)nimu * 931 * sizeof(double),
                         hipMemcpyDeviceToDevice, s);
    ctx->dbg_cap_n = nout + nimu * 931;
    ctx->dbg_capture = 2;
  }
  k_ba_prep<<<ntile, 256, 0, s>>>(W, nimu, ctx->cfg.imu_coef, hlx, d.imuout, d.Hcalc, d.Jcalc, d.timg, d.bvec,
                                  d.dvec, d.jvec, d.ipg, d.st, ctx->ba_structural ? 1 : 0, shard_on ? sh.world : 0,
                                  ctx->map.counters + kCntErr);
  if (solve_ev) (void)hipEventRecord(ctx->solve_ev[k][0], s);
  k_ba_solve<<<1, 1024, solve_lds, s>>>(W, nimu, d.timg, d.bvec, d.dvec, d.jvec, d.ipg, d.xs, d.xt, d.bias, d.dxi,
                                       d.st, &ctx->st->clk);
  if (solve_ev) (void)hipEventRecord(ctx->solve_ev[k][1], s);
  if (rh == 1)
    k_ba_resid_hess<<<kRhChunkWg + 1 + nimu, kHessThreads, hess_lds, s>>>(
        nfp, W, ctx->ba.fac_node, ctx->map.pcr_fix, ctx->map.pcrs, d.mpring, d.xt, ctx->ba.fac_eig, ctx->ba.fac_pcr,
        d.part, d.rpart, d.st, nimu, d.imurec, &ctx->st->imu_head, d.bias, d.imures, d.imuout, ctl_fused);
  else
    k_ba_resid<<<nrb + 1, kResidThreads, 0, s>>>(nfp, W, ctx->ba.fac_node, ctx->map.pcr_fix, ctx->map.pcrs, d.mpring,
                                                 d.xt, ctx->ba.fac_eig, ctx->ba.fac_pcr, d.rpart, d.st, nrb, nimu,
                                                 d.imurec, &ctx->st->imu_head, d.bias, d.imures, ctl_fused);
  if (shard_on) {  // the residual over every shard's factors
    k_ba_rsum<<<1, 64, 0, s>>>(nrb, d.rpart, d.st,
                               XchgArg{sh.d_frame, sh.d_seq, ctx->map.counters + kCntErr, kShardSmall, sh.world});
    if (xerr == VG_OK) xerr = shard_exchange(ctx, kShardSmall);
  }
  if (!ctl_fused.err) k_ba_control<<<1, 256, 0, s>>>(ctl);
}

// k_ba_init: seq0 > 0 the LM's first flag number, else (the scan graph) read
// on the device from DState::ph
static void ba_init_kernel(vg_ctx* ctx, const int* mp_ring, int seq0) {
  const int W = ctx->cfg.win_size;
  BaDev d = carve(ctx);
  const int L = 6 * W, nout = L * (L + 1) / 2 + L + 1;
  // the IMU records are in DState's ring (k_push_state), the mp ring rides in k_ba_init's arguments
  MpRing ring;
  for (int i = 0; i < kMaxW; i++) ring.mp[i] = i < W ? mp_ring[i] : 0;
  const bool fin = ctx->rc_finish_in_init;  // the asynchronous recut left tras_opt's bookkeeping to this launch
  ctx->rc_finish_in_init = false;
  k_ba_init<<<fin ? 64 : 1, 256, 0, ctx->stream>>>(d.st, d.hl, ctx->ba.hout_part, nout, ring, d.mpring, W,
                                                    map_rc_status(ctx), seq0, d.rpart, kResidBlocks,
                                                    seq0 > 0 ? nullptr : ctx->st->ph, ctx->d_sync + 3, fin ? 1 : 0,
                                                    ctx->map, ctx->ba.fac_node, ctx->ba.fac_eig, ctx->ba.fac_pcr);
}

// the two-iteration LM graphs take k_ba_resid_hess (unsharded, bookkeeping
// fused, hess_fs(W) two residual chunks)
static bool ba_rh_on(vg_ctx* ctx) {
  return ctx->ba_resid_hess && ctx->ba_fuse_ctl && !sharded(ctx) && resid_hess_ok(ctx->cfg.win_size);
}

// the scan graph's LM part (pipeline.cpp stage_insert_recut), captured on the
// context stream: k_ba_init reading its per-scan numbers from the device,
// then the first two iterations
int ba_capture_scan_lm(vg_ctx* ctx, const int* mp_ring) {
  int xerr = VG_OK;
  const bool rh = ba_rh_on(ctx);
  if (ctx->ba_init_hess && !sharded(ctx)) {  // k_ba_init inside the first Hessian pass
    InitHessArg ih;
    for (int i = 0; i < kMaxW; i++) ih.ring.mp[i] = i < ctx->cfg.win_size ? mp_ring[i] : 0;
    ih.fin = ctx->rc_finish_in_init ? 1 : 0;
    ih.seq0 = 0;
    ctx->rc_finish_in_init = false;
    ba_iter_kernels(ctx, 0, false, xerr, rh ? 1 : 0, &ih);
  } else {
    ba_init_kernel(ctx, mp_ring, 0);
    ba_iter_kernels(ctx, 0, false, xerr, rh ? 1 : 0);
  }
  ba_iter_kernels(ctx, 1, false, xerr, rh ? 2 : 0);
  VG_HIP(hipGetLastError());
  return xerr;
}

// Run damping_iter on the device state. imurec: (W-1) x kImuRec host records
// (pinned staging, uploaded asynchronously). The window states and the IMU
// bias records are read and written in DState.
// pre > 0: k_ba_init, the first `pre` iterations and the gated margi tail are
// already on the stream (the scan graph), with the flag numbers from
// ctx->ba_seq0_pre
int ba_run(vg_ctx* ctx, int nf, const int* mp_ring, int* iters, const std::function<int()>& before_first_wait,
           const std::function<int(bool*)>& spec_tail, bool* tail_ok, bool* pending, int pre) {
  if (pending) *pending = false;
  const int W = ctx->cfg.win_size;
  if (15 * W > kMaxNB * kTile) {
    ctx->err = "win_size > 11 unsupported by the BA solve (LDS-resident 15W x 15W tile store)";
    return VG_E_ARG;
  }
  hipStream_t s = ctx->stream;
  (void)nf;
  const bool shard_on = sharded(ctx);
  int seq0;
  // sharded (direct launches, exchanges between): k_ba_init inside the first
  // Hessian pass and the first residual pass forming the second iteration's
  // Hessian, as the unsharded graphs do; the residual's bookkeeping stays in
  // k_ba_control, behind the residual exchange
  const bool shard_fused = shard_on && ctx->ba_init_hess && ctx->ba_resid_hess && resid_hess_ok(W);
  InitHessArg ih;
  if (pre > 0) {
    seq0 = ctx->ba_seq0_pre;
  } else {
    seq0 = ctx->pub_seq + 1;
    ctx->pub_seq += 10;
    if (shard_fused) {
      for (int i = 0; i < kMaxW; i++) ih.ring.mp[i] = i < W ? mp_ring[i] : 0;
      ih.fin = ctx->rc_finish_in_init ? 1 : 0;
      ctx->rc_finish_in_init = false;
      ih.seq0 = seq0;
    } else {
      ba_init_kernel(ctx, mp_ring, seq0);
    }
    VG_HIP(flush_insert_events(ctx));
  }
  int xerr = VG_OK;  // exchange errors (sharded mode)
  // k_ba_solve launch events (vg_profile): on every prof_every-th run only, so
  // that timing a long run costs the stream little (each record is a gap)
  const bool solve_ev = pre == 0 && ctx->prof_on && !ctx->prof_clock &&
                        (ctx->prof_every <= 1 || ctx->prof_runs++ % ctx->prof_every == 0);
  auto enqueue = [&](int k) {
    if (shard_fused && pre == 0 && k < 2) ba_iter_kernels(ctx, k, solve_ev, xerr, k + 1, k == 0 ? &ih : nullptr);
    else ba_iter_kernels(ctx, k, solve_ev, xerr);
  };
  const bool graph = ctx->use_graphs && ctx->ba_graph && !shard_on && !solve_ev && ctx->dbg_capture != 1;
  if (graph && !ctx->g_ba) {
    std::lock_guard<std::recursive_mutex> cap_lk_(capture_mutex());  // (vg_internal.h)
    VG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    enqueue(0);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    VG_HIP(e);
    VG_HIP(hipGraphInstantiate(&ctx->g_ba, g, nullptr, nullptr, 0));
    VG_HIP(hipGraphDestroy(g));
  }
  // the two iterations of the steady state as ONE graph (no graph boundary
  // between them: each boundary left the stream idle ~9 us)
  const bool graph2 = pre == 0 && graph && ctx->ba_graph2 && ctx->ba_last_iters >= 2;
  if (graph2 && !ctx->g_ba2) {
    std::lock_guard<std::recursive_mutex> cap_lk_(capture_mutex());  // (vg_internal.h)
    VG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const bool rh = ba_rh_on(ctx);
    ba_iter_kernels(ctx, 0, solve_ev, xerr, rh ? 1 : 0);
    ba_iter_kernels(ctx, 1, solve_ev, xerr, rh ? 2 : 0);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    VG_HIP(e);
    VG_HIP(hipGraphInstantiate(&ctx->g_ba2, g, nullptr, nullptr, 0));
    VG_HIP(hipGraphDestroy(g));
  }
  auto iteration = [&](int k) {
    if (!graph) return enqueue(k);
    const hipError_t e = hipGraphLaunch(ctx->g_ba, s);
    if (e != hipSuccess && xerr == VG_OK) {
      ctx->err = std::string("hipGraphLaunch (LM iteration): ") + hipGetErrorString(e);
      xerr = VG_E_HIP;
    }
  };
  // One iteration ahead: iteration k+1 is enqueued before the host waits for
  // iteration k's flags, so the stream never drains; a converged LM leaves at
  // most one early-exiting iteration behind (optimizers.cpp:449, at most 10).
  // Except at the iteration count the previous LM run converged at: there the
  // host waits first (a round trip, ~15 us) rather than queue an iteration
  // that most likely early-exits (~35 us of dispatches). Results do not depend
  // on it: the device-side flags decide.
  // The margi tail goes in right behind the iteration count the previous run
  // converged at (steady state: 2 of 2), gated on the device: if the LM needs
  // more, that copy runs as no-ops and the caller enqueues it again after the
  // last iteration. So the tail starts as soon as the LM ends instead of one
  // host round trip later.
  int enq = 1, done_iters = 0, tail_at = 0;  // iterations enqueued so far / ahead of the speculative tail
  if (pre > 0) {
    enq = pre;
    tail_at = pre;
  } else if (graph2) {
    const hipError_t e = hipGraphLaunch(ctx->g_ba2, s);
    if (e != hipSuccess) {
      ctx->err = std::string("hipGraphLaunch (LM iterations 0-1): ") + hipGetErrorString(e);
      return VG_E_HIP;
    }
    enq = 2;
  } else {
    iteration(0);
  }
  for (int k = 0; k < 10; k++) {
    if (enq == k + 1 && enq < 10 && enq < ctx->ba_last_iters) iteration(enq++);  // one ahead
    VG_HIP(hipGetLastError());
    VG_TRY(xerr);
    if (k == 0 && before_first_wait) VG_TRY(before_first_wait());
    if (spec_tail && !tail_at && enq >= ctx->ba_last_iters) {
      bool queued = false;
      VG_TRY(spec_tail(&queued));
      if (queued) tail_at = enq;
    }
    // the outcome is read later (ba_resolve): the tail is queued, every
    // further iteration is a replay of the same graph
    if (pending && tail_at > 0 && graph && !ctx->ba_no_defer) {
      ctx->ba_loop.seq0 = seq0;
      ctx->ba_loop.enq = enq;
      ctx->ba_loop.tail_at = tail_at;
      ctx->ba_loop.k = k;
      ctx->ba_loop.active = true;
      *pending = true;
      *iters = -1;
      if (tail_ok) *tail_ok = true;
      return VG_OK;
    }
    VG_TRY(pub_wait(ctx, &ctx->h_pub->seq_ba, seq0 + k, "k_ba_control"));
    // The flags may already come from iteration k+1 (queued ahead, possibly
    // finished by now): decide on iteration k's outcome only — done at or
    // before it (the device stops counting once done) — so the number of
    // iterations enqueued never depends on timing (sharded mode: every
    // enqueue is an exchange, all ranks must enqueue alike)
    const int bw = __atomic_load_n(&ctx->h_pub->ba_word, __ATOMIC_ACQUIRE);
    done_iters = bw >> 1;
    if ((bw & 1) && done_iters <= k + 1) break;
    done_iters = k + 1;
    if (enq == k + 1 && enq < 10) iteration(enq++);  // not queued ahead: now
  }
  if (tail_ok) *tail_ok = tail_at > 0 && done_iters <= tail_at;  // the gate opened for that copy
  *iters = done_iters;
  ctx->ba_last_iters = done_iters > 0 ? done_iters : 2;
  if (solve_ev)  // k_ba_solve of the executed iterations only (the bench's roofline)
    for (int it = 0; it < done_iters && it < 10; it++) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ctx->solve_ev[it][0], ctx->solve_ev[it][1]) == hipSuccess) {
        ctx->prof_ms[kProfBaSolve] += ms;
        ctx->prof_n[kProfBaSolve] += 1;
      }
    }
  (void)g_dummy;
  return VG_OK;
}

// The rest of ba_run's loop for a run it left pending: the same decisions on
// the same flags (iteration k's own outcome), every iteration a replay of the
// one-iteration graph.
int ba_resolve(vg_ctx* ctx, bool block, bool* finished, int* iters, bool* tail_ok) {
  BaLoop& L = ctx->ba_loop;
  *finished = true;
  if (!L.active) return VG_OK;
  hipStream_t s = ctx->stream;
  auto launch = [&]() -> int {
    const hipError_t e = hipGraphLaunch(ctx->g_ba, s);
    if (e != hipSuccess) {
      L.active = false;
      ctx->err = std::string("hipGraphLaunch (LM iteration): ") + hipGetErrorString(e);
      return VG_E_HIP;
    }
    L.enq++;
    return VG_OK;
  };
  int done_iters = 0;
  for (int k = L.k; k < 10; k++) {
    L.k = k;
    if (L.enq == k + 1 && L.enq < 10 && L.enq < ctx->ba_last_iters) VG_TRY(launch());  // one ahead
    if (!block && __atomic_load_n(&ctx->h_pub->seq_ba, __ATOMIC_ACQUIRE) < L.seq0 + k) {
      *finished = false;
      return VG_OK;
    }
    const int r = pub_wait(ctx, &ctx->h_pub->seq_ba, L.seq0 + k, "k_ba_control");
    if (r != VG_OK) {
      L.active = false;
      return r;
    }
    const int bw = __atomic_load_n(&ctx->h_pub->ba_word, __ATOMIC_ACQUIRE);
    done_iters = bw >> 1;
    if ((bw & 1) && done_iters <= k + 1) break;
    done_iters = k + 1;
    if (L.enq == k + 1 && L.enq < 10) VG_TRY(launch());  // not queued ahead: now
  }
  L.active = false;
  *tail_ok = L.tail_at > 0 && done_iters <= L.tail_at;
  *iters = done_iters;
  ctx->ba_last_iters = done_iters > 0 ? done_iters : 2;
  return VG_OK;
}

// ---- LiDAR factor passes for a host-driven LM (the initialisation's
// LI_BA_OptimizerGravity, optimizers.cpp:640-743): the same kernels, no IMU
// factors (the host evaluates those), synchronous.
// poses: W x kX frame states (R 9, p 3, v 3, bg 3, ba 3, g 3) by ord.
// out (Hessian pass): the 6W x 6W LiDAR Hessian as packed lower rows, then the
// 6W gradient, then the residual (acc_evaluate2 summed over the factors);
// out (residual pass): the residual (evaluate_only_residual, which also stores
// each factor's eigen system and merged cluster at these poses, as the
// reference's does).
int ba_lidar_pass(vg_ctx* ctx, bool hessian, const double* poses, const int* mp_ring, double* out) {
  const int W = ctx->cfg.win_size;
  hipStream_t s = ctx->stream;
  BaDev d = carve(ctx);
  const int L = 6 * W, nout = L * (L + 1) / 2 + L + 1;
  BaState bs;
  memset(&bs, 0, sizeof(bs));
  bs.calc_hess = 1;
  int ring[kMaxW];
  for (int i = 0; i < kMaxW; i++) ring[i] = i < W ? mp_ring[i] : 0;
  double* h = ctx->h_stage;  // pinned staging
  memcpy(h, poses, (size_t)W * kX * sizeof(double));
  memcpy(h + W * kX, &bs, sizeof(bs));
  memcpy(h + W * kX + 8, ring, sizeof(ring));
  double* target = hessian ? d.xs : d.xt;
  VG_HIP(hipMemcpyAsync(target, h, (size_t)W * kX * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.st, h + W * kX, sizeof(bs), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.mpring, h + W * kX + 8, sizeof(ring), hipMemcpyHostToDevice, s));
  const int* nfp = ctx->map.counters + kCntFactors;
  if (hessian) {
    const int G = std::min(kHessGridMax, ctx->ba.cap_f / hess_chunk(W) + 1);
    k_ba_hess<<<G, kHessThreads, hess_lds_bytes(W), s>>>(nfp, W, ctx->ba.fac_node, ctx->ba.fac_eig, ctx->ba.fac_pcr,
                                                        ctx->map.pcrs, d.mpring, d.xs, d.part, d.st, G, 0, d.imurec,
                                                        &ctx->st->imu_head, d.bias, d.imuout, nullptr);
    k_ba_hfinal<<<(nout * 8 + 255) / 256, 256, 0, s>>>(nfp, hess_chunk(W), nout, d.part, d.hl, d.st, XchgArg{});
    VG_HIP(hipGetLastError());
    VG_HIP(hipMemcpyAsync(h, d.hl, nout * sizeof(double), hipMemcpyDeviceToHost, s));
    VG_HIP(hipStreamSynchronize(s));
    memcpy(out, h, nout * sizeof(double));
    return VG_OK;
  }
  const int nrb = kResidBlocks;
  k_ba_resid<<<nrb, 256, 0, s>>>(nfp, W, ctx->ba.fac_node, ctx->map.pcr_fix, ctx->map.pcrs, d.mpring, d.xt,
                                 ctx->ba.fac_eig, ctx->ba.fac_pcr, d.rpart, d.st, nrb, 0, d.imurec, &ctx->st->imu_head,
                                 d.bias, d.imures, CtlArg{});
  VG_HIP(hipGetLastError());
  VG_HIP(hipMemcpyAsync(h, d.rpart, nrb * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  double r = 0.0;
  for (int b = 0; b < nrb; b++) r += h[b];
  *out = r;
  return VG_OK;
}

// Test-only (vgx_ba_solve): k_ba_solve on a given m x m symmetric system
// (m = 15W - 15, row-major A, right-hand side b) in identity pivot order;
// x = the solution. Runs the kernel exactly as an LM iteration does (the
// trial-state tail writes the context's scratch trial states and bias
// records, so use a context that is not stepped afterwards).
int ba_solve_test(vg_ctx* ctx, const double* A, const double* b, double* x) {
  const int W = ctx->cfg.win_size, n = 15 * W, m = n - 15;
  const int NB = (m + kTile - 1) / kTile, N = NB * kTile, ntile = NB * (NB + 1) / 2;
  hipStream_t s = ctx->stream;
  BaDev d = carve(ctx);
  std::vector<double> img((size_t)ntile * 256), bv(N, 0.0), dv(n, 1.0), jv(n, 0.0);
  std::vector<int> ipv(N, 0);
  for (int I = 0; I < NB; I++)
    for (int J = 0; J <= I; J++)
      for (int r = 0; r < 16; r++)
        for (int c = 0; c < 16; c++) {
          const int R = I * 16 + r, C = J * 16 + c;
          const double v = (R < m && C < m) ? A[(size_t)R * m + C] : (R == C ? 1.0 : 0.0);
          img[(size_t)(I * (I + 1) / 2 + J) * 256 + r * 16 + (c ^ r)] = v;
        }
  for (int t = 0; t < m; t++) {
    bv[t] = b[t];
    ipv[t] = 15 + t;
  }
  BaState bs;
  memset(&bs, 0, sizeof(bs));
  VG_HIP(hipMemcpyAsync(d.timg, img.data(), img.size() * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.bvec, bv.data(), N * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.dvec, dv.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.jvec, jv.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.ipg, ipv.data(), N * sizeof(int), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(d.st, &bs, sizeof(bs), hipMemcpyHostToDevice, s));
  VG_HIP(hipStreamSynchronize(s));
  k_ba_solve<<<1, 1024, solve_lds_bytes(W), s>>>(W, W - 1, d.timg, d.bvec, d.dvec, d.jvec, d.ipg, d.xs, d.xt, d.bias,
                                                 d.dxi, d.st, nullptr);
  VG_HIP(hipGetLastError());
  std::vector<double> out(n);
  VG_HIP(hipMemcpyAsync(out.data(), d.dxi, n * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  for (int t = 0; t < m; t++) x[t] = out[15 + t];
  return VG_OK;
}

// the factors' eigenvectors (column 0 = the plane normal) and count, host copy
int ba_factor_normals(vg_ctx* ctx, std::vector<double>& normals) {
  hipStream_t s = ctx->stream;  // stream-ordered: the context stream is non-blocking
  VG_HIP(hipMemcpyAsync(ctx->h_pinned, ctx->map.counters + kCntFactors, sizeof(int), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  const int nf = ctx->h_pinned[0];
  std::vector<double> e((size_t)nf * 12);
  if (nf > 0) VG_HIP(hipMemcpyAsync(e.data(), ctx->ba.fac_eig, e.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  normals.resize((size_t)nf * 3);
  for (int a = 0; a < nf; a++)
    for (int k = 0; k < 3; k++) normals[(size_t)a * 3 + k] = e[(size_t)a * 12 + 3 + k * 3];  // U(k, 0), row-major
  return VG_OK;
}

}  // namespace vg

#ifdef VG_PROBE
VG_PROBE_READER(vg_probe_read)
#endif
