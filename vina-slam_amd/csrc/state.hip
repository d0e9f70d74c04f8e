// state.hip — the device-resident estimator state machine.
//
// The reference keeps x_curr / x_prop / x_buf as host objects and runs the
// IEKF update (odometry.cpp:192-230) on the odometry thread between point
// loops. Here that state lives in HBM (DState) and every step that reads or
// writes it is a kernel on the context stream:
//   k_scan_begin     x_curr after IMU propagation (kernel argument), x_prop =
//                    x_curr, cov_inv = cov^-1 (odometry.cpp:67, 82)
//   k_iekf_update    one workgroup per IEKF iteration: ordered sum of the
//                    k_iekf block partials, K_1 = (H_T_H + cov_inv)^-1 by
//                    Gauss-Jordan with partial pivoting (Eigen's fixed-size
//                    inverse stand-in), G, the ⊞ update, the convergence /
//                    rematch rule and, on the last iteration, cov = (I-G) cov
//                    and the degeneracy test (odometry.cpp:192-254)
//   k_push_state     x_buf.push_back(x_curr) and a fresh IMU_PRE bias record
//                    (local_mapping.cpp:434-441)
//   k_make_win       the window view (poses by ord, mp ring, point counts) the
//                    map kernels read; optionally x_curr.R/p <- x_buf.back()
//                    first (local_mapping.cpp:501-502)
//   k_slide_state    x_buf / imu_pre_buf slide by one (local_mapping.cpp:536-546)
//   k_publish_*      copies to the host-mapped Pub block, closed by a sequence
//                    flag (system-scope release), so the host reads results
//                    without draining the stream
// The fp64 expression trees are the host code's (vg_la.h, -ffp-contract=off),
// so the device update is the same arithmetic the host update was.
#include "vg_dev.h"

namespace vg {

struct XcArg {
  double x[kXC];
};

__device__ __forceinline__ void pub_store(double* dst, double v) {
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void pub_store(int* dst, int v) {
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void pub_flag(int* dst, int v) {
  __threadfence_system();
  __hip_atomic_store(dst, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Gauss-Jordan inverse of the 15 x 15 block a[0..15)[0..15) of the augmented
// 15 x 30 LDS matrix (right half = identity on entry, inverse on exit), by the
// whole workgroup. Pivot rule and every update expression are vg_la.h
// inverse<15>'s: first max |a(r,c)| for r >= c, row swap, scale the pivot row
// by 1/a(c,c), then a(r,j) -= f a(c,j) for rows with f != 0.
__device__ void gj_inverse15(double (*a)[30]) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int c = 0; c < 15; c++) {
    int p = c;
    double best = fabs(a[c][c]);
    for (int r = c + 1; r < 15; r++)
      if (fabs(a[r][c]) > best) {
        best = fabs(a[r][c]);
        p = r;
      }
    if (p != c && tid < 30) {
      const double t = a[c][tid];
      a[c][tid] = a[p][tid];
      a[p][tid] = t;
    }
    __syncthreads();
    const double inv = 1.0 / a[c][c];
    __syncthreads();
    if (tid < 30) a[c][tid] *= inv;
    __syncthreads();
    double f[2], pc[2];
    int e[2];
    for (int k = 0; k < 2; k++) {
      e[k] = tid + k * nt;
      f[k] = 0.0;
      pc[k] = 0.0;
      if (e[k] < 450) {
        const int r = e[k] / 30, j = e[k] % 30;
        f[k] = a[r][c];
        pc[k] = a[c][j];
      }
    }
    __syncthreads();
    for (int k = 0; k < 2; k++) {
      if (e[k] >= 450) continue;
      const int r = e[k] / 30, j = e[k] % 30;
      if (r == c || f[k] == 0.0) continue;
      a[r][j] -= f[k] * pc[k];
    }
    __syncthreads();
  }
}

// x_curr after propagation; x_prop; cov_inv; IEKF flags
__global__ void __launch_bounds__(256) k_scan_begin(XcArg xa, DState* __restrict__ st) {
  __shared__ double a[15][30];
  const int tid = threadIdx.x;
  for (int t = tid; t < kXC; t += blockDim.x) {
    st->xc[t] = xa.x[t];
    st->xp[t] = xa.x[t];
  }
  for (int e = tid; e < 450; e += blockDim.x) {
    const int r = e / 30, j = e % 30;
    a[r][j] = j < 15 ? xa.x[kXS + r * 15 + j] : ((j - 15 == r) ? 1.0 : 0.0);
  }
  __syncthreads();
  gj_inverse15(a);
  for (int e = tid; e < 225; e += blockDim.x) st->cinv[e] = a[e / 15][15 + e % 15];
  if (tid == 0) {
    st->it = 0;
    st->rematch = 0;
    st->done = 0;
    st->iters = 0;
    st->degenerate = 0;
    for (int k = 0; k < 4; k++) st->matches[k] = 0;
  }
}

constexpr int kIekfVals = 34;

// One IEKF update (odometry.cpp:192-230) after the k_iekf point loop of
// iteration `it` wrote nb block partials.
__global__ void __launch_bounds__(256) k_iekf_update(int nb, const double* __restrict__ partials,
                                                     DState* __restrict__ st, int it) {
  if (st->done) return;
  __shared__ double red[256][kIekfVals + 1];
  __shared__ double a[15][30];
  __shared__ double o[kIekfVals], K6[15][6], G6[15][6], vec[15], sol[15], IG[15][15];
  __shared__ int fin;
  const int tid = threadIdx.x;
  {  // ordered two-level sum of the block partials (deterministic)
    double acc[kIekfVals];
    for (int j = 0; j < kIekfVals; j++) acc[j] = 0.0;
    for (int b = tid; b < nb; b += 256)
      for (int j = 0; j < kIekfVals; j++) acc[j] += partials[(size_t)b * kIekfVals + j];
    for (int j = 0; j < kIekfVals; j++) red[tid][j] = acc[j];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (tid < w)
        for (int j = 0; j < kIekfVals; j++) red[tid][j] += red[tid + w][j];
      __syncthreads();
    }
    if (tid < kIekfVals) o[tid] = red[0][tid];
    __syncthreads();
  }
  // HTH (upper 21 -> full), HTz, nnt; A = H_T_H + cov_inv (H_T_H zero outside 6x6)
  for (int e = tid; e < 450; e += blockDim.x) {
    const int r = e / 30, j = e % 30;
    double v;
    if (j < 15) {
      double h = 0.0;
      if (r < 6 && j < 6) {
        const int lo = r < j ? r : j, hi = r < j ? j : r;
        h = o[lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
      }
      v = h + st->cinv[r * 15 + j];
    } else {
      v = (j - 15 == r) ? 1.0 : 0.0;
    }
    a[r][j] = v;
  }
  if (tid == 0) {
    st->iters = it + 1;
    st->matches[it] = (int)o[33];
    st->nnt[0] = o[27];
    st->nnt[1] = o[28];
    st->nnt[2] = o[29];
    st->nnt[3] = o[30];
    st->nnt[4] = o[31];
    st->nnt[5] = o[32];
  }
  __syncthreads();
  gj_inverse15(a);
  // K6 = K_1(:, 0:6); G6 = K6 * HTH (mul: s = x0 y0; s += ...)
  if (tid < 90) K6[tid / 6][tid % 6] = a[tid / 6][15 + tid % 6];
  __syncthreads();
  if (tid < 90) {
    const int r = tid / 6, c = tid % 6;
    auto hth = [&](int i, int j) {
      const int lo = i < j ? i : j, hi = i < j ? j : i;
      return o[lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
    };
    double s = K6[r][0] * hth(0, c);
    for (int k = 1; k < 6; k++) s += K6[r][k] * hth(k, c);
    G6[r][c] = s;
    st->G6[r * 6 + c] = s;
  }
  if (tid == 64) {  // vec = x_prop ⊟ x_curr (IMUST::operator-, types.hpp:80-86)
    const double* xp = st->xp;
    const double* xc = st->xc;
    const V3 rr = Log(mul(tr(ld_m3(xc)), ld_m3(xp)));
    for (int k = 0; k < 3; k++) {
      vec[k] = rr[k];
      vec[3 + k] = xp[9 + k] - xc[9 + k];
      vec[6 + k] = xp[12 + k] - xc[12 + k];
      vec[9 + k] = xp[15 + k] - xc[15 + k];
      vec[12 + k] = xp[18 + k] - xc[18 + k];
    }
  }
  __syncthreads();
  if (tid < 15) {  // sol = (K6 HTz + vec) - G6 v6
    double s1 = K6[tid][0] * o[21];
    for (int k = 1; k < 6; k++) s1 += K6[tid][k] * o[21 + k];
    double s2 = G6[tid][0] * vec[0];
    for (int k = 1; k < 6; k++) s2 += G6[tid][k] * vec[k];
    sol[tid] = (s1 + vec[tid]) - s2;
  }
  __syncthreads();
  if (tid == 0) {  // x_curr ⊞= sol (types.hpp:67-78); convergence / rematch (odometry.cpp:205-227)
    double* xc = st->xc;
    const M3 Rn = mul(ld_m3(xc), Exp(v3(sol[0], sol[1], sol[2])));
    for (int k = 0; k < 9; k++) xc[k] = Rn[k];
    for (int k = 0; k < 3; k++) {
      xc[9 + k] += sol[3 + k];
      xc[12 + k] += sol[6 + k];
      xc[15 + k] += sol[9 + k];
      xc[18 + k] += sol[12 + k];
    }
    const double rot_add = norm3(v3(sol[0], sol[1], sol[2])), tra_add = norm3(v3(sol[3], sol[4], sol[5]));
    const bool conv = (rot_add * 57.3 < 0.01) && (tra_add * 100 < 0.015);
    int rm = st->rematch;
    if (conv || ((rm == 0) && (it == 4 - 2))) rm++;
    st->rematch = rm;
    fin = (rm >= 2 || it == 4 - 1) ? 1 : 0;
  }
  __syncthreads();
  if (!fin) return;
  // cov = (I - G) cov (G zero outside columns 0..5)
  for (int e = tid; e < 225; e += blockDim.x) {
    const int r = e / 15, c = e % 15;
    IG[r][c] = ((r == c) ? 1.0 : 0.0) - (c < 6 ? G6[r][c] : 0.0);
  }
  __syncthreads();
  double cv = 0.0;
  if (tid < 225) {
    const int r = tid / 15, c = tid % 15;
    const double* cov = st->xc + kXS;
    double s = IG[r][0] * cov[c];
    for (int k = 1; k < 15; k++) s += IG[r][k] * cov[k * 15 + c];
    cv = s;
  }
  __syncthreads();
  if (tid < 225) st->xc[kXS + tid] = cv;
  if (tid == 0) {
    M3 nn;
    nn(0, 0) = st->nnt[0];
    nn(0, 1) = nn(1, 0) = st->nnt[1];
    nn(0, 2) = nn(2, 0) = st->nnt[2];
    nn(1, 1) = st->nnt[3];
    nn(1, 2) = nn(2, 1) = st->nnt[4];
    nn(2, 2) = st->nnt[5];
    V3 ev;
    M3 U;
    eig3(nn, ev, U);
    st->degenerate = (ev[0] < 14) ? 1 : 0;  // odometry.cpp:244-254
    for (int k = 0; k < 12; k++) st->traj[k] = st->xc[k];
    st->done = 1;
  }
}

// x_buf.push_back(x_curr) at ord; a new IMU_PRE (when win_count > 1) starts
// with zero bias deltas (imu_preintegration.cpp:10-29)
__global__ void k_push_state(DState* __restrict__ st, int ord, int new_imu) {
  const int t = threadIdx.x;
  if (t < kXS) st->xs[ord * kXS + t] = st->xc[t];
  if (new_imu >= 0 && t < 12) st->bias[new_imu * 12 + t] = 0.0;
}

// window view for the map kernels: poses by ord, ring, per-ord counts / slots
__global__ void k_make_win(DState* __restrict__ st, WinArg wa, WinD* __restrict__ win, int* __restrict__ nper,
                           int* __restrict__ slot_of) {
  const int t = threadIdx.x;
  const int wc = wa.win_count;
  if (wa.set_xc && wc > 0) {
    if (t < 12) st->xc[t] = st->xs[(wc - 1) * kXS + t];
    __syncthreads();
  }
  for (int e = t; e < kMaxWin * 12; e += blockDim.x) {
    const int i = e / 12, k = e % 12;
    const double v = i < wc ? st->xs[i * kXS + k] : 0.0;
    if (k < 9) win->R[i][k] = v;
    else win->p[i][k - 9] = v;
  }
  if (t < kMaxWin) {
    win->mp[t] = wa.mp[t];
    nper[t] = t < wc ? wa.nper[t] : 0;
    slot_of[t] = wa.mp[t];
  }
  if (t == 0) {
    win->win_count = wc;
    win->pad = 0;
  }
}

// slide the window states and the IMU bias records by one
__global__ void k_slide_state(DState* __restrict__ st, int win_count, int nimu) {
  const int t = threadIdx.x;
  double v[4], b[2];
  for (int k = 0; k < 4; k++) {
    const int e = t + k * blockDim.x;
    v[k] = (e < (win_count - 1) * kXS) ? st->xs[kXS + e] : 0.0;
  }
  for (int k = 0; k < 2; k++) {
    const int e = t + k * blockDim.x;
    b[k] = (e < (nimu - 1) * 12) ? st->bias[12 + e] : 0.0;
  }
  __syncthreads();
  for (int k = 0; k < 4; k++) {
    const int e = t + k * blockDim.x;
    if (e < (win_count - 1) * kXS) st->xs[e] = v[k];
  }
  for (int k = 0; k < 2; k++) {
    const int e = t + k * blockDim.x;
    if (e < (nimu - 1) * 12) st->bias[e] = b[k];
  }
}

// P1: x_curr, the post-IEKF pose, window states, IEKF / BA summary
__global__ void k_publish_state(const DState* __restrict__ st, int win_count, int ba_iters_valid,
                                const int* __restrict__ ba_iters, Pub* __restrict__ pub, int seq) {
  const int t = threadIdx.x;
  for (int e = t; e < kXC; e += blockDim.x) pub_store(&pub->xc[e], st->xc[e]);
  for (int e = t; e < 12; e += blockDim.x) pub_store(&pub->traj[e], st->traj[e]);
  for (int e = t; e < win_count * kXS; e += blockDim.x) pub_store(&pub->xs[e], st->xs[e]);
  if (t == 0) {
    pub_store(&pub->iekf_iters, st->iters);
    pub_store(&pub->degenerate, st->degenerate);
    for (int k = 0; k < 4; k++) pub_store(&pub->matches[k], st->matches[k]);
    pub_store(&pub->ba_iters1, ba_iters_valid ? *ba_iters : 0);
  }
  __syncthreads();
  if (t == 0) pub_flag(&pub->seq1, seq);
}

// P2: map counters at the end of the scan
__global__ void k_publish_counters(const int* __restrict__ counters, Pub* __restrict__ pub, int seq) {
  const int t = threadIdx.x;
  if (t < kCntN) pub_store(&pub->counters[t], counters[t]);
  __syncthreads();
  if (t == 0) pub_flag(&pub->seq2, seq);
}

// downsample result (n_out, range error) -> host
__global__ void k_publish_ds(const int* __restrict__ flags, Pub* __restrict__ pub, int seq) {
  if (threadIdx.x == 0) {
    pub_store(&pub->ds_err, flags[0]);
    pub_store(&pub->n_ds, flags[1]);
    pub_flag(&pub->seq_ds, seq);
  }
}

// ---- host wrappers ----
int state_alloc(vg_ctx* ctx) {
  ctx->st = ctx->arena.take<DState>(1);
  if (!ctx->st) {
    ctx->err = "arena exhausted (state)";
    return VG_E_CAPACITY;
  }
  return VG_OK;
}

int state_scan_begin(vg_ctx* ctx, const double* xc249) {
  XcArg a;
  memcpy(a.x, xc249, sizeof(a.x));
  k_scan_begin<<<1, 256, 0, ctx->stream>>>(a, ctx->st);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_iekf_update(vg_ctx* ctx, int nb, const double* partials, int it) {
  k_iekf_update<<<1, 256, 0, ctx->stream>>>(nb, partials, ctx->st, it);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_push(vg_ctx* ctx, int ord, int new_imu) {
  k_push_state<<<1, 64, 0, ctx->stream>>>(ctx->st, ord, new_imu);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_make_win(vg_ctx* ctx, const WinArg& wa, WinD* dwin, int* dnper, int* dslot) {
  k_make_win<<<1, 256, 0, ctx->stream>>>(ctx->st, wa, dwin, dnper, dslot);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_slide(vg_ctx* ctx, int win_count, int nimu) {
  if (win_count * kXS > 4 * 256 || nimu * 12 > 2 * 256) {
    ctx->err = "state_slide: window too large";
    return VG_E_ARG;
  }
  k_slide_state<<<1, 256, 0, ctx->stream>>>(ctx->st, win_count, nimu);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_publish(vg_ctx* ctx, int win_count, const int* ba_iters_dev, int seq) {
  k_publish_state<<<1, 256, 0, ctx->stream>>>(ctx->st, win_count, ba_iters_dev != nullptr, ba_iters_dev, ctx->d_pub,
                                              seq);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_publish_counters(vg_ctx* ctx, int seq) {
  k_publish_counters<<<1, 64, 0, ctx->stream>>>(ctx->map.counters, ctx->d_pub, seq);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_publish_ds(vg_ctx* ctx, int seq) {
  k_publish_ds<<<1, 64, 0, ctx->stream>>>(ctx->ds.flags, ctx->d_pub, seq);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

}  // namespace vg
