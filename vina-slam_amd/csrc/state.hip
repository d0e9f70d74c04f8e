// state.hip — the device-resident estimator state machine.
//
// The reference keeps x_curr / x_prop / x_buf as host objects and runs the
// IEKF update (odometry.cpp:192-230) on the odometry thread between point
// loops. Here that state lives in HBM (DState) and every step that reads or
// writes it is a kernel on the context stream:
//   k_scan_begin     x_curr after IMU propagation (kernel argument), x_prop =
//                    x_curr (odometry.cpp:67)
//   iekf_update_block (vg_iekf.h) — run by the last k_iekf workgroup of each
//                    IEKF iteration: ordered sum of the block partials,
//                    K_1 = (H_T_H + cov_inv)^-1, G, the ⊞ update, the
//                    convergence / rematch rule and, on the last iteration,
//                    cov = (I-G) cov and the degeneracy test (odometry.cpp:192-254)
//   k_push_state     x_buf.push_back(x_curr) and a fresh IMU_PRE bias record
//                    (local_mapping.cpp:434-441)
//   make_win_block   (vg_dev.h) the window view (poses by ord, mp ring, point
//                    counts) the map kernels read; optionally x_curr.R/p <-
//                    x_buf.back() first (local_mapping.cpp:501-502): run by
//                    k_make_win_recut_begin and by k_margi_leaf's workgroup 0
//   k_slide_state    x_buf / imu_pre_buf slide by one (local_mapping.cpp:536-546)
//   k_publish_*      copies to the host-mapped Pub block, closed by a sequence
//                    flag (system-scope release), so the host reads results
//                    without draining the stream
// The fp64 expression trees are the host code's (vg_la.h, -ffp-contract=off),
// so the device update is the same arithmetic the host update was.
#include <cstddef>

#include "vg_iekf.h"

namespace vg {

struct XcArg {
  double x[kXC];
};

// x_curr after propagation; x_prop; cov_inv; IEKF flags; the scan the IEKF
// reads (set_scan: one launch for both)
__global__ void __launch_bounds__(256) k_scan_begin(XcArg xa, DState* __restrict__ st, const float* x, const float* y,
                                                    const float* z, int n, int set_scan) {
  const int tid = threadIdx.x;
  if (set_scan && tid == 64) {
    st->sx = x;
    st->sy = y;
    st->sz = z;
    st->sn = n;
  }
  for (int t = tid; t < kXC; t += blockDim.x) {
    st->xc[t] = xa.x[t];
    st->xp[t] = xa.x[t];
  }
  if (tid == 0) {
    st->it = 0;
    st->rematch = 0;
    st->done = 0;
    st->iters = 0;
    st->degenerate = 0;
    st->ticket = 0;
    for (int k = 0; k < 4; k++) st->matches[k] = 0;
    for (int k = 0; k < 4; k++) st->planes[k] = 0;
    st->iekf_pts = 0;
    if (st->clk.on) {  // this scan's k_iekf clock slots (KClock)
      const int sc = st->clk.scan + 1;
      st->clk.scan = sc;
      for (int k = 0; k < 4; k++) st->clk.exec[(sc * 4 + k) & (kClkRing - 1)] = 0;
    }
  }
}

// IMUEKF::process's state / covariance propagation (imu_ekf.cpp:13-86, the
// host's propagate() in pipeline.cpp, same expression trees) from the device's
// x_curr, then the scan opening (k_scan_begin). One workgroup: the per-sample
// rotations (Exp, the sin / cos) in parallel, the rotation / velocity /
// position chain on one lane in registers (inputs loaded a step ahead), the F
// / noise blocks of each sample in parallel, then cov <- F cov F^T + Q sample
// by sample, one lane per entry, each sum in ascending column order over F's
// non-zeros (the host's sandwich()), one wave per row (column) group so that
// every wave runs one row shape. Round 4's forms: the chain on one lane with
// per-lane index arrays for F's rows 54 us (11 chain, 37 covariance); the chain
// on wave 0 by shuffles and 256 lanes of mixed shapes 32 us (8.3 chain, 16.4
// covariance, scripts/probe_prop.py).
// Hand-offs inside the kernel (the split IEKF stream, pipeline.cpp): the
// per-sample rotations need only the biases, final since the previous scan's
// IEKF, so they run before the margi head's flag (head_flag >= head_target:
// x_curr.R/p <- x_buf.back() stored); the kernel then waits for the margi
// leaves' plane updates (leaf_flag >= leaf_target) before it ends, so the
// IEKF behind it needs no polling kernel and no launch gap of its own. A wait
// that times out (~1 s) sets error bit 64 and closes the IEKF (st->done).
__device__ __forceinline__ bool flag_wait(const unsigned* flag, unsigned target) {
  for (long it = 0; (int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0; it++) {
    __builtin_amdgcn_s_sleep(2);
    if (it > (1l << 24)) return false;
  }
  return true;
}
constexpr int kPropThreads = 320;  // five waves: one 3-row (3-column) group of the covariance each
__global__ void __launch_bounds__(kPropThreads) k_scan_prop(PropArg arg, DState* __restrict__ st, const float* x,
                                                            const float* y, const float* z, int n, int set_scan,
                                                            const unsigned* __restrict__ head_flag, unsigned head_target,
                                                            const unsigned* __restrict__ leaf_flag, unsigned leaf_target,
                                                            int* __restrict__ err) {
  // the arguments once into LDS, by all lanes (the kernel-argument block is
  // host memory: the serial chain below would pay a round trip per sample)
  __shared__ PropArg a;
  {
    const int words = (int)((offsetof(PropArg, imu) + (size_t)(arg.n > 0 ? arg.n : 0) * 7 * sizeof(double)) / 8);
    const double* src = reinterpret_cast<const double*>(&arg);
    double* dst = reinterpret_cast<double*>(&a);
    for (int i = threadIdx.x; i < words; i += blockDim.x) dst[i] = src[i];
  }
  VG_PROBE_BEGIN();
  __syncthreads();
  VG_PROBE_MARK(1);
  __shared__ double sExp[kPropMax][9], sF00[kPropMax][9], sRi[kPropMax][9], sAsk[kPropMax][9];
  __shared__ double sF60[kPropMax][9], sF612[kPropMax][9], sCw[kPropMax][9], sDt[kPropMax];
  __shared__ double sAa[kPropMax][3], sAng[kPropMax][3];
  __shared__ int sOk[kPropMax];
  __shared__ double C[225], A[225];
  const int tid = threadIdx.x;
  const double* xc = st->xc;
  const V3 bg = v3(xc[15], xc[16], xc[17]), ba = v3(xc[18], xc[19], xc[20]);
  const int ns = a.n > 1 ? a.n - 1 : 0;  // sample pairs
  // 1. per pair: skip rule, angvel, acc_avr, dt, Exp(angvel, dt), F00 = Exp(angvel, -dt), hat(acc_avr)
  if (tid < ns) {
    const double* h = &a.imu[7 * tid];
    const double* t = &a.imu[7 * (tid + 1)];
    const bool ok = !(h[0] < a.last_end);
    V3 angvel, acc_avr;
    for (int j = 0; j < 3; j++) {
      angvel[j] = 0.5 * (h[1 + j] + t[1 + j]);
      acc_avr[j] = 0.5 * (h[4 + j] + t[4 + j]);
    }
    angvel = sub(angvel, bg);
    acc_avr = sub(scl(acc_avr, a.sg), ba);
    double cur = h[0];
    if (cur < a.last_end) cur = a.last_end;
    const double dt = t[0] - cur;
    const M3 e = Exp(angvel, dt), f = Exp(angvel, -dt), k = hat(acc_avr);
    for (int q = 0; q < 9; q++) {
      sExp[tid][q] = e[q];
      sF00[tid][q] = f[q];
      sAsk[tid][q] = k[q];
    }
    for (int q = 0; q < 3; q++) {
      sAa[tid][q] = acc_avr[q];
      sAng[tid][q] = angvel[q];
    }
    sDt[tid] = dt;
    sOk[tid] = ok ? 1 : 0;
  }
  VG_PROBE_MARK(2);
  if (head_flag) {  // x_curr.R/p of the previous scan's margi head
    __shared__ int s_late;
    if (tid == 0) s_late = flag_wait(head_flag, head_target) ? 0 : 1;
    __syncthreads();
    if (s_late) {
      if (tid == 0) {
        atomicOr(err, 64);
        st->done = 1;
      }
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  VG_PROBE_MARK(7);
  // 2. the rotation / velocity / position chain on one lane, everything in
  // registers, the next pair's inputs loaded one step ahead (the host's mul /
  // add / scl trees term for term; the wave-0 form with one entry per lane
  // paid a shuffle round trip per dependent step: 8.3 us)
  if (tid < 225) C[tid] = xc[kXS + tid];  // (cov: final since the previous scan's IEKF)
  if (tid == 0) {
    double R[9], p[3], v[3], g[3];
    for (int q = 0; q < 9; q++) R[q] = xc[q];
    for (int j = 0; j < 3; j++) {
      p[j] = xc[9 + j];
      v[j] = xc[12 + j];
      g[j] = xc[21 + j];
    }
    double acc[3] = {0.0, 0.0, 0.0}, ang[3] = {0.0, 0.0, 0.0};
    double nE[9], nA[3], nG[3], ndt = 0.0;
    int nok = 0;
    auto load = [&](int k) {
      for (int q = 0; q < 9; q++) nE[q] = sExp[k][q];
      for (int q = 0; q < 3; q++) {
        nA[q] = sAa[k][q];
        nG[q] = sAng[k][q];
      }
      ndt = sDt[k];
      nok = sOk[k];
    };
    if (ns > 0) load(0);
    for (int k = 0; k < ns; k++) {
      double E[9], aa[3], an[3];
      for (int q = 0; q < 9; q++) E[q] = nE[q];
      for (int q = 0; q < 3; q++) {
        aa[q] = nA[q];
        an[q] = nG[q];
      }
      const double dt = ndt;
      const int ok = nok;
      if (k + 1 < ns) load(k + 1);
      if (!ok) continue;
      for (int i = 0; i < 3; i++) {  // acc_imu = R_imu acc_avr + g
        double t = R[3 * i] * aa[0];
        t += R[3 * i + 1] * aa[1];
        t += R[3 * i + 2] * aa[2];
        acc[i] = t + g[i];
      }
      for (int q = 0; q < 9; q++) sRi[k][q] = R[q];
      const double hdt2 = 0.5 * dt * dt;
      for (int j = 0; j < 3; j++) {
        p[j] = (p[j] + v[j] * dt) + acc[j] * hdt2;
        v[j] = v[j] + acc[j] * dt;
        ang[j] = an[j];
      }
      double Rn[9];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          double t = R[3 * i] * E[j];
          t += R[3 * i + 1] * E[3 + j];
          t += R[3 * i + 2] * E[6 + j];
          Rn[3 * i + j] = t;
        }
      for (int q = 0; q < 9; q++) R[q] = Rn[q];
    }
    if (a.n > 0) {  // imu_ekf.cpp:81-86
      M3 R_imu;
      for (int q = 0; q < 9; q++) R_imu[q] = R[q];
      const V3 pos = v3(p[0], p[1], p[2]), vel = v3(v[0], v[1], v[2]);
      const V3 acc_imu = v3(acc[0], acc[1], acc[2]), angvel = v3(ang[0], ang[1], ang[2]);
      const double tb = a.imu[7 * (a.n - 1)];
      const double note = a.end > tb ? 1.0 : -1.0;
      const double dt = note * (a.end - tb);
      const V3 vv = add(vel, scl(acc_imu, note * dt));
      const M3 Rr = mul(R_imu, Exp(scl(angvel, note), dt));
      const V3 pp = add(add(pos, scl(vel, note * dt)), scl(acc_imu, note * 0.5 * dt * dt));
      for (int q = 0; q < 9; q++) st->xc[q] = Rr[q];
      for (int j2 = 0; j2 < 3; j2++) {
        st->xc[9 + j2] = pp[j2];
        st->xc[12 + j2] = vv[j2];
      }
    }
  }
  __syncthreads();
  VG_PROBE_MARK(3);
  // 3. per pair: F60, F612 and the acceleration noise block
  if (tid < ns && sOk[tid]) {
    const M3 Ri = ld_m3(sRi[tid]);
    const double dt = sDt[tid];
    M3 ca = M3::Z();
    for (int j = 0; j < 3; j++) ca(j, j) = a.cov_acc;
    const M3 f60 = scl(mul(Ri, ld_m3(sAsk[tid])), -dt), f612 = scl(Ri, -dt);
    const M3 cw = scl(mul(mul(Ri, ca), tr(Ri)), dt * dt);
    for (int q = 0; q < 9; q++) {
      sF60[tid][q] = f60[q];
      sF612[tid][q] = f612[q];
      sCw[tid][q] = cw[q];
    }
  }
  __syncthreads();
  VG_PROBE_MARK(4);
  // 4. cov = F cov F^T + Q per pair, F's non-zero columns ascending (sandwich()),
  // F's four row shapes written out. Wave w takes rows 3w..3w+2 of F C, then
  // columns 3w..3w+2 of (F C) F^T: every lane of a wave runs the same shape
  // (the 256-lane form mixed all four shapes in each wave: 16.4 us)
  const int wv = tid >> 6, ln = tid & 63;
  const bool act = ln < 45;
  const int ai = 3 * wv + ln / 15, aj = ln % 15;  // phase A entry (row group wv)
  const int bi = ln % 15, bj = 3 * wv + ln / 15;  // phase B entry (column group wv)
  auto a_ent = [&](int k, int i, int j) -> double {  // (F C)(i, j)
    const double dt = sDt[k];
    if (i < 3) {
      double s = sF00[k][i * 3] * C[j];
      s += sF00[k][i * 3 + 1] * C[15 + j];
      s += sF00[k][i * 3 + 2] * C[30 + j];
      s += (-dt) * C[(9 + i) * 15 + j];
      return s;
    }
    if (i < 6) {
      double s = 1.0 * C[i * 15 + j];
      s += dt * C[(i + 3) * 15 + j];
      return s;
    }
    if (i < 9) {
      const int q = i - 6;
      double s = sF60[k][q * 3] * C[j];
      s += sF60[k][q * 3 + 1] * C[15 + j];
      s += sF60[k][q * 3 + 2] * C[30 + j];
      s += 1.0 * C[i * 15 + j];
      s += sF612[k][q * 3] * C[180 + j];
      s += sF612[k][q * 3 + 1] * C[195 + j];
      s += sF612[k][q * 3 + 2] * C[210 + j];
      return s;
    }
    return 1.0 * C[i * 15 + j];
  };
  auto o_ent = [&](int k, int i, int j) -> double {  // (A F^T)(i, j) + Q(i, j)
    const double dt = sDt[k];
    const double* Ai = &A[i * 15];
    double s;
    if (j < 3) {
      s = Ai[0] * sF00[k][j * 3];
      s += Ai[1] * sF00[k][j * 3 + 1];
      s += Ai[2] * sF00[k][j * 3 + 2];
      s += Ai[9 + j] * (-dt);
    } else if (j < 6) {
      s = Ai[j] * 1.0;
      s += Ai[j + 3] * dt;
    } else if (j < 9) {
      const int q = j - 6;
      s = Ai[0] * sF60[k][q * 3];
      s += Ai[1] * sF60[k][q * 3 + 1];
      s += Ai[2] * sF60[k][q * 3 + 2];
      s += Ai[j] * 1.0;
      s += Ai[12] * sF612[k][q * 3];
      s += Ai[13] * sF612[k][q * 3 + 1];
      s += Ai[14] * sF612[k][q * 3 + 2];
    } else {
      s = Ai[j] * 1.0;
    }
    double q = 0.0;
    if (i >= 6 && i < 9 && j >= 6 && j < 9) q = sCw[k][(i - 6) * 3 + (j - 6)];
    else if (i == j && i < 3) q = a.cov_gyr * dt * dt;
    else if (i == j && i >= 9 && i < 12) q = a.rdw_gyr * dt * dt;
    else if (i == j && i >= 12) q = a.rdw_acc * dt * dt;
    return s + q;
  };
  for (int k = 0; k < ns; k++) {
    if (!sOk[k]) continue;  // uniform
    if (act) A[ai * 15 + aj] = a_ent(k, ai, aj);
    __syncthreads();
    if (act) C[bi * 15 + bj] = o_ent(k, bi, bj);
    __syncthreads();
  }
  VG_PROBE_MARK(5);
  // 5. the scan opening (k_scan_begin) with the propagated state
  if (tid < 225) st->xc[kXS + tid] = C[tid];
  __syncthreads();
  for (int t = tid; t < kXC; t += blockDim.x) st->xp[t] = st->xc[t];
  if (set_scan && tid == 64) {
    st->sx = x;
    st->sy = y;
    st->sz = z;
    st->sn = n;
  }
  if (tid == 0) {
    st->it = 0;
    st->rematch = 0;
    st->done = 0;
    st->iters = 0;
    st->degenerate = 0;
    st->ticket = 0;
    for (int k = 0; k < 4; k++) st->matches[k] = 0;
    for (int k = 0; k < 4; k++) st->planes[k] = 0;
    st->iekf_pts = 0;
    if (st->clk.on) {  // this scan's k_iekf clock slots (KClock)
      const int sc = st->clk.scan + 1;
      st->clk.scan = sc;
      for (int k = 0; k < 4; k++) st->clk.exec[(sc * 4 + k) & (kClkRing - 1)] = 0;
    }
  }
  VG_PROBE_MARK(6);
#ifdef VG_PROBE
  if (tid == 0) atomicAdd(&g_probe[63], 1ull);
#endif
  if (leaf_flag && tid == 0 && !flag_wait(leaf_flag, leaf_target)) {  // the margi leaves' plane updates
    atomicOr(err, 64);
    st->done = 1;
  }
}

// ---- cross-stream hand-offs on the critical path (vg_ctx::flag_sync)
// A hipStreamWaitEvent whose event is still pending when the waiting queue
// reaches it releases late: measured ~18 us after the event on an idle GPU,
// and not before the producer's queue drained when that queue stays busy (the
// next scan's IEKF behind the margi remainder: ~97 us). So the two waits the
// scan's critical path crosses — the IEKF stream on k_margi_leaf, the main
// stream on the IEKF — are a counter instead: the producer's stream bumps it
// (k_sync_set, one lane, behind the producing kernel, so that kernel's
// end-of-kernel release has made its writes visible), a one-lane kernel on
// the consumer's stream polls it (k_sync_wait) and ends; the consumer's
// kernels then start with the usual kernel-start acquire. The flag carries a
// host-chosen increasing number (the margi's publication number, a count of
// split IEKFs), so a gated-off producer (a speculative margi tail the LM did
// not reach) simply does not store it; a poll gives up after ~1 s (error bit
// 64) instead of hanging.
__global__ void k_sync_set(unsigned* __restrict__ flag, const int* __restrict__ gate, unsigned value) {
  if (threadIdx.x != 0 || (gate && !*gate)) return;
  __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// close: the consumer is the IEKF — a wait that timed out also closes it
// (st->done: its iterations exit), so it never runs on a half-updated map
__global__ void k_sync_wait(const unsigned* __restrict__ flag, unsigned target, int* __restrict__ err,
                            DState* __restrict__ close) {
  if (threadIdx.x != 0) return;
  for (long it = 0; (int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0; it++) {
    __builtin_amdgcn_s_sleep(4);
    if (it > (1l << 24)) {
      atomicOr(err, 64);
      if (close) close->done = 1;
      return;
    }
  }
}
// the same poll with the target read from the device (a replayed graph's
// per-scan value) and a gate (the margi tail's: the LM finished)
__global__ void k_sync_wait_dev(const unsigned* __restrict__ flag, const int* __restrict__ target,
                                const int* __restrict__ gate, int* __restrict__ err) {
  if (threadIdx.x != 0 || (gate && !*gate)) return;
  const unsigned t = (unsigned)*target;
  for (long it = 0; (int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - t) < 0; it++) {
    __builtin_amdgcn_s_sleep(4);
    if (it > (1l << 24)) {
      atomicOr(err, 64);
      return;
    }
  }
}
int sync_wait_dev(vg_ctx* ctx, hipStream_t s, int k, const int* target, const int* gate) {
  k_sync_wait_dev<<<1, 64, 0, s>>>(ctx->d_sync + k, target, gate, ctx->map.counters + kCntErr);
  VG_HIP(hipGetLastError());
  return VG_OK;
}
int sync_set(vg_ctx* ctx, hipStream_t s, int k, unsigned value, const int* gate) {
  k_sync_set<<<1, 64, 0, s>>>(ctx->d_sync + k, gate, value);
  VG_HIP(hipGetLastError());
  return VG_OK;
}
int sync_wait(vg_ctx* ctx, hipStream_t s, int k, unsigned target) {
  k_sync_wait<<<1, 64, 0, s>>>(ctx->d_sync + k, target, ctx->map.counters + kCntErr, k == 0 ? ctx->st : nullptr);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

__global__ void k_set_scan(DState* __restrict__ st, const float* x, const float* y, const float* z, int n) {
  if (threadIdx.x == 0) {
    st->sx = x;
    st->sy = y;
    st->sz = z;
    st->sn = n;
  }
}

// x_buf.push_back(x_curr) at ord; a new IMU_PRE (when win_count > 1) starts
// with zero bias deltas (imu_preintegration.cpp:10-29)
// the IMU_PRE record rides in the kernel arguments (2.3 KB): no copy-engine
// transfer on the stream
__global__ void k_push_state(DState* __restrict__ st, PushArg pa) { push_state_block(st, pa); }


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
  if (t == 0) st->imu_head = (st->imu_head + 1) % kMaxWin;
}

__global__ void k_publish_state(const DState* __restrict__ st, int win_count, int ba_iters_valid,
                                const int* __restrict__ ba_iters, const int* __restrict__ ba_hess,
                                Pub* __restrict__ pub, int seq, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  publish_state_block(st, win_count, ba_iters_valid, ba_iters, ba_hess, pub, seq);
}

// P2: map counters at the end of the scan
__global__ void k_publish_counters(const int* __restrict__ counters, Pub* __restrict__ pub, int seq) {
  const int t = threadIdx.x;
  if (t < kCntN) pub_store(&pub->counters[t], counters[t]);
  pub_drain();
  __syncthreads();
  if (t == 0) pub_flag(&pub->seq2, seq);
}

// downsample result (n_out, range error) -> host
__global__ void k_publish_ds(int* __restrict__ flags, Pub* __restrict__ pub, int seq, int reset) {
  if (threadIdx.x == 0) {
    pub_store(&pub->ds_err, flags[0]);
    pub_store(&pub->n_ds, flags[1]);
    if (reset) flags[0] = 0;  // ready for the next run (the hashed path's insert takes it instead)
    pub_flag(&pub->seq_ds, seq);
  }
}

// ---- IMUEKF::motion_blur's per-point deskew (imu_ekf.cpp:114-144)
// par: [0..9) x_curr.R (after propagation), [9..12) x_curr.p, [12..21) the
// LiDAR-to-IMU rotation, [21..24) offset, then npose records of 22 doubles
// (t offset, R 9, p 3, v 3, w 3, a 3), ascending in t.
constexpr int kDeskewHead = 24, kDeskewPose = 22;
__device__ __forceinline__ V3 deskew_point(const double* par, const double* h, double t, V3 P) {
  const double dt = t - h[0];
  const M3 R_i = mul(ld_m3(h + 1), Exp(ld_v3(h + 16), dt));
  const V3 hp = ld_v3(h + 10), hv = ld_v3(h + 13), ha = ld_v3(h + 19), xp = ld_v3(par + 9);
  V3 T;
  for (int j = 0; j < 3; j++) T[j] = ((hp[j] + hv[j] * dt) + ((ha[j] * 0.5) * dt) * dt) - xp[j];
  const M3 Lr = ld_m3(par + 12);
  const V3 Lo = ld_v3(par + 21);
  const V3 a = add(mul(Lr, P), Lo);
  const V3 b = add(mul(R_i, a), T);
  const V3 c = sub(mul(tr(ld_m3(par)), b), Lo);
  return mul(tr(Lr), c);
}
// One lane per point: the segment is the last IMU pose starting strictly
// before the point (the reference's backward walk over a time-sorted cloud);
// points at or before the first pose stay. Point 0 also gets the reference
// loop's tail: after its own compensation every earlier pose that starts
// before it compensates it again.
__global__ void __launch_bounds__(256) k_deskew(int n, int npose, const double* __restrict__ par,
                                                const float* __restrict__ x, const float* __restrict__ y,
                                                const float* __restrict__ z, const float* __restrict__ in,
                                                const float* __restrict__ t, float* __restrict__ ox,
                                                float* __restrict__ oy, float* __restrict__ oz,
                                                float* __restrict__ oi) {
  const double* poses = par + kDeskewHead;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double ti = (double)t[i];
    V3 P = v3((double)x[i], (double)y[i], (double)z[i]);
    int lo = -1, hi = npose - 1;  // last pose with start < ti
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (poses[(size_t)mid * kDeskewPose] < ti) lo = mid;
      else hi = mid - 1;
    }
    float fx = x[i], fy = y[i], fz = z[i];
    if (lo >= 0) {
      P = deskew_point(par, poses + (size_t)lo * kDeskewPose, ti, P);
      fx = (float)P[0];
      fy = (float)P[1];
      fz = (float)P[2];
      if (i == 0)
        for (int k = lo - 1; k >= 0 && ti > poses[(size_t)k * kDeskewPose]; k--) {
          P = deskew_point(par, poses + (size_t)k * kDeskewPose, ti, v3((double)fx, (double)fy, (double)fz));
          fx = (float)P[0];
          fy = (float)P[1];
          fz = (float)P[2];
        }
    }
    ox[i] = fx;
    oy[i] = fy;
    oz[i] = fz;
    if (oi != in) oi[i] = in ? in[i] : 0.0f;
  }
}

// ---- Initialization::motion_blur (initialization.cpp:64-156),
// the per-point part. The host integrates the IMU poses backwards from the
// scan-end state (one record per IMU segment, descending start time, the
// deskew's 22-double layout) and plans the output: the reference walks the
// time-sorted cloud backwards, giving each point the first pose (in list
// order) that starts strictly before it, and, once point 0 is reached, pushes
// point 0 again with every later pose. Output o < n - j0 is point n-1-o; the
// rest are point 0 with poses q0+1, q0+2, ... One lane per output point:
//   pnt = R_c^T (R_i (R_L P + t_L) + T_ei)   (IMU frame at the scan end, fp64)
// par: [0..9) x_buf[i].R, [9..12) x_buf[i].p, [12..21) R_L, [21..24) t_L,
// then the pose records.
__global__ void __launch_bounds__(256) k_blur_init(int nout, int n, int j0, int npose, int q0,
                                                   const float4* __restrict__ pts, const double* __restrict__ par,
                                                   double* __restrict__ pnt) {
  const double* poses = par + kDeskewHead;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < nout; o += gridDim.x * blockDim.x) {
    int j, q;
    if (o < n - j0) {
      j = n - 1 - o;
      const double tj = (double)pts[j].w;
      int lo = 0, hi = npose - 1;  // first pose (descending starts) with start < tj; exists for j >= j0
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (poses[(size_t)mid * kDeskewPose] < tj) hi = mid;
        else lo = mid + 1;
      }
      q = lo;
    } else {
      j = 0;
      q = q0 + 1 + (o - (n - j0));
    }
    const float4 pt = pts[j];
    const double* h = poses + (size_t)q * kDeskewPose;
    const double dt = (double)pt.w - h[0];
    const M3 R_i = mul(ld_m3(h + 1), Exp(ld_v3(h + 16), dt));
    const V3 hp = ld_v3(h + 10), hv = ld_v3(h + 13), ha = ld_v3(h + 19), xp = ld_v3(par + 9);
    V3 T;
    for (int k = 0; k < 3; k++) T[k] = ((hp[k] + hv[k] * dt) + ((ha[k] * 0.5) * dt) * dt) - xp[k];
    const V3 a = add(mul(ld_m3(par + 12), v3((double)pt.x, (double)pt.y, (double)pt.z)), ld_v3(par + 21));
    const V3 r = mul(tr(ld_m3(par)), add(mul(R_i, a), T));
    for (int k = 0; k < 3; k++) pnt[(size_t)o * 3 + k] = r[k];
  }
}

// ---- host wrappers ----
int state_blur_init(vg_ctx* ctx, const double* par, int npose, const float4* pts, int n, int j0, int q0, int nout,
                    double* d_par, double* pnt) {
  const size_t nd = kDeskewHead + (size_t)npose * kDeskewPose;
  if (nd > (size_t)kDeskewBuf) {
    ctx->err = "motion_blur (init): too many IMU segments in one scan";
    return VG_E_CAPACITY;
  }
  double* stage = ctx->h_stage + kStageDeskewOff;
  memcpy(stage, par, nd * sizeof(double));
  VG_HIP(hipMemcpyAsync(d_par, stage, nd * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if (nout > 0) k_blur_init<<<grid_for(nout), 256, 0, ctx->stream>>>(nout, n, j0, npose, q0, pts, d_par, pnt);
  VG_HIP(hipGetLastError());
  VG_HIP(stream_wait(ctx));  // the staging block is reused by the next call
  return VG_OK;
}

// the window states x_buf (kXS each, by ord), x_curr (kXC), the IMU_PRE records
// of the window factors (ring from slot 0) with zero bias deltas: the
// initialisation's hand-over to the steady state (and the recut's poses)
int state_load(vg_ctx* ctx, const double* xs, int nw, const double* xc, const double* recs, int nrec) {
  hipStream_t s = ctx->stream;
  DState* st = ctx->st;
  if (nw > kMaxWin || nrec > kMaxWin) {
    ctx->err = "state_load: window too large";
    return VG_E_ARG;
  }
  if (nw > 0) VG_HIP(hipMemcpyAsync(st->xs, xs, (size_t)nw * kXS * sizeof(double), hipMemcpyHostToDevice, s));
  if (xc) VG_HIP(hipMemcpyAsync(st->xc, xc, kXC * sizeof(double), hipMemcpyHostToDevice, s));
  if (recs) {
    if (nrec > 0)
      VG_HIP(hipMemcpyAsync(st->imurec, recs, (size_t)nrec * kBaImuRec * sizeof(double), hipMemcpyHostToDevice, s));
    VG_HIP(hipMemsetAsync(st->bias, 0, sizeof(st->bias), s));
    VG_HIP(hipMemsetAsync(&st->imu_head, 0, sizeof(int), s));
  }
  VG_HIP(hipStreamSynchronize(s));
  return VG_OK;
}

int state_alloc(vg_ctx* ctx) {
  ctx->st = ctx->arena.take<DState>(1);
  ctx->d_deskew = ctx->arena.take<double>(kDeskewBuf);
  ctx->d_sync = ctx->arena.take<unsigned>(8);
  if (!ctx->st || !ctx->d_deskew || !ctx->d_sync) {
    ctx->err = "arena exhausted (state)";
    return VG_E_CAPACITY;
  }
  return VG_OK;
}

int state_scan_begin(vg_ctx* ctx, const double* xc249, const float* x, const float* y, const float* z, int n,
                     hipStream_t s, const PropArg* prop, const unsigned* head_flag, unsigned head_target,
                     const unsigned* leaf_flag, unsigned leaf_target) {
  if (prop) {
    k_scan_prop<<<1, kPropThreads, 0, s ? s : ctx->stream>>>(*prop, ctx->st, x, y, z, n, x != nullptr ? 1 : 0, head_flag,
                                                    head_target, leaf_flag, leaf_target, ctx->map.counters + kCntErr);
    VG_HIP(hipGetLastError());
    return VG_OK;
  }
  XcArg a;
  memcpy(a.x, xc249, sizeof(a.x));
  k_scan_begin<<<1, 256, 0, s ? s : ctx->stream>>>(a, ctx->st, x, y, z, n, x != nullptr ? 1 : 0);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_set_scan(vg_ctx* ctx, const float* x, const float* y, const float* z, int n, hipStream_t s) {
  k_set_scan<<<1, 64, 0, s ? s : ctx->stream>>>(ctx->st, x, y, z, n);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_push(vg_ctx* ctx, int ord, int new_imu, const double* imurec) {
  PushArg pa;
  pa.ord = ord;
  pa.new_imu = new_imu;
  if (new_imu >= 0) memcpy(pa.rec, imurec, sizeof(pa.rec));
  else memset(pa.rec, 0, sizeof(pa.rec));
  k_push_state<<<1, 64, 0, ctx->stream>>>(ctx->st, pa);
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


int state_publish(vg_ctx* ctx, int win_count, const int* ba_iters_dev, int seq, const int* gate) {
  k_publish_state<<<1, 256, 0, ctx->stream>>>(ctx->st, win_count, ba_iters_dev != nullptr, ba_iters_dev,
                                              ba_iters_dev ? ba_hess_dev(ctx) : nullptr, ctx->d_pub, seq, gate);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_publish_counters(vg_ctx* ctx, int seq) {
  k_publish_counters<<<1, 64, 0, ctx->stream>>>(ctx->map.counters, ctx->d_pub, seq);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// deskew the scan into the context's staging buffers (in place when the scan
// already is there). par: the head and the poses (host), uploaded through the
// pinned staging block.
int state_deskew(vg_ctx* ctx, const double* par, int npose, const float* x, const float* y, const float* z,
                 const float* in, const float* t, int n) {
  const size_t nd = kDeskewHead + (size_t)npose * kDeskewPose;
  if (nd > (size_t)kDeskewBuf) {
    ctx->err = "deskew: too many IMU segments in one scan";
    return VG_E_CAPACITY;
  }
  double* stage = ctx->h_stage + kStageDeskewOff;
  memcpy(stage, par, nd * sizeof(double));
  VG_HIP(hipMemcpyAsync(ctx->d_deskew, stage, nd * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if (n > 0)
    k_deskew<<<grid_for(n), 256, 0, ctx->stream>>>(n, npose, ctx->d_deskew, x, y, z, in, t, ctx->d_x, ctx->d_y,
                                                    ctx->d_z, ctx->d_i);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// host-input scans: the DMA image of the caller's arrays (xyz AoS, intensity,
// time, packed by n) -> the SoA planes every per-scan kernel reads; a missing
// intensity reads as 0 (as the synchronous staging did)
__global__ void __launch_bounds__(256) k_unpack_scan(int n, const float* __restrict__ img, int has_i, int has_t,
                                                     float* __restrict__ x, float* __restrict__ y,
                                                     float* __restrict__ z, float* __restrict__ in,
                                                     float* __restrict__ t) {
  const float* xyz = img;
  const float* si = img + 3 * (size_t)n;
  const float* st = si + (has_i ? n : 0);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    x[i] = xyz[3 * (size_t)i];
    y[i] = xyz[3 * (size_t)i + 1];
    z[i] = xyz[3 * (size_t)i + 2];
    in[i] = has_i ? si[i] : 0.0f;
    if (has_t) t[i] = st[i];
  }
}

int state_unpack_scan(vg_ctx* ctx, hipStream_t s, int n, const float* img, bool has_i, bool has_t, float* x, float* y, float* z,
                      float* in, float* t) {
  if (n <= 0) return VG_OK;
  k_unpack_scan<<<grid_for(n), 256, 0, s>>>(n, img, has_i ? 1 : 0, has_t ? 1 : 0, x, y, z, in, t);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int state_publish_ds(vg_ctx* ctx, hipStream_t s, int seq, int* flags, bool reset) {
  k_publish_ds<<<1, 64, 0, s>>>(flags, ctx->d_pub, seq, reset ? 1 : 0);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

}  // namespace vg

#ifdef VG_PROBE
VG_PROBE_READER(vg_probe_read_state)
#endif
