// vg_iekf.h — the IEKF update (odometry.cpp:192-254) as a workgroup-level
// device routine, run by k_iekf_update after each k_iekf point loop (map.hip).
//
// The reference forms K_1 = (H_T_H + cov^-1)^-1 with two 15 x 15 inverses
// (odometry.cpp:82, 194) but only ever uses its first six columns (K_1.block<15,6>,
// 198-201). Since H_T_H is zero outside its 6 x 6 block, the push-through
// (Woodbury) identity gives exactly those columns from one 6 x 6 system:
//   K6 = K_1(:, 0:6) = cov(:, 0:6) (I + HTH cov(0:6, 0:6))^-1,
// solved here by one wave (Gauss-Jordan with partial pivoting, one column of
// [M^T | cov(:,0:6)^T] per lane, no barriers). Identical in exact arithmetic;
// rounding differs from the 15 x 15 route at the 1e-13 relative level (the
// parity tests bound the trajectory).
#pragma once
#include "vg_dev.h"

namespace vg {

constexpr int kIekfVals = 34;  // HTH upper 21, HTz 6, nnt upper 6, match count

// LDS of iekf_update_block
constexpr int kIekfGroups = 60;  // row groups of the partial sums (1024-lane update: 60 x 17 lanes)
struct IekfLds {
  double red[kIekfGroups][kIekfVals];
  double o[kIekfVals], K6[15][6], G6[15][6], vec[15], sol[15], IG[15][15];
  int fin;
};

// One IEKF update after iteration `it`'s point loop wrote nb block partials
// (row-major nb x kIekfVals; nb < 0: `partials` is the final 34 sums). Whole
// workgroup (>= 256 threads), uniform.
// ordered sum of nb block partials (row-major nb x kIekfVals) into L.o: row
// group g = tid / 17 (rows g, g+G, ...; G = blockDim / 17 groups, at most
// kIekfGroups), lane pair 2*(tid % 17); then the G groups in order
// (deterministic). A 1024-lane update runs 60 groups of ~9 rows each: the
// dependent chains of L2 / cross-XCD loads are 4x shorter than with 15.
// (nact: the workgroups whose chunk holds points, iekf_chunk below; the
// others' rows are +0 and skipped — the same sums)
__device__ __forceinline__ int iekf_chunk(int b, int nb);
__device__ __forceinline__ void iekf_reduce_block(int nb, const double* __restrict__ partials, IekfLds& L,
                                                  int nact) {
  const int tid = threadIdx.x;
  const int G = (int)blockDim.x / 17 < kIekfGroups ? (int)blockDim.x / 17 : kIekfGroups;
  const int g = tid / 17, j2 = 2 * (tid % 17);
  if (g < G) {
    // the group's first kRows rows loaded at once (one memory round trip, not
    // one per row), then summed in the same row order
    constexpr int kRows = 9;  // ceil(512 / 60): a 512-workgroup grid in one batch
    double2 v[kRows];
    bool ok[kRows];
#pragma unroll
    for (int k = 0; k < kRows; k++) {
      const int b = g + k * G;
      ok[k] = b < nb && iekf_chunk(b, nb) < nact;
      v[k] = ok[k] ? *reinterpret_cast<const double2*>(&partials[(size_t)b * kIekfVals + j2]) : make_double2(0.0, 0.0);
    }
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int k = 0; k < kRows; k++)
      if (ok[k]) {
        a0 += v[k].x;
        a1 += v[k].y;
      }
    for (int b = g + kRows * G; b < nb; b += G) {
      if (iekf_chunk(b, nb) >= nact) continue;
      const double2 w = *reinterpret_cast<const double2*>(&partials[(size_t)b * kIekfVals + j2]);
      a0 += w.x;
      a1 += w.y;
    }
    L.red[g][j2] = a0;
    L.red[g][j2 + 1] = a1;
  }
  __syncthreads();
  if (tid < kIekfVals) {
    double s = L.red[0][tid];
    for (int k = 1; k < G; k++) s += L.red[k][tid];
    L.o[tid] = s;
  }
  __syncthreads();
}

// 64-bit broadcast of lane `ln` (a compile-time constant after unrolling)
__device__ __forceinline__ double bcast_lane(double v, int ln) {
  const long long b = __double_as_longlong(v);
  const int lo32 = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), ln);
  const int hi32 = __builtin_amdgcn_readlane((int)(b >> 32), ln);
  return __longlong_as_double(((long long)hi32 << 32) | (unsigned int)lo32);
}

// The point loop's chunk of workgroup b (XCD-aware: consecutive chunks on one
// XCD); the reduction skips the rows of chunks without points (an exact no-op:
// their sums are +0)
__device__ __forceinline__ int iekf_chunk(int b, int nb) { return (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b; }

__device__ __forceinline__ void iekf_update_tail(DState* __restrict__ st, int it, IekfLds& L, bool vec_done = false);
// vec = x_prop ⊟ x_curr (IMUST::operator-, types.hpp:80-86), one thread
__device__ __forceinline__ void iekf_vec(const DState* __restrict__ st, IekfLds& L) {
  const double* xp = st->xp;
  const double* xc = st->xc;
  const V3 rr = Log(mul(tr(ld_m3(xc)), ld_m3(xp)));
  for (int k = 0; k < 3; k++) {
    L.vec[k] = rr[k];
    L.vec[3 + k] = xp[9 + k] - xc[9 + k];
    L.vec[6 + k] = xp[12 + k] - xc[12 + k];
    L.vec[9 + k] = xp[15 + k] - xc[15 + k];
    L.vec[12 + k] = xp[18 + k] - xc[18 + k];
  }
}
// nb < 0 (sharded): `partials` is the all-reduced exchange frame; xworld > 0:
// its guard is checked here (a mismatch sets error bit 32 and the update runs
// on zeros, as a separately unpacked frame's consumers did)
__device__ void iekf_update_block(int nb, const double* __restrict__ partials, DState* __restrict__ st, int it,
                                  IekfLds& L, int xworld = 0, int* xerr = nullptr) {
  const int tid = threadIdx.x;
  VG_PROBE_BEGIN();
  // x_curr does not change before the update's end: vec on a lane the
  // ordered sum leaves idle (17 x 60 = 1020 of 1024), beside the sum. (Copies
  // of x_curr and its covariance loaded with the partials, read from LDS after
  // the sum, measured -0.8 %: profiles/r05/ab_iekf_state_copy_r05p.txt.)
  const bool vec_early = (int)blockDim.x > 17 * kIekfGroups;
  if (vec_early && tid == (int)blockDim.x - 1) iekf_vec(st, L);
  if (nb >= 0) {
    const int n = iekf_n(st);
    iekf_reduce_block(nb, partials, L, n < nb * 256 ? (n + 255) / 256 : nb);
  } else {  // sharded mode: `partials` holds the all-reduced sums
    const bool ok = xworld <= 0 || xchg_ok(partials, kShardSmall, xworld);
    if (!ok && tid == 0) atomicOr(xerr, 32);
    if (tid < kIekfVals) L.o[tid] = ok ? partials[tid] : 0.0;
    __syncthreads();
  }
  VG_PROBE_MARK(23);  // the ordered sum of the block partials
  iekf_update_tail(st, it, L, vec_early);
}
// the update once L.o holds the 34 sums
__device__ __forceinline__ void iekf_update_tail(DState* __restrict__ st, int it, IekfLds& L, bool vec_done) {
  const int tid = threadIdx.x;
  VG_PROBE_BEGIN();
  const double* o = L.o;
  auto hth = [&](int i, int j) {
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    return o[lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
  };
  if (tid == 0) {
    st->iters = it + 1;
    st->matches[it] = (int)o[33];
    for (int k = 0; k < 6; k++) st->nnt[k] = o[27 + k];
  }
  VG_PROBE_MARK(24);
  if (tid < 64) {  // K6 = cov(:, 0:6) M^-1, M = I + HTH cov66: solve M^T X = cov(:, 0:6)^T, K6 = X^T
    const int lane = tid;
    const double* cov = st->xc + kXS;
    double col[6];
    if (lane < 6) {  // column `lane` of M^T = row `lane` of M
      for (int r = 0; r < 6; r++) {
        double sm = hth(lane, 0) * cov[0 * 15 + r];
        for (int l = 1; l < 6; l++) sm += hth(lane, l) * cov[l * 15 + r];
        col[r] = ((lane == r) ? 1.0 : 0.0) + sm;
      }
    } else {
      const int i = lane < 21 ? lane - 6 : 0;  // column i of cov(:, 0:6)^T = row i of cov, cols 0..5
      for (int r = 0; r < 6; r++) col[r] = cov[i * 15 + r];
    }
#pragma unroll
    for (int c = 0; c < 6; c++) {
      double pc[6];
#pragma unroll
      for (int r = 0; r < 6; r++) pc[r] = bcast_lane(col[r], c);
      int p = c;
      double best = fabs(pc[c]);
#pragma unroll
      for (int r = c + 1; r < 6; r++)
        if (fabs(pc[r]) > best) {
          best = fabs(pc[r]);
          p = r;
        }
      // swap rows c, p (pivot column and this lane's column)
      double pv = pc[c], cv = col[c];
#pragma unroll
      for (int r = c + 1; r < 6; r++)
        if (r == p) {
          const double t = pc[r];
          pc[r] = pv;
          pv = t;
          const double u = col[r];
          col[r] = cv;
          cv = u;
        }
      const double inv = 1.0 / pv;
      cv *= inv;
      col[c] = cv;
#pragma unroll
      for (int r = 0; r < 6; r++)
        if (r != c && pc[r] != 0.0) col[r] -= pc[r] * cv;
    }
    if (!vec_done) {  // (iekf_update_block computes it beside the sum)
      if (lane == 63) iekf_vec(st, L);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // G6 = K6 HTH and sol = (K6 HTz + vec) - G6 v6 on the lanes that hold K6's
    // rows (lane 6 + r: row r), in the same operation order as a separate
    // pass would take them from LDS, so no workgroup barrier sits between
    // the 6 x 6 solve and the state update
    if (lane >= 6 && lane < 21) {
      const int r = lane - 6;
      double g[6];
#pragma unroll
      for (int c = 0; c < 6; c++) {
        double sv = col[0] * hth(0, c);
        for (int k = 1; k < 6; k++) sv += col[k] * hth(k, c);
        g[c] = sv;
        L.G6[r][c] = sv;
        st->G6[r * 6 + c] = sv;
      }
      double s1 = col[0] * o[21];
      for (int k = 1; k < 6; k++) s1 += col[k] * o[21 + k];
      double s2 = g[0] * L.vec[0];
      for (int k = 1; k < 6; k++) s2 += g[k] * L.vec[k];
      L.sol[r] = (s1 + L.vec[r]) - s2;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // lane 0 reads every row's sol
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    VG_PROBE_MARK(25);
    VG_PROBE_MARK(26);
    if (lane == 0) {  // x_curr ⊞= sol (types.hpp:67-78); convergence / rematch (odometry.cpp:205-227)
      double* xc = st->xc;
      const double* sol = L.sol;
      const M3 Rn = mul(ld_m3(xc), Exp(v3(sol[0], sol[1], sol[2])));
      for (int k = 0; k < 9; k++) xc[k] = Rn[k];
      double pn[3];
      for (int k = 0; k < 3; k++) {
        pn[k] = xc[9 + k] + sol[3 + k];
        xc[9 + k] = pn[k];
        xc[12 + k] += sol[6 + k];
        xc[15 + k] += sol[9 + k];
        xc[18 + k] += sol[12 + k];
      }
      const double rot_add = norm3(v3(sol[0], sol[1], sol[2])), tra_add = norm3(v3(sol[3], sol[4], sol[5]));
      const bool conv = (rot_add * 57.3 < 0.01) && (tra_add * 100 < 0.015);
      int rm = st->rematch;
      if (conv || ((rm == 0) && (it == 4 - 2))) rm++;
      st->rematch = rm;
      L.fin = (rm >= 2 || it == 4 - 1) ? 1 : 0;
      if (L.fin) {  // the trajectory row (the pose the IEKF ends at), from registers
        for (int k = 0; k < 9; k++) st->traj[k] = Rn[k];
        for (int k = 0; k < 3; k++) st->traj[9 + k] = pn[k];
      }
    }
  }
  __syncthreads();
  VG_PROBE_MARK(27);
#ifdef VG_PROBE
  if (tid == 0) atomicAdd(&g_probe[61], 1ull);
#endif
  if (!L.fin) return;
  // cov = (I - G) cov (G zero outside columns 0..5)
  for (int e = tid; e < 225; e += blockDim.x) {
    const int r = e / 15, c = e % 15;
    L.IG[r][c] = ((r == c) ? 1.0 : 0.0) - (c < 6 ? L.G6[r][c] : 0.0);
  }
  __syncthreads();
  double cv = 0.0;
  if (tid < 225) {
    const int r = tid / 15, c = tid % 15;
    const double* cov = st->xc + kXS;
    double s = L.IG[r][0] * cov[c];
    for (int k = 1; k < 15; k++) s += L.IG[r][k] * cov[k * 15 + c];
    cv = s;
  }
  __syncthreads();
  if (tid < 225) st->xc[kXS + tid] = cv;
  VG_PROBE_MARK(28);
  if (tid == 0) st->done = 1;  // (the degeneracy test, odometry.cpp:244-254, runs on the host from nnt)
  VG_PROBE_MARK(29);
#ifdef VG_PROBE
  if (tid == 0) atomicAdd(&g_probe[60], 1ull);
#endif
}

}  // namespace vg
