// kdlio.hip — SURVEY §8(a) row A14: the initialisation-phase LIO,
// VINA_SLAM::lio_state_estimation_kdtree (src/pipeline/odometry.cpp:267-439).
//
// The reference keeps the registered init scans in a float point cloud
// (pl_tree, re-downsampled at 0.5 m after every scan) behind a PCL
// KdTreeFLANN and, per scan point and IEKF iteration with refind set, takes
// the 5 nearest map points (exact search), fits a plane A n = -1 by
// ColPivHouseholderQR, rejects the point if any neighbour is off the plane by
// more than 0.1, and accumulates a unit-weight point-to-plane row.
//
// MI355X mapping: the map is bucketed by 1 m cells (sort by cell key, one
// hash entry per occupied cell); one lane per scan point searches the 27
// cells around it, then wider shells until the 5th distance is provably
// below the unsearched region (exact, the same neighbours as the kd-tree up
// to ties), fits the plane in fp64 registers, and the block reduces the 28
// normal-equation sums (HTH upper 21, HTz 6, valid count). The 15x15 update
// runs on the host (init phase only: a handful of scans). The map update
// reuses the downsample kernels (downsample.hip), bit-exact float means.
#include <hipcub/hipcub.hpp>
#include "vg_internal.h"
#include "vg_dev.h"

namespace vg {

constexpr float kCell = 1.0f;  // m
constexpr int kKdSums = 28;
constexpr int kKdBlock = 256;
constexpr int kNn = 5;  // NMATCH

__host__ __device__ __forceinline__ int kd_cell(float c) { return (int)floorf(c / kCell); }
__device__ __forceinline__ uint64_t kd_pack(int cx, int cy, int cz) {
  return ((uint64_t)(cx + (1 << 20)) << 42) | ((uint64_t)(cy + (1 << 20)) << 21) | (uint64_t)(cz + (1 << 20));
}
__device__ __forceinline__ uint32_t kd_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (uint32_t)k;
}

__global__ void k_kd_keys(int n, const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                          uint64_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    keys[i] = kd_pack(kd_cell(x[i]), kd_cell(y[i]), kd_cell(z[i]));
    idx[i] = (uint32_t)i;
  }
}

// grouped copies + one hash entry per occupied cell (its run [start, end))
__global__ void k_kd_index(int n, const uint64_t* __restrict__ keys_s, const uint32_t* __restrict__ idx_s,
                           const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                           KdMap kd) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint32_t i = idx_s[j];
    kd.sx[j] = x[i];
    kd.sy[j] = y[i];
    kd.sz[j] = z[i];
    kd.sidx[j] = (int)i;
    const uint64_t k = keys_s[j];
    if (j > 0 && keys_s[j - 1] == k) continue;
    int e = j + 1;
    while (e < n && keys_s[e] == k) e++;
    uint32_t h = kd_hash(k) & kd.hmask;
    while (true) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&kd.hkey[h], ~0ull, (unsigned long long)k);
      if (prev == ~0ull) break;
      h = (h + 1) & kd.hmask;
    }
    kd.hstart[h] = j;
    kd.hend[h] = e;
  }
}

__device__ __forceinline__ bool kd_less(float d, int id, float e, int je) { return d < e || (d == e && id < je); }
// insertion into the ascending top-5 (distance, then map index)
__device__ __forceinline__ void kd_offer(float d, int id, float* bd, int* bi, int& cnt) {
  if (cnt == kNn && !kd_less(d, id, bd[kNn - 1], bi[kNn - 1])) return;
  int pos = cnt < kNn ? cnt++ : kNn - 1;
  while (pos > 0 && kd_less(d, id, bd[pos - 1], bi[pos - 1])) {
    bd[pos] = bd[pos - 1];
    bi[pos] = bi[pos - 1];
    pos--;
  }
  bd[pos] = d;
  bi[pos] = id;
}

__device__ __forceinline__ void kd_scan_cell(const KdMap& kd, int cx, int cy, int cz, float qx, float qy, float qz,
                                             float* bd, int* bi, int& cnt) {
  const uint64_t k = kd_pack(cx, cy, cz);
  uint32_t h = kd_hash(k) & kd.hmask;
  while (true) {
    const uint64_t hk = kd.hkey[h];
    if (hk == ~0ull) return;
    if (hk == k) break;
    h = (h + 1) & kd.hmask;
  }
  const int e = kd.hend[h];
  for (int j = kd.hstart[h]; j < e; j++) {
    const float dx = kd.sx[j] - qx, dy = kd.sy[j] - qy, dz = kd.sz[j] - qz;
    kd_offer((dx * dx + dy * dy) + dz * dz, kd.sidx[j], bd, bi, cnt);
  }
}

// exact 5 nearest (float squared distance, ties by map index)
__device__ void kd_knn(const KdMap& kd, float qx, float qy, float qz, float* bd, int* bi) {
  int cnt = 0;
  const int cx = kd_cell(qx), cy = kd_cell(qy), cz = kd_cell(qz);
  for (int r = 1; r <= 3; r++) {
    for (int dz = -r; dz <= r; dz++)
      for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
          const int a = max(abs(dx), max(abs(dy), abs(dz)));
          if (r > 1 && a < r) continue;  // shells beyond the first
          kd_scan_cell(kd, cx + dx, cy + dy, cz + dz, qx, qy, qz, bd, bi, cnt);
        }
    // every unsearched point is farther than r cells from the query
    const float bound = (float)r * kCell;
    if (cnt == kNn && bd[kNn - 1] < bound * bound * 0.999999f) return;
  }
  cnt = 0;  // far from the map: the whole map
  for (int j = 0; j < kd.n; j++) {
    const float dx = kd.x[j] - qx, dy = kd.y[j] - qy, dz = kd.z[j] - qz;
    kd_offer((dx * dx + dy * dy) + dz * dz, j, bd, bi, cnt);
  }
}

struct KdPose {
  double R[9], p[3], eR[9], et[3];
};

// odometry.cpp:342-381 per point with refind set: the 5 nearest map points,
// the plane fit and its check -> ds[i] (-1: rejected) and the unit normal
__global__ void __launch_bounds__(kKdBlock) k_kd_pass(int n, const float* __restrict__ px, const float* __restrict__ py,
                                                      const float* __restrict__ pz, KdPose ps, KdMap kd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const M3 R = ld_m3(ps.R);
  const V3 pnt = rigid(ld_m3(ps.eR), v3(px[i], py[i], pz[i]), ld_v3(ps.et));  // var_init (point_utils.cpp:36-52)
  const V3 wld = rigid(R, pnt, ld_v3(ps.p));
  float bd[kNn];
  int bi[kNn];
  kd_knn(kd, (float)wld[0], (float)wld[1], (float)wld[2], bd, bi);
  double A[kNn * 3], b[kNn];
  for (int r = 0; r < kNn; r++) {
    A[r * 3 + 0] = kd.x[bi[r]];
    A[r * 3 + 1] = kd.y[bi[r]];
    A[r * 3 + 2] = kd.z[bi[r]];
    b[r] = -1.0;
  }
  double dir[3];
  colpiv_qr_solve(A, kNn, b, dir);
  bool off = false;
  for (int r = 0; r < kNn; r++)
    if (fabs(((dir[0] * A[r * 3] + dir[1] * A[r * 3 + 1]) + dir[2] * A[r * 3 + 2]) + 1.0) > 0.1) off = true;
  if (off) {
    kd.ds[i] = -1.0;
  } else {
    const double d = 1.0 / sqrt((dir[0] * dir[0] + dir[1] * dir[1]) + dir[2] * dir[2]);
    kd.ds[i] = d;
    for (int c = 0; c < 3; c++) kd.dir[(size_t)i * 3 + c] = dir[c] * d;
  }
}

// the iteration's normal equations (odometry.cpp:367-378): HTH += jac jac^T,
// HTz += jac (-pd2), valid++ over the scan's points IN POINT ORDER, as the
// reference accumulates them — one workgroup: 1024 points at a time get their
// Jacobian row in parallel (LDS), then lane k of wave 0 adds sum k's terms in
// order (HTH upper 21, HTz 6, the count). The sums, and so the 15x15 update
// on the host, are the reference's bit for bit.
constexpr int kKdSumThreads = 1024;
__global__ void __launch_bounds__(kKdSumThreads) k_kd_sum(int n, const float* __restrict__ px,
                                                          const float* __restrict__ py, const float* __restrict__ pz,
                                                          KdPose ps, KdMap kd) {
  __shared__ double sj[7][kKdSumThreads];  // jac 0..5, -pd2
  __shared__ unsigned char sv[kKdSumThreads];
  const int tid = threadIdx.x;
  const M3 R = ld_m3(ps.R);
  const M3 Rt = tr(R);
  double acc = 0.0;
  int cnt = 0;
  // sum k (wave 0, lane k < 27): HTH (r, c) upper row-major, then HTz r
  int kr = 0, kc = 0;
  if (tid < 21) {
    int k = tid;
    while (k >= 6 - kr) {
      k -= 6 - kr;
      kr++;
    }
    kc = kr + k;
  } else if (tid < 27) {
    kr = tid - 21;
    kc = 6;
  }
  for (int c0 = 0; c0 < n; c0 += kKdSumThreads) {
    const int i = c0 + tid;
    unsigned char v = 0;
    if (i < n) {
      const double dsi = kd.ds[i];
      if (dsi >= 0) {
        const V3 pnt = rigid(ld_m3(ps.eR), v3(px[i], py[i], pz[i]), ld_v3(ps.et));
        const V3 wld = rigid(R, pnt, ld_v3(ps.p));
        const V3 nv = v3(kd.dir[(size_t)i * 3], kd.dir[(size_t)i * 3 + 1], kd.dir[(size_t)i * 3 + 2]);
        const double pd2 = ((nv[0] * wld[0] + nv[1] * wld[1]) + nv[2] * wld[2]) + dsi;
        const V3 j0 = mul(mul(hat(pnt), Rt), nv);
        for (int c = 0; c < 3; c++) {
          sj[c][tid] = j0[c];
          sj[3 + c][tid] = nv[c];
        }
        sj[6][tid] = -pd2;
        v = 1;
      }
    }
    sv[tid] = v;
    __syncthreads();
    if (tid < kKdSums) {
      const int m = n - c0 < kKdSumThreads ? n - c0 : kKdSumThreads;
      if (tid == kKdSums - 1) {
        for (int t = 0; t < m; t++) cnt += sv[t];
      } else {
        for (int t = 0; t < m; t++)
          if (sv[t]) acc += sj[kr][t] * sj[kc][t];
      }
    }
    __syncthreads();
  }
  if (tid < kKdSums) kd.part[tid] = tid == kKdSums - 1 ? (double)cnt : acc;
}

// the registered scan (world, float) appended to the map (odometry.cpp:427-435)
__global__ void k_kd_append(int n, const float* __restrict__ px, const float* __restrict__ py,
                            const float* __restrict__ pz, KdPose ps, int base, KdMap kd) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const V3 pnt = rigid(ld_m3(ps.eR), v3(px[i], py[i], pz[i]), ld_v3(ps.et));
    const V3 w = rigid(ld_m3(ps.R), pnt, ld_v3(ps.p));
    kd.x[base + i] = (float)w[0];
    kd.y[base + i] = (float)w[1];
    kd.z[base + i] = (float)w[2];
  }
}

int kd_alloc(vg_ctx* ctx) {
  KdMap& kd = ctx->kd;
  const int np = ctx->cap.max_points_per_scan;
  kd.cap = np;  // map + appended scan must fit the downsample buffers
  int hs = 1;
  while (hs < 2 * kd.cap) hs <<= 1;
  kd.hmask = hs - 1;
  bool good = true;
  good &= (kd.x = ctx->arena.take<float>(kd.cap)) != nullptr;
  good &= (kd.y = ctx->arena.take<float>(kd.cap)) != nullptr;
  good &= (kd.z = ctx->arena.take<float>(kd.cap)) != nullptr;
  good &= (kd.sx = ctx->arena.take<float>(kd.cap)) != nullptr;
  good &= (kd.sy = ctx->arena.take<float>(kd.cap)) != nullptr;
  good &= (kd.sz = ctx->arena.take<float>(kd.cap)) != nullptr;
  good &= (kd.sidx = ctx->arena.take<int>(kd.cap)) != nullptr;
  good &= (kd.keys = ctx->arena.take<uint64_t>(kd.cap)) != nullptr;
  good &= (kd.keys_s = ctx->arena.take<uint64_t>(kd.cap)) != nullptr;
  good &= (kd.idx = ctx->arena.take<uint32_t>(kd.cap)) != nullptr;
  good &= (kd.idx_s = ctx->arena.take<uint32_t>(kd.cap)) != nullptr;
  good &= (kd.hkey = ctx->arena.take<uint64_t>(hs)) != nullptr;
  good &= (kd.hstart = ctx->arena.take<int>(hs)) != nullptr;
  good &= (kd.hend = ctx->arena.take<int>(hs)) != nullptr;
  good &= (kd.ds = ctx->arena.take<double>(np)) != nullptr;
  good &= (kd.dir = ctx->arena.take<double>((size_t)np * 3)) != nullptr;
  good &= (kd.part = ctx->arena.take<double>((size_t)(np / kKdBlock + 1) * kKdSums)) != nullptr;
  size_t tb = 0;
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kd.keys, kd.keys_s, kd.idx, kd.idx_s, kd.cap, 0, 64,
                                            ctx->stream));
  kd.tmp_bytes = tb;
  good &= (kd.tmp = ctx->arena.take<char>(tb)) != nullptr;
  if (!good) {
    ctx->err = "arena exhausted (kd map)";
    return VG_E_CAPACITY;
  }
  kd.n = 0;
  return VG_OK;
}

int kd_reset(vg_ctx* ctx) {
  ctx->kd.n = 0;
  return VG_OK;
}

static int kd_index(vg_ctx* ctx) {
  KdMap& kd = ctx->kd;
  hipStream_t s = ctx->stream;
  VG_HIP(hipMemsetAsync(kd.hkey, 0xff, (size_t)(kd.hmask + 1) * sizeof(uint64_t), s));
  if (kd.n > 0) {
    k_kd_keys<<<grid_for(kd.n), kBlock, 0, s>>>(kd.n, kd.x, kd.y, kd.z, kd.keys, kd.idx);
    size_t tb = kd.tmp_bytes;
    VG_HIP(hipcub::DeviceRadixSort::SortPairs(kd.tmp, tb, kd.keys, kd.keys_s, kd.idx, kd.idx_s, kd.n, 0, 64, s));
    k_kd_index<<<grid_for(kd.n), kBlock, 0, s>>>(kd.n, kd.keys_s, kd.idx_s, kd.x, kd.y, kd.z, kd);
  }
  VG_HIP(hipGetLastError());
  return VG_OK;
}

static KdPose kd_pose(vg_ctx* ctx, const double* R, const double* p) {
  KdPose ps;
  for (int i = 0; i < 9; i++) {
    ps.R[i] = R[i];
    ps.eR[i] = ctx->cfg.ext_R[i];
  }
  for (int i = 0; i < 3; i++) {
    ps.p[i] = p[i];
    ps.et[i] = ctx->cfg.ext_t[i];
  }
  return ps;
}

int kd_pass(vg_ctx* ctx, int n, const double* R, const double* p, int refind, double* out28) {
  KdMap& kd = ctx->kd;
  hipStream_t s = ctx->stream;
  for (int k = 0; k < kKdSums; k++) out28[k] = 0.0;
  if (n <= 0) return VG_OK;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "kd pass: scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  const KdPose ps = kd_pose(ctx, R, p);
  if (refind) k_kd_pass<<<(n + kKdBlock - 1) / kKdBlock, kKdBlock, 0, s>>>(n, ctx->d_x, ctx->d_y, ctx->d_z, ps, kd);
  k_kd_sum<<<1, kKdSumThreads, 0, s>>>(n, ctx->d_x, ctx->d_y, ctx->d_z, ps, kd);
  VG_HIP(hipGetLastError());
  VG_HIP(hipMemcpyAsync(out28, kd.part, kKdSums * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  return VG_OK;
}

int kd_update(vg_ctx* ctx, int n, const double* R, const double* p, bool downsample) {
  KdMap& kd = ctx->kd;
  hipStream_t s = ctx->stream;
  if (kd.n + n > kd.cap) {
    ctx->err = "kd map: map + scan exceed max_points_per_scan";
    return VG_E_CAPACITY;
  }
  if (n > 0) k_kd_append<<<grid_for(n), kBlock, 0, s>>>(n, ctx->d_x, ctx->d_y, ctx->d_z, kd_pose(ctx, R, p), kd.n, kd);
  VG_HIP(hipGetLastError());
  kd.n += n;
  if (downsample && kd.n > 0) {  // down_sampling_voxel(*pl_tree, 0.5) (odometry.cpp:436)
    int nout = 0;
    VG_TRY(ds_run(ctx, kd.x, kd.y, kd.z, nullptr, kd.n, 0.5, &nout));
    VG_HIP(hipMemcpyAsync(kd.x, ctx->ds.ox, (size_t)nout * sizeof(float), hipMemcpyDeviceToDevice, s));
    VG_HIP(hipMemcpyAsync(kd.y, ctx->ds.oy, (size_t)nout * sizeof(float), hipMemcpyDeviceToDevice, s));
    VG_HIP(hipMemcpyAsync(kd.z, ctx->ds.oz, (size_t)nout * sizeof(float), hipMemcpyDeviceToDevice, s));
    kd.n = nout;
  }
  VG_TRY(kd_index(ctx));
  VG_HIP(hipStreamSynchronize(s));
  return VG_OK;
}

}  // namespace vg
