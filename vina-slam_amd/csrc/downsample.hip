// downsample.hip — A1 voxel-grid downsample.
//
// Replaces down_sampling_voxel (include/vina_slam/core/point_utils.hpp:7-44):
// per voxel, the running mean (x*c + p)/(c+1) in float over the voxel's points
// in input order, intensity of the first point, curvature := count.
//
// MI355X mapping (HBM-bound integer/byte work, no MFMA):
//  1. k_ds_keys   — one lane per point: coalesced SoA fp32 loads, the exact
//                   reference key rule (fp64 divide -> fp32 round -> "-1 if
//                   negative" in fp32 -> int64 truncation), 21-bit-per-axis
//                   packing into one u64.
//  2. radix sort  — (packed key, point index) pairs, stable (hipCUB/rocPRIM
//                   onesweep): groups each voxel and keeps input order inside.
//  3. k_ds_heads + exclusive scan — voxel ranks (output order = key order).
//  4. k_ds_mean   — one lane per voxel walks its segment in input order and
//                   reproduces the reference's float recurrence bit-for-bit
//                   (the library is built with -ffp-contract=off).
#include <algorithm>
#include <hipcub/hipcub.hpp>
#include "vg_internal.h"

namespace vg {

__device__ __forceinline__ int64_t key_axis_f(float c, double size) {
  // point_utils.hpp:18-21: loc = p_c.data[j] / voxel_size (float / double ->
  // double divide), stored to float; if (loc < 0) loc -= 1.0; (int64_t)loc.
  float l = (float)((double)c / size);
  if (l < 0) l -= 1.0f;
  return (int64_t)l;
}

// 1/(k+1) in fp64, correctly rounded (constant-evaluated IEEE division)
constexpr int kRcpN = 264;  // >= kHdsMid + 1
struct RcpTable {
  double v[kRcpN];
  constexpr RcpTable() : v() {
    for (int k = 0; k < kRcpN; k++) v[k] = 1.0 / (double)(k + 1);
  }
};
__constant__ RcpTable kRcp = RcpTable();

// One step of point_utils.hpp:34-37's running mean, p <- (p*c + v) / (c+1) in
// float: the product and the sum rounded as written (no contraction), the
// quotient as t * r in fp64 with r = RN64(1/(c+1)), rounded once to float.
// That is the correctly rounded float quotient RN32(t/(c+1)) (for c+1 <=
// 2^24): the fp64 value is within 2^-52 (relative) of t/b, while a float t
// over an integer b <= 2^24 is either exact, or an exact rounding midpoint
// only where r is exact too (b a power of two, or a subnormal quotient: taken
// by the division below), or at least 2^-26/b >= 2^-50 (relative) away from
// every midpoint between floats, so both round to the same float. It takes
// the fp32 division's long correctly rounded sequence off the serial chain.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ float mean_step(float p, float c, float v, double r) {
  const float t = p * c + v;
  if (__builtin_expect(fabsf(t) < 0x1p-100f, 0)) return t / (c + 1);
  return (float)((double)t * r);
}

__global__ void k_ds_keys(int n, const float* __restrict__ x, const float* __restrict__ y,
                          const float* __restrict__ z, double size, uint64_t* __restrict__ keys,
                          uint32_t* __restrict__ idx, int* __restrict__ flags) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int64_t kx = key_axis_f(x[i], size) + kKeyOff;
    int64_t ky = key_axis_f(y[i], size) + kKeyOff;
    int64_t kz = key_axis_f(z[i], size) + kKeyOff;
    bool bad = (kx < 0) | (ky < 0) | (kz < 0) | (kx >= 2 * kKeyOff) | (ky >= 2 * kKeyOff) | (kz >= 2 * kKeyOff);
    if (bad) {
      atomicOr(&flags[0], 1);
      kx = ky = kz = 0;
    }
    keys[i] = ((uint64_t)kx << 42) | ((uint64_t)ky << 21) | (uint64_t)kz;
    idx[i] = (uint32_t)i;
  }
}

__global__ void k_ds_heads(int n, const uint64_t* __restrict__ ks, uint32_t* __restrict__ head) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    head[j] = (j == 0 || ks[j] != ks[j - 1]) ? 1u : 0u;
}

__global__ void k_ds_segs(int n, const uint32_t* __restrict__ head, const uint32_t* __restrict__ pos,
                          uint32_t* __restrict__ seg, int* __restrict__ flags) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    if (head[j]) seg[pos[j]] = (uint32_t)j;
    if (j == n - 1) {
      flags[1] = (int)(pos[j] + head[j]);
      seg[pos[j] + head[j]] = (uint32_t)n;  // sentinel end
    }
  }
}

__global__ void k_ds_mean(const int* __restrict__ flags, const uint32_t* __restrict__ seg,
                          const uint32_t* __restrict__ order, const float* __restrict__ x,
                          const float* __restrict__ y, const float* __restrict__ z, const float* __restrict__ in,
                          float* __restrict__ ox, float* __restrict__ oy, float* __restrict__ oz,
                          float* __restrict__ oi, float* __restrict__ oc) {
  const int nv = flags[1];
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gridDim.x * blockDim.x) {
    uint32_t b = seg[v], e = seg[v + 1];
    uint32_t i0 = order[b];
    float px = x[i0], py = y[i0], pz = z[i0], c = 1.0f;
    for (uint32_t j = b + 1; j < e; j++) {
      uint32_t i = order[j];
      // point_utils.hpp:34-37 (mean_step: exactly the float recurrence as written)
      const uint32_t jj = j - b;  // == c
      const double r = jj < (uint32_t)kRcpN ? kRcp.v[jj] : 1.0 / (double)(jj + 1);
      px = mean_step(px, c, x[i], r);
      py = mean_step(py, c, y[i], r);
      pz = mean_step(pz, c, z[i], r);
      c += 1;
    }
    ox[v] = px;
    oy[v] = py;
    oz[v] = pz;
    oi[v] = in ? in[i0] : 0.0f;
    oc[v] = c;
  }
}

// ---- down_sampling_close (point_utils.hpp:46-113), the initialisation's raw
// cloud reduction (node.cpp:337-343): per voxel the real point nearest the
// float mean of the voxel's points. The voxel grouping is the A1 pipeline
// above (keys, stable sort, segments); one lane per voxel then
//  - sums its points in input order in fp32 (pb.x += ...), divides by the
//    count in fp32, and picks the first point at the smallest fp64 squared
//    distance (float differences widened, as the reference's `double xx =
//    pb.x - v[i].x`), starting from ndis = 100;
//  - emits it with its time; voxels come out in ascending packed-key order,
//    i.e. (x, y, z) lexicographic, and a stable sort by time follows (the
//    reference std::sorts unordered_map order by time; the order of equal
//    times is unspecified there, this one is the oracle's).
__device__ __forceinline__ uint32_t time_key(float t) {  // order-preserving float -> u32 (-0 as +0)
  uint32_t b = __float_as_uint(t == 0.0f ? 0.0f : t);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ void k_close_pick(const int* __restrict__ flags, const uint32_t* __restrict__ seg,
                             const uint32_t* __restrict__ order, const float* __restrict__ x,
                             const float* __restrict__ y, const float* __restrict__ z, const float* __restrict__ t,
                             float tconst, float* __restrict__ ox, float* __restrict__ oy, float* __restrict__ oz,
                             float* __restrict__ ot, uint32_t* __restrict__ tkey, uint32_t* __restrict__ tidx) {
  const int nv = flags[1];
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gridDim.x * blockDim.x) {
    const uint32_t b = seg[v], e = seg[v + 1];
    const uint32_t i0 = order[b];
    float px = x[i0], py = y[i0], pz = z[i0];
    for (uint32_t j = b + 1; j < e; j++) {
      const uint32_t i = order[j];
      px += x[i];
      py += y[i];
      pz += z[i];
    }
    const float cnt = (float)(int)(e - b);
    px /= cnt;
    py /= cnt;
    pz /= cnt;
    double ndis = 100;
    uint32_t best = i0;
    for (uint32_t j = b; j < e; j++) {
      const uint32_t i = order[j];
      const double xx = (double)(px - x[i]), yy = (double)(py - y[i]), zz = (double)(pz - z[i]);
      const double dis = xx * xx + yy * yy + zz * zz;
      if (dis < ndis) {
        best = i;
        ndis = dis;
      }
    }
    const float tb = t ? t[best] : tconst;
    ox[v] = x[best];
    oy[v] = y[best];
    oz[v] = z[best];
    ot[v] = tb;
    tkey[v] = time_key(tb);
    tidx[v] = (uint32_t)v;
  }
}

__global__ void k_close_gather(int nv, const uint32_t* __restrict__ perm, const float* __restrict__ ox,
                               const float* __restrict__ oy, const float* __restrict__ oz,
                               const float* __restrict__ ot, float4* __restrict__ out) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < nv; r += gridDim.x * blockDim.x) {
    const uint32_t v = perm[r];
    out[r] = make_float4(ox[v], oy[v], oz[v], ot[v]);
  }
}

// voxel segments of a cloud in the ds buffers: keys, stable sort, heads, ranks
static int ds_segments(vg_ctx* ctx, hipStream_t s, const float* x, const float* y, const float* z, int n,
                       double voxel) {
  DownsampleBufs& d = ctx->ds;
  k_ds_keys<<<grid_for(n), kBlock, 0, s>>>(n, x, y, z, voxel, d.keys, d.idx, d.flags);
  size_t tb = d.tmp_bytes;
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(d.tmp, tb, d.keys, d.keys_sorted, d.idx, d.idx_sorted, n, 0, 63, s));
  k_ds_heads<<<grid_for(n), kBlock, 0, s>>>(n, d.keys_sorted, d.head);
  tb = d.tmp_bytes;
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(d.tmp, tb, d.head, d.pos, n, s));
  k_ds_segs<<<grid_for(n), kBlock, 0, s>>>(n, d.head, d.pos, d.seg, d.flags);
  return VG_OK;
}

int ds_close(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* t, float tconst, int n,
             double voxel, float4* out, int* n_out) {
  DownsampleBufs& d = ctx->ds;
  hipStream_t s = ctx->stream;
  *n_out = 0;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  if (n <= 0) return VG_OK;
  VG_TRY(ds_segments(ctx, s, x, y, z, n, voxel));
  // the sorted pair buffers are free once the segments exist: time keys and
  // voxel ranks go into the key/index buffers, sorted into their twins
  uint32_t* tkey = reinterpret_cast<uint32_t*>(d.keys);
  uint32_t* tkey_s = reinterpret_cast<uint32_t*>(d.keys_sorted);
  k_close_pick<<<grid_for(n), kBlock, 0, s>>>(d.flags, d.seg, d.idx_sorted, x, y, z, t, tconst, d.ox, d.oy, d.oz,
                                              d.oi, tkey, d.idx);
  VG_HIP(hipMemcpyAsync(ctx->h_pinned, d.flags, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  VG_HIP(hipMemsetAsync(d.flags, 0, 4 * sizeof(int), s));
  VG_HIP(stream_wait(ctx));
  if (ctx->h_pinned[0]) {
    ctx->err = "voxel key out of packed range (|key| >= 2^20)";
    return VG_E_RANGE;
  }
  const int nv = ctx->h_pinned[1];
  size_t tb = d.tmp_bytes;
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(d.tmp, tb, tkey, tkey_s, d.idx, d.idx_sorted, nv, 0, 32, s));
  k_close_gather<<<grid_for(nv), kBlock, 0, s>>>(nv, d.idx_sorted, d.ox, d.oy, d.oz, d.oi, out);
  VG_HIP(hipGetLastError());
  VG_HIP(stream_wait(ctx));  // `out` is complete on return (callers copy it on other streams)
  *n_out = nv;
  return VG_OK;
}

// ---- the per-scan pipeline's downsample (down_sampling_voxel + the /2
// fallback, local_mapping.cpp:396-403) without a sort and without the host:
//  1. k_hds_insert  one lane per point: the key, insert-or-find in an open
//                   addressing table, atomicMin of the voxel's first point
//                   index, atomicAdd of its point count;
//  2. k_hds_tiles   per 1024-point tile: first points and their voxels' points;
//  3. k_hds_rank    per tile: prefix over the earlier tiles + block scan ->
//                   each voxel's output rank (= order of first occurrence, so
//                   deterministic) and the offset of its point segment; the
//                   voxel count; the fallback flag (fewer than 2000 voxels);
//  4. k_hds_scatter point indices into their voxel's segment (atomic slots);
//  5. k_hds_mean    one lane per voxel: insertion-sorts its segment back to
//                   input order, runs the reference's float recurrence
//                   (bit-identical to k_ds_mean), writes the voxel at its rank
//                   and clears its table slot for the next scan.
// The fallback pass at half the voxel size is enqueued behind it on the same
// stream and early-exits on the device flag, so no count ever travels to the
// host. Output order = first-occurrence order (the sorted path's is key order;
// the reference's is unordered_map order: the set is the same).
__device__ __forceinline__ uint32_t hds_hash(uint64_t k, int mask) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (uint32_t)k & (uint32_t)mask;
}
constexpr int kHdsTile = 1024;  // points per tile (256 lanes x 4)
constexpr int kHdsSmall = 16;   // a lane sorts a voxel's segment itself (in registers) up to this many points
constexpr int kHdsMid = 256;    // a wave puts a voxel's segment back in order (LDS ranks) up to this many
static_assert(kRcpN > kHdsMid, "the reciprocal table covers a mid-size voxel");
constexpr int kHdsEmptyFirst = 0x7f7f7f7f;  // above every point index (ds_reset's memset byte)

// the scan's input cloud as a kernel argument -> device memory, so that the
// chain behind it (captured once as a graph) reads it from there
__global__ void k_hds_args(HdsIn* __restrict__ dst, HdsIn a) {
  if (threadIdx.x == 0) *dst = a;
}

__global__ void __launch_bounds__(256) k_hds_insert(double size, DownsampleBufs d, const int* __restrict__ need) {
  if (need && !*need) return;
  const HdsIn a = *d.arg;
  const float *x = a.x, *y = a.y, *z = a.z;
  const int n = a.n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int64_t kx = key_axis_f(x[i], size) + kKeyOff;
    int64_t ky = key_axis_f(y[i], size) + kKeyOff;
    int64_t kz = key_axis_f(z[i], size) + kKeyOff;
    const bool bad = (kx < 0) | (ky < 0) | (kz < 0) | (kx >= 2 * kKeyOff) | (ky >= 2 * kKeyOff) | (kz >= 2 * kKeyOff);
    if (bad) {
      atomicOr(&d.hflags[0], 1);
      kx = ky = kz = 0;
    }
    const uint64_t key = ((uint64_t)kx << 42) | ((uint64_t)ky << 21) | (uint64_t)kz;
    uint32_t s = hds_hash(key, d.hmask);
    while (true) {
      const unsigned long long prev =
          atomicCAS((unsigned long long*)&d.hkey[s], (unsigned long long)kKeyEmpty, (unsigned long long)key);
      if (prev == kKeyEmpty || prev == key) break;
      s = (s + 1) & (uint32_t)d.hmask;
    }
    atomicMin(&d.hfirst[s], i);
    atomicAdd(&d.hcnt[s], 1);
    d.pslot[i] = s;
  }
}

// (first point?, its voxel's point count) of point i
__device__ __forceinline__ void hds_code(const DownsampleBufs& d, int i, int n, int& f, int& c) {
  f = 0;
  c = 0;
  if (i >= n) return;
  const uint32_t s = d.pslot[i];
  if (d.hfirst[s] == i) {
    f = 1;
    c = d.hcnt[s];
  }
}

__global__ void __launch_bounds__(256) k_hds_tiles(DownsampleBufs d, const int* __restrict__ need) {
  if (need && !*need) return;
  const int n = d.arg->n;
  if ((int)blockIdx.x * kHdsTile >= n) return;  // the grid covers the capacity
  __shared__ int s_f[4], s_c[4];
  const int i0 = blockIdx.x * kHdsTile + threadIdx.x * 4;
  int F = 0, C = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int f, c;
    hds_code(d, i0 + k, n, f, c);
    F += f;
    C += c;
  }
  for (int o = 32; o > 0; o >>= 1) {
    F += __shfl_down(F, o, 64);
    C += __shfl_down(C, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_f[threadIdx.x >> 6] = F;
    s_c[threadIdx.x >> 6] = C;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    d.tsum[2 * blockIdx.x] = s_f[0] + s_f[1] + s_f[2] + s_f[3];
    d.tsum[2 * blockIdx.x + 1] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
  }
}

// need_in: this pass's predicate (nullptr: always); need_out: the fallback flag
// this pass decides (nullptr: none)
__global__ void __launch_bounds__(256) k_hds_rank(DownsampleBufs d, const int* __restrict__ need_in,
                                                  int* __restrict__ need_out, int min_out) {
  if (need_in && !*need_in) return;
  const int n = d.arg->n, ntile = (n + kHdsTile - 1) / kHdsTile;
  if ((int)blockIdx.x >= ntile) return;  // the grid covers the capacity
  __shared__ unsigned long long s_w[4];
  __shared__ int s_b[2][4];
  // prefix of the earlier tiles (first points, points)
  int bf = 0, bc = 0;
  for (int t = threadIdx.x; t < (int)blockIdx.x; t += blockDim.x) {
    bf += d.tsum[2 * t];
    bc += d.tsum[2 * t + 1];
  }
  for (int o = 32; o > 0; o >>= 1) {
    bf += __shfl_down(bf, o, 64);
    bc += __shfl_down(bc, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    s_b[0][wv] = bf;
    s_b[1][wv] = bc;
  }
  __syncthreads();
  bf = s_b[0][0] + s_b[0][1] + s_b[0][2] + s_b[0][3];
  bc = s_b[1][0] + s_b[1][1] + s_b[1][2] + s_b[1][3];
  // exclusive scan of (f, c) packed in 64 bits (c < 2^32: points per scan)
  const int i0 = blockIdx.x * kHdsTile + threadIdx.x * 4;
  int f[4], c[4];
  unsigned long long v = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    hds_code(d, i0 + k, n, f[k], c[k]);
    v += ((unsigned long long)f[k] << 32) | (unsigned long long)c[k];
  }
  unsigned long long x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long yv = __shfl_up(x, o, 64);
    if (lane >= o) x += yv;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  unsigned long long base = 0, tot = 0;
  for (int k = 0; k < 4; k++) {
    if (k < wv) base += s_w[k];
    tot += s_w[k];
  }
  unsigned long long r = base + x - v;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (f[k]) {
      const uint32_t s = d.pslot[i0 + k];
      const int v = bf + (int)(r >> 32);
      d.hrank[s] = v;
      d.hoff[s] = bc + (int)(r & 0xffffffffull);
      d.vfirst[v] = i0 + k;  // k_hds_mean walks the voxels, not the points
    }
    r += ((unsigned long long)f[k] << 32) | (unsigned long long)c[k];
  }
  if (blockIdx.x == ntile - 1 && threadIdx.x == 0) {
    const int nv = bf + (int)(tot >> 32);
    d.hflags[1] = nv;
    d.hflags[3] = 0;  // dense voxels deferred by k_hds_mean
    d.hflags[4] = 0;  // mid-size voxels deferred by k_hds_mean
    if (need_out) *need_out = nv < min_out ? 1 : 0;
  }
}

__global__ void __launch_bounds__(256) k_hds_scatter(DownsampleBufs d, const int* __restrict__ need) {
  if (need && !*need) return;
  const int n = d.arg->n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = d.pslot[i];
    const int pos = atomicAdd(&d.hfill[s], 1);
    d.pseg[d.hoff[s] + pos] = (uint32_t)i;
  }
}

// A voxel's segment (N >= cnt point indices, padded with ~0u) back to input
// order in registers — a static Batcher odd-even merge network, no memory
// traffic — then the reference's float recurrence over the points in that
// order (point_utils.hpp:34-37, evaluated exactly as written, no contraction).
template <int N>
__device__ __forceinline__ void hds_sorted_mean(const uint32_t* __restrict__ sg, int cnt, const float* __restrict__ x,
                                                const float* __restrict__ y, const float* __restrict__ z,
                                                float& px, float& py, float& pz, float& c) {
  uint32_t u[N];
#pragma unroll
  for (int a = 0; a < N; a++) u[a] = a < cnt ? sg[a] : ~0u;
#pragma unroll
  for (int p = 1; p < N; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k; i++)
          if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const uint32_t lo = u[i + j] < u[i + j + k] ? u[i + j] : u[i + j + k];
            const uint32_t hi = u[i + j] < u[i + j + k] ? u[i + j + k] : u[i + j];
            u[i + j] = lo;
            u[i + j + k] = hi;
          }
  float vx[N], vy[N], vz[N];  // the loads are independent of the recurrence: issue them all first
#pragma unroll
  for (int a = 0; a < N; a++)
    if (a < cnt) {
      vx[a] = x[u[a]];
      vy[a] = y[u[a]];
      vz[a] = z[u[a]];
    }
  px = vx[0];
  py = vy[0];
  pz = vz[0];
  c = 1.0f;
#pragma unroll
  for (int a = 1; a < N; a++)
    if (a < cnt) {
      const double r = kRcp.v[a];  // c == a
      px = mean_step(px, c, vx[a], r);
      py = mean_step(py, c, vy[a], r);
      pz = mean_step(pz, c, vz[a], r);
      c += 1;
    }
}

__global__ void __launch_bounds__(256) k_hds_mean(DownsampleBufs d, const int* __restrict__ need) {
  if (need && !*need) return;
  const HdsIn a = *d.arg;
  const float *__restrict__ x = a.x, *__restrict__ y = a.y, *__restrict__ z = a.z, *__restrict__ in = a.in;
  const int nv = d.hflags[1];
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gridDim.x * blockDim.x) {
    const int i = d.vfirst[v];
    const uint32_t s = d.pslot[i];
    const int b = d.hoff[s], cnt = d.hcnt[s];
    if (cnt > kHdsSmall) {  // mid-size: a wave puts it back in order (k_hds_mid); dense: a workgroup (k_hds_big)
      if (cnt <= kHdsMid) d.bigv[d.cap - 1 - atomicAdd(&d.hflags[4], 1)] = v;
      else d.bigv[atomicAdd(&d.hflags[3], 1)] = v;
      continue;
    }
    const uint32_t* sg = d.pseg + b;
    float px, py, pz, c;
    if (cnt <= 2) hds_sorted_mean<2>(sg, cnt, x, y, z, px, py, pz, c);
    else if (cnt <= 4) hds_sorted_mean<4>(sg, cnt, x, y, z, px, py, pz, c);
    else if (cnt <= 8) hds_sorted_mean<8>(sg, cnt, x, y, z, px, py, pz, c);
    else hds_sorted_mean<kHdsSmall>(sg, cnt, x, y, z, px, py, pz, c);
    d.ox[v] = px;
    d.oy[v] = py;
    d.oz[v] = pz;
    d.oi[v] = in ? in[i] : 0.0f;
    d.oc[v] = c;
    d.hkey[s] = kKeyEmpty;  // the slot is this lane's alone: clear it for the next run
    d.hfirst[s] = kHdsEmptyFirst;
    d.hcnt[s] = 0;
    d.hfill[s] = 0;
  }
}

// Mid-size voxels (kHdsSmall < points <= kHdsMid): one wave each. The
// segment's point indices go to LDS, each lane ranks its (up to four) indices
// against the whole segment (distinct indices: rank = input order), the
// coordinates are gathered in that order into LDS, and lanes 0..2 run the x, y
// and z recurrences (point_utils.hpp:34-37, mean_step).
__global__ void __launch_bounds__(256) k_hds_mid(DownsampleBufs d, const int* __restrict__ need) {
  if (need && !*need) return;
  const HdsIn a = *d.arg;
  __shared__ __attribute__((aligned(16))) uint32_t s_idx[4][kHdsMid];
  __shared__ uint32_t s_ord[4][kHdsMid];
  __shared__ float s_c[4][3][kHdsMid];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nmid = d.hflags[4];
  for (int q = blockIdx.x * 4 + w; q < nmid; q += gridDim.x * 4) {
    const int v = d.bigv[d.cap - 1 - q];
    const int i0 = d.vfirst[v];
    const uint32_t s = d.pslot[i0];
    const int b = d.hoff[s], cnt = d.hcnt[s];
    uint32_t u[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int e = lane + 64 * k;
      u[k] = e < cnt ? d.pseg[b + e] : 0xffffffffu;
      s_idx[w][e] = u[k];
    }
    wave_lds_sync();
    int r[4] = {0, 0, 0, 0};
    const uint4* s4 = reinterpret_cast<const uint4*>(s_idx[w]);
    for (int j = 0; j < (cnt + 3) >> 2; j++) {
      const uint4 t = s4[j];
#pragma unroll
      for (int k = 0; k < 4; k++) r[k] += (t.x < u[k]) + (t.y < u[k]) + (t.z < u[k]) + (t.w < u[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (lane + 64 * k < cnt) s_ord[w][r[k]] = u[k];
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int e = lane + 64 * k;
      if (e < cnt) {
        const uint32_t i = s_ord[w][e];
        s_c[w][0][e] = a.x[i];
        s_c[w][1][e] = a.y[i];
        s_c[w][2][e] = a.z[i];
      }
    }
    wave_lds_sync();
    if (lane < 3) {
      const float* cv = s_c[w][lane];
      float p = cv[0], c = 1.0f;
#pragma unroll 4
      for (int e = 1; e < cnt; e++) {
        p = mean_step(p, c, cv[e], kRcp.v[e]);  // c == e
        c += 1.0f;
      }
      (lane == 0 ? d.ox : (lane == 1 ? d.oy : d.oz))[v] = p;
      if (lane == 0) {
        d.oi[v] = a.in ? a.in[i0] : 0.0f;
        d.oc[v] = c;
        d.hkey[s] = kKeyEmpty;
        d.hfirst[s] = kHdsEmptyFirst;
        d.hcnt[s] = 0;
        d.hfill[s] = 0;
      }
    }
    wave_lds_sync();
  }
}

// Dense voxels (more than kHdsSmall points): one workgroup each restores the
// input order of the voxel's segment with an LDS bitmap over its index range
// (windows of kHdsBits indices; set bits compacted by a block scan — O(points +
// range/32), exact for any size), then three lanes run the x, y and z
// recurrences (the same arithmetic as k_hds_mean, bit for bit).
constexpr int kHdsBits = 1 << 18;          // indices per bitmap window (32 KB of LDS)
constexpr int kHdsWords = kHdsBits / 32;
// one dense voxel v by the whole workgroup (any size, a multiple of 64 that
// divides kHdsWords); bm: kHdsWords LDS words, s_w: one int per wave
constexpr int kHdsChunk = 2048;  // ordered points per LDS chunk of the recurrence
__device__ void hds_big_voxel(DownsampleBufs& d, int v, const float* x, const float* y, const float* z, const float* in,
                              uint32_t* bm, int* s_w, int* s_base, float* cb, double* rb) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = blockDim.x, nw = nt >> 6;
  const int i0 = d.vfirst[v];  // the voxel's smallest index
  const uint32_t s = d.pslot[i0];
  const int b = d.hoff[s], cnt = d.hcnt[s];
  const uint32_t* sg = d.pseg + b;
  uint32_t* out = d.pseg2 + b;
  int hi = i0;
  for (int e = tid; e < cnt; e += nt) hi = max(hi, (int)sg[e]);
  for (int o = 32; o > 0; o >>= 1) hi = max(hi, __shfl_down(hi, o, 64));
  if (lane == 0) s_w[wv] = hi;
  __syncthreads();
  hi = s_w[0];
  for (int k = 1; k < nw; k++) hi = max(hi, s_w[k]);
  if (tid == 0) *s_base = 0;
  __syncthreads();
  for (int w0 = i0; w0 <= hi; w0 += kHdsBits) {
    for (int k = tid; k < kHdsWords; k += nt) bm[k] = 0u;
    __syncthreads();
    for (int e = tid; e < cnt; e += nt) {
      const int off = (int)sg[e] - w0;
      if (off >= 0 && off < kHdsBits) atomicOr(&bm[off >> 5], 1u << (off & 31));
    }
    __syncthreads();
    const int per = kHdsWords / nt;  // words per thread, contiguous
    int mine = 0;
    for (int k = 0; k < per; k++) mine += __popc(bm[tid * per + k]);
    int xs = mine;  // block exclusive scan
    for (int o = 1; o < 64; o <<= 1) {
      const int yv = __shfl_up(xs, o, 64);
      if (lane >= o) xs += yv;
    }
    __syncthreads();
    if (lane == 63) s_w[wv] = xs;
    __syncthreads();
    int base = *s_base;
    for (int k = 0; k < wv; k++) base += s_w[k];
    base += xs - mine;
    for (int k = 0; k < per; k++) {
      uint32_t m = bm[tid * per + k];
      while (m) {
        const int bit = __ffs(m) - 1;
        m &= m - 1;
        out[base++] = (uint32_t)(w0 + (tid * per + k) * 32 + bit);
      }
    }
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int k = 0; k < nw; k++) t += s_w[k];
      *s_base += t;
    }
    __syncthreads();
  }
  // point_utils.hpp:34-37 per coordinate (mean_step): the ordered points'
  // coordinates and the fp64 reciprocals staged in LDS chunks by the whole
  // workgroup, lanes 0..2 walking each chunk
  float p = 0.0f, c = 1.0f;
  for (int e0 = 0; e0 < cnt; e0 += kHdsChunk) {
    const int m = cnt - e0 < kHdsChunk ? cnt - e0 : kHdsChunk;
    for (int e = tid; e < m; e += nt) {
      const uint32_t i = out[e0 + e];
      cb[e] = x[i];
      cb[kHdsChunk + e] = y[i];
      cb[2 * kHdsChunk + e] = z[i];
      rb[e] = 1.0 / (double)(e0 + e + 1);
    }
    __syncthreads();
    if (tid < 3) {
      const float* cv = cb + tid * kHdsChunk;
      int e = 0;
      if (e0 == 0) {
        p = cv[0];
        e = 1;
      }
#pragma unroll 4
      for (; e < m; e++) {
        p = mean_step(p, c, cv[e], rb[e]);  // c == e0 + e
        c += 1.0f;
      }
    }
    __syncthreads();
  }
  if (tid < 3) {
    (tid == 0 ? d.ox : (tid == 1 ? d.oy : d.oz))[v] = p;
    if (tid == 0) {
      d.oi[v] = in ? in[i0] : 0.0f;
      d.oc[v] = c;
    }
  }
  __syncthreads();
  if (tid == 0) {
    d.hkey[s] = kKeyEmpty;
    d.hfirst[s] = kHdsEmptyFirst;
    d.hcnt[s] = 0;
    d.hfill[s] = 0;
  }
}

// Dense voxels (more than kHdsSmall points): one workgroup each restores the
// input order of the voxel's segment with an LDS bitmap over its index range
// (windows of kHdsBits indices; set bits compacted by a block scan — O(points +
// range/32), exact for any size), then three lanes run the x, y and z
// recurrences (the same arithmetic as k_hds_mean, bit for bit).
__global__ void __launch_bounds__(256) k_hds_big(DownsampleBufs d, const int* __restrict__ need) {
  if (need && !*need) return;
  const HdsIn a = *d.arg;
  __shared__ uint32_t bm[kHdsWords];
  __shared__ float cb[3 * kHdsChunk];
  __shared__ double rb[kHdsChunk];
  __shared__ int s_w[4], s_base;
  const int nbig = d.hflags[3];
  for (int q = blockIdx.x; q < nbig; q += gridDim.x)
    hds_big_voxel(d, d.bigv[q], a.x, a.y, a.z, a.in, bm, s_w, &s_base, cb, rb);
}

// The /2 fallback pass of local_mapping.cpp:399-403 as ONE workgroup (it is
// needed only when the first pass kept fewer than 2000 voxels): the first four
// steps of k_hds_insert .. k_hds_mean, separated by workgroup barriers instead
// of kernel boundaries, the ranks by a block scan over the points in 1024-point
// tiles, so the output (order, float means) is bit for bit the multi-kernel
// pass's; its dense voxels go to the k_hds_big launch behind it (256
// workgroups, not one after the other). On the common path it is two
// early-exiting launches instead of seven.
constexpr int kHdsFbThreads = 1024;
__global__ void __launch_bounds__(kHdsFbThreads) k_hds_fallback(double size, DownsampleBufs d,
                                                                const int* __restrict__ need) {
  if (!*need) return;
  __shared__ unsigned long long s_w64[kHdsFbThreads / 64];
  const HdsIn a = *d.arg;
  const float *x = a.x, *y = a.y, *z = a.z, *in = a.in;
  const int n = a.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = kHdsFbThreads / 64;
  // 1. keys, insert-or-find, first index, count (k_hds_insert)
  for (int i = tid; i < n; i += kHdsFbThreads) {
    int64_t kx = key_axis_f(x[i], size) + kKeyOff;
    int64_t ky = key_axis_f(y[i], size) + kKeyOff;
    int64_t kz = key_axis_f(z[i], size) + kKeyOff;
    const bool bad = (kx < 0) | (ky < 0) | (kz < 0) | (kx >= 2 * kKeyOff) | (ky >= 2 * kKeyOff) | (kz >= 2 * kKeyOff);
    if (bad) {
      atomicOr(&d.hflags[0], 1);
      kx = ky = kz = 0;
    }
    const uint64_t key = ((uint64_t)kx << 42) | ((uint64_t)ky << 21) | (uint64_t)kz;
    uint32_t s = hds_hash(key, d.hmask);
    while (true) {
      const unsigned long long prev =
          atomicCAS((unsigned long long*)&d.hkey[s], (unsigned long long)kKeyEmpty, (unsigned long long)key);
      if (prev == kKeyEmpty || prev == key) break;
      s = (s + 1) & (uint32_t)d.hmask;
    }
    atomicMin(&d.hfirst[s], i);
    atomicAdd(&d.hcnt[s], 1);
    d.pslot[i] = s;
  }
  __syncthreads();
  // 2. ranks in first-occurrence order and segment offsets (k_hds_tiles + k_hds_rank)
  int bf = 0, bc = 0;  // first points / points of the earlier tiles
  for (int t0 = 0; t0 < n; t0 += kHdsFbThreads) {
    const int i = t0 + tid;
    int f, c;
    hds_code(d, i, n, f, c);
    const unsigned long long v = ((unsigned long long)f << 32) | (unsigned long long)c;
    unsigned long long xs = v;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long yv = __shfl_up(xs, o, 64);
      if (lane >= o) xs += yv;
    }
    if (lane == 63) s_w64[wv] = xs;
    __syncthreads();
    unsigned long long base = 0, tot = 0;
    for (int k = 0; k < nw; k++) {
      if (k < wv) base += s_w64[k];
      tot += s_w64[k];
    }
    const unsigned long long r = base + xs - v;
    if (f) {
      const uint32_t s = d.pslot[i];
      const int rk = bf + (int)(r >> 32);
      d.hrank[s] = rk;
      d.hoff[s] = bc + (int)(r & 0xffffffffull);
      d.vfirst[rk] = i;
    }
    bf += (int)(tot >> 32);
    bc += (int)(tot & 0xffffffffull);
    __syncthreads();
  }
  const int nv = bf;
  if (tid == 0) {
    d.hflags[1] = nv;
    d.hflags[3] = 0;
  }
  __syncthreads();
  // 3. point indices into their voxel's segment (k_hds_scatter)
  for (int i = tid; i < n; i += kHdsFbThreads) {
    const uint32_t s = d.pslot[i];
    const int pos = atomicAdd(&d.hfill[s], 1);
    d.pseg[d.hoff[s] + pos] = (uint32_t)i;
  }
  __syncthreads();
  // 4. small voxels' means (k_hds_mean); dense ones listed for step 5
  for (int v = tid; v < nv; v += kHdsFbThreads) {
    const int i = d.vfirst[v];
    const uint32_t s = d.pslot[i];
    const int b = d.hoff[s], cnt = d.hcnt[s];
    if (cnt > kHdsSmall) {  // dense: k_hds_big behind this launch, one workgroup each
      d.bigv[atomicAdd(&d.hflags[3], 1)] = v;
      continue;
    }
    const uint32_t* sg = d.pseg + b;
    float px, py, pz, c;
    if (cnt <= 2) hds_sorted_mean<2>(sg, cnt, x, y, z, px, py, pz, c);
    else if (cnt <= 4) hds_sorted_mean<4>(sg, cnt, x, y, z, px, py, pz, c);
    else if (cnt <= 8) hds_sorted_mean<8>(sg, cnt, x, y, z, px, py, pz, c);
    else hds_sorted_mean<kHdsSmall>(sg, cnt, x, y, z, px, py, pz, c);
    d.ox[v] = px;
    d.oy[v] = py;
    d.oz[v] = pz;
    d.oi[v] = in ? in[i] : 0.0f;
    d.oc[v] = c;
    d.hkey[s] = kKeyEmpty;
    d.hfirst[s] = kHdsEmptyFirst;
    d.hcnt[s] = 0;
    d.hfill[s] = 0;
  }
  // 5. dense voxels: the k_hds_big launch behind this one (gated on the same flag)
}

// the pipeline's downsample, asynchronous on stream s; with `fallback`, the
// /2 pass of local_mapping.cpp:399-403 runs on the device when fewer than
// 2000 voxels came out. hflags[1] = the voxel count (device), published to
// Pub (seq_ds) when pub_seq > 0.
int ds_enqueue_hashed(vg_ctx* ctx, hipStream_t s, const float* x, const float* y, const float* z, const float* in,
                      int n, double voxel, bool fallback, int pub_seq) {
  DownsampleBufs& d = ctx->ds;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  int* need = d.hflags + 2;
  if (n == 0) {
    VG_HIP(hipMemsetAsync(d.hflags + 1, 0, 2 * sizeof(int), s));
  } else {
    k_hds_args<<<1, 64, 0, s>>>(d.arg, HdsIn{x, y, z, in, n, 0});
    // every count and size below is read on the device (grids cover the
    // context's capacity, surplus blocks exit), so the chain is one graph
    // per (voxel, fallback), replayed for every scan: one launch instead of 12
    const int cap = ctx->cap.max_points_per_scan;
    const int g = grid_for(cap, kBlock, 1024), ntile = (cap + kHdsTile - 1) / kHdsTile;
    auto chain = [&](hipStream_t st) {
      k_hds_insert<<<g, kBlock, 0, st>>>(voxel, d, nullptr);
      k_hds_tiles<<<ntile, kBlock, 0, st>>>(d, nullptr);
      k_hds_rank<<<ntile, kBlock, 0, st>>>(d, nullptr, fallback ? need : nullptr, 2000);
      k_hds_scatter<<<g, kBlock, 0, st>>>(d, nullptr);
      k_hds_mean<<<g, kBlock, 0, st>>>(d, nullptr);
      k_hds_mid<<<grid_for(cap / kHdsSmall + 1, kBlock / 64, 256), kBlock, 0, st>>>(d, nullptr);
      k_hds_big<<<256, kBlock, 0, st>>>(d, nullptr);
      if (fallback) {
        k_hds_fallback<<<1, kHdsFbThreads, 0, st>>>(voxel / 2, d, need);
        k_hds_big<<<256, kBlock, 0, st>>>(d, need);
      }
    };
    const bool use_graph = ctx->use_graphs && fallback && voxel == ctx->cfg.down_size;
    if (use_graph && !ctx->g_ds) {
      std::lock_guard<std::recursive_mutex> cap_lk_(capture_mutex());  // (vg_internal.h)
      VG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      chain(s);
      hipGraph_t gr = nullptr;
      VG_HIP(hipStreamEndCapture(s, &gr));
      VG_HIP(hipGraphInstantiate(&ctx->g_ds, gr, nullptr, nullptr, 0));
      VG_HIP(hipGraphDestroy(gr));
    }
    if (use_graph) VG_HIP(hipGraphLaunch(ctx->g_ds, s));
    else chain(s);
  }
  if (pub_seq > 0) VG_TRY(state_publish_ds(ctx, s, pub_seq, d.hflags, false));
  VG_HIP(hipGetLastError());
  return VG_OK;
}

int ds_alloc(vg_ctx* ctx) {
  const int n = ctx->cap.max_points_per_scan;
  DownsampleBufs& d = ctx->ds;
  d.keys = ctx->arena.take<uint64_t>(n);
  d.keys_sorted = ctx->arena.take<uint64_t>(n);
  d.idx = ctx->arena.take<uint32_t>(n);
  d.idx_sorted = ctx->arena.take<uint32_t>(n);
  d.head = ctx->arena.take<uint32_t>(n);
  d.pos = ctx->arena.take<uint32_t>(n);
  d.seg = ctx->arena.take<uint32_t>(n + 1);
  d.ox = ctx->arena.take<float>(n);
  d.oy = ctx->arena.take<float>(n);
  d.oz = ctx->arena.take<float>(n);
  d.oi = ctx->arena.take<float>(n);
  d.oc = ctx->arena.take<float>(n);
  d.flags = ctx->arena.take<int>(4);
  d.arg = ctx->arena.take<HdsIn>(1);
  size_t b1 = 0, b2 = 0, b3 = 0;
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, d.keys, d.keys_sorted, d.idx, d.idx_sorted, n, 0, 63,
                                            ctx->stream));
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, d.head, d.pos, n, ctx->stream));
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b3, (uint32_t*)d.keys, (uint32_t*)d.keys_sorted, d.idx,
                                            d.idx_sorted, n, 0, 32, ctx->stream));  // ds_close's time sort
  d.tmp_bytes = std::max(b1, std::max(b2, b3));
  d.tmp = ctx->arena.take<char>(d.tmp_bytes);
  int hs = 1024;
  while (hs < 2 * n) hs <<= 1;
  d.hmask = hs - 1;
  d.hkey = ctx->arena.take<uint64_t>(hs);
  d.hfirst = ctx->arena.take<int>(hs);
  d.hcnt = ctx->arena.take<int>(hs);
  d.hfill = ctx->arena.take<int>(hs);
  d.hrank = ctx->arena.take<int>(hs);
  d.hoff = ctx->arena.take<int>(hs);
  d.pslot = ctx->arena.take<uint32_t>(n);
  d.pseg = ctx->arena.take<uint32_t>(n);
  d.vfirst = ctx->arena.take<int>(n);
  d.bigv = ctx->arena.take<int>(n);
  d.pseg2 = ctx->arena.take<uint32_t>(n);
  d.tsum = ctx->arena.take<int>(2 * ((size_t)n / kHdsTile + 2));
  d.hflags = ctx->arena.take<int>(8);
  d.cap = n;
  if (!d.keys || !d.seg || !d.oc || !d.tmp || !d.hkey || !d.hoff || !d.pseg || !d.tsum || !d.hflags) {
    ctx->err = "arena exhausted (downsample)";
    return VG_E_CAPACITY;
  }
  return VG_OK;
}

int ds_enqueue(vg_ctx* ctx, hipStream_t s, const float* x, const float* y, const float* z, const float* in, int n,
               double voxel, int pub_seq) {
  DownsampleBufs& d = ctx->ds;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  // d.flags are zero here: zeroed at creation and by every k_publish_ds / ds_run
  if (n > 0) {
    VG_TRY(ds_segments(ctx, s, x, y, z, n, voxel));
    k_ds_mean<<<grid_for(n), kBlock, 0, s>>>(d.flags, d.seg, d.idx_sorted, x, y, z, in, d.ox, d.oy, d.oz, d.oi,
                                             d.oc);
  }
  if (pub_seq > 0) VG_TRY(state_publish_ds(ctx, s, pub_seq, d.flags, true));
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// the hashed downsample's tables at rest: empty keys, no first points, zero
// counts (vg_create, vg_reset; k_hds_mean restores this after every run)
int ds_reset(vg_ctx* ctx) {
  DownsampleBufs& d = ctx->ds;
  hipStream_t s = ctx->stream;
  const size_t hs = (size_t)d.hmask + 1;
  VG_HIP(hipMemsetAsync(d.hkey, 0xff, hs * sizeof(uint64_t), s));
  VG_HIP(hipMemsetAsync(d.hfirst, 0x7f, hs * sizeof(int), s));  // 0x7f7f7f7f: above every point index
  VG_HIP(hipMemsetAsync(d.hcnt, 0, hs * sizeof(int), s));
  VG_HIP(hipMemsetAsync(d.hfill, 0, hs * sizeof(int), s));
  VG_HIP(hipMemsetAsync(d.hflags, 0, 8 * sizeof(int), s));
  VG_HIP(hipStreamSynchronize(s));
  return VG_OK;
}

int ds_run(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* in, int n, double voxel,
           int* n_out) {
  DownsampleBufs& d = ctx->ds;
  hipStream_t s = ctx->stream;
  if (n <= 0) {
    *n_out = 0;
    return VG_OK;
  }
  VG_TRY(ds_enqueue(ctx, s, x, y, z, in, n, voxel, 0));
  VG_HIP(hipMemcpyAsync(ctx->h_pinned, d.flags, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  VG_HIP(hipMemsetAsync(d.flags, 0, 4 * sizeof(int), s));
  VG_HIP(stream_wait(ctx));
  if (ctx->h_pinned[0]) {
    ctx->err = "voxel key out of packed range (|key| >= 2^20)";
    return VG_E_RANGE;
  }
  *n_out = ctx->h_pinned[1];
  return VG_OK;
}

}  // namespace vg
