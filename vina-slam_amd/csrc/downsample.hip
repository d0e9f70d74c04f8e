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
      // point_utils.hpp:34-37, evaluated exactly as written (no contraction)
      px = (px * c + x[i]) / (c + 1);
      py = (py * c + y[i]) / (c + 1);
      pz = (pz * c + z[i]) / (c + 1);
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
  size_t b1 = 0, b2 = 0, b3 = 0;
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, d.keys, d.keys_sorted, d.idx, d.idx_sorted, n, 0, 63,
                                            ctx->stream));
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, d.head, d.pos, n, ctx->stream));
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b3, (uint32_t*)d.keys, (uint32_t*)d.keys_sorted, d.idx,
                                            d.idx_sorted, n, 0, 32, ctx->stream));  // ds_close's time sort
  d.tmp_bytes = std::max(b1, std::max(b2, b3));
  d.tmp = ctx->arena.take<char>(d.tmp_bytes);
  if (!d.keys || !d.seg || !d.oc || !d.tmp) {
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
  if (pub_seq > 0) VG_TRY(state_publish_ds(ctx, s, pub_seq));
  VG_HIP(hipGetLastError());
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
