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
  size_t b1 = 0, b2 = 0;
  VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, d.keys, d.keys_sorted, d.idx, d.idx_sorted, n, 0, 63,
                                            ctx->stream));
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, d.head, d.pos, n, ctx->stream));
  d.tmp_bytes = b1 > b2 ? b1 : b2;
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
    k_ds_keys<<<grid_for(n), kBlock, 0, s>>>(n, x, y, z, voxel, d.keys, d.idx, d.flags);
    size_t tb = d.tmp_bytes;
    VG_HIP(hipcub::DeviceRadixSort::SortPairs(d.tmp, tb, d.keys, d.keys_sorted, d.idx, d.idx_sorted, n, 0, 63, s));
    k_ds_heads<<<grid_for(n), kBlock, 0, s>>>(n, d.keys_sorted, d.head);
    tb = d.tmp_bytes;
    VG_HIP(hipcub::DeviceScan::ExclusiveSum(d.tmp, tb, d.head, d.pos, n, s));
    k_ds_segs<<<grid_for(n), kBlock, 0, s>>>(n, d.head, d.pos, d.seg, d.flags);
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
