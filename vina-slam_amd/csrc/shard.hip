// shard.hip — spatial-tile sharding of one sequence across contexts (one per
// GPU): the collective transport behind the exchange points of map.hip / ba.hip
// (SURVEY §8(e)). Two transports:
//   RCCL  ncclAllReduce on the context stream (stream-ordered, no host sync);
//         `ncclComm_t` lives in the context.
//   host  a caller-supplied in-place host all-reduce (e.g. torch.distributed
//         gloo); the library synchronises the stream, stages through pinned
//         memory and copies the sum back. For tests and CPU-mediated transports.
//
// Exchange guard. Every all-reduce carries a frame of its call site's class
// (kShardSmall = 64 doubles for the IEKF's normal equations and the counts,
// Shard::frame_n for the LM's Hessian: the payload, ints as doubles, zeros,
// then the guard pair (x, x^2) with x = (seq mod 2^16) * 16 + site; seq is the
// device's count of this context's exchanges, site the call site). The summed
// pair equals (world x, world x^2) exactly when every rank sent the same x
// (sum over ranks of (x_r - x)^2 = 0; all terms < 2^44, exact in fp64), i.e.
// the ranks are at the same exchange of the same call site. A rank that
// enqueued a different exchange sequence gets VG_E_STATE ("sharded exchange
// out of step"), and the consumers of that exchange read zeros; within a
// frame class the out-of-step collectives still complete, so every rank
// reaches the error (ranks drifting across classes would pair frames of
// different sizes: the cost of not sending the 15 KB Hessian frame for every
// 34-value IEKF exchange).
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>
#include <cstring>
#include "vg_internal.h"

namespace vg {

__global__ void k_xchg_pack(const void* __restrict__ send, int count, int dtype, int site, int n,
                            double* __restrict__ frame, unsigned* __restrict__ seq) {
  for (int i = threadIdx.x; i < n - 2; i += blockDim.x)
    frame[i] = i < count ? (dtype == 0 ? static_cast<const double*>(send)[i]
                                       : (double)static_cast<const int*>(send)[i])
                         : 0.0;
  if (threadIdx.x == 0) {
    const unsigned s = *seq;
    *seq = s + 1;
    const double x = (double)((s & 0xffffu) * 16u + (unsigned)site);
    frame[n - 2] = x;
    frame[n - 1] = x * x;
    frame[n] = x;  // this rank's own x (not exchanged)
  }
}
__global__ void k_xchg_unpack(const double* __restrict__ frame, void* __restrict__ recv, int count, int dtype, int n,
                              int world, int* __restrict__ err) {
  const double x = frame[n];
  const bool ok = frame[n - 2] == world * x && frame[n - 1] == world * (x * x);
  if (!ok) {  // the consumers read zeros, not another exchange's (or a stale) sum
    if (threadIdx.x == 0) atomicOr(err, 32);
    for (int i = threadIdx.x; i < count; i += blockDim.x) {
      if (dtype == 0) static_cast<double*>(recv)[i] = 0.0;
      else static_cast<int*>(recv)[i] = 0;
    }
    return;
  }
  for (int i = threadIdx.x; i < count; i += blockDim.x) {
    if (dtype == 0) static_cast<double*>(recv)[i] = frame[i];
    else static_cast<int*>(recv)[i] = (int)llrint(frame[i]);
  }
}

int shard_alloc(vg_ctx* ctx) {
  ctx->shard.d_buf = ctx->arena.take<double>(kShardBuf);
  // the frame: the largest message (the LM's 6W x 6W LiDAR Hessian, gradient
  // and residual) + the guard pair + this rank's x; then the exchange counter
  const int W = ctx->cfg.win_size;
  ctx->shard.frame_n = 3 * W * (6 * W + 1) + 6 * W + 1 + 2;
  if (ctx->shard.frame_n < 64 + 2) ctx->shard.frame_n = 64 + 2;
  ctx->shard.d_frame = ctx->arena.take<double>((size_t)ctx->shard.frame_n + 2);
  ctx->shard.d_seq = ctx->arena.take<unsigned>(4);
  const size_t cap = (size_t)ctx->cap.max_points_per_scan;
  Shard& sh = ctx->shard;
  sh.keep_flag = ctx->arena.take<int>(cap);
  sh.keep_pos = ctx->arena.take<int>(cap);
  sh.keep_list = ctx->arena.take<int>(cap);
  sh.keep_rmax = ctx->arena.take<unsigned>(4);
  sh.keep_tmp_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sh.keep_tmp_bytes, (int*)nullptr, (int*)nullptr, (int)cap);
  sh.keep_tmp = ctx->arena.take<char>(sh.keep_tmp_bytes + 256);
  if (!ctx->shard.d_buf || !ctx->shard.d_frame || !ctx->shard.d_seq || !sh.keep_flag || !sh.keep_pos ||
      !sh.keep_list || !sh.keep_rmax || !sh.keep_tmp) {
    ctx->err = "arena exhausted (shard)";
    return VG_E_CAPACITY;
  }
  return VG_OK;
}

void shard_free(vg_ctx* ctx) {
  if (ctx->shard.comm) (void)ncclCommDestroy((ncclComm_t)ctx->shard.comm);
  ctx->shard.comm = nullptr;
  if (ctx->shard.h_buf) (void)hipHostFree(ctx->shard.h_buf);
  ctx->shard.h_buf = nullptr;
}

// sum-all-reduce of `count` elements (dtype 0 double, 1 int32) from call site
// `site` (< 16), ordered on the context stream, in the guarded frame; send may
// equal recv
int shard_allreduce(vg_ctx* ctx, const void* send, void* recv, int count, int dtype, int site) {
  Shard& sh = ctx->shard;
  if (sh.mode == 0 || count <= 0) return VG_OK;
  // the frame of the call site's class: the IEKF's normal equations and the
  // counts (<= 62 values) travel in a 64-double frame, the LM's Hessian in the
  // largest; a site always sends the same count, so ranks at the same exchange
  // agree on the size (the guard catches a rank at another exchange of the class)
  const int n = count <= kShardSmall - 2 ? kShardSmall : sh.frame_n;
  if (count > n - 2) {
    ctx->err = "shard_allreduce: message larger than the exchange frame";
    return VG_E_ARG;
  }
  k_xchg_pack<<<1, 256, 0, ctx->stream>>>(send, count, dtype, site, n, sh.d_frame, sh.d_seq);
  if (sh.mode == 1) {
    const ncclResult_t r =
        ncclAllReduce(sh.d_frame, sh.d_frame, (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)sh.comm, ctx->stream);
    if (r != ncclSuccess) {
      ctx->err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
      return VG_E_HIP;
    }
    // out of step: counters[kCntErr] bit 32, reported with the scan's counters (VG_E_STATE)
    k_xchg_unpack<<<1, 256, 0, ctx->stream>>>(sh.d_frame, recv, count, dtype, n, sh.world,
                                              ctx->map.counters + kCntErr);
    VG_HIP(hipGetLastError());
    return VG_OK;
  }
  VG_HIP(hipMemcpyAsync(sh.h_buf, sh.d_frame, (size_t)(n + 1) * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  VG_HIP(stream_wait(ctx));
  const double x = sh.h_buf[n];
  if (sh.host_fn(sh.h_buf, n, 0, sh.user) != 0) {
    ctx->err = "host all-reduce callback failed";
    return VG_E_HIP;
  }
  if (!(sh.h_buf[n - 2] == sh.world * x && sh.h_buf[n - 1] == sh.world * (x * x))) {
    ctx->err = "sharded exchange out of step: the ranks' exchange sequences differ (site " +
               std::to_string((int)x & 15) + ", exchange " + std::to_string((int)x >> 4) + " mod 2^16)";
    return VG_E_STATE;
  }
  sh.h_buf[n] = x;
  VG_HIP(hipMemcpyAsync(sh.d_frame, sh.h_buf, (size_t)(n + 1) * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  k_xchg_unpack<<<1, 256, 0, ctx->stream>>>(sh.d_frame, recv, count, dtype, n, sh.world,
                                            ctx->map.counters + kCntErr);
  VG_HIP(hipGetLastError());
  VG_HIP(stream_wait(ctx));  // the staging buffer is reused by the next exchange
  return VG_OK;
}

// the all-reduce of a frame its producer kernel packed (xchg_close) and its
// consumer kernel checks (xchg_ok): RCCL on the stream, or the host transport
// (which checks the guard itself as well, to fail at once)
int shard_exchange(vg_ctx* ctx, int n, hipStream_t s) {
  Shard& sh = ctx->shard;
  if (!s) s = ctx->stream;
  if (sh.mode == 1) {
    const ncclResult_t r =
        ncclAllReduce(sh.d_frame, sh.d_frame, (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)sh.comm, s);
    if (r != ncclSuccess) {
      ctx->err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
      return VG_E_HIP;
    }
    return VG_OK;
  }
  VG_HIP(hipMemcpyAsync(sh.h_buf, sh.d_frame, (size_t)(n + 1) * sizeof(double), hipMemcpyDeviceToHost, s));
  VG_HIP(stream_wait(ctx, s));
  const double x = sh.h_buf[n];
  if (sh.host_fn(sh.h_buf, n, 0, sh.user) != 0) {
    ctx->err = "host all-reduce callback failed";
    return VG_E_HIP;
  }
  if (!(sh.h_buf[n - 2] == sh.world * x && sh.h_buf[n - 1] == sh.world * (x * x))) {
    ctx->err = "sharded exchange out of step: the ranks' exchange sequences differ (site " +
               std::to_string((int)x & 15) + ", exchange " + std::to_string((int)x >> 4) + " mod 2^16)";
    return VG_E_STATE;
  }
  sh.h_buf[n] = x;
  VG_HIP(hipMemcpyAsync(sh.d_frame, sh.h_buf, (size_t)(n + 1) * sizeof(double), hipMemcpyHostToDevice, s));
  VG_HIP(stream_wait(ctx, s));  // the staging buffer is reused by the next exchange
  return VG_OK;
}

static int shard_common(vg_ctx* ctx, int rank, int world) {
  if (world < 1 || rank < 0 || rank >= world) {
    ctx->err = "vg_shard: rank/world out of range";
    return VG_E_ARG;
  }
  if (host_win_count(ctx) != 0 || ctx->shard.mode != 0) {
    ctx->err = "vg_shard: call once, before the first scan";
    return VG_E_STATE;
  }
  ctx->shard.rank = rank;
  ctx->shard.world = world;
  ctx->map.shard_rank = rank;
  ctx->map.shard_world = world;
  return VG_OK;
}

}  // namespace vg

using namespace vg;

extern "C" {

int vg_rccl_unique_id(void* id128) {
  if (!id128) return VG_E_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return VG_E_HIP;
  memcpy(id128, &id, sizeof(id));
  return VG_OK;
}

int vg_shard_rccl(vg_ctx* ctx, int rank, int world, const void* id128) {
  if (!ctx || !id128) return VG_E_ARG;
  VG_TRY(shard_common(ctx, rank, world));
  if (world == 1 && !ctx->shard_force) return VG_OK;  // (vgx_debug 30: the sharded path on one GPU)
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t comm;
  VG_HIP(hipSetDevice(ctx->device));
  const ncclResult_t r = ncclCommInitRank(&comm, world, id, rank);
  if (r != ncclSuccess) {
    ctx->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    ctx->shard.world = 1;
    ctx->map.shard_world = 1;
    return VG_E_HIP;
  }
  ctx->shard.comm = comm;
  ctx->shard.mode = 1;
  return VG_OK;
}

int vg_shard_host(vg_ctx* ctx, int rank, int world, vg_host_allreduce_fn fn, void* user) {
  if (!ctx || !fn) return VG_E_ARG;
  VG_TRY(shard_common(ctx, rank, world));
  if (world == 1) return VG_OK;
  VG_HIP(hipHostMalloc((void**)&ctx->shard.h_buf, ((size_t)ctx->shard.frame_n + 2) * sizeof(double),
                       hipHostMallocDefault));
  ctx->shard.host_fn = fn;
  ctx->shard.user = user;
  ctx->shard.mode = 2;
  return VG_OK;
}

}  // extern "C"
