// shard.cpp — spatial-tile sharding of one sequence across contexts (one per
// GPU): the collective transport behind the exchange points of map.hip / ba.hip
// (SURVEY §8(e)). Two transports:
//   RCCL  ncclAllReduce on the context stream (stream-ordered, no host sync);
//         `ncclComm_t` lives in the context.
//   host  a caller-supplied in-place host all-reduce (e.g. torch.distributed
//         gloo); the library synchronises the stream, stages through pinned
//         memory and copies the sum back. For tests and CPU-mediated transports.
#include <rccl/rccl.h>
#include <cstring>
#include "vg_internal.h"

namespace vg {

int shard_alloc(vg_ctx* ctx) {
  ctx->shard.d_buf = ctx->arena.take<double>(kShardBuf);
  if (!ctx->shard.d_buf) {
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

// sum-all-reduce of `count` elements (dtype 0 double, 1 int32), ordered on the
// context stream; send may equal recv
int shard_allreduce(vg_ctx* ctx, const void* send, void* recv, int count, int dtype) {
  Shard& sh = ctx->shard;
  if (sh.world <= 1 || count <= 0) return VG_OK;
  const size_t bytes = (size_t)count * (dtype == 0 ? 8 : 4);
  if (sh.mode == 1) {
    const ncclResult_t r = ncclAllReduce(send, recv, (size_t)count, dtype == 0 ? ncclFloat64 : ncclInt32, ncclSum,
                                         (ncclComm_t)sh.comm, ctx->stream);
    if (r != ncclSuccess) {
      ctx->err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
      return VG_E_HIP;
    }
    return VG_OK;
  }
  if (bytes > kShardBuf * sizeof(double)) {
    ctx->err = "shard_allreduce: message too large";
    return VG_E_ARG;
  }
  VG_HIP(hipMemcpyAsync(sh.h_buf, send, bytes, hipMemcpyDeviceToHost, ctx->stream));
  VG_HIP(stream_wait(ctx));
  if (sh.host_fn(sh.h_buf, count, dtype, sh.user) != 0) {
    ctx->err = "host all-reduce callback failed";
    return VG_E_HIP;
  }
  VG_HIP(hipMemcpyAsync(recv, sh.h_buf, bytes, hipMemcpyHostToDevice, ctx->stream));
  VG_HIP(stream_wait(ctx));  // the staging buffer is reused by the next exchange
  return VG_OK;
}

static int shard_common(vg_ctx* ctx, int rank, int world) {
  if (world < 1 || rank < 0 || rank >= world) {
    ctx->err = "vg_shard: rank/world out of range";
    return VG_E_ARG;
  }
  if (host_win_count(ctx) != 0 || ctx->shard.world > 1) {
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
  if (world == 1) return VG_OK;
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
  VG_HIP(hipHostMalloc((void**)&ctx->shard.h_buf, kShardBuf * sizeof(double), hipHostMallocDefault));
  ctx->shard.host_fn = fn;
  ctx->shard.user = user;
  ctx->shard.mode = 2;
  return VG_OK;
}

}  // extern "C"
