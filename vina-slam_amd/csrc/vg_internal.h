// vg_internal.h — device context of the MI355X LIO hot path (not part of the
// C-ABI). One vg_ctx owns every device buffer of one LiDAR-inertial sequence:
// the scan staging area, the downsample workspace, the device-resident voxel
// map (root hash + octree node pool + per-slot window point arrays + point_fix
// arena) and the sliding-window state.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>
#include "../../include/vina_gpu.h"

#define VG_HIP(call)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ctx->err = std::string(#call) + ": " + hipGetErrorString(e_);                    \
      return VG_E_HIP;                                                                  \
    }                                                                                   \
  } while (0)

#define VG_TRY(expr)            \
  do {                          \
    int r_ = (expr);            \
    if (r_ != VG_OK) return r_; \
  } while (0)

namespace vg {

constexpr int kBlock = 256;
constexpr int64_t kKeyOff = 1 << 20;  // packed voxel key: 21 bits per axis
constexpr uint64_t kKeyEmpty = ~0ull;

inline int grid_for(long n, int block = kBlock, int cap = 8192) {
  long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// Bump allocator over one hipMalloc'd slab (16-byte aligned carve-outs).
struct Arena {
  char* base = nullptr;
  size_t size = 0, used = 0;
  template <class T>
  T* take(size_t n) {
    size_t b = (n * sizeof(T) + 255) & ~size_t(255);
    if (used + b > size) return nullptr;
    T* p = (T*)(base + used);
    used += b;
    return p;
  }
};

struct DownsampleBufs {
  uint64_t *keys = nullptr, *keys_sorted = nullptr;
  uint32_t *idx = nullptr, *idx_sorted = nullptr;
  uint32_t *head = nullptr, *pos = nullptr, *seg = nullptr;
  float *ox = nullptr, *oy = nullptr, *oz = nullptr, *oi = nullptr, *oc = nullptr;
  int* flags = nullptr;  // [0] range error, [1] n_out
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
};

}  // namespace vg

struct vg_ctx {
  vg_config cfg;
  vg_capacity cap;
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  vg::Arena arena;
  // raw scan staging (SoA)
  float *d_x = nullptr, *d_y = nullptr, *d_z = nullptr, *d_i = nullptr;
  vg::DownsampleBufs ds;
  int* h_pinned = nullptr;  // small pinned host scratch for counters
  vg_stats stats;
};

namespace vg {
// downsample.hip
int ds_alloc(vg_ctx* ctx);
// Voxel-grid downsample of a device-resident SoA cloud; results land in
// ctx->ds.o* (n_out voxels, ascending packed-key order). Host-synchronous
// (returns n_out).
int ds_run(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* in, int n, double voxel,
           int* n_out);
}  // namespace vg
