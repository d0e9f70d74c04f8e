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
#include "vg_la.h"

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
// In measure mode (base == nullptr) take() only accumulates the size and hands
// out placeholder addresses, so vg_create can size the slab exactly.
struct Arena {
  char* base = nullptr;
  size_t size = 0, used = 0;
  bool measure = false;
  template <class T>
  T* take(size_t n) {
    size_t b = (n * sizeof(T) + 255) & ~size_t(255);
    if (measure) {
      T* p = (T*)(uintptr_t)(4096 + used);
      used += b;
      return p;
    }
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

// ---- device-resident voxel map (replaces unordered_map<VOXEL_LOC, OctoTree*>
// surf_map, octree.hpp:21-97, slide_window.hpp:6-20) ----
struct NodeHdr {            // 96 B: everything the correspondence descent reads
  double center[3];         // voxel_center
  int child[8];             // leaves[8] (-1 = none)
  float qlen;               // quater_length
  int8_t layer, octo, isexist, is_plane;
  int8_t has_sw, pad0, pad1, pad2;
  int opt_state, last_num;
  int fix_off, fix_cnt, fix_cap;
  int parent;
};
struct PlaneRec {           // 224 B: Plane (plane.hpp:5-24) as read by OctoTree::match
  double center[3], normal[3];
  double var[21];           // plane_var, packed upper 6x6
  float radius;
  int pad;
};
constexpr int kCovN = 45;   // cov_add packed upper 9x9

struct DevMap {
  int cap_nodes = 0, cap_fix = 0, hash_mask = 0, W = 0, cap_wp = 0;
  NodeHdr* hdr = nullptr;
  PlaneRec* pl = nullptr;
  Clu* pcr_add = nullptr;
  Clu* pcr_fix = nullptr;
  double* cov_add = nullptr;   // cap_nodes * 45
  double* eig = nullptr;       // cap_nodes * 12 (eig_value 3, eig_vector 9 row-major)
  double* jour = nullptr;
  Clu* pcrs = nullptr;         // cap_nodes * W (SlideWindow::pcrs_local, physical slot)
  int* nscr = nullptr;         // per-node scratch (cap_nodes * 4)
  int* cfirst = nullptr;       // per-node per-octant first-event scratch (cap_nodes * 8)
  uint64_t* hkey = nullptr;    // root hash
  int* hval = nullptr;
  int* hfirst = nullptr;
  int* slide = nullptr;        // surf_map_slide (root ids)
  uint8_t* in_slide = nullptr;
  double* fix_pnt = nullptr;   // point_fix arena: pnt (world) 3, var 6
  double* fix_var = nullptr;
  double* wp_pnt = nullptr;    // window points per physical slot: body pnt
  double* wp_var = nullptr;    // world var (after pvec_update), packed 6
  int* wp_leaf = nullptr;      // leaf holding the point in its list, -1 = not listed
  int* counters = nullptr;     // device counters (see kCnt*)
};
enum {
  kCntNodes = 0, kCntFix = 1, kCntSlide = 2, kCntNew = 3, kCntTouched = 4, kCntWork = 5, kCntNext = 6,
  kCntSub = 7, kCntEvents = 8, kCntFactors = 9, kCntCreate = 10, kCntErr = 11, kCntLeaves = 12, kCntMisc = 13, kCntSeg = 14, kCntRoots = 15,
  kCntN = 16
};

// per-scan work buffers
struct Work {
  int cap = 0;                 // entries
  uint64_t *k0 = nullptr, *k1 = nullptr;
  uint32_t *v0 = nullptr, *v1 = nullptr;
  uint32_t *u0 = nullptr, *u1 = nullptr;
  uint32_t* evsrc = nullptr;   // subdivision event source index
  uint32_t *ac_cnt = nullptr, *ac_off = nullptr;  // child allocation scratch
  int *list0 = nullptr, *list1 = nullptr, *list2 = nullptr, *cand = nullptr;
  int* leaf = nullptr;         // per ds point leaf / per event target
  double* pw = nullptr;        // per ds point world coords
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  double* partials = nullptr;  // reduction partials
  int* iekf_cache = nullptr;   // per raw point cached leaf
  int* rc = nullptr;           // device-side level counts (recut / margi, map.hip kRc*)
  int* plan = nullptr;         // per-leaf point_fix copy plan (margi)
  int nparts = 0;
};

// BA device buffers
struct BaBufs {
  int cap_f = 0;
  int* fac_node = nullptr;
  double* fac_eig = nullptr;   // trial eig values/vectors (12) per factor
  Clu* fac_pcr = nullptr;      // trial merged cluster per factor
  double* hpart = nullptr;     // chunk partials
  double* hout = nullptr;      // reduced 60x60 upper + 60 + 1
  double* rpart = nullptr;
  double* xs = nullptr;        // window poses (W x 12: R9 p3)
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
  // the scan the stage-level API works on (own staging or caller's HBM)
  const float *cur_x = nullptr, *cur_y = nullptr, *cur_z = nullptr, *cur_i = nullptr;
  int cur_n = -1;
  vg::DownsampleBufs ds;
  vg::DevMap map;
  vg::Work wk;
  vg::BaBufs ba;
  int* h_pinned = nullptr;  // small pinned host scratch for counters
  double* h_pinned_d = nullptr;
  double* h_zc = nullptr;         // host-mapped zero-copy results (k_iekf): 64 doubles + flag
  double* d_zc = nullptr;         // its device address
  int zc_seq = 0;

  vg_stats stats;
  void* host = nullptr;     // host-side pipeline state (pipeline.cpp)
  // stage timing with HIP events on the context stream (vg_profile)
  bool prof_on = false;      // k_iekf launch events (vg_profile bit 0)
  bool prof_stages = false;  // per-stage events (vg_profile bit 1)
  hipEvent_t prof_ev[8][2] = {};
  hipEvent_t sync_ev = nullptr;  // host-spin synchronisation (vg::stream_wait)
  hipEvent_t iekf_ev[8][2] = {};  // k_iekf launches since the last full sync (vg_profile)
  int iekf_ring_n = 0;
  hipEvent_t solve_ev[10][2] = {};  // k_ba_solve launches of the current BA run (vg_profile)
  int dbg_apply_cap = -1;        // test knob (vgx_debug): recut apply event capacity
  bool prof_pending[8] = {};
  double prof_ms[8] = {};
  int prof_n[8] = {};
};

namespace vg {
enum { kProfDownsample = 0, kProfIekfKernel = 1, kProfInsert = 2, kProfRecut = 3, kProfBA = 4, kProfMargi = 5,
       kProfIekf = 6, kProfBaSolve = 7, kProfN = 8 };
inline void prof_begin(vg_ctx* c, int id) {
  if (c->prof_stages) (void)hipEventRecord(c->prof_ev[id][0], c->stream);
}
inline void prof_end(vg_ctx* c, int id) {
  if (c->prof_stages) {
    (void)hipEventRecord(c->prof_ev[id][1], c->stream);
    c->prof_pending[id] = true;
  }
}
// Wait for the context stream by spinning on an event: a blocking
// hipStreamSynchronize may sleep and costs up to ~100+ us of wake-up latency
// per round trip, and the map stages make several per scan.
inline hipError_t stream_wait(vg_ctx* c) {
  hipError_t e = hipEventRecord(c->sync_ev, c->stream);
  if (e != hipSuccess) return e;
  while ((e = hipEventQuery(c->sync_ev)) == hipErrorNotReady) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  return e;
}
// call only after the stream has been synchronised past the recorded events
inline void prof_collect(vg_ctx* c) {
  for (int r = 0; r < c->iekf_ring_n; r++) {  // k_iekf launches (one event pair each)
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->iekf_ev[r][0], c->iekf_ev[r][1]) == hipSuccess) {
      c->prof_ms[kProfIekfKernel] += ms;
      c->prof_n[kProfIekfKernel] += 1;
    }
  }
  c->iekf_ring_n = 0;
  for (int i = 0; i < kProfN; i++)
    if (c->prof_pending[i]) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, c->prof_ev[i][0], c->prof_ev[i][1]) == hipSuccess) {
        c->prof_ms[i] += ms;
        c->prof_n[i] += 1;
      }
      c->prof_pending[i] = false;
    }
}
}  // namespace vg

namespace vg {
// Hot-path parameters in kernel-argument form (node.cpp:52-291 values).
struct MP {
  double vs;          // Odometry.voxel_size
  double min_eig;     // Odometry.min_eigen_value
  double thre[4];     // 1 / LocalBA.plane_eigen_value_thre (node.cpp:256-259)
  double minpt[4];    // min_point (node.cpp:219)
  double extR[9], extt[3];
  float dept, beam;   // dept_err / beam_err as the float params of calcBodyVar
  int max_layer, max_points, W, pad;
};

struct WinD {           // window poses x_buf (by ord) and the ring mp[] (octree.cpp:75)
  double R[32][9];
  double p[32][3];
  int mp[32];
  int win_count;
  int pad;
};

struct IekfPose {
  double R[9], p[3], rot_var[9], tsl_var[9];
};

struct InsPose {
  double R[9], p[3], rot_var[9], tsl_var[9];
};


// downsample.hip
int ds_alloc(vg_ctx* ctx);
// Voxel-grid downsample of a device-resident SoA cloud; results land in
// ctx->ds.o* (n_out voxels, ascending packed-key order). Host-synchronous
// (returns n_out).
int ds_run(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* in, int n, double voxel,
           int* n_out);
// map.hip
int map_alloc(vg_ctx* ctx);
int map_reset(vg_ctx* ctx);
int iekf_reset_cache(vg_ctx* ctx, int n);
int iekf_iter(vg_ctx* ctx, const MP& mp, const float* x, const float* y, const float* z, int n,
              const IekfPose& pose, double* out34);
int map_insert(vg_ctx* ctx, const MP& mp, int slot, const InsPose& pose, int n, int epoch, int thread_num,
               int* roots_new, int* touched);
int map_recut(vg_ctx* ctx, const MP& mp, const WinD& win, const int* nper, int thread_num, int* n_factors);
int map_margi(vg_ctx* ctx, const MP& mp, const WinD& win, int n_oldest, int thread_num, double jour);
// ba.hip
constexpr int kBaX = 24;        // per-frame state: R 9, p 3, v 3, bg 3, ba 3, g 3
constexpr int kBaImuRec = 64 + 225;
int ba_alloc(vg_ctx* ctx);
int ba_run(vg_ctx* ctx, int nf, const int* mp_ring, double* xs_io, const double* imurec, double* bias_io,
           int* iters);
// pipeline.cpp
void host_init(vg_ctx* ctx);
void host_free(vg_ctx* ctx);
void host_reset(vg_ctx* ctx);
void host_seed(vg_ctx* ctx, const double* s);
void host_state(vg_ctx* ctx, double* s);
int host_window(vg_ctx* ctx, double* out);
int host_traj(vg_ctx* ctx, double* out, int cap);
int host_step(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n, double beg,
              double end, const double* imu, int m);
int host_win_count(vg_ctx* ctx);
int stage_propagate(vg_ctx* ctx, const double* imu, int m, double end);
int stage_downsample(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n,
                     int* n_ds_out);
int stage_iekf(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, int n, int* degenerate_out);
int stage_window_push(vg_ctx* ctx, const double* imu, int m);
int stage_insert(vg_ctx* ctx);
int stage_recut(vg_ctx* ctx, int* nf_out);
int stage_ba(vg_ctx* ctx, int* iters_out);
int stage_margi_slide(vg_ctx* ctx);
int stage_finish(vg_ctx* ctx);
}  // namespace vg

// ---- phase probes (instrumented build only, make probe) -------------------
#ifdef VG_PROBE
// one probe array per translation unit (no relocatable device code); each
// .hip exports its reader with VG_PROBE_READER(name)
namespace vg {
static __device__ unsigned long long g_probe[64];
}
#define VG_PROBE_READER(fn)                                                                        \
  extern "C" int fn(unsigned long long* out, int n) {                                              \
    if (n > 64) n = 64;                                                                            \
    if (hipDeviceSynchronize() != hipSuccess) return -2;                                           \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vg::g_probe), n * sizeof(unsigned long long)) != hipSuccess) \
      return -2;                                                                                   \
    unsigned long long z[64] = {0};                                                                \
    if (hipMemcpyToSymbol(HIP_SYMBOL(vg::g_probe), z, sizeof(z)) != hipSuccess) return -2;         \
    return 0;                                                                                      \
  }
#define VG_PROBE_BEGIN() unsigned long long vg_probe_t = wall_clock64()
#define VG_PROBE_MARK(k)                                  \
  do {                                                    \
    if (threadIdx.x == 0) {                               \
      const unsigned long long now_ = wall_clock64();     \
      atomicAdd(&vg::g_probe[(k)], now_ - vg_probe_t);    \
      vg_probe_t = now_;                                  \
    }                                                     \
  } while (0)
#else
#define VG_PROBE_BEGIN() (void)0
#define VG_PROBE_MARK(k) (void)0
#endif
