// vg_internal.h — device context of the MI355X LIO hot path (not part of the
// C-ABI). One vg_ctx owns every device buffer of one LiDAR-inertial sequence:
// the scan staging area, the downsample workspace, the device-resident voxel
// map (root hash + octree node pool + per-slot window point arrays + point_fix
// arena) and the sliding-window state.
#pragma once
#include <hip/hip_runtime.h>
#include <chrono>
#include <functional>
#include <mutex>
#include <cstdint>
#include <string>
#include <thread>
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

// Initialisation map of lio_state_estimation_kdtree (odometry.cpp:267-439,
// SURVEY A14): float points (0.5 m downsampled), bucketed by 1 m cells for an
// exact k = 5 nearest-neighbour search (kdlio.hip)
struct KdMap {
  float *x = nullptr, *y = nullptr, *z = nullptr;     // map points (key order of the last downsample)
  float *sx = nullptr, *sy = nullptr, *sz = nullptr;  // the same, grouped by cell
  int* sidx = nullptr;                                // map index of each grouped point
  uint64_t *keys = nullptr, *keys_s = nullptr;
  uint32_t *idx = nullptr, *idx_s = nullptr;
  uint64_t* hkey = nullptr;                           // cell hash: key -> [start, end) in s*
  int *hstart = nullptr, *hend = nullptr;
  int hmask = 0, cap = 0, n = 0;
  double *ds = nullptr, *dir = nullptr, *part = nullptr;  // per scan point: plane offset, normal; block partials
  double* h_part = nullptr;                           // pinned copy of the partials
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
};

struct HdsIn {  // the per-scan downsample's input (k_hds_args -> device, read by every k_hds_* kernel)
  const float *x, *y, *z, *in;
  int n, pad;
};
struct DownsampleBufs {
  HdsIn* arg = nullptr;       // the current scan's input cloud (device copy, see k_hds_args)
  uint64_t *keys = nullptr, *keys_sorted = nullptr;
  uint32_t *idx = nullptr, *idx_sorted = nullptr;
  uint32_t *head = nullptr, *pos = nullptr, *seg = nullptr;
  float *ox = nullptr, *oy = nullptr, *oz = nullptr, *oi = nullptr, *oc = nullptr;
  int* flags = nullptr;  // [0] range error, [1] n_out
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  // the per-scan pipeline's downsample (ds_enqueue): hashed grouping, every
  // count on the device. Voxel table (open addressing, cleared by its users):
  uint64_t* hkey = nullptr;
  int *hfirst = nullptr, *hcnt = nullptr, *hfill = nullptr, *hrank = nullptr, *hoff = nullptr;
  int hmask = 0;
  int cap = 0;                // max points per scan (bigv's length: dense voxels from the front, mid-size from the back)
  uint32_t* pslot = nullptr;  // per point: its voxel's table slot
  uint32_t* pseg = nullptr;   // point indices grouped by voxel
  int* vfirst = nullptr;      // per voxel (output rank): its first point
  int* bigv = nullptr;        // dense voxels (output ranks) deferred to k_hds_big
  uint32_t* pseg2 = nullptr;  // dense voxels' segments back in input order
  int* tsum = nullptr;        // per 1024-point tile: first points, their points
  int* hflags = nullptr;      // [0] range error (until the insert takes it), [1] n_out, [2] fallback needed, [3] dense voxels, [4] mid-size voxels
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
  int shard_rank = 0, shard_world = 1;  // spatial-tile sharding (shard.cpp)
  NodeHdr* hdr = nullptr;
  PlaneRec* pl = nullptr;
  Clu* pcr_add = nullptr;
  Clu* pcr_fix = nullptr;
  double* cov_add = nullptr;   // cap_nodes * 45
  double* eig = nullptr;       // cap_nodes * 12 (eig_value 3, eig_vector 9 row-major)
  double* jour = nullptr;
  double* dbox = nullptr;      // cap_nodes * 6: the descent's region per node (lo[3] exclusive, hi[3] inclusive; vg_dev.h dbox_*)
  Clu* pcrs = nullptr;         // cap_nodes * W (SlideWindow::pcrs_local, physical slot)
  int* nscr = nullptr;         // per-node scratch (cap_nodes * 4)
  unsigned long long* pend = nullptr;  // margi: per internal node, children still to report (high 32) | existing ones (low 32)
  int* cfirst = nullptr;       // per-node per-octant first-event scratch (cap_nodes * 8)
  uint64_t* hkey = nullptr;    // root hash
  int* hval = nullptr;
  int* hfirst = nullptr;
  int* slide = nullptr;        // surf_map_slide (root ids)
  uint8_t* in_slide = nullptr;
  int* leaf_cnt = nullptr;     // insert bucketing: points of this scan per leaf (0 between inserts)
  int* leaf_seg = nullptr;     // insert bucketing: the leaf's segment
  double* fix_pnt = nullptr;   // point_fix arena: pnt (world) 3, var 6
  double* fix_var = nullptr;
  double* wp_pnt = nullptr;    // window points per physical slot: body pnt
  double* wp_var = nullptr;    // world var (after pvec_update), packed 6
  int* wp_leaf = nullptr;      // leaf holding the point in its list, -1 = not listed
  float* wp_int = nullptr;     // intensity of the window point (pointVar::intensity; /map_cmap only)
  // SlideWindow::points per leaf (octree.cpp:151-177): per physical slot, the
  // slot's listed point indices grouped by leaf, each leaf's run in index order
  // — [0, cap_wp) written by the insert, then an arena the recut's children
  // take their runs from (a point moves one layer down per subdivision, so
  // max_layer arenas of cap_wp suffice); lseg locates a leaf's run per slot
  int* wp_ord = nullptr;       // W * ord_stride
  uint64_t* lseg = nullptr;    // cap_nodes * W: start 24 | count 21 | slot epoch 19 bits (lseg_pack)
  int* slot_epoch = nullptr;   // per physical slot: inserts into it so far (a run of an older epoch is stale)
  int* arena = nullptr;        // per physical slot: next free wp_ord entry of the children's arena
  int ord_stride = 0;
  int* counters = nullptr;     // device counters (see kCnt*)
  int* stamp = nullptr;        // per-node tag of the last IEKF iteration that read its plane (P_k, profiling pass)
  int* wpn = nullptr;          // window points per physical slot (written by the insert, read by k_make_win)
};
enum {
  kCntNodes = 0, kCntFix = 1, kCntSlide = 2, kCntNew = 3, kCntTouched = 4, kCntWork = 5, kCntNext = 6,
  kCntSub = 7, kCntEvents = 8, kCntFactors = 9, kCntCreate = 10, kCntErr = 11, kCntLeaves = 12, kCntMisc = 13, kCntSeg = 14, kCntRoots = 15,
  kCntGTouched = 16, kCntGSlide = 17,  // all-reduced copies (sharded mode) for the thread_num quirks
  kCntPlaneUpd = 18, kCntFixFull = 19,  // margi: plane_update calls, leaves with pcr_fix.N >= max_points
  kCntSlideBase = 20,                   // insert: surf_map_slide size before the scan's roots
  kCntNds = 21,                         // insert: the downsampled points it took (N_ds of the scan)
  kCntN = 22
};

// per-scan work buffers
struct Work {
  int cap = 0;                 // entries
  uint64_t *k0 = nullptr, *k1 = nullptr;
  uint32_t *v0 = nullptr, *v1 = nullptr;
  uint32_t *u0 = nullptr, *u1 = nullptr;
  uint32_t *ac_cnt = nullptr, *ac_off = nullptr;  // child allocation scratch
  int *list0 = nullptr, *list1 = nullptr, *list2 = nullptr, *cand = nullptr;
  int* leaf = nullptr;         // per ds point leaf / per event target
  double* pw = nullptr;        // per ds point world coords
  void* tmp = nullptr;
  void* tmp2 = nullptr;        // sort workspace of the second stream
  size_t tmp_bytes = 0;
  double* partials = nullptr;  // reduction partials
  int* iekf_cache = nullptr;   // per raw point cached leaf
  int* pk_leaf = nullptr;      // per raw point leaf read by the profiled IEKF iteration (P_k count)
  int* rc = nullptr;           // device-side level counts (recut / margi, map.hip kRc*)
  uint32_t* cand_bits = nullptr;  // factor candidates of an asynchronous recut, one bit per node id
  int* plan = nullptr;         // per-leaf point_fix copy plan (margi)
  // the recut's odd levels: subdividing leaves, rcinfo, events (even levels: list2, v1, k0)
  unsigned long long* gran = nullptr;  // per 1024-point tile: the root registration's look-back granules
  int ngran = 0;
  int* sub_odd = nullptr;
  int* info_odd = nullptr;
  uint64_t* ev_odd = nullptr;
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
  double* hout_part = nullptr; // this shard's part of it (sharded mode)
  double* rpart = nullptr;
  double* xs = nullptr;        // window poses (W x 12: R9 p3)
};

// ---- device-resident estimator state (state.hip) ----
// The per-scan state lives in HBM for the whole scan: the IEKF update, the
// window push, the BA and the slide all read and write it on the device, so
// the host never waits for an intermediate result. The host mirror (pipeline.cpp)
// is refreshed from the host-mapped publication block below.
constexpr int kXS = 24;             // per-frame state: R 9, p 3, v 3, bg 3, ba 3, g 3
constexpr int kXC = kXS + 225;      // x_curr: frame state + cov 15x15 (row-major)
constexpr int kMaxWin = 32;
constexpr int kBaImuRec = 64 + 225;  // IMU_PRE record (doubles): deltas, bias Jacobians, dtime, cov_inv
// In-kernel clocks of the roofline kernels (vg_profile bit 2): the device's
// constant-rate wall clock (wall_clock64), kernel-only spans, no atomics on
// the timed kernels' paths (a hot atomic from every workgroup cost k_iekf
// ~3 us per launch). A k_iekf launch runs from workgroup 0's start to the
// last workgroup's end: workgroup 0 stores the start, every workgroup its end,
// into a ring slot per (scan, iteration); the host takes the maximum when it
// reads the clock (vg_profile_read). k_ba_solve is one workgroup, timed by its
// thread 0.
constexpr int kClkRing = 256;    // k_iekf launch slots: the last 64 scans x 4 iterations
constexpr int kClkBlocks = 512;  // >= the IEKF grid (iekf_blocks)
// The recut's level kernels (k_rc_level0 + max_layer x k_rc_level), one span
// per scan: k_rc_level0's workgroup 0 stamps the start, every workgroup of the
// last level kernel its end. k_ba_hess: executed launches like k_iekf, slot
// (scan, LM iteration).
constexpr int kClkRcScans = 64;   // recut spans of the last 64 scans
constexpr int kClkRcBlocks = 256; // the level kernels' grid
constexpr int kClkHRing = 512;    // k_ba_hess slots: 64 scans x 8 LM iterations
constexpr int kClkHBlocks = 272;  // >= k_ba_hess's grid (chunk workgroups + IMU workgroups)
struct KClock {
  unsigned long long solve_ticks, solve_n;  // executed k_ba_solve launches
  int on, scan;                             // scans opened since vg_profile (k_scan_begin / k_scan_prop)
  int exec[kClkRing];                       // the slot's k_iekf ran (not a no-op after convergence)
  unsigned long long t0[kClkRing];
  unsigned long long tend[kClkRing][kClkBlocks];
  int rc_exec[kClkRcScans];
  unsigned long long rc_t0[kClkRcScans];
  unsigned long long rc_tend[kClkRcScans][kClkRcBlocks];
  int h_exec[kClkHRing];
  unsigned long long h_t0[kClkHRing];
  unsigned long long h_tend[kClkHRing][kClkHBlocks];
};

struct DState {
  double xc[256];                   // x_curr (IMUST, types.hpp:43-113)
  double xp[256];                   // x_prop (odometry.cpp:67)
  double G6[96];                    // G(:, 0:6) of the last IEKF iteration (odometry.cpp:198)
  double nnt[8];                    // sum n n^T of the last iteration (odometry.cpp:145)
  double traj[16];                  // R, p right after the IEKF (pub_localtraj, local_mapping.cpp:427)
  double xs[kMaxWin * kXS];         // window states x_buf by ord (local_mapping.cpp:434)
  double bias[kMaxWin * 12];        // IMU_PRE bias state per window factor: dbg, dba, dbg_buf, dba_buf
  int it, rematch, done, iters, degenerate, matches[4], ticket, planes[4], rc_ctr, pad1;  // planes: P_k (profiling pass)
  // rc_ctr: asynchronous recuts so far (k_fac_sort publishes it; vg_ctx::rc_pub mirrors it)
  // the scan this IEKF reads (set by k_scan_begin's caller, so the IEKF
  // launches are the same every scan and replay as one hipGraph)
  const float *sx, *sy, *sz;
  int sn, seq2;
  // IMU_PRE records of the window factors (preintegrated deltas, bias
  // Jacobians, cov_inv; constant once pushed): a ring, factor k at slot
  // (imu_head + k) % kMaxWin, so the slide is one index step
  int imu_head, margi_seq;  // margi_seq: the last margi head's publication number (k_margi_copy signals it)
  // the scan graph's per-scan numbers (HostIn::ph, copied by k_ins_prep's block 0):
  // [0] the LM's first flag number, [1] / [2] the margi tail's publication
  // numbers, [3] the recut-done flag value, [4] the margi prefix's flag value,
  // [5] the tail's jour_check (WinArg::jour_check)
  int ph[6];
  // jour (local_mapping.cpp:510-518) on the device, so the margi prefix's
  // stamps (k_set_jour) never wait for the host: jour_check is set by the margi
  // head, the update runs in k_slide_compact (x_buf.back().p before the slide)
  int jour_check, pad_j;
  double jour, last_pos[3];
  double imurec[kMaxWin * kBaImuRec];
  KClock clk;
  // sharded mode (world > 1): the scan's points this rank can match, made
  // once per scan at the opening pose (map.hip k_keep_*): raw indices,
  // ascending; null: every point. The IEKF uses the list while the pose
  // stays within kmargin of kpose for every point (|dR|_F krmax + |dp|).
  const int* skeep;
  int snk, iekf_pts;  // kept points; points the point loop processed this scan (vg_stats::iekf_points)
  double kpose[12], krmax, kmargin;
};
// x_buf.push_back(x_curr) + a new IMU_PRE record, as kernel arguments (k_push_state,
// or folded into the insert's first launch, map_insert)
struct PushArg {
  int ord, new_imu;
  double rec[kBaImuRec];
};
// IMUEKF::process's propagation (imu_ekf.cpp:13-86) on the device: the scan's
// IMU samples and times as kernel arguments; the state it starts from is the
// device's x_curr (the previous scan's, after its BA), so the host never waits
// for that state before opening the next scan (state.hip k_scan_prop)
constexpr int kPropMax = 48;  // IMU samples per scan in the arguments (more: the host path)
struct PropArg {
  int n, pad;
  double last_end, beg, end, sg;                 // last_pcl_end_time, pcl_beg/end, imupre_scale_gravity
  double cov_gyr, cov_acc, rdw_gyr, rdw_acc;     // Odometry.* (node.cpp:211-214)
  double imu[kPropMax * 7];                      // t, gyr[3], acc[3] per sample
};
// per-scan inputs of the replayed graphs, in host-mapped memory: the host
// writes them before the launch, the kernels read them in place. One per ring
// position (the steady state's graphs are per ring position, so a slot is
// rewritten W scans after the graph that read it)
struct HostIn {
  PushArg push;
  int ph[6];  // DState::ph
};
// Spatial-tile sharding of one sequence over `world` contexts (one per GPU):
// every context keeps the root voxels of the tiles it owns (tile_owner) and
// sums only its own points / factors; the normal equations are all-reduced
// (RCCL on the context stream, or a host callback for CPU-mediated tests).
constexpr int kShardBuf = 4096;  // doubles of exchange scratch / staging
constexpr int kShardSmall = 64;   // doubles of a small exchange frame (payload + guard pair)
// a frame its producer kernel packed and its consumer kernel checks (the IEKF
// sums, the LM's Hessian and residual): the all-reduce alone, no pack / unpack
// launches (shard.hip)
int shard_exchange(vg_ctx* ctx, int n, hipStream_t s = nullptr);  // s: the producer's stream (default ctx->stream)
struct Shard {
  int rank = 0, world = 1;
  int mode = 0;              // 0 none, 1 RCCL, 2 host callback
  void* comm = nullptr;      // ncclComm_t
  vg_host_allreduce_fn host_fn = nullptr;
  void* user = nullptr;
  double* h_buf = nullptr;   // pinned staging (host mode)
  double* d_buf = nullptr;   // device scratch for the exchanged sums (4096 doubles)
  int frame_n = 0;           // doubles per exchange (shard.hip: payload + guard pair)
  double* d_frame = nullptr; // the exchange frame (+ this rank's guard value)
  unsigned* d_seq = nullptr; // the device's count of exchanges (the guard's sequence number)
  // the scan's kept points (world > 1, map.hip k_keep_*): per raw point its
  // flag and exclusive prefix, the kept list, max |pnt| (float bits), scan scratch
  int *keep_flag = nullptr, *keep_pos = nullptr, *keep_list = nullptr;
  unsigned* keep_rmax = nullptr;
  void* keep_tmp = nullptr;
  size_t keep_tmp_bytes = 0;
};

// Host-mapped publication block (written by the device with system-scope
// stores, each part closed by a sequence flag the host spins on).
struct Pub {
  int seq_ds, n_ds, ds_err, pad0;          // downsample (after k_ds_*)
  int seq_ba, ba_word, pad1, pad1b;  // LM iteration flags (k_ba_control): iterations * 2 + done, one word (no torn pair)
  int seq_rc, rc_status, rc_nf, pad5;      // asynchronous recut status (k_fac_sort)
  int seq1, iekf_iters, degenerate, matches[4], ba_iters1, ba_hess1, planes[4], iekf_pts, pad2[2];  // P1: state after IEKF/BA
  int seq2, pad3[3];
  int counters[kCntN];                      // P2: map counters at the end of the scan
  double xc[256];
  double traj[16];
  double nnt[8];
  double xs[kMaxWin * kXS];
};
// An LM run whose outcome the host has not read yet (ba_run's loop state,
// continued by ba_resolve): the fused step returns once the LM iterations and
// the speculative margi tail are enqueued, and the next step enqueues its
// downsample, propagation and IEKF before it waits for that outcome
struct BaLoop {
  int seq0 = 0, enq = 0, tail_at = 0, k = 0;  // first iteration flag number, iterations enqueued, ahead of the tail, next k
  bool active = false;
};
// window view for the map kernels, built on the device from DState::xs
struct WinArg {
  int mp[kMaxWin];      // mp[] ring (octree.cpp:75)
  int nper[kMaxWin];    // window points per ord
  int win_count;
  int set_xc;           // x_curr.R/p <- x_buf.back() first (local_mapping.cpp:501-502)
  int seq2;             // end-of-scan publication number (stored in DState::seq2)
  int jour_check;       // (win_base + win_count) % 10 == 0: the jour update follows the margi (local_mapping.cpp:510)
};

}  // namespace vg

struct vg_ctx {
  vg_config cfg;
  vg_capacity cap;
  int device = 0;
  hipStream_t stream = nullptr;
  // the downsample runs on its own stream: it reads only the raw scan, so it
  // overlaps the previous scan's recut/BA/margi and this scan's IEKF
  hipStream_t stream_ds = nullptr;
  // the downsample / margi prefix get a stream of their own, created on the
  // first scan; the multi-sequence mode turns it off before any scan, so its
  // contexts never hold a second hardware queue (vg_multi_create)
  bool want_ds_stream = true;
  hipEvent_t ev_ds_done = nullptr, ev_ds_free = nullptr;
  hipEvent_t ds_free_ev = nullptr;  // what the next downsample waits for: ev_ds_free, or ev_recut_done when one record marks both
  hipEvent_t ev_recut_done = nullptr, ev_prefix_done = nullptr;  // margi prefix on the second stream
  // The next scan's IEKF overlaps the margi's map-only remainder: it runs on
  // stream_iekf behind ev_tail_a (recorded after k_margi_leaf's plane updates,
  // the last margi work the IEKF reads), and the main stream waits for it
  // (ev_iekf_done) before anything else (map_margi, pipeline.cpp lio_state_estimation)
  hipStream_t stream_iekf = nullptr;
  hipEvent_t ev_tail_a = nullptr, ev_iekf_done = nullptr;
  bool tail_a_valid = false;  // ev_tail_a marks the latest main-stream work the next IEKF depends on
  hipEvent_t ev_scan_ready = nullptr;  // deskew done (row f1)
  // the IEKF's 8 launches captured once and replayed (map.hip iekf_run)
  hipGraphExec_t g_iekf[4] = {nullptr, nullptr, nullptr, nullptr};  // [0] the four iterations, [3] the same, signalling the insert ([1], [2] unused)
  hipGraphExec_t g_margi[4] = {};  // margi after the window view (map.hip map_margi): [gated + 2 * signalling]
  hipGraphExec_t g_ba = nullptr;     // one LM iteration (ba.hip ba_run)
  hipGraphExec_t g_ba2 = nullptr;    // the first two LM iterations
  hipGraphExec_t g_ds = nullptr;     // the per-scan downsample chain (downsample.hip ds_enqueue_hashed)
  // steady state: the insert + recut of one scan, per ring position mp[0] (pipeline.cpp stage_insert_recut)
  hipGraphExec_t g_mid[vg::kMaxWin] = {};
  bool capturing = false;  // a stream capture is open (host-side steps that cannot be captured are deferred)
  int rc_pub = 0;          // asynchronous recuts enqueued (mirrors DState::rc_ctr, k_fac_sort)
  int ba_last_iters = 2;   // LM iterations of the previous run (ba_run's enqueue-ahead policy)
  vg::BaLoop ba_loop;      // a deferred LM run (ba_run / ba_resolve)
  bool lm_defer = true;    // the fused step returns before the LM outcome (vgx_debug 26: 0 = waits for it)
  // kernels do not run concurrently (AMD_SERIALIZE_KERNEL, or VG_SERIAL_KERNELS=1 as rocprofv3 --pmc
  // runs set): no device-flag hand-offs (a polling kernel would wait for a producer queued behind it)
  bool serial_kernels = false;
  bool counted = false;          // in the per-device live-context count (dev_ctx_count)
  bool shard_force = false;       // vg_shard_rccl at world 1 still sets up the sharded path (vgx_debug 30)
  bool flag_force = false;       // flag hand-offs even beside other contexts (vgx_debug 14 = 2: the caller drains between them)
  vg::HostIn* h_in = nullptr;  // host-mapped per-scan inputs of replayed graphs, kMaxWin slots (host address)
  vg::HostIn* d_in = nullptr;  // its device address
  int in_sel = 0;              // the slot map_insert uses (the ring position of a scan graph)
  bool in_ph = false;          // map_insert copies the slot's per-scan numbers into DState::ph (scan graph capture)
  // the scan graph (pipeline.cpp stage_insert_recut): insert + recut + k_ba_init
  // + two LM iterations + the gated margi tail, one per ring position
  hipGraphExec_t g_scan[vg::kMaxWin] = {};
  bool scan_graph = true;   // vgx_debug 27: 0 = separate insert+recut graph, LM graph, margi tail
  int ba_seq0_pre = 0;      // the LM flag numbers a scan graph's k_ba_init uses (ba_run pre > 0)
  bool ba_no_defer = false; // set by stage_ba's prefix step when the recut needs the host (no deferral)
  unsigned rc_flag_ctr = 0, pre_flag_ctr = 0;  // d_sync[3] / d_sync[4] values (scan graph hand-offs)
  bool pool_zeroed = false;
  bool ins_ev_pending = false;  // ev_ds_free / ev_recut_done of the last insert+recut graph not recorded yet  // map_reset has cleared the node records once (then only the used ids)
  bool use_graphs = true;  // margi prefix on the second stream
  bool overlap_iekf = true;  // the next IEKF under the margi remainder (lio_state_estimation)
  int pub_flags = 0;         // vg_set_publish: bit 0 = /map_cmap after each window BA (k_local_map)
  float4* d_cmap = nullptr;  // the last /map_cmap cloud (x, y, z, intensity) and its size
  int* d_cmap_n = nullptr;
  bool ds_early = true;      // a fused step's downsample enqueued before the host waits for the previous state (host_step)
  bool ds_after_iekf = true; // vgx_debug 37: ... behind the device propagation's launch (0: ahead of it)
  bool spec_tail = true;     // the margi tail behind the predicted LM iterations (stage_ba)
  std::string err;
  vg::Arena arena;
  // raw scan staging (SoA)
  float *d_x = nullptr, *d_y = nullptr, *d_z = nullptr, *d_i = nullptr, *d_t = nullptr;
  // the scan the stage-level API works on (own staging or caller's HBM)
  const float *cur_x = nullptr, *cur_y = nullptr, *cur_z = nullptr, *cur_i = nullptr;
  int cur_n = -1;
  vg::DownsampleBufs ds;
  vg::KdMap kd;
  vg::DevMap map;
  vg::Work wk;
  vg::BaBufs ba;
  vg::DState* st = nullptr;     // device-resident estimator state
  vg::Shard shard;              // spatial-tile sharding across contexts (shard.cpp)
  vg::Pub* h_pub = nullptr;     // host-mapped publication block (host address)
  vg::Pub* d_pub = nullptr;     // its device address
  double* h_stage = nullptr;    // pinned staging for asynchronous H2D copies (kStageBytes)
  double* d_deskew = nullptr;   // deskew parameters (x_curr pose, extrinsic, IMU poses)
  int pub_seq = 0;
  int wait_spin_us = 0, wait_sleep_us = 0;  // vg_set_wait_policy (0 sleep: spin)
  int plane_tag = 0;        // IEKF iteration tag of the P_k count (vg_profile stages)
  int* h_pinned = nullptr;  // small pinned host scratch for counters
  // host-input scans (vg_step / vg_step_deskew): two slots in flight, each the
  // caller's arrays copied once into pinned memory, one DMA to HBM and an
  // AoS -> SoA unpack on stream_ds ahead of the scan's kernels, no host wait
  // on the device (vina_gpu.cpp upload_scan)
  struct InSlot {
    char* h = nullptr;          // pinned: xyz AoS (12 B/pt) | intensity | time, packed by n
    float* d = nullptr;         // HBM: the DMA image (5 cap floats), then the SoA planes x y z i t
    hipEvent_t up = nullptr;    // unpack done (stream_ds): the DMA has read h
    hipEvent_t done = nullptr;  // main stream past the scan that read the planes
    bool live = false;
  } in_slot[2];
  size_t in_cap = 0;  // points per slot
  void* copy_pool = nullptr;  // helper threads of the pinned copy (vina_gpu.cpp CopyPool)
  int in_next = 0;
  hipEvent_t in_ev = nullptr;  // the current scan's unpack (the split IEKF stream waits for it)

  vg_stats stats;
  void* host = nullptr;     // host-side pipeline state (pipeline.cpp)
  // stage timing with HIP events on the context stream (vg_profile)
  bool prof_on = false;      // k_iekf launch events (vg_profile bit 0)
  int prof_every = 0;        // sample k_ba_solve events on every n-th BA run (vg_profile bits 8-15)
  long prof_runs = 0;
  int rc_total = 0, rc_thread_num = 0;  // the last recut's window point total / thread_num (its resume)
  bool prof_stages = false;  // per-stage events (vg_profile bit 1)
  bool roots_lb = true;      // root registration in one look-back launch (vgx_debug 16: 0 = two launches)
  bool ba_graph2 = true;     // the first two LM iterations as one graph (vgx_debug 17: 0 = one graph each)
  bool margi_batch = true;    // vgx_debug 24: k_margi_leaf reads a leaf's frame clusters four at a time (r04k +0.4 %)
  bool margi_fused = true;    // margi isexist bottom-up in k_margi_copy, erase in one launch (vgx_debug 21: 0 = per-level launches)
  bool iekf_prefetch = true;  // vgx_debug 23: k_iekf touches a cached match's plane record beside its header (r04i A/B +0.9 %)
  bool ba_structural = true;      // vgx_debug 31: k_ba_prep's structural elimination order (0: Eigen's |diag| order)
  bool ba_resid_hess = true;      // vgx_debug 34: k_ba_resid_hess in the two-iteration LM graphs (0: k_ba_resid + k_ba_hess)
  bool ba_init_hess = true;       // vgx_debug 35: k_ba_init inside the scan graph's first Hessian pass (0: its own launch)
  bool rc_init_finish = true;     // vgx_debug 32: the asynchronous recut's factor bookkeeping inside k_ba_init (0: k_factor_finish_dev)
  bool rc_finish_in_init = false; // set by map_recut for the next k_ba_init
  bool rc_begin_fold = true;      // vgx_debug 33: the recut's head in the insert's k_push_window (insert + recut graph)
  const vg::WinArg* rc_begin_wa = nullptr;  // set for one map_insert: its k_push_window runs the recut's head
  bool rc_begun = false;          // ... and the map_recut after it skips k_make_win_recut_begin
  bool ba_fuse_ctl = true;    // vgx_debug 19: the LM bookkeeping in k_ba_resid's IMU workgroup (A/Bs r04e 0, r04g/h +0.8-0.9 %)
  bool ba_graph = true;      // LM iterations replay one captured graph each (vgx_debug 15: 0 = direct launches)
  bool flag_sync = true;     // counter hand-offs instead of event waits on the critical path (vgx_debug 14)
  unsigned* d_sync = nullptr;  // hand-off flags: [0] margi leaf -> next IEKF, [1] IEKF -> insert, [2] margi head -> propagation,
                               // [3] recut done -> margi prefix, [4] margi prefix -> tail (scan graph)
  bool sync_tail_armed = false;  // the last margi's leaf pass stores sync_tail_value into d_sync[0]
  unsigned sync_tail_value = 0, sync_iekf_value = 0;
  bool dev_prop = false;     // host_step propagates on the device (k_scan_prop; vgx_debug 13: 1 = on the device)
  bool rc_fused = true;      // the fused recut levels (vgx_debug 11: 0 = the four-launch level loop)
  bool prof_clock = false;   // in-kernel clocks instead of k_ba_solve events (vg_profile bit 2, KClock)
  hipEvent_t prof_ev[8][2] = {};
  hipEvent_t sync_ev = nullptr;  // host-spin synchronisation (vg::stream_wait)
  hipEvent_t iekf_ev[16][2] = {};  // k_iekf launches of the last two scans (vg_profile), 8 per scan
  int iekf_ring_n = 0, iekf_ring_base = 0;
  hipEvent_t solve_ev[10][2] = {};  // k_ba_solve launches of the current BA run (vg_profile)
  int dbg_apply_cap = -1;        // test knob (vgx_debug): recut apply event capacity
  int dbg_ins_cap = -1;   // vgx_debug 3: k_ins_alloc capacity override (forces the insert replay)
  int dbg_fac_max = -1;   // vgx_debug 4: device factor-sort limit override (forces the host factor path)
  int dbg_capture = 0;    // vgx_debug 5: capture the next LM run's first Hessian pass (vgx_ba_capture)
  double* dbg_cap_buf = nullptr;  // device copy: LiDAR hl (lower) + IMU factor blocks
  int dbg_cap_n = 0;
  bool prof_pending[16] = {};
  double prof_ms[16] = {};  // [0, 8): device time (events); [8, 16): host time of the stage calls
  int prof_n[16] = {};
};

namespace vg {
constexpr int kTrajRow = 13;  // vg_trajectory: t, R 9, p 3
constexpr int kPathRow = 14;  // vg_path: t, R 9, p 3, jour (the path point's curvature)
constexpr size_t kStageBytes = 1 << 17;
constexpr size_t kStageDeskewOff = 8192;  // doubles: the deskew block's part of the staging area
constexpr int kDeskewBuf = 4096;          // doubles (up to 180 IMU segments per scan)
// Spin until a Pub sequence flag reaches seq (the device publishes with a
// system-scope release); checks the stream for errors while spinning.
// Wait policy (vg_set_wait_policy): spin for spin_us, then sleep sleep_us per
// poll. Pure spinning (the default) has the lowest latency for one context;
// several contexts driven from their own threads under a CPU quota need the
// sleeping polls, or the spinning threads starve each other's launches.
inline void wait_pause(const vg_ctx* c, long spin, std::chrono::steady_clock::time_point t0);
inline int pub_wait(vg_ctx* c, const int* flag, int seq, const char* what, hipStream_t producer = nullptr) {
  hipStream_t st = producer ? producer : c->stream;  // the stream the publishing kernel runs on
  const auto t0 = std::chrono::steady_clock::now();
  for (long spin = 0; __atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq; spin++) {
    wait_pause(c, spin, t0);
    if ((spin & 4095) == 4095) {
      const hipError_t e = hipStreamQuery(st);
      if (e != hipSuccess && e != hipErrorNotReady) {
        c->err = std::string(what) + ": " + hipGetErrorString(e);
        return VG_E_HIP;
      }
      if (e == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq) {
        c->err = std::string(what) + ": stream drained without publishing";
        return VG_E_HIP;
      }
    }
  }
  return VG_OK;
}
enum { kProfDownsample = 0, kProfIekfKernel = 1, kProfInsert = 2, kProfRecut = 3, kProfBA = 4, kProfMargi = 5,
       kProfIekf = 6, kProfBaSolve = 7, kProfN = 8,
       // host (CPU) time spent in the stage calls: enqueue work plus any wait
       kHostPropagate = 8, kHostDownsample = 9, kHostIekf = 10, kHostPush = 11, kHostInsert = 12, kHostRecut = 13,
       kHostBA = 14, kHostMargi = 15, kProfAll = 16 };
// host-time scope for a stage call (vg_profile bit 0)
struct HostTimer {
  vg_ctx* c;
  int id;
  std::chrono::steady_clock::time_point t0;
  HostTimer(vg_ctx* ctx, int i) : c(ctx), id(i), t0(std::chrono::steady_clock::now()) {}
  ~HostTimer() {
    if (!c->prof_on) return;
    c->prof_ms[id] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->prof_n[id] += 1;
  }
};
inline void prof_begin(vg_ctx* c, int id, hipStream_t s = nullptr) {
  if (c->prof_stages) (void)hipEventRecord(c->prof_ev[id][0], s ? s : c->stream);
}
inline void prof_end(vg_ctx* c, int id, hipStream_t s = nullptr) {
  if (c->prof_stages) {
    (void)hipEventRecord(c->prof_ev[id][1], s ? s : c->stream);
    c->prof_pending[id] = true;
  }
}
// Wait for the context stream by spinning on an event: a blocking
// hipStreamSynchronize may sleep and costs up to ~100+ us of wake-up latency
// per round trip, and the map stages make several per scan.
inline hipError_t stream_wait(vg_ctx* c, hipStream_t s = nullptr) {
  hipError_t e = hipEventRecord(c->sync_ev, s ? s : c->stream);
  if (e != hipSuccess) return e;
  const auto t0 = std::chrono::steady_clock::now();
  for (long spin = 0; (e = hipEventQuery(c->sync_ev)) == hipErrorNotReady; spin++) wait_pause(c, spin, t0);
  return e;
}
inline void wait_pause(const vg_ctx* c, long spin, std::chrono::steady_clock::time_point t0) {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
  if (c->wait_sleep_us <= 0 || (spin & 63) != 63) return;
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  if (us >= c->wait_spin_us) std::this_thread::sleep_for(std::chrono::microseconds(c->wait_sleep_us));
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
  double beam_dv;     // sin^2(beam * pi / 180) of calcBodyVar (point_utils.cpp:13-14), with beam in float
};

struct WinD {           // window poses x_buf (by ord) and the ring mp[] (octree.cpp:75)
  double R[32][9];
  double p[32][3];
  int mp[32];
  int win_count;
  int pad;
};


// downsample.hip
int ds_alloc(vg_ctx* ctx);
// kdlio.hip
int kd_alloc(vg_ctx* ctx);
int kd_reset(vg_ctx* ctx);
// one pass of the kd-tree IEKF over the scan in ctx->d_x/y/z (n points, raw
// LiDAR frame) at pose (R row-major 9, p 3): refind -> kNN + plane fits, then
// the 28 sums (HTH upper 21, HTz 6, valid count) -> out28 (synchronous)
int kd_pass(vg_ctx* ctx, int n, const double* R, const double* p, int refind, double* out28);
// append the scan at pose (R, p) to the map, re-downsample at 0.5 m, rebuild
// the cell index (synchronous); or only append + index when the map is seeding
int kd_update(vg_ctx* ctx, int n, const double* R, const double* p, bool downsample);
// Voxel-grid downsample of a device-resident SoA cloud; results land in
// ctx->ds.o* (n_out voxels, ascending packed-key order). Host-synchronous
// (returns n_out).
int ds_run(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* in, int n, double voxel,
           int* n_out);
// down_sampling_close of a device cloud (the initialisation's raw-cloud
// reduction): out = the chosen points (x, y, z, t) sorted by time, stable over
// ascending voxel keys; t == nullptr gives every point the time tconst.
// Host-synchronous.
int ds_close(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* t, float tconst, int n,
             double voxel, float4* out, int* n_out);
// The per-scan pipeline's downsample (hashed, no sort, no host count; output
// in first-occurrence order), asynchronous on s, with the /2 fallback on the
// device when `fallback`; the voxel count stays in ds.hflags[1].
int ds_enqueue_hashed(vg_ctx* ctx, hipStream_t s, const float* x, const float* y, const float* z, const float* in,
                      int n, double voxel, bool fallback, int pub_seq);
int ds_reset(vg_ctx* ctx);
// Same, asynchronous: n_out and the range flag are published to Pub (seq_ds).
int ds_enqueue(vg_ctx* ctx, hipStream_t s, const float* x, const float* y, const float* z, const float* in, int n,
               double voxel, int pub_seq);
// map.hip
int map_alloc(vg_ctx* ctx);
// The insert+recut graph's completion events are recorded lazily: right
// behind the LM's k_ba_init when the LM follows (a marker packet straight
// after the graph delays the next dispatch), else before their first waiter.
// Recording later only makes the waiters wait longer.
inline hipError_t flush_insert_events(vg_ctx* ctx) {
  if (!ctx->ins_ev_pending) return hipSuccess;
  ctx->ins_ev_pending = false;
  ctx->ds_free_ev = ctx->ev_recut_done;  // one record marks both (each record is a gap in the stream)
  return hipEventRecord(ctx->ev_recut_done, ctx->stream);
}
int map_reset(vg_ctx* ctx);
int iekf_iteration(vg_ctx* ctx, const MP& mp, const float* x, const float* y, const float* z, int n, int it,
                   hipEvent_t ev0, hipEvent_t ev1, int tag = 0, hipStream_t s = nullptr,
                   unsigned* done_flag = nullptr);
// all four iterations; replays the captured graph when possible
// begin_xc != nullptr: open the scan on the device first (x_curr after
// propagation, one launch with the scan binding)
// *signalled: the run itself advanced the IEKF -> insert hand-off flag
// (d_sync[1], by one; k_iekf_all's update workgroup after a release), so the
// caller need not enqueue k_sync_set (signal: the caller wants it)
int iekf_run(vg_ctx* ctx, const MP& mp, const float* x, const float* y, const float* z, int n, int bank,
             const double* begin_xc = nullptr, hipStream_t s = nullptr, const PropArg* begin_prop = nullptr,
             bool signal = false, bool* signalled = nullptr, bool opened = false);  // opened: scan already bound
constexpr int kNeedInsertReplay = 1;  // map_recut: the insert overflowed k_ins_alloc, replay it first
// the initialisation's insert source (cut_voxel, initialization.cpp:229-246):
// n fp64 body points, the kXC pose/covariance block of x_buf[i], both device
struct InsPre {
  const double* pnt;
  const double* pose;
  int var_identity;  // 1: identity body covariance, no pvec_update (before convergence)
};
// push: the window push to fold into the insert's first launch (or nullptr);
// pre: insert precomputed body points instead of the downsampled scan
// nd: the point count on the device (n is then an upper bound, for grid sizes)
int map_insert(vg_ctx* ctx, const MP& mp, int slot, int n, int epoch, int thread_num, const PushArg* push = nullptr,
               const InsPre* pre = nullptr, const int* nd = nullptr);
int map_insert_replay(vg_ctx* ctx, const MP& mp, int slot, int n, int thread_num);
int map_recut(vg_ctx* ctx, const MP& mp, const WinArg& wa, int thread_num, int* n_factors, bool replay = false,
              int pub_seq = 0);
int map_recut_resume(vg_ctx* ctx, const MP& mp, int* n_factors);
int map_set_attrs(vg_ctx* ctx);
const int* map_rc_status(vg_ctx* ctx);
int map_factor_finish(vg_ctx* ctx);  // k_factor_finish_dev when no k_ba_init took it (map.hip)  // the asynchronous recut's status word (k_fac_sort)
int map_memo_probe(vg_ctx* ctx, const MP& mp, int* out);  // test-only (vgx_memo_probe)
int iekf_grid(vg_ctx* ctx);  // k_iekf's workgroups (map.hip iekf_blocks)
int sync_set(vg_ctx* ctx, hipStream_t s, int k, unsigned value, const int* gate = nullptr);  // state.hip: cross-stream flags
int sync_wait(vg_ctx* ctx, hipStream_t s, int k, unsigned target);
int sync_wait_dev(vg_ctx* ctx, hipStream_t s, int k, const int* target, const int* gate);  // target / gate on the device
// multi_margi + the device-state slide; publishes the state (pub_seq, before
// the margi kernels) and the end-of-scan counters (pub_seq2)
// flags (the scan graph): {recut-done value of d_sync[3] to wait for, value to
// store into d_sync[4] at the end}; nullptr: event waits
int map_margi_prefix(vg_ctx* ctx, const MP& mp, int slot0, int n_oldest, int thread_num,
                     const unsigned* flags = nullptr);
int map_margi(vg_ctx* ctx, const MP& mp, const WinArg& wa, int n_oldest, int thread_num, int pub_seq, int pub_seq2,
              const int* gate);
int map_margi_tail_capture(vg_ctx* ctx, const MP& mp, const WinArg& wa);  // the scan graph's gated margi tail
// state.hip
int state_alloc(vg_ctx* ctx);
// x_curr / x_prop / IEKF flags; with x != nullptr also the scan the IEKF reads
// prop: propagate on the device (k_scan_prop), optionally waiting inside for
// the margi head's flag (before the rotation chain) and the leaves' flag (at
// its end); see state.hip
int state_scan_begin(vg_ctx* ctx, const double* xc249, const float* x = nullptr, const float* y = nullptr,
                     const float* z = nullptr, int n = 0, hipStream_t s = nullptr, const PropArg* prop = nullptr,
                     const unsigned* head_flag = nullptr, unsigned head_target = 0,
                     const unsigned* leaf_flag = nullptr, unsigned leaf_target = 0);
int state_set_scan(vg_ctx* ctx, const float* x, const float* y, const float* z, int n, hipStream_t s = nullptr);
int state_push(vg_ctx* ctx, int ord, int new_imu, const double* imurec);  // imurec: kBaImuRec doubles (new_imu >= 0)
int state_publish(vg_ctx* ctx, int win_count, const int* ba_iters_dev, int seq, const int* gate = nullptr);
int state_publish_counters(vg_ctx* ctx, int seq);
int state_publish_ds(vg_ctx* ctx, hipStream_t s, int seq, int* flags, bool reset);
int state_deskew(vg_ctx* ctx, const double* par, int npose, const float* x, const float* y, const float* z,
                 const float* in, const float* t, int n);
int state_unpack_scan(vg_ctx* ctx, hipStream_t s, int n, const float* img, bool has_i, bool has_t, float* x, float* y, float* z,
                      float* in, float* t);
// initialisation: motion_blur's per-point part on a close-downsampled
// cloud (pts, ascending time) -> nout fp64 body points; par (host): frame pose,
// extrinsic, npose IMU pose records (descending start); synchronous
int state_blur_init(vg_ctx* ctx, const double* par, int npose, const float4* pts, int n, int j0, int q0, int nout,
                    double* d_par, double* pnt);
// window states / x_curr / IMU records (+ zero bias, ring head 0) -> DState; synchronous
int state_load(vg_ctx* ctx, const double* xs, int nw, const double* xc, const double* recs, int nrec);
// ba.hip
constexpr int kBaX = 24;        // per-frame state: R 9, p 3, v 3, bg 3, ba 3, g 3
int ba_alloc(vg_ctx* ctx);
// LM on the device state (window states, IMU_PRE records and bias records in
// DState; the factor count in the map counters). Returns once the LM has
// converged on the device (the flags are read without draining the stream).
// before_first_wait: enqueued once the first iterations are; spec_tail (may
// decline through its flag): the margi tail, enqueued right behind the
// iteration count the previous run converged at and gated on the device by
// ba_gate_dev; *tail_ok tells whether that copy is the one that runs
// pending != nullptr: the run may return once the speculative tail is queued
// (*pending = true, *iters = -1); ba_resolve then continues it
// pre > 0: the scan graph already holds k_ba_init, the first `pre`
// iterations and the gated margi tail (flag numbers from ctx->ba_seq0_pre)
int ba_run(vg_ctx* ctx, int nf, const int* mp_ring, int* iters,
           const std::function<int()>& before_first_wait = nullptr,
           const std::function<int(bool*)>& spec_tail = nullptr, bool* tail_ok = nullptr, bool* pending = nullptr,
           int pre = 0);
// the scan graph's LM part, captured on the context stream (k_ba_init with its
// numbers from DState::ph, iterations 0 and 1)
int ba_capture_scan_lm(vg_ctx* ctx, const int* mp_ring);
// the rest of a deferred run (ctx->ba_loop): waits for the iteration flags and
// enqueues further iterations as ba_run would have. block = false: returns
// with *finished = false as soon as a flag it needs is not published yet.
// *tail_ok: the speculative tail is the copy that runs (else the caller
// enqueues the real one)
int ba_resolve(vg_ctx* ctx, bool block, bool* finished, int* iters, bool* tail_ok);
const int* ba_iters_dev(vg_ctx* ctx);
const int* ba_gate_dev(vg_ctx* ctx);  // 1 once the LM run has finished (converged or 10 iterations)
const int* ba_hess_dev(vg_ctx* ctx);  // Hessian passes of the last LM run (I_H of SURVEY 8(d))
// LiDAR factor passes for a host-driven LM (initialisation): Hessian pass at
// `poses` (lower 6W x 6W, gradient, residual into out) or residual pass at
// `poses` (*out); synchronous
int ba_lidar_pass(vg_ctx* ctx, bool hessian, const double* poses, const int* mp_ring, double* out);
int ba_factor_normals(vg_ctx* ctx, std::vector<double>& normals);
int ba_solve_test(vg_ctx* ctx, const double* A, const double* b, double* x);  // vgx_ba_solve  // column 0 of each factor's eigenvectors
// pipeline.cpp
void host_init(vg_ctx* ctx);
void host_free(vg_ctx* ctx);
void host_reset(vg_ctx* ctx);
void host_seed(vg_ctx* ctx, const double* s);
int host_state(vg_ctx* ctx, double* s);
int host_window(vg_ctx* ctx, double* out);
int host_traj(vg_ctx* ctx, double* out, int cap, int from = 0);  // rows [from, from + cap), returns the row count
int host_path(vg_ctx* ctx, double* out, int cap);
int host_poll(vg_ctx* ctx);
int host_step(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n, double beg,
              double end, const double* imu, int m);
int host_win_count(vg_ctx* ctx);
int host_memo_probe(vg_ctx* ctx, int* out);  // map_memo_probe with the context's map parameters
// shard.cpp
int shard_alloc(vg_ctx* ctx);
void shard_free(vg_ctx* ctx);
int shard_allreduce(vg_ctx* ctx, const void* send, void* recv, int count, int dtype, int site);
int host_sync(vg_ctx* ctx);
// the sharded path (collectives at the exchange points, direct launches): a
// shard transport is set (vg_shard_rccl / vg_shard_host with world > 1, or
// world 1 with vgx_debug 30: the sharded path's own cost on one GPU)
inline bool sharded(const vg_ctx* c) { return c->shard.mode != 0; }
// live contexts on a HIP device in this process (vina_gpu.cpp): with more than
// one, each context's three streams share the device's hardware queues
// (GPU_MAX_HW_QUEUES, 4 by default) with another's, and a polling hand-off
// kernel could wait on a producer queued behind it: the flag hand-offs are off
int dev_ctx_count(int device);
// Graph capture and instantiation are serialised across the process's
// contexts (one-time work per context): the multi-sequence mode's worker
// threads otherwise capture concurrently (B = 16: sixteen threads at once).
std::recursive_mutex& capture_mutex();
int host_release_far(vg_ctx* ctx, int flags, long long* out);
bool host_release_pending(vg_ctx* ctx);  // jour advanced in an absorbed scan since the last release
// lifetime.hip: the journey release + the node pool / point_fix arena compaction
int map_release(vg_ctx* ctx, bool release, int thr, double jour, int compact, long long* out);
int map_roots(vg_ctx* ctx, long long* key, double* jour, int* flags, int* nodes, int* nfix, int cap, int* count);
int host_lio_kdtree(vg_ctx* ctx, const float* xyz, int n, double* state, int* valid, int* iters);
int decode_scan(vg_ctx* ctx, const void* records, int n, const vg_lidar_format* fmt, float* xyz, float* inten,
                float* time, int* n_out);  // decode.hip
int host_stats_log(vg_ctx* ctx, vg_stats* out, int cap);
int stage_propagate(vg_ctx* ctx, const double* imu, int m, double beg, double end, bool dev = false);  // dev: k_scan_prop
int stage_deskew(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* in, const float* t,
                 int n);
int host_step_deskew(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di,
                     const float* dt, int n, double beg, double end, const double* imu, int m);
int stage_downsample(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n,
                     int* n_ds_out);
int stage_iekf(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, int n, int* degenerate_out);
int stage_window_push(vg_ctx* ctx, const double* imu, int m);
int stage_insert(vg_ctx* ctx);
int stage_recut(vg_ctx* ctx, int* nf_out);
int stage_ba(vg_ctx* ctx, int* iters_out, bool margi_follows = false);  // margi_follows: the fused step
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
#define VG_PROBE_MARK_T(k, t)                             \
  do {                                                    \
    if (threadIdx.x == (t)) {                             \
      const unsigned long long now_ = wall_clock64();     \
      atomicAdd(&vg::g_probe[(k)], now_ - vg_probe_t);    \
      vg_probe_t = now_;                                  \
    }                                                     \
  } while (0)
#else
#define VG_PROBE_BEGIN() (void)0
#define VG_PROBE_MARK(k) (void)0
#define VG_PROBE_MARK_T(k, t) (void)0
#endif
