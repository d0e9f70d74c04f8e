// vg_host.h — host-side pipeline state shared by pipeline.cpp (the
// steady-state loop) and init.cpp (the cold-start initialisation, SURVEY row
// f2): the host mirror of the estimator state, the IMU preintegration, the
// pending-publication queue.
#pragma once
#include <deque>
#include <functional>
#include <vector>
#include "vg_internal.h"

namespace vg {

struct HX {  // IMUST (types.hpp:43-113)
  double t = 0;
  M3 R = M3::I();
  V3 p = V3::Z(), v = V3::Z(), bg = V3::Z(), ba = V3::Z(), g = v3(0, 0, -9.8);
  M15 cov;
  HX() {
    cov = M15::Z();
    for (int i = 0; i < 15; i++) cov(i, i) = (i < 9) ? 0.0001 : 0.00001;
  }
  void plus(const V15& d) {
    R = mul(R, Exp(v3(d[0], d[1], d[2])));
    for (int k = 0; k < 3; k++) {
      p[k] += d[3 + k];
      v[k] += d[6 + k];
      bg[k] += d[9 + k];
      ba[k] += d[12 + k];
    }
  }
  V15 minus(const HX& b) const {  // *this - b
    V15 a;
    V3 r = Log(mul(tr(b.R), R));
    for (int k = 0; k < 3; k++) {
      a[k] = r[k];
      a[3 + k] = p[k] - b.p[k];
      a[6 + k] = v[k] - b.v[k];
      a[9 + k] = bg[k] - b.bg[k];
      a[12 + k] = ba[k] - b.ba[k];
    }
    return a;
  }
};

struct Imu {
  double t;
  double gyr[3], acc[3];
};

// IMUEKF::scale_gravity = imupre_scale_gravity (vg_config; 0 reads as 1)
static inline double gravity_scale(const vg_config& c) { return c.scale_gravity > 0 ? c.scale_gravity : 1.0; }

// IMU_PRE host part (preintegration.hpp:12-51)
struct HImuPre {
  M3 R_delta = M3::I(), R_bg = M3::Z(), p_bg = M3::Z(), p_ba = M3::Z(), v_bg = M3::Z(), v_ba = M3::Z();
  V3 p_delta = V3::Z(), v_delta = V3::Z(), bg, ba;
  double dtime = 0;
  M15 cov = M15::Z();
  std::vector<double> rec;  // the BA's device record, fixed once integrated (record())
  HImuPre(const V3& bg1, const V3& ba1) : bg(bg1), ba(ba1) {}
  void add_imu(V3 gyr, V3 acc, double dt, const M6& nm, const M6& nw) {  // imu_preintegration.cpp:57-95
    dtime += dt;
    M3 rinc = Exp(gyr, dt);
    M3 rj = jr(scl(gyr, dt));
    M3 rdt = scl(R_delta, dt);
    M3 rdt2 = scl(R_delta, 0.5 * dt * dt);
    M3 ask = hat(acc);
    p_ba = sub(add(p_ba, scl(v_ba, dt)), rdt2);
    p_bg = sub(add(p_bg, scl(v_bg, dt)), mul(mul(rdt2, ask), R_bg));
    v_ba = sub(v_ba, rdt);
    v_bg = sub(v_bg, mul(mul(rdt, ask), R_bg));
    R_bg = sub(mul(tr(rinc), R_bg), scl(rj, dt));
    M<9, 9> A = M<9, 9>::I();
    M<9, 6> B = M<9, 6>::Z();
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        A(r, c) = rinc(c, r);
        A(3 + r, c) = -mul(rdt2, ask)(r, c);
        A(3 + r, 6 + c) = (r == c) ? dt : 0.0;
        A(6 + r, c) = -mul(rdt, ask)(r, c);
        B(r, c) = rj(r, c) * dt;
        B(3 + r, 3 + c) = rdt2(r, c);
        B(6 + r, 3 + c) = rdt(r, c);
      }
    M<9, 9> c9;
    for (int r = 0; r < 9; r++)
      for (int c = 0; c < 9; c++) c9(r, c) = cov(r, c);
    M<9, 9> nc = add(mul(mul(A, c9), tr(A)), mul(mul(B, nm), tr(B)));
    for (int r = 0; r < 9; r++)
      for (int c = 0; c < 9; c++) cov(r, c) = nc(r, c);
    for (int r = 0; r < 6; r++)
      for (int c = 0; c < 6; c++) cov(9 + r, 9 + c) += nw(r, c) * dt;
    V3 dp = add(scl(v_delta, dt), mul(rdt2, acc));
    V3 dv = mul(rdt, acc);
    for (int k = 0; k < 3; k++) {
      p_delta[k] += dp[k];
      v_delta[k] += dv[k];
    }
    R_delta = mul(R_delta, rinc);
  }
  // imu_preintegration.cpp:31-55; sg = imupre_scale_gravity (line 51)
  void push_imu(const std::vector<Imu>& buf, const M6& nm, const M6& nw, double sg) {
    for (size_t k = 1; k < buf.size(); k++) {
      const Imu& a = buf[k - 1];
      const Imu& b = buf[k];
      double dt = b.t - a.t;
      V3 gyr, acc;
      for (int j = 0; j < 3; j++) {
        gyr[j] = 0.5 * (a.gyr[j] + b.gyr[j]) - bg[j];
        acc[j] = 0.5 * (a.acc[j] + b.acc[j]) * sg - ba[j];
      }
      add_imu(gyr, acc, dt, nm, nw);
    }
  }
  void record(double* rec) const {
    memset(rec, 0, kBaImuRec * sizeof(double));
    memcpy(rec, R_delta.a, 72);
    memcpy(rec + 9, p_delta.a, 24);
    memcpy(rec + 12, v_delta.a, 24);
    memcpy(rec + 15, R_bg.a, 72);
    memcpy(rec + 24, p_bg.a, 72);
    memcpy(rec + 33, p_ba.a, 72);
    memcpy(rec + 42, v_bg.a, 72);
    memcpy(rec + 51, v_ba.a, 72);
    rec[60] = dtime;
    M15 ci = inverse(cov);
    memcpy(rec + 64, ci.a, 225 * sizeof(double));
  }
};

struct Pend {          // a scan whose device results the host has not absorbed yet
  int seq1 = 0, seq2 = 0;  // P1 (state) and P2 (counters) sequence numbers
  int shift = 0;           // x_buf slid on the host after P1 was published
  int jour_check = 0;      // local_mapping.cpp:525-533 pending on the BA result
  int pushed = -1;         // x_buf index pushed by this scan (cov from x_curr)
  int ins_slot = -1;       // physical window slot its insert filled (wp_n once absorbed)
  int ev_base = 0, ev_n = 0;  // this scan's k_iekf event pairs (vg_profile)
  double t = 0;            // scan end time (trajectory row)
  bool init_tail = false;  // the scan motion_init succeeded on: its trajectory row and
                           // IEKF fields come from the initialisation (init.cpp)
  vg_stats st;
};

struct InitState;  // init.cpp

struct HostPipe {
  std::function<int()> ds_hook;  // host_step: the early downsample's enqueue, run inside lio_state_estimation
  HX x_curr;
  std::vector<HX> x_buf;
  std::deque<HImuPre> imu_pre;
  std::vector<int> mp;
  int win_count = 0, win_base = 0, epoch = 0;
  double jour = 0, last_pcl_end_time = 0;
  bool release_flag = false;  // local_mapping.cpp:272, 517: jour advanced since the last release (vg_release_far)
  V3 last_pos = V3::Z();
  bool first = true;
  int wp_n[32] = {0};
  MP mpd;
  M6 noiseMeas = M6::Z(), noiseWalk = M6::Z();
  std::vector<double> traj;  // save_pose_tum rows (io.cpp:67-77): steady-state scans only, kTrajRow each
  std::vector<double> path;  // pcl_path (publishers.cpp:65-131): every pub_localtraj, cleared by system_reset,
                             // the window's rows re-written by pub_localmap after the BA; kPathRow each
  std::vector<vg_stats> stats_log;
  std::vector<double> poses;  // this scan's IMUEKF::imu_poses, 22 doubles each (deskew)
  int n_factors = 0;
  // current scan
  Pend cur;
  bool in_scan = false;
  int ds_seq = 0, ds_n = -1, n_raw = 0;
  const float *sx = nullptr, *sy = nullptr, *sz = nullptr, *si = nullptr;
  int ins_slot = -1, ins_n = 0;
  bool published = false;
  bool prefix = false;     // map_margi_prefix enqueued for this scan
  bool tail_queued = false;  // the margi tail went in behind the LM and its gate opened (ba_run)
  int tail_seq1 = 0, tail_seq2 = 0;  // that tail's publication numbers
  WinArg tail_wa;                    // and its window view (before the host's slide)
  // the previous fused step's LM, not resolved yet (stage_ba, ctx->ba_loop):
  // if its speculative tail turns out not to run, the real one is enqueued
  // with the same publication numbers and window view (resolve_lm)
  struct LmPend {
    bool active = false;
    int seq1 = 0, seq2 = 0;
    WinArg wa;
  } lmp;
  int rc_seq = 0;          // > 0: this scan's recut ran asynchronously (status with Pub::seq_rc == rc_seq)
  bool scan_g = false;     // this scan's insert + recut + LM + tail went in as the scan graph (stage_insert_recut)
  unsigned sg_flags[2] = {0, 0};  // its hand-off values: recut done (d_sync[3]), margi prefix done (d_sync[4])
  std::deque<Pend> pend;   // enqueued scans awaiting absorption (oldest first)
  int sticky = VG_OK;      // deferred device error
  // device work deferred to the next launch that can carry it (one launch
  // fewer each): the scan opening rides with the IEKF's scan binding, the
  // window push with the insert's first kernel
  bool begin_pending = false;
  double begin_xc[kXC];
  bool begin_prop = false;  // the opening propagates on the device (k_scan_prop) from `prop`
  PropArg prop;
  bool push_pending = false;
  PushArg push;
  // IMUEKF::scale_gravity as used by the propagation and the preintegration
  // (imupre_scale_gravity): the configuration's, or IMU_init's on a cold start
  double sg = 1.0;
  InitState* init = nullptr;  // cold start (vg_config::cold_start): the initialisation's state
};

static inline HostPipe* hp(vg_ctx* ctx) { return (HostPipe*)ctx->host; }

static inline std::vector<Imu> to_imus(const double* imu, int m) {
  std::vector<Imu> imus(m > 0 ? m : 0);
  for (int i = 0; i < m; i++) {
    imus[i].t = imu[7 * i];
    for (int j = 0; j < 3; j++) {
      imus[i].gyr[j] = imu[7 * i + 1 + j];
      imus[i].acc[j] = imu[7 * i + 4 + j];
    }
  }
  return imus;
}

// pipeline.cpp
void propagate(vg_ctx* ctx, HostPipe* P, const std::vector<Imu>& imus, double pcl_beg, double pcl_end);
int absorb(vg_ctx* ctx, HostPipe* P, bool full);
int kd_lio(vg_ctx* ctx, int n, HX& x_curr, int* valid, int* iters);  // on the scan in ctx->d_x/y/z
// init.cpp
InitState* init_create(vg_ctx* ctx);
void init_destroy(InitState* I);
bool init_active(const HostPipe* P);
int init_step(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, const float* dt, int n,
              double beg, double end, const double* imu, int m);

}  // namespace vg
