// pipeline.cpp — host side of the drop-in: the per-scan steady-state loop of
// VINA_SLAM::thd_odometry_localmapping (local_mapping.cpp:389-547), reshaped
// around device-resident stages. Host C++ keeps only what is O(IMU samples):
// IMU propagation (imu_ekf.cpp:28-94) and preintegration
// (imu_preintegration.cpp:31-95). Every per-point / per-voxel / per-factor
// loop and the estimator state itself (x_curr, x_prop, x_buf, the IMU bias
// records, the IEKF 15x15 update) live on the device (state.hip).
//
// Asynchrony: a scan is enqueued without draining the stream. The host waits
// only (a) for the downsampled point count, while the GPU runs the IEKF; (b)
// for the recut's factor count; (c) for each LM iteration's flags, one
// iteration ahead. The state the next scan's propagation needs is published to
// host-mapped memory right after the BA, while the GPU still runs the margi;
// the host mirror (x_curr, x_buf, trajectory, stats) absorbs it lazily.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>

#include "vg_host.h"

namespace vg {

// enqueue deferred device work on its own when the next stage cannot carry it
static int flush_begin(vg_ctx* ctx, HostPipe* P) {
  if (!P->begin_pending) return VG_OK;
  P->begin_pending = false;
  return P->begin_prop ? state_scan_begin(ctx, nullptr, nullptr, nullptr, nullptr, 0, nullptr, &P->prop)
                       : state_scan_begin(ctx, P->begin_xc);
}
static int flush_deferred(vg_ctx* ctx, HostPipe* P) {
  VG_TRY(flush_begin(ctx, P));
  if (!P->push_pending) return VG_OK;
  P->push_pending = false;
  return state_push(ctx, P->push.ord, P->push.new_imu, P->push.rec);
}


void host_init(vg_ctx* ctx) {
  HostPipe* P = new HostPipe();
  const vg_config& c = ctx->cfg;
  P->mp.resize(c.win_size);
  for (int i = 0; i < c.win_size; i++) P->mp[i] = i;
  MP& m = P->mpd;
  memset(&m, 0, sizeof(m));
  m.vs = c.voxel_size;
  m.min_eig = c.min_eigen_value;
  for (int i = 0; i < 4; i++) {
    m.thre[i] = 1.0 / c.plane_eigen_value_thre[i];
    m.minpt[i] = c.min_point[i];
  }
  for (int i = 0; i < 9; i++) m.extR[i] = c.ext_R[i];
  for (int i = 0; i < 3; i++) m.extt[i] = c.ext_t[i];
  m.dept = (float)c.dept_err;
  m.beam = (float)c.beam_err;
  {
    const double sb = sin(m.beam * M_PI / 180.0);  // calcBodyVar's (float degree_inc) * M_PI / 180.0
    m.beam_dv = sb * sb;
  }
  m.max_layer = c.max_layer;
  m.max_points = c.max_points;
  m.W = c.win_size;
  for (int i = 0; i < 3; i++) {
    P->noiseMeas(i, i) = c.ba_cov_gyr;
    P->noiseMeas(3 + i, 3 + i) = c.ba_cov_acc;
    P->noiseWalk(i, i) = c.ba_rdw_gyr;
    P->noiseWalk(3 + i, 3 + i) = c.ba_rdw_acc;
  }
  P->sg = gravity_scale(c);
  if (c.cold_start) P->init = init_create(ctx);
  ctx->host = P;
}
void host_free(vg_ctx* ctx) {
  if (hp(ctx) && hp(ctx)->init) init_destroy(hp(ctx)->init);
  delete hp(ctx);
  ctx->host = nullptr;
}
void host_reset(vg_ctx* ctx) {
  host_free(ctx);
  host_init(ctx);
}

// ---- absorbing published device results into the host mirror

static int map_error(vg_ctx* ctx, int e) {
  ctx->err = std::string("device map error flags=") + std::to_string(e) + ((e & 4) ? " (node pool full)" : "") +
             ((e & 8) ? " (point_fix arena full)" : "") + ((e & 1) ? " (voxel key out of packed range)" : "") +
             ((e & 2) ? " (root hash full)" : "") + ((e & 16) ? " (subdivision event buffer full)" : "") +
             ((e & 32) ? " (sharded exchange out of step: the ranks' exchange sequences differ)" : "") +
             ((e & 64) ? " (cross-stream hand-off timed out)" : "");
  if (e & (32 | 64)) return VG_E_STATE;  // out-of-step exchange, or a hand-off that timed out: not a capacity limit
  return (e & 1) ? VG_E_RANGE : VG_E_CAPACITY;
}

// LioStateEstimation's return value (odometry.cpp:244-254): lambda_min of
// sum n n^T >= 14; bookkeeping only (degrade_cnt, local_mapping.cpp:413-423)
static int degenerate_of(const double* nnt) {
  M3 nn;
  nn(0, 0) = nnt[0];
  nn(0, 1) = nn(1, 0) = nnt[1];
  nn(0, 2) = nn(2, 0) = nnt[2];
  nn(1, 1) = nnt[3];
  nn(1, 2) = nn(2, 1) = nnt[4];
  nn(2, 2) = nnt[5];
  V3 ev;
  M3 U;
  eig3(nn, ev, U);
  return (ev[0] < 14) ? 1 : 0;
}

// P1 of the oldest pending scan: x_curr, post-IEKF pose, window states
static int absorb_p1(vg_ctx* ctx, HostPipe* P, Pend& q) {
  if (q.seq1 == 0) return VG_OK;
  VG_TRY(pub_wait(ctx, &ctx->h_pub->seq1, q.seq1, "state publication"));
  const Pub& pb = *ctx->h_pub;
  HX& xc = P->x_curr;
  memcpy(xc.R.a, pb.xc, 72);
  memcpy(xc.p.a, pb.xc + 9, 24);
  memcpy(xc.v.a, pb.xc + 12, 24);
  memcpy(xc.bg.a, pb.xc + 15, 24);
  memcpy(xc.ba.a, pb.xc + 18, 24);
  memcpy(xc.g.a, pb.xc + 21, 24);
  memcpy(xc.cov.a, pb.xc + kXS, 225 * sizeof(double));
  for (size_t i = 0; i < P->x_buf.size(); i++) {
    const double* o = pb.xs + (i + q.shift) * kXS;
    HX& h = P->x_buf[i];
    memcpy(h.R.a, o, 72);
    memcpy(h.p.a, o + 9, 24);
    memcpy(h.v.a, o + 12, 24);
    memcpy(h.bg.a, o + 15, 24);
    memcpy(h.ba.a, o + 18, 24);
    memcpy(h.g.a, o + 21, 24);
  }
  if (q.pushed >= 0 && q.pushed < (int)P->x_buf.size()) P->x_buf[q.pushed].cov = xc.cov;
  if (!q.init_tail) {  // pub_localtraj's path point and save_pose_tum's row (local_mapping.cpp:427-430)
    P->traj.push_back(q.t);
    for (int i = 0; i < 12; i++) P->traj.push_back(pb.traj[i]);
    P->path.push_back(q.t);
    for (int i = 0; i < 12; i++) P->path.push_back(pb.traj[i]);
    P->path.push_back(P->jour);
    q.st.iekf_iters = pb.iekf_iters;
    for (int i = 0; i < 4; i++) q.st.iekf_matches[i] = pb.matches[i];
    q.st.iekf_points = pb.iekf_pts;
    q.st.degenerate = degenerate_of(pb.nnt);
  }
  q.st.ba_iters = pb.ba_iters1;
  q.st.ba_hess = pb.ba_hess1;
  for (int i = 0; i < 4; i++) q.st.iekf_planes[i] = pb.planes[i];
  if (q.shift) {  // pub_localmap (publishers.cpp:121-129, local_mapping.cpp:505): the window's path rows
                  // [win_base, win_base + win_count) take x_buf[i].p after the BA (pb.xs: the window before the slide)
    const int W = ctx->cfg.win_size;
    const int rows = (int)P->path.size() / kPathRow;
    if (rows >= W)
      for (int i = 0; i < W; i++) memcpy(&P->path[(size_t)(rows - W + i) * kPathRow + 10], pb.xs + (size_t)i * kXS + 9, 24);
  }
  if (q.jour_check) {  // local_mapping.cpp:525-533 with x_curr.p = x_buf.back().p after the BA
    double spat = norm3(sub(xc.p, P->last_pos));
    if (spat > 0.5) {
      P->jour += spat;
      P->last_pos = xc.p;
      P->release_flag = true;
    }
  }
  q.seq1 = 0;
  return VG_OK;
}

// k_iekf launches of the executed IEKF iterations (vg_profile bit 0)
static void collect_iekf_events(vg_ctx* ctx, const Pend& q) {
  for (int r = 0; r < q.ev_n && r < q.st.iekf_iters; r++) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ctx->iekf_ev[q.ev_base + r][0], ctx->iekf_ev[q.ev_base + r][1]) == hipSuccess) {
      ctx->prof_ms[kProfIekfKernel] += ms;
      ctx->prof_n[kProfIekfKernel] += 1;
    }
  }
}

// P2: end-of-scan counters; the scan's stats are complete
static int absorb_p2(vg_ctx* ctx, HostPipe* P, Pend& q) {
  VG_TRY(absorb_p1(ctx, P, q));
  VG_TRY(pub_wait(ctx, &ctx->h_pub->seq2, q.seq2, "counter publication"));
  const int* c = ctx->h_pub->counters;
  q.st.n_slide = c[kCntSlide];
  q.st.nodes_used = c[kCntNodes];
  q.st.fix_used = c[kCntFix];
  if (!q.init_tail) q.st.roots_new = c[kCntRoots];  // init: the rebuilt map's roots (init.cpp)
  q.st.plane_updates = c[kCntPlaneUpd];
  if (!q.init_tail) {  // the insert's downsampled count (the insert read it on the device)
    q.st.n_ds = c[kCntNds];
    if (q.ins_slot >= 0) P->wp_n[q.ins_slot] = c[kCntNds];
  }
  q.st.fix_full = c[kCntFixFull];
  q.st.v_ins = c[kCntSeg];
  // events recorded while this scan was enqueued are complete now
  collect_iekf_events(ctx, q);
  for (int i = 0; i < kProfN; i++)
    if (ctx->prof_pending[i] && i != kProfIekfKernel) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ctx->prof_ev[i][0], ctx->prof_ev[i][1]) == hipSuccess) {
        ctx->prof_ms[i] += ms;
        ctx->prof_n[i] += 1;
      }
      ctx->prof_pending[i] = false;
    }
  ctx->stats = q.st;
  P->stats_log.push_back(q.st);
  if (c[kCntErr]) return map_error(ctx, c[kCntErr]);
  return VG_OK;
}

// The outcome of the previous fused step's LM (stage_ba left it pending):
// ba_resolve waits for its flags and enqueues any further iteration; if the
// speculative margi tail did not run, the real one follows with the same
// publication numbers and window view, so every wait already enqueued on
// those numbers (the next IEKF's hand-off flags, the host's P1 / P2) holds.
// block = false: returns without waiting when a flag is not published yet.
static int resolve_lm(vg_ctx* ctx, HostPipe* P, bool block = true) {
  if (!P->lmp.active) return VG_OK;
  HostTimer ht_(ctx, kHostBA);
  bool fin = true, tail_ok = true;
  int iters = 0;
  int r = ba_resolve(ctx, block, &fin, &iters, &tail_ok);
  if (r == VG_OK && !fin) return VG_OK;
  P->lmp.active = false;
  if (r == VG_OK && !tail_ok)
    r = map_margi(ctx, P->mpd, P->lmp.wa, 0, ctx->cfg.thread_num, P->lmp.seq1, P->lmp.seq2, nullptr);
  if (r != VG_OK) P->sticky = r;
  return r;
}

// absorb every pending scan whose results are needed (all of P1, and P2 when
// `full`); blocking
int absorb(vg_ctx* ctx, HostPipe* P, bool full) {
  if (P->sticky != VG_OK) return P->sticky;
  VG_TRY(resolve_lm(ctx, P));
  int r = VG_OK;
  while (!P->pend.empty()) {
    Pend& q = P->pend.front();
    r = full || P->pend.size() > 1 ? absorb_p2(ctx, P, q) : absorb_p1(ctx, P, q);
    if (r != VG_OK) break;
    if (q.seq1 == 0 && (full || P->pend.size() > 1)) {
      P->pend.pop_front();
    } else {
      break;
    }
  }
  if (r != VG_OK) P->sticky = r;
  return r;
}

// non-blocking: absorb, oldest first, every pending scan whose publications
// (state and end-of-scan counters) have both arrived; stops at the first that
// has not. Only the newest pending scan can be unpublished (the host absorbs a
// scan's state before the next scan publishes), so the Pub block holds the
// scan being absorbed.
int absorb_ready(vg_ctx* ctx, HostPipe* P) {
  if (P->sticky != VG_OK) return P->sticky;
  VG_TRY(resolve_lm(ctx, P, false));
  if (P->lmp.active) return VG_OK;  // the LM is still running: nothing of that scan is published
  while (!P->pend.empty()) {
    Pend& q = P->pend.front();
    if (q.seq1 != 0 && __atomic_load_n(&ctx->h_pub->seq1, __ATOMIC_ACQUIRE) < q.seq1) break;
    if (__atomic_load_n(&ctx->h_pub->seq2, __ATOMIC_ACQUIRE) < q.seq2) break;
    const int r = absorb_p2(ctx, P, q);
    if (r != VG_OK) {
      P->sticky = r;
      return r;
    }
    P->pend.pop_front();
  }
  return VG_OK;
}

int host_sync(vg_ctx* ctx) {
  HostPipe* P = hp(ctx);
  if (P->in_scan) {
    ctx->err = "host_sync inside a scan";
    return VG_E_STATE;
  }
  VG_TRY(resolve_lm(ctx, P));  // before the drain: it may enqueue work
  VG_HIP(stream_wait(ctx));
  return absorb(ctx, P, true);
}

// IMUEKF::motion_blur state/covariance propagation (imu_ekf.cpp:28-94); the
// per-point deskew (114-144) is SURVEY row f1 (callers pass compensated scans).
// one row of a sparse 15x15 matrix: its non-zero columns, ascending
struct SpRow {
  int n;
  int k[7];
  double v[7];
};
// F C F^T + Q with F given by its rows; every sum in ascending column order
// (the dense product's order, zero terms dropped)
static M15 sandwich(const SpRow* F, const M15& C, const M15& Q) {
  M15 A, out;
  for (int i = 0; i < 15; i++)
    for (int j = 0; j < 15; j++) {
      double s = F[i].v[0] * C(F[i].k[0], j);
      for (int t = 1; t < F[i].n; t++) s += F[i].v[t] * C(F[i].k[t], j);
      A(i, j) = s;
    }
  for (int i = 0; i < 15; i++)
    for (int j = 0; j < 15; j++) {
      double s = A(i, F[j].k[0]) * F[j].v[0];
      for (int t = 1; t < F[j].n; t++) s += A(i, F[j].k[t]) * F[j].v[t];
      out(i, j) = s + Q(i, j);
    }
  return out;
}

void propagate(vg_ctx* ctx, HostPipe* P, const std::vector<Imu>& imus, double pcl_beg, double pcl_end) {
  P->poses.clear();
  const vg_config& c = ctx->cfg;
  HX& xc = P->x_curr;
  V3 acc_imu = V3::Z(), angvel = V3::Z(), acc_avr, vel = xc.v, pos = xc.p;
  M3 R_imu = xc.R;
  double dt = 0;
  for (size_t k = 0; k + 1 < imus.size(); k++) {
    const Imu& head = imus[k];
    const Imu& tail = imus[k + 1];
    if (head.t < P->last_pcl_end_time) continue;
    for (int j = 0; j < 3; j++) {
      angvel[j] = 0.5 * (head.gyr[j] + tail.gyr[j]);
      acc_avr[j] = 0.5 * (head.acc[j] + tail.acc[j]);
    }
    angvel = sub(angvel, xc.bg);
    acc_avr = sub(scl(acc_avr, P->sg), xc.ba);  // imu_ekf.cpp:51
    acc_imu = add(mul(R_imu, acc_avr), xc.g);
    double cur = head.t;
    if (cur < P->last_pcl_end_time) cur = P->last_pcl_end_time;
    dt = tail.t - cur;
    {  // imu_poses.emplace_back(offt, R_imu, pos_imu, vel_imu, angvel_avr, acc_imu) (imu_ekf.cpp:64)
      double rec[22];
      rec[0] = cur - pcl_beg;
      memcpy(rec + 1, R_imu.a, 72);
      memcpy(rec + 10, pos.a, 24);
      memcpy(rec + 13, vel.a, 24);
      memcpy(rec + 16, angvel.a, 24);
      memcpy(rec + 19, acc_imu.a, 24);
      P->poses.insert(P->poses.end(), rec, rec + 22);
    }
    M3 ask = hat(acc_avr);
    M3 Exp_f = Exp(angvel, dt);
    M15 cw = M15::Z();
    M3 F00 = Exp(angvel, -dt), F60 = scl(mul(R_imu, ask), -dt), F612 = scl(R_imu, -dt);
    M3 ca = M3::Z();
    for (int j = 0; j < 3; j++) ca(j, j) = c.odo_cov_acc;
    M3 cw66 = scl(mul(mul(R_imu, ca), tr(R_imu)), dt * dt);
    for (int r = 0; r < 3; r++) {
      for (int q = 0; q < 3; q++) cw(6 + r, 6 + q) = cw66(r, q);
      cw(r, r) = c.odo_cov_gyr * dt * dt;
      cw(9 + r, 9 + r) = c.odo_rdw_gyr * dt * dt;
      cw(12 + r, 12 + r) = c.odo_rdw_acc * dt * dt;
    }
    // cov = F cov F^T + cw (imu_ekf.cpp:79) with F's non-zeros only: F is the
    // identity but for rows 0-2 (F00, -dt I), 3-5 (I, dt I) and 6-8 (F60, I,
    // F612). Terms are summed in ascending column order, as the dense product
    // does, and the zero terms it adds are exact no-ops: same bits, 5x fewer
    // flops on the host's per-scan critical path.
    SpRow Fr[15];
    for (int r = 0; r < 3; r++) {
      Fr[r] = SpRow{4, {0, 1, 2, 9 + r}, {F00(r, 0), F00(r, 1), F00(r, 2), -dt}};
      Fr[3 + r] = SpRow{2, {3 + r, 6 + r}, {1.0, dt}};
      Fr[6 + r] = SpRow{7, {0, 1, 2, 6 + r, 12, 13, 14}, {F60(r, 0), F60(r, 1), F60(r, 2), 1.0, F612(r, 0),
                                                           F612(r, 1), F612(r, 2)}};
    }
    for (int r = 9; r < 15; r++) Fr[r] = SpRow{1, {r}, {1.0}};
    xc.cov = sandwich(Fr, xc.cov, cw);
    pos = add(add(pos, scl(vel, dt)), scl(acc_imu, 0.5 * dt * dt));
    vel = add(vel, scl(acc_imu, dt));
    R_imu = mul(R_imu, Exp_f);
  }
  if (!imus.empty()) {
    double note = pcl_end > imus.back().t ? 1.0 : -1.0;
    dt = note * (pcl_end - imus.back().t);
    xc.v = add(vel, scl(acc_imu, note * dt));
    xc.R = mul(R_imu, Exp(scl(angvel, note), dt));
    xc.p = add(add(pos, scl(vel, note * dt)), scl(acc_imu, note * 0.5 * dt * dt));
  }
  xc.t = pcl_end;
  P->last_pcl_end_time = pcl_end;
}

// LioStateEstimation (odometry.cpp:64-255) with use_vnc = true (4 iterations),
// enqueued: each iteration is the k_iekf point loop and the device update
// (state.hip k_iekf_update); iterations after convergence are no-ops on the
// device. The VNC scan-plane prep (84-96, 150-190) contributes nothing
// (SURVEY finding 3: matchVoxelMap always returns 0) and is skipped as
// output-invariant.
static int flush_deferred_push(vg_ctx* ctx, HostPipe* P) {
  if (!P->push_pending) return VG_OK;
  VG_TRY(flush_begin(ctx, P));
  P->push_pending = false;
  return state_push(ctx, P->push.ord, P->push.new_imu, P->push.rec);
}
static int lio_state_estimation(vg_ctx* ctx, HostPipe* P, const float* x, const float* y, const float* z, int n) {
  // event pairs alternate between two banks: scan k's are collected while
  // scan k+1 is being enqueued
  ctx->iekf_ring_base = ctx->iekf_ring_base == 0 ? 8 : 0;
  P->cur.ev_base = ctx->iekf_ring_base;
  P->cur.ev_n = (ctx->prof_on && (ctx->prof_stages || !ctx->use_graphs || sharded(ctx))) ? 4 : 0;
  VG_TRY(flush_deferred_push(ctx, P));
  const bool begin = P->begin_pending;
  P->begin_pending = false;
  // behind the previous margi's plane updates only (map_margi): its
  // remainder on the main stream runs under this IEKF, and the main stream
  // then waits for the IEKF. The opening (k_scan_begin) goes with it.
  // (sharded: the IEKF's exchanges go on the IEKF stream, shard_exchange; the
  // hand-offs are events, sync_tail_armed being off)
  const bool split = ctx->tail_a_valid && ctx->overlap_iekf && ctx->use_graphs && !ctx->prof_stages;
  ctx->tail_a_valid = false;
  const double* bxc = begin && !P->begin_prop ? P->begin_xc : nullptr;
  const PropArg* bprop = begin && P->begin_prop ? &P->prop : nullptr;
  // host_step's early downsample: enqueued behind this IEKF's launches when
  // those go out without a host wait (below), else first
  auto ds_hook = [&]() -> int {
    if (!P->ds_hook) return VG_OK;
    const std::function<int()> h = std::move(P->ds_hook);
    P->ds_hook = nullptr;
    return h();
  };
  // a pending LM is resolved before this IEKF is enqueued unless the IEKF
  // stream waits for the margi on device flags (the numbers the real tail
  // stores as well) and starts from the device's state
  if (!(split && ctx->flag_sync && ctx->sync_tail_armed && bprop)) {
    VG_TRY(ds_hook());
    VG_TRY(resolve_lm(ctx, P));
  }
  if (!split) return iekf_run(ctx, P->mpd, x, y, z, n, ctx->iekf_ring_base, bxc, nullptr, bprop);
  // created on first use: a context of the multi-sequence mode never makes
  // it (vg_multi_create), as a third stream per sequence makes sequences
  // share hardware queues (B = 4: 2,742 -> 1,430 scans/s)
  if (!ctx->stream_iekf) VG_HIP(hipStreamCreateWithFlags(&ctx->stream_iekf, hipStreamNonBlocking));
  const bool flags = ctx->flag_sync && ctx->sync_tail_armed;  // state.hip k_sync_*: no late-released event waits
  // (flag_sync is off when kernels run serialised: vg_create, VG_SERIAL_KERNELS)
  ctx->sync_tail_armed = false;
  bool opened = false;
  if (flags && bprop) {
    // the device propagation needs only x_curr, final once the margi head
    // (k_margi_leaf's workgroup 0) stored it: it runs under the leaves'
    // plane updates, and the IEKF waits for those alone
    // (both waits inside k_scan_prop: no polling kernels, no launch gap)
    if (ctx->in_ev) VG_HIP(hipStreamWaitEvent(ctx->stream_iekf, ctx->in_ev, 0));  // a host-input scan's unpack
    VG_TRY(state_scan_begin(ctx, nullptr, x, y, z, n, ctx->stream_iekf, bprop, ctx->d_sync + 2, ctx->sync_tail_value,
                            ctx->d_sync, ctx->sync_tail_value));
    bprop = nullptr;
    opened = true;
  } else {
    if (flags) VG_TRY(sync_wait(ctx, ctx->stream_iekf, 0, ctx->sync_tail_value));
    else VG_HIP(hipStreamWaitEvent(ctx->stream_iekf, ctx->ev_tail_a, 0));
    if (ctx->in_ev) VG_HIP(hipStreamWaitEvent(ctx->stream_iekf, ctx->in_ev, 0));  // a host-input scan's unpack
  }
  // the early downsample between the device propagation's launch and the
  // IEKF's: k_scan_prop (queued) waits on the device for the margi while the
  // host enqueues the downsample, which still runs under the previous LM, and
  // the IEKF's graph goes in before k_scan_prop ends
  VG_TRY(ds_hook());
  bool signalled = false;  // k_iekf_all advanced the flag itself (no k_sync_set launch)
  VG_TRY(iekf_run(ctx, P->mpd, x, y, z, n, ctx->iekf_ring_base, bxc, ctx->stream_iekf, bprop, flags, &signalled,
                  opened));
  if (flags) {
    const unsigned v = ++ctx->sync_iekf_value;
    if (!signalled) VG_TRY(sync_set(ctx, ctx->stream_iekf, 1, v));
    // the previous LM's further iterations and real margi tail, if any, go
    // onto the main stream ahead of its wait for this IEKF
    VG_TRY(resolve_lm(ctx, P));
    VG_TRY(sync_wait(ctx, ctx->stream, 1, v));
  } else {
    VG_HIP(hipEventRecord(ctx->ev_iekf_done, ctx->stream_iekf));
    VG_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_iekf_done, 0));
  }
  return VG_OK;
}

static WinArg make_winarg(const HostPipe* P, int set_xc) {
  WinArg w;
  memset(&w, 0, sizeof(w));
  for (size_t i = 0; i < P->mp.size() && i < 32; i++) w.mp[i] = P->mp[i];
  for (int i = 0; i < P->win_count && i < 32; i++) w.nper[i] = P->wp_n[P->mp[i]];
  w.win_count = P->win_count;
  w.set_xc = set_xc;
  w.jour_check = ((P->win_base + P->win_count) % 10 == 0) ? 1 : 0;  // local_mapping.cpp:510 (stage_margi_slide)
  return w;
}

// ---- stage entry points (one per reference call in local_mapping.cpp:389-547)

static int need_open(vg_ctx* ctx, HostPipe* P, const char* what) {
  if (P->sticky != VG_OK) return P->sticky;
  if (!P->in_scan) {
    ctx->err = std::string(what) + ": no scan in progress (vg_propagate first)";
    return VG_E_STATE;
  }
  return VG_OK;
}

// the scan propagates on the device (k_scan_prop) rather than on the host
// after a wait for the previous scan's state
static bool prop_on_device(vg_ctx* ctx, const HostPipe* P, int m, bool dev) {
  return dev && (ctx->dev_prop || P->lmp.active) && !P->first && m <= kPropMax && P->sticky == VG_OK;
}

// odom_ekf.process -> motion_blur state/covariance part (local_mapping.cpp:389);
// opens the scan on the device (x_curr, x_prop, cov_inv)
int stage_propagate(vg_ctx* ctx, const double* imu, int m, double beg, double end, bool dev) {
  HostTimer ht_(ctx, kHostPropagate);
  HostPipe* P = hp(ctx);
  if (P->in_scan) {
    ctx->err = "vg_propagate: previous scan not finished (vg_step_end)";
    return VG_E_STATE;
  }
  if (init_active(P)) {
    ctx->err = "vg_propagate: cold-start initialisation in progress (use vg_step* until init_phase 3)";
    return VG_E_STATE;
  }
  if (ctx->flag_sync && !ctx->flag_force && dev_ctx_count(ctx->device) > 1) {  // another context on the device: event waits from here
    VG_TRY(host_sync(ctx));
    ctx->flag_sync = false;
  }
  // device propagation (k_scan_prop): from the device's x_curr, so the host
  // does not wait for the previous scan's state here (the window push absorbs
  // it, behind the IEKF's enqueue); the first scan has nothing to propagate
  // A pending LM (the previous fused step returned before its outcome):
  // only the device has that scan's state, so it propagates there
  P->begin_prop = prop_on_device(ctx, P, m, dev);
  if (P->begin_prop) {
    PropArg& a = P->prop;
    const vg_config& c = ctx->cfg;
    a.n = m;
    a.last_end = P->last_pcl_end_time;
    a.beg = beg;
    a.end = end;
    a.sg = P->sg;
    a.cov_gyr = c.odo_cov_gyr;
    a.cov_acc = c.odo_cov_acc;
    a.rdw_gyr = c.odo_rdw_gyr;
    a.rdw_acc = c.odo_rdw_acc;
    if (m > 0) memcpy(a.imu, imu, (size_t)m * 7 * sizeof(double));
    P->poses.clear();
    P->x_curr.t = end;
    P->last_pcl_end_time = end;
  } else {
    VG_TRY(absorb(ctx, P, false));  // x_curr / x_buf of the previous scan
    P->poses.clear();
    if (!P->first) {
      propagate(ctx, P, to_imus(imu, m), beg, end);
    } else {
      P->x_curr.t = end;
      P->last_pcl_end_time = end;
    }
    double* xc = P->begin_xc;  // opened on the device with the IEKF's first launch (flush_begin otherwise)
    const HX& h = P->x_curr;
    memcpy(xc, h.R.a, 72);
    memcpy(xc + 9, h.p.a, 24);
    memcpy(xc + 12, h.v.a, 24);
    memcpy(xc + 15, h.bg.a, 24);
    memcpy(xc + 18, h.ba.a, 24);
    memcpy(xc + 21, h.g.a, 24);
    memcpy(xc + kXS, h.cov.a, 225 * sizeof(double));
  }
  P->begin_pending = true;
  P->push_pending = false;
  P->cur = Pend();
  memset(&P->cur.st, 0, sizeof(P->cur.st));
  P->cur.t = end;
  P->in_scan = true;
  P->published = false;
  P->ds_seq = 0;
  P->ds_n = -1;
  P->ins_slot = -1;
  P->prefix = false;
  P->tail_queued = false;
  return VG_OK;
}

// the downsampled point count for a caller of the stage-level API (the
// pipeline itself never waits for it: the insert reads it on the device)
static int resolve_ds(vg_ctx* ctx, HostPipe* P) {
  if (P->ds_n >= 0) return VG_OK;
  VG_TRY(pub_wait(ctx, &ctx->h_pub->seq_ds, P->ds_seq, "downsample", ctx->stream_ds));
  if (ctx->h_pub->ds_err) {
    ctx->err = "voxel key out of packed range (|key| >= 2^20)";
    return VG_E_RANGE;
  }
  P->ds_n = ctx->h_pub->n_ds;
  P->cur.st.n_ds = P->ds_n;
  return VG_OK;
}

// down_sampling_voxel(pl_down, down_size) and its /2 fallback below 2000
// voxels (local_mapping.cpp:396-403), both decided on the device
// (ds_enqueue_hashed): the host never waits for the count, the GPU runs the
// IEKF meanwhile and the insert reads the count where it lands
// the downsample's device work on its own stream, which waits only until the
// previous insert has read the ds buffers (and for a deskewed scan)
static int ds_enqueue_scan(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n,
                           int pub_seq) {
  if (ctx->want_ds_stream && ctx->stream_ds == ctx->stream) {
    // the new stream starts behind everything already on the main stream: the
    // scan's upload + unpack (upload_scan ran while the two were one stream)
    // and the previous scans' inserts, none of which recorded an event it waits on
    VG_HIP(hipStreamCreateWithFlags(&ctx->stream_ds, hipStreamNonBlocking));
    VG_HIP(hipEventRecord(ctx->ev_ds_done, ctx->stream));
    VG_HIP(hipStreamWaitEvent(ctx->stream_ds, ctx->ev_ds_done, 0));
  }
  VG_HIP(flush_insert_events(ctx));
  VG_HIP(hipStreamWaitEvent(ctx->stream_ds, ctx->ds_free_ev ? ctx->ds_free_ev : ctx->ev_ds_free, 0));
  VG_HIP(hipStreamWaitEvent(ctx->stream_ds, ctx->ev_scan_ready, 0));  // a deskewed scan (no-op otherwise)
  prof_begin(ctx, kProfDownsample, ctx->stream_ds);
  VG_TRY(ds_enqueue_hashed(ctx, ctx->stream_ds, dx, dy, dz, di, n, ctx->cfg.down_size, true, pub_seq));
  prof_end(ctx, kProfDownsample, ctx->stream_ds);
  VG_HIP(hipEventRecord(ctx->ev_ds_done, ctx->stream_ds));
  return VG_OK;
}

// the scan's raw cloud as the insert's input; early: its downsample is already
// enqueued (host_step)
static void ds_adopt(HostPipe* P, const float* dx, const float* dy, const float* dz, const float* di, int n) {
  P->sx = dx;
  P->sy = dy;
  P->sz = dz;
  P->si = di;
  P->n_raw = n;
  P->cur.st.n_raw = n;
  P->ds_n = -1;
}

int stage_downsample(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n,
                     int* n_ds_out) {
  HostTimer ht_(ctx, kHostDownsample);
  HostPipe* P = hp(ctx);
  VG_TRY(need_open(ctx, P, "vg_downsample_scan"));
  ds_adopt(P, dx, dy, dz, di, n);
  P->ds_seq = n_ds_out ? ++ctx->pub_seq : -1;  // published only for a stage-level caller
  VG_TRY(ds_enqueue_scan(ctx, dx, dy, dz, di, n, n_ds_out ? P->ds_seq : 0));
  if (n_ds_out) {
    VG_TRY(resolve_ds(ctx, P));
    *n_ds_out = P->ds_n;
  }
  return VG_OK;
}

// VNC_lio(no_ds_pptr) on the full cloud (local_mapping.cpp:408-430)
int stage_iekf(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, int n, int* degenerate_out) {
  HostTimer ht_(ctx, kHostIekf);
  HostPipe* P = hp(ctx);
  VG_TRY(need_open(ctx, P, "vg_lio_state_estimation"));
  prof_begin(ctx, kProfIekf);
  VG_TRY(lio_state_estimation(ctx, P, dx, dy, dz, n));
  prof_end(ctx, kProfIekf);
  if (degenerate_out) {  // stage API caller wants the flag now: read it from the device state
    double* h = ctx->h_stage;
    VG_HIP(hipMemcpyAsync(h, ctx->st->nnt, 6 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    VG_HIP(stream_wait(ctx));
    *degenerate_out = degenerate_of(h);
  }
  return VG_OK;
}

// x_buf / pvec_buf / imu_pre_buf push (local_mapping.cpp:434-441)
int stage_window_push(vg_ctx* ctx, const double* imu, int m) {
  HostTimer ht_(ctx, kHostPush);
  HostPipe* P = hp(ctx);
  VG_TRY(need_open(ctx, P, "vg_window_push"));
  // the previous scan's window after its BA (the IMU_PRE bias below); already
  // absorbed unless this scan propagated on the device
  VG_TRY(absorb(ctx, P, false));
  if (P->win_count >= 32) {
    ctx->err = "vg_window_push: window full";
    return VG_E_STATE;
  }
  P->win_count++;
  P->x_buf.push_back(P->x_curr);  // device values arrive with the scan's publication
  P->x_buf.back().t = P->cur.t;
  P->cur.pushed = P->win_count - 1;
  int new_imu = -1;
  if (P->win_count > 1) {
    const HX& xb = P->x_buf[P->win_count - 2];
    P->imu_pre.emplace_back(xb.bg, xb.ba);
    P->imu_pre.back().push_imu(to_imus(imu, m), P->noiseMeas, P->noiseWalk, P->sg);
    P->imu_pre.back().rec.resize(kBaImuRec);
    P->imu_pre.back().record(P->imu_pre.back().rec.data());  // off the BA's critical path
    new_imu = P->win_count - 2;
  }
  // deferred: the insert's first launch carries it (map_insert), else flush_deferred
  P->push.ord = P->win_count - 1;
  P->push.new_imu = new_imu;
  if (new_imu >= 0) memcpy(P->push.rec, P->imu_pre.back().rec.data(), sizeof(P->push.rec));
  else memset(P->push.rec, 0, sizeof(P->push.rec));
  P->push_pending = true;
  return VG_OK;
}

// pvec_update + cut_voxel_multi of the downsampled scan (local_mapping.cpp:425-448)
int stage_insert(vg_ctx* ctx) {
  HostTimer ht_(ctx, kHostInsert);
  HostPipe* P = hp(ctx);
  const vg_config& c = ctx->cfg;
  VG_TRY(need_open(ctx, P, "vg_cut_voxel_multi"));
  if (P->win_count <= 0) {
    ctx->err = "vg_map_insert: window is empty (push the scan first)";
    return VG_E_STATE;
  }
  if (P->ds_seq == 0) {
    ctx->err = "vg_cut_voxel_multi: no downsampled scan";
    return VG_E_STATE;
  }
  VG_TRY(absorb(ctx, P, true));  // earlier scans are complete by now (stream order)
  const int ord = P->win_count - 1;
  const int slot = P->mp[ord];
  P->epoch++;
  VG_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_ds_done, 0));
  VG_TRY(flush_begin(ctx, P));
  prof_begin(ctx, kProfInsert);
  const bool push = P->push_pending;
  P->push_pending = false;
  // the downsampled count stays on the device (n_raw bounds the grids)
  VG_TRY(map_insert(ctx, P->mpd, slot, P->n_raw, P->epoch, c.thread_num, push ? &P->push : nullptr, nullptr,
                    ctx->ds.hflags + 1));
  prof_end(ctx, kProfInsert);
  VG_HIP(hipEventRecord(ctx->ev_ds_free, ctx->stream));  // the insert has read the ds buffers
  ctx->ds_free_ev = ctx->ev_ds_free;
  P->wp_n[slot] = P->n_raw;  // an upper bound until the scan's counters are absorbed (absorb_p2)
  P->ins_slot = slot;
  P->cur.ins_slot = slot;
  P->ins_n = -1;
  return VG_OK;
}

// the insert's downsampled count, read back (the rare insert-replay path only)
static int insert_replay(vg_ctx* ctx, HostPipe* P) {
  if (P->ins_n < 0) {
    VG_HIP(hipMemcpyAsync(ctx->h_pinned, ctx->ds.hflags + 1, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    VG_HIP(hipStreamSynchronize(ctx->stream));
    P->ins_n = ctx->h_pinned[0];
  }
  return map_insert_replay(ctx, P->mpd, P->ins_slot, P->ins_n, ctx->cfg.thread_num);
}

// The steady state's insert + recut (local_mapping.cpp:425-451) as one
// replayed graph per ring position mp[0]: every argument is fixed for a full
// window (slot = mp[W-1], the window view, grids sized by the capacity), every
// count lives on the device, and the scan's push record is read from
// host-mapped memory. One launch instead of ~26, each kernel ~2-3 us cheaper
// to dispatch. Conditions: graphs on, unsharded, the LM follows (the recut's
// factor extraction is the asynchronous one), no debug capacity overrides.
static bool mid_graph_ok(vg_ctx* ctx, const HostPipe* P) {
  const vg_config& c = ctx->cfg;
  return ctx->use_graphs && !ctx->prof_stages && !sharded(ctx) && c.if_BA == 1 &&
         P->win_count == c.win_size && P->push_pending && P->push.ord == c.win_size - 1 && !P->begin_pending &&
         ctx->dbg_apply_cap < 0 && ctx->dbg_ins_cap < 0 && ctx->dbg_fac_max < 0 && P->ds_seq != 0;
}
// The scan graph: the same insert + recut, then k_ba_init, the first two LM
// iterations and the margi tail gated on the LM's end (a speculative tail
// inside the graph), one launch per scan on the main stream — no graph
// boundaries between the recut, the LM and the margi (each left the stream
// idle 5-14 us). Per-scan numbers (the LM's flag numbers, the tail's
// publication numbers, two hand-off values) go through the ring position's
// host-mapped slot into DState::ph (k_ins_prep). Events cannot be recorded
// inside it, so the margi prefix waits for the recut on a device flag
// (k_ba_init raises d_sync[3]) and the tail for the prefix on another
// (d_sync[4]); the next downsample follows the prefix on its stream.
// Conditions: the steady state predicted 2 LM iterations (the graph holds 2),
// the flag hand-offs, no /map_cmap publication in the tail.
static bool scan_graph_ok(vg_ctx* ctx, const HostPipe* P) {
  return ctx->scan_graph && ctx->spec_tail && ctx->ba_graph && ctx->ba_graph2 && ctx->ba_last_iters == 2 &&
         ctx->flag_sync && !ctx->serial_kernels && ctx->overlap_iekf && ctx->want_ds_stream &&
         !(ctx->prof_on && !ctx->prof_clock) &&
         ctx->dbg_capture != 1 && !(ctx->pub_flags & 1) && !P->lmp.active;
}
static int stage_insert_recut(vg_ctx* ctx) {
  HostTimer ht_(ctx, kHostInsert);
  HostPipe* P = hp(ctx);
  const vg_config& c = ctx->cfg;
  VG_TRY(need_open(ctx, P, "vg_cut_voxel_multi"));
  VG_TRY(absorb(ctx, P, true));  // earlier scans are complete by now (stream order)
  const int W = c.win_size;
  const int slot = P->mp[W - 1], ring0 = P->mp[0];
  P->epoch++;
  VG_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_ds_done, 0));
  P->push_pending = false;
  const bool sg = scan_graph_ok(ctx, P);
  P->scan_g = sg;
  ctx->in_sel = ring0;  // this ring position's host-mapped inputs
  HostIn& hin = ctx->h_in[ring0];
  hin.push = P->push;  // this scan's record, read by the replay
  if (sg) {
    const int seq0 = ctx->pub_seq + 1;  // the LM's flag numbers (ba_run's)
    ctx->pub_seq += 10;
    ctx->ba_seq0_pre = seq0;
    P->tail_seq1 = ++ctx->pub_seq;  // the tail's publication numbers (margi_enqueue's)
    P->tail_seq2 = ++ctx->pub_seq;
    P->tail_wa = make_winarg(P, 1);
    P->sg_flags[0] = ++ctx->rc_flag_ctr;
    P->sg_flags[1] = ++ctx->pre_flag_ctr;
    const int ph[6] = {seq0, P->tail_seq1, P->tail_seq2, (int)P->sg_flags[0], (int)P->sg_flags[1],
                       P->tail_wa.jour_check};
    memcpy(hin.ph, ph, sizeof(ph));
  }
  hipGraphExec_t& ge = sg ? ctx->g_scan[ring0] : ctx->g_mid[ring0];
  if (!ge) {
    const int cap = ctx->cap.max_points_per_scan;
    WinArg wa = make_winarg(P, 0);
    for (int i = 0; i < W; i++) wa.nper[i] = cap;  // grid bounds only: the kernels read the device counts
    hipStream_t s = ctx->stream;
    std::lock_guard<std::recursive_mutex> cap_lk_(capture_mutex());  // (vg_internal.h)
    VG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    ctx->capturing = true;
    ctx->in_ph = sg;
    ctx->rc_begin_wa = ctx->rc_begin_fold ? &wa : nullptr;  // the recut's head rides in the insert's last launch
    int nf = 0;
    int r = map_insert(ctx, P->mpd, slot, cap, P->epoch, c.thread_num, &P->push, nullptr, ctx->ds.hflags + 1);
    ctx->rc_begin_wa = nullptr;
    ctx->in_ph = false;
    if (r == VG_OK) r = map_recut(ctx, P->mpd, wa, c.thread_num, &nf, false, 1);
    if (r == VG_OK && sg) r = ba_capture_scan_lm(ctx, P->mp.data());
    if (r == VG_OK && sg) r = map_margi_tail_capture(ctx, P->mpd, P->tail_wa);
    ctx->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    VG_TRY(r);
    VG_HIP(e);
    VG_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    VG_HIP(hipGraphDestroy(g));
  }
  prof_begin(ctx, kProfInsert);
  VG_HIP(hipGraphLaunch(ge, ctx->stream));
  prof_end(ctx, kProfInsert);
  // the insert + recut graph's asynchronous recut leaves tras_opt's factor
  // bookkeeping to the LM's k_ba_init (the scan graph holds that k_ba_init)
  if (!sg) ctx->rc_finish_in_init = ctx->rc_init_finish;
  if (sg) {  // nothing to record: the prefix and the next downsample order themselves on the flags
    ctx->ins_ev_pending = false;
    ctx->tail_a_valid = true;  // the next IEKF waits for this graph's tail (device flags)
    P->wp_n[slot] = P->n_raw;
    P->ins_slot = slot;
    P->cur.ins_slot = slot;
    P->ins_n = -1;
    P->rc_seq = ++ctx->rc_pub;
    return VG_OK;
  }
  // ev_ds_free (the insert has read the ds buffers) and ev_recut_done (the
  // margi prefix starts from here): recorded by their first waiter's flush,
  // the LM's right behind k_ba_init (a record right behind the graph leaves
  // the stream idle before k_ba_init). With the early downsample the next
  // scan's downsample is enqueued after this LM anyway; without it the
  // records stay right behind the graph, so that downsample does not wait
  // for k_ba_init.
  ctx->ins_ev_pending = true;
  if (!ctx->ds_early) VG_HIP(flush_insert_events(ctx));
  P->wp_n[slot] = P->n_raw;  // an upper bound until the scan's counters are absorbed (absorb_p2)
  P->ins_slot = slot;
  P->cur.ins_slot = slot;
  P->ins_n = -1;
  P->rc_seq = ++ctx->rc_pub;  // k_fac_sort in the graph publishes the same number
  return VG_OK;
}

// multi_recut + tras_opt (local_mapping.cpp:451)
int stage_recut(vg_ctx* ctx, int* nf_out) {
  HostTimer ht_(ctx, kHostRecut);
  HostPipe* P = hp(ctx);
  const vg_config& c = ctx->cfg;
  VG_TRY(need_open(ctx, P, "vg_multi_recut"));
  VG_TRY(flush_deferred(ctx, P));
  const WinArg wa = make_winarg(P, 0);
  int nf = 0;
  prof_begin(ctx, kProfRecut);
  P->rc_seq = 0;
  if (!nf_out && P->win_count >= c.win_size && c.if_BA == 1) {
    // the LM follows: its kernels read the factor count on the device, and the
    // host learns the recut's outcome only once the LM is enqueued (stage_ba);
    // sharded, the status is all-reduced first (map.hip k_pub_rc), so every
    // rank takes the same host-sized completion and LM rerun
    P->rc_seq = ++ctx->rc_pub;  // the device counts its asynchronous recuts the same way (k_fac_sort)
    VG_TRY(map_recut(ctx, P->mpd, wa, c.thread_num, &nf, false, 1));
    prof_end(ctx, kProfRecut);
    return VG_OK;
  }
  int r = map_recut(ctx, P->mpd, wa, c.thread_num, &nf);
  if (r == kNeedInsertReplay) {  // per shard; the replayed recut has no collective
    VG_TRY(insert_replay(ctx, P));
    r = map_recut(ctx, P->mpd, wa, c.thread_num, &nf, true);
  }
  VG_TRY(r);
  prof_end(ctx, kProfRecut);
  P->cur.st.n_factors = nf;
  P->n_factors = nf;
  if (nf_out) *nf_out = nf;
  return VG_OK;
}

static int margi_enqueue(vg_ctx* ctx, HostPipe* P, const int* gate, int* seq1, int* seq2);

// LI_BA_Optimizer::damping_iter (local_mapping.cpp:492-497) on the device state
int stage_ba(vg_ctx* ctx, int* iters_out, bool margi_follows) {
  HostTimer ht_(ctx, kHostBA);
  HostPipe* P = hp(ctx);
  const int W = ctx->cfg.win_size;
  VG_TRY(need_open(ctx, P, "vg_damping_iter"));
  VG_TRY(flush_deferred(ctx, P));
  if (P->win_count < W) {
    ctx->err = "vg_ba: window not full";
    return VG_E_STATE;
  }
  VG_TRY(resolve_lm(ctx, P));  // (resolved by the IEKF's enqueue already)
  const bool pre = P->scan_g;  // the scan graph holds k_ba_init, two iterations and the gated tail
  P->scan_g = false;
  ctx->ba_no_defer = false;
  int iters = 0;
  prof_begin(ctx, kProfBA);
  // margi's BA-independent part goes onto the second stream once the first LM
  // iterations are enqueued, so it runs under them (map_margi_prefix). After
  // an asynchronous recut, the host first reads its published outcome: a
  // status other than 0 means the recut needs the host-sized path, and the LM
  // kernels skip (k_ba_init read the same status).
  int rc_status = 0;
  auto prefix = [&]() -> int {
    if (P->rc_seq > 0) {
      VG_TRY(pub_wait(ctx, &ctx->h_pub->seq_rc, P->rc_seq, "k_fac_sort"));
      rc_status = __atomic_load_n(&ctx->h_pub->rc_status, __ATOMIC_ACQUIRE);
      if (rc_status) {
        ctx->ba_no_defer = true;  // the scan graph's LM skipped: the host completes the recut below
        return VG_OK;
      }
      P->n_factors = __atomic_load_n(&ctx->h_pub->rc_nf, __ATOMIC_ACQUIRE);
      P->cur.st.n_factors = P->n_factors;
    }
    // after a scan graph whose recut completed on the device, the prefix and the
    // graph's tail meet on device flags (the host-completed recut records events)
    VG_TRY(map_margi_prefix(ctx, P->mpd, P->mp[0], P->wp_n[P->mp[0]], ctx->cfg.thread_num,
                            pre && !rc_status ? P->sg_flags : nullptr));
    P->prefix = true;
    return VG_OK;
  };
  // the margi tail behind the LM (see ba_run): fused step, plain graph path
  // (sharded: the gated tail holds no exchange, and the LM's iteration count —
  // the only thing it depends on — is the same on every rank)
  const bool spec_ok = margi_follows && ctx->spec_tail && ctx->use_graphs && !ctx->prof_stages;
  std::function<int(bool*)> spec = [&](bool* queued) -> int {
    if (rc_status || !P->prefix) return VG_OK;
    VG_TRY(margi_enqueue(ctx, P, ba_gate_dev(ctx), &P->tail_seq1, &P->tail_seq2));
    *queued = true;
    return VG_OK;
  };
  bool tail_ok = false;
  // The outcome may stay pending (ba_run returns once the speculative tail is
  // queued): the next fused step enqueues its downsample, device propagation
  // and IEKF first — all behind the margi on device flags — and reads it then
  // (resolve_lm). Needs the flag hand-offs and the IEKF stream.
  const bool defer = spec_ok && ctx->lm_defer && ctx->flag_sync && !ctx->serial_kernels && ctx->overlap_iekf &&
                     ctx->want_ds_stream && !sharded(ctx);
  bool pending = false;
  VG_TRY(ba_run(ctx, P->n_factors, P->mp.data(), &iters, prefix,
                spec_ok && !pre ? spec : std::function<int(bool*)>(), &tail_ok, defer ? &pending : nullptr, pre ? 2 : 0));
  P->tail_queued = tail_ok && !rc_status;  // (a skipped LM left the graph's tail shut)
  if (pending) {
    P->lmp.active = true;
    P->lmp.seq1 = P->tail_seq1;
    P->lmp.seq2 = P->tail_seq2;
    P->lmp.wa = P->tail_wa;
    P->rc_seq = 0;
    prof_end(ctx, kProfBA);
    P->cur.st.ba_iters = 0;  // absorb_p1 takes the device's count
    if (iters_out) *iters_out = -1;
    return VG_OK;
  }
  if (rc_status) {  // complete the recut on the host (stream order), then the LM again
    P->rc_seq = 0;
    int nf = 0;
    int r = map_recut_resume(ctx, P->mpd, &nf);
    if (r == kNeedInsertReplay) {
      VG_TRY(insert_replay(ctx, P));
      const WinArg wa = make_winarg(P, 0);
      r = map_recut(ctx, P->mpd, wa, ctx->cfg.thread_num, &nf, true);
    }
    VG_TRY(r);
    P->n_factors = nf;
    P->cur.st.n_factors = nf;
    VG_TRY(ba_run(ctx, nf, P->mp.data(), &iters, prefix));
  }
  P->rc_seq = 0;
  prof_end(ctx, kProfBA);
  P->cur.st.ba_iters = iters;
  if (iters_out) *iters_out = iters;
  return VG_OK;
}

// the device part of multi_margi (x_curr.R/p <- x_buf.back(), the window
// view, the state publication, the margi kernels); gate: see ba_run
static int margi_enqueue(vg_ctx* ctx, HostPipe* P, const int* gate, int* seq1, int* seq2) {
  const vg_config& c = ctx->cfg;
  const WinArg wa = make_winarg(P, 1);
  P->tail_wa = wa;
  VG_TRY(map_factor_finish(ctx));  // an asynchronous recut no k_ba_init followed (stage API without the LM)
  *seq1 = ++ctx->pub_seq;
  *seq2 = ++ctx->pub_seq;
  if (!P->prefix) {
    VG_TRY(map_margi_prefix(ctx, P->mpd, P->mp[0], P->wp_n[P->mp[0]], c.thread_num));
    P->prefix = true;
  }
  return map_margi(ctx, P->mpd, wa, P->wp_n[P->mp[0]], c.thread_num, *seq1, *seq2, gate);
}

// x_curr.R/p <- x_buf.back(), multi_margi, jour, mp[] rotation and buffer slide
// (local_mapping.cpp:499-546)
int stage_margi_slide(vg_ctx* ctx) {
  HostTimer ht_(ctx, kHostMargi);
  HostPipe* P = hp(ctx);
  const vg_config& c = ctx->cfg;
  const int W = c.win_size;
  if (P->win_count < W) {
    ctx->err = "vg_margi: window not full";
    return VG_E_STATE;
  }
  VG_TRY(need_open(ctx, P, "vg_multi_margi"));
  VG_TRY(flush_deferred(ctx, P));
  int seq1, seq2;
  if (P->tail_queued) {  // already on the stream behind the LM (stage_ba)
    seq1 = P->tail_seq1;
    seq2 = P->tail_seq2;
  } else {
    prof_begin(ctx, kProfMargi);
    VG_TRY(margi_enqueue(ctx, P, nullptr, &seq1, &seq2));
    prof_end(ctx, kProfMargi);
  }
  P->prefix = false;
  P->tail_queued = false;
  // the margi that stands (the speculative tail or the one just enqueued) stores seq1 into the
  // IEKF hand-off flag (map_margi), which the next scan's IEKF stream polls (lio_state_estimation)
  ctx->sync_tail_armed = ctx->flag_sync && ctx->overlap_iekf && ctx->use_graphs && !ctx->prof_stages;
  ctx->sync_tail_value = (unsigned)seq1;
  P->cur.seq1 = seq1;
  P->cur.seq2 = seq2;
  P->cur.shift = 1;
  P->published = true;
  const int mgsize = 1;
  P->cur.jour_check = ((P->win_base + P->win_count) % 10 == 0) ? 1 : 0;
  for (int i = 0; i < W; i++) {
    P->mp[i] += mgsize;
    if (P->mp[i] >= W) P->mp[i] -= W;
  }
  for (int i = mgsize; i < P->win_count; i++) P->x_buf[i - mgsize] = P->x_buf[i];
  P->x_buf.pop_back();
  P->imu_pre.pop_front();
  P->cur.pushed -= mgsize;
  P->win_base += mgsize;
  P->win_count -= mgsize;
  return VG_OK;
}

// end of the scan: publish what is not yet published, no drain
int stage_finish(vg_ctx* ctx) {
  HostPipe* P = hp(ctx);
  VG_TRY(need_open(ctx, P, "vg_step_end"));
  VG_TRY(flush_deferred(ctx, P));
  if (!P->published) {
    P->cur.seq1 = ++ctx->pub_seq;
    VG_TRY(state_publish(ctx, P->win_count, nullptr, P->cur.seq1));
  }
  if (P->cur.seq2 == 0) {
    P->cur.seq2 = ++ctx->pub_seq;
    VG_TRY(state_publish_counters(ctx, P->cur.seq2));
  }
  P->pend.push_back(P->cur);
  P->in_scan = false;
  P->first = false;
  if (ctx->prof_stages) return host_sync(ctx);  // stage events are single-buffered
  return VG_OK;
}

int host_win_count(vg_ctx* ctx) { return hp(ctx)->win_count; }

// The idle branch's journey release (local_mapping.cpp:317-344) after
// host_sync: pending once jour has advanced (release_flag, :510-518); the
// device erases the far roots and compacts (lifetime.hip map_release). The
// device keeps its own jour (DState::jour, for the margi stamps): it must be
// the host's, bit for bit.
bool host_release_pending(vg_ctx* ctx) { return hp(ctx)->release_flag; }
int host_release_far(vg_ctx* ctx, int flags, long long* out) {
  HostPipe* P = hp(ctx);
  if (P->in_scan) {
    ctx->err = "vg_release_far inside a scan";
    return VG_E_STATE;
  }
  if (init_active(P)) {
    ctx->err = "vg_release_far: cold-start initialisation in progress";
    return VG_E_STATE;
  }
  double dj = 0;
  VG_HIP(hipMemcpy(&dj, &ctx->st->jour, sizeof(double), hipMemcpyDeviceToHost));
  if (memcmp(&dj, &P->jour, sizeof(double)) != 0) {
    ctx->err = "vg_release_far: device jour " + std::to_string(dj) + " != host jour " + std::to_string(P->jour);
    return VG_E_STATE;
  }
  const bool release = P->release_flag;
  const int thr = ctx->cfg.release_dis > 0 ? ctx->cfg.release_dis : 700;
  const int r = map_release(ctx, release, thr, P->jour, flags & 1, out);
  if (r == VG_OK) P->release_flag = false;  // a failed release (e.g. its scratch allocation) stays pending
  return r;
}
int host_memo_probe(vg_ctx* ctx, int* out) { return map_memo_probe(ctx, hp(ctx)->mpd, out); }

// IMUEKF::motion_blur's per-point deskew (imu_ekf.cpp:114-144), SURVEY row
// f1: after the propagation (which recorded the IMU poses), the scan is moved
// into the LiDAR frame at pcl_end_time by one lane per point, into the
// context's staging buffers. Nothing to do on the first scan (no poses).
int stage_deskew(vg_ctx* ctx, const float* x, const float* y, const float* z, const float* in, const float* t,
                 int n) {
  HostPipe* P = hp(ctx);
  VG_TRY(need_open(ctx, P, "vg_deskew"));
  const int npose = (int)P->poses.size() / 22;
  std::vector<double> par(24 + P->poses.size());
  const HX& xc = P->x_curr;
  memcpy(par.data(), xc.R.a, 72);
  memcpy(par.data() + 9, xc.p.a, 24);
  for (int i = 0; i < 9; i++) par[12 + i] = ctx->cfg.ext_R[i];
  for (int i = 0; i < 3; i++) par[21 + i] = ctx->cfg.ext_t[i];
  if (!P->poses.empty()) memcpy(par.data() + 24, P->poses.data(), P->poses.size() * sizeof(double));
  VG_TRY(state_deskew(ctx, par.data(), npose, x, y, z, in, t, n));
  ctx->tail_a_valid = false;  // the IEKF reads the deskewed scan: behind the whole main stream
  VG_HIP(hipEventRecord(ctx->ev_scan_ready, ctx->stream));  // the downsample stream reads the result
  return VG_OK;
}

// one scan with the deskew: the rest of the pipeline reads the staging buffers
int host_step_deskew(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di,
                     const float* dt, int n, double beg, double end, const double* imu, int m) {
  const vg_config& c = ctx->cfg;
  if (init_active(hp(ctx))) return init_step(ctx, dx, dy, dz, di, dt, n, beg, end, imu, m);
  VG_TRY(stage_propagate(ctx, imu, m, beg, end));
  VG_TRY(stage_deskew(ctx, dx, dy, dz, di, dt, n));
  const float *x = ctx->d_x, *y = ctx->d_y, *z = ctx->d_z, *i = ctx->d_i;
  VG_TRY(stage_iekf(ctx, x, y, z, n, nullptr));
  VG_TRY(stage_downsample(ctx, x, y, z, i, n, nullptr));
  VG_TRY(stage_window_push(ctx, imu, m));
  if (mid_graph_ok(ctx, hp(ctx))) {
    VG_TRY(stage_insert_recut(ctx));
  } else {
    VG_TRY(stage_insert(ctx));
    VG_TRY(stage_recut(ctx, nullptr));
  }
  if (hp(ctx)->win_count >= c.win_size) {
    if (c.if_BA == 1) VG_TRY(stage_ba(ctx, nullptr, true));
    VG_TRY(stage_margi_slide(ctx));
  }
  return stage_finish(ctx);
}

// slack probe (scripts/slack_probe.sh): VG_HOST_DELAY="point,us" busy-waits
// the host at one point of the step; ms/scan rises by the delay only where the
// host is on the critical path (0: before the IEKF, 1: before the LM, 2: after
// the LM wait, 3: before the insert, 4: before the downsample)
static void host_delay(int point) {
  static int p = -2, us = 0;
  if (p == -2) {
    const char* e = getenv("VG_HOST_DELAY");
    p = -1;
    if (e && sscanf(e, "%d,%d", &p, &us) != 2) p = -1;
  }
  if (p != point) return;
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < us) {
  }
}

// one scan of thd_odometry_localmapping's steady-state branch
int host_step(vg_ctx* ctx, const float* dx, const float* dy, const float* dz, const float* di, int n, double beg,
              double end, const double* imu, int m) {
  const vg_config& c = ctx->cfg;
  if (init_active(hp(ctx))) return init_step(ctx, dx, dy, dz, di, nullptr, n, beg, end, imu, m);
  // both read only the raw scan (local_mapping.cpp:396-413). The downsample
  // (its count stays on the device) goes first, on its own stream, before the
  // host waits for the previous scan's state: it runs under that scan's margi
  // and this scan's IEKF instead of behind the IEKF's enqueue. The IEKF then
  // opens the main stream's critical path.
  HostPipe* P = hp(ctx);
  host_delay(5);
  const bool early = ctx->ds_early && ctx->want_ds_stream && !P->in_scan && P->sticky == VG_OK && !ctx->prof_stages;
  if (early) {
    // ds_after_iekf: behind the device propagation's launch (lio_state_estimation
    // runs the hook), so k_scan_prop is queued before the host enqueues it
    auto enq = [=]() -> int {
      HostTimer ht_(ctx, kHostDownsample);
      return ds_enqueue_scan(ctx, dx, dy, dz, di, n, 0);
    };
    if (ctx->ds_after_iekf && prop_on_device(ctx, P, m, true)) P->ds_hook = enq;  // (no host wait before it)
    else VG_TRY(enq());
  }
  VG_TRY(stage_propagate(ctx, imu, m, beg, end, true));
  host_delay(0);
  const int r_iekf = stage_iekf(ctx, dx, dy, dz, n, nullptr);
  if (P->ds_hook) {  // not run inside (an error, or a path without the IEKF's enqueue)
    const std::function<int()> h = std::move(P->ds_hook);
    P->ds_hook = nullptr;
    if (r_iekf == VG_OK) VG_TRY(h());
  }
  VG_TRY(r_iekf);
  host_delay(4);
  if (early) {
    ds_adopt(P, dx, dy, dz, di, n);
    P->ds_seq = -1;
  } else {
    VG_TRY(stage_downsample(ctx, dx, dy, dz, di, n, nullptr));
  }
  VG_TRY(stage_window_push(ctx, imu, m));
  host_delay(3);
  if (mid_graph_ok(ctx, hp(ctx))) {
    VG_TRY(stage_insert_recut(ctx));
  } else {
    VG_TRY(stage_insert(ctx));
    VG_TRY(stage_recut(ctx, nullptr));
  }
  if (hp(ctx)->win_count >= c.win_size) {
    host_delay(1);
    if (c.if_BA == 1) VG_TRY(stage_ba(ctx, nullptr, true));
    host_delay(2);
    VG_TRY(stage_margi_slide(ctx));
  }
  return stage_finish(ctx);
}

void host_seed(vg_ctx* ctx, const double* s) {
  HX& x = hp(ctx)->x_curr;
  x.t = s[0];
  memcpy(x.R.a, s + 1, 72);
  memcpy(x.p.a, s + 10, 24);
  memcpy(x.v.a, s + 13, 24);
  memcpy(x.bg.a, s + 16, 24);
  memcpy(x.ba.a, s + 19, 24);
  memcpy(x.g.a, s + 22, 24);
  memcpy(x.cov.a, s + 25, 225 * sizeof(double));
}
static void state_out(const HX& x, double* s) {
  s[0] = x.t;
  memcpy(s + 1, x.R.a, 72);
  memcpy(s + 10, x.p.a, 24);
  memcpy(s + 13, x.v.a, 24);
  memcpy(s + 16, x.bg.a, 24);
  memcpy(s + 19, x.ba.a, 24);
  memcpy(s + 22, x.g.a, 24);
  memcpy(s + 25, x.cov.a, 225 * sizeof(double));
}
// lio_state_estimation_kdtree (odometry.cpp:267-439) on an
// explicit state (250 doubles in/out): the per-point kNN, plane fit and
// normal-equation sums on the device (kdlio.hip), the 15x15 update here. The
// scan is the init-phase cloud downsampled at max(down_size, 0.5), raw LiDAR
// frame (xyz AoS). *valid = -1 when the map held < 100 points and the scan
// only seeded it.
int host_lio_kdtree(vg_ctx* ctx, const float* xyz, int n, double* state, int* valid, int* iters) {
  VG_TRY(host_sync(ctx));  // the scan staging and downsample buffers are shared with the pipeline
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "vg_lio_kdtree: scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  *valid = -1;
  *iters = 0;
  HX x_curr;
  x_curr.t = state[0];
  memcpy(x_curr.R.a, state + 1, 72);
  memcpy(x_curr.p.a, state + 10, 24);
  memcpy(x_curr.v.a, state + 13, 24);
  memcpy(x_curr.bg.a, state + 16, 24);
  memcpy(x_curr.ba.a, state + 19, 24);
  memcpy(x_curr.g.a, state + 22, 24);
  memcpy(x_curr.cov.a, state + 25, 225 * sizeof(double));
  {
    std::vector<float> soa((size_t)3 * n);
    for (int i = 0; i < n; i++) {
      soa[i] = xyz[3 * i];
      soa[(size_t)n + i] = xyz[3 * i + 1];
      soa[(size_t)2 * n + i] = xyz[3 * i + 2];
    }
    VG_HIP(hipMemcpy(ctx->d_x, soa.data(), (size_t)n * sizeof(float), hipMemcpyHostToDevice));
    VG_HIP(hipMemcpy(ctx->d_y, soa.data() + n, (size_t)n * sizeof(float), hipMemcpyHostToDevice));
    VG_HIP(hipMemcpy(ctx->d_z, soa.data() + 2 * (size_t)n, (size_t)n * sizeof(float), hipMemcpyHostToDevice));
  }
  if (n == 0) return VG_OK;
  VG_TRY(kd_lio(ctx, n, x_curr, valid, iters));
  state_out(x_curr, state);
  return VG_OK;
}

// the kd-tree IEKF on the scan in ctx->d_x/y/z (n points, raw LiDAR frame);
// x_curr in/out; the map is extended with the scan at the result
int kd_lio(vg_ctx* ctx, int n, HX& x_curr, int* valid, int* iters) {
  *valid = -1;
  *iters = 0;
  if (ctx->kd.n < 100) {  // 275-310: seed the map with the scan at the current pose
    VG_TRY(kd_update(ctx, n, x_curr.R.a, x_curr.p.a, false));
    return VG_OK;
  }
  const int num_max_iter = 4;
  const HX x_prop = x_curr;
  bool flg_conv = false;
  int rematch_num = 0;
  M15 G = M15::Z(), cov_inv = inverse(x_curr.cov);
  bool refind = true;
  for (int it = 0; it < num_max_iter; it++) {
    (*iters)++;
    double sums[28];
    VG_TRY(kd_pass(ctx, n, x_curr.R.a, x_curr.p.a, refind ? 1 : 0, sums));
    M15 HTH15 = M15::Z();
    double HTz[6];
    int k = 0;
    for (int r = 0; r < 6; r++)
      for (int c = r; c < 6; c++, k++) HTH15(r, c) = HTH15(c, r) = sums[k];
    for (int r = 0; r < 6; r++) HTz[r] = sums[21 + r];
    *valid = (int)sums[27];
    M15 Kin;  // H_T_H + cov_inv / 1000 (odometry.cpp:393)
    for (int r = 0; r < 15; r++)
      for (int c = 0; c < 15; c++) Kin(r, c) = HTH15(r, c) + cov_inv(r, c) / 1000;
    const M15 K_1 = inverse(Kin);
    for (int r = 0; r < 15; r++)  // G(:, 0:6) = K_1(:, 0:6) HTH
      for (int c = 0; c < 6; c++) {
        double g = 0.0;
        for (int q = 0; q < 6; q++) g += K_1(r, q) * HTH15(q, c);
        G(r, c) = g;
      }
    const V15 vec = x_prop.minus(x_curr);
    V15 sol;
    for (int r = 0; r < 15; r++) {  // K_1(:,0:6) HTz + vec - G(:,0:6) vec(0:6)
      double a = 0.0, b = 0.0;
      for (int q = 0; q < 6; q++) a += K_1(r, q) * HTz[q];
      for (int q = 0; q < 6; q++) b += G(r, q) * vec[q];
      sol[r] = (a + vec[r]) - b;
    }
    x_curr.plus(sol);
    const double rn = sqrt((sol[0] * sol[0] + sol[1] * sol[1]) + sol[2] * sol[2]);
    const double tn = sqrt((sol[3] * sol[3] + sol[4] * sol[4]) + sol[5] * sol[5]);
    refind = false;
    if ((rn * 57.3 < 0.01) && (tn * 100 < 0.015)) {
      refind = true;
      flg_conv = true;
      rematch_num++;
    }
    if (it == num_max_iter - 2 && !flg_conv) refind = true;
    if (rematch_num >= 2 || it == num_max_iter - 1) {  // cov = (I - G) cov
      M15 nc;
      for (int r = 0; r < 15; r++)
        for (int c = 0; c < 15; c++) {
          double a = 0.0;
          for (int q = 0; q < 15; q++) a += ((r == q ? 1.0 : 0.0) - G(r, q)) * x_curr.cov(q, c);
          nc(r, c) = a;
        }
      x_curr.cov = nc;
      break;
    }
  }
  VG_TRY(kd_update(ctx, n, x_curr.R.a, x_curr.p.a, true));  // 427-437
  return VG_OK;
}

// x_curr now: between scans the absorbed host mirror; inside a scan (e.g.
// save_pose_tum right after VNC_lio, local_mapping.cpp:429) the device state
int host_state(vg_ctx* ctx, double* s) {
  HostPipe* P = hp(ctx);
  if (!P->in_scan) {
    VG_TRY(host_sync(ctx));
    state_out(P->x_curr, s);
    return VG_OK;
  }
  VG_TRY(flush_deferred(ctx, P));
  double* h = ctx->h_stage;
  VG_HIP(hipMemcpyAsync(h, ctx->st->xc, kXC * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  VG_HIP(stream_wait(ctx));
  s[0] = P->cur.t;
  memcpy(s + 1, h, kXS * sizeof(double));  // R, p, v, bg, ba, g
  memcpy(s + 25, h + kXS, 225 * sizeof(double));
  return VG_OK;
}
int host_window(vg_ctx* ctx, double* out) {
  HostPipe* P = hp(ctx);
  for (size_t i = 0; i < P->x_buf.size(); i++) state_out(P->x_buf[i], out + 250 * i);
  return (int)P->x_buf.size();
}
int host_traj(vg_ctx* ctx, double* out, int cap, int from) {
  HostPipe* P = hp(ctx);
  int n = (int)P->traj.size() / kTrajRow;
  const int k = from < n ? (n - from < cap ? n - from : cap) : 0;
  if (out && k > 0) memcpy(out, P->traj.data() + (size_t)from * kTrajRow, (size_t)k * kTrajRow * sizeof(double));
  return n;
}
int host_path(vg_ctx* ctx, double* out, int cap) {
  HostPipe* P = hp(ctx);
  int n = (int)P->path.size() / kPathRow;
  if (out) memcpy(out, P->path.data(), (size_t)(n < cap ? n : cap) * kPathRow * sizeof(double));
  return n;
}
int host_poll(vg_ctx* ctx) {
  HostPipe* P = hp(ctx);
  if (P->in_scan) return VG_OK;  // a stage-level scan is open: nothing to absorb mid-scan
  return absorb_ready(ctx, P);
}
int host_stats_log(vg_ctx* ctx, vg_stats* out, int cap) {
  HostPipe* P = hp(ctx);
  int n = (int)P->stats_log.size();
  if (out)
    for (int i = 0; i < n && i < cap; i++) out[i] = P->stats_log[i];
  return n;
}

}  // namespace vg
