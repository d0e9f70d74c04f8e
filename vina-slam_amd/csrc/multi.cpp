// multi.cpp — multi-sequence mode: B independent sequences on one GPU
// (BASELINE config 5, SURVEY §7 "Hard parts"). Up to four sequences: each
// context on its own stream, driven by its own native worker thread; past
// four, the sequences share four streams, one worker per stream stepping its
// sequences one scan each in turn (a graph capture then never meets another
// thread's work on its stream). vg_multi_step_dev queues one scan per sequence
// and returns; the workers run free (no lock-step between streams), so the
// streams overlap on the device. Each worker runs exactly the single-sequence
// path (host_step), so every sequence's results are those of a lone context,
// bit for bit.
//
// Why threads and not one launch for B sequences: the per-scan path is ~90
// small dependent kernels whose cost is dispatch + cross-XCD memory latency,
// not arithmetic; on MI355X independent per-stream launches overlap
// (scripts/micro/concurrency.hip: 1.6M kernels/s over 16 streams vs 0.3M for
// one graph holding the same parallel chains), so per-sequence streams are the
// shape that fills the chip. The workers sleep-poll their waits
// (vg_set_wait_policy) because the box's CPU quota is shared by all of them.
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>
#include "vg_host.h"

namespace {
constexpr int kMultiStreams = 4;  // default shared streams past this many sequences
struct Job {
  vg_scan_dev sc;
  std::vector<double> imu;  // the scan's IMU samples (the caller's buffer may be reused)
};
struct Worker {
  std::deque<Job> q;
  int rc = VG_OK;
};
}  // namespace

struct vg_multi {
  std::vector<vg_ctx*> ctx;
  std::vector<Worker> wk;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv_job, cv_room;
  bool quit = false;
  int depth = 4;  // scans queued per sequence before vg_multi_step_dev blocks
  int busy = 0;   // workers inside a step
  std::vector<char> split;  // context b ran with its own downsample stream + IEKF overlap (restored on destroy)
  // At most `cap` sequences on the device at once (0: no cap). Measured
  // (profiles/r04/multi_pmc_r04g.json): at B = 8 every kernel's L2 hit rate and
  // request count equal B = 4's, yet every kernel takes >= ~47 us — the
  // hardware queues are oversubscribed and time-sliced, not the caches; idle
  // queues count too (a cap of 4 busy sequences over 8 queues changes
  // nothing). So with GPU_MAX_HW_QUEUES = cap the B streams share cap
  // queues, and sequence b runs only while no other sequence of its slot
  // b % cap does: a worker takes its slot, runs its scan, waits for that
  // scan's device work and gives the slot back.
  int cap = 0, active = 0;
  std::vector<char> slot_busy;  // sequence b runs in slot b % cap (its stream shares a hardware queue with
                                // the other sequences of that slot when GPU_MAX_HW_QUEUES = cap)
  std::condition_variable cv_slot;
  // Shared streams (VG_MULTI_STREAMS = G < B): sequence b runs on stream
  // b % G, driven by worker b % G, which steps its sequences one scan each in
  // turn. G busy hardware queues instead of B time-sliced ones; one thread per
  // stream, so a graph capture never sees another thread's work on it.
  int groups = 0;                 // 0: one stream + one worker per sequence
  std::vector<hipStream_t> own;   // each context's own stream (restored on destroy)
};

// one queued scan of sequence b (busy already counted)
static void run_job(vg_multi* M, int b, Job& j) {
  vg_ctx* c = M->ctx[b];
  const vg_scan_dev& sc = j.sc;
  const double* imu = j.imu.empty() ? nullptr : j.imu.data();
  const bool capped = M->cap > 0;
  const int slot = capped ? b % M->cap : 0;
  if (capped) {
    std::unique_lock<std::mutex> lk(M->mu);
    M->cv_slot.wait(lk, [&] { return !M->slot_busy[slot]; });
    M->slot_busy[slot] = 1;
    M->active++;
  }
  int r;
  if (sc.d_time)
    r = vg_step_deskew_dev(c, sc.d_x, sc.d_y, sc.d_z, sc.d_intensity, sc.d_time, sc.n, sc.pcl_beg_time,
                           sc.pcl_end_time, imu, sc.m);
  else
    r = vg_step_dev(c, sc.d_x, sc.d_y, sc.d_z, sc.d_intensity, sc.n, sc.pcl_beg_time, sc.pcl_end_time, imu, sc.m);
  if (capped) {  // the scan's device work done before the slot goes to another sequence
    const int r2 = vg::host_sync(c);
    if (r == VG_OK) r = r2;
    {
      std::lock_guard<std::mutex> lk(M->mu);
      M->slot_busy[slot] = 0;
      M->active--;
    }
    M->cv_slot.notify_all();
  }
  {
    std::lock_guard<std::mutex> lk(M->mu);
    if (r != VG_OK && M->wk[b].rc == VG_OK) M->wk[b].rc = r;
    M->busy--;
  }
  M->cv_room.notify_all();
}

// worker g: sequences g, g + G, ... (G = groups, or one sequence when 0), one
// scan each in turn; returns on quit once its queues are empty
static void worker(vg_multi* M, int g) {
  const int B = (int)M->ctx.size(), G = M->groups > 0 ? M->groups : B;
  for (;;) {
    bool any = false;
    for (int b = g; b < B; b += G) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(M->mu);
        M->cv_job.wait(lk, [&] { return M->quit || !M->wk[b].q.empty(); });
        if (M->wk[b].q.empty()) continue;  // quit with nothing left for this sequence
        j = std::move(M->wk[b].q.front());
        M->wk[b].q.pop_front();
        M->busy++;
      }
      any = true;
      M->cv_room.notify_all();
      run_job(M, b, j);
    }
    if (!any) return;
  }
}

extern "C" {

vg_multi* vg_multi_create(vg_ctx** ctxs, int B, int spin_us, int sleep_us) {
  if (!ctxs || B <= 0) return nullptr;
  vg_multi* M = new vg_multi();
  M->ctx.assign(ctxs, ctxs + B);
  M->wk.resize(B);
  M->split.assign(B, 0);
  for (int b = 0; b < B; b++) {
    vg_set_wait_policy(ctxs[b], spin_us, sleep_us);
    if (B > 1) {
      // one stream per sequence: the concurrency comes from the B sequences,
      // and every stream beyond the hardware queues makes sequences share a
      // queue (measured: B = 4 at 1,465-2,704 scans/s with two streams each,
      // depending on how the queues fell); the downsample and the margi prefix
      // then run in enqueue order on the context stream
      vg_ctx* c = ctxs[b];
      M->split[b] = (char)((c->overlap_iekf ? 1 : 0) | (c->want_ds_stream ? 2 : 0));
      c->overlap_iekf = false;
      c->want_ds_stream = false;
      if (c->stream_ds && c->stream_ds != c->stream) {
        (void)hipStreamSynchronize(c->stream_ds);
        (void)hipStreamDestroy(c->stream_ds);
        c->stream_ds = c->stream;
      }
    }
  }
  // shared streams past four sequences (vina_gpu.h; measured in
  // profiles/r06/multi_streams_r06.txt: B = 8 3,837 scans/s on four shared
  // streams against 2,970 on eight, B = 4 3,824)
  const char* gs = getenv("VG_MULTI_STREAMS");
  const int G = gs ? atoi(gs) : (B > kMultiStreams ? kMultiStreams : 0);
  if (B > 1 && G > 0 && G < B) {  // sequence b on sequence (b % G)'s stream
    M->groups = G;
    M->own.resize(B);
    for (int b = 0; b < B; b++) {
      vg_ctx* c = ctxs[b];
      (void)hipStreamSynchronize(c->stream);  // (its seed / setup work)
      M->own[b] = c->stream;
    }
    for (int b = G; b < B; b++) {
      vg_ctx* c = ctxs[b];
      c->stream = M->own[b % G];
      c->stream_ds = c->stream;
    }
  }
  const int nw = M->groups > 0 ? M->groups : B;
  for (int g = 0; g < nw; g++) M->th.emplace_back(worker, M, g);
  return M;
}

// All-or-nothing: every queue has room and no worker has failed before any
// scan is queued, so the sequences never go out of step on an error.
int vg_multi_step_dev(vg_multi* M, const vg_scan_dev* scans) {
  if (!M || !scans) return VG_E_ARG;
  std::unique_lock<std::mutex> lk(M->mu);
  M->cv_room.wait(lk, [&] {
    for (const Worker& w : M->wk)
      if (w.rc != VG_OK || (int)w.q.size() >= M->depth) return w.rc != VG_OK;
    return true;
  });
  for (const Worker& w : M->wk)
    if (w.rc != VG_OK) return w.rc;
  for (size_t b = 0; b < M->ctx.size(); b++) {
    Job j;
    j.sc = scans[b];
    if (scans[b].imu && scans[b].m > 0) j.imu.assign(scans[b].imu, scans[b].imu + 7 * (size_t)scans[b].m);
    j.sc.imu = nullptr;
    M->wk[b].q.push_back(std::move(j));
  }
  lk.unlock();
  M->cv_job.notify_all();
  return VG_OK;
}

int vg_multi_set_active(vg_multi* M, int cap) {
  if (!M || cap < 0) return VG_E_ARG;
  std::lock_guard<std::mutex> lk(M->mu);
  if (M->busy || M->active) return VG_E_STATE;  // between steps only
  for (const Worker& w : M->wk)
    if (!w.q.empty()) return VG_E_STATE;
  M->cap = cap >= (int)M->ctx.size() ? 0 : cap;
  M->slot_busy.assign(M->cap > 0 ? M->cap : 0, 0);
  return VG_OK;
}

int vg_multi_sync(vg_multi* M) {
  if (!M) return VG_E_ARG;
  {
    std::unique_lock<std::mutex> lk(M->mu);
    M->cv_room.wait(lk, [&] {
      if (M->busy) return false;
      for (const Worker& w : M->wk)
        if (!w.q.empty()) return false;
      return true;
    });
    for (const Worker& w : M->wk)
      if (w.rc != VG_OK) return w.rc;
  }
  int rc = VG_OK;
  for (vg_ctx* c : M->ctx) {
    vg_stats st;
    const int r = vg_get_stats(c, &st);  // completes every enqueued scan of the context
    if (r != VG_OK && rc == VG_OK) rc = r;
  }
  return rc;
}

void vg_multi_destroy(vg_multi* M) {
  if (!M) return;
  {
    std::lock_guard<std::mutex> lk(M->mu);
    M->quit = true;
  }
  M->cv_job.notify_all();
  for (auto& t : M->th) t.join();
  // hand each context back as it came: its own downsample stream and the
  // IEKF / margi overlap of the single-sequence path
  for (size_t b = 0; b < M->ctx.size(); b++) {
    vg_ctx* c = M->ctx[b];
    (void)hipStreamSynchronize(c->stream);
    if (!M->own.empty()) {  // back on its own stream
      c->stream = M->own[b];
      c->stream_ds = c->stream;
    }
    if (M->split[b] & 2) c->want_ds_stream = true;  // made again on the next scan (stage_downsample)
    if (M->split[b] & 1) c->overlap_iekf = true;
  }
  delete M;
}

}  // extern "C"
