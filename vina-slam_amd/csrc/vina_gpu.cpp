// vina_gpu.cpp — C-ABI entry points (include/vina_gpu.h) and context lifecycle.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <csignal>
#include <cstdio>
#include <execinfo.h>
#include <unistd.h>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <new>
#include <vector>
#include "vg_internal.h"

using namespace vg;

// The pinned copy of a host-input scan split over the calling thread and a few
// helper threads (VG_COPY_THREADS, default 4 in all): one core copies ~10 GB/s,
// and this copy sits before the scan's first kernel. Helpers sleep on a
// condition variable between scans (no spinning core in a ROS process).
namespace {
struct CopyPool {
  struct Job {
    char* dst;
    const char* src;
    size_t bytes;
  };
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Job> jobs;            // rewritten only once every job of the previous run is done
  std::atomic<uint64_t> claim{0};   // (run << 32) | next job: a claim of a finished run cannot succeed
  std::atomic<int> left{0};         // jobs of the current run not yet copied
  uint32_t runs = 0;
  int njobs = 0;
  bool stop = false;
  static constexpr size_t kChunk = 128 << 10;
  explicit CopyPool(int nhelp) {
    for (int i = 0; i < nhelp; i++) th.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void work(uint32_t run, int n) {
    uint64_t v = claim.load(std::memory_order_acquire);
    for (;;) {
      if ((uint32_t)(v >> 32) != run || (int)(uint32_t)v >= n) return;
      if (!claim.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) continue;
      const Job& jb = jobs[(uint32_t)v];
      memcpy(jb.dst, jb.src, jb.bytes);
      left.fetch_sub(1, std::memory_order_release);
      v = claim.load(std::memory_order_acquire);
    }
  }
  void loop() {
    uint32_t seen = 0;
    for (;;) {
      uint32_t run;
      int n;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || runs != seen; });
        if (stop) return;
        seen = run = runs;
        n = njobs;
      }
      work(run, n);
    }
  }
  // copies every (dst, src, bytes) piece; returns when all are done
  void run(const std::vector<Job>& pieces) {
    uint32_t r;
    int n;
    {
      std::lock_guard<std::mutex> g(mu);
      jobs.clear();
      for (const Job& p : pieces)
        for (size_t o = 0; o < p.bytes; o += kChunk)
          jobs.push_back({p.dst + o, p.src + o, std::min(kChunk, p.bytes - o)});
      r = ++runs;
      n = njobs = (int)jobs.size();
      left.store(n, std::memory_order_relaxed);
      claim.store((uint64_t)r << 32, std::memory_order_release);
    }
    if (!th.empty() && n > 1) cv.notify_all();
    work(r, n);
    while (left.load(std::memory_order_acquire) > 0) std::this_thread::yield();
  }
};
}  // namespace

static void pinned_copy(vg_ctx* ctx, const std::vector<CopyPool::Job>& pieces) {
  if (!ctx->copy_pool) {
    const char* e = getenv("VG_COPY_THREADS");
    const int n = std::max(1, std::min(16, e ? atoi(e) : 4));
    ctx->copy_pool = new CopyPool(n - 1);
  }
  static_cast<CopyPool*>(ctx->copy_pool)->run(pieces);
}


static std::atomic<int> g_dev_ctx[64];
namespace vg {
int dev_ctx_count(int device) { return (device >= 0 && device < 64) ? g_dev_ctx[device].load() : 1; }
std::recursive_mutex& capture_mutex() {
  static std::recursive_mutex mu;
  return mu;
}
}  // namespace vg

// VG_SEGV_TRACE=1: a fatal signal prints the native stack (the frames of this
// library and of the HIP runtime) to stderr before the default action, so a
// crash inside a worker thread of the multi-sequence mode names its call site.
static void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "vina_gpu: fatal signal, native stack:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
static void segv_trace_install() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = getenv("VG_SEGV_TRACE");
    if (!e || atoi(e) == 0) return;
    signal(SIGSEGV, segv_trace);
    signal(SIGBUS, segv_trace);
    signal(SIGABRT, segv_trace);
  });
}

static void fill_capacity(vg_capacity& c) {
  if (c.max_points_per_scan <= 0) c.max_points_per_scan = 2000000;
  if (c.max_nodes <= 0) c.max_nodes = 4000000;
  if (c.max_fix_points <= 0) c.max_fix_points = 16000000;
  if (c.hash_log2 <= 0) c.hash_log2 = 23;
}

extern "C" {

int vg_create(const vg_config* cfg, const vg_capacity* cap, int device, vg_ctx** out) {
  if (!cfg || !out) return VG_E_ARG;
  *out = nullptr;
  segv_trace_install();
  vg_ctx* ctx = new (std::nothrow) vg_ctx();
  if (!ctx) return VG_E_CAPACITY;
  ctx->cfg = *cfg;
  memset(&ctx->cap, 0, sizeof(ctx->cap));
  if (cap) ctx->cap = *cap;
  fill_capacity(ctx->cap);
  ctx->device = device;
  memset(&ctx->stats, 0, sizeof(ctx->stats));
  // Kernels serialised (AMD_SERIALIZE_KERNEL, or a counter-collection run:
  // rocprofv3 --pmc dispatches one kernel at a time; VG_SERIAL_KERNELS=1 says
  // so): a polling hand-off kernel would wait for a producer queued behind it,
  // so the context uses event waits and waits for each LM's outcome in its step
  {
    const char* a = getenv("AMD_SERIALIZE_KERNEL");
    const char* v = getenv("VG_SERIAL_KERNELS");
    const char* p = getenv("ROCPROF_COUNTER_COLLECTION");  // rocprofv3 --pmc sets it for its target
    if ((a && atoi(a) != 0) || (v && atoi(v) != 0) || (p && atoi(p) != 0)) {
      ctx->serial_kernels = true;
      ctx->flag_sync = false;
    }
  }
  auto fail = [&](int code) {
    fprintf(stderr, "vg_create: %s\n", ctx->err.c_str());
    vg_destroy(ctx);
    return code;
  };
  if (cfg->win_size <= 0 || cfg->win_size > 32 || cfg->max_layer < 0 || cfg->max_layer > 3 ||
      cfg->voxel_size <= 0) {
    ctx->err = "invalid config (win_size in [1,32], max_layer in [0,3], voxel_size > 0)";
    return fail(VG_E_ARG);
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    ctx->err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  if ((e = hipEventCreateWithFlags(&ctx->ev_ds_done, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&ctx->ev_ds_free, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&ctx->ev_recut_done, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&ctx->ev_prefix_done, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&ctx->ev_scan_ready, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&ctx->ev_tail_a, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&ctx->ev_iekf_done, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess) {
    ctx->err = std::string("hipStreamCreate: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) {
    ctx->err = std::string("hipStreamCreate: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  ctx->stream_ds = ctx->stream;  // its own stream on the first scan (stage_downsample), unless multi-sequence
  if ((e = hipHostMalloc((void**)&ctx->h_pinned, 4096, hipHostMallocDefault)) != hipSuccess) {
    ctx->err = std::string("hipHostMalloc: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  // size the slab exactly (measure pass), then carve it for real
  auto carve = [&]() -> int {
    const size_t n = (size_t)ctx->cap.max_points_per_scan;
    ctx->d_x = ctx->arena.take<float>(n);
    ctx->d_y = ctx->arena.take<float>(n);
    ctx->d_z = ctx->arena.take<float>(n);
    ctx->d_i = ctx->arena.take<float>(n);
    ctx->d_t = ctx->arena.take<float>(n);
    int r = state_alloc(ctx);
    if (r == VG_OK) r = shard_alloc(ctx);
    if (r == VG_OK) r = ds_alloc(ctx);
    if (r == VG_OK) r = map_alloc(ctx);
    if (r == VG_OK) r = ba_alloc(ctx);
    if (r == VG_OK) r = kd_alloc(ctx);
    return r;
  };
  ctx->arena.measure = true;
  int r = carve();
  if (r != VG_OK) return fail(r);
  size_t need = ctx->arena.used + (1 << 20);
  ctx->arena = vg::Arena();
  if ((e = hipMalloc((void**)&ctx->arena.base, need)) != hipSuccess) {
    ctx->err = std::string("hipMalloc arena (") + std::to_string(need >> 20) + " MiB): " + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  ctx->arena.size = need;
  if ((e = hipMemsetAsync(ctx->arena.base, 0, need, ctx->stream)) != hipSuccess) {
    ctx->err = std::string("hipMemset arena: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  r = carve();
  if (r == VG_OK) r = map_reset(ctx);
  if (r != VG_OK) return fail(r);
  if ((e = hipHostMalloc((void**)&ctx->h_stage, kStageBytes, hipHostMallocDefault)) != hipSuccess) {
    ctx->err = std::string("hipHostMalloc: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  for (int i = 0; i < 10; i++)
    for (int j = 0; j < 2; j++)
      if ((e = hipEventCreate(&ctx->solve_ev[i][j])) != hipSuccess) {
        ctx->err = std::string("hipEventCreate: ") + hipGetErrorString(e);
        return fail(VG_E_HIP);
      }
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 2; j++)
      if ((e = hipEventCreate(&ctx->iekf_ev[i][j])) != hipSuccess) {
        ctx->err = std::string("hipEventCreate: ") + hipGetErrorString(e);
        return fail(VG_E_HIP);
      }
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 2; j++)
      if ((e = hipEventCreate(&ctx->prof_ev[i][j])) != hipSuccess) {
        ctx->err = std::string("hipEventCreate: ") + hipGetErrorString(e);
        return fail(VG_E_HIP);
      }
  if ((e = hipHostMalloc((void**)&ctx->h_pub, sizeof(Pub), hipHostMallocMapped | hipHostMallocCoherent)) !=
          hipSuccess ||
      (e = hipHostGetDevicePointer((void**)&ctx->d_pub, ctx->h_pub, 0)) != hipSuccess) {
    ctx->err = std::string("hipHostMalloc (mapped): ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  memset(ctx->h_pub, 0, sizeof(Pub));
  if ((e = hipHostMalloc((void**)&ctx->h_in, kMaxWin * sizeof(HostIn), hipHostMallocMapped | hipHostMallocCoherent)) !=
          hipSuccess ||
      (e = hipHostGetDevicePointer((void**)&ctx->d_in, ctx->h_in, 0)) != hipSuccess) {
    ctx->err = std::string("hipHostMalloc (mapped inputs): ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  memset(ctx->h_in, 0, kMaxWin * sizeof(HostIn));
  if ((e = hipEventCreateWithFlags(&ctx->sync_ev, hipEventDisableTiming)) != hipSuccess) {
    ctx->err = std::string("hipEventCreate: ") + hipGetErrorString(e);
    return fail(VG_E_HIP);
  }
  host_init(ctx);
  if (device >= 0 && device < 64) {
    ctx->counted = true;
    if (g_dev_ctx[device].fetch_add(1) > 0) ctx->flag_sync = false;  // (stage_propagate: the others follow)
  }
  *out = ctx;
  return VG_OK;
}

int vg_destroy(vg_ctx* ctx) {
  if (!ctx) return VG_OK;
  // a pending LM (vg_step returned before its outcome) needs nothing more:
  // its speculative tail either ran or ran as no-ops, and nothing waits on it
  ctx->ba_loop.active = false;
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream_ds && ctx->stream_ds != ctx->stream) (void)hipStreamSynchronize(ctx->stream_ds);
  if (ctx->stream_iekf) (void)hipStreamSynchronize(ctx->stream_iekf);
  if (ctx->counted) g_dev_ctx[ctx->device].fetch_sub(1);
  if (ctx->arena.base) (void)hipFree(ctx->arena.base);
  if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
  if (ctx->dbg_cap_buf) (void)hipFree(ctx->dbg_cap_buf);
  shard_free(ctx);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_pub) (void)hipHostFree(ctx->h_pub);
  if (ctx->host) host_free(ctx);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 2; j++)
      if (ctx->prof_ev[i][j]) (void)hipEventDestroy(ctx->prof_ev[i][j]);
  if (ctx->sync_ev) (void)hipEventDestroy(ctx->sync_ev);
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 2; j++)
      if (ctx->iekf_ev[i][j]) (void)hipEventDestroy(ctx->iekf_ev[i][j]);
  for (int i = 0; i < 10; i++)
    for (int j = 0; j < 2; j++)
      if (ctx->solve_ev[i][j]) (void)hipEventDestroy(ctx->solve_ev[i][j]);
  for (auto& g : ctx->g_iekf)
    if (g) (void)hipGraphExecDestroy(g);
  for (auto& g : ctx->g_margi)
    if (g) (void)hipGraphExecDestroy(g);
  if (ctx->g_ba) (void)hipGraphExecDestroy(ctx->g_ba);
  if (ctx->g_ba2) (void)hipGraphExecDestroy(ctx->g_ba2);
  if (ctx->g_ds) (void)hipGraphExecDestroy(ctx->g_ds);
  for (auto& g : ctx->g_mid)
    if (g) (void)hipGraphExecDestroy(g);
  for (auto& g : ctx->g_scan)
    if (g) (void)hipGraphExecDestroy(g);
  if (ctx->h_in) (void)hipHostFree(ctx->h_in);
  if (ctx->stream_ds && ctx->stream_ds != ctx->stream) (void)hipStreamSynchronize(ctx->stream_ds);
  delete static_cast<CopyPool*>(ctx->copy_pool);
  for (auto& sl : ctx->in_slot) {
    if (sl.h) (void)hipHostFree(sl.h);
    if (sl.d) (void)hipFree(sl.d);
    if (sl.up) (void)hipEventDestroy(sl.up);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->stream_ds && ctx->stream_ds != ctx->stream) (void)hipStreamSynchronize(ctx->stream_ds);
  if (ctx->stream_ds && ctx->stream_ds != ctx->stream) (void)hipStreamDestroy(ctx->stream_ds);
  if (ctx->ev_ds_done) (void)hipEventDestroy(ctx->ev_ds_done);
  if (ctx->ev_ds_free) (void)hipEventDestroy(ctx->ev_ds_free);
  if (ctx->ev_recut_done) (void)hipEventDestroy(ctx->ev_recut_done);
  if (ctx->ev_prefix_done) (void)hipEventDestroy(ctx->ev_prefix_done);
  if (ctx->ev_scan_ready) (void)hipEventDestroy(ctx->ev_scan_ready);
  if (ctx->stream_iekf) (void)hipStreamSynchronize(ctx->stream_iekf);
  if (ctx->stream_iekf) (void)hipStreamDestroy(ctx->stream_iekf);
  if (ctx->ev_tail_a) (void)hipEventDestroy(ctx->ev_tail_a);
  if (ctx->ev_iekf_done) (void)hipEventDestroy(ctx->ev_iekf_done);
  delete ctx;
  return VG_OK;
}

const char* vg_last_error(const vg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* vg_stream(vg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int vg_reset(vg_ctx* ctx) {
  if (!ctx) return VG_E_ARG;
  VG_HIP(hipStreamSynchronize(ctx->stream_ds));
  VG_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->stream_iekf) VG_HIP(hipStreamSynchronize(ctx->stream_iekf));
  ctx->ba_loop.active = false;  // the HostPipe's record of it goes with host_reset
  VG_TRY(map_reset(ctx));
  // the device's jour with the host's (host_reset: 0)
  VG_HIP(hipMemset(&ctx->st->jour_check, 0, offsetof(DState, imurec) - offsetof(DState, jour_check)));
  VG_TRY(kd_reset(ctx));
  host_reset(ctx);
  return VG_OK;
}

static int upload_aos(vg_ctx* ctx, const float* xyz, const float* inten, int n) {
  std::vector<float> soa((size_t)n * 4);
  for (int i = 0; i < n; i++) {
    soa[i] = xyz[3 * i];
    soa[(size_t)n + i] = xyz[3 * i + 1];
    soa[2 * (size_t)n + i] = xyz[3 * i + 2];
    soa[3 * (size_t)n + i] = inten ? inten[i] : 0.0f;
  }
  hipStream_t s = ctx->stream;
  VG_HIP(hipMemcpyAsync(ctx->d_x, soa.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(ctx->d_y, soa.data() + n, n * sizeof(float), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(ctx->d_z, soa.data() + 2 * (size_t)n, n * sizeof(float), hipMemcpyHostToDevice, s));
  VG_HIP(hipMemcpyAsync(ctx->d_i, soa.data() + 3 * (size_t)n, n * sizeof(float), hipMemcpyHostToDevice, s));
  VG_HIP(hipStreamSynchronize(s));
  return VG_OK;
}

int vg_downsample(vg_ctx* ctx, const float* xyz, const float* intensity, int n, double voxel_size,
                  float* out_xyzic, int* n_out) {
  if (!ctx || (!xyz && n > 0) || !out_xyzic || !n_out || n < 0) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  *n_out = 0;
  if (voxel_size < 0.001) {  // point_utils.hpp:9-10: no-op
    for (int i = 0; i < n; i++) {
      out_xyzic[5 * i] = xyz[3 * i];
      out_xyzic[5 * i + 1] = xyz[3 * i + 1];
      out_xyzic[5 * i + 2] = xyz[3 * i + 2];
      out_xyzic[5 * i + 3] = intensity ? intensity[i] : 0.0f;
      out_xyzic[5 * i + 4] = 0.0f;
    }
    *n_out = n;
    return VG_OK;
  }
  if (n == 0) return VG_OK;
  VG_HIP(hipStreamSynchronize(ctx->stream_ds));  // the pipeline's downsample shares the buffers
  VG_TRY(upload_aos(ctx, xyz, intensity, n));
  int m = 0;
  VG_TRY(ds_run(ctx, ctx->d_x, ctx->d_y, ctx->d_z, ctx->d_i, n, voxel_size, &m));
  std::vector<float> buf((size_t)m * 5);
  hipStream_t s = ctx->stream;
  const DownsampleBufs& d = ctx->ds;
  float* cols[5] = {d.ox, d.oy, d.oz, d.oi, d.oc};
  for (int c = 0; c < 5; c++)
    VG_HIP(hipMemcpyAsync(buf.data() + (size_t)c * m, cols[c], m * sizeof(float), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  for (int v = 0; v < m; v++)
    for (int c = 0; c < 5; c++) out_xyzic[5 * v + c] = buf[(size_t)c * m + v];
  *n_out = m;
  return VG_OK;
}

int vg_downsample_close(vg_ctx* ctx, const float* xyz, const float* time, int n, double voxel_size, float* out_xyzt,
                        int* n_out) {
  if (!ctx || (!xyz && n > 0) || !out_xyzt || !n_out || n < 0) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  *n_out = 0;
  if (n == 0) return VG_OK;
  if (voxel_size < 0.001) {  // point_utils.hpp:48: no-op (the time sort still applies in the caller's use)
    ctx->err = "vg_downsample_close: voxel_size < 0.001 is a no-op in the reference";
    return VG_E_ARG;
  }
  VG_TRY(host_sync(ctx));
  VG_HIP(hipStreamSynchronize(ctx->stream_ds));
  VG_TRY(upload_aos(ctx, xyz, nullptr, n));
  if (time) VG_HIP(hipMemcpy(ctx->d_t, time, (size_t)n * sizeof(float), hipMemcpyHostToDevice));
  float4* out = nullptr;
  VG_HIP(hipMalloc((void**)&out, (size_t)n * sizeof(float4)));
  int m = 0;
  const int r = ds_close(ctx, ctx->d_x, ctx->d_y, ctx->d_z, time ? ctx->d_t : nullptr, 0.0f, n, voxel_size, out, &m);
  if (r == VG_OK && m > 0) {
    const hipError_t e = hipMemcpy(out_xyzt, out, (size_t)m * sizeof(float4), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      (void)hipFree(out);
      ctx->err = std::string("vg_downsample_close: ") + hipGetErrorString(e);
      return VG_E_HIP;
    }
  }
  (void)hipFree(out);
  VG_TRY(r);
  *n_out = m;
  return VG_OK;
}

int vg_seed(vg_ctx* ctx, const double* state) {
  if (!ctx || !state) return VG_E_ARG;
  host_seed(ctx, state);
  return VG_OK;
}

// A host-input scan into one of the two in-flight slots: the caller's arrays
// are copied once into the slot's pinned block (the only host work per point),
// one DMA takes them to HBM and k_unpack_scan writes the SoA planes, both on
// stream_ds; the main stream waits for the unpack on the device. The slot is
// reused two scans later: the host waits for its previous DMA (long done in
// the steady state), the device for the main stream to pass the scan that read
// it. *slot receives the index for upload_done.
static int upload_scan(vg_ctx* ctx, const float* xyz, const float* inten, const float* time, int n, float* soa[5],
                       int* slot) {
  // slots sized to the largest scan so far (grown with headroom; the old ones
  // are released once both streams have drained)
  if ((size_t)n > ctx->in_cap) {
    VG_HIP(hipStreamSynchronize(ctx->stream_ds));
    VG_HIP(hipStreamSynchronize(ctx->stream));
    for (auto& sl : ctx->in_slot) {
      if (sl.h) VG_HIP(hipHostFree(sl.h));
      if (sl.d) VG_HIP(hipFree(sl.d));
      sl.h = nullptr;
      sl.d = nullptr;
      sl.live = false;
    }
    ctx->in_cap = std::min((size_t)ctx->cap.max_points_per_scan, ((size_t)n * 5 / 4 + 65535) & ~(size_t)65535);
  }
  const size_t cap = ctx->in_cap;
  if (!ctx->in_slot[0].h) {
    for (auto& sl : ctx->in_slot) {
      VG_HIP(hipHostMalloc((void**)&sl.h, cap * 5 * sizeof(float), hipHostMallocDefault));
      VG_HIP(hipMalloc((void**)&sl.d, cap * 10 * sizeof(float)));
      if (!sl.up) VG_HIP(hipEventCreateWithFlags(&sl.up, hipEventDisableTiming | hipEventDisableSystemFence));
      if (!sl.done) VG_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming | hipEventDisableSystemFence));
    }
  }
  *slot = ctx->in_next;
  vg_ctx::InSlot& sl = ctx->in_slot[ctx->in_next];
  ctx->in_next ^= 1;
  if (sl.live) VG_HIP(hipEventSynchronize(sl.up));
  const size_t nn = (size_t)n;
  size_t nf = 3 * nn;
  std::vector<CopyPool::Job> pieces;
  pieces.push_back({sl.h, (const char*)xyz, nn * 3 * sizeof(float)});
  if (inten) {
    pieces.push_back({sl.h + nf * sizeof(float), (const char*)inten, nn * sizeof(float)});
    nf += nn;
  }
  if (time) {
    pieces.push_back({sl.h + nf * sizeof(float), (const char*)time, nn * sizeof(float)});
    nf += nn;
  }
  pinned_copy(ctx, pieces);
  hipStream_t s = ctx->stream_ds;
  if (sl.live) VG_HIP(hipStreamWaitEvent(s, sl.done, 0));
  VG_HIP(hipMemcpyAsync(sl.d, sl.h, nf * sizeof(float), hipMemcpyHostToDevice, s));
  float* pl = sl.d + 5 * cap;
  for (int c = 0; c < 5; c++) soa[c] = pl + (size_t)c * cap;
  VG_TRY(state_unpack_scan(ctx, s, n, sl.d, inten != nullptr, time != nullptr, soa[0], soa[1], soa[2], soa[3], soa[4]));
  VG_HIP(hipEventRecord(sl.up, s));
  if (s != ctx->stream) VG_HIP(hipStreamWaitEvent(ctx->stream, sl.up, 0));
  ctx->in_ev = sl.up;
  sl.live = true;
  return VG_OK;
}

// after the scan's enqueue: the main stream has everything that reads the slot
// (the IEKF stream and the downsample stream join it before the insert)
static int upload_done(vg_ctx* ctx, int slot, int r) {
  ctx->in_ev = nullptr;
  const hipError_t e = hipEventRecord(ctx->in_slot[slot].done, ctx->stream);
  if (r == VG_OK && e != hipSuccess) {
    ctx->err = std::string("upload_done: ") + hipGetErrorString(e);
    return VG_E_HIP;
  }
  return r;
}

int vg_step(vg_ctx* ctx, const float* xyz, const float* intensity, int n, double pcl_beg_time,
            double pcl_end_time, const double* imu, int m) {
  if (!ctx || (!xyz && n > 0) || n < 0 || m < 0 || (m > 0 && !imu)) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  if (n == 0) return host_step(ctx, ctx->d_x, ctx->d_y, ctx->d_z, ctx->d_i, n, pcl_beg_time, pcl_end_time, imu, m);
  float* p[5];
  int slot = 0;
  VG_TRY(upload_scan(ctx, xyz, intensity, nullptr, n, p, &slot));
  return upload_done(ctx, slot, host_step(ctx, p[0], p[1], p[2], p[3], n, pcl_beg_time, pcl_end_time, imu, m));
}

int vg_step_dev(vg_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, const float* d_intensity, int n,
                double pcl_beg_time, double pcl_end_time, const double* imu, int m) {
  if (!ctx || n < 0 || m < 0 || (m > 0 && !imu) || (n > 0 && (!d_x || !d_y || !d_z))) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  return host_step(ctx, d_x, d_y, d_z, d_intensity, n, pcl_beg_time, pcl_end_time, imu, m);
}

int vg_step_deskew_dev(vg_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, const float* d_intensity,
                       const float* d_time, int n, double pcl_beg_time, double pcl_end_time, const double* imu,
                       int m) {
  if (!ctx || n < 0 || m < 0 || (m > 0 && !imu) || (n > 0 && (!d_x || !d_y || !d_z || !d_time))) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  return host_step_deskew(ctx, d_x, d_y, d_z, d_intensity, d_time, n, pcl_beg_time, pcl_end_time, imu, m);
}

int vg_step_deskew(vg_ctx* ctx, const float* xyz, const float* intensity, const float* time, int n,
                   double pcl_beg_time, double pcl_end_time, const double* imu, int m) {
  if (!ctx || (n > 0 && (!xyz || !time)) || n < 0 || m < 0 || (m > 0 && !imu)) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  if (n == 0)
    return host_step_deskew(ctx, ctx->d_x, ctx->d_y, ctx->d_z, ctx->d_i, ctx->d_t, n, pcl_beg_time, pcl_end_time, imu,
                            m);
  float* p[5];
  int slot = 0;
  VG_TRY(upload_scan(ctx, xyz, intensity, time, n, p, &slot));
  return upload_done(ctx, slot,
                     host_step_deskew(ctx, p[0], p[1], p[2], p[3], p[4], n, pcl_beg_time, pcl_end_time, imu, m));
}

int vg_get_state(vg_ctx* ctx, double* state) {
  if (!ctx || !state) return VG_E_ARG;
  VG_TRY(host_state(ctx, state));
  return VG_OK;
}

// the last completed scan's downsampled cloud (body frame after the deskew,
// the map path's pl_down, local_mapping.cpp:396-406): the points
// pub_localtraj publishes on /map_scan once moved to the world
// (publishers.cpp:65-97). Completes the outstanding work first.
int vg_scan_points(vg_ctx* ctx, float* xyz, int cap, int* n) {
  if (!ctx || !n || cap < 0 || (cap > 0 && !xyz)) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  int cnt = 0;
  VG_HIP(hipMemcpy(&cnt, ctx->ds.hflags + 1, sizeof(int), hipMemcpyDeviceToHost));
  *n = cnt;
  const int k = cnt < cap ? cnt : cap;
  if (k > 0) {
    std::vector<float> b((size_t)3 * k);
    VG_HIP(hipMemcpy(b.data(), ctx->ds.ox, k * sizeof(float), hipMemcpyDeviceToHost));
    VG_HIP(hipMemcpy(b.data() + k, ctx->ds.oy, k * sizeof(float), hipMemcpyDeviceToHost));
    VG_HIP(hipMemcpy(b.data() + 2 * k, ctx->ds.oz, k * sizeof(float), hipMemcpyDeviceToHost));
    for (int i = 0; i < k; i++) {
      xyz[3 * i] = b[i];
      xyz[3 * i + 1] = b[k + i];
      xyz[3 * i + 2] = b[2 * k + i];
    }
  }
  return VG_OK;
}

int vg_release_far(vg_ctx* ctx, int flags, long long* out) {
  if (!ctx || !out || (flags & ~3)) return VG_E_ARG;
  if (!(flags & 3)) {  // nothing asked but the release: no wait unless one is pending
    VG_TRY(host_poll(ctx));
    if (!host_release_pending(ctx)) {
      for (int i = 0; i < 6; i++) out[i] = -1;
      return VG_OK;
    }
  }
  VG_TRY(host_sync(ctx));
  return host_release_far(ctx, flags, out);
}

int vg_get_stats(vg_ctx* ctx, vg_stats* out) {
  if (!ctx || !out) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  *out = ctx->stats;
  return VG_OK;
}

int vg_stats_log(vg_ctx* ctx, vg_stats* out, int cap, int* n) {
  if (!ctx || !n || cap < 0) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  *n = host_stats_log(ctx, out, cap);
  return VG_OK;
}

int vg_window_states(vg_ctx* ctx, double* out, int* n) {
  if (!ctx || !n || !out) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  *n = host_window(ctx, out);
  return VG_OK;
}

int vg_trajectory(vg_ctx* ctx, double* out, int cap, int* n) {
  if (!ctx || !n) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  *n = host_traj(ctx, out, cap);
  return VG_OK;
}

int vg_path(vg_ctx* ctx, double* out, int cap, int* n) {
  if (!ctx || !n || cap < 0) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  *n = host_path(ctx, out, cap);
  return VG_OK;
}

int vg_set_publish(vg_ctx* ctx, int flags) {
  if (!ctx || (flags & ~1)) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  if ((flags & 1) && !(ctx->pub_flags & 1)) VG_HIP(hipMemset(ctx->d_cmap_n, 0, sizeof(int)));
  ctx->pub_flags = flags;
  return VG_OK;
}

int vg_local_map(vg_ctx* ctx, float* out_xyzi, int cap, int* n) {
  if (!ctx || !n || cap < 0 || (cap > 0 && !out_xyzi)) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  int k = 0;
  if (ctx->pub_flags & 1) VG_HIP(hipMemcpy(&k, ctx->d_cmap_n, sizeof(int), hipMemcpyDeviceToHost));
  *n = k;
  const int c = k < cap ? k : cap;
  if (c > 0) VG_HIP(hipMemcpy(out_xyzi, ctx->d_cmap, (size_t)c * sizeof(float4), hipMemcpyDeviceToHost));
  return VG_OK;
}

int vg_poll(vg_ctx* ctx, int* n_scans, int* n_traj, int* n_path) {
  if (!ctx) return VG_E_ARG;
  VG_TRY(host_poll(ctx));
  if (n_scans) *n_scans = host_stats_log(ctx, nullptr, 0);
  if (n_traj) *n_traj = host_traj(ctx, nullptr, 0);
  if (n_path) *n_path = host_path(ctx, nullptr, 0);
  return VG_OK;
}

int vg_poll_rows(vg_ctx* ctx, double* traj, int traj_from, int traj_cap, double* path, int path_cap) {
  if (!ctx || traj_from < 0 || traj_cap < 0 || path_cap < 0) return VG_E_ARG;
  if (traj && traj_cap > 0) host_traj(ctx, traj, traj_cap, traj_from);
  if (path && path_cap > 0) host_path(ctx, path, path_cap);
  return VG_OK;
}

// ---- stage-level API (include/vina_gpu.h "Stage-level API") ----
int vg_scan_load(vg_ctx* ctx, const float* xyz, const float* intensity, int n) {
  if (!ctx || n < 0 || (n > 0 && !xyz)) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  if (n > 0) VG_TRY(upload_aos(ctx, xyz, intensity, n));
  ctx->cur_x = ctx->d_x;
  ctx->cur_y = ctx->d_y;
  ctx->cur_z = ctx->d_z;
  ctx->cur_i = ctx->d_i;
  ctx->cur_n = n;
  return VG_OK;
}

int vg_scan_bind_dev(vg_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, const float* d_intensity,
                     int n) {
  if (!ctx || n < 0 || (n > 0 && (!d_x || !d_y || !d_z))) return VG_E_ARG;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "scan larger than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  ctx->cur_x = d_x;
  ctx->cur_y = d_y;
  ctx->cur_z = d_z;
  ctx->cur_i = d_intensity;
  ctx->cur_n = n;
  return VG_OK;
}

static int need_scan(vg_ctx* ctx) {
  if (ctx->cur_n < 0) {
    ctx->err = "no scan loaded (vg_scan_load / vg_scan_bind_dev)";
    return VG_E_STATE;
  }
  return VG_OK;
}

int vg_propagate(vg_ctx* ctx, const double* imu, int m, double pcl_beg_time, double pcl_end_time) {
  if (!ctx || m < 0 || (m > 0 && !imu)) return VG_E_ARG;
  return stage_propagate(ctx, imu, m, pcl_beg_time, pcl_end_time);
}

int vg_downsample_scan(vg_ctx* ctx, int* n_ds) {
  if (!ctx) return VG_E_ARG;
  VG_TRY(need_scan(ctx));
  return stage_downsample(ctx, ctx->cur_x, ctx->cur_y, ctx->cur_z, ctx->cur_i, ctx->cur_n, n_ds);
}

int vg_lio_state_estimation(vg_ctx* ctx, int* degenerate) {
  if (!ctx) return VG_E_ARG;
  VG_TRY(need_scan(ctx));
  return stage_iekf(ctx, ctx->cur_x, ctx->cur_y, ctx->cur_z, ctx->cur_n, degenerate);
}

int vg_window_push(vg_ctx* ctx, const double* imu, int m) {
  if (!ctx || m < 0 || (m > 0 && !imu)) return VG_E_ARG;
  return stage_window_push(ctx, imu, m);
}

int vg_cut_voxel_multi(vg_ctx* ctx) {
  if (!ctx) return VG_E_ARG;
  return stage_insert(ctx);
}

int vg_multi_recut(vg_ctx* ctx, int* n_factors) {
  if (!ctx) return VG_E_ARG;
  return stage_recut(ctx, n_factors);
}

int vg_damping_iter(vg_ctx* ctx, int* lm_iters) {
  if (!ctx) return VG_E_ARG;
  return stage_ba(ctx, lm_iters);
}

int vg_multi_margi(vg_ctx* ctx) {
  if (!ctx) return VG_E_ARG;
  return stage_margi_slide(ctx);
}

int vg_step_end(vg_ctx* ctx) {
  if (!ctx) return VG_E_ARG;
  return stage_finish(ctx);
}

int vg_win_count(vg_ctx* ctx, int* n) {
  if (!ctx || !n) return VG_E_ARG;
  *n = host_win_count(ctx);
  return VG_OK;
}

int vg_set_wait_policy(vg_ctx* ctx, int spin_us, int sleep_us) {
  if (!ctx || spin_us < 0 || sleep_us < 0) return VG_E_ARG;
  ctx->wait_spin_us = spin_us;
  ctx->wait_sleep_us = sleep_us;
  return VG_OK;
}

int vg_profile(vg_ctx* ctx, int on) {
  if (!ctx) return VG_E_ARG;
  ctx->prof_on = (on & 1) != 0;
  ctx->prof_stages = (on & 2) != 0;
  ctx->prof_clock = (on & 4) != 0;
  ctx->prof_every = (on >> 8) & 0xff;  // k_ba_solve events on every prof_every-th BA run (0/1: every run)
  ctx->prof_runs = 0;
  {  // bit 2: the in-kernel clocks (KClock), reset; set behind everything already enqueued
    VG_TRY(host_sync(ctx));
    VG_HIP(hipMemset(&ctx->st->clk, 0, sizeof(vg::KClock)));
    const int clk_on = (on & 4) ? 1 : 0;
    VG_HIP(hipMemcpy(&ctx->st->clk.on, &clk_on, sizeof(int), hipMemcpyHostToDevice));
  }
  ctx->iekf_ring_n = 0;
  for (int i = 0; i < vg::kProfAll; i++) {
    ctx->prof_ms[i] = 0;
    ctx->prof_n[i] = 0;
    ctx->prof_pending[i] = false;
  }
  return VG_OK;
}

int vg_profile_read(vg_ctx* ctx, int stage, double* total_ms, int* count) {
  if (!ctx || stage < 0 || stage >= vg::kProfAll + 4 || !total_ms || !count) return VG_E_ARG;
  // 16 k_iekf, 17 k_ba_solve, 18 the recut level kernels (per scan), 19 k_ba_hess:
  // kernel-only time from the in-kernel clocks
  if (stage >= vg::kProfAll) {
    VG_TRY(host_sync(ctx));
    std::vector<vg::KClock> kv(1);
    vg::KClock& k = kv[0];
    VG_HIP(hipMemcpy(&k, &ctx->st->clk, sizeof(k), hipMemcpyDeviceToHost));
    int khz = 0;
    VG_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
    unsigned long long t = k.solve_ticks, nl = k.solve_n;
    const int s1 = k.scan, s0 = k.scan - 63 > 1 ? k.scan - 63 : 1;  // the last <= 64 scans
    if (stage == vg::kProfAll + 2) {  // recut level kernels: one span per scan
      t = 0;
      nl = 0;
      for (int sc = s0; sc <= s1; sc++) {
        const int slot = sc & (vg::kClkRcScans - 1);
        if (!k.rc_exec[slot]) continue;
        unsigned long long e = 0;
        for (int b = 0; b < vg::kClkRcBlocks; b++) e = k.rc_tend[slot][b] > e ? k.rc_tend[slot][b] : e;
        if (e > k.rc_t0[slot]) {
          t += e - k.rc_t0[slot];
          nl++;
        }
      }
    }
    if (stage == vg::kProfAll + 3) {  // k_ba_hess: the executed launches
      t = 0;
      nl = 0;
      for (int sc = s0; sc <= s1; sc++)
        for (int it = 0; it < 8; it++) {
          const int slot = (sc * 8 + it) & (vg::kClkHRing - 1);
          if (!k.h_exec[slot]) continue;
          unsigned long long e = 0;
          for (int b = 0; b < vg::kClkHBlocks; b++) e = k.h_tend[slot][b] > e ? k.h_tend[slot][b] : e;
          if (e > k.h_t0[slot]) {
            t += e - k.h_t0[slot];
            nl++;
          }
        }
    }
    if (stage == vg::kProfAll) {  // k_iekf: the executed launches of the last <= 64 scans
      t = 0;
      nl = 0;
      const int nb = vg::iekf_grid(ctx) < vg::kClkBlocks ? vg::iekf_grid(ctx) : vg::kClkBlocks;
      // (s0, s1: kClkRing / 4 = 64 scans)
      for (int sc = s0; sc <= s1; sc++)
        for (int it = 0; it < 4; it++) {
          const int slot = (sc * 4 + it) & (vg::kClkRing - 1);
          if (!k.exec[slot]) continue;
          unsigned long long e = 0;
          for (int b = 0; b < nb; b++) e = k.tend[slot][b] > e ? k.tend[slot][b] : e;
          if (e > k.t0[slot]) {
            t += e - k.t0[slot];
            nl++;
          }
        }
    }
    *total_ms = khz > 0 ? (double)t / (double)khz : 0.0;
    *count = (int)nl;
    return VG_OK;
  }
  *total_ms = ctx->prof_ms[stage];
  *count = ctx->prof_n[stage];
  return VG_OK;
}

}  // extern "C"

// Test-only knobs (not part of include/vina_gpu.h): key 1 = event capacity of
// the single-workgroup recut apply (0 forces the host-sized replay path).
extern "C" int vgx_debug(vg_ctx* ctx, int key, int value) {
  if (!ctx) return VG_E_ARG;
  if (key == 2) {  // 0: direct launches only (no hipGraph replay)
    ctx->use_graphs = value != 0;
    return VG_OK;
  }
  if (key == 1) {
    ctx->dbg_apply_cap = value;
    return VG_OK;
  }
  if (key == 3) {
    ctx->dbg_ins_cap = value;
    return VG_OK;
  }
  if (key == 4) {
    ctx->dbg_fac_max = value;
    return VG_OK;
  }
  if (key == 12) {  // sharded: add `value` to this context's exchange counter (desynchronises the guard)
    if (!ctx->shard.d_seq) return VG_E_STATE;
    unsigned s = 0;
    VG_HIP(hipMemcpy(&s, ctx->shard.d_seq, sizeof(s), hipMemcpyDeviceToHost));
    s += (unsigned)value;
    VG_HIP(hipMemcpy(ctx->shard.d_seq, &s, sizeof(s), hipMemcpyHostToDevice));
    return VG_OK;
  }
  if (key == 24) {  // 1: k_margi_leaf batches a leaf's frame-cluster loads
    ctx->margi_batch = value != 0;
    return VG_OK;
  }
  if (key == 23) {  // 1: k_iekf prefetches a cached match's plane record
    ctx->iekf_prefetch = value != 0;
    return VG_OK;
  }
  if (key == 21) {  // 0: margi's isexist / erase passes as per-level launches
    ctx->margi_fused = value != 0;
    return VG_OK;
  }
  if (key == 19) {  // 0: the LM bookkeeping as its own k_ba_control launch
    ctx->ba_fuse_ctl = value != 0;
    return VG_OK;
  }
  if (key == 17) {  // 0: one graph per LM iteration (no two-iteration graph)
    ctx->ba_graph2 = value != 0;
    return VG_OK;
  }
  if (key == 16) {  // 0: root registration as k_ins_flags + k_ins_roots_alloc
    ctx->roots_lb = value != 0;
    return VG_OK;
  }
  if (key == 15) {  // 0: the LM iterations as direct launches (no graph per iteration)
    ctx->ba_graph = value != 0;
    return VG_OK;
  }
  if (key == 37) {  // 0: host_step enqueues the early downsample ahead of the propagation / IEKF launches
    ctx->ds_after_iekf = value != 0;
    return VG_OK;
  }
  if (key == 35) {  // 0: k_ba_init as its own launch ahead of the scan graph's first k_ba_hess
    ctx->ba_init_hess = value != 0;
    return VG_OK;
  }
  if (key == 34) {  // 0: the second LM iteration's Hessian by its own k_ba_hess, not inside the first's residual pass
    ctx->ba_resid_hess = value != 0;
    return VG_OK;
  }
  if (key == 33) {  // 0: k_make_win_recut_begin as its own launch in the insert + recut graph
    ctx->rc_begin_fold = value != 0;
    return VG_OK;
  }
  if (key == 32) {  // 0: k_factor_finish_dev after k_fac_sort instead of inside k_ba_init
    ctx->rc_init_finish = value != 0;
    return VG_OK;
  }
  if (key == 31) {  // 0: the LM system in Eigen's pivot order (descending |diag|) instead of the structural one
    ctx->ba_structural = value != 0;
    return VG_OK;
  }
  if (key == 30) {  // 1: vg_shard_rccl(ctx, 0, 1, id) sets up the sharded path on one GPU (RCCL, one rank)
    ctx->shard_force = value != 0;
    return VG_OK;
  }
  if (key == 14) {  // 0: event waits for the margi leaf -> IEKF and IEKF -> insert hand-offs;
                    // 2: the flag hand-offs even beside other contexts on the device (a caller that
                    // drains each context before stepping another, as the A/B tests do)
    ctx->flag_sync = value != 0;
    ctx->flag_force = value == 2;
    return VG_OK;
  }
  if (key == 27) {  // 0: no scan graph (separate insert+recut graph, LM launches, margi tail)
    ctx->scan_graph = value != 0;
    return VG_OK;
  }
  if (key == 26) {  // 0: a fused step waits for its LM's outcome (no deferral to the next step)
    ctx->lm_defer = value != 0;
    return VG_OK;
  }
  if (key == 13) {  // 1: host_step always propagates on the device (0: only while an LM is pending)
    ctx->dev_prop = value != 0;
    return VG_OK;
  }
  if (key == 11) {  // 0: the recut's four-launch level loop instead of the fused levels
    ctx->rc_fused = value != 0;
    return VG_OK;
  }
  if (key == 7) {  // 0: the IEKF waits for the whole margi (no cross-scan overlap)
    ctx->overlap_iekf = value != 0;
    return VG_OK;
  }
  if (key == 9) {  // 0: a fused step enqueues its downsample after the IEKF, not before the state wait
    ctx->ds_early = value != 0;
    return VG_OK;
  }
  if (key == 8) {  // 0: the margi tail is enqueued only after the LM is seen done
    ctx->spec_tail = value != 0;
    return VG_OK;
  }
  if (key == 5) {  // arm: the next LM run copies its first Hessian pass (LiDAR hl + IMU blocks)
    if (!ctx->dbg_cap_buf)
      VG_HIP(hipMalloc((void**)&ctx->dbg_cap_buf, (size_t)(4096 + 32 * 931) * sizeof(double)));
    ctx->dbg_capture = value ? 1 : 0;
    ctx->dbg_cap_n = 0;
    return VG_OK;
  }
  return VG_E_ARG;
}

// Test-only: the IEKF memo against fresh descents at internal nodes' centre
// planes (map.hip k_memo_probe); out[4]: samples, mismatches of the inclusive
// box, mismatches of the descent region k_iekf uses, samples split by the plane
extern "C" int vgx_memo_probe(vg_ctx* ctx, int* out) {
  if (!ctx || !out) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  return host_memo_probe(ctx, out);
}

// Test-only: every root voxel of the device map (lifetime.hip map_roots) —
// key x/y/z, jour stamp, flags (1: in the slide map, 2: isexist), subtree
// nodes and point_fix points — for a per-root comparison with the oracle's
// surf_map (orc_roots). *n = the root count; rows past cap are not written.
extern "C" int vgx_roots(vg_ctx* ctx, long long* key, double* jour, int* flags, int* nodes, int* nfix, int cap,
                         int* n) {
  if (!ctx || !n || cap < 0 || (cap > 0 && (!key || !jour || !flags || !nodes || !nfix))) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  return map_roots(ctx, key, jour, flags, nodes, nfix, cap, n);
}

// Test-only: the per-scan pipeline's hashed downsample (ds_enqueue_hashed,
// fallback off) of a host cloud: [x, y, z, intensity, count] per voxel in its
// first-occurrence order.
extern "C" int vgx_downsample_hashed(vg_ctx* ctx, const float* xyz, const float* intensity, int n, double voxel,
                                     float* out_xyzic, int* n_out) {
  if (!ctx || !xyz || !out_xyzic || !n_out || n <= 0) return VG_E_ARG;
  VG_TRY(host_sync(ctx));
  VG_HIP(hipStreamSynchronize(ctx->stream_ds));
  VG_TRY(upload_aos(ctx, xyz, intensity, n));
  const bool fallback = voxel < 0;  // test knob: a negative size runs the pipeline's /2 fallback pass as well
  if (fallback) voxel = -voxel;
  VG_TRY(ds_enqueue_hashed(ctx, ctx->stream, ctx->d_x, ctx->d_y, ctx->d_z, ctx->d_i, n, voxel, fallback, 0));
  hipStream_t s = ctx->stream;
  VG_HIP(hipMemcpyAsync(ctx->h_pinned, ctx->ds.hflags, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  const int m = ctx->h_pinned[1];
  const DownsampleBufs& d = ctx->ds;
  std::vector<float> buf((size_t)m * 5);
  const float* cols[5] = {d.ox, d.oy, d.oz, d.oi, d.oc};
  for (int c = 0; c < 5; c++)
    VG_HIP(hipMemcpyAsync(buf.data() + (size_t)c * m, cols[c], m * sizeof(float), hipMemcpyDeviceToHost, s));
  VG_HIP(hipMemsetAsync(ctx->ds.hflags, 0, sizeof(int), s));  // the range flag (no insert consumes it here)
  VG_HIP(hipStreamSynchronize(s));
  for (int v = 0; v < m; v++)
    for (int c = 0; c < 5; c++) out_xyzic[5 * v + c] = buf[(size_t)c * m + v];
  *n_out = m;
  return ctx->h_pinned[0] ? VG_E_RANGE : VG_OK;
}

// Test-only: the captured first Hessian pass of an LM run (vgx_debug 5), as
// [6W x 6W LiDAR Hessian (full, row-major), 6W gradient, residual, then per
// IMU factor k: J^T C J 30 x 30, J^T C r 30, r^T C r] — the oracle's
// orc_capture_get layout (acc_evaluate2 summed over factors, factors.cpp:22-126;
// give_evaluate, imu_preintegration.cpp:97-163). *n = doubles written.
extern "C" int vgx_ba_capture(vg_ctx* ctx, double* out, int cap, int* n) {
  if (!ctx || !n) return VG_E_ARG;
  VG_TRY(vg::host_sync(ctx));
  *n = 0;
  if (ctx->dbg_capture != 2 || ctx->dbg_cap_n <= 0) return VG_OK;
  const int W = ctx->cfg.win_size, L = 6 * W, nl = L * (L + 1) / 2, nout = nl + L + 1;
  std::vector<double> raw(ctx->dbg_cap_n);
  VG_HIP(hipMemcpy(raw.data(), ctx->dbg_cap_buf, raw.size() * sizeof(double), hipMemcpyDeviceToHost));
  std::vector<double> o;
  o.resize((size_t)L * L);
  for (int r = 0; r < L; r++)
    for (int c = 0; c <= r; c++) o[(size_t)r * L + c] = o[(size_t)c * L + r] = raw[(size_t)r * (r + 1) / 2 + c];
  o.insert(o.end(), raw.begin() + nl, raw.begin() + nout);
  o.insert(o.end(), raw.begin() + nout, raw.end());
  const int m = (int)o.size() < cap ? (int)o.size() : cap;
  if (out) memcpy(out, o.data(), (size_t)m * sizeof(double));
  *n = (int)o.size();
  return VG_OK;
}

// Test-only: k_ba_solve on a given (15W-15)-unknown symmetric system (row-major
// A, rhs b) in identity pivot order -> x. The context must not be stepped after.
extern "C" int vgx_ba_solve(vg_ctx* ctx, const double* A, const double* b, double* x) {
  if (!ctx || !A || !b || !x) return VG_E_ARG;
  VG_TRY(vg::host_sync(ctx));
  return vg::ba_solve_test(ctx, A, b, x);
}

int vg_lio_kdtree(vg_ctx* ctx, const float* xyz, int n, double* state, int* valid, int* iters) {
  if (!ctx || (!xyz && n > 0) || n < 0 || !state || !valid || !iters) return VG_E_ARG;
  return host_lio_kdtree(ctx, xyz, n, state, valid, iters);
}

int vg_kdmap_get(vg_ctx* ctx, float* xyz, int cap, int* n) {
  if (!ctx || !n) return VG_E_ARG;
  *n = ctx->kd.n;
  if (!xyz || cap <= 0) return VG_OK;
  const int m = ctx->kd.n < cap ? ctx->kd.n : cap;
  std::vector<float> t((size_t)3 * m);
  if (m > 0) {
    VG_HIP(hipMemcpy(t.data(), ctx->kd.x, (size_t)m * sizeof(float), hipMemcpyDeviceToHost));
    VG_HIP(hipMemcpy(t.data() + m, ctx->kd.y, (size_t)m * sizeof(float), hipMemcpyDeviceToHost));
    VG_HIP(hipMemcpy(t.data() + 2 * (size_t)m, ctx->kd.z, (size_t)m * sizeof(float), hipMemcpyDeviceToHost));
  }
  for (int i = 0; i < m; i++) {
    xyz[3 * i] = t[i];
    xyz[3 * i + 1] = t[(size_t)m + i];
    xyz[3 * i + 2] = t[2 * (size_t)m + i];
  }
  return VG_OK;
}

int vg_decode_scan(vg_ctx* ctx, const void* records, int n, const vg_lidar_format* fmt, float* xyz, float* intensity,
                   float* time, int* n_out) {
  if (!ctx || !fmt || (!records && n > 0) || n < 0 || !xyz || !time || !n_out) return VG_E_ARG;
  return decode_scan(ctx, records, n, fmt, xyz, intensity, time, n_out);
}

