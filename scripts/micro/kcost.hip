// micro-benchmark: GPU time per dependent kernel in one stream, as a function
// of the kernel-argument size, block count, LDS, and whether the kernel writes
// host-mapped memory — what sets the ~4-5 us per small kernel seen in the
// per-scan traces. Direct launches are timed with events around a chain of
// 200 (the host enqueues faster than that: the chain is queued up first).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int B>
struct Big {
  double a[B / 8];
};

template <int B>
__global__ void k_arg(Big<B> g, float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += (float)g.a[0];
}
__global__ void k_lds(float* p) {
  extern __shared__ float s[];
  s[threadIdx.x] = p[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) p[0] = s[1] + 1.0f;
}
__global__ void k_host(int* hp, float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    p[0] += 1.0f;
    __hip_atomic_store(hp, (int)p[0], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <class F>
static void chain(const char* name, hipStream_t s, F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++) {
    // queue a long kernel first so the chain is fully enqueued before it runs
    hipEventRecord(e0, s);
    for (int i = 0; i < 200; i++) launch();
    hipEventRecord(e1, s);
    hipStreamSynchronize(s);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("%-34s %.2f us/kernel\n", name, ms * 1000 / 200);
  }
  // graph of the same chain
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < 200; i++) launch();
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEventRecord(e0, s);
  hipGraphLaunch(ge, s);
  hipEventRecord(e1, s);
  hipStreamSynchronize(s);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-34s %.2f us/kernel (graph)\n", name, ms * 1000 / 200);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
}

int main() {
  float* p;
  hipMalloc(&p, 4096 * sizeof(float));
  hipMemset(p, 0, 4096 * sizeof(float));
  int* hp;
  hipHostMalloc((void**)&hp, 64, hipHostMallocMapped | hipHostMallocCoherent);
  int* dhp;
  hipHostGetDevicePointer((void**)&dhp, hp, 0);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  Big<16> b16{};
  Big<256> b256{};
  Big<2048> b2k{};
  chain("arg 16 B, 1 block", s, [&] { k_arg<16><<<1, 64, 0, s>>>(b16, p); });
  chain("arg 16 B, 64 blocks", s, [&] { k_arg<16><<<64, 256, 0, s>>>(b16, p); });
  chain("arg 16 B, 1024 blocks", s, [&] { k_arg<16><<<1024, 256, 0, s>>>(b16, p); });
  chain("arg 256 B, 64 blocks", s, [&] { k_arg<256><<<64, 256, 0, s>>>(b256, p); });
  chain("arg 2 KB, 64 blocks", s, [&] { k_arg<2048><<<64, 256, 0, s>>>(b2k, p); });
  chain("LDS 64 KB, 1 block x 1024", s, [&] { k_lds<<<1, 1024, 65536, s>>>(p); });
  chain("host-mapped system store", s, [&] { k_host<<<1, 64, 0, s>>>(dhp, p); });
  return 0;
}
