// Can an ncclAllReduce be captured into a hipGraph on this ROCm / RCCL?
// One rank, one GPU: capture pack -> allreduce -> unpack, replay, check sums.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <chrono>

__global__ void k_fill(double* a, int n, double v) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] += v;
}
int main() {
  ncclUniqueId id;
  ncclGetUniqueId(&id);
  ncclComm_t comm;
  hipSetDevice(0);
  if (ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess) { printf("init failed\n"); return 1; }
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int n = 1024;
  double* d;
  hipMalloc(&d, n * sizeof(double));
  hipMemsetAsync(d, 0, n * sizeof(double), s);
  hipStreamSynchronize(s);
  // direct: time 200 allreduces of 64 doubles
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 200; i++) {
    k_fill<<<1, 64, 0, s>>>(d, 64, 1.0);
    ncclAllReduce(d, d, 64, ncclFloat64, ncclSum, comm, s);
  }
  hipStreamSynchronize(s);
  auto t1 = std::chrono::steady_clock::now();
  printf("direct: %.2f us per fill+allreduce\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 200);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  printf("begin capture: %s\n", hipGetErrorString(e));
  for (int i = 0; i < 4; i++) {
    k_fill<<<1, 64, 0, s>>>(d, 64, 1.0);
    ncclResult_t r = ncclAllReduce(d, d, 64, ncclFloat64, ncclSum, comm, s);
    if (r != ncclSuccess) printf("allreduce in capture: %s\n", ncclGetErrorString(r));
  }
  e = hipStreamEndCapture(s, &g);
  printf("end capture: %s\n", hipGetErrorString(e));
  if (e != hipSuccess) return 2;
  size_t nn = 0;
  hipGraphGetNodes(g, nullptr, &nn);
  printf("graph nodes: %zu\n", nn);
  e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  printf("instantiate: %s\n", hipGetErrorString(e));
  if (e != hipSuccess) return 3;
  hipMemsetAsync(d, 0, n * sizeof(double), s);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 50; i++) hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  t1 = std::chrono::steady_clock::now();
  printf("graph: %.2f us per fill+allreduce\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 200);
  double h[64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("value %.1f (expect 200)\n", h[0]);
  ncclCommDestroy(comm);
  return h[0] == 200.0 ? 0 : 4;
}
