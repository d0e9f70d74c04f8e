// micro-benchmark: host cost of a kernel launch, direct vs replayed hipGraph
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void k_empty(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && v < 0) p[0] = v;
}
int main() {
  int* d;
  hipMalloc(&d, 64);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  using clk = std::chrono::steady_clock;
  for (int rep = 0; rep < 2; rep++) {
    hipStreamSynchronize(s);
    auto t0 = clk::now();
    for (int i = 0; i < 1000; i++) k_empty<<<64, 256, 0, s>>>(d, i);
    auto t1 = clk::now();
    hipStreamSynchronize(s);
    auto t2 = clk::now();
    printf("direct: host %.2f us/launch, drain %.2f us/launch\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / 1000);
  }
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; i++) k_empty<<<64, 256, 0, s>>>(d, i);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int rep = 0; rep < 3; rep++) {
    hipStreamSynchronize(s);
    auto t0 = clk::now();
    for (int i = 0; i < 10; i++) hipGraphLaunch(ge, s);
    auto t1 = clk::now();
    hipStreamSynchronize(s);
    auto t2 = clk::now();
    printf("graph(100 nodes): host %.2f us/node, drain %.2f us/node\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / 1000);
  }
  return 0;
}
