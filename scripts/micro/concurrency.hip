// micro-benchmark: how many dependent kernel launches per second the device
// completes when S independent chains (one per stream, like S sequences) run
// concurrently — direct launches, one graph per chain, or one graph holding
// all S chains. A chain of `len` dependent kernels stands for one scan.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_work(float* p, int n) {  // a few us of real work per launch
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.999f + 1.0f;
}

int main(int argc, char** argv) {
  const int len = 100, reps = 20, blocks = argc > 1 ? atoi(argv[1]) : 64;
  const int n = blocks * 256;
  using clk = std::chrono::steady_clock;
  for (int S : {1, 2, 4, 8, 16, 32}) {
    std::vector<hipStream_t> st(S);
    std::vector<float*> buf(S);
    for (int s = 0; s < S; s++) {
      hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking);
      hipMalloc(&buf[s], n * sizeof(float));
      hipMemset(buf[s], 0, n * sizeof(float));
    }
    hipDeviceSynchronize();
    // (a) direct launches, round robin over the streams
    auto t0 = clk::now();
    for (int r = 0; r < reps; r++)
      for (int k = 0; k < len; k++)
        for (int s = 0; s < S; s++) k_work<<<blocks, 256, 0, st[s]>>>(buf[s], n);
    hipDeviceSynchronize();
    const double ta = std::chrono::duration<double>(clk::now() - t0).count();
    // (b) one graph per chain, replayed on its stream
    std::vector<hipGraphExec_t> ge(S);
    for (int s = 0; s < S; s++) {
      hipGraph_t g;
      hipStreamBeginCapture(st[s], hipStreamCaptureModeThreadLocal);
      for (int k = 0; k < len; k++) k_work<<<blocks, 256, 0, st[s]>>>(buf[s], n);
      hipStreamEndCapture(st[s], &g);
      hipGraphInstantiate(&ge[s], g, nullptr, nullptr, 0);
      hipGraphDestroy(g);
    }
    for (int s = 0; s < S; s++) hipGraphLaunch(ge[s], st[s]);
    hipDeviceSynchronize();
    t0 = clk::now();
    for (int r = 0; r < reps; r++)
      for (int s = 0; s < S; s++) hipGraphLaunch(ge[s], st[s]);
    hipDeviceSynchronize();
    const double tb = std::chrono::duration<double>(clk::now() - t0).count();
    // (c) one graph with S parallel chains (fork from stream 0)
    hipGraph_t g;
    hipEvent_t fork;
    hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    std::vector<hipEvent_t> join(S);
    hipStreamBeginCapture(st[0], hipStreamCaptureModeThreadLocal);
    hipEventRecord(fork, st[0]);
    for (int s = 1; s < S; s++) hipStreamWaitEvent(st[s], fork, 0);
    for (int k = 0; k < len; k++)
      for (int s = 0; s < S; s++) k_work<<<blocks, 256, 0, st[s]>>>(buf[s], n);
    for (int s = 1; s < S; s++) {
      hipEventCreateWithFlags(&join[s], hipEventDisableTiming);
      hipEventRecord(join[s], st[s]);
      hipStreamWaitEvent(st[0], join[s], 0);
    }
    hipStreamEndCapture(st[0], &g);
    hipGraphExec_t gall;
    hipGraphInstantiate(&gall, g, nullptr, nullptr, 0);
    hipGraphLaunch(gall, st[0]);
    hipDeviceSynchronize();
    t0 = clk::now();
    for (int r = 0; r < reps; r++) hipGraphLaunch(gall, st[0]);
    hipDeviceSynchronize();
    const double tc = std::chrono::duration<double>(clk::now() - t0).count();
    const double nk = (double)reps * len * S;
    printf("S=%2d blocks=%d  direct %.0f kern/s (%.2f us/chain-kernel)  graph/stream %.0f kern/s  one-graph %.0f kern/s\n",
           S, blocks, nk / ta, ta * 1e6 / (reps * len), nk / tb, nk / tc);
    fflush(stdout);
    hipGraphExecDestroy(gall);
    hipGraphDestroy(g);
    for (int s = 0; s < S; s++) {
      hipGraphExecDestroy(ge[s]);
      hipFree(buf[s]);
      hipStreamDestroy(st[s]);
    }
  }
  return 0;
}
