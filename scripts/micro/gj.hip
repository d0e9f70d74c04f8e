// micro-benchmark: 15x15 Gauss-Jordan in one workgroup (vg_iekf.h) vs copies only
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../vina-slam_amd/csrc/vg_iekf.h"
using namespace vg;
__global__ void __launch_bounds__(256) k_gj(const double* in, double* out, int mode) {
  __shared__ double a[15][30], b[15][30];
  const int tid = threadIdx.x;
  for (int e = tid; e < 450; e += blockDim.x) {
    const int r = e / 30, j = e % 30;
    a[r][j] = j < 15 ? in[r * 15 + j] : ((j - 15 == r) ? 1.0 : 0.0);
  }
  __syncthreads();
  double(*K)[30] = a;
  unsigned long long t0 = wall_clock64();
  if (mode == 1) gj_inverse15(a, b, &K);
  if (mode == 2) for (int c = 0; c < 15; c++) __syncthreads();
  unsigned long long t1 = wall_clock64();
  for (int e = tid; e < 225; e += blockDim.x) out[e] = K[e / 15][15 + e % 15];
  if (tid == 0) out[256] = (double)(t1 - t0);
}
int main() {
  double *in, *out;
  hipMalloc(&in, 225 * 8);
  hipMalloc(&out, 512 * 8);
  double h[225];
  for (int i = 0; i < 225; i++) h[i] = (i % 16 == 0) ? 4.0 : 0.01 * (i % 7);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 3; mode++) {
    for (int w = 0; w < 10; w++) k_gj<<<1, 256>>>(in, out, mode);
    hipEventRecord(e0);
    for (int w = 0; w < 200; w++) k_gj<<<1, 256>>>(in, out, mode);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double ticks;
    hipMemcpy(&ticks, out + 256, 8, hipMemcpyDeviceToHost);
    printf("mode %d: %.2f us/launch, in-kernel %.2f us\n", mode, ms * 1e3 / 200, ticks * 0.01);
  }
  return 0;
}
