// micro-benchmark: latency of one symmetric 3x3 eigen-decomposition (vg_la.h eig3)
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../vina-slam_amd/csrc/vg_la.h"
using namespace vg;
__global__ void k_eig(const double* in, double* out, int reps) {
  M3 A;
  for (int i = 0; i < 9; i++) A[i] = in[i];
  unsigned long long t0 = wall_clock64();
  V3 w;
  M3 V;
  for (int r = 0; r < reps; r++) {
    eig3(A, w, V);
    A(0, 0) += w[0] * 1e-30;
  }
  unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = (double)(t1 - t0) / reps;
    out[1] = w[0] + V[0];
  }
}
int main() {
  double *in, *out;
  hipMalloc(&in, 9 * 8);
  hipMalloc(&out, 8 * 8);
  // a thin planar cluster covariance (lambda ~ 1e-5, 0.02, 0.05)
  double h[9] = {0.05, 0.001, 0.0002, 0.001, 0.02, 0.0003, 0.0002, 0.0003, 0.00002};
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  for (int it = 0; it < 3; it++) {
    k_eig<<<1, 64>>>(in, out, 20);
    hipDeviceSynchronize();
    double r[2];
    hipMemcpy(r, out, 16, hipMemcpyDeviceToHost);
    printf("eig3: %.2f us per call (one wave)\n", r[0] * 0.01);
  }
  return 0;
}
