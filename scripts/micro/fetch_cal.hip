// FETCH_SIZE / WRITE_SIZE calibration on the access shapes of the per-scan
// kernels (MI355X_MICROARCH.md, HBM: the x2 correction is stated for 16 B/lane
// coalesced streaming reads only; "other access widths are uncalibrated").
// Every kernel touches each byte of its region exactly once, regions larger
// than the L2s and never read twice, so the algorithmic bytes are known:
//   stream16  float4 per lane, coalesced                 (the guide's case)
//   soa4      float per lane, 4 planes (k_iekf's x, y, z + the leaf cache)
//   rec224    one 224 B PlaneRec per lane, records in a random permutation
//             (k_iekf's gate: center, normal, 21 plane_var doubles, radius)
//   hdr96     one 96 B NodeHdr per lane, random permutation (the descent)
//   gather8   one double per lane, random permutation over the whole array
//   store16 / store8 / store4  coalesced stores of 16 / 8 / 4 B per lane
//   fachess   k_ba_hess's reads: lane (f, i) of ten lanes per factor reads
//             frame cluster i (80 B) of factor f's ten-cluster block (blocks in
//             a random order, as factor nodes are) plus factor f's 96 B eigen
//             record (all ten lanes the same address, records contiguous)
//   storerun  k_ba_hess's old partial stores: runs of 16 doubles (128 B) at
//             offsets 8 B past a 128 B boundary, four runs per wave, runs in a
//             random order
// Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) --kernel-trace;
// scripts/fetch_cal.py divides the counters by the byte counts printed here.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Rec224 {
  double c[3], n[3], var[21];
  float radius;
  int pad;
};
struct Hdr96 {
  double center[3];
  int child[8];
  int octo, layer, is_plane, isexist;
  double qlen;
  int fix_off, fix_cnt, pad[2];
};
static_assert(sizeof(Rec224) == 224 && sizeof(Hdr96) == 96, "record sizes");

// i -> (i * odd) mod 2^k: a permutation of [0, 2^k)
__device__ __forceinline__ unsigned perm(unsigned i, unsigned mask) { return (i * 2654435761u) & mask; }

__global__ void k_stream16(const float4* __restrict__ a, size_t n, float* __restrict__ sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) sink[0] = s;  // never true: keeps the loads, no store traffic
}
__global__ void k_soa4(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                       const int* __restrict__ c, size_t n, float* __restrict__ sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += x[i] + y[i] + z[i] + (float)c[i];
  if (s == 1234.5f) sink[0] = s;
}
__global__ void k_rec224(const Rec224* __restrict__ r, unsigned mask, float* __restrict__ sink) {
  double s = 0.0;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i <= mask; i += gridDim.x * blockDim.x) {
    const Rec224& q = r[perm(i, mask)];
    for (int k = 0; k < 3; k++) s += q.c[k] * q.n[k];
    for (int k = 0; k < 21; k++) s += q.var[k];
    s += q.radius;
  }
  if (s == 1234.5) sink[0] = (float)s;
}
__global__ void k_hdr96(const Hdr96* __restrict__ h, unsigned mask, float* __restrict__ sink) {
  double s = 0.0;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i <= mask; i += gridDim.x * blockDim.x) {
    const Hdr96& q = h[perm(i, mask)];
    s += q.center[0] + q.center[1] + q.center[2] + q.qlen;
    int t = q.octo + q.layer + q.is_plane + q.isexist + q.fix_off + q.fix_cnt;
    for (int k = 0; k < 8; k++) t += q.child[k];
    s += t;
  }
  if (s == 1234.5) sink[0] = (float)s;
}
__global__ void k_gather8(const double* __restrict__ a, unsigned mask, float* __restrict__ sink) {
  double s = 0.0;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i <= mask; i += gridDim.x * blockDim.x)
    s += a[perm(i, mask)];
  if (s == 1234.5) sink[0] = (float)s;
}
struct Clu80 {
  double v[10];
};
__global__ void k_fachess(const Clu80* __restrict__ clu, const double* __restrict__ eig, unsigned nf,
                          unsigned gmask, float* __restrict__ sink) {
  double s = 0.0;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < nf * 10; t += gridDim.x * blockDim.x) {
    const unsigned f = t / 10, i = t % 10;
    const Clu80& c = clu[(size_t)perm(f, gmask) * 10 + i];
    for (int k = 0; k < 10; k++) s += c.v[k];
    for (int k = 0; k < 12; k++) s += eig[(size_t)f * 12 + k];
  }
  if (s == 1234.5) sink[0] = (float)s;
}
__global__ void k_storerun(double* __restrict__ a, unsigned rmask) {
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < (rmask + 1) * 16; t += gridDim.x * blockDim.x) {
    const unsigned run = perm(t >> 4, rmask);
    a[1 + (size_t)run * 16 + (t & 15)] = 0.0;
  }
}
#define STORE_KERNEL(name, T)                                                                              \
  __global__ void name(T* __restrict__ a, size_t n) {                                                      \
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) \
      a[i] = T{};                                                                                          \
  }
STORE_KERNEL(k_flush, float4)
STORE_KERNEL(k_store16, float4)
STORE_KERNEL(k_store8, double)
STORE_KERNEL(k_store4, float)

int main() {
  const size_t MB = 1 << 20;
  float* sink;
  CK(hipMalloc(&sink, 64));
  char *A, *F;
  const size_t bytesA = 512 * MB;
  CK(hipMalloc(&A, bytesA));
  CK(hipMalloc(&F, 512 * MB));  // a flush buffer written between the measured launches
  CK(hipMemset(A, 0, bytesA));
  CK(hipDeviceSynchronize());
  const int grid = 2048, blk = 256;
  auto flush = [&]() { k_flush<<<grid, blk>>>((float4*)F, 512 * MB / 16); };
  printf("kernel,read_bytes,write_bytes\nk_flush,0,%zu\n", 512 * MB);
  for (int rep = 0; rep < 3; rep++) {
    const size_t nS = 256 * MB / 16;
    flush();
    k_stream16<<<grid, blk>>>((const float4*)A, nS, sink);
    if (rep == 0) printf("k_stream16,%zu,0\n", nS * 16);
    const size_t nP = 64 * MB / 4;  // four 64 MB planes
    flush();
    k_soa4<<<grid, blk>>>((const float*)A, (const float*)(A + 64 * MB), (const float*)(A + 128 * MB),
                          (const int*)(A + 192 * MB), nP, sink);
    if (rep == 0) printf("k_soa4,%zu,0\n", nP * 16);
    const unsigned nR = 1u << 21;  // 2 M records x 224 B = 448 MiB
    flush();
    k_rec224<<<grid, blk>>>((const Rec224*)A, nR - 1, sink);
    if (rep == 0) printf("k_rec224,%zu,0\n", (size_t)nR * 224);
    const unsigned nH = 1u << 22;  // 4 M headers x 96 B = 384 MiB
    flush();
    k_hdr96<<<grid, blk>>>((const Hdr96*)A, nH - 1, sink);
    if (rep == 0) printf("k_hdr96,%zu,0\n", (size_t)nH * 96);
    const unsigned nG = 1u << 25;  // 32 M doubles = 256 MiB, each read once in a random order
    flush();
    k_gather8<<<grid, blk>>>((const double*)A, nG - 1, sink);
    if (rep == 0) printf("k_gather8,%zu,0\n", (size_t)nG * 8);
    const unsigned nF = 1u << 18;  // 256 k factors x (800 B clusters + 96 B eigen record) = 224 MiB
    flush();
    k_fachess<<<grid, blk>>>((const Clu80*)A, (const double*)(A + (size_t)nF * 800), nF, nF - 1, sink);
    if (rep == 0) printf("k_fachess,%zu,0\n", (size_t)nF * 896);
    const unsigned nRun = 1u << 20;  // 1 M runs x 128 B = 128 MiB (+8 B)
    flush();
    k_storerun<<<grid, blk>>>((double*)A, nRun - 1);
    if (rep == 0) printf("k_storerun,0,%zu\n", (size_t)nRun * 128);
    flush();
    k_store16<<<grid, blk>>>((float4*)A, 256 * MB / 16);
    if (rep == 0) printf("k_store16,0,%zu\n", 256 * MB);
    flush();
    k_store8<<<grid, blk>>>((double*)A, 256 * MB / 8);
    if (rep == 0) printf("k_store8,0,%zu\n", 256 * MB);
    flush();
    k_store4<<<grid, blk>>>((float*)A, 256 * MB / 4);
    if (rep == 0) printf("k_store4,0,%zu\n", 256 * MB);
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(A));
  CK(hipFree(F));
  CK(hipFree(sink));
  return 0;
}
