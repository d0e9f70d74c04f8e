// micro-benchmark: rocPRIM radix sort at the pipeline's sizes, default dispatch
// (block sort + merge passes below 1M keys) vs forced onesweep
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
using onesweep_cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;
template <class Cfg>
float time_keys(uint64_t* in, uint64_t* out, int n, int b0, int b1, hipStream_t s) {
  size_t tb = 0;
  rocprim::radix_sort_keys<Cfg>(nullptr, tb, in, out, n, b0, b1, s);
  void* tmp;
  hipMalloc(&tmp, tb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 5; i++) rocprim::radix_sort_keys<Cfg>(tmp, tb, in, out, n, b0, b1, s);
  hipEventRecord(e0, s);
  for (int i = 0; i < 100; i++) rocprim::radix_sort_keys<Cfg>(tmp, tb, in, out, n, b0, b1, s);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipFree(tmp);
  return ms * 10.0f;  // us per sort
}
template <class Cfg>
float time_pairs(uint64_t* in, uint64_t* out, uint32_t* vi, uint32_t* vo, int n, int b0, int b1, hipStream_t s) {
  size_t tb = 0;
  rocprim::radix_sort_pairs<Cfg>(nullptr, tb, in, out, vi, vo, n, b0, b1, s);
  void* tmp;
  hipMalloc(&tmp, tb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 5; i++) rocprim::radix_sort_pairs<Cfg>(tmp, tb, in, out, vi, vo, n, b0, b1, s);
  hipEventRecord(e0, s);
  for (int i = 0; i < 100; i++) rocprim::radix_sort_pairs<Cfg>(tmp, tb, in, out, vi, vo, n, b0, b1, s);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipFree(tmp);
  return ms * 10.0f;
}
int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  std::mt19937_64 rng(1);
  const int N = 1 << 17;
  std::vector<uint64_t> h(N);
  std::vector<uint32_t> hv(N);
  for (int i = 0; i < N; i++) {
    h[i] = ((rng() % 20000ull) << 27) | (uint64_t)i;
    hv[i] = i;
  }
  uint64_t *in, *out;
  uint32_t *vi, *vo;
  hipMalloc(&in, N * 8);
  hipMalloc(&out, N * 8);
  hipMalloc(&vi, N * 4);
  hipMalloc(&vo, N * 4);
  hipMemcpy(in, h.data(), N * 8, hipMemcpyHostToDevice);
  hipMemcpy(vi, hv.data(), N * 4, hipMemcpyHostToDevice);
  using m1 = rocprim::radix_sort_config<rocprim::default_config, rocprim::merge_sort_config<256, 256, 16>, rocprim::default_config>;
  using m2 = rocprim::radix_sort_config<rocprim::default_config, rocprim::merge_sort_config<512, 512, 8>, rocprim::default_config>;
  using m3 = rocprim::radix_sort_config<rocprim::default_config, rocprim::merge_sort_config<1024, 1024, 8>, rocprim::default_config>;
  using m4 = rocprim::radix_sort_config<rocprim::default_config, rocprim::merge_sort_config<256, 512, 16>, rocprim::default_config>;
  for (int n : {6700, 39000, 96000}) {
    printf("keys n=%d: 256x16 %.1f, 512x8 %.1f, 1024x8 %.1f, 512x16 %.1f us\n", n, time_keys<m1>(in, out, n, 27, 48, s),
           time_keys<m2>(in, out, n, 27, 48, s), time_keys<m3>(in, out, n, 27, 48, s), time_keys<m4>(in, out, n, 27, 48, s));
    printf("pairs n=%d: 256x16 %.1f, 512x8 %.1f, 1024x8 %.1f, 512x16 %.1f us\n", n, time_pairs<m1>(in, out, vi, vo, n, 0, 63, s),
           time_pairs<m2>(in, out, vi, vo, n, 0, 63, s), time_pairs<m3>(in, out, vi, vo, n, 0, 63, s), time_pairs<m4>(in, out, vi, vo, n, 0, 63, s));
  }
  for (int n : {6700, 20000, 39000}) {
    printf("keys n=%d bits 27..48: default %.1f us, onesweep %.1f us\n", n,
           time_keys<rocprim::default_config>(in, out, n, 27, 48, s), time_keys<onesweep_cfg>(in, out, n, 27, 48, s));
  }
  for (int nb : {21, 27, 33, 63}) {
    printf("pairs n=96000 bits 0..%d: default %.1f us, onesweep %.1f us\n", nb,
           time_pairs<rocprim::default_config>(in, out, vi, vo, 96000, 0, nb, s),
           time_pairs<onesweep_cfg>(in, out, vi, vo, 96000, 0, nb, s));
  }
  return 0;
}
