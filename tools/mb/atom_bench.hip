// same-address returning 64-bit atomicAdd throughput: W waves, each K atomics from lane 0
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
__global__ void k(unsigned long long* p, int K, unsigned long long* sink) {
  unsigned long long acc = 0;
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < K; i++) acc += atomicAdd(p, 1024ull);
  if (acc == 0x123456789ull) sink[0] = acc;
}
__global__ void k_spread(unsigned long long* p, int K, unsigned long long* sink) {
  unsigned long long acc = 0;
  const int w = (blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) & 63;
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < K; i++) acc += atomicAdd(p + 32 * w, 1024ull);
  if (acc == 0x123456789ull) sink[0] = acc;
}
int main() {
  unsigned long long *p, *s;
  hipMalloc(&p, 1 << 16); hipMalloc(&s, 64); hipMemset(p, 0, 1 << 16);
  for (int spread = 0; spread < 2; spread++)
  for (int blocks : {1024, 4096, 16384}) {
    for (int K : {1, 4, 16}) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      if (spread) k_spread<<<blocks, 256>>>(p, K, s); else k<<<blocks, 256>>>(p, K, s);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 5; r++) { if (spread) k_spread<<<blocks, 256>>>(p, K, s); else k<<<blocks, 256>>>(p, K, s); }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
      const double n = (double)blocks * 4 * K;
      printf("%s blocks %6d K %3d atomics %9.0f  %8.3f ms  %6.2f ns/atomic\n", spread ? "64 addrs" : "1 addr  ", blocks, K, n, ms, ms * 1e6 / n);
    }
  }
  return 0;
}
