// diag_kernel.hip — measured HBM bandwidth for the roofline (SURVEY.md §8d
// asks for a stream-copy figure beside the 8 TB/s spec): a 16-byte-per-lane
// grid-stride copy, timed with HIP events on the caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "engine_internal.hpp"

namespace ose {
namespace {
// one 16-byte element per lane, a grid over the whole buffer
__global__ __launch_bounds__(256) void stream_copy_flat_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                               uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  if (i < n16) reinterpret_cast<v4u*>(dst)[i] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + i);
}
__global__ __launch_bounds__(256) void stream_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                          uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // four loads in flight per lane
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}
}  // namespace
}  // namespace ose

using namespace ose;

extern "C" {
// Device-to-device copy of `bytes` (a multiple of 16) `reps` times; *gbps =
// (read + written bytes) / average kernel time.  Diagnostics for bench.py.
int osehost_stream_copy(void* dst, const void* src, size_t bytes, int reps, void* hip_stream, double* gbps) {
  if (!dst || !src || !gbps || bytes % 16 || reps < 1) return fail(OSE_EINVAL, "bad argument");
  int rc = ensure_device();
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  const uint64_t n16 = bytes / 16;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, (uint64_t)cus * 16);
  if ((n16 + 255) / 256 > 0x7FFFFFFFull) return fail(OSE_ERANGE, "buffer too large");
  const uint32_t flat_blocks = (uint32_t)((n16 + 255) / 256);
  hipEvent_t a = nullptr, b = nullptr;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return fail(OSE_EDEVICE, "hipEventCreate failed");
  double best = 0;
  // two shapes (grid-stride with four loads in flight per lane; one element
  // per lane over a grid of the whole buffer): the faster one is reported
  for (int shape = 0; shape < 2; shape++) {
    auto launch = [&] {
      if (shape == 0)
        hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(256), 0, st, static_cast<uint4*>(dst),
                           static_cast<const uint4*>(src), n16);
      else
        hipLaunchKernelGGL(stream_copy_flat_kernel, dim3(flat_blocks), dim3(256), 0, st, static_cast<uint4*>(dst),
                           static_cast<const uint4*>(src), n16);
    };
    launch();   // warm-up
    (void)hipEventRecord(a, st);
    for (int r = 0; r < reps; r++) launch();
    (void)hipEventRecord(b, st);
    float ms = 0;
    const hipError_t e = hipEventSynchronize(b);
    if (e == hipSuccess) (void)hipEventElapsedTime(&ms, a, b);
    if (e != hipSuccess || ms <= 0) {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
      return fail(OSE_EDEVICE, "stream copy timing failed");
    }
    best = std::max(best, 2.0 * (double)bytes * reps / (ms * 1e-3) / 1e9);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *gbps = best;
  return 0;
}
}  // extern "C"
