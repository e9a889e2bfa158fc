// size_kernel.hip — odigostrafficmetrics on CDNA4 (gfx950).
//
// Replaces dataSizesMetricsProcessor.processTraces (odigostrafficmetrics/
// processor.go:71-84): per surviving ResourceSpans, its protobuf wire size
// (ptrace.ProtoMarshaler.ResourceSpansSize, pdata v1.47.0) times
// inverseSamplingFraction, added to the counter of its resource attribute
// set, and the surviving span count.  The host sizes the immutable parts of
// each message once when it columnarises (span_size, scope_size, res_size);
// the GPU adds what the earlier gateway stages changed — spans dropped by
// odigossampling, the attribute and name odigosurltemplate wrote — and the
// length framing of every level, which depends on the final sizes:
//   K1 spans     framed span sizes, wave-segmented by scope  -> scope sums
//   K2 scopes    framed scope sizes, segmented by resource   -> resource sums
//   K3 resources ResourceSpans sizes x inverse -> LDS-privatised attribute-set
//                histogram -> one global atomic per non-empty bin per block
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "device_common.hpp"
#include "kernels.hpp"
#include "size_device.hpp"

namespace ose {
namespace {

using namespace sizedev;
constexpr int kSThreads = 256;
constexpr uint32_t kLdsAttrsets = 2048;   // attribute sets privatised in LDS (16 KiB of int64)

__device__ __forceinline__ bool batch_dropped(const SizeKernelArgs& a) { return size_batch_dropped(a); }

// Grid-stride over 256-span tiles (a capped grid: the surviving-span count
// is reduced per block and added with ONE atomic per block — a per-wave
// atomic on that single word serialises at the memory side).
__global__ __launch_bounds__(kSThreads) void size_span_kernel(SizeKernelArgs a) {
  if (batch_dropped(a)) return;
  __shared__ uint32_t wk[kSThreads / kWave];
  uint32_t kept_total = 0;
  // two tiles per iteration: both tiles' loads are in flight together
  const uint64_t stride = (uint64_t)gridDim.x * kSThreads;
  for (uint64_t base = (uint64_t)blockIdx.x * kSThreads; base < a.n_spans; base += 2 * stride) {
    const SpanCols x0 = size_span_load(a, base + threadIdx.x);
    const SpanCols x1 = size_span_load(a, base + stride + threadIdx.x);
    kept_total += size_span_finish(a, x0);
    if (base + stride < a.n_spans) kept_total += size_span_finish(a, x1);   // wave-uniform
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kept_total += __shfl_xor(kept_total, o, kWave);
  if ((threadIdx.x & 63) == 0) wk[threadIdx.x >> 6] = kept_total;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t k = 0;
    for (int w = 0; w < kSThreads / kWave; w++) k += wk[w];
    if (k) atomicAdd((unsigned long long*)a.accepted, (unsigned long long)k);
  }
}

__global__ __launch_bounds__(kSThreads) void size_scope_kernel(SizeKernelArgs a) {
  if (batch_dropped(a)) return;
  const uint32_t s = blockIdx.x * kSThreads + threadIdx.x;
  const bool valid = s < a.n_scopes;
  uint32_t r = 0, alive = 0, had = 0;
  uint64_t contrib = 0;
  if (valid) {
    r = a.scope_resource[s];
    const uint64_t sb = a.scope_body[s];
    const uint64_t body = sb & kSumMask;
    had = (sb >> kSumBits) != 0;   // some run of spans added to it
    alive = !a.remove_empty || !had || body != 0;   // an emptied ScopeSpans is removed
    if (alive) contrib = field_len((uint64_t)a.scope_size[s] + body);
  }
  uint64_t v = contrib;
  uint32_t c = alive;
  const bool tail = wave_seg_sum(r, valid, v, c);
  // any scope of the run had spans: OR over the run == (run's had bits != 0)
  // (keys are non-decreasing: the run is lanes [its head, this lane]; two
  // ballots and a bit search instead of a 6-step shuffle scan)
  const int lane = threadIdx.x & 63;
  const uint32_t pr = dpp_mov<0x138>(r, r);   // lane - 1's key (wave_shr:1)
  const uint64_t heads = __ballot(lane == 0 || pr != r);
  const uint64_t hadm = __ballot(had != 0);
  const uint64_t upto = ~0ull >> (63 - lane);
  const int start = 63 - __clzll((long long)(heads & upto));   // lane 0 is always a head
  const uint32_t h = (hadm & upto & (~0ull << start)) ? 1u : 0u;
  // (plain stores for the runs inside a wave measured slower: C4 0.23 ->
  // 0.32 ms; these atomics resolve in L2)
  if (tail) {   // the body sum and the alive scopes' count in one word (kSumBits)
    if (v | c) atomicAdd((unsigned long long*)&a.res_body[r], (unsigned long long)(v + ((uint64_t)c << kSumBits)));
    if (h) a.res_had[r] = 1;
  }
}

__global__ __launch_bounds__(kSThreads) void size_res_kernel(SizeKernelArgs a) {
  if (batch_dropped(a)) {   // nothing survived: every ResourceSpans is 0 bytes (and no span is counted)
    if (a.res_bytes)
      for (uint32_t r = blockIdx.x * kSThreads + threadIdx.x; r < a.n_resources; r += gridDim.x * kSThreads) a.res_bytes[r] = 0;
    return;
  }
  __shared__ unsigned long long hist[kLdsAttrsets];   // two's-complement sums
  const bool lds = a.n_attrsets <= kLdsAttrsets;
  if (lds)
    for (uint32_t k = threadIdx.x; k < a.n_attrsets; k += kSThreads) hist[k] = 0;
  __syncthreads();
  for (uint32_t r = blockIdx.x * kSThreads + threadIdx.x; r < a.n_resources; r += gridDim.x * kSThreads) {
    const uint64_t rb = a.res_body[r];
    const bool removed = a.remove_empty && a.res_had[r] && (rb >> kSumBits) == 0;   // no alive scope left
    const uint64_t size = removed ? 0 : (uint64_t)a.res_size[r] + (rb & kSumMask);
    if (a.res_bytes) a.res_bytes[r] = size;
    if (removed) continue;
    const long long add = (long long)size * a.inverse;
    const uint32_t set = a.res_attrset[r];
    if (lds) atomicAdd(&hist[set], (unsigned long long)add);
    else atomicAdd((unsigned long long*)&a.attrset_bytes[set], (unsigned long long)add);
  }
  if (a.kept_partials) {   // the surviving spans counted per block by url_copy_kernel (fused spans pass)
    uint32_t k = 0;
    for (uint32_t b = blockIdx.x * kSThreads + threadIdx.x; b < a.n_kept_partials; b += gridDim.x * kSThreads)
      k += a.kept_partials[b];
    __shared__ uint32_t wk[kSThreads / kWave];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o, kWave);
    if ((threadIdx.x & 63) == 0) wk[threadIdx.x >> 6] = k;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kSThreads / kWave; w++) t += wk[w];
      if (t) atomicAdd((unsigned long long*)a.accepted, (unsigned long long)t);
    }
  }
  if (!lds) return;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < a.n_attrsets; k += kSThreads)
    if (hist[k]) atomicAdd((unsigned long long*)&a.attrset_bytes[k], hist[k]);
}

}  // namespace

void launch_size_spans(const SizeKernelArgs& a, hipStream_t st) {
  constexpr uint64_t cap = 1024;   // swept on C4: 512 0.127 ms, 1024 0.088, 2048 0.094, 8192 0.126
  const uint64_t blocks = std::min<uint64_t>((a.n_spans + kSThreads - 1) / kSThreads, cap);
  if (blocks) hipLaunchKernelGGL(size_span_kernel, dim3((uint32_t)blocks), dim3(kSThreads), 0, st, a);
}
void launch_size_scopes(const SizeKernelArgs& a, hipStream_t st) {
  const uint32_t blocks = (a.n_scopes + kSThreads - 1) / kSThreads;
  if (blocks) hipLaunchKernelGGL(size_scope_kernel, dim3(blocks), dim3(kSThreads), 0, st, a);
}
void launch_size_resources(const SizeKernelArgs& a, hipStream_t st) {
  if (!a.n_resources && !a.kept_partials) return;
  constexpr uint32_t per_thread = 16;   // swept on C4: 4 0.058 ms, 16 0.044, 32 0.058, 64 0.102
  uint32_t blocks = (a.n_resources + kSThreads * per_thread - 1) / (kSThreads * per_thread);
  if (a.kept_partials) blocks = std::max<uint32_t>(blocks, std::min<uint32_t>(64, (a.n_kept_partials + 4095) / 4096));
  if (blocks > 2048) blocks = 2048;
  if (blocks) hipLaunchKernelGGL(size_res_kernel, dim3(blocks), dim3(kSThreads), 0, st, a);
}

}  // namespace ose
