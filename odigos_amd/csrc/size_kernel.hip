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

// One ResourceSpans finished: its size (ptrace ResourceSpansSize: the fixed
// part the host sized plus the framed scopes that survive), 0 when the
// emptied resource is removed, into res_bytes and, times inverse, into its
// attribute set's sum (LDS when the sets fit, else global).
__device__ __forceinline__ void size_finish_res(const SizeKernelArgs& a, unsigned long long* hist, bool lds, uint32_t r,
                                                uint64_t body, uint32_t alive, bool had, uint32_t rsz, uint32_t set) {
  const bool removed = a.remove_empty && had && alive == 0;   // no alive scope left
  const uint64_t size = removed ? 0 : (uint64_t)rsz + body;
  if (a.res_bytes) a.res_bytes[r] = size;
  if (removed) return;
  const long long add = (long long)size * a.inverse;
  if (lds) atomicAdd(&hist[set], (unsigned long long)add);
  else atomicAdd((unsigned long long*)&a.attrset_bytes[set], (unsigned long long)add);
}

// K2+K3 in one pass over the scopes (replaces a scopes pass whose per-run
// atomics summed into per-resource words, a zeroing of those words and a
// resources pass that read them back).  A 64-scope window's lanes take its
// scopes; a wave-segmented sum by resource gives every resource run of the
// window its framed body bytes, alive scopes and whether any scope had
// spans.  A run whose resource has no scope outside the window is finished
// at its tail lane; the window's first and last runs (the only ones that can
// reach into a neighbour) are also written to the window's two part slots,
// and a window holding the end of a run that began earlier is flagged for
// size_fix_kernel.  Resources without scopes (the gaps between consecutive
// runs' resources, and those after the last scope) are finished by the lane
// that sees the gap.  Grid-stride over 256-scope tiles, the attribute-set
// sums privatised in LDS per block.
__global__ __launch_bounds__(kSThreads) void size_tail_kernel(SizeKernelArgs a) {
  __shared__ unsigned long long hist[kLdsAttrsets];   // two's-complement sums
  __shared__ uint32_t wk[kSThreads / kWave];
  const bool lds = a.n_attrsets <= kLdsAttrsets;
  const int lane = threadIdx.x & 63;
  const uint64_t gstride = (uint64_t)gridDim.x * kSThreads;
  if (batch_dropped(a)) {   // nothing survived: every ResourceSpans is 0 bytes (and no span is counted)
    if (a.res_bytes)
      for (uint64_t r = (uint64_t)blockIdx.x * kSThreads + threadIdx.x; r < a.n_resources; r += gstride) a.res_bytes[r] = 0;
    return;
  }
  if (lds)
    for (uint32_t k = threadIdx.x; k < a.n_attrsets; k += kSThreads) hist[k] = 0;
  __syncthreads();
  const uint32_t S = a.n_scopes, R = a.n_resources;
  if (S == 0) {   // no scopes: every resource keeps its fixed size
    for (uint64_t r = (uint64_t)blockIdx.x * kSThreads + threadIdx.x; r < R; r += gstride)
      size_finish_res(a, hist, lds, (uint32_t)r, 0, 0, false, a.res_size[r], a.res_attrset[r]);
  }
  for (uint64_t t0 = (uint64_t)blockIdx.x * kSThreads; t0 < S; t0 += gstride) {
    const uint64_t s = t0 + threadIdx.x;
    const uint64_t s0 = s - lane;                      // the window's first scope
    const bool valid = s < S;
    uint32_t r = 0xFFFFFFFFu, alive = 0, had = 0;
    uint64_t contrib = 0;
    uint32_t nb = 0xFFFFFFFFu;                         // lane 0: the scope before the window's resource
    if (valid) {
      r = a.scope_resource[s];
      const uint64_t sb = a.scope_body[s];
      const uint64_t body = sb & kSumMask;
      had = (sb >> kSumBits) != 0;                     // some run of spans added to it
      alive = !a.remove_empty || !had || body != 0;    // an emptied ScopeSpans is removed
      if (alive) contrib = field_len((uint64_t)a.scope_size[s] + body);
      if (lane == 0 && s > 0) nb = a.scope_resource[s - 1];
    }
    // the resource's fixed size and attribute set, read with the scope's
    // columns (a run's tail lane finishes its own resource)
    uint32_t rsz = 0, rset = 0;
    if (valid) {
      rsz = a.res_size[r];
      rset = a.res_attrset[r];
    }
    const uint64_t vmask = __ballot(valid);            // window lanes [0, lastv]
    if (!vmask) continue;                              // a window past the last scope (wave-uniform)
    const int lastv = 63 - __clzll((long long)vmask);
    uint32_t na = 0xFFFFFFFFu;                         // lane lastv: the scope after the window's resource
    if (lane == lastv && s + 1 < S) na = a.scope_resource[s + 1];
    uint64_t v = contrib;
    uint32_t c = alive;
    const bool tail = wave_seg_sum(r, valid, v, c);
    const uint32_t pr = dpp_mov<0x138>(r, r);          // lane - 1's resource (wave_shr:1)
    const bool head = valid && (lane == 0 || pr != r);
    const uint64_t heads = __ballot(head);
    const uint64_t hadm = __ballot(had != 0);
    const uint64_t upto = ~0ull >> (63 - lane);
    const int start = 63 - __clzll((long long)(heads & upto));   // this lane's run head (lane 0 is a head)
    const uint32_t h = (hadm & upto & (~0ull << start)) ? 1u : 0u;
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(r);
    const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)r, lastv);
    const uint32_t before = __builtin_amdgcn_readfirstlane(nb);
    const uint32_t after = (uint32_t)__builtin_amdgcn_readlane((int)na, lastv);
    const bool whole_head = s0 == 0 || before != r0;   // the window's first run starts in it
    const bool whole_tail = s0 + lastv + 1 >= S || after != rl;   // its last run ends in it
    const int end0 = __builtin_ctzll(__ballot(tail));  // the first run's tail lane
    const bool single = end0 == lastv;
    // runs with a side outside the window: the first (head missing), the last (tail missing)
    const bool cut = tail && ((start == 0 && !whole_head) || (lane == lastv && !whole_tail));
    if (tail && !cut) size_finish_res(a, hist, lds, r, v, c, h != 0, rsz, rset);
    if (valid && head) {
      // resources with no scope between the previous run's and this one
      const uint32_t prev = lane ? pr : (s0 == 0 ? 0xFFFFFFFFu : before);
      for (uint32_t g = prev + 1; g < r; g++) size_finish_res(a, hist, lds, g, 0, 0, false, a.res_size[g], a.res_attrset[g]);
    }
    if (valid && s + 1 == S)   // resources after the last scope
      for (uint32_t g = r + 1; g < R; g++) size_finish_res(a, hist, lds, g, 0, 0, false, a.res_size[g], a.res_attrset[g]);
    // the window's part slots and fix flag
    const uint64_t w = s0 >> 6;
    const uint32_t ch0 = (uint32_t)__builtin_amdgcn_readlane((int)(c | (h << 30)), end0);
    const uint64_t v0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), end0) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, end0);
    const uint32_t chl = (uint32_t)__builtin_amdgcn_readlane((int)(c | (h << 30)), lastv);
    const uint64_t vl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lastv) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lastv);
    if (lane == 0 && valid) {
      a.parts[2 * w] = SizePart{r0, ch0 | (whole_head ? 1u << 31 : 0u), v0};
      a.parts[2 * w + 1] = SizePart{rl, chl | (whole_tail ? 1u << 31 : 0u), vl};
      // a run that began in an earlier window ends here
      a.fix[w] = (!whole_head && (!single || whole_tail)) ? 1u : 0u;
    }
  }
  if (a.kept_partials) {   // the surviving spans counted per block by url_copy_kernel (fused spans pass)
    uint32_t k = 0;
    for (uint32_t b = blockIdx.x * kSThreads + threadIdx.x; b < a.n_kept_partials; b += gridDim.x * kSThreads)
      k += a.kept_partials[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o, kWave);
    if (lane == 0) wk[threadIdx.x >> 6] = k;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int q = 0; q < kSThreads / kWave; q++) t += wk[q];
      if (t) atomicAdd((unsigned long long*)a.accepted, (unsigned long long)t);
    }
  }
  if (!lds) return;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < a.n_attrsets; k += kSThreads)
    if (hist[k]) atomicAdd((unsigned long long*)&a.attrset_bytes[k], hist[k]);
}

// The resources whose scopes span windows: from the window holding a run's
// end, its head part there plus the last-run parts of the windows before it
// (walking back while a window is that run alone), finished with global
// atomics.  A handful per batch (one per resource run that crosses a window
// edge).
__global__ __launch_bounds__(kSThreads) void size_fix_kernel(SizeKernelArgs a) {
  const uint64_t w = (uint64_t)blockIdx.x * kSThreads + threadIdx.x;
  if (w >= a.n_swin || !a.fix[w] || size_batch_dropped(a)) return;
  const SizePart hp = a.parts[2 * w];
  const uint32_t r = hp.r;
  uint64_t body = hp.v;
  uint32_t alive = hp.ch & 0x3FFFFFFFu;
  bool had = (hp.ch >> 30) & 1u;
  for (uint64_t k = w; k-- > 0;) {
    const SizePart lp = a.parts[2 * k + 1];            // window k's last run: this resource's
    body += lp.v;
    alive += lp.ch & 0x3FFFFFFFu;
    had |= (lp.ch >> 30) & 1u;
    const SizePart fp = a.parts[2 * k];
    // window k is this run alone and the run began before it: keep walking
    if (fp.r != r || (fp.ch >> 31)) break;
  }
  size_finish_res(a, nullptr, false, r, body, alive, had, a.res_size[r], a.res_attrset[r]);
}
}  // namespace

void launch_size_spans(const SizeKernelArgs& a, hipStream_t st) {
  constexpr uint64_t cap = 1024;   // swept on C4: 512 0.127 ms, 1024 0.088, 2048 0.094, 8192 0.126
  const uint64_t blocks = std::min<uint64_t>((a.n_spans + kSThreads - 1) / kSThreads, cap);
  if (blocks) hipLaunchKernelGGL(size_span_kernel, dim3((uint32_t)blocks), dim3(kSThreads), 0, st, a);
}
void launch_size_tail(const SizeKernelArgs& a, hipStream_t st) {
  // grid-stride over 256-scope tiles (fewer per-block attribute-set flushes)
  uint64_t blocks = ((uint64_t)a.n_scopes + kSThreads - 1) / kSThreads;
#ifndef OSE_SIZE_TAIL_CAP
#define OSE_SIZE_TAIL_CAP 4096
#endif
  if (blocks > OSE_SIZE_TAIL_CAP) blocks = OSE_SIZE_TAIL_CAP;
  if (a.kept_partials) blocks = std::max<uint64_t>(blocks, std::min<uint32_t>(64, (a.n_kept_partials + 4095) / 4096));
  if (!blocks && a.n_resources) blocks = std::min<uint64_t>(((uint64_t)a.n_resources + kSThreads - 1) / kSThreads, 1024);
  if (blocks) hipLaunchKernelGGL(size_tail_kernel, dim3((uint32_t)blocks), dim3(kSThreads), 0, st, a);
}
void launch_size_fix(const SizeKernelArgs& a, hipStream_t st) {
  if (a.n_swin) hipLaunchKernelGGL(size_fix_kernel, dim3((a.n_swin + kSThreads - 1) / kSThreads), dim3(kSThreads), 0, st, a);
}

}  // namespace ose
