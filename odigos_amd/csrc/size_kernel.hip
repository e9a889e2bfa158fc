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

namespace ose {
namespace {

constexpr int kSThreads = 256;
constexpr uint32_t kLdsAttrsets = 2048;   // attribute sets privatised in LDS (16 KiB of int64)

__device__ __forceinline__ uint32_t sov(uint64_t x) {
  // varint length: 1 + floor(log2(x|1) / 7)
  return 1u + (uint32_t)((63 - __clzll((long long)(x | 1))) / 7);
}
__device__ __forceinline__ uint64_t field_len(uint64_t l) { return 1 + sov(l) + l; }

__device__ __forceinline__ bool batch_dropped(const SizeKernelArgs& a) {
  return a.batch_keep && __hip_atomic_load(a.batch_keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

// Segmented (by non-decreasing key) inclusive sums over one wave; returns
// true on the lane that ends its key's run inside the wave.
// One DPP step of the segmented sum: (h, v, c) elements, earlier ⊕ later =
// (h_e | h_l, h_l ? (v_l, c_l) : (v_e + v_l, c_e + c_l)); a source lane
// outside the row yields the identity (0, 0, 0).
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_sum_step(uint32_t& h, uint64_t& v, uint32_t& c) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h), oc = dpp_mov<CTRL, ROWS>(0u, c);
  const uint64_t ov = dpp_mov64<CTRL, ROWS>(0ull, v);
  if (!h) {
    v += ov;
    c += oc;
  }
  h |= oh;
}
template <typename T>
__device__ __forceinline__ bool wave_seg_sum(uint32_t key, bool valid, T& v, uint32_t& c) {
  const int lane = threadIdx.x & 63;
  const uint64_t vmask = __ballot(valid);
  // neighbours' keys by DPP wave_shl:1 / wave_shr:1 (every lane takes them)
  const uint32_t nk = dpp_mov<0x130>(key, key);
  const uint32_t pk = dpp_mov<0x138>(key, key);
  const bool last = valid && (lane == 63 || !((vmask >> (lane + 1)) & 1) || nk != key);
  // lanes whose key differs from lane-1's start a run; invalid lanes are runs of their own
  const uint32_t h = valid ? ((lane == 0 || pk != key) ? 1u : 0u) : 1u;
  uint64_t w = v;
  uint32_t hh = h;
  seg_sum_step<0x111, 0xF>(hh, w, c);
  seg_sum_step<0x112, 0xF>(hh, w, c);
  seg_sum_step<0x114, 0xF>(hh, w, c);
  seg_sum_step<0x118, 0xF>(hh, w, c);
  seg_sum_step<0x142, 0xA>(hh, w, c);
  seg_sum_step<0x143, 0xC>(hh, w, c);
  v = (T)w;
  return last;
}

struct SpanCols {
  uint32_t s, kept, span_size, tl, old;
  uint8_t u, kd;
  bool valid;
};
__device__ __forceinline__ SpanCols size_span_load(const SizeKernelArgs& a, uint64_t i);
__device__ __forceinline__ uint32_t size_span_finish(const SizeKernelArgs& a, const SpanCols& x);

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

__device__ __forceinline__ SpanCols size_span_load(const SizeKernelArgs& a, uint64_t i) {
  // every column is loaded up front, whatever keep and url_out say: one
  // memory round trip per tile instead of three dependent ones (the kernel
  // is latency-bound; the extra bytes of dropped/untemplated spans are cheap)
  SpanCols x{};
  x.valid = i < a.n_spans;
  if (x.valid) {
    x.s = a.scope[i];
    x.kept = a.sampled ? a.keep[i] : 1u;
    x.span_size = a.span_size[i];
    if (a.templated) {
      x.u = a.url_out[i];
      x.tl = a.tmpl[i].len;
      x.kd = a.kind[i];
      x.old = a.name_len[i];
    }
  }
  return x;
}

__device__ __forceinline__ uint32_t size_span_finish(const SizeKernelArgs& a, const SpanCols& x) {
  uint64_t contrib = 0;
  if (x.valid && x.kept) {
    uint64_t sz = x.span_size;
    const uint64_t tl = x.tl;
    if (x.u & OSE_OUT_SET_ATTR) {   // PutStr(http.route | url.template, tmpl): one more KeyValue
      const uint64_t keylen = x.kd == OSE_KIND_CLIENT ? 12 : 10;
      sz += field_len(field_len(keylen) + field_len(field_len(tl)));
    }
    if (x.u & OSE_OUT_RENAME) {     // SetName(method + " " + tmpl), old name == method
      const uint64_t old = x.old;
      sz += field_len(old + 1 + tl) - (old ? field_len(old) : 0);
    }
    contrib = field_len(sz);
  }
  uint64_t v = contrib;
  uint32_t c = x.valid ? x.kept : 0u;
  const uint32_t s = x.s;
  const bool tail = wave_seg_sum(s, x.valid, v, c);
  if (tail) {
    if (v) atomicAdd((unsigned long long*)&a.scope_body[s], (unsigned long long)v);
    if (c) atomicAdd(&a.scope_kept[s], c);
    a.scope_had[s] = 1;
  }
  return x.valid ? x.kept : 0u;
}

__global__ __launch_bounds__(kSThreads) void size_scope_kernel(SizeKernelArgs a) {
  if (batch_dropped(a)) return;
  const uint32_t s = blockIdx.x * kSThreads + threadIdx.x;
  const bool valid = s < a.n_scopes;
  uint32_t r = 0, alive = 0, had = 0;
  uint64_t contrib = 0;
  if (valid) {
    r = a.scope_resource[s];
    had = a.scope_had[s];
    alive = !a.remove_empty || !had || a.scope_kept[s];   // an emptied ScopeSpans is removed
    if (alive) contrib = field_len((uint64_t)a.scope_size[s] + a.scope_body[s]);
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
  if (tail) {
    if (v) atomicAdd((unsigned long long*)&a.res_body[r], (unsigned long long)v);
    if (c) atomicAdd(&a.res_alive[r], c);
    if (h) a.res_had[r] = 1;
  }
}

__global__ __launch_bounds__(kSThreads) void size_res_kernel(SizeKernelArgs a) {
  if (batch_dropped(a)) {   // nothing survived: every ResourceSpans is 0 bytes
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
    const bool removed = a.remove_empty && a.res_had[r] && !a.res_alive[r];
    const uint64_t size = removed ? 0 : (uint64_t)a.res_size[r] + a.res_body[r];
    if (a.res_bytes) a.res_bytes[r] = size;
    if (removed) continue;
    const long long add = (long long)size * a.inverse;
    const uint32_t set = a.res_attrset[r];
    if (lds) atomicAdd(&hist[set], (unsigned long long)add);
    else atomicAdd((unsigned long long*)&a.attrset_bytes[set], (unsigned long long)add);
  }
  if (!lds) return;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < a.n_attrsets; k += kSThreads)
    if (hist[k]) atomicAdd((unsigned long long*)&a.attrset_bytes[k], hist[k]);
}

}  // namespace

void launch_size_spans(const SizeKernelArgs& a, hipStream_t st) {
  static const uint64_t cap = [] {
    const char* g = getenv("OSE_SIZE_GRID");   // tuning
    return g ? std::max<uint64_t>(1, strtoull(g, nullptr, 0)) : 1024ull;   // swept on C4: 512 0.127 ms, 1024 0.088, 2048 0.094, 8192 0.126
  }();
  const uint64_t blocks = std::min<uint64_t>((a.n_spans + kSThreads - 1) / kSThreads, cap);
  if (blocks) hipLaunchKernelGGL(size_span_kernel, dim3((uint32_t)blocks), dim3(kSThreads), 0, st, a);
}
void launch_size_scopes(const SizeKernelArgs& a, hipStream_t st) {
  const uint32_t blocks = (a.n_scopes + kSThreads - 1) / kSThreads;
  if (blocks) hipLaunchKernelGGL(size_scope_kernel, dim3(blocks), dim3(kSThreads), 0, st, a);
}
void launch_size_resources(const SizeKernelArgs& a, hipStream_t st) {
  static const uint32_t per_thread = [] {
    const char* g = getenv("OSE_SIZE_RES_PER_THREAD");   // tuning
    return g ? std::max<uint32_t>(1, (uint32_t)strtoul(g, nullptr, 0)) : 16u;   // swept on C4: 4 0.058 ms, 16 0.044, 32 0.058, 64 0.102
  }();
  uint32_t blocks = (a.n_resources + kSThreads * per_thread - 1) / (kSThreads * per_thread);
  if (blocks > 2048) blocks = 2048;
  if (blocks) hipLaunchKernelGGL(size_res_kernel, dim3(blocks), dim3(kSThreads), 0, st, a);
}

}  // namespace ose
