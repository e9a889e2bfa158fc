// size_device.hpp — the per-span part of odigostrafficmetrics' size
// (odigostrafficmetrics/processor.go:71-84 via ptrace.ProtoMarshaler.
// ResourceSpansSize): the framed size of one surviving span after the
// earlier gateway stages, summed per scope.  Shared by size_span_kernel
// (size_kernel.hip) and url_copy_kernel (url_kernel.hip), which runs the
// same pass fused when TEMPLATE and SIZE are in one call.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"

namespace ose {
namespace sizedev {

__device__ __forceinline__ uint32_t sov(uint64_t x) {
  // varint length: 1 + floor(log2(x|1) / 7)
  return 1u + (uint32_t)((63 - __clzll((long long)(x | 1))) / 7);
}
__device__ __forceinline__ uint64_t field_len(uint64_t l) { return 1 + sov(l) + l; }

// The per-scope and per-resource sums carry a count in their top bits: the
// byte sum in the low kSumBits (a batch's arena offsets are 32-bit, so no
// scope or resource body reaches 2^40 bytes) and, above it, the number of
// runs that added to a scope (> 0: the scope had spans) or of alive scopes
// a resource holds -- one atomic per run instead of a sum and a flag.
constexpr uint32_t kSumBits = 40;
constexpr uint64_t kSumMask = (1ull << kSumBits) - 1;

// One DPP step of the segmented sum: (h, v, c) elements, earlier + later =
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
// Segmented (by non-decreasing key) inclusive sums over one wave; returns
// true on the lane that ends its key's run inside the wave.
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

// the columns of one span
struct SpanCols {
  uint32_t s, kept, span_size, tl, old;
  uint8_t u, kd;
  bool valid;
};
// every column is loaded up front, whatever keep and url_out say: one
// memory round trip instead of three dependent ones (the pass is
// latency-bound; the extra bytes of dropped/untemplated spans are cheap).
// tl: the template length (tmpl[i].len, or the plan length in url_copy).
__device__ __forceinline__ SpanCols size_span_load(const SizeKernelArgs& a, uint64_t i, bool with_tmpl = true) {
  SpanCols x{};
  x.valid = i < a.n_spans;
  if (x.valid) {
    x.s = a.scope[i];
    x.kept = a.sampled ? a.keep[i] : 1u;
    x.span_size = a.span_size[i];
    if (a.templated) {
      x.u = a.url_out[i];
      if (with_tmpl) x.tl = a.tmpl[i].len;
      x.kd = a.kind[i];
      x.old = a.name_len[i];
    }
  }
  return x;
}

// the span's framed size into its scope's sums (one atomic per scope run of
// the wave; plain stores for the scopes that lie inside one wave measured
// slower, C4 url_copy 0.81 -> 1.51 ms: profiles/r4u_size_plain_stores_ab.txt);
// returns 1 when the span survives
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
  // a scope keeps a span iff its body sum is non-zero (a kept span adds its
  // framed size, >= 2 bytes): no per-scope kept count (C4 url_copy 0.80 ->
  // 0.77 ms, profiles/r4za_size_nokept_ab.txt); "had spans" is the run count
  // in the sum's top bits (one atomic per run; an atomic OR on a flag word
  // beside it before)
  if (tail) atomicAdd((unsigned long long*)&a.scope_body[s], (unsigned long long)(v + (1ull << kSumBits)));
  return x.valid ? x.kept : 0u;
}

__device__ __forceinline__ bool size_batch_dropped(const SizeKernelArgs& a) {
  return a.batch_keep && __hip_atomic_load(a.batch_keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

}  // namespace sizedev
}  // namespace ose
