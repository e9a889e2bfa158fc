// device_common.hpp — device helpers shared by the HIP kernels: wave64
// reductions, the decoupled look-back tile scan, UTF-8 decoding, the 16-byte
// cached byte reader and the DFA evaluator.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "devcfg.hpp"

namespace ose {

constexpr int kWave = 64;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// ---------------------------------------------------------------------------
// Decoupled look-back (single-pass tile prefix).  Tile ids come from an
// atomic counter taken at block start, so every tile a block waits on was
// already running (no dispatch-order assumption).  Each tile publishes one
// 8-byte granule {status:2 | value:62} with relaxed agent-scope atomics (the
// granule IS the flag: MI355X_MICROARCH.md "R2"); nothing else is handed
// between workgroups.  Status words and the counter are zeroed by a
// hipMemsetAsync before every launch.  Spins are bounded; a timeout sets
// *err bit 0 and the tile proceeds with a wrong prefix (the call fails).
constexpr uint64_t kLbAgg = 1ull << 62;
constexpr uint64_t kLbIncl = 2ull << 62;
constexpr uint64_t kLbVal = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by all 64 lanes of ONE wave; returns the exclusive prefix of `tile`.
__device__ inline uint64_t lookback_prefix(uint64_t* status, uint32_t tile, uint64_t agg, uint32_t* err) {
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0) lb_store(&status[0], kLbIncl | agg);
    return 0;
  }
  if (lane == 0) lb_store(&status[tile], kLbAgg | agg);
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    int64_t idx = base - lane;
    uint64_t v = idx >= 0 ? lb_load(&status[idx]) : kLbIncl;
    uint64_t st = v & ~kLbVal;
    uint64_t incl = __ballot(st == kLbIncl);
    uint64_t inval = __ballot(st == 0);
    int first = incl ? __ffsll((unsigned long long)incl) - 1 : 64;
    uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);
    if (inval & need) {
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t c = lane <= first ? (v & kLbVal) : 0;
    excl += wave_sum_u64(c);
    if (first < 64) break;
    base -= 64;
  }
  if (lane == 0) lb_store(&status[tile], kLbIncl | (excl + agg));
  return excl;
}

// ---------------------------------------------------------------------------
// Byte reader over one string: 16-byte aligned vector loads cached in
// registers.  Strings live in an arena allocated with >= 16 bytes of slack
// and a 16-byte aligned base (ose_columns contract), so the aligned load of
// the last chunk never leaves the allocation.
struct ByteReader {
  const uint8_t* base;
  uint64_t cached = ~0ull;
  uint4 chunk;
  __device__ explicit ByteReader(const uint8_t* b) : base(b) {}
  __device__ __forceinline__ uint32_t at(uint32_t i) {
    uint64_t addr = (uint64_t)(base + i);
    uint64_t al = addr & ~15ull;
    if (al != cached) {
      chunk = *reinterpret_cast<const uint4*>(al);
      cached = al;
    }
    uint32_t o = (uint32_t)(addr & 15);
    uint32_t w = (o & 8) ? ((o & 4) ? chunk.w : chunk.z) : ((o & 4) ? chunk.y : chunk.x);
    return (w >> ((o & 3) * 8)) & 0xFFu;
  }
};

// unicode/utf8.DecodeRune on [i, e): invalid -> (U+FFFD, 1)
__device__ inline uint32_t decode_rune(ByteReader& rd, uint32_t i, uint32_t e, uint32_t& w) {
  uint32_t c = rd.at(i);
  if (c < 0x80) { w = 1; return c; }
  uint32_t need, r, lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { need = 1; r = c & 0x1F; }
  else if (c == 0xE0) { need = 2; r = c & 0x0F; lo = 0xA0; }
  else if (c >= 0xE1 && c <= 0xEC) { need = 2; r = c & 0x0F; }
  else if (c == 0xED) { need = 2; r = c & 0x0F; hi = 0x9F; }
  else if (c >= 0xEE && c <= 0xEF) { need = 2; r = c & 0x0F; }
  else if (c == 0xF0) { need = 3; r = c & 0x07; lo = 0x90; }
  else if (c >= 0xF1 && c <= 0xF3) { need = 3; r = c & 0x07; }
  else if (c == 0xF4) { need = 3; r = c & 0x07; hi = 0x8F; }
  else { w = 1; return 0xFFFD; }
  if (i + need >= e) { w = 1; return 0xFFFD; }
  for (uint32_t k = 1; k <= need; k++) {
    uint32_t b = rd.at(i + k);
    if (b < (k == 1 ? lo : 0x80u) || b > (k == 1 ? hi : 0xBFu)) { w = 1; return 0xFFFD; }
    r = (r << 6) | (b & 0x3F);
  }
  w = need + 1;
  return r;
}

// regexp.MatchString via a compiled DFA (regex_dfa.cpp) over bytes [s, e).
__device__ inline bool dfa_match(const uint8_t* blob, uint32_t dfa_off, ByteReader& rd, uint32_t s, uint32_t e) {
  const DfaDev* d = reinterpret_cast<const DfaDev*>(blob + dfa_off);
  const uint16_t* trans = reinterpret_cast<const uint16_t*>(blob + d->trans_off);
  const uint32_t ncls = d->nclasses, match = d->match;
  uint32_t st = d->start;
  uint32_t i = s;
  while (i < e) {
    if (st == match) return true;
    uint32_t w;
    uint32_t r = decode_rune(rd, i, e, w);
    i += w;
    uint32_t cls;
    if (r < 0x80) {
      cls = d->ascii[r];
    } else {
      const uint32_t* hr = reinterpret_cast<const uint32_t*>(blob + d->hi_off);
      uint32_t lo = 0, hi = d->hi_n;
      cls = 0;
      while (lo < hi) {
        uint32_t m = (lo + hi) >> 1;
        if (r < hr[3 * m]) hi = m;
        else if (r > hr[3 * m + 1]) lo = m + 1;
        else { cls = hr[3 * m + 2]; break; }
      }
    }
    st = trans[st * ncls + cls];
  }
  const uint8_t* acc = blob + d->acc_off;
  return st == match || acc[st];
}

}  // namespace ose
