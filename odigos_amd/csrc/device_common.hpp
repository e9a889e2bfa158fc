// device_common.hpp — device helpers shared by the HIP kernels: wave64
// reductions, the decoupled look-back tile scan, UTF-8 decoding, the 16-byte
// cached byte reader and the DFA evaluator.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "devcfg.hpp"

#ifndef OSE_LDS_WORD1
#define OSE_LDS_WORD1 0
#endif

namespace ose {

constexpr int kWave = 64;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// DPP wave64 scans and reductions (gfx9 row_shr / row_bcast): register-only,
// no ds_bpermute round trip through the LDS pipeline per step.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t old, uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint64_t dpp_mov64(uint64_t old, uint64_t x) {
  return (uint64_t)dpp_mov<CTRL, ROWS>((uint32_t)old, (uint32_t)x) |
         ((uint64_t)dpp_mov<CTRL, ROWS>((uint32_t)(old >> 32), (uint32_t)(x >> 32)) << 32);
}
// inclusive prefix sum over the wave's lanes
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t x) {
  x += dpp_mov<0x111>(0, x);   // row_shr:1
  x += dpp_mov<0x112>(0, x);   // row_shr:2
  x += dpp_mov<0x114>(0, x);   // row_shr:4
  x += dpp_mov<0x118>(0, x);   // row_shr:8
  x += dpp_mov<0x142, 0xA>(0, x);   // row_bcast:15 into rows 1, 3
  x += dpp_mov<0x143, 0xC>(0, x);   // row_bcast:31 into rows 2, 3
  return x;
}
__device__ __forceinline__ uint32_t lane_value(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
// wave-uniform min / max (lanes 15, 31, 47, 63 hold their row's after the row_shr steps)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  x = min(x, dpp_mov<0x111>(x, x));
  x = min(x, dpp_mov<0x112>(x, x));
  x = min(x, dpp_mov<0x114>(x, x));
  x = min(x, dpp_mov<0x118>(x, x));
  return min(min(lane_value(x, 15), lane_value(x, 31)), min(lane_value(x, 47), lane_value(x, 63)));
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t x) {
  x |= dpp_mov<0x111>(0u, x);
  x |= dpp_mov<0x112>(0u, x);
  x |= dpp_mov<0x114>(0u, x);
  x |= dpp_mov<0x118>(0u, x);
  return lane_value(x, 15) | lane_value(x, 31) | lane_value(x, 47) | lane_value(x, 63);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
  x = max(x, dpp_mov<0x111>(x, x));
  x = max(x, dpp_mov<0x112>(x, x));
  x = max(x, dpp_mov<0x114>(x, x));
  x = max(x, dpp_mov<0x118>(x, x));
  return max(max(lane_value(x, 15), lane_value(x, 31)), max(lane_value(x, 47), lane_value(x, 63)));
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
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;   // named registers: a uint4 member with a runtime
                                             // word index is lowered to scratch (guide §5.4 rule 20)
  __device__ explicit ByteReader(const uint8_t* b) : base(b) {}
  __device__ __forceinline__ uint32_t at(uint32_t i) {
    uint64_t addr = (uint64_t)(base + i);
    uint64_t al = addr & ~15ull;
    if (al != cached) {
      uint4 v = *reinterpret_cast<const uint4*>(al);
      c0 = v.x; c1 = v.y; c2 = v.z; c3 = v.w;
      cached = al;
    }
    uint32_t o = (uint32_t)(addr & 15);
    uint32_t m4 = 0u - ((o >> 2) & 1u), m8 = 0u - ((o >> 3) & 1u);
    uint32_t lo = (c0 & ~m4) | (c1 & m4);
    uint32_t hi = (c2 & ~m4) | (c3 & m4);
    uint32_t w = (lo & ~m8) | (hi & m8);
    return (w >> ((o & 3) * 8)) & 0xFFu;
  }
  // bytes i..i+3, little-endian (reads up to 3 bytes past the string: arena slack)
  __device__ __forceinline__ uint32_t word(uint32_t i) {
    return at(i) | (at(i + 1) << 8) | (at(i + 2) << 16) | (at(i + 3) << 24);
  }
  struct Stream {
    ByteReader* rd;
    uint32_t q;
    __device__ __forceinline__ uint32_t next() { uint32_t x = rd->word(q); q += 4; return x; }
  };
  __device__ __forceinline__ Stream stream(uint32_t i) { return Stream{this, i}; }
};

// Reader over bytes staged in LDS.  Single bytes are ds_read_u8; words are
// two aligned ds_read_b32 funnel-shifted with v_alignbyte_b32, and a stream
// carries the upper dword into the next step (one LDS read per 4 bytes).
typedef const __attribute__((address_space(3))) uint8_t lds_u8;
typedef const __attribute__((address_space(3))) uint32_t lds_u32;
struct LdsReader {
  lds_u32* base;   // 4-byte aligned slice
  uint32_t off;    // string start within the slice
  __device__ LdsReader(lds_u32* b, uint32_t o) : base(b), off(o) {}
  __device__ __forceinline__ uint32_t at(uint32_t i) const { return ((lds_u8*)base)[off + i]; }
  // two aligned reads and a funnel shift: gfx950 takes a misaligned
  // ds_read_b32 but replays it (64 cycles per wave instruction, PMC
  // SQ_LDS_UNALIGNED_STALL), which cost url_plan_kernel more LDS cycles
  // than all its aligned accesses (OSE_LDS_WORD1=1 builds the single
  // misaligned read, diagnostics only)
  __device__ __forceinline__ uint32_t word(uint32_t i) const {
#if OSE_LDS_WORD1
    typedef uint32_t __attribute__((aligned(1))) u32_ua;
    return *reinterpret_cast<const __attribute__((address_space(3))) u32_ua*>((lds_u8*)base + off + i);
#else
    const uint32_t p = off + i;
    return __builtin_amdgcn_alignbyte(base[(p >> 2) + 1], base[p >> 2], p & 3);
#endif
  }
  // the dword after next is loaded one step ahead so its latency overlaps
  // the caller's work on the current word (reads up to 11 bytes past i)
  struct Stream {
    lds_u32* w;
    uint32_t sh, lo, mid;
    __device__ __forceinline__ uint32_t next() {
      const uint32_t x = __builtin_amdgcn_alignbyte(mid, lo, sh);
      lo = mid;
      mid = w[2];
      w++;
      return x;
    }
  };
  __device__ __forceinline__ Stream stream(uint32_t i) const {
    const uint32_t p = off + i;
    return Stream{base + (p >> 2), p & 3, base[p >> 2], base[(p >> 2) + 1]};
  }
};

// ---------------------------------------------------------------------------
// SWAR byte classes over a little-endian word of 4 bytes: each result has bit
// 7 of byte k set when byte k is in the class.  t = (x & 0x7F7F7F7F) | kH;
// bytes >= 0x80 are masked out by the caller.
constexpr uint32_t kH = 0x80808080u, kL = 0x01010101u;
__device__ __forceinline__ uint32_t swar_t(uint32_t x) { return (x & 0x7F7F7F7Fu) | kH; }
__device__ __forceinline__ uint32_t swar_ge(uint32_t t, uint32_t k) { return (t - k * kL) & kH; }   // byte >= k (k <= 128)
__device__ __forceinline__ uint32_t swar_eq(uint32_t x, uint32_t k) {                               // byte == k (any byte)
  const uint32_t y = x ^ (k * kL);
  return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & kH;
}
// high bits of the bytes at index >= rem (rem < 4), 0 when rem >= 4
__device__ __forceinline__ uint32_t swar_end(uint32_t rem) { return rem >= 4 ? 0u : kH << (8 * rem); }
// high bits of the bytes before the first flagged byte of stop
__device__ __forceinline__ uint32_t swar_before(uint32_t stop) { return ((stop & (0u - stop)) - 1u) & kH; }
// index of the first flagged byte (4 when none)
__device__ __forceinline__ uint32_t swar_first(uint32_t m) { return m ? (uint32_t)(__ffs(m) - 1) >> 3 : 4u; }

// first index >= q in [q, n) holding byte ch, or n
template <class Reader>
__device__ __forceinline__ uint32_t scan_to(Reader& rd, uint32_t q, uint32_t n, uint32_t ch) {
  auto st = rd.stream(q);
  for (;;) {
    const uint32_t stop = swar_eq(st.next(), ch) | swar_end(n - q);
    if (stop) return q + swar_first(stop);
    q += 4;
  }
}
// number of bytes ch in [q, n)
template <class Reader>
__device__ __forceinline__ uint32_t count_byte(Reader& rd, uint32_t q, uint32_t n, uint32_t ch) {
  auto st = rd.stream(q);
  uint32_t c = 0;
  for (;;) {
    const uint32_t end = swar_end(n - q);
    c += __builtin_popcount(swar_eq(st.next(), ch) & swar_before(end));
    if (end) return c;
    q += 4;
  }
}

// unicode/utf8.DecodeRune on [i, e): invalid -> (U+FFFD, 1)
template <class Reader>
__device__ inline uint32_t decode_rune(Reader& rd, uint32_t i, uint32_t e, uint32_t& w) {
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
template <class Reader>
__device__ inline bool dfa_match(const uint8_t* blob, uint32_t dfa_off, Reader& rd, uint32_t s, uint32_t e) {
  const DfaDev* d = reinterpret_cast<const DfaDev*>(blob + dfa_off);
  const uint16_t* trans = reinterpret_cast<const uint16_t*>(blob + d->trans_off);
  const uint32_t* trans32 = reinterpret_cast<const uint32_t*>(blob + d->trans_off);
  const bool wide = d->wide != 0;
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
    st = wide ? trans32[st * ncls + cls] : (uint32_t)trans[st * ncls + cls];
  }
  const uint8_t* acc = blob + d->acc_off;
  return st == match || acc[st];
}

}  // namespace ose
