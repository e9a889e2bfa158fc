// trace_kernel.hip — odigossampling on CDNA4 (gfx950).
//
// Replaces RuleEngine.ShouldSample over every trace of a batch
// (odigossamplingprocessor/rule_engine.go:55-115 with the Evaluate functions
// of internal/sampling/{error,latency,servicename}.go), grouped by trace_id
// as groupbytrace would release them (sampling_controller.go:193-220).
//
// Fast path (one launch): positions are batch order.  A run is a maximal
// stretch of consecutive spans with one trace_id; when every trace_id forms
// exactly one run (groupbytrace release order) each run is a trace.  One
// wave owns the runs whose head lies in its 64-span window and walks them in
// 64-span steps: per-span contributions (error bit, endpoint-match bits of
// the latency rules of the span's service, service-rule bits) are combined
// by wave-segmented scans (shuffles, no LDS), the latency state (min start
// with the Go sentinel quirk, max end) by a segmented scan of the monoid
// below, once per distinct latency service present in the step.  A run that
// continues past the step is carried in wave-uniform registers plus one lane
// per latency service.  Every run head also inserts its trace_id into an
// exact hash table; a trace_id found twice sets *dup.
//
// Slow path (only when *dup; every launch checks the flag first): key every
// span by its trace's first run-head position (table lookup), stable LSD
// radix sort of the spans by that key, then the same evaluation kernel over
// the sorted positions, which makes every trace one run in batch order.
//
// Latency monoid (latency.go:69-80): minStart is replaced when it is 0 or the
// new start is smaller, so a span with start 0 resets it.  Element
// (f, m, e): f bit0 = contains a zero start, bit1 = contains a span of the
// service; m = min start after the last zero start (+inf if none); e = max
// end.  later∘earlier = {f_a|f_b, b.reset ? b.m : min(a.m, b.m), max}.  The
// final minStart is m, or 0 when m = +inf.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "devcfg.hpp"
#include "device_common.hpp"
#include "kernels.hpp"

namespace ose {
namespace {

// Owner-side record columns (ose_shard_unpack): status bit 7 says the
// record's latency element begins with a zero start (a reset of minStart
// before its min start), include/odigos_amd.h "trace-id exchange".
constexpr uint32_t kStatusReset = 0x80u;
constexpr int kTWaves = 4;
constexpr int kTThreads = kTWaves * kWave;
constexpr uint64_t kInf = ~0ull;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t tid_hash(uint64_t hi, uint64_t lo) { return splitmix64(hi ^ splitmix64(lo)); }

// include/odigos_amd.h "injected randomness"
__device__ __forceinline__ double trace_uniform(uint64_t hi, uint64_t lo, uint64_t seed) {
  const uint64_t x = hi ^ ((lo << 29) | (lo >> 35)) ^ seed;
  return (double)(splitmix64(x) >> 11) * 0x1.0p-53;
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1; }
__device__ __forceinline__ uint64_t lanemask_le(int lane) { return lane == 63 ? ~0ull : ((2ull << lane) - 1); }
__device__ __forceinline__ int ffs64(uint64_t x) { return __ffsll((unsigned long long)x) - 1; }
__device__ __forceinline__ int fls64(uint64_t x) { return 63 - __clzll((long long)x); }

__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int l) {
  return (uint64_t)rdl((uint32_t)v, l) | ((uint64_t)rdl((uint32_t)(v >> 32), l) << 32);
}
// ---- DPP segmented scans ------------------------------------------------------
// Inclusive scans over the wave in lane order with (head, value) elements:
// earlier ⊕ later = (h_e | h_l, h_l ? v_l : v_e ∘ v_l).  row_shr 1/2/4/8 scan
// each 16-lane row, row_bcast:15 and :31 carry the row totals (the pattern of
// wave_incl_sum_u32); a source lane outside the row yields the identity.
// Register-only: no ds_bpermute round trip per step.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t x) {
  return (uint64_t)dpp_mov<CTRL, ROWS>((uint32_t)old, (uint32_t)x) |
         ((uint64_t)dpp_mov<CTRL, ROWS>((uint32_t)(old >> 32), (uint32_t)(x >> 32)) << 32);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_or_step(uint32_t& h, uint32_t& err, uint64_t& ep, uint64_t& sv) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h), oe = dpp_mov<CTRL, ROWS>(0u, err);
  const uint64_t oep = dpp64<CTRL, ROWS>(0ull, ep), osv = dpp64<CTRL, ROWS>(0ull, sv);
  if (!h) {
    err |= oe;
    ep |= oep;
    sv |= osv;
  }
  h |= oh;
}
__device__ __forceinline__ void seg_or_scan(uint32_t h, uint32_t& err, uint64_t& ep, uint64_t& sv) {
  seg_or_step<0x111, 0xF>(h, err, ep, sv);
  seg_or_step<0x112, 0xF>(h, err, ep, sv);
  seg_or_step<0x114, 0xF>(h, err, ep, sv);
  seg_or_step<0x118, 0xF>(h, err, ep, sv);
  seg_or_step<0x142, 0xA>(h, err, ep, sv);
  seg_or_step<0x143, 0xC>(h, err, ep, sv);
}
// two 64-bit words (the latency stretches' threshold bits and latency-slot bits)
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_or2_step(uint32_t& h, uint64_t& x, uint64_t& y) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h);
  const uint64_t ox = dpp64<CTRL, ROWS>(0ull, x), oy = dpp64<CTRL, ROWS>(0ull, y);
  if (!h) {
    x |= ox;
    y |= oy;
  }
  h |= oh;
}
__device__ __forceinline__ void seg_or2_scan(uint32_t h, uint64_t& x, uint64_t& y) {
  seg_or2_step<0x111, 0xF>(h, x, y);
  seg_or2_step<0x112, 0xF>(h, x, y);
  seg_or2_step<0x114, 0xF>(h, x, y);
  seg_or2_step<0x118, 0xF>(h, x, y);
  seg_or2_step<0x142, 0xA>(h, x, y);
  seg_or2_step<0x143, 0xC>(h, x, y);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_or3_step(uint32_t& h, uint64_t& x, uint64_t& y, uint64_t& z) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h);
  const uint64_t ox = dpp64<CTRL, ROWS>(0ull, x), oy = dpp64<CTRL, ROWS>(0ull, y), oz = dpp64<CTRL, ROWS>(0ull, z);
  if (!h) {
    x |= ox;
    y |= oy;
    z |= oz;
  }
  h |= oh;
}
__device__ __forceinline__ void seg_or_scan3(uint32_t h, uint64_t& x, uint64_t& y, uint64_t& z) {
  seg_or3_step<0x111, 0xF>(h, x, y, z);
  seg_or3_step<0x112, 0xF>(h, x, y, z);
  seg_or3_step<0x114, 0xF>(h, x, y, z);
  seg_or3_step<0x118, 0xF>(h, x, y, z);
  seg_or3_step<0x142, 0xA>(h, x, y, z);
  seg_or3_step<0x143, 0xC>(h, x, y, z);
}

// one 32-bit word (kNarrow: the error bit, endpoint bits and service bits packed)
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_or1_step(uint32_t& h, uint32_t& x) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h), ox = dpp_mov<CTRL, ROWS>(0u, x);
  if (!h) x |= ox;
  h |= oh;
}
__device__ __forceinline__ void seg_or1_scan(uint32_t h, uint32_t& x) {
  seg_or1_step<0x111, 0xF>(h, x);
  seg_or1_step<0x112, 0xF>(h, x);
  seg_or1_step<0x114, 0xF>(h, x);
  seg_or1_step<0x118, 0xF>(h, x);
  seg_or1_step<0x142, 0xA>(h, x);
  seg_or1_step<0x143, 0xC>(h, x);
}
// two 32-bit words (kNarrow: the latency rules and latency slots fit 32 bits)
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_or2n_step(uint32_t& h, uint32_t& x, uint32_t& y) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h), ox = dpp_mov<CTRL, ROWS>(0u, x), oy = dpp_mov<CTRL, ROWS>(0u, y);
  if (!h) {
    x |= ox;
    y |= oy;
  }
  h |= oh;
}
__device__ __forceinline__ void seg_or2n_scan(uint32_t h, uint32_t& x, uint32_t& y) {
  seg_or2n_step<0x111, 0xF>(h, x, y);
  seg_or2n_step<0x112, 0xF>(h, x, y);
  seg_or2n_step<0x114, 0xF>(h, x, y);
  seg_or2n_step<0x118, 0xF>(h, x, y);
  seg_or2n_step<0x142, 0xA>(h, x, y);
  seg_or2n_step<0x143, 0xC>(h, x, y);
}

// OR over the wave, broadcast: DPP row_shr within each 16-lane row, then the
// four row results read out (no ds_bpermute round trips)
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
  v |= dpp64<0x111, 0xF>(0ull, v);
  v |= dpp64<0x112, 0xF>(0ull, v);
  v |= dpp64<0x114, 0xF>(0ull, v);
  v |= dpp64<0x118, 0xF>(0ull, v);
  return rdl64(v, 15) | rdl64(v, 31) | rdl64(v, 47) | rdl64(v, 63);
}

struct Cfg {
  const SampCfgDev* h;
  const SampRuleDev* rules;
  const SampLatDev* lat;
  const uint32_t* svc_slot;
  const uint64_t* slot_rules;
  const uint64_t* svc_bits;
  const uint8_t* bytes;
};
// the bytes of a rule table a kernel copies into LDS: a table longer than
// kSampCfgLds is one whose route bytes spill (one rule with a very long
// http_route: build_sampling_tables); the endpoint bits of such a chunk come
// precomputed (endpoint_plane_kernel), so its route bytes are never read
// from the LDS copy
__device__ __forceinline__ uint32_t cfg_lds_copy_bytes(const uint8_t* g) {
  const uint32_t t = reinterpret_cast<const SampCfgDev*>(g)->total_bytes;
  return t < kSampCfgLds ? t : kSampCfgLds;
}
__device__ __forceinline__ Cfg load_cfg(const uint8_t* b) {
  Cfg c;
  c.h = reinterpret_cast<const SampCfgDev*>(b);
  c.rules = reinterpret_cast<const SampRuleDev*>(b + c.h->rules_off);
  c.lat = reinterpret_cast<const SampLatDev*>(b + c.h->lat_off);
  c.svc_slot = reinterpret_cast<const uint32_t*>(b + c.h->svc_slot_off);
  c.slot_rules = reinterpret_cast<const uint64_t*>(b + c.h->slot_rules_off);
  c.svc_bits = reinterpret_cast<const uint64_t*>(b + c.h->svc_bits_off);
  c.bytes = b + c.h->bytes_off;
  return c;
}

// The span_attribute bits of span j under a rule chunk's tables: its rules'
// attr_match bits [attr_base, attr_base + n_attr) (one 64-bit window: a
// chunk holds at most 64 service + span_attribute bits; attr_match is
// word-major, `words` planes of `stride` spans), placed after the chunk's
// service-rule bits
__device__ __forceinline__ uint64_t chunk_attr_bits(const uint64_t* am, uint64_t stride, uint32_t words,
                                                    const SampCfgDev* h, uint64_t j) {
  const uint32_t b = h->attr_base, w0 = b >> 6, sh = b & 63, na = h->n_attr;
  if (!na) return 0;
  uint64_t x = am[(uint64_t)w0 * stride + j] >> sh;
  if (sh && w0 + 1 < words) x |= am[(uint64_t)(w0 + 1) * stride + j] << (64 - sh);
  return (na >= 64 ? x : x & ((1ull << na) - 1)) << h->attr_shift;
}

struct Lat {
  uint32_t f;
  uint64_t m, e;
};
__device__ __forceinline__ Lat lat_comb(const Lat& a, const Lat& b) {   // a earlier, b later
  Lat r;
  r.f = a.f | b.f;
  r.m = (b.f & 1u) ? b.m : (a.m < b.m ? a.m : b.m);
  r.e = a.e > b.e ? a.e : b.e;
  return r;
}

template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_lat_step(uint32_t& h, Lat& v) {
  const uint32_t oh = dpp_mov<CTRL, ROWS>(0u, h);
  Lat o;
  o.f = dpp_mov<CTRL, ROWS>(0u, v.f);
  o.m = dpp64<CTRL, ROWS>(kInf, v.m);
  o.e = dpp64<CTRL, ROWS>(0ull, v.e);
  if (!h) v = lat_comb(o, v);
  h |= oh;
}
__device__ __forceinline__ void seg_lat_scan(uint32_t h, Lat& v) {
  seg_lat_step<0x111, 0xF>(h, v);
  seg_lat_step<0x112, 0xF>(h, v);
  seg_lat_step<0x114, 0xF>(h, v);
  seg_lat_step<0x118, 0xF>(h, v);
  seg_lat_step<0x142, 0xA>(h, v);
  seg_lat_step<0x143, 0xC>(h, v);
}

// strings.HasPrefix(route, rule.HttpRoute) (latency.go:97-100)
__device__ __forceinline__ bool route_has_prefix(const uint8_t* arena, ose_strref r, const uint8_t* pre, uint32_t n) {
  if (r.len < n) return false;
  const uint8_t* s = arena + r.off;
  for (uint32_t k = 0; k < n; k++)
    if (s[k] != pre[k]) return false;
  return true;
}

// The first 16 bytes of a string at arena offset `off` with `len` bytes:
// one aligned dwordx4 load, a second only when the bytes cross into the next
// 16-byte chunk (never past the string's own last chunk: the arena contract
// pads allocations to 16 bytes), funnel-shifted with v_alignbyte.
__device__ __forceinline__ uint4 head16(const uint8_t* arena, uint32_t off, uint32_t len) {
  const uint8_t* b = arena + (off & ~15u);
  const uint4 c0 = *reinterpret_cast<const uint4*>(b);
  uint4 c1 = make_uint4(0, 0, 0, 0);
  const uint32_t o = off & 15u;
  if (o + (len < 16u ? len : 16u) > 16u) c1 = *reinterpret_cast<const uint4*>(b + 16);
  const uint32_t q = o >> 2, sh = o & 3u;
  const uint32_t d0 = c0.x, d1 = c0.y, d2 = c0.z, d3 = c0.w, d4 = c1.x, d5 = c1.y, d6 = c1.z, d7 = c1.w;
  auto pick = [&](uint32_t j0, uint32_t j1, uint32_t j2, uint32_t j3) {   // d[k + q] for q = 0..3
    return q == 0 ? j0 : q == 1 ? j1 : q == 2 ? j2 : j3;
  };
  const uint32_t e0 = pick(d0, d1, d2, d3), e1 = pick(d1, d2, d3, d4), e2 = pick(d2, d3, d4, d5),
                 e3 = pick(d3, d4, d5, d6), e4 = pick(d4, d5, d6, d7);
  return make_uint4(__builtin_amdgcn_alignbyte(e1, e0, sh), __builtin_amdgcn_alignbyte(e2, e1, sh),
                    __builtin_amdgcn_alignbyte(e3, e2, sh), __builtin_amdgcn_alignbyte(e4, e3, sh));
}

// Endpoint bits of one span: the latency rules of its service whose
// http_route prefixes the span's AsString(http.route) (strings.HasPrefix,
// latency.go:97-100): one 16-byte window of the route, compared under each
// rule's byte mask; prefixes longer than 16 bytes finish bytewise.
__device__ __forceinline__ uint64_t endpoint_bits_w(const Cfg& c, uint32_t slot, const uint8_t* arena, ose_strref rt,
                                                    const uint4 w) {
  uint64_t rules = c.slot_rules[slot], ep = 0;
  if (!rules || rt.len == 0) return 0;
  while (rules) {
    const int k = ffs64(rules);
    rules &= rules - 1;
    const SampLatDev& L = c.lat[k];
    if (rt.len < L.route_len) continue;
    const bool head_ok = ((w.x & L.msk[0]) == L.pre[0]) && ((w.y & L.msk[1]) == L.pre[1]) &&
                         ((w.z & L.msk[2]) == L.pre[2]) && ((w.w & L.msk[3]) == L.pre[3]);
    if (!head_ok) continue;
    if (L.route_len > 16) {
      ose_strref tail{rt.off + 16, rt.len - 16};
      if (!route_has_prefix(arena, tail, c.bytes + L.route_off + 16, L.route_len - 16)) continue;
    }
    ep |= 1ull << k;
  }
  return ep;
}
__device__ __forceinline__ uint64_t endpoint_bits(const Cfg& c, uint32_t slot, const uint8_t* arena, ose_strref rt) {
  if (rt.len == 0 || !c.slot_rules[slot]) return 0;
  return endpoint_bits_w(c, slot, arena, rt, head16(arena, rt.off, rt.len));
}

// Latency rules of `slot` that matched (endpoint found) and whose duration
// reaches the threshold.  Duration: maxEnd.AsTime().Sub(minStart.AsTime())
// .Milliseconds() — int64 ns difference saturated like time.Sub, truncated.
__device__ __forceinline__ uint64_t latency_satisfied(const Cfg& c, uint32_t slot, uint64_t ep, uint64_t m, uint64_t e) {
  uint64_t rules = c.slot_rules[slot] & ep;
  if (!rules) return 0;
  const int64_t t = (int64_t)e, u = (int64_t)(m == kInf ? 0 : m);
  int64_t d;
  if (__builtin_sub_overflow(t, u, &d)) d = t < u ? INT64_MIN : INT64_MAX;
  // d / 1e6 >= threshold  <=>  d >= threshold_ns (no 64-bit division)
  uint64_t sat = 0;
  while (rules) {
    const int r = ffs64(rules);
    rules &= rules - 1;
    const int64_t tn = c.lat[r].threshold_ns;
    if (tn != INT64_MAX && d >= tn) sat |= 1ull << r;
  }
  return sat;
}

// A latency slot with two or more stretches in one closed trace (rep: a
// stretch head whose slot the trace already had): the OR of its stretches'
// results (lsat = lraw & ep, set by the caller) is not the trace's, so that
// slot's monoid is scanned over the whole trace and its rules' bits replaced
// at the trace's tail.  Only the repeated slots are rescanned (a step with
// one repeat used to rescan every slot of its closed traces).
__device__ __forceinline__ void rep_slots(const Cfg& c, bool rep, uint32_t slot, uint32_t hseg, bool ttail, uint64_t st,
                                       uint64_t en, uint32_t rst, uint64_t ep, uint64_t& lsat) {
  // the trace's repeated slots (a segmented OR of the rep lanes' slot bits)
  uint32_t rlo = rep && slot < 32 ? 1u << slot : 0u, rhi = rep && slot >= 32 && slot != kNoSlot ? 1u << (slot - 32) : 0u;
  seg_or2n_scan(hseg, rlo, rhi);
  const uint64_t rm = (uint64_t)rlo | ((uint64_t)rhi << 32);
  for (uint64_t pend = __ballot(rep); pend;) {
    const uint32_t ks = rdl(slot, ffs64(pend));
    const bool ink = slot == ks;
    pend &= ~__ballot(ink);
    Lat v = ink ? Lat{(st == 0 || rst) ? 3u : 2u, st == 0 ? kInf : st, en} : Lat{0u, kInf, 0ull};
    seg_lat_scan(hseg, v);
    if (ttail && ((rm >> ks) & 1))
      lsat = (lsat & ~c.slot_rules[ks]) | ((v.f & 2u) ? latency_satisfied(c, ks, ep, v.m, v.e) : 0ull);
  }
}

// uniform (scalar) copies of a rule's fields: the rule table lives in LDS,
// so its fields arrive in vector registers although every lane reads the
// same rule; branching on the vector copy cost exec-mask bookkeeping per rule
__device__ __forceinline__ uint32_t sgpr(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ double sgpr(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  return __builtin_bit_cast(double, (uint64_t)sgpr((uint32_t)b) | ((uint64_t)sgpr((uint32_t)(b >> 32)) << 32));
}

// ShouldSample's level walk (rule_engine.go:55-83) over evaluateLevel's fold
// (rule_engine.go:89-115).  level: 0..2 satisfied level, 3 min fallback, 4 none.
// Without branches on per-trace values (the lanes of a flush decide 64
// traces together): every level is folded, the first satisfied one is kept
// (the early return of ShouldSample), and the min fallback of the matched
// levels is only read when no level was satisfied.  The rule fields are
// scalar, so the per-type cases are scalar branches.
__device__ __forceinline__ void decide(const Cfg& c, uint32_t err, uint64_t ep, uint64_t lsat, uint64_t svc, double u,
                              uint8_t& keep, uint8_t& level, double& ratio_out) {
  bool have_min = false, done = false;
  double min_fb = 0, out_ratio = 100.0;
  uint32_t out_level = 4;
  for (int L = 0; L < 3; L++) {
    double ratio = 0;
    bool sat = false, matched = false, found_fb = false;
    const uint32_t k0 = sgpr(c.h->level_first[L]), k1 = sgpr(c.h->level_first[L + 1]);
    for (uint32_t k = k0; k < k1; k++) {
      const SampRuleDev& r = c.rules[k];
      const uint32_t type = sgpr(r.type), bit = sgpr(r.bit);
      bool mt, st;
      double p;
      if (type == kSampError) {            // error.go:29-44
        mt = true;
        st = err != 0;
        p = st ? 100.0 : sgpr(r.fallback);
      } else if (type == kSampLatency) {   // latency.go:84-95
        mt = (ep >> bit) & 1;
        st = mt & (((lsat >> bit) & 1) != 0);
        p = st ? 100.0 : (mt ? sgpr(r.fallback) : 0.0);
      } else {                             // servicename.go:35-51
        mt = st = (svc >> bit) & 1;
        p = st ? sgpr(r.ratio) : sgpr(r.fallback);
      }
      // evaluateLevel: satisfied rules raise the ratio to their max; matched
      // unsatisfied ones take the first fallback, then the min of fallbacks
      const double rmax = ratio > p ? ratio : p;
      const double rfb = found_fb ? (ratio < p ? ratio : p) : p;
      ratio = st ? rmax : (mt ? rfb : ratio);
      found_fb |= !st & mt;
      sat |= st;
      matched |= mt;
    }
    const bool take = sat & !done;
    out_level = take ? (uint32_t)L : out_level;
    out_ratio = take ? ratio : out_ratio;
    done |= sat;
    const bool upd = matched & (!have_min | (ratio < min_fb));
    min_fb = upd ? ratio : min_fb;
    have_min |= matched;
  }
  if (!done) {
    out_level = have_min ? 3u : 4u;
    out_ratio = have_min ? min_fb : 100.0;
  }
  level = (uint8_t)out_level;
  ratio_out = out_ratio;
  keep = out_level == 4 ? 1 : (u * 100 < out_ratio);
}

// ShouldSample's walk (decide()) split at rule-chunk boundaries: walk_chunk
// takes one chunk's rules (level order, config order) from the state s (the
// open level, its evaluateLevel accumulators, the min fallback of the closed
// levels) and leaves it there; walk_finish closes the remaining levels and
// decides.  Chunk by chunk it is decide() over the whole rule list.
__device__ __forceinline__ void walk_close(FoldState& s) {   // the end of evaluateLevel for level s.level
  if (s.flags & kFsSat) {
    s.flags = kFsDone | (s.flags & kFsHaveMin);
    return;
  }
  if ((s.flags & kFsMatched) && (!(s.flags & kFsHaveMin) || s.ratio < s.min_fb)) {
    s.min_fb = s.ratio;
    s.flags |= kFsHaveMin;
  }
  s.flags &= kFsHaveMin;
  s.ratio = 0;
  s.level++;
}
__device__ void walk_chunk(const Cfg& c, FoldState& s, uint32_t err, uint64_t ep, uint64_t lsat, uint64_t svc) {
  for (uint32_t L = 0; L < 3 && !(s.flags & kFsDone); L++) {
    const uint32_t k0 = c.h->level_first[L], k1 = c.h->level_first[L + 1];
    if (k0 == k1) continue;
    while (s.level < L && !(s.flags & kFsDone)) walk_close(s);
    if (s.flags & kFsDone) break;
    for (uint32_t k = k0; k < k1; k++) {
      const SampRuleDev& r = c.rules[k];
      bool mt, st;
      double p;
      if (r.type == kSampError) {
        mt = true;
        st = err != 0;
        p = st ? 100.0 : r.fallback;
      } else if (r.type == kSampLatency) {
        mt = (ep >> r.bit) & 1;
        st = mt && ((lsat >> r.bit) & 1);
        p = st ? 100.0 : (mt ? r.fallback : 0.0);
      } else {
        mt = st = (svc >> r.bit) & 1;
        p = st ? r.ratio : r.fallback;
      }
      if (st) {
        s.ratio = s.ratio > p ? s.ratio : p;
        s.flags |= kFsSat | kFsMatched;
      } else if (mt) {
        s.flags |= kFsMatched;
        if (!(s.flags & kFsFoundFb)) {
          s.ratio = p;
          s.flags |= kFsFoundFb;
        } else {
          s.ratio = s.ratio < p ? s.ratio : p;
        }
      }
    }
  }
}
// walk_chunk over the matched rules only (trace_multi_kernel: a chunk of at
// most 128 rules, SampWalkDev): an unmatched rule changes nothing, and a
// level is closed when a matched rule of a later level comes (or by the
// next chunk / walk_finish) — the same state as walk_chunk leaves
__device__ __forceinline__ void walk_sparse(const Cfg& c, const SampWalkDev& W, FoldState& s, uint32_t err, uint64_t ep,
                                            uint64_t lsat, uint64_t svc) {
  uint64_t m[2] = {W.err[0], W.err[1]};
  for (uint64_t b = ep; b; b &= b - 1) {
    const uint32_t r = W.lat_rule[ffs64(b)];
    m[r >> 6] |= 1ull << (r & 63);
  }
  for (uint64_t b = svc; b; b &= b - 1) {
    const int x = ffs64(b);
    m[0] |= W.svc[x][0];
    m[1] |= W.svc[x][1];
  }
  const uint32_t lf1 = c.h->level_first[1], lf2 = c.h->level_first[2];
  for (int w = 0; w < 2; w++) {
    for (uint64_t mm = m[w]; mm && !(s.flags & kFsDone); mm &= mm - 1) {
      const uint32_t k = (uint32_t)(w * 64 + ffs64(mm));
      const uint32_t L = (k >= lf1 ? 1u : 0u) + (k >= lf2 ? 1u : 0u);
      while (s.level < L && !(s.flags & kFsDone)) walk_close(s);
      if (s.flags & kFsDone) break;
      const SampRuleDev& r = c.rules[k];
      bool mt, st;
      double p;
      if (r.type == kSampError) {
        mt = true;
        st = err != 0;
        p = st ? 100.0 : r.fallback;
      } else if (r.type == kSampLatency) {
        mt = (ep >> r.bit) & 1;
        st = mt && ((lsat >> r.bit) & 1);
        p = st ? 100.0 : (mt ? r.fallback : 0.0);
      } else {
        mt = st = (svc >> r.bit) & 1;
        p = st ? r.ratio : r.fallback;
      }
      if (st) {
        s.ratio = s.ratio > p ? s.ratio : p;
        s.flags |= kFsSat | kFsMatched;
      } else if (mt) {
        s.flags |= kFsMatched;
        if (!(s.flags & kFsFoundFb)) {
          s.ratio = p;
          s.flags |= kFsFoundFb;
        } else {
          s.ratio = s.ratio < p ? s.ratio : p;
        }
      }
    }
  }
}
__device__ __forceinline__ void walk_finish(FoldState& s, double u, uint8_t& keep, uint8_t& level, double& ratio_out) {
  while (s.level < 3 && !(s.flags & kFsDone)) walk_close(s);
  if (s.flags & kFsDone) {
    level = (uint8_t)s.level;
    ratio_out = s.ratio;
    keep = u * 100 < s.ratio;
  } else if (s.flags & kFsHaveMin) {
    level = 3;
    ratio_out = s.min_fb;
    keep = u * 100 < s.min_fb;
  } else {
    level = 4;
    ratio_out = 100.0;
    keep = 1;
  }
}

// One chunk of a rule-chunked configuration in a pass per chunk: the walk
// resumed from and saved to the trace's FoldState (first: the trace's first
// span); the last pass decides.
__device__ void decide_chunk(const TraceKernelArgs& a, const Cfg& c, uint64_t first, uint32_t err, uint64_t ep,
                             uint64_t lsat, uint64_t svc, double u, uint8_t& keep, uint8_t& level, double& ratio_out) {
  FoldState s = a.fold_in ? a.fold_in[first] : FoldState{0.0, 0.0, 0u, 0u};
  walk_chunk(c, s, err, ep, lsat, svc);
  if (a.fold_out) {   // more chunks follow: save the walk (this pass's keep is rewritten by the last)
    a.fold_out[first] = s;
    keep = 1;
    level = 4;
    ratio_out = 100.0;
    return;
  }
  walk_finish(s, u, keep, level, ratio_out);
}
// decide() or, in a rule-chunked pass, decide_chunk(); first: the trace's
// first span in batch order (the FoldState index)
__device__ __forceinline__ void decide_at(const TraceKernelArgs& a, const Cfg& c, uint64_t first, uint32_t err,
                                          uint64_t ep, uint64_t lsat, uint64_t svc, double u, uint8_t& keep,
                                          uint8_t& level, double& ratio_out) {
  if (a.fold_in || a.fold_out)
    decide_chunk(a, c, first, err, ep, lsat, svc, u, keep, level, ratio_out);
  else
    decide(c, err, ep, lsat, svc, u, keep, level, ratio_out);
}

// ---- exact trace_id table -------------------------------------------------
// Insert protocol: CAS the state from a stale epoch to BUSY, store the key
// with sc1 (agent-scope relaxed) stores, drain them (s_waitcnt vmcnt(0)), then
// store READY; readers poll the state and read the key with sc1 loads
// (MI355X_MICROARCH.md "Valid forms": sc1 payload + drained flag).  A lane
// that finds the key ready and equal is a second run of that trace_id.
// Returns kInsNew (the slot was claimed; with run lists, the run is listed
// as the trace's first), kInsFound (the id was there: a repeated trace id)
// or kInsFail (error flagged).  Callers gated on *dup do not set it again:
// one word hit by every repeated head of the batch is a serialised
// device-scope atomic per head.
constexpr int kInsNew = 0, kInsFound = 1, kInsFail = -1;
__device__ inline int table_insert(const TraceKernelArgs& a, uint64_t hi, uint64_t lo, uint32_t pos,
                                    uint64_t* slot_out = nullptr) {
  const uint32_t busy = (a.epoch << 2) | 1u, ready = (a.epoch << 2) | 2u;
  uint64_t h = tid_hash(hi, lo) & a.table_mask;
  uint32_t probes = 0, spins = 0;
  for (;;) {
    TraceSlot* s = &a.table[h];
    const uint32_t st = __hip_atomic_load(&s->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((st >> 2) != a.epoch) {
      uint32_t expect = st;
      if (__hip_atomic_compare_exchange_strong(&s->state, &expect, busy, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(&s->hi, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->lo, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->first, pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.run_count) {   // this run is the trace's first listed run
          __hip_atomic_store(&a.run_count[h], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (a.runs) a.runs[h * kMaxRuns] = pos;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&s->state, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (slot_out) *slot_out = h;
        return kInsNew;
      }
      continue;   // lost the race for this slot: look at it again
    }
    if ((st & 3u) != 2u) {   // another lane is publishing this slot
      if (++spins > (1u << 20)) {
        atomicOr(a.error, 1u);
        return kInsFail;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint64_t h2 = __hip_atomic_load(&s->hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t l2 = __hip_atomic_load(&s->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (h2 == hi && l2 == lo) {
      atomicMin(&s->first, pos);
      if (slot_out) *slot_out = h;
      return kInsFound;
    }
    h = (h + 1) & a.table_mask;
    if (++probes > a.table_mask) {
      atomicOr(a.error, 4u);
      return kInsFail;
    }
  }
}

// ---- per-step columns ---------------------------------------------------------
// Raw loads of one 64-span step, issued one step ahead of their use (the
// compiler places the waits at the first use, in the next iteration), so a
// wave keeps two steps of HBM reads in flight.
struct StepRaw {
  uint64_t i;          // span index (perm[p] in kTracePerm)
  uint64_t hi, lo;     // trace id
  uint64_t ph, pl;     // lane 0: trace id of position p-1 (head test); lane 63: of p+1 (kTraceRuns)
  uint32_t k, pk;      // kTracePerm: canonical key of p and (lane 0) of p-1
  uint32_t res;
  uint32_t status;
  ose_strref route;
  uint64_t start, end;
  uint64_t svm;        // svc_match (owner-side record columns)
  bool full;           // the per-span columns below the trace id were loaded
};
// full = false loads only what the head test needs: a wave skipping windows
// inside a run an earlier wave owns reads 16 B per span, not every column.
__device__ __forceinline__ StepRaw load_raw(const TraceKernelArgs& a, uint64_t base, int lane, bool full = true) {
  StepRaw r{};
  r.full = full;
  const uint64_t p = base + lane;
  const bool valid = p < a.n_spans;
  if (!valid) return r;
  if (a.mode == kTracePerm) {
    r.i = a.perm[p];
    r.k = a.key[r.i];
    if (lane == 0 && p > 0) r.pk = a.key[a.perm[p - 1]];
  } else {
    r.i = p;
    if (lane == 0 && p > 0 && a.mode == kTraceRuns) {
      r.ph = a.tid[2 * p - 2];
      r.pl = a.tid[2 * p - 1];
    }
    if (lane == kWave - 1 && p + 1 < a.n_spans && a.mode == kTraceRuns) {   // the span after the step
      r.ph = a.tid[2 * p + 2];
      r.pl = a.tid[2 * p + 3];
    }
  }
  const uint4 v = reinterpret_cast<const uint4*>(a.tid)[r.i];
  r.hi = (uint64_t)v.x | ((uint64_t)v.y << 32);
  r.lo = (uint64_t)v.z | ((uint64_t)v.w << 32);
  if (!full) return r;
  r.res = a.resource[r.i];
  r.status = a.status[r.i];
  if (a.start) {
    r.start = a.start[r.i];
    r.end = a.end[r.i];
  }
  if (a.route) r.route = a.route[r.i];
  if (a.svc_match) r.svm = a.svc_match[r.i];
  return r;
}
// head flag of every lane of a step (all lanes take the shuffles)
__device__ __forceinline__ bool step_head(const TraceKernelArgs& a, const StepRaw& r, uint64_t base, int lane) {
  const uint64_t p = base + lane;
  const bool valid = p < a.n_spans;
  if (a.mode == kTracePerm) {
    uint32_t pk = __shfl_up(r.k, 1, kWave);
    if (lane == 0) pk = r.pk;
    return valid && (p == 0 || pk != r.k);
  }
  // wave_shr:1 (DPP): lane l gets lane l-1's trace id, lane 0 its own prefetched p-1 id
  const uint64_t ph = dpp64<0x138, 0xF>(r.ph, r.hi), pl = dpp64<0x138, 0xF>(r.pl, r.lo);
  if (a.mode == kTraceBatch) return valid && p == 0;
  return valid && (p == 0 || ph != r.hi || pl != r.lo);
}
__device__ __forceinline__ bool head_at(const TraceKernelArgs& a, uint64_t p) {   // p < n, p > 0
  if (a.mode == kTraceBatch) return false;
  if (a.mode == kTracePerm) return a.key[a.perm[p]] != a.key[a.perm[p - 1]];
  return a.tid[2 * p] != a.tid[2 * p - 2] || a.tid[2 * p + 1] != a.tid[2 * p - 1];
}

__device__ __forceinline__ void write_rec(const TraceKernelArgs& a, uint64_t pos, uint8_t keep, uint8_t level,
                                          double ratio) {
  if (a.mode == kTraceBatch && a.batch_keep) *a.batch_keep = keep;
  if (!a.rec) return;
  TraceRec r;
  r.first_span = a.mode == kTracePerm ? a.perm[pos] : (uint32_t)pos;
  r.keep = keep;
  r.level = level;
  r._p0 = r._p1 = 0;
  r.ratio = ratio;
  a.rec[pos] = r;
}

// Run heads are collected per wave in LDS and inserted 64 at a time: each
// insert is a load and a dependent CAS, so batching turns a per-step pair of
// round trips into one pair per 64 heads.
constexpr int kHeadQ = 128;
struct HeadQ {
  uint64_t cell[kHeadQ];
};
__device__ void flush_heads(const TraceKernelArgs& a, HeadQ& H, uint32_t& hn, int lane) {
  __builtin_amdgcn_wave_barrier();
  bool dup = false;
  // bucketed: one returning atomic per head, the fingerprint stored after it
  for (uint32_t b = 0; b < hn; b += kWave) {
    if (b + lane < hn) {
      const uint64_t h = H.cell[b + lane];
      const uint32_t bk = (uint32_t)(h >> (64 - a.dup_bkt_bits));   // dup_bkt_bits in [1, 32] (the host's)
      const uint32_t at = atomicAdd(&a.dup_bkt_count[bk], 1u);
      if (at < kDupBucketCap) a.dup_bkt[(uint64_t)bk * kDupBucketCap + at] = h | 1ull;   // (0 marks an empty set slot)
      else dup = true;
    }
  }
  // one *dup store per wave flush (a per-head atomic on one word serialises)
  if (__ballot(dup) && lane == 0) atomicOr(a.dup, 1u);
  __builtin_amdgcn_wave_barrier();
  hn = 0;
}

// ---- decide queue ---------------------------------------------------------------
// Closed traces are queued per wave in LDS and decided 64 at a time, so the
// rule fold runs with every lane busy instead of once per trace tail.
constexpr int kQ = 64;
struct DecideQ {
  uint64_t ep[kQ], lsat[kQ], svc[kQ], hi[kQ], lo[kQ];
  uint32_t pos[kQ], len[kQ], err[kQ];
};

__device__ __forceinline__ void write_keep_range(const TraceKernelArgs& a, uint64_t pos, uint32_t len, uint8_t k,
                                                 int lane) {
  for (uint32_t q = lane; q < len; q += kWave) a.keep[a.mode == kTracePerm ? a.perm[pos + q] : pos + q] = k;
}

__device__ void flush_queue(const TraceKernelArgs& a, const Cfg& c, DecideQ& Q, uint32_t& qn, int lane) {
  if (!qn) return;
  __builtin_amdgcn_wave_barrier();
  uint8_t dk = 0, dl = 0;
  double dr = 0;
  uint32_t pos = 0, len = 0;
  if ((uint32_t)lane < qn) {
    pos = Q.pos[lane];
    len = Q.len[lane];
    if (!(a.ablate & 4))
      decide_at(a, c, a.mode == kTracePerm ? a.perm[pos] : (a.mode == kTraceBatch ? 0u : pos), Q.err[lane], Q.ep[lane],
                Q.lsat[lane], Q.svc[lane], trace_uniform(Q.hi[lane], Q.lo[lane], a.seed), dk, dl, dr);
    write_rec(a, pos, dk, dl, dr);
  }
  const uint32_t mlen = wave_max_u32((uint32_t)lane < qn ? len : 0u);
  if (a.mode != kTracePerm && mlen <= 32) {
    // short traces: each lane writes its own trace's keep bytes (at most 32
    // store instructions per 64 traces instead of one per trace)
    if ((uint32_t)lane < qn)
      for (uint32_t q = 0; q < len; q++) a.keep[pos + q] = dk;
  } else {
    for (uint32_t e = 0; e < qn; e++)
      write_keep_range(a, rdl(pos, e), rdl(len, e), (uint8_t)rdl(dk, e), lane);
  }
  __builtin_amdgcn_wave_barrier();
  qn = 0;
}



// kLean: the instance for the common call — batch order (kTraceRuns), no
// owner-side record columns, no precomputed endpoint bits, no span_attribute
// bits, no diagnostics.  Those arguments are constants in it, so their code
// and the kernel-argument registers that hold them fold away (the general
// instance spills ~90 scalar registers into vector lanes).
// kNarrow (with kLean): the error bit, the endpoint bits of the latency rules
// and the service-rule bits fit one 32-bit word (1 + n_lat + service bits <=
// 32, n_lat_slots <= 32; the host checks): the segmented ORs scan one word
// instead of five, the latency stretches' words two instead of four.
// kChunk (with kLean): one pass of a rule-chunked configuration, the walk
// resumed from fold_in and saved to fold_out (decide_chunk) — the lean
// instance's loads and scans instead of the general instance's.
template <bool kLean, bool kNarrow, bool kChunk>
__global__ __launch_bounds__(kTThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void trace_eval_kernel(TraceKernelArgs a) {
  if (kLean) {
    a.mode = kTraceRuns;
    a.svc_match = nullptr;
    a.route_match = nullptr;
    a.attr_match = nullptr;
    a.perm = nullptr;
    a.key = nullptr;
    a.batch_keep = nullptr;
#if !OSE_DIAG
    a.ablate = 0;   // (diagnostics builds keep OSE_TRACE_ABLATE for the lean instances too)
#endif
    if (!kChunk) {
      a.fold_in = nullptr;
      a.fold_out = nullptr;
    }
  }
  if (a.mode == kTracePerm && __hip_atomic_load(a.dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  __shared__ DecideQ queues[kTWaves];
  __shared__ HeadQ headqs[kTWaves];
  __shared__ __attribute__((aligned(16))) uint8_t cfg_lds[kSampCfgLds];
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  DecideQ& Q = queues[wv];
  HeadQ& HQ = headqs[wv];
  {
    // the rule tables (<= kSampCfgLds bytes, checked by the host) live in LDS:
    // every lookup below is a ds_read instead of a dependent L2 round trip
    const uint32_t nb = cfg_lds_copy_bytes(a.cfg);
    for (uint32_t k = threadIdx.x * 16; k < nb; k += kTThreads * 16)
      *reinterpret_cast<uint4*>(cfg_lds + k) = *reinterpret_cast<const uint4*>(a.cfg + k);
    __syncthreads();
  }
  const uint64_t wpw = a.win_per_wave;
  const uint64_t w0 = ((uint64_t)blockIdx.x * kTWaves + wv) * wpw;   // first owned window
  if (w0 >= a.n_windows) return;
  const Cfg c = load_cfg(cfg_lds);
  const uint64_t n = a.n_spans;
  const uint32_t nsvc = c.h->n_services;

  // OSE_GROUP_BATCH: ServiceNameRule looks at every resource of the call,
  // spanless ones included (servicename.go:38-47).
  uint64_t batch_svc = 0;
  if (a.mode == kTraceBatch && w0 == 0) {
    for (uint32_t r = lane; r < a.n_resources; r += kWave) {
      const uint32_t s = a.res_svc_str[r];
      if (s < nsvc) batch_svc |= c.svc_bits[s];
    }
    batch_svc = wave_or64(batch_svc);
  }
  if (n == 0) {   // kTraceBatch only: one trace with no spans
    uint8_t k, l;
    double r;
    decide_at(a, c, 0, 0, 0, 0, batch_svc, trace_uniform(0, 0, a.seed), k, l, r);
    if (lane == 0) {
      if (a.batch_keep) *a.batch_keep = k;
      if (a.win_heads) a.win_heads[0] = 1;
      if (a.rec) {
        TraceRec rr{0, k, l, 0, 0, r};
        a.rec[0] = rr;
      }
    }
    return;
  }

  const uint64_t range_end = min((w0 + wpw) * kWave, n);
  uint32_t qn = 0, hn = 0;
  bool started = false, open = false;
  uint32_t c_err = 0;
  uint64_t c_ep = 0, c_svc = 0, c_kmask = 0, c_pos = 0, c_hi = 0, c_lo = 0;
  Lat cur{0, kInf, 0};
  uint64_t base = w0 * kWave;
  const bool want_route = c.h->n_lat && !a.route_match && a.route;
  StepRaw nx = load_raw(a, base, lane);
  for (;;) {
    // Order of the memory operations per step: this step's dependent loads
    // (resource service ids, the route window, the fingerprint cell), then
    // the next step's column loads, then the arithmetic — a wait for a load
    // also waits for every load issued before it (vmcnt counts in order),
    // so nothing this step consumes may be issued after the prefetch.
    StepRaw r = nx;
    const bool valid = base + lane < n;
    const bool hd = step_head(a, r, base, lane);
    const bool work = started || __ballot(hd) != 0;   // wave-uniform: this step is evaluated
    if (work && !r.full) r = load_raw(a, base, lane);   // first owned step after skipped ones
    uint32_t sv = 0xFFFFFFFFu, ss = 0xFFFFFFFFu;
    uint4 rw = make_uint4(0, 0, 0, 0);
    if (valid && work) {
      if (a.ablate & 16) {   // diagnostics: no dependent service-id loads
        sv = r.res % (nsvc + 1);
        ss = sv;
      } else {
        sv = a.res_svc[r.res];
        ss = a.res_svc_str[r.res];
      }
      // route bytes only for spans of a latency-rule service (strings.HasPrefix
      // is evaluated for nothing else): one dependent LDS lookup, and the
      // random 16-byte arena reads of every other routed span are skipped
      if (want_route && r.route.len && sv < nsvc && c.svc_slot[sv] != kNoSlot && !(a.ablate & 32))
        rw = head16(a.arena, r.route.off, r.route.len);
    }
    const uint64_t vmask = __ballot(valid);
    const uint64_t hmask = __ballot(hd);
    const bool in_range = base < range_end;
    if (in_range) {
      if (lane == 0 && a.win_heads) a.win_heads[base / kWave] = hmask;
      // (no dup_bkt: a later rule-chunk pass, whose batch layout the first
      // pass already checked — *dup carries that pass's answer)
      if (a.mode == kTraceRuns && !(a.ablate & 1) && a.dup_bkt && hmask) {
        const uint32_t nh = __popcll(hmask);
        if (hn + nh > kHeadQ) flush_heads(a, HQ, hn, lane);
        if (hd) {
          const uint32_t e = hn + __popcll(hmask & lanemask_lt(lane));
          // one multiply (odd: a bijection) on the folded id; its top bits
          // (the bucket) depend on every bit of the id
          HQ.cell[e] = (r.lo ^ ((r.hi << 29) | (r.hi >> 35))) * 0x9E3779B97F4A7C15ull;
        }
        hn += nh;
      }
    }
    // (the service ids loaded a step ahead too, the resource index two steps
    // ahead: C3 -1 %, C4 -1.3 %, C5 +13 % — skipped steps then load every
    // column; profiles/r4q_te_pipe_ab.txt)
    if (base + kWave < n) nx = load_raw(a, base + kWave, lane, work);   // prefetch the next step
    uint64_t own;
    if (in_range) {
      if (!started) {
        if (!hmask) {   // still inside a trace an earlier wave owns
          base += kWave;
          if (base >= range_end) break;
          continue;
        }
        started = true;
        own = vmask & ~lanemask_lt(ffs64(hmask));
      } else {
        own = vmask;
      }
    } else {
      if (!open) break;
      own = vmask & (hmask ? lanemask_lt(ffs64(hmask)) : ~0ull);
    }
    const uint64_t segmask = (hmask & own) | (open ? 1ull : 0ull);
    const int last_own = fls64(own);
    bool cont_next = false;
    if (last_own == 63 && base + kWave < n) {
      bool h = false;
      // kTraceRuns: lane 63 loaded the next step's first trace id with this step
      if (lane == 63) h = a.mode == kTraceRuns ? (r.ph != r.hi || r.pl != r.lo) : head_at(a, base + kWave);
      cont_next = !rdl((uint32_t)h, 63);
    }
    const bool mine = (own >> lane) & 1;
    const int sst = mine ? fls64(segmask & lanemask_le(lane)) : lane;
    const bool tail = mine && (lane == last_own || ((segmask >> (lane + 1)) & 1));
    const uint64_t tails = __ballot(tail);
    const int t0 = ffs64(tails);
    const bool seg0_cont = open;
    const bool single = t0 == last_own;
    const bool last_open = cont_next && !(single && seg0_cont);   // a new trace opens in this step and continues
    const int sst_last = rdl((uint32_t)sst, last_own);

    // ---- per-span contributions ----
    uint32_t err = 0, slot = kNoSlot;
    uint64_t ep = 0, svcb = 0, st = 0, en = 0;
    const uint32_t rst = (r.status & kStatusReset) ? 1u : 0u;   // owner-side record: a zero start came first
    if (mine) {
      const uint32_t s = sv;
      err = (r.status & ~kStatusReset) == OSE_STATUS_ERROR;
      if (a.svc_match) {
        svcb = r.svm;
      } else {
        if (a.mode != kTraceBatch && ss < nsvc) svcb = c.svc_bits[ss];
        if (a.attr_match) svcb |= chunk_attr_bits(a.attr_match, a.attr_stride, a.attr_words, c.h, r.i);
      }
      if (s < nsvc) {
        slot = c.svc_slot[s];
        if (slot != kNoSlot) {
          if (!(a.ablate & 8))
            ep = a.route_match ? a.route_match[r.i] & c.slot_rules[slot]
                               : endpoint_bits_w(c, slot, a.arena, r.route, rw);
          st = r.start;
          en = r.end;
        }
      }
    }
    // ---- latency state (latency.go:69-80) ----
    // One segmented scan of the monoid over stretches: maximal runs of lanes
    // with one trace and one latency slot (a trace's spans of a service come
    // together, ResourceSpans by ResourceSpans).  A stretch's element is its
    // trace's element for that slot when the slot has no other stretch in the
    // trace within this step; the step checks that (slot bits OR-scanned per
    // trace) and otherwise takes the per-slot scans below.  At a stretch tail
    // the slot's rules whose threshold the duration reaches are found without
    // the endpoint mask; ORed per trace and masked by the trace's endpoint bits
    // at its tail, they are the per-slot result.  The carried trace (segment 0)
    // and the trace left open at the end combine their stretches into the
    // per-slot carry registers in lane order.
    const uint32_t hseg = mine ? (uint32_t)((segmask >> lane) & 1) : 1u;
    // ---- segmented OR of the flag masks (DPP scan; h = segment head) ----
    if constexpr (kNarrow) {
      const uint32_t nsh = 1 + c.h->n_lat;   // <= 32 (host-checked)
      uint32_t pk = err | ((uint32_t)ep << 1) | (nsh < 32 ? (uint32_t)svcb << nsh : 0u);
      seg_or1_scan(hseg, pk);
      err = pk & 1u;
      ep = (pk >> 1) & (uint32_t)((1ull << c.h->n_lat) - 1);
      svcb = nsh < 32 ? pk >> nsh : 0u;
    } else {
      seg_or_scan(hseg, err, ep, svcb);
    }
    uint64_t lsat = 0, n_kmask = 0;
    Lat nxt{0, kInf, 0};
    const bool carried_tail = (lane == t0 && seg0_cont) || (lane == last_own && last_open);
    const bool lat_on = !(a.ablate & 2) && __ballot(slot != kNoSlot) != 0;   // wave-uniform
    uint64_t lraw = 0, smask = 0;
    bool stail = false, shead = false;
    if (lat_on) {
      const uint32_t pslot = dpp_mov<0x138>(kNoSlot, slot);   // lane - 1's slot (wave_shr:1)
      shead = !mine || hseg || pslot != slot;
      const uint32_t hs = shead ? 1u : 0u;
      stail = mine && dpp_mov<0x130>(1u, hs) != 0;            // lane + 1 starts a stretch (wave_shl:1)
      Lat v = slot != kNoSlot ? Lat{(st == 0 || rst) ? 3u : 2u, st == 0 ? kInf : st, en} : Lat{0u, kInf, 0ull};
      seg_lat_scan(hs, v);
      const bool lt = stail && (v.f & 2u);
      if (lt) lraw = latency_satisfied(c, slot, ~0ull, v.m, v.e);
      if (slot != kNoSlot) smask = 1ull << slot;
      if (seg0_cont) {   // the carried trace's stretches, in order
        for (uint64_t m0 = __ballot(lt && lane <= t0); m0; m0 &= m0 - 1) {
          const int L = ffs64(m0);
          const uint32_t ks = rdl(slot, L);
          const Lat v0{rdl(v.f, L), rdl64(v.m, L), rdl64(v.e, L)};
          if ((uint32_t)lane == ks) cur = lat_comb(cur, v0);
          c_kmask |= 1ull << ks;
        }
      }
      if (last_open) {   // the open trace's stretches, in order
        for (uint64_t m1 = __ballot(lt && lane >= sst_last); m1; m1 &= m1 - 1) {
          const int L = ffs64(m1);
          const uint32_t ks = rdl(slot, L);
          const Lat v1{rdl(v.f, L), rdl64(v.m, L), rdl64(v.e, L)};
          if ((uint32_t)lane == ks) nxt = lat_comb(nxt, v1);
          n_kmask |= 1ull << ks;
        }
      }
    }
    if (lat_on) {
      if constexpr (kNarrow) {
        uint32_t lr = (uint32_t)lraw, sm = (uint32_t)smask;
        seg_or2n_scan(hseg, lr, sm);
        lraw = lr;
        smask = sm;
      } else {
        seg_or2_scan(hseg, lraw, smask);
      }
      // a slot with two stretches in a trace this step closes: per-slot scans
      const uint64_t psm = dpp64<0x138, 0xF>(0ull, smask);   // lane - 1's inclusive slot bits
      const bool in_closed = mine && !(seg0_cont && lane <= t0) && !(last_open && lane >= sst_last);
      const bool rep = in_closed && shead && !hseg && slot != kNoSlot && ((psm >> slot) & 1);
      if (tail && !carried_tail) lsat = lraw & ep;
      if (__ballot(rep)) rep_slots(c, rep, slot, hseg, tail && !carried_tail, st, en, rst, ep, lsat);
    }
    // ---- the carried trace closes in this step: queue it ----
    const bool cont_close = seg0_cont && !(single && cont_next);
    if (cont_close) {
      const uint32_t E = c_err | rdl(err, t0);
      const uint64_t EP = c_ep | rdl64(ep, t0);
      const uint64_t SV = batch_svc | c_svc | rdl64(svcb, t0);
      uint64_t s_l = 0;
      if ((c_kmask >> lane) & 1) s_l = latency_satisfied(c, (uint32_t)lane, EP, cur.m, cur.e);
      s_l = wave_or64(s_l);
      if (qn == kQ) flush_queue(a, c, Q, qn, lane);
      if (lane == 0) {
        Q.err[qn] = E;
        Q.ep[qn] = EP;
        Q.lsat[qn] = s_l;
        Q.svc[qn] = SV;
        Q.hi[qn] = c_hi;
        Q.lo[qn] = c_lo;
        Q.pos[qn] = (uint32_t)c_pos;
        Q.len[qn] = (uint32_t)(base + t0 + 1 - c_pos);
      }
      qn++;
      open = false;
      cur = Lat{0, kInf, 0};
      c_kmask = 0;
    }
    // ---- traces that start and end in this step: queue them ----
    const uint64_t qmask = __ballot(tail && !carried_tail);
    const uint32_t nq = __popcll(qmask);
    if (nq) {
      if (qn + nq > kQ) flush_queue(a, c, Q, qn, lane);
      // the trace's first span's id (the injected uniform): in batch order and
      // in the sorted permutation every span of a segment has that id; only a
      // whole-batch trace (OSE_GROUP_BATCH) mixes ids
      uint64_t hh = r.hi, hl = r.lo;
      if (a.mode == kTraceBatch) {
        hh = __shfl(r.hi, sst, kWave);
        hl = __shfl(r.lo, sst, kWave);
      }
      if ((qmask >> lane) & 1) {
        const uint32_t e = qn + __popcll(qmask & lanemask_lt(lane));
        Q.err[e] = err;
        Q.ep[e] = ep;
        Q.lsat[e] = lsat;
        Q.svc[e] = batch_svc | svcb;   // batch mode: resource bits of the call + span_attribute bits
        Q.hi[e] = hh;
        Q.lo[e] = hl;
        Q.pos[e] = (uint32_t)(base + sst);
        Q.len[e] = (uint32_t)(lane - sst + 1);
      }
      qn += nq;
    }
    // ---- carry into the next step ----
    if (last_open) {
      open = true;
      c_pos = base + sst_last;
      c_hi = rdl64(r.hi, sst_last);
      c_lo = rdl64(r.lo, sst_last);
      c_err = rdl(err, last_own);
      c_ep = rdl64(ep, last_own);
      c_svc = rdl64(svcb, last_own);
      cur = nxt;
      c_kmask = n_kmask;
    } else if (seg0_cont && single && cont_next) {
      c_err |= rdl(err, t0);
      c_ep |= rdl64(ep, t0);
      c_svc |= rdl64(svcb, t0);
    }
    base += kWave;
    if (!open && base >= range_end) break;
    if (open && a.long_runs && base >= range_end + (uint64_t)a.long_steps * kWave) {
      // a long run: trace_long_kernel splits it over a workgroup's waves
      if (lane == 0) a.long_runs[atomicAdd(a.n_long, 1u)] = (uint32_t)c_pos;
      break;
    }
  }
  flush_queue(a, c, Q, qn, lane);
  if (a.dup_bkt) flush_heads(a, HQ, hn, lane);
}

// ---- rule-chunked lists in one pass ---------------------------------------------
// A rule list cut into K (2..kMaxMulti) chunks — no span_attribute rules, no
// spilled routes, grouped by trace id — in one pass over the columns instead
// of one per chunk: every chunk's table sits in LDS, each step evaluates each
// chunk's endpoint, service and latency words exactly as trace_eval_kernel
// does for one table, and a closed trace is queued with all K; the flush
// walks the chunks in order (walk_chunk, then walk_finish: decide() over the
// whole list, rule_engine.go:55-115).  Duplicate detection is the lean
// instance's; a batch whose trace ids repeat is redone by the pass-per-chunk
// path (run_sampling).  No long-run hand-off: a run's owner wave follows it.
template <int K>
struct MultiQ {
  uint64_t hi[kQ], lo[kQ];
  uint32_t pos[kQ], len[kQ], err[kQ];
  uint64_t ep[K][kQ], lsat[K][kQ], svc[K][kQ];
};

template <int K>
__device__ __forceinline__ void flush_multi(const TraceKernelArgs& a, const uint8_t* lds, const uint32_t (&coff)[K],
                                            const SampWalkDev* walks, MultiQ<K>& Q, uint32_t& qn, int lane) {
  if (!qn) return;
  __builtin_amdgcn_wave_barrier();
  uint8_t dk = 0, dl = 0;
  double dr = 0;
  uint32_t pos = 0, len = 0;
  if ((uint32_t)lane < qn) {
    pos = Q.pos[lane];
    len = Q.len[lane];
    FoldState s{0.0, 0.0, 0u, 0u};
    const uint32_t err = Q.err[lane];
#pragma unroll
    for (int k = 0; k < K; k++)
      walk_sparse(load_cfg(lds + coff[k]), walks[k], s, err, Q.ep[k][lane], Q.lsat[k][lane], Q.svc[k][lane]);
    walk_finish(s, trace_uniform(Q.hi[lane], Q.lo[lane], a.seed), dk, dl, dr);
    write_rec(a, pos, dk, dl, dr);
  }
  const uint32_t mlen = wave_max_u32((uint32_t)lane < qn ? len : 0u);
  if (mlen <= 32) {
    if ((uint32_t)lane < qn)
      for (uint32_t q = 0; q < len; q++) a.keep[pos + q] = dk;
  } else {
    for (uint32_t e = 0; e < qn; e++) write_keep_range(a, rdl(pos, e), rdl(len, e), (uint8_t)rdl(dk, e), lane);
  }
  __builtin_amdgcn_wave_barrier();
  qn = 0;
}

template <int K>
__global__ __launch_bounds__(kTThreads) __attribute__((amdgpu_waves_per_eu(2, 4))) void trace_multi_kernel(TraceKernelArgs a) {
  extern __shared__ uint4 multi_cfg4[];
  uint8_t* mcfg = reinterpret_cast<uint8_t*>(multi_cfg4);
  __shared__ MultiQ<K> queues[kTWaves];
  __shared__ HeadQ headqs[kTWaves];
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  MultiQ<K>& Q = queues[wv];
  HeadQ& HQ = headqs[wv];
  uint32_t coff[K];
  const uint32_t nsvc = reinterpret_cast<const SampCfgDev*>(a.cfgs[0])->n_services;   // (the engine's: every chunk's)
  const uint32_t* gslot_of;   // LDS: latency-service index of each service, then the service of each index
  const SampWalkDev* wlk;     // LDS: each chunk's rules by what matches them
  {
    // every chunk's table (each <= kSampCfgLds, together <= kMultiCfgLds with
    // the latency-service ids: the host checks) into LDS
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint8_t* g = a.cfgs[k];
      const uint32_t nb = cfg_lds_copy_bytes(g);
      for (uint32_t x = threadIdx.x * 16; x < nb; x += kTThreads * 16)
        *reinterpret_cast<uint4*>(mcfg + o + x) = *reinterpret_cast<const uint4*>(g + x);
      coff[k] = o;
      o += (nb + 15u) & ~15u;
    }
    uint32_t* gl = reinterpret_cast<uint32_t*>(mcfg + o);
    for (uint32_t x = threadIdx.x; x < nsvc + 64; x += kTThreads) gl[x] = a.lat_gslot[x];
    gslot_of = gl;
    o += ((nsvc + 64) * 4 + 15u) & ~15u;
    // each chunk's SampWalkDev (16-byte multiples)
    const uint4* wg = reinterpret_cast<const uint4*>(a.walks);
    uint4* wl = reinterpret_cast<uint4*>(mcfg + o);
    for (uint32_t x = threadIdx.x; x < K * sizeof(SampWalkDev) / 16; x += kTThreads) wl[x] = wg[x];
    wlk = reinterpret_cast<const SampWalkDev*>(mcfg + o);
    __syncthreads();
  }
  const uint32_t* gsvc = gslot_of + nsvc;
  const uint64_t wpw = a.win_per_wave;
  const uint64_t w0 = ((uint64_t)blockIdx.x * kTWaves + wv) * wpw;   // first owned window
  if (w0 >= a.n_windows) return;
  const uint64_t n = a.n_spans;

  const uint64_t range_end = min((w0 + wpw) * kWave, n);
  uint32_t qn = 0, hn = 0;
  bool started = false, open = false;
  uint32_t c_err = 0;
  uint64_t c_pos = 0, c_hi = 0, c_lo = 0, c_kmask = 0;
  Lat cur{0, kInf, 0};   // lane g: the open trace's latency monoid for latency service g
  uint64_t c_ep[K], c_svc[K];
#pragma unroll
  for (int k = 0; k < K; k++) c_ep[k] = c_svc[k] = 0;
  uint64_t base = w0 * kWave;
  StepRaw nx = load_raw(a, base, lane);
  for (;;) {
    StepRaw r = nx;
    const bool valid = base + lane < n;
    const bool hd = step_head(a, r, base, lane);
    const bool work = started || __ballot(hd) != 0;   // wave-uniform: this step is evaluated
    if (work && !r.full) r = load_raw(a, base, lane);
    uint32_t sv = 0xFFFFFFFFu, ss = 0xFFFFFFFFu, gs0 = kNoSlot;
    uint4 rw = make_uint4(0, 0, 0, 0);
    if (valid && work) {
      sv = a.res_svc[r.res];
      ss = a.res_svc_str[r.res];
      if (sv < nsvc) {
        gs0 = gslot_of[sv];
        // route bytes only for a service with latency rules (in some chunk)
        if (gs0 != kNoSlot && r.route.len) rw = head16(a.arena, r.route.off, r.route.len);
      }
    }
    const uint64_t vmask = __ballot(valid);
    const uint64_t hmask = __ballot(hd);
    const bool in_range = base < range_end;
    if (in_range) {
      if (lane == 0 && a.win_heads) a.win_heads[base / kWave] = hmask;
      if (hmask) {
        const uint32_t nh = __popcll(hmask);
        if (hn + nh > kHeadQ) flush_heads(a, HQ, hn, lane);
        if (hd) {
          const uint32_t e = hn + __popcll(hmask & lanemask_lt(lane));
          HQ.cell[e] = (r.lo ^ ((r.hi << 29) | (r.hi >> 35))) * 0x9E3779B97F4A7C15ull;
        }
        hn += nh;
      }
    }
    if (base + kWave < n) nx = load_raw(a, base + kWave, lane, work);   // prefetch the next step
    uint64_t own;
    if (in_range) {
      if (!started) {
        if (!hmask) {   // still inside a trace an earlier wave owns
          base += kWave;
          if (base >= range_end) break;
          continue;
        }
        started = true;
        own = vmask & ~lanemask_lt(ffs64(hmask));
      } else {
        own = vmask;
      }
    } else {
      if (!open) break;
      own = vmask & (hmask ? lanemask_lt(ffs64(hmask)) : ~0ull);
    }
    const uint64_t segmask = (hmask & own) | (open ? 1ull : 0ull);
    const int last_own = fls64(own);
    bool cont_next = false;
    if (last_own == 63 && base + kWave < n) {
      bool h = false;
      if (lane == 63) h = r.ph != r.hi || r.pl != r.lo;   // lane 63 loaded the next step's first id
      cont_next = !rdl((uint32_t)h, 63);
    }
    const bool mine = (own >> lane) & 1;
    const int sst = mine ? fls64(segmask & lanemask_le(lane)) : lane;
    const bool tail = mine && (lane == last_own || ((segmask >> (lane + 1)) & 1));
    const uint64_t tails = __ballot(tail);
    const int t0 = ffs64(tails);
    const bool seg0_cont = open;
    const bool single = t0 == last_own;
    const bool last_open = cont_next && !(single && seg0_cont);
    const int sst_last = rdl((uint32_t)sst, last_own);
    const uint32_t hseg = mine ? (uint32_t)((segmask >> lane) & 1) : 1u;
    const uint32_t rst = (r.status & kStatusReset) ? 1u : 0u;
    const bool carried_tail = (lane == t0 && seg0_cont) || (lane == last_own && last_open);
    const bool ttail = tail && !carried_tail;   // the tail of a trace that opens and closes in this step
    const bool in_closed = mine && !(seg0_cont && lane <= t0) && !(last_open && lane >= sst_last);

    // ---- per-span words of every chunk ----
    const uint32_t gs = mine ? gs0 : kNoSlot;
    uint32_t err = mine && (r.status & ~kStatusReset) == OSE_STATUS_ERROR ? 1u : 0u;
    uint64_t st = 0, en = 0;
    if (gs != kNoSlot) {
      st = r.start;
      en = r.end;
    }
    uint64_t ep[K], svcb[K], lsat[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const Cfg c = load_cfg(mcfg + coff[k]);
      ep[k] = svcb[k] = lsat[k] = 0;
      if (mine && ss < nsvc) svcb[k] = c.svc_bits[ss];
      if (gs != kNoSlot) {
        const uint32_t slot = c.svc_slot[sv];
        if (slot != kNoSlot) ep[k] = endpoint_bits_w(c, slot, a.arena, r.route, rw);
      }
    }
    // ---- latency state, once for every chunk: stretches of one trace and
    // one latency service (a chunk's slots are its services with rules: the
    // same stretches); the stretch tails' threshold tests per chunk ----
    uint64_t n_kmask = 0, smask = 0;
    Lat nxt{0, kInf, 0};
    bool rep = false;
    if (__ballot(gs != kNoSlot)) {
      const uint32_t pgs = dpp_mov<0x138>(kNoSlot, gs);
      const bool shead = !mine || hseg || pgs != gs;
      const uint32_t hs = shead ? 1u : 0u;
      const bool stail = mine && dpp_mov<0x130>(1u, hs) != 0;
      Lat v = gs != kNoSlot ? Lat{(st == 0 || rst) ? 3u : 2u, st == 0 ? kInf : st, en} : Lat{0u, kInf, 0ull};
      seg_lat_scan(hs, v);
      const bool lt = stail && (v.f & 2u);
      if (lt) {
#pragma unroll
        for (int k = 0; k < K; k++) {
          const Cfg c = load_cfg(mcfg + coff[k]);
          const uint32_t slot = c.svc_slot[sv];
          if (slot != kNoSlot) lsat[k] = latency_satisfied(c, slot, ~0ull, v.m, v.e);   // (ORed over the trace below)
        }
      }
      if (gs != kNoSlot) smask = 1ull << gs;
      if (seg0_cont) {   // the carried trace's stretches, in order
        for (uint64_t m0 = __ballot(lt && lane <= t0); m0; m0 &= m0 - 1) {
          const int L = ffs64(m0);
          const uint32_t ks = rdl(gs, L);
          const Lat v0{rdl(v.f, L), rdl64(v.m, L), rdl64(v.e, L)};
          if ((uint32_t)lane == ks) cur = lat_comb(cur, v0);
          c_kmask |= 1ull << ks;
        }
      }
      if (last_open) {   // the open trace's stretches, in order
        for (uint64_t m1 = __ballot(lt && lane >= sst_last); m1; m1 &= m1 - 1) {
          const int L = ffs64(m1);
          const uint32_t ks = rdl(gs, L);
          const Lat v1{rdl(v.f, L), rdl64(v.m, L), rdl64(v.e, L)};
          if ((uint32_t)lane == ks) nxt = lat_comb(nxt, v1);
          n_kmask |= 1ull << ks;
        }
      }
      uint32_t slo = (uint32_t)smask, shi = (uint32_t)(smask >> 32);
      seg_or2n_scan(hseg, slo, shi);
      const uint64_t psm = dpp64<0x138, 0xF>(0ull, (uint64_t)slo | ((uint64_t)shi << 32));   // lane - 1's inclusive bits
      rep = in_closed && shead && !hseg && gs != kNoSlot && ((psm >> gs) & 1);
    }
    // ---- segmented ORs per trace: error, then each chunk's words ----
    seg_or1_scan(hseg, err);
#pragma unroll
    for (int k = 0; k < K; k++) {
      seg_or_scan3(hseg, ep[k], svcb[k], lsat[k]);
      lsat[k] = ttail ? lsat[k] & ep[k] : 0ull;
    }
    if (__ballot(rep)) {
      // a latency service with two or more stretches in a closed trace: its
      // monoid over the whole trace, and its rules' bits replaced per chunk
      uint32_t rlo = rep && gs < 32 ? 1u << gs : 0u, rhi = rep && gs >= 32 && gs != kNoSlot ? 1u << (gs - 32) : 0u;
      seg_or2n_scan(hseg, rlo, rhi);
      const uint64_t rm = (uint64_t)rlo | ((uint64_t)rhi << 32);
      for (uint64_t pend = __ballot(rep); pend;) {
        const uint32_t ks = rdl(gs, ffs64(pend));
        const bool ink = gs == ks;
        pend &= ~__ballot(ink);
        Lat w = ink ? Lat{(st == 0 || rst) ? 3u : 2u, st == 0 ? kInf : st, en} : Lat{0u, kInf, 0ull};
        seg_lat_scan(hseg, w);
        if (ttail && ((rm >> ks) & 1)) {
#pragma unroll
          for (int k = 0; k < K; k++) {
            const Cfg c = load_cfg(mcfg + coff[k]);
            const uint32_t slot = c.svc_slot[gsvc[ks]];
            if (slot != kNoSlot)
              lsat[k] = (lsat[k] & ~c.slot_rules[slot]) | ((w.f & 2u) ? latency_satisfied(c, slot, ep[k], w.m, w.e) : 0ull);
          }
        }
      }
    }
    // ---- queue the carried trace (if it closes) and this step's traces ----
    const bool cont_close = seg0_cont && !(single && cont_next);
    const uint64_t qmask = __ballot(ttail);
    const uint32_t ncl = cont_close ? 1u : 0u, nq = __popcll(qmask);
    if (qn + ncl + nq > (uint32_t)kQ) flush_multi<K>(a, mcfg, coff, wlk, Q, qn, lane);
    const uint32_t qcl = qn;
    const uint32_t qe = qn + ncl + __popcll(qmask & lanemask_lt(lane));
    if (cont_close && lane == 0) {
      Q.err[qcl] = c_err | rdl(err, t0);
      Q.hi[qcl] = c_hi;
      Q.lo[qcl] = c_lo;
      Q.pos[qcl] = (uint32_t)c_pos;
      Q.len[qcl] = (uint32_t)(base + t0 + 1 - c_pos);
    }
    if (ttail) {
      Q.err[qe] = err;
      Q.hi[qe] = r.hi;
      Q.lo[qe] = r.lo;
      Q.pos[qe] = (uint32_t)(base + sst);
      Q.len[qe] = (uint32_t)(lane - sst + 1);
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      if (cont_close) {
        const Cfg c = load_cfg(mcfg + coff[k]);
        const uint64_t EP = c_ep[k] | rdl64(ep[k], t0);
        uint64_t s_l = 0;
        if ((c_kmask >> lane) & 1) {
          const uint32_t slot = c.svc_slot[gsvc[lane]];
          if (slot != kNoSlot) s_l = latency_satisfied(c, slot, EP, cur.m, cur.e);
        }
        s_l = wave_or64(s_l);
        if (lane == 0) {
          Q.ep[k][qcl] = EP;
          Q.lsat[k][qcl] = s_l;
          Q.svc[k][qcl] = c_svc[k] | rdl64(svcb[k], t0);
        }
      }
      if (ttail) {
        Q.ep[k][qe] = ep[k];
        Q.lsat[k][qe] = lsat[k];
        Q.svc[k][qe] = svcb[k];
      }
      // ---- carry into the next step ----
      if (last_open) {
        c_ep[k] = rdl64(ep[k], last_own);
        c_svc[k] = rdl64(svcb[k], last_own);
      } else if (seg0_cont && single && cont_next) {
        c_ep[k] |= rdl64(ep[k], t0);
        c_svc[k] |= rdl64(svcb[k], t0);
      }
    }
    qn += ncl + nq;
    if (cont_close) {
      open = false;
      cur = Lat{0, kInf, 0};
      c_kmask = 0;
    }
    if (last_open) {
      open = true;
      c_pos = base + sst_last;
      c_hi = rdl64(r.hi, sst_last);
      c_lo = rdl64(r.lo, sst_last);
      c_err = rdl(err, last_own);
      cur = nxt;
      c_kmask = n_kmask;
    } else if (seg0_cont && single && cont_next) {
      c_err |= rdl(err, t0);
    }
    base += kWave;
    if (!open && base >= range_end) break;
  }
  flush_multi<K>(a, mcfg, coff, wlk, Q, qn, lane);
  flush_heads(a, HQ, hn, lane);
}

// ---- long runs ------------------------------------------------------------------
// A run the fast path listed (kTraceRuns; still open long_steps steps past
// its owner's windows) is one trace.  Zipf run lengths put most of a batch's
// spans in a few runs, so a run is not one workgroup's work (one workgroup
// per run: C5 0.98 ms, most of it the few workgroups holding 50k-span runs):
//  - trace_long_plan_kernel finds each run's end from the window head masks
//    and cuts it into pieces of at most kLongPiece spans;
//  - trace_long_kernel's waves take the pieces in turn, each on its own (no
//    workgroup barrier): a piece's per-span contributions exactly as
//    trace_eval_kernel computes them, the latency monoid reduced in lane
//    order, then step order; a one-piece run is decided there, a piece of a
//    longer run leaves its partial in long_part;
//  - trace_long_decide_kernel combines each longer run's partials in piece
//    order, decides, and writes the run's keep bytes.
// The partials cross workgroups (and XCDs) through the kernel boundary: a
// release / acquire pair per piece inside one kernel writes back the L2 each
// time (2.8 ms at 1024-span pieces).  C5: 0.98 -> 0.66 ms (profiles/r5l_long_pieces.txt).
// the columns of one span of a long run (loaded two steps ahead)
struct LongRaw {
  uint32_t res, status;
  uint64_t st, en, am, rm, svm;
  ose_strref rt;
};
__device__ __forceinline__ LongRaw long_raw(const TraceKernelArgs& a, const SampCfgDev* h, uint64_t p, uint64_t hi) {
  LongRaw r{};
  if (p >= hi) return r;
  r.res = a.resource[p];
  r.status = a.status[p];
  if (a.start) {
    r.st = a.start[p];
    r.en = a.end[p];
  }
  if (a.attr_match) r.am = chunk_attr_bits(a.attr_match, a.attr_stride, a.attr_words, h, p);
  if (a.svc_match) r.svm = a.svc_match[p];
  if (a.route_match) r.rm = a.route_match[p];
  else if (a.route) r.rt = a.route[p];
  return r;
}

// one wave per listed run: its end (the first head after it), its pieces;
// a workgroup's 16 runs take their piece and partial ranges with one atomic
// each (per-wave atomics on two counters serialised 0.1 ms on C5)
constexpr int kPlanWaves = 16;
__global__ __launch_bounds__(kPlanWaves * kWave) void trace_long_plan_kernel(TraceKernelArgs a) {
  __shared__ uint32_t s_np[kPlanWaves];
  __shared__ uint32_t s_q, s_p;
  const uint32_t nl = __hip_atomic_load(a.n_long, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  for (uint32_t r0 = blockIdx.x * kPlanWaves; r0 < nl; r0 += gridDim.x * kPlanWaves) {
    const uint32_t r = r0 + wv;
    uint64_t pos = 0, end = a.n_spans;
    uint32_t np = 0;
    if (r < nl) {
      pos = a.long_runs[r];
      const uint32_t w0 = (uint32_t)(pos / kWave);
      const uint64_t m0 = a.win_heads[w0] & ~lanemask_le((int)(pos % kWave));
      if (m0) {
        end = (uint64_t)w0 * kWave + ffs64(m0);
      } else {
        for (uint64_t wb = (uint64_t)w0 + 1; wb < a.n_windows; wb += kWave) {
          const uint64_t w = wb + lane;
          const uint64_t h = w < a.n_windows ? a.win_heads[w] : 0ull;
          const uint64_t b = __ballot(h != 0);
          if (b) {
            const int l = (int)ffs64(b);
            end = (wb + l) * kWave + ffs64(rdl64(h, l));
            break;
          }
        }
      }
      np = (uint32_t)((end - pos + kLongPiece - 1) / kLongPiece);
    }
    if (lane == 0) s_np[wv] = np;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tq = 0, tp = 0;
      for (int w = 0; w < kPlanWaves; w++) {
        tq += s_np[w];
        tp += s_np[w] > 1 ? s_np[w] : 0u;
      }
      s_q = tq ? atomicAdd(a.n_long + 1, tq) : 0u;
      s_p = tp ? atomicAdd(a.n_long + 3, tp) : 0u;
    }
    __syncthreads();
    if (r < nl) {
      uint32_t q0 = s_q, pb = s_p;
      for (uint32_t w = 0; w < wv; w++) {
        q0 += s_np[w];
        pb += s_np[w] > 1 ? s_np[w] : 0u;
      }
      if (lane == 0) a.long_meta[r] = make_uint4((uint32_t)end, np, np > 1 ? pb : 0u, 0u);
      for (uint32_t k = lane; k < np; k += kWave) a.long_pieces[q0 + k] = make_uint2(r, k);
    }
    __syncthreads();   // s_np / s_q / s_p are read before the next round's writes
  }
}

constexpr int kLWaves = 8;
constexpr int kLThreads = kLWaves * kWave;
struct LongPart {   // kLongPartBytes
  uint64_t m[kWave], e[kWave];
  uint32_t f[kWave];
  uint64_t ep, svc, kmask;
  uint32_t err;
  uint32_t _pad[9];   // 21 cache lines
};
static_assert(sizeof(LongPart) == kLongPartBytes, "long-run partial layout");
// keep bytes [x0, x1) = k, 16-byte stores in the aligned middle
__device__ __forceinline__ void long_keep_fill(uint8_t* keep, uint64_t x0, uint64_t x1, uint8_t k, int lane) {
  const uint64_t b = reinterpret_cast<uintptr_t>(keep);
  const uint64_t a0 = min(x1, ((b + x0 + 15) & ~15ull) - b), a1 = max(a0, ((b + x1) & ~15ull) - b);
  for (uint64_t x = x0 + lane; x < a0; x += kWave) keep[x] = k;
  const uint32_t k4 = k * 0x01010101u;
  for (uint64_t x = a0 + 16ull * lane; x < a1; x += 16ull * kWave) *reinterpret_cast<uint4*>(keep + x) = make_uint4(k4, k4, k4, k4);
  for (uint64_t x = a1 + lane; x < x1; x += kWave) keep[x] = k;
}
// a long run's decision (wave-wide: lane k holds latency slot k's monoid)
// and its keep bytes
__device__ __forceinline__ void long_decide(const TraceKernelArgs& a, const Cfg& c, int lane, uint64_t pos, uint64_t end,
                                            uint32_t E, uint64_t EP, uint64_t SV, uint64_t K, const Lat& tot) {
  uint64_t s_l = 0;
  if ((K >> lane) & 1) s_l = latency_satisfied(c, (uint32_t)lane, EP, tot.m, tot.e);
  s_l = wave_or64(s_l);
  uint32_t dk32 = 0;
  if (lane == 0) {
    const uint4 t = reinterpret_cast<const uint4*>(a.tid)[pos];
    uint8_t dk = 0, dl = 0;
    double dr = 0;
    decide_at(a, c, pos, E, EP, s_l, SV,
              trace_uniform((uint64_t)t.x | ((uint64_t)t.y << 32), (uint64_t)t.z | ((uint64_t)t.w << 32), a.seed), dk, dl,
              dr);
    write_rec(a, pos, dk, dl, dr);
    dk32 = dk;
  }
  long_keep_fill(a.keep, pos, end, (uint8_t)rdl(dk32, 0), lane);
}
// Each wave takes pieces in turn, on its own (no workgroup barrier after
// the table copy): a piece's latency chain overlaps the other waves' folds
__global__ __launch_bounds__(kLThreads) void trace_long_kernel(TraceKernelArgs a) {
  const uint32_t npieces = __hip_atomic_load(a.n_long + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x * kLWaves >= npieces) return;
  __shared__ __attribute__((aligned(16))) uint8_t cfg_lds[kSampCfgLds];
  {
    const uint32_t nb = cfg_lds_copy_bytes(a.cfg);
    for (uint32_t k = threadIdx.x * 16; k < nb; k += kLThreads * 16)
      *reinterpret_cast<uint4*>(cfg_lds + k) = *reinterpret_cast<const uint4*>(a.cfg + k);
    __syncthreads();   // every wave reads the tables (n_services, n_lat below) after the copy
  }
  const Cfg c = load_cfg(cfg_lds);
  const int lane = threadIdx.x & 63;
  const uint32_t nsvc = c.h->n_services;
  const bool want_route = c.h->n_lat && !a.route_match && a.route;
  const uint32_t stride = gridDim.x * kLWaves;
  for (uint32_t q = blockIdx.x * kLWaves + (threadIdx.x >> 6); q < npieces; q += stride) {
    const uint2 pk = a.long_pieces[q];
    const uint4 meta = a.long_meta[pk.x];   // {end, pieces, first partial, pieces done}
    const uint64_t pos = a.long_runs[pk.x], end = meta.x;
    const uint64_t lo = pos + (uint64_t)pk.y * kLongPiece, hi = min(end, lo + kLongPiece);
    uint32_t err = 0;
    uint64_t ep_acc = 0, svc_acc = 0, kmask = 0;
    Lat cur{0, kInf, 0};   // lane k: latency slot k
    // two steps of columns in flight, the service ids of the next step
    // gathered a step ahead: a step's route head waits on nothing of its own
    LongRaw r0 = long_raw(a, c.h, lo + lane, hi), r1 = long_raw(a, c.h, lo + kWave + lane, hi);
    uint32_t nsv = 0xFFFFFFFFu, nss = 0xFFFFFFFFu;
    if (lo + lane < hi) {
      nsv = a.res_svc[r0.res];
      nss = a.res_svc_str[r0.res];
    }
    for (uint64_t base = lo; base < hi; base += kWave) {
      const uint64_t p = base + lane;
      const bool valid = p < hi;
      const LongRaw r = r0;
      const uint32_t sv = nsv, ss = nss;
      uint4 rw = make_uint4(0, 0, 0, 0);
      if (valid && want_route && r.rt.len && sv < nsvc && c.svc_slot[sv] != kNoSlot)
        rw = head16(a.arena, r.rt.off, r.rt.len);
      r0 = r1;
      if (base + 2 * kWave < hi) r1 = long_raw(a, c.h, p + 2 * kWave, hi);
      if (p + kWave < hi) {
        nsv = a.res_svc[r0.res];
        nss = a.res_svc_str[r0.res];
      }
      uint32_t slot = kNoSlot;
      uint64_t st = 0, en = 0;
      const uint32_t rst = (r.status & kStatusReset) ? 1u : 0u;
      if (valid) {
        err |= (r.status & ~kStatusReset) == OSE_STATUS_ERROR;
        if (a.svc_match) {
          svc_acc |= r.svm;
        } else {
          if (ss < nsvc) svc_acc |= c.svc_bits[ss];
          svc_acc |= r.am;
        }
        if (sv < nsvc) {
          slot = c.svc_slot[sv];
          if (slot != kNoSlot) {
            ep_acc |= a.route_match ? r.rm & c.slot_rules[slot] : endpoint_bits_w(c, slot, a.arena, r.rt, rw);
            st = r.st;
            en = r.en;
          }
        }
      }
      uint64_t pend = __ballot(slot != kNoSlot);
      while (pend) {
        const uint32_t ks = rdl(slot, ffs64(pend));
        const bool ink = slot == ks;
        pend &= ~__ballot(ink);
        Lat v = ink ? Lat{(st == 0 || rst) ? 3u : 2u, st == 0 ? kInf : st, en} : Lat{0u, kInf, 0ull};
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {   // lane-order reduction into lane 0
          Lat o;
          o.f = __shfl_down(v.f, d, kWave);
          o.m = __shfl_down(v.m, d, kWave);
          o.e = __shfl_down(v.e, d, kWave);
          if ((lane & (2 * d - 1)) == 0) v = lat_comb(v, o);
        }
        const Lat v0{rdl(v.f, 0), rdl64(v.m, 0), rdl64(v.e, 0)};
        if ((uint32_t)lane == ks) cur = lat_comb(cur, v0);
        kmask |= 1ull << ks;
      }
    }
    uint32_t E = __ballot(err != 0) ? 1u : 0u;
    uint64_t EP = wave_or64(ep_acc), SV = wave_or64(svc_acc), K = kmask;
    Lat tot = cur;
    if (meta.y > 1) {   // trace_long_decide_kernel combines the run's partials
      LongPart* part = reinterpret_cast<LongPart*>(a.long_part + (size_t)kLongPartBytes * (meta.z + pk.y));
      part->m[lane] = tot.m;
      part->e[lane] = tot.e;
      part->f[lane] = tot.f;
      if (lane == 0) {
        part->ep = EP;
        part->svc = SV;
        part->kmask = K;
        part->err = E;
      }
      continue;
    }
    long_decide(a, c, lane, pos, end, E, EP, SV, K, tot);
  }
}

// one wave per run of several pieces: its partials in piece order, the
// decision, the run's keep bytes
__global__ __launch_bounds__(kPlanWaves * kWave) void trace_long_decide_kernel(TraceKernelArgs a) {
  const uint32_t nl = __hip_atomic_load(a.n_long, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x * kPlanWaves >= nl) return;
  __shared__ __attribute__((aligned(16))) uint8_t cfg_lds[kSampCfgLds];
  {
    const uint32_t nb = cfg_lds_copy_bytes(a.cfg);
    for (uint32_t k = threadIdx.x * 16; k < nb; k += kPlanWaves * kWave * 16)
      *reinterpret_cast<uint4*>(cfg_lds + k) = *reinterpret_cast<const uint4*>(a.cfg + k);
    __syncthreads();
  }
  const Cfg c = load_cfg(cfg_lds);
  const int lane = threadIdx.x & 63;
  for (uint32_t r = blockIdx.x * kPlanWaves + (threadIdx.x >> 6); r < nl; r += gridDim.x * kPlanWaves) {
    const uint4 meta = a.long_meta[r];
    if (meta.y <= 1) continue;
    uint32_t E = 0;
    uint64_t EP = 0, SV = 0, K = 0;
    Lat tot{0, kInf, 0};
    const LongPart* pp = reinterpret_cast<const LongPart*>(a.long_part + (size_t)kLongPartBytes * meta.z);
    for (uint32_t k0 = 0; k0 < meta.y; k0 += 4) {   // piece order, 4 partials' loads in flight
      uint64_t kk[4], m[4], e[4];
      uint32_t f[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const LongPart& q = pp[k0 + j < meta.y ? k0 + j : k0];
        kk[j] = k0 + j < meta.y ? q.kmask : 0ull;
        E |= q.err;
        EP |= q.ep;
        SV |= q.svc;
        f[j] = q.f[lane];
        m[j] = q.m[lane];
        e[j] = q.e[lane];
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        K |= kk[j];
        if ((kk[j] >> lane) & 1) tot = lat_comb(tot, Lat{f[j], m[j], e[j]});
      }
    }
    long_decide(a, c, lane, a.long_runs[r], meta.x, E, EP, SV, K, tot);
  }
}

// ---- slow path ---------------------------------------------------------------
__device__ __forceinline__ bool gated(const uint32_t* g) {
  return g && __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

// Exact table of the slow path: every run head inserts its full trace id
// (table_insert's publish protocol); a trace's entry keeps its smallest
// run-head position.
// Gated kernels use a grid-stride loop over a capped grid: when the gate is
// closed (the common case) the launch costs a few microseconds, not one
// block per 256 spans.
constexpr uint32_t kGatedBlocks = 2048;
__global__ __launch_bounds__(256) void trace_insert_exact_kernel(TraceKernelArgs a) {
  if (__hip_atomic_load(a.dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < a.n_spans; p += (uint64_t)gridDim.x * 256) {
    const uint64_t hi = a.tid[2 * p], lo = a.tid[2 * p + 1];
    if (p > 0 && a.tid[2 * p - 2] == hi && a.tid[2 * p - 1] == lo) continue;
    (void)table_insert(a, hi, lo, (uint32_t)p);   // gated on *dup: already set
  }
}

// ---- run-list path ---------------------------------------------------------
// A batch with repeated trace ids (resource-shuffled input, or the records a
// trace's owner GPU receives from several sources) usually holds each trace
// in a few runs.  trace_runs_kernel inserts every run head (the window head
// masks of the fast pass) into the exact table and lists the run in the
// trace's slot; trace_fold_kernel then folds, for every trace with 2 or
// more runs, its runs in batch order on one lane (exactly the fold
// trace_eval_kernel does over a contiguous trace), decides and writes keep
// over all its runs.  Traces with more than kMaxRuns runs, more than
// kMaxFoldSpans spans or more than kMaxFoldSlots latency services set
// *overflow, and the sort-based path (gated on it) recomputes the batch.
__global__ __launch_bounds__(256) void trace_runs_kernel(TraceKernelArgs a) {
  if (__hip_atomic_load(a.dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  if (a.path_count && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.path_count, 1ull);
  const int lane = threadIdx.x & 63;
  for (uint64_t w = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / kWave; w < a.n_windows;
       w += (uint64_t)gridDim.x * (256 / kWave)) {
    const uint64_t heads = a.win_heads[w];
    const uint64_t p = w * kWave + lane;
    if (!((heads >> lane) & 1) || p >= a.n_spans) continue;
    const uint64_t hi = a.tid[2 * p], lo = a.tid[2 * p + 1];
    uint64_t slot = ~0ull;
    const int ins = table_insert(a, hi, lo, (uint32_t)p, &slot);   // gated on *dup: not set again
    if (ins == kInsFail || slot == ~0ull) {   // table full / spin gave up: error already flagged
      atomicOr(a.overflow, 1u);
      continue;
    }
    if (ins == kInsFound) {   // a later run: append (the claiming lane listed the first)
      const uint32_t k = atomicAdd(&a.run_count[slot], 1u);
      if (k < kMaxRuns) a.runs[slot * kMaxRuns + k] = (uint32_t)p;
      else atomicOr(a.overflow, 1u);
    }
    a.head_slot[p] = (uint32_t)slot;
  }
}

// end of the run starting at head position p: the next head after it
__device__ __forceinline__ uint64_t run_end(const TraceKernelArgs& a, uint64_t p) {
  uint64_t w = p / kWave;
  uint64_t m = a.win_heads[w] & ~lanemask_le((int)(p % kWave));
  while (!m) {
    if (++w >= a.n_windows) return a.n_spans;
    m = a.win_heads[w];
  }
  return w * kWave + (uint64_t)ffs64(m);
}

__global__ __launch_bounds__(kTThreads) void trace_fold_kernel(TraceKernelArgs a) {
  if (__hip_atomic_load(a.dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  // the sort-based path already has the batch (it redoes every trace)
  if (__hip_atomic_load(a.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  __shared__ __attribute__((aligned(16))) uint8_t cfg_lds[kSampCfgLds];
  {
    const uint32_t nb = cfg_lds_copy_bytes(a.cfg);
    for (uint32_t k = threadIdx.x * 16; k < nb; k += kTThreads * 16)
      *reinterpret_cast<uint4*>(cfg_lds + k) = *reinterpret_cast<const uint4*>(a.cfg + k);
    __syncthreads();
  }
  const Cfg c = load_cfg(cfg_lds);
  const uint32_t nsvc = c.h->n_services;
  const bool want_route = c.h->n_lat && !a.route_match && a.route;
  const int lane = threadIdx.x & 63;
  for (uint64_t w = ((uint64_t)blockIdx.x * kTThreads + threadIdx.x) / kWave; w < a.n_windows;
       w += (uint64_t)gridDim.x * kTWaves) {
    const uint64_t heads = a.win_heads[w];
    const uint64_t p = w * kWave + lane;
    const bool head = ((heads >> lane) & 1) && p < a.n_spans;
    uint32_t slot = 0, nr = 0;
    bool first = false;
    if (head) {
      slot = a.head_slot[p];
      first = a.table[slot].first == (uint32_t)p;
      nr = __hip_atomic_load(&a.run_count[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint64_t fm = __ballot(first);
    if (lane == 0) a.win_first[w] = fm;
    if (!first || nr < 2 || nr > kMaxRuns) continue;   // one run: the fast pass decided it
    // the trace's runs in batch order
    uint32_t rs[kMaxRuns];
#pragma unroll
    for (uint32_t k = 0; k < kMaxRuns; k++) rs[k] = k < nr ? a.runs[(uint64_t)slot * kMaxRuns + k] : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t k = 1; k < kMaxRuns; k++)   // insertion sort, unrolled (nr <= 8)
#pragma unroll
      for (uint32_t j = k; j > 0; j--)
        if (rs[j - 1] > rs[j]) { const uint32_t t = rs[j]; rs[j] = rs[j - 1]; rs[j - 1] = t; }
    uint32_t err = 0, nslots = 0;
    uint64_t ep = 0, svcb = 0, spans = 0;
    uint32_t ks[kMaxFoldSlots];
    Lat ls[kMaxFoldSlots];
    bool over = false;
    for (uint32_t r = 0; r < nr && !over; r++) {
      const uint64_t s0 = rs[r], s1 = run_end(a, s0);
      spans += s1 - s0;
      if (spans > kMaxFoldSpans) { over = true; break; }
      for (uint64_t q = s0; q < s1; q++) {
        const uint32_t res = a.resource[q], stt = a.status[q];
        err |= (stt & ~kStatusReset) == OSE_STATUS_ERROR;
        const uint32_t sv = a.res_svc[res];
        if (a.svc_match) {
          svcb |= a.svc_match[q];
        } else {
          const uint32_t ss = a.res_svc_str[res];
          if (ss < nsvc) svcb |= c.svc_bits[ss];
          if (a.attr_match) svcb |= chunk_attr_bits(a.attr_match, a.attr_stride, a.attr_words, c.h, q);
        }
        if (sv >= nsvc) continue;
        const uint32_t slt = c.svc_slot[sv];
        if (slt == kNoSlot) continue;
        ep |= a.route_match ? a.route_match[q] & c.slot_rules[slt]
                            : (want_route ? endpoint_bits(c, slt, a.arena, a.route[q]) : 0ull);
        const uint64_t st = a.start ? a.start[q] : 0, en = a.end ? a.end[q] : 0;
        const Lat v{(st == 0 || (stt & kStatusReset)) ? 3u : 2u, st == 0 ? kInf : st, en};
        uint32_t k = 0;
        while (k < nslots && ks[k] != slt) k++;
        if (k == nslots) {
          if (nslots == kMaxFoldSlots) { over = true; break; }
          ks[nslots] = slt;
          ls[nslots] = Lat{0u, kInf, 0ull};
          nslots++;
        }
        ls[k] = lat_comb(ls[k], v);
      }
    }
    if (over) {
      atomicOr(a.overflow, 1u);
      continue;
    }
    uint64_t lsat = 0;
    for (uint32_t k = 0; k < nslots; k++)
      if (ls[k].f & 2u) lsat |= latency_satisfied(c, ks[k], ep, ls[k].m, ls[k].e);
    const uint64_t hi = a.tid[2 * p], lo = a.tid[2 * p + 1];
    uint8_t dk = 0, dl = 0;
    double dr = 0;
    decide_at(a, c, p, err, ep, lsat, svcb, trace_uniform(hi, lo, a.seed), dk, dl, dr);
    write_rec(a, p, dk, dl, dr);
    for (uint32_t r = 0; r < nr; r++) {
      const uint64_t s0 = rs[r], s1 = run_end(a, s0);
      for (uint64_t q = s0; q < s1; q++) a.keep[q] = dk;
    }
  }
}

// the per-trace outputs list first runs only, unless the sort-based path
// (gated on *overflow) rewrites the head masks itself
__global__ __launch_bounds__(256) void trace_first_select_kernel(TraceKernelArgs a) {
  if (__hip_atomic_load(a.dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  if (__hip_atomic_load(a.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < a.n_windows; w += (uint64_t)gridDim.x * 256)
    a.win_heads[w] = a.win_first[w];
}

// key[i] = first run-head position of span i's trace_id (read-only probe of
// the table the fast path filled).
__global__ __launch_bounds__(256) void trace_key_kernel(TraceSortArgs a) {
  if (gated(a.gate)) return;
  if (a.path_count && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.path_count + 1, 1ull);
  const uint32_t ready = (a.epoch << 2) | 2u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n_spans; i += (uint64_t)gridDim.x * 256) {
    const uint64_t hi = a.tid[2 * i], lo = a.tid[2 * i + 1];
    uint64_t h = tid_hash(hi, lo) & a.table_mask;
    bool found = false;
    for (uint64_t probes = 0; probes <= a.table_mask; probes++) {
      const TraceSlot& s = a.table[h];
      if (s.state == ready && s.hi == hi && s.lo == lo) {
        a.key[i] = s.first;
        found = true;
        break;
      }
      if ((s.state >> 2) != a.epoch) break;
      h = (h + 1) & a.table_mask;
    }
    if (!found) {
      atomicOr(a.error, 4u);
      a.key[i] = 0;
    }
  }
}

constexpr int kSortThreads = 256;
constexpr int kSortRounds = kSortTile / kSortThreads;

__global__ __launch_bounds__(kSortThreads) void sort_hist_kernel(TraceSortArgs a) {
  if (gated(a.gate)) return;
  __shared__ uint32_t hist[256];
  const int t = threadIdx.x;
  if (a.scan_status) {
    for (uint32_t k = blockIdx.x * kSortThreads + t; k < a.scan_status_n; k += gridDim.x * kSortThreads)
      a.scan_status[k] = 0;
    if (blockIdx.x == 0 && t == 0) *a.scan_counter = 0;
  }
  hist[t] = 0;
  __syncthreads();
  const uint32_t* keys = a.keys_in ? a.keys_in : a.key;
  const uint64_t b = (uint64_t)blockIdx.x * kSortTile;
  for (int r = 0; r < kSortRounds; r++) {
    const uint64_t j = b + (uint64_t)r * kSortThreads + t;
    if (j < a.n_spans) atomicAdd(&hist[(keys[j] >> a.shift) & 255u], 1u);
  }
  __syncthreads();
  a.hist[(uint64_t)t * a.n_tiles + blockIdx.x] = hist[t];
}

// Stable scatter: items keep tile order (round-major, lane order inside a
// wave); ranks among equal digits come from per-wave match masks (8 ballots)
// and per-round wave offsets in LDS.
__global__ __launch_bounds__(kSortThreads) void sort_scatter_kernel(TraceSortArgs a) {
  if (gated(a.gate)) return;
  __shared__ uint32_t goff[256], run[256];
  __shared__ uint32_t wcnt[kSortThreads / kWave][256], woff[kSortThreads / kWave][256];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  goff[t] = a.hist[(uint64_t)t * a.n_tiles + blockIdx.x];
  run[t] = 0;
  for (int k = 0; k < kSortThreads / kWave; k++) wcnt[k][t] = 0;
  __syncthreads();
  const uint32_t* keys = a.keys_in ? a.keys_in : a.key;
  const uint64_t b = (uint64_t)blockIdx.x * kSortTile;
  for (int r = 0; r < kSortRounds; r++) {
    const uint64_t j = b + (uint64_t)r * kSortThreads + t;
    const bool valid = j < a.n_spans;
    const uint32_t k = valid ? keys[j] : 0;
    const uint32_t v = valid ? (a.vals_in ? a.vals_in[j] : (uint32_t)j) : 0;
    const uint32_t d = (k >> a.shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; bit++) {
      const uint64_t bal = __ballot((d >> bit) & 1u);
      peers &= ((d >> bit) & 1u) ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lanemask_lt(lane));
    const uint32_t cnt = __popcll(peers);
    if (valid && rank == cnt - 1) wcnt[wv][d] = cnt;
    __syncthreads();
    {
      uint32_t acc = run[t];
      for (int k2 = 0; k2 < kSortThreads / kWave; k2++) {
        woff[k2][t] = acc;
        acc += wcnt[k2][t];
        wcnt[k2][t] = 0;
      }
      run[t] = acc;
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = goff[d] + woff[wv][d] + rank;
      a.keys_out[pos] = k;
      a.vals_out[pos] = v;
    }
  }
}

// ---- exclusive scan of u32 counts --------------------------------------------
__global__ __launch_bounds__(kScanTileItems) void scan_u32_kernel(ScanArgs a) {
  if (gated(a.gate)) return;
  __shared__ uint64_t wsum[kScanTileItems / kWave];
  __shared__ uint64_t prefix;
  __shared__ uint32_t tile_s;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) tile_s = atomicAdd(a.counter, 1u);
  __syncthreads();
  const uint32_t tile = tile_s;
  const uint64_t k = (uint64_t)tile * kScanTileItems + t;
  uint64_t v = 0;
  if (k < a.n)
    v = a.popcount ? (uint64_t)__popcll(static_cast<const uint64_t*>(a.in)[k]) : static_cast<const uint32_t*>(a.in)[k];
  uint64_t incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint64_t x = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += x;
  }
  if (lane == kWave - 1) wsum[wv] = incl;
  __syncthreads();
  uint64_t wbase = 0, total = 0;
#pragma unroll
  for (int q = 0; q < kScanTileItems / kWave; q++) {
    const uint64_t x = wsum[q];
    if (q < wv) wbase += x;
    total += x;
  }
  if (wv == 0) {
    const uint64_t pfx = lookback_prefix(a.status, tile, total, a.error);
    if (lane == 0) {
      prefix = pfx;
      if (tile == a.n_tiles - 1 && a.total) *a.total = (uint32_t)(pfx + total);
    }
  }
  __syncthreads();
  if (k < a.n) a.out[k] = (uint32_t)(prefix + wbase + incl - v);
}

// ---- dense per-trace outputs ---------------------------------------------------
__global__ __launch_bounds__(kTThreads) void trace_compact_kernel(TraceCompactArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x * kTWaves + (threadIdx.x >> 6);
  if (w >= a.n_windows) return;
  const uint64_t heads = a.win_heads[w];
  if (!((heads >> lane) & 1)) return;
  const uint32_t t = a.win_base[w] + __popcll(heads & lanemask_lt(lane));
  const TraceRec r = a.rec[(uint64_t)w * kWave + lane];
  if (a.trace_first_span) a.trace_first_span[t] = r.first_span;
  if (a.trace_keep) a.trace_keep[t] = r.keep;
  if (a.trace_level) a.trace_level[t] = r.level;
  if (a.trace_ratio) a.trace_ratio[t] = r.ratio;
}

// ---- trace-id exchange ---------------------------------------------------------
// Partial records (include/odigos_amd.h "trace-id exchange"): the source
// folds each stretch of its batch that shares a trace id and a latency
// service (and lies in one 64-span step) into one record, so the owner GPU
// receives one record per stretch instead of one per span.  The record is
// the stretch's share of what trace_eval_kernel combines per trace: the
// error bit, the latency monoid element (reset, min start after the last
// reset, max end) of its service, and per rule chunk the endpoint
// (HasPrefix) bits and the service_name / span_attribute bits of that
// chunk's tables.  The owner folds records in (source rank, source order),
// which is the global batch order restricted to the trace, so the fold
// equals the single-GPU one (the monoid is associative, the rest are ORs),
// chunk by chunk.
constexpr uint32_t kXNone = 0xFFFFFFu;   // 24-bit "no latency service"
constexpr uint32_t kXErr = 1u, kXLat = 2u, kXReset = 4u;
__device__ __forceinline__ uint32_t shard_owner(uint64_t hi, uint64_t lo, uint32_t n) {
  return (uint32_t)((tid_hash(hi, lo) >> 32) % n);
}

// one span of a 64-span step: its trace id and latency service (the record
// boundary test) and, with `full`, its chunk-independent contributions.
// XRaw holds the span's column loads, issued one step ahead of their use
// (a wave walks its chunk's steps in order, two steps of loads in flight).
struct XRaw {
  uint4 t;
  uint32_t res, status;
  uint64_t st, en;
  ose_strref rt;
};
__device__ __forceinline__ XRaw x_load(const ShardArgs& a, uint64_t j, bool full) {
  XRaw r{};
  if (j >= a.n_spans) return r;
  r.t = reinterpret_cast<const uint4*>(a.tid)[j];
  r.res = a.resource[j];
  if (!full) return r;
  r.status = a.status[j];
  if (a.start) r.st = a.start[j];
  if (a.end) r.en = a.end[j];
  if (a.route && !a.route_match) r.rt = a.route[j];
  return r;
}
struct XSpan {
  bool valid;
  uint64_t hi, lo;
  uint32_t sv, res, err;
  uint64_t st, en;
  ose_strref rt;
};
__device__ __forceinline__ XSpan x_span(const ShardArgs& a, uint32_t nsvc, const XRaw& r, uint64_t j, bool full) {
  XSpan x{};
  x.valid = j < a.n_spans;
  x.sv = kXNone;
  if (!x.valid) return x;
  x.hi = (uint64_t)r.t.x | ((uint64_t)r.t.y << 32);
  x.lo = (uint64_t)r.t.z | ((uint64_t)r.t.w << 32);
  x.res = r.res;
  const uint32_t s = a.res_svc[x.res];   // global id (nsvc = the engine's interned services)
  if (s < nsvc && ((a.lat_svc[s >> 5] >> (s & 31)) & 1u)) x.sv = s;
  if (!full) return x;
  x.err = r.status == OSE_STATUS_ERROR;
  if (x.sv != kXNone) {
    x.st = r.st;
    x.en = r.en;
  }
  x.rt = r.rt;
  return x;
}
// the span's endpoint bits and rule bits under rule chunk k's tables
__device__ __forceinline__ void x_chunk(const ShardArgs& a, const Cfg& c, const XSpan& x, uint64_t j, uint32_t k,
                                        uint64_t& ep, uint64_t& svcb) {
  ep = svcb = 0;
  if (!x.valid) return;
  const uint32_t nsvc = c.h->n_services;
  // chunk-local tables: global ids through the chunk's map (ids past the
  // engine's services and ids the chunk does not name map to none)
  const uint32_t* map = a.svc_maps ? a.svc_maps[k] : nullptr;
  const uint32_t sg = a.res_svc_str[x.res];
  const uint32_t ss = map ? (sg < a.n_global_svc ? map[sg] : kXNone) : sg;
  svcb = ss < nsvc ? c.svc_bits[ss] : 0;
  if (a.attr_match) svcb |= chunk_attr_bits(a.attr_match, a.attr_stride, a.attr_words, c.h, j);
  const uint32_t sv = map && x.sv != kXNone ? map[x.sv] : x.sv;
  if (sv < nsvc) {
    const uint32_t slot = c.svc_slot[sv];
    if (slot != kNoSlot)
      ep = a.route_match ? a.route_match[(uint64_t)k * a.rm_stride + j] & c.slot_rules[slot]
                         : endpoint_bits(c, slot, a.arena, x.rt);
  }
}
// record heads of the step (lane 0 always starts one) and tails (where a
// record's folded value sits after the inclusive segmented scans)
__device__ __forceinline__ void x_bounds(const XSpan& x, int lane, uint64_t& heads, uint64_t& tails) {
  const uint64_t ph = __shfl_up(x.hi, 1, kWave), pl = __shfl_up(x.lo, 1, kWave);
  const uint32_t ps = __shfl_up(x.sv, 1, kWave);
  const bool head = x.valid && (lane == 0 || ph != x.hi || pl != x.lo || ps != x.sv);
  const uint64_t vm = __ballot(x.valid);
  heads = __ballot(head);
  const uint64_t nxt = (heads | ~vm) >> 1 | (1ull << 63);   // bit l: span l+1 starts a record or is past the end
  tails = vm & nxt;
}

// Each wave packs one chunk of kXSteps consecutive 64-span steps, with no
// block barriers: shard_hist_kernel counts the chunk's records per owner,
// a scan over (owner, chunk) gives every (owner, chunk) its first slot, and
// shard_scatter_kernel writes the records in source order (chunks, steps,
// lanes), each wave advancing its own per-owner offsets (lane d: owner d).
// The first form interleaved a block's four waves step by step and ranked
// their records per owner through LDS with two block barriers per step.
__global__ __launch_bounds__(kSortThreads) void shard_hist_kernel(ShardArgs a) {
  __shared__ uint32_t hist[kSortThreads / kWave][64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t ch = blockIdx.x * (kSortThreads / kWave) + wv;
  if (ch >= a.n_tiles) return;   // wave-uniform; no block barriers below
  hist[wv][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t nsvc = a.n_global_svc;
  const uint64_t b0 = (uint64_t)ch * kXChunk;
  XRaw nx = x_load(a, b0 + lane, false);
  for (uint32_t s = 0; s < kXSteps; s++) {
    const uint64_t base = b0 + (uint64_t)s * kWave;
    if (base >= a.n_spans) break;   // wave-uniform
    const XRaw cur = nx;
    if (s + 1 < kXSteps) nx = x_load(a, base + kWave + lane, false);
    const XSpan x = x_span(a, nsvc, cur, base + lane, false);
    uint64_t heads, tails;
    x_bounds(x, lane, heads, tails);
    if ((tails >> lane) & 1) atomicAdd(&hist[wv][shard_owner(x.hi, x.lo, a.n_ranks)], 1u);
  }
  __builtin_amdgcn_wave_barrier();
  if ((uint32_t)lane < a.n_ranks) a.hist[(uint64_t)lane * a.n_tiles + ch] = hist[wv][lane];
}
// records per owner from the scanned (owner, chunk) offsets (a device-scope
// atomic per wave and owner on n_ranks words serialised the count pass)
__global__ __launch_bounds__(64) void shard_counts_kernel(ShardArgs a) {
  const uint32_t d = threadIdx.x;
  if (d >= a.n_ranks) return;
  const uint64_t T = a.n_tiles;
  const uint32_t lo = a.hoff[d * T];
  const uint32_t hi = d + 1 < a.n_ranks ? a.hoff[(d + 1) * T] : a.hoff[d * T + T - 1] + a.hist[d * T + T - 1];
  a.counts[d] = hi - lo;
}

// The records in source order; pack_pos[span] = its record's slot in `send`.
// The rule chunks' tables are copied into LDS first (cfg_lds_bytes, when
// they fit): the endpoint tests and service lookups of every span are then
// ds_reads, as in trace_eval_kernel.
__global__ __launch_bounds__(kSortThreads) void shard_scatter_kernel(ShardArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t xcfg[];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (a.cfg_lds_bytes) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < a.n_chunks; k++) {
      const uint8_t* src = a.cfgs[k];
      const uint32_t nb = (cfg_lds_copy_bytes(src) + 15u) & ~15u;
      for (uint32_t q = (uint32_t)t * 16; q < nb; q += kSortThreads * 16)
        *reinterpret_cast<uint4*>(xcfg + off + q) = *reinterpret_cast<const uint4*>(src + q);
      off += nb;
    }
    __syncthreads();
  }
  const uint32_t ch = blockIdx.x * (kSortThreads / kWave) + wv;
  if (ch >= a.n_tiles) return;   // wave-uniform; no block barriers below
  uint32_t off = (uint32_t)lane < a.n_ranks ? a.hoff[(uint64_t)lane * a.n_tiles + ch] : 0u;
  const uint32_t nsvc = a.n_global_svc;
  const uint32_t words = x_rec_words(a.n_chunks);
  const uint64_t b0 = (uint64_t)ch * kXChunk;
  XRaw nx = x_load(a, b0 + lane, true);
  for (uint32_t s = 0; s < kXSteps; s++) {
    const uint64_t base = b0 + (uint64_t)s * kWave;
    if (base >= a.n_spans) break;   // wave-uniform
    const XRaw cur = nx;
    if (s + 1 < kXSteps) nx = x_load(a, base + kWave + lane, true);
    const XSpan x = x_span(a, nsvc, cur, base + lane, true);
    uint64_t heads, tails;
    x_bounds(x, lane, heads, tails);
    const bool tail = (tails >> lane) & 1;
    // fold each record (inclusive segmented scans; invalid lanes are lone segments)
    const uint32_t h = x.valid ? (uint32_t)((heads >> lane) & 1) : 1u;
    uint32_t err = x.err;
    Lat v = x.sv != kXNone ? Lat{x.st == 0 ? 3u : 2u, x.st == 0 ? kInf : x.st, x.en} : Lat{0u, kInf, 0ull};
    {
      uint64_t z0 = 0, z1 = 0;
      seg_or_scan(h, err, z0, z1);
      seg_lat_scan(h, v);
    }
    // slot: the owner's running offset + rank among this step's records of that owner
    const uint32_t d = tail ? shard_owner(x.hi, x.lo, a.n_ranks) : 0u;
    uint32_t pos = __shfl(off, (int)d, kWave);
    uint64_t mine = 0;
    for (uint32_t o = 0; o < a.n_ranks; o++) {
      const uint64_t bo = __ballot(tail && d == o);
      if (d == o) mine = bo;
      if ((uint32_t)lane == o) off += (uint32_t)__popcll(bo);
    }
    pos += (uint32_t)__popcll(mine & lanemask_lt(lane));
    uint64_t* rec = nullptr;
    if (tail) {
      rec = reinterpret_cast<uint64_t*>(a.send) + (uint64_t)pos * words;
      const uint32_t flags = (err ? kXErr : 0u) | ((v.f & 2u) ? kXLat : 0u) | ((v.f & 1u) ? kXReset : 0u);
      rec[0] = x.hi;
      rec[1] = x.lo;
      rec[2] = v.m;
      rec[3] = v.e;
      rec[4] = (uint64_t)(x.sv | (flags << 24));
    }
    // per rule chunk: the endpoint and rule bits under that chunk's tables
    uint32_t coff = 0;
    for (uint32_t k = 0; k < a.n_chunks; k++) {
      const Cfg c = load_cfg(a.cfg_lds_bytes ? xcfg + coff : a.cfgs[k]);
      coff += ((c.h->total_bytes < kSampCfgLds ? c.h->total_bytes : kSampCfgLds) + 15u) & ~15u;
      uint64_t ep = 0, svcb = 0;
      x_chunk(a, c, x, base + lane, k, ep, svcb);
      uint32_t z = 0;
      seg_or_scan(h, z, ep, svcb);
      if (tail) {
        rec[kXFixedWords + 2 * k] = ep;
        rec[kXFixedWords + 2 * k + 1] = svcb;
      }
    }
    // every span learns its record's slot from the record's tail lane
    const int tl = ffs64(tails & ~lanemask_lt(lane));
    const uint32_t my = __shfl(pos, tl < 0 ? lane : tl, kWave);
    if (x.valid) a.pack_pos[base + lane] = my;
  }
}

// Records -> the owner's SAMPLE columns: one "span" per record with its own
// resource.  The record's latency element becomes start / end plus status
// bit 7 (kStatusReset) when a zero start came before its min start; chunk
// k's endpoint bits go to plane k of route_match, its rule bits to plane k
// of svc_match.
__global__ __launch_bounds__(256) void shard_unpack_kernel(UnpackArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t* rec = reinterpret_cast<const uint64_t*>(a.recv) + i * x_rec_words(a.n_chunks);
  const uint64_t m = rec[2], e = rec[3], w4 = rec[4];
  const uint32_t sv = (uint32_t)(w4 & kXNone), flags = (uint32_t)(w4 >> 24) & 0xFFu;
  const bool lat = flags & kXLat;
  a.tid[2 * i] = rec[0];
  a.tid[2 * i + 1] = rec[1];
  a.start[i] = lat && m != kInf ? m : 0;
  a.end[i] = lat ? e : 0;
  a.status[i] = (uint8_t)(((flags & kXErr) ? OSE_STATUS_ERROR : 0u) |
                          ((lat && (flags & kXReset) && m != kInf) ? kStatusReset : 0u));
  for (uint32_t k = 0; k < a.n_chunks; k++) {
    a.route_match[k * a.n + i] = rec[kXFixedWords + 2 * k];
    a.svc_match[k * a.n + i] = rec[kXFixedWords + 2 * k + 1];
  }
  a.res_svc[i] = lat && sv != kXNone ? sv : 0xFFFFFFFFu;
  a.res_svc_str[i] = 0xFFFFFFFFu;
  a.resource[i] = (uint32_t)i;   // one "resource" per record carries its latency service
}

// ---- owner side: decisions from the received records ------------------------------
// A rank receives each trace it owns as pieces, one record per source
// stretch, in (source rank, source order) = global batch order.
// owner_bucket_kernel reads the records in order (coalesced) and moves each
// into a 64-byte slot of its trace-id hash bucket (one atomic per record;
// the slot keeps the record's index, since order inside a bucket is lost
// here).  One workgroup per bucket (owner_fold_kernel):
//   1. loads the bucket's slots (one round trip: slot t by thread t,
//      issued with the count, not after it) into LDS and groups them by
//      trace id with an LDS hash table (exact 128-bit compare): group = the
//      entry that claimed the trace's slot;
//   2. sorts the keys (group : 8 | record index : 32 | entry : 8) with a
//      bitonic sort in LDS: every trace's records become adjacent and in
//      batch order;
//   3. folds each trace on one lane: the error bit, then chunk by chunk the
//      endpoint and rule words, the latency monoid of each latency service
//      (lat_comb in order: the zero-start reset is order-dependent; services
//      taken one at a time in increasing id, so no per-lane arrays, which
//      would live in scratch) and ShouldSample's walk (walk_chunk), and
//      writes keep on every record of the trace.
// This replaces unpacking into span columns and the general run-list path
// (an exact table in HBM, run lists, one lane chasing a trace's runs through
// the head masks).  Only a bucket past kOwnerCap records sets *overflow,
// and the host then runs the general path on the whole batch.
// Measured forms (owner workload, profiles/r4_owner_fold_forms.txt): an
// index per slot with the records read through it (two more dependent round
// trips per workgroup), persistent workgroups, the rule tables read from
// HBM (the fold phase 89% of the clocks), and per-trace member lists built
// by a scan and an insertion sort instead of the bitonic sort, with the
// traces' lanes packed into the first waves, were slower.
constexpr uint32_t kOwnerTable = 2 * kOwnerCap;   // LDS hash slots: load <= 1/2
constexpr uint32_t kOwnerNone = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t owner_bucket_of(uint64_t h, uint32_t n_buckets) {
  return (uint32_t)(((h & 0xFFFFFFFFull) * n_buckets) >> 32);   // the low half: owner = high half mod N
}
__global__ __launch_bounds__(256) void owner_bucket_kernel(OwnerArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t* r = reinterpret_cast<const uint64_t*>(a.recv) + i * a.words;
  const uint64_t hi = r[0], lo = r[1], m = r[2], e = r[3], w4 = r[4], ep = r[kXFixedWords], sv = r[kXFixedWords + 1];
  const uint32_t b = owner_bucket_of(tid_hash(hi, lo), a.n_buckets);
  const uint32_t at = atomicAdd(&a.bkt_count[b], 1u);
  if (at >= kOwnerCap) return;
  uint4* d = reinterpret_cast<uint4*>(a.bkt_rec + ((uint64_t)b * kOwnerCap + at) * kOwnerSlotWords);
  d[0] = make_uint4((uint32_t)hi, (uint32_t)(hi >> 32), (uint32_t)lo, (uint32_t)(lo >> 32));
  d[1] = make_uint4((uint32_t)m, (uint32_t)(m >> 32), (uint32_t)e, (uint32_t)(e >> 32));
  d[2] = make_uint4((uint32_t)w4, (uint32_t)i, (uint32_t)ep, (uint32_t)(ep >> 32));
  d[3] = make_uint4((uint32_t)sv, (uint32_t)(sv >> 32), 0u, 0u);
}

// One chunk's share of a trace's fold: the chunk's endpoint and rule words
// ORed over the trace's entries [k, e) of the sorted keys, the latency
// element of each latency service (in batch order; services one at a time
// in increasing id), ShouldSample's walk over the chunk's rules
__device__ void owner_chunk(const Cfg& c, const uint32_t* map, uint32_t n_global, const uint64_t* s_key,
                            const uint32_t* s_w4, const uint64_t* s_m, const uint64_t* s_e, const uint64_t* s_ep,
                            const uint64_t* s_sv, uint32_t k, uint32_t e, uint32_t err, bool any_lat, FoldState& s) {
  uint64_t ep = 0, svc = 0;
  for (uint32_t j = k; j < e; j++) {
    const uint32_t x = (uint32_t)s_key[j] & 255u;
    ep |= s_ep[x];
    svc |= s_sv[x];
  }
  uint64_t lsat = 0;
  const uint32_t nsvc = c.h->n_services;
  uint32_t last = 0;
  bool first = true;
  while (any_lat) {
    uint32_t nxt = kXNone;
    for (uint32_t j = k; j < e; j++) {
      const uint32_t w4 = s_w4[(uint32_t)s_key[j] & 255u];
      const uint32_t sv = w4 & kXNone;
      if (((w4 >> 24) & kXLat) && sv != kXNone && (first || sv > last) && sv < nxt) nxt = sv;
    }
    if (nxt == kXNone) break;
    Lat l{0u, kInf, 0ull};
    for (uint32_t j = k; j < e; j++) {
      const uint32_t x = (uint32_t)s_key[j] & 255u;
      const uint32_t w4 = s_w4[x];
      if ((w4 & kXNone) != nxt || !((w4 >> 24) & kXLat)) continue;
      l = lat_comb(l, Lat{2u | (((w4 >> 24) & kXReset) ? 1u : 0u), s_m[x], s_e[x]});
    }
    // the record's latency service is a global id; a chunk-local table
    // takes it through the chunk's map
    const uint32_t sl = map ? (nxt < n_global ? map[nxt] : kXNone) : nxt;
    if (sl < nsvc) {
      const uint32_t slot = c.svc_slot[sl];
      if (slot != kNoSlot) lsat |= latency_satisfied(c, slot, ep, l.m, l.e);
    }
    last = nxt;
    first = false;
  }
  walk_chunk(c, s, err, ep, lsat, svc);
}

// OSE_DIAG: wall-clock ticks per phase, summed over workgroups (thread 0
// after a barrier; the diagnostic instance adds barriers between phases)
#if OSE_DIAG
#define OWNER_TICK(ph)                                                                       \
  do {                                                                                       \
    if (a.clocks) {                                                                          \
      __syncthreads();                                                                       \
      if (t == 0) {                                                                          \
        const uint64_t now = wall_clock64();                                                 \
        atomicAdd((unsigned long long*)&a.clocks[ph], (unsigned long long)(now - tick));     \
        tick = now;                                                                          \
      }                                                                                      \
    }                                                                                        \
  } while (0)
#else
#define OWNER_TICK(ph) \
  do {                 \
  } while (0)
#endif

// One workgroup per bucket; thread t holds entry t.  The rule tables of the
// chunk being walked are copied into LDS without their route bytes (the
// endpoint bits came with the records): every lookup of latency_satisfied
// and walk_chunk is then a ds_read, not a dependent L2 round trip (with the
// tables in HBM the fold was 89% of the kernel's clocks).
__device__ __forceinline__ void owner_cfg_copy(const OwnerArgs& a, uint8_t* dst, uint32_t ck, uint32_t t) {
  const uint8_t* src = a.cfgs[ck];
  const uint32_t nb = (reinterpret_cast<const SampCfgDev*>(src)->bytes_off + 15u) & ~15u;   // <= cfg_lds_bytes
  for (uint32_t k = t * 16; k < nb; k += 256 * 16)
    *reinterpret_cast<uint4*>(dst + k) = *reinterpret_cast<const uint4*>(src + k);
}
__global__ __launch_bounds__(256) void owner_fold_kernel(OwnerArgs a) {
  static_assert(kOwnerCap == 256, "one entry per thread; 8-bit entry and group indices");
  extern __shared__ __attribute__((aligned(16))) uint8_t cfg_lds[];
  __shared__ uint64_t s_hi[kOwnerCap], s_lo[kOwnerCap], s_key[kOwnerCap];
  __shared__ uint64_t s_m[kOwnerCap], s_e[kOwnerCap], s_ep[kOwnerCap], s_sv[kOwnerCap];
  __shared__ uint32_t s_w4[kOwnerCap], s_tab[kOwnerTable];
  const uint32_t t = threadIdx.x, b = blockIdx.x;
  uint64_t tick = OSE_DIAG ? wall_clock64() : 0;
  (void)tick;
  // the slot load does not wait for the count: slot t is read whether or not
  // it is filled (a bucket's slots are contiguous; unfilled ones are ignored)
  const uint4* sl = reinterpret_cast<const uint4*>(a.bkt_rec + ((uint64_t)b * kOwnerCap + t) * kOwnerSlotWords);
  const uint4 q0 = sl[0], q1 = sl[1], q2 = sl[2], q3 = sl[3];
  const uint32_t cnt = a.bkt_count[b];
  if (cnt == 0) return;   // block-uniform
  if (cnt > kOwnerCap) {
    if (t == 0) atomicOr(a.overflow, 1u);
    return;
  }
  owner_cfg_copy(a, cfg_lds, 0, t);
  s_tab[t] = kOwnerNone;
  s_tab[t + 256] = kOwnerNone;
  uint32_t ri = 0;
  if (t < cnt) {
    s_hi[t] = (uint64_t)q0.x | ((uint64_t)q0.y << 32);
    s_lo[t] = (uint64_t)q0.z | ((uint64_t)q0.w << 32);
    s_m[t] = (uint64_t)q1.x | ((uint64_t)q1.y << 32);
    s_e[t] = (uint64_t)q1.z | ((uint64_t)q1.w << 32);
    s_w4[t] = q2.x;
    ri = q2.y;
    s_ep[t] = (uint64_t)q2.z | ((uint64_t)q2.w << 32);
    s_sv[t] = (uint64_t)q3.x | ((uint64_t)q3.y << 32);
  }
  uint32_t P = 1;
  while (P < cnt) P <<= 1;
  __syncthreads();
  OWNER_TICK(0);
  // 1. group by trace id; key = group : 8 | record index : 32 | entry : 8
  if (t < P) {
    uint64_t key = ~0ull;   // padding sorts last
    if (t < cnt) {
      const uint64_t hi = s_hi[t], lo = s_lo[t];
      uint32_t slot = ((uint32_t)(tid_hash(hi, lo) >> 32) * 0x9E3779B1u) >> 23;   // 9 bits: kOwnerTable
      uint32_t g = t;
      for (;;) {   // the table never fills (cnt <= kOwnerTable / 2)
        const uint32_t prev = atomicCAS(&s_tab[slot], kOwnerNone, t);
        if (prev == kOwnerNone) break;
        if (s_hi[prev] == hi && s_lo[prev] == lo) {
          g = prev;
          break;
        }
        slot = (slot + 1) & (kOwnerTable - 1);
      }
      key = ((uint64_t)g << 40) | ((uint64_t)ri << 8) | t;
    }
    s_key[t] = key;
  }
  __syncthreads();
  OWNER_TICK(1);
  // 2. bitonic sort of s_key[0, P) ascending: a trace's records adjacent, in batch order
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      if (t < P / 2) {
        const uint32_t i0 = 2 * t - (t & (stride - 1)), i1 = i0 + stride;
        const bool up = (i0 & size) == 0;
        const uint64_t x = s_key[i0], y = s_key[i1];
        if ((x > y) == up) {
          s_key[i0] = y;
          s_key[i1] = x;
        }
      }
      __syncthreads();
    }
  }
  OWNER_TICK(2);
  // 3. the trace whose first entry (in sorted order) is t
  bool hv = false, hlat = false;
  uint32_t he = 0, herr = 0, g = 0;
  if (t < cnt) {
    g = (uint32_t)(s_key[t] >> 40);
    if (t == 0 || (uint32_t)(s_key[t - 1] >> 40) != g) {
      uint32_t lat = 0;
      for (uint32_t j = t; j < cnt; j++) {
        if (j > t && (uint32_t)(s_key[j] >> 40) != g) break;
        const uint32_t fl = s_w4[(uint32_t)s_key[j] & 255u] >> 24;
        herr |= fl & kXErr;
        lat |= fl & kXLat;
        he = j + 1;
      }
      hv = true;
      hlat = lat != 0;
    }
  }
  FoldState fs{0.0, 0.0, 0u, 0u};
  const uint64_t* R = reinterpret_cast<const uint64_t*>(a.recv);
  for (uint32_t ck = 0; ck < a.n_chunks; ck++) {
    if (ck) {   // chunk ck's tables and words of entry t (block-uniform loop)
      __syncthreads();
      owner_cfg_copy(a, cfg_lds, ck, t);
      if (t < cnt) {
        const uint64_t* r = R + (uint64_t)ri * a.words + kXFixedWords + 2 * ck;
        s_ep[t] = r[0];
        s_sv[t] = r[1];
      }
      __syncthreads();
    }
    if (hv)
      owner_chunk(load_cfg(cfg_lds), a.svc_maps ? a.svc_maps[ck] : nullptr, a.n_global_svc, s_key, s_w4, s_m, s_e,
                  s_ep, s_sv, t, he, herr, hlat, fs);
  }
  OWNER_TICK(3);
  if (hv) {
    uint8_t dk = 0, dl = 0;
    double dr = 0;
    walk_finish(fs, trace_uniform(s_hi[g], s_lo[g], a.seed), dk, dl, dr);
    for (uint32_t j = t; j < he; j++) a.keep[(s_key[j] >> 8) & 0xFFFFFFFFull] = dk;
  }
  OWNER_TICK(4);
}

// The endpoint bits of every span under one rule chunk's tables read from
// HBM (a chunk whose route bytes spill past the kernels' LDS copy): the
// plane the trace stage and the pack then take as route_match
__global__ __launch_bounds__(256) void endpoint_plane_kernel(const uint8_t* cfg, const uint32_t* resource,
                                                             const uint32_t* res_svc, const ose_strref* route,
                                                             const uint8_t* arena, uint64_t n, uint64_t* out) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const Cfg c = load_cfg(cfg);
  const uint32_t sv = res_svc[resource[j]];
  uint64_t ep = 0;
  if (sv < c.h->n_services) {
    const uint32_t slot = c.svc_slot[sv];
    if (slot != kNoSlot) ep = endpoint_bits(c, slot, arena, route[j]);
  }
  out[j] = ep;
}

__global__ __launch_bounds__(256) void scatter_keep_kernel(const uint8_t* back, const uint32_t* pos, uint64_t n,
                                                           uint8_t* keep) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) keep[i] = back[pos[i]];
}

}  // namespace

uint32_t shard_owner_host(uint64_t hi, uint64_t lo, uint32_t n) {
  auto sm = [](uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  return (uint32_t)((sm(hi ^ sm(lo)) >> 32) % n);
}
void launch_shard_hist(const ShardArgs& a, hipStream_t st) {
  const uint32_t waves = kSortThreads / kWave;
  hipLaunchKernelGGL(shard_hist_kernel, dim3((a.n_tiles + waves - 1) / waves), dim3(kSortThreads), 0, st, a);
}
void launch_shard_counts(const ShardArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(shard_counts_kernel, dim3(1), dim3(64), 0, st, a);
}
void launch_shard_scatter(const ShardArgs& a, hipStream_t st) {
  const uint32_t waves = kSortThreads / kWave;
  hipLaunchKernelGGL(shard_scatter_kernel, dim3((a.n_tiles + waves - 1) / waves), dim3(kSortThreads), a.cfg_lds_bytes, st,
                     a);
}
void launch_shard_unpack(const UnpackArgs& a, hipStream_t st) {
  if (a.n) hipLaunchKernelGGL(shard_unpack_kernel, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, st, a);
}
namespace {
__global__ __launch_bounds__(256) void add_i64_kernel(int64_t* dst, const int64_t* src, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] += src[i];
}
// the in-process transport's phase: every peer's piece in one launch
// (blockIdx.y = piece; 16-, 8- or 1-byte moves by the pieces' alignment)
__global__ __launch_bounds__(256) void peer_copy_kernel(PeerCopies c) {
  const uint32_t p = blockIdx.y;
  const uint8_t* src = c.src[p];
  uint8_t* dst = c.dst[p];
  const uint64_t len = c.len[p];
  const uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, step = (uint64_t)gridDim.x * 256;
  const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst);
  uint64_t done = 0;
  if ((al & 15) == 0) {
    const uint64_t m = len / 16;
    for (uint64_t i = t0; i < m; i += step)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    done = m * 16;
  } else if ((al & 7) == 0) {
    const uint64_t m = len / 8;
    for (uint64_t i = t0; i < m; i += step)
      reinterpret_cast<uint64_t*>(dst)[i] = reinterpret_cast<const uint64_t*>(src)[i];
    done = m * 8;
  }
  for (uint64_t i = done + t0; i < len; i += step) dst[i] = src[i];
}
}  // namespace
void launch_peer_copies(const PeerCopies& c, uint64_t max_len, hipStream_t st) {
  if (!c.n || !max_len) return;
  const uint32_t bx = (uint32_t)std::min<uint64_t>((max_len + 4095) / 4096, 1024);
  hipLaunchKernelGGL(peer_copy_kernel, dim3(bx, c.n), dim3(256), 0, st, c);
}
void launch_add_i64(int64_t* dst, const int64_t* src, uint64_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(add_i64_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, dst, src, n);
}
void launch_owner_bucket(const OwnerArgs& a, hipStream_t st) {
  if (a.n) hipLaunchKernelGGL(owner_bucket_kernel, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, st, a);
}
void launch_owner_fold(const OwnerArgs& a, hipStream_t st) {
  if (a.n) hipLaunchKernelGGL(owner_fold_kernel, dim3(a.n_buckets), dim3(256), a.cfg_lds_bytes, st, a);
}
void launch_endpoint_plane(const uint8_t* cfg, const uint32_t* resource, const uint32_t* res_svc, const ose_strref* route,
                           const uint8_t* arena, uint64_t n, uint64_t* out, hipStream_t st) {
  if (n) hipLaunchKernelGGL(endpoint_plane_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, cfg, resource,
                            res_svc, route, arena, n, out);
}
void launch_scatter_keep(const uint8_t* back, const uint32_t* pos, uint64_t n, uint8_t* keep, hipStream_t st) {
  if (n) hipLaunchKernelGGL(scatter_keep_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, back, pos, n, keep);
}

void launch_trace_eval(const TraceKernelArgs& a, hipStream_t st) {
  const uint32_t per_block = kTWaves * a.win_per_wave;
  const uint32_t blocks = (a.n_windows + per_block - 1) / per_block;
  if (a.n_multi) {   // every rule chunk in one pass (run_sampling checks the conditions)
    if (a.n_multi == 2)
      hipLaunchKernelGGL((trace_multi_kernel<2>), dim3(blocks), dim3(kTThreads), a.cfg_lds_bytes, st, a);
    else
      hipLaunchKernelGGL((trace_multi_kernel<3>), dim3(blocks), dim3(kTThreads), a.cfg_lds_bytes, st, a);
    return;
  }
  if (a.mode == kTraceRuns && !a.svc_match && !a.route_match && !a.attr_match && (OSE_DIAG || !a.ablate)) {
    const bool chunk = a.fold_in || a.fold_out;
    if (a.narrow && chunk)
      hipLaunchKernelGGL((trace_eval_kernel<true, true, true>), dim3(blocks), dim3(kTThreads), 0, st, a);
    else if (a.narrow)
      hipLaunchKernelGGL((trace_eval_kernel<true, true, false>), dim3(blocks), dim3(kTThreads), 0, st, a);
    else if (chunk)
      hipLaunchKernelGGL((trace_eval_kernel<true, false, true>), dim3(blocks), dim3(kTThreads), 0, st, a);
    else
      hipLaunchKernelGGL((trace_eval_kernel<true, false, false>), dim3(blocks), dim3(kTThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL((trace_eval_kernel<false, false, false>), dim3(blocks), dim3(kTThreads), 0, st, a);
  }
}
// One workgroup per fingerprint bucket: its entries into an LDS hash set; an
// entry met twice (or a bucket past its capacity) sets *dup
__global__ __launch_bounds__(256) void trace_dup_check_kernel(TraceKernelArgs a) {
  constexpr uint32_t kSet = 2 * kDupBucketCap;
  static_assert(kSet == 2048, "the set hash takes at most 11 bits");
  __shared__ uint64_t set[kSet];
  __shared__ uint32_t found;
  const uint32_t bk = blockIdx.x;
  const uint32_t c = a.dup_bkt_count[bk];
  if (c <= 1) return;
  if (c > kDupBucketCap) {
    if (threadIdx.x == 0) atomicOr(a.dup, 1u);
    return;
  }
  // the set: the power of two >= 2c (>= 256), so a bucket of ~c entries
  // clears ~2c slots instead of all kSet
  uint32_t bits = 8;
  while ((1u << bits) < 2 * c) bits++;
  const uint32_t nset = 1u << bits;   // <= kSet (c <= kDupBucketCap)
  for (uint32_t k = threadIdx.x; k < nset; k += 256) set[k] = 0ull;
  if (threadIdx.x == 0) found = 0;
  __syncthreads();
  const uint64_t* e = a.dup_bkt + (uint64_t)bk * kDupBucketCap;
  bool hit = false;
  for (uint32_t k = threadIdx.x; k < c; k += 256) {
    const uint64_t v = e[k];   // never 0
    uint32_t s = ((uint32_t)v * 0x9E3779B1u) >> (32 - bits);
    for (uint32_t probes = 0; probes < nset; probes++) {
      const uint64_t old = atomicCAS((unsigned long long*)&set[s], 0ull, (unsigned long long)v);
      if (old == 0) break;
      if (old == v) { hit = true; break; }
      s = (s + 1) & (nset - 1);
    }
  }
  if (hit) found = 1;
  __syncthreads();
  if (threadIdx.x == 0 && found) atomicOr(a.dup, 1u);
}
// Chunk-local service ids (sampling_host.cpp local_service_ids)
__global__ __launch_bounds__(256) void svc_translate_kernel(const uint32_t* map, uint32_t n_global, const uint32_t* in1,
                                                            const uint32_t* in2, uint32_t* out1, uint32_t* out2,
                                                            uint64_t n) {
  const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const uint32_t a = in1[r], b = in2[r];
  out1[r] = a < n_global ? map[a] : 0xFFFFFFFFu;
  out2[r] = b < n_global ? map[b] : 0xFFFFFFFFu;
}
void launch_svc_translate(const uint32_t* map, uint32_t n_global, const uint32_t* in1, const uint32_t* in2, uint32_t* out1,
                          uint32_t* out2, uint64_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(svc_translate_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, map, n_global, in1,
                            in2, out1, out2, n);
}
void launch_trace_dup_check(const TraceKernelArgs& a, hipStream_t st) {
  if (a.dup_bkt) hipLaunchKernelGGL(trace_dup_check_kernel, dim3(1u << a.dup_bkt_bits), dim3(256), 0, st, a);
}

void launch_trace_long(const TraceKernelArgs& a, hipStream_t st, uint32_t known_runs) {
  // known_runs: the listed-run count the host read (host-gated form); else
  // grids for the most runs the fast path can list, workgroups past the
  // device counts exit
  const uint64_t most = known_runs ? known_runs : a.n_spans / ((uint64_t)a.long_steps * kWave) + 1;
  hipLaunchKernelGGL(trace_long_plan_kernel, dim3((uint32_t)std::min<uint64_t>((most + kPlanWaves - 1) / kPlanWaves, 1024)),
                     dim3(kPlanWaves * kWave), 0, st, a);
  const uint64_t pieces = most + a.n_spans / kLongPiece + 1;
  hipLaunchKernelGGL(trace_long_kernel, dim3((uint32_t)std::min<uint64_t>((pieces + kLWaves - 1) / kLWaves, 1024)),
                     dim3(kLThreads), 0, st, a);
  hipLaunchKernelGGL(trace_long_decide_kernel, dim3((uint32_t)std::min<uint64_t>((most + kPlanWaves - 1) / kPlanWaves, 1024)),
                     dim3(kPlanWaves * kWave), 0, st, a);
}
void launch_trace_insert_exact(const TraceKernelArgs& a, hipStream_t st) {
  if (a.n_spans)
    hipLaunchKernelGGL(trace_insert_exact_kernel, dim3((uint32_t)std::min<uint64_t>((a.n_spans + 255) / 256, kGatedBlocks)),
                       dim3(256), 0, st, a);
}
void launch_trace_runs(const TraceKernelArgs& a, hipStream_t st) {
  const uint64_t blocks = std::min<uint64_t>((a.n_windows + 3) / 4, kGatedBlocks);
  hipLaunchKernelGGL(trace_runs_kernel, dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(256), 0, st, a);
}
void launch_trace_fold(const TraceKernelArgs& a, hipStream_t st) {
  const uint64_t blocks = std::min<uint64_t>((a.n_windows + kTWaves - 1) / kTWaves, kGatedBlocks);
  hipLaunchKernelGGL(trace_fold_kernel, dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(kTThreads), 0, st, a);
}
void launch_trace_first_select(const TraceKernelArgs& a, hipStream_t st) {
  const uint64_t blocks = std::min<uint64_t>((a.n_windows + 255) / 256, kGatedBlocks);
  hipLaunchKernelGGL(trace_first_select_kernel, dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(256), 0, st, a);
}
void launch_trace_key(const TraceSortArgs& a, hipStream_t st) {
  const uint64_t blocks = std::min<uint64_t>((a.n_spans + 255) / 256, kGatedBlocks);
  hipLaunchKernelGGL(trace_key_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, a);
}
void launch_sort_hist(const TraceSortArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sort_hist_kernel, dim3(a.n_tiles), dim3(kSortThreads), 0, st, a);
}
void launch_sort_scatter(const TraceSortArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sort_scatter_kernel, dim3(a.n_tiles), dim3(kSortThreads), 0, st, a);
}
void launch_scan_u32(const ScanArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(scan_u32_kernel, dim3(a.n_tiles), dim3(kScanTileItems), 0, st, a);
}
void launch_trace_compact(const TraceCompactArgs& a, hipStream_t st) {
  const uint32_t blocks = (a.n_windows + kTWaves - 1) / kTWaves;
  hipLaunchKernelGGL(trace_compact_kernel, dim3(blocks), dim3(kTThreads), 0, st, a);
}

}  // namespace ose
