// url_kernel.hip — odigosurltemplate on CDNA4 (gfx950).
//
// One wave per 64-span group; a persistent grid of four 4-wave workgroups per
// CU (16x that beside the trace stage), waves independent after the config
// load:
//   url_plan_kernel   per group: the arena bytes its paths reference are
//                     staged into a 3 KiB per-wave LDS buffer by LDS-DMA
//                     (global_load_lds_dwordx4; paths gathered as 16-byte
//                     chunks when the range is wider), the next group's copy
//                     in flight while this one is planned; 12 bit-sliced
//                     class bitmaps of the staged rows (url_classes.hpp);
//                     the segment list (enumerated from the slash / '?' rows)
//                     classified 64 segments per step, branch-free
//                     (templatize.go:242-269), each lane folding its span's
//                     plan (processor.go:149-186); then the group's template
//                     bytes assembled into an LDS image over the dead bitmaps
//                     and stored to the wave's scratch region (refs form: to
//                     its place in the output arena, the refs written here).
//                     Groups it cannot take (user-rule matches, name ids past
//                     the braced table, a list or image overflow) are listed.
//   url_plan_slow_kernel  the groups whose paths overflow the stage or hold a
//                     segment over 64 bytes, planned in stage-sized subsets.
//   url_scan_kernel   exclusive scan of the group sums (decoupled look-back).
//   url_emit_slow_kernel  the listed groups, written per span at their bases.
//   url_copy_kernel   template refs of the other groups and the images moved
//                     to the compact output arena (with SIZE: the fused spans
//                     pass of odigostrafficmetrics).
// Byte-identical to the oracle (oracle/url.c) including the compact arena.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../../include/odigos_amd.h"
#include "device_common.hpp"
#include "kernels.hpp"
#include "size_device.hpp"
#include "url_classes.hpp"

#ifndef OSE_ASM_BATCH
#define OSE_ASM_BATCH 0
#endif

namespace ose {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr uint32_t kStage = 4 * 1024;            // per-wave LDS copy of one group's bytes (slow kernels)

enum : uint32_t { M_NONE = 0, M_RENAME_SLASH, M_SLASH, M_RULE, M_DEFAULT, M_ORIG };

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }
__device__ __forceinline__ bool is_alpha(uint32_t c) { return (c | 0x20u) - 'a' < 26u; }
__device__ __forceinline__ bool is_hex(uint32_t c) { return is_digit(c) || (c | 0x20u) - 'a' < 6u; }
// noLettersRegex class (templatize.go:14): digits and _-!@#$%^&*()=+{}[]:;"'<>,.?/\|`~
__device__ __forceinline__ bool is_nolet(uint32_t c) {
  constexpr uint64_t lo = (1ull << '!') | (1ull << '"') | (1ull << '#') | (1ull << '$') | (1ull << '%') |
                          (1ull << '&') | (1ull << '\'') | (1ull << '(') | (1ull << ')') | (1ull << '*') |
                          (1ull << '+') | (1ull << ',') | (1ull << '-') | (1ull << '.') | (1ull << '/') |
                          (0x3FFull << '0') | (1ull << ':') | (1ull << ';') | (1ull << '<') | (1ull << '=') |
                          (1ull << '>') | (1ull << '?');
  constexpr uint64_t hi = (1ull << ('@' - 64)) | (1ull << ('[' - 64)) | (1ull << ('\\' - 64)) |
                          (1ull << (']' - 64)) | (1ull << ('^' - 64)) | (1ull << ('_' - 64)) |
                          (1ull << ('`' - 64)) | (1ull << ('{' - 64)) | (1ull << ('|' - 64)) |
                          (1ull << ('}' - 64)) | (1ull << ('~' - 64));
  uint64_t m = c < 64 ? lo : hi;
  return c < 128 && ((m >> (c & 63)) & 1);
}
// emailRegex classes (templatize.go:70)
__device__ __forceinline__ bool is_email_local(uint32_t c) {
  return is_alpha(c) || is_digit(c) || c == '.' || c == '_' || c == '%' || c == '+' || c == '-';
}
__device__ __forceinline__ bool is_email_domain(uint32_t c) { return is_alpha(c) || is_digit(c) || c == '.' || c == '-'; }

// datesRegex (templatize.go:67) accepts exactly these lengths
__device__ __forceinline__ bool date_len(uint32_t n) {
  return n == 10 || n == 11 || n == 15 || n == 16 || n == 17 || n == 19 || n == 20 || n == 21 || n == 22 || n == 24;
}
// `^\d{4}-\d{2}-\d{2}(?:T\d{2}:\d{2}(?::\d{2})?)?(?:Z|[+-]\d{4})?$`: each
// optional group starts with a byte nothing later may start with, so the
// greedy parse is the only possible match.
template <class R>
__device__ bool date_match(R& rd, uint32_t s, uint32_t n) {
  auto d = [&](uint32_t k) { return is_digit(rd.at(s + k)); };
  if (!(d(0) && d(1) && d(2) && d(3) && rd.at(s + 4) == '-' && d(5) && d(6) && rd.at(s + 7) == '-' && d(8) && d(9)))
    return false;
  uint32_t p = 10;
  if (p < n && rd.at(s + p) == 'T') {
    if (p + 6 > n || !d(p + 1) || !d(p + 2) || rd.at(s + p + 3) != ':' || !d(p + 4) || !d(p + 5)) return false;
    p += 6;
    if (p < n && rd.at(s + p) == ':') {
      if (p + 3 > n || !d(p + 1) || !d(p + 2)) return false;
      p += 3;
    }
  }
  if (p < n) {
    uint32_t c = rd.at(s + p);
    if (c == 'Z') p += 1;
    else if (c == '+' || c == '-') {
      if (p + 5 > n || !d(p + 1) || !d(p + 2) || !d(p + 3) || !d(p + 4)) return false;
      p += 5;
    }
  }
  return p == n;
}
// one 8-4-4-4-12 hex UUID at s
template <class R>
__device__ bool uuid_at(R& rd, uint32_t s) {
  for (uint32_t k = 0; k < 36; k++) {
    uint32_t c = rd.at(s + k);
    bool ok = (k == 8 || k == 13 || k == 18 || k == 23) ? c == '-' : is_hex(c);
    if (!ok) return false;
  }
  return true;
}
// `^[a-zA-Z0-9._%+-]+@[a-zA-Z0-9.-]+\.[a-zA-Z]{2,}$` given exactly one '@':
// local part >= 1 byte, domain all [A-Za-z0-9.-] with its last '.' at index
// >= 1 followed by >= 2 ASCII letters.
template <class R>
__device__ bool email_match(R& rd, uint32_t s, uint32_t e) {
  uint32_t q = s;
  while (q < e && rd.at(q) != '@') {
    if (!is_email_local(rd.at(q))) return false;
    q++;
  }
  if (q == s || q >= e) return false;
  const uint32_t d0 = q + 1;
  int32_t lastdot = -1;
  for (uint32_t k = d0; k < e; k++) {
    uint32_t c = rd.at(k);
    if (!is_email_domain(c)) return false;
    if (c == '.') lastdot = (int32_t)(k - d0);
  }
  if (lastdot < 1) return false;
  const uint32_t t0 = d0 + (uint32_t)lastdot + 1;
  if (e - t0 < 2) return false;
  for (uint32_t k = t0; k < e; k++)
    if (!is_alpha(rd.at(k))) return false;
  return true;
}
// replacementChar (templatize.go:73): Go decodes invalid UTF-8 as U+FFFD
// (width 1), so the regexp matches EF BF BD or any undecodable byte.
template <class R>
__device__ bool has_fffd(R& rd, uint32_t s, uint32_t e) {
  uint32_t q = s;
  while (q < e) {
    uint32_t c = rd.at(q);
    if (c < 0x80) { q++; continue; }
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return true;
    if (q + need >= e) return true;
    for (uint32_t k = 1; k <= need; k++) {
      uint32_t b = rd.at(q + k);
      if (b < (k == 1 ? lo : 0x80u) || b > (k == 1 ? hi : 0xBFu)) return true;
    }
    if (need == 2 && c == 0xEF && rd.at(q + 1) == 0xBF && rd.at(q + 2) == 0xBD) return true;
    q += need + 1;
  }
  return false;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr uint32_t kNameTab = 64;
// The header is copied into registers once per workgroup: read through the
// blob pointer the compiler cannot prove it unclobbered by the kernel's own
// stores and reloads it (vector load + full wait) in every segment loop.
typedef const __attribute__((address_space(3))) UrlCfgDev lds_cfg;
struct Cfg {
  const uint8_t* blob;
  lds_cfg* h;             // header copy in LDS: fields are read where used, no registers held
  uint32_t n_custom, n_rules, max_rule_nseg;   // the fields every span's plan tests
  uint32_t names_off;
  uint32_t names_tab_all;   // every name id < kNameTab (the LDS name table holds them all)
  lds_u8* names;          // first kNamesLds bytes of the bytes section, staged in LDS
  uint32_t names_len;
  uint32_t ablate;        // diagnostics (UrlKernelArgs::ablate)
  const __attribute__((address_space(3))) NameDev* name_tab;   // first kNameTab entries of the name table, in LDS
  __device__ NameDev name(uint32_t id) const {
    if (id < kNameTab) return NameDev{name_tab[id].off, name_tab[id].len};
    return reinterpret_cast<const NameDev*>(blob + h->names_off)[id];
  }
  __device__ uint32_t dfa_off(int32_t i) const {
    return reinterpret_cast<const uint32_t*>(blob + h->dfa_off)[i];
  }
};

// getSegmentTemplatizationString (templatize.go:242-269) for the segment
// starting at s (it ends at the next '/' or n; the end is returned in *e_out):
// the name id, or -1 when the segment stays as is.  One pass over 4-byte
// words computes every cheap predicate branch-free:
//   noLetters   every byte in [!-~] and not a letter
//   hex         every byte [0-9A-Fa-f] (length >= 16 and even checked after)
//   \d{7,}      longest digit run, carried across words
//   '@' count and "any byte >= 0x80" gate the email and U+FFFD passes.
template <class R>
__device__ __forceinline__ int classify_segment(const Cfg& cfg, R& rd, uint32_t s, uint32_t n, uint32_t* e_out) {
  uint32_t bad_nl = 0, bad_hex = 0, any_hi = 0, ats = 0, run = 0, longnum = 0;
  auto st = rd.stream(s);
  uint32_t q = s;
  for (;;) {
    const uint32_t x = st.next();
    const uint32_t hi = x & kH, asc = hi ^ kH;
    const uint32_t t = swar_t(x), tl = t | 0x20202020u;
    const uint32_t digit = swar_ge(t, '0') & ~swar_ge(t, '9' + 1) & asc;
    const uint32_t ga = swar_ge(tl, 'a');
    const uint32_t alpha = ga & ~swar_ge(tl, 'z' + 1) & asc;
    const uint32_t hexl = ga & ~swar_ge(tl, 'f' + 1) & asc;
    const uint32_t print = swar_ge(t, '!') & ~swar_ge(t, 127) & asc;
    const uint32_t at = swar_ge(t, '@') & ~swar_ge(t, 'A') & asc;
    const uint32_t slash = swar_ge(t, '/') & ~swar_ge(t, '0') & asc;
    const uint32_t stop = slash | swar_end(n - q);
    const uint32_t v = swar_before(stop);
    bad_nl |= ~(print & ~alpha) & v;
    bad_hex |= ~(digit | hexl) & v;
    any_hi |= hi & v;
    ats += __builtin_popcount(at & v);
    const uint32_t nd = ~(digit & v) & kH;   // non-digit (or past the end) bytes
    const uint32_t lead = swar_first(nd);
    longnum |= (run + lead >= 7) ? 1u : 0u;
    if (stop) {
      q += swar_first(stop);
      break;
    }
    const uint32_t trail = nd ? (uint32_t)__clz(nd) >> 3 : 4u;
    run = lead == 4 ? run + 4 : trail;
    q += 4;
  }
  *e_out = q;
  const uint32_t e = q, len = e - s;
  for (uint32_t k = 0; k < cfg.n_custom; k++) {   // custom ids first, in config order
    const UrlCustomDev& cu = reinterpret_cast<const UrlCustomDev*>(cfg.blob + cfg.h->custom_off)[k];
    if (dfa_match(cfg.blob, cfg.dfa_off(cu.dfa), rd, s, e)) return (int)cu.name;
  }
  if (date_len(len) && date_match(rd, s, len)) return kNameDate;
  if (ats == 1 && !any_hi && email_match(rd, s, e)) return kNameEmail;
  if ((bad_nl == 0 && len > 0) || longnum || (bad_hex == 0 && len >= 16 && (len & 1) == 0)) return kNameId;
  if (len >= 36 && (uuid_at(rd, s) || uuid_at(rd, e - 36))) return kNameId;
  if (any_hi && has_fffd(rd, s, e)) return kNameId;
  return -1;
}

// attemptTemplateWithRule (templatize.go:192-237): output body length
// (without the leading '/') or -1.
template <class R>
__device__ int64_t attempt_rule(const Cfg& cfg, const UrlRuleDev& r, R& rd, uint32_t b0, uint32_t n) {
  const UrlRuleSegDev* segs = reinterpret_cast<const UrlRuleSegDev*>(cfg.blob + cfg.h->segs_off) + r.seg_first;
  const uint8_t* bytes = cfg.blob + cfg.h->bytes_off;
  uint32_t s = b0;
  int64_t len = 0;
  for (uint32_t k = 0; k < r.nseg; k++) {
    const uint32_t e = scan_to(rd, s, n, '/');
    const UrlRuleSegDev& sg = segs[k];
    const uint32_t sl = e - s;
    if (sg.kind == kRuleStatic && sg.text_len != 0) {
      if (sg.text_len != sl) return -1;
      for (uint32_t q = 0; q < sl; q++)
        if (bytes[sg.text_off + q] != rd.at(s + q)) return -1;
    }
    if (sg.dfa >= 0 && !dfa_match(cfg.blob, cfg.dfa_off(sg.dfa), rd, s, e)) return -1;
    if (k) len += 1;
    if (sg.kind == kRuleTemplate) len += sg.text_len + 2;
    else if (sg.kind == kRuleWildcard || sg.kind == kRuleRegex) len += sl;
    else len += sg.text_len;
    s = e + 1;
  }
  return len;
}

// path end after the http.target '?' cut (strings.SplitN(target, "?", 2)[0])
template <class R>
__device__ __forceinline__ uint32_t path_end(R& rd, uint32_t len, uint32_t f) {
  return (f & OSE_URL_PATH_MASK) == OSE_URL_PATH_TARGET ? scan_to(rd, 0, len, '?') : len;
}

// Output writers.  word(x, nv) appends the low nv (<= 4) bytes of x; while
// at least 4 bytes of the span's own output remain it stores all 4 (the
// extra bytes are overwritten by this lane later), so the common case has no
// per-byte branches.
template <class P>
struct Put {
  P dst;
  uint32_t w, cap;
  __device__ __forceinline__ void byte(uint32_t c) { dst[w++] = (uint8_t)c; }
  __device__ __forceinline__ void word(uint32_t x, uint32_t nv) {
    if (w + 4 <= cap) {
      dst[w] = (uint8_t)x;
      dst[w + 1] = (uint8_t)(x >> 8);
      dst[w + 2] = (uint8_t)(x >> 16);
      dst[w + 3] = (uint8_t)(x >> 24);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < 4; k++)
        if (k < nv) dst[w + k] = (uint8_t)(x >> (8 * k));
    }
    w += nv;
  }
};
typedef __attribute__((address_space(3))) uint8_t lds_out_u8;
// unaligned LDS accesses (gfx950 LDS supports them: the compiler emits
// ds_read_b64 / ds_write_b64 for 1-byte-aligned 8-byte accesses)
typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;
typedef const __attribute__((address_space(3))) u64_ua lds_u64u;
typedef __attribute__((address_space(3))) u64_ua lds_w64u;
typedef __attribute__((address_space(3))) u32_ua lds_w32u;
typedef __attribute__((address_space(3))) u16_ua lds_w16u;

// copies [q, n)
template <class R, class W>
__device__ __forceinline__ void copy_range(R& rd, uint32_t q, uint32_t n, W& put) {
  auto st = rd.stream(q);
  for (; q < n; q += 4) put.word(st.next(), min(4u, n - q));
}
// copies the segment starting at q (up to '/' or n); returns its end
template <class R, class W>
__device__ __forceinline__ uint32_t copy_segment(R& rd, uint32_t q, uint32_t n, W& put) {
  auto st = rd.stream(q);
  for (;;) {
    const uint32_t x = st.next();
    const uint32_t stop = swar_eq(x, '/') | swar_end(n - q);
    const uint32_t nv = swar_first(stop);
    put.word(x, nv);
    q += nv;
    if (stop) return q;
  }
}
template <class W>
__device__ __forceinline__ void put_name(const Cfg& cfg, uint32_t id, W& put) {
  const NameDev nm = cfg.name(id);
  put.byte('{');
  if (nm.off + nm.len <= cfg.names_len) {
    for (uint32_t q = 0; q < nm.len; q++) put.byte(cfg.names[nm.off + q]);
  } else {
    const uint8_t* bytes = cfg.blob + cfg.h->bytes_off;
    for (uint32_t q = 0; q < nm.len; q++) put.byte(bytes[nm.off + q]);
  }
  put.byte('}');
}

template <class R, class W>
__device__ void emit_rule(const Cfg& cfg, const UrlRuleDev& r, R& rd, uint32_t b0, uint32_t n, W& put) {
  const UrlRuleSegDev* segs = reinterpret_cast<const UrlRuleSegDev*>(cfg.blob + cfg.h->segs_off) + r.seg_first;
  const uint8_t* bytes = cfg.blob + cfg.h->bytes_off;
  uint32_t s = b0;
  for (uint32_t k = 0; k < r.nseg; k++) {
    const uint32_t e = scan_to(rd, s, n, '/');
    const UrlRuleSegDev& sg = segs[k];
    if (k) put.byte('/');
    if (sg.kind == kRuleTemplate) {
      put.byte('{');
      for (uint32_t q = 0; q < sg.text_len; q++) put.byte(bytes[sg.text_off + q]);
      put.byte('}');
    } else if (sg.kind == kRuleWildcard || sg.kind == kRuleRegex) {
      copy_range(rd, s, e, put);
    } else {
      for (uint32_t q = 0; q < sg.text_len; q++) put.byte(bytes[sg.text_off + q]);
    }
    s = e + 1;
  }
}

// The plan of one span (phase 1 -> phase 2).  `n` (path end after the '?'
// cut) is carried in the meta word when it fits, sparing phase 2 the scan.
constexpr uint32_t kNField = (1u << 25) - 1;   // "recompute n"
struct Plan {
  uint32_t mode = M_NONE, len = 0, lead = 0, field = 0;   // field: rule index (M_RULE) or n
  uint64_t code = 0;
  bool slow = false;
};

// phase 1 for one span whose path is available through rd (url_flags f)
template <class R>
__device__ __forceinline__ Plan plan_path(const Cfg& cfg, R& rd, uint32_t plen, uint32_t f) {
  Plan p;
  const uint32_t n = path_end(rd, plen, f);
  p.lead = (n > 0 && rd.at(0) == '/') ? 1 : 0;
  if (n == p.lead) {   // "" or "/" -> "/" (processor.go:156-160)
    p.mode = M_SLASH;
    p.len = 1;
    return p;
  }
  if (cfg.n_rules) {
    const uint32_t nseg = 1 + count_byte(rd, p.lead, n, '/');
    if (nseg <= cfg.max_rule_nseg) {
      const uint32_t* by_len = reinterpret_cast<const uint32_t*>(cfg.blob + cfg.h->rules_by_len_off);
      const UrlRuleDev* rules = reinterpret_cast<const UrlRuleDev*>(cfg.blob + cfg.h->rules_off);
      for (uint32_t r = by_len[nseg]; r < by_len[nseg + 1]; r++) {
        int64_t l = attempt_rule(cfg, rules[r], rd, p.lead, n);
        if (l >= 0) { p.mode = M_RULE; p.field = r; p.len = p.lead + (uint32_t)l; return p; }
      }
    }
  }
  uint32_t s = p.lead, seg = 0, l = p.lead;
  bool templated = false;
  for (;;) {
    uint32_t e;
    const int id = classify_segment(cfg, rd, s, n, &e);
    if (seg) l += 1;
    if (id >= 0) {
      templated = true;
      l += cfg.name((uint32_t)id).len + 2;
      if (seg < 16 && id < 15) p.code |= (uint64_t)(id + 1) << (seg * 4);
      else p.slow = true;
    } else {
      l += e - s;
    }
    seg++;
    if (e >= n) break;
    s = e + 1;
  }
  if (templated) { p.mode = M_DEFAULT; p.len = l; }
  else { p.mode = M_ORIG; p.len = 1 + (n - p.lead); }   // "/" + body (processor.go:182-185)
  p.field = n < kNField ? n : kNField;
  return p;
}

// phase 2 for one span: writes the template through put
template <class R, class W>
__device__ __forceinline__ void emit_path(const Cfg& cfg, R& rd, uint32_t plen, uint32_t f, uint32_t mode,
                                          uint32_t lead, bool slow, uint32_t field, uint64_t code, W& put) {
  if (mode == M_RENAME_SLASH || mode == M_SLASH) { put.byte('/'); return; }
  if (mode == M_RULE) {
    const uint32_t n = path_end(rd, plen, f);
    if (lead) put.byte('/');
    const UrlRuleDev* rules = reinterpret_cast<const UrlRuleDev*>(cfg.blob + cfg.h->rules_off);
    emit_rule(cfg, rules[field], rd, lead, n, put);
    return;
  }
  const uint32_t n = field != kNField ? field : path_end(rd, plen, f);
  if (mode == M_ORIG) {
    put.byte('/');
    copy_range(rd, lead, n, put);
    return;
  }
  if (lead) put.byte('/');
  uint32_t s = lead, seg = 0;
  for (;;) {
    if (seg) put.byte('/');
    uint32_t e;
    int id;
    if (seg < 16 && !slow) {
      id = (int)((code >> (seg * 4)) & 15u) - 1;
      e = id >= 0 ? scan_to(rd, s, n, '/') : copy_segment(rd, s, n, put);
    } else {
      id = classify_segment(cfg, rd, s, n, &e);
      if (id < 0) copy_range(rd, s, e, put);
    }
    if (id >= 0) put_name(cfg, (uint32_t)id, put);
    seg++;
    if (e >= n) break;
    s = e + 1;
  }
}

// ---------------------------------------------------------------------------
// Class bitmaps of one wave's staged bytes.  Row r covers stage bytes
// [32r, 32r+32) and holds one 32-bit mask per class (bit k = byte 32r+k), so
// the 64-bit windows of all classes at any byte come from 3 rows (6 x
// ds_read_b128).  Built cooperatively, 32 bytes per lane, branch-free.
// Classes 0-7 are read for every segment; 8-11 (the email classes) only for
// segments holding exactly one '@'.  A row is 3 x 16 bytes: [0-3] [4-7] [8-11].
// classes 0-5 are what the segment classifier reads (a row's first vector and
// half of its second), 6-7 what the enumeration reads, 8-11 the email checks
enum : uint32_t { C_BNL = 0, C_BHX, C_DG, C_AT, C_HI, C_DASH, C_SL, C_QM, C_BLOC, C_BDOM, C_DOT, C_NAL, kClasses };
constexpr uint32_t kBase = 8;
constexpr uint32_t kRowVec = 3;   // u32x4 per row
constexpr uint32_t kBmRows = kStage / 32 + 3;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;
typedef const __attribute__((address_space(3))) u32x4 lds_cu4;

// One 32-byte row: the class words as boolean functions of the row's 8 bit
// planes (url_classes.hpp; tests/lut_check.cpp checks them on the host).
// C_* above is uc::BNL.. in the same order.
static_assert(C_BNL == uc::BNL && C_DG == uc::DG && C_HI == uc::HI && C_QM == uc::QM && C_NAL == uc::NAL &&
                  kClasses == uc::kN,
              "class order");
__device__ __forceinline__ void build_row(lds_u32* stage32, lds_u4* bm, uint32_t r) {
  const lds_cu4* src = (lds_cu4*)(stage32 + 8 * r);
  const u32x4 v0 = src[0], v1 = src[1];
  const uint32_t x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  uint32_t w[kClasses];
  uc::row_classes(x, w);
  bm[kRowVec * r] = u32x4{w[0], w[1], w[2], w[3]};
  bm[kRowVec * r + 1] = u32x4{w[4], w[5], w[6], w[7]};
  bm[kRowVec * r + 2] = u32x4{w[8], w[9], w[10], w[11]};
}
// A quarter of row r (bytes 8q..8q+7, one 8 x 8 block) per lane, the four
// lanes of a quad together building the row: each lane's transposed block
// is broadcast over the quad (DPP quad_perm) and every lane assembles the
// plane words with the 4 x 4 byte transposes; the quad's first lane derives
// and writes the row.  For the last few rows of a group (a full round would
// leave most lanes idle).
__device__ __forceinline__ void build_quarter_row(lds_u32* stage32, lds_u4* bm, uint32_t r, uint32_t q, bool valid) {
  uint32_t B0 = 0, B1 = 0;
  if (valid) {
    B0 = stage32[8 * r + 2 * q];
    B1 = stage32[8 * r + 2 * q + 1];
    uc::xpose8(B0, B1);
  }
  uint32_t p[8];
  uc::xpose4(dpp_mov<0x00>(0u, B0), dpp_mov<0x55>(0u, B0), dpp_mov<0xAA>(0u, B0), dpp_mov<0xFF>(0u, B0), p);
  uc::xpose4(dpp_mov<0x00>(0u, B1), dpp_mov<0x55>(0u, B1), dpp_mov<0xAA>(0u, B1), dpp_mov<0xFF>(0u, B1), p + 4);
  if (valid && q == 0) {
    uint32_t w[kClasses];
    uc::derive_planes(p, w);
    bm[kRowVec * r] = u32x4{w[0], w[1], w[2], w[3]};
    bm[kRowVec * r + 1] = u32x4{w[4], w[5], w[6], w[7]};
    bm[kRowVec * r + 2] = u32x4{w[8], w[9], w[10], w[11]};
  }
}
__device__ __forceinline__ void build_bitmaps(lds_u32* stage32, lds_u4* bm, uint32_t bytes) {
  const int lane = threadIdx.x & 63;
  const uint32_t rows = (bytes + 31) / 32;
  for (uint32_t r = lane; r < rows; r += kWave) build_row(stage32, bm, r);
}
// Only the rows (bit r of the 96-bit mask {m0, m1, m2}) that hold path bytes:
// every reader of the bitmaps masks its windows to a path's own bytes, so the
// rows between paths (other strings of the arena) are never looked at.  The
// k-th set row is found through a list in LDS (`list`, >= 96 words of the
// wave's free segment list): lane L enters rows L and 64 + L at their rank
// among the set rows (mbcnt), then lane k reads entry k.  (Selecting the k-th
// set bit per lane with a popcount bisection cost about 75 vector
// instructions per row, half of building the row.)
__device__ __forceinline__ void build_bitmaps_rows(lds_u32* stage32, lds_u4* bm, uint32_t m0, uint32_t m1,
                                                   uint32_t m2, uint32_t* list) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t c01 = __builtin_popcount(m0) + __builtin_popcount(m1), total = c01 + __builtin_popcount(m2);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi(m1, __builtin_amdgcn_mbcnt_lo(m0, 0u));   // set rows < lane
  if ((((lane < 32 ? m0 : m1) >> (lane & 31)) & 1u) != 0) list[below] = lane;
  if (lane < 32 && ((m2 >> lane) & 1u) != 0) list[c01 + __builtin_amdgcn_mbcnt_lo(m2, 0u)] = 64 + lane;
  wave_lds_sync();
  // full rounds while 64 rows are left; a last round of at most 16 rows in
  // quarter rows (four lanes per row)
  const uint32_t full = total > kWave && total - (total & ~(kWave - 1)) <= 16 ? total & ~(kWave - 1) : total;
  for (uint32_t k = lane; k < full; k += kWave) build_row(stage32, bm, list[k]);
  if (full < total) {
    const uint32_t k = full + (lane >> 2);
    const bool valid = k < total;
    build_quarter_row(stage32, bm, valid ? list[k] : 0u, lane & 3u, valid);
  }
}
// bits [lo, hi] (rows) of the 32-row word starting at row w0
__device__ __forceinline__ uint32_t row_bits(uint32_t lo, uint32_t hi, uint32_t w0) {
  if (hi < w0 || lo > w0 + 31) return 0u;
  const uint32_t l = lo > w0 ? lo - w0 : 0u, h = min(hi - w0, 31u);
  return (h == 31 ? ~0u : ((2u << h) - 1u)) & ~((1u << l) - 1u);
}

// 64-bit windows of classes [c0, c0+4*nv) starting at stage byte a
template <int NV>
struct WinT {
  uint64_t c[4 * NV];
};
template <int V0, int NV>
__device__ __forceinline__ WinT<NV> load_win(lds_cu4* bm, uint32_t a) {
  const uint32_t r = a >> 5, sh = a & 31;
  WinT<NV> w;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    const u32x4 x0 = bm[kRowVec * r + V0 + v];
    const u32x4 x1 = bm[kRowVec * (r + 1) + V0 + v];
    const u32x4 x2 = bm[kRowVec * (r + 2) + V0 + v];
    const uint32_t w0[4] = {x0.x, x0.y, x0.z, x0.w}, w1[4] = {x1.x, x1.y, x1.z, x1.w}, w2[4] = {x2.x, x2.y, x2.z, x2.w};
#pragma unroll
    for (int c = 0; c < 4; c++)
      w.c[4 * v + c] =
          ((uint64_t)__builtin_amdgcn_alignbit(w2[c], w1[c], sh) << 32) | __builtin_amdgcn_alignbit(w1[c], w0[c], sh);
  }
  return w;
}
// the 64-bit windows of classes 0-5 at stage byte a (what the segment
// classifier reads): per row one 16-byte and one 8-byte read
struct Win {
  uint64_t c[6];
};
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(3))) u32x2 lds_cu2;
__device__ __forceinline__ Win load_win6(lds_cu4* bm, uint32_t a) {
  const uint32_t r = a >> 5, sh = a & 31;
  const lds_cu2* b2 = (const lds_cu2*)bm;
  const u32x4 x0 = bm[kRowVec * r], x1 = bm[kRowVec * (r + 1)], x2 = bm[kRowVec * (r + 2)];
  const u32x2 y0 = b2[2 * (kRowVec * r + 1)], y1 = b2[2 * (kRowVec * (r + 1) + 1)], y2 = b2[2 * (kRowVec * (r + 2) + 1)];
  const uint32_t w0[6] = {x0.x, x0.y, x0.z, x0.w, y0.x, y0.y}, w1[6] = {x1.x, x1.y, x1.z, x1.w, y1.x, y1.y},
                 w2[6] = {x2.x, x2.y, x2.z, x2.w, y2.x, y2.y};
  Win w;
#pragma unroll
  for (int c = 0; c < 6; c++)
    w.c[c] = ((uint64_t)__builtin_amdgcn_alignbit(w2[c], w1[c], sh) << 32) | __builtin_amdgcn_alignbit(w1[c], w0[c], sh);
  return w;
}
__device__ __forceinline__ uint64_t low_mask(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

// first byte of class c in [a, e) (stage coordinates), or e
__device__ __forceinline__ uint32_t first_of(lds_cu4* bm, uint32_t c, uint32_t a, uint32_t e) {
  const lds_u32* b32 = (const lds_u32*)bm;
  while (a < e) {
    const uint32_t r = a >> 5, sh = a & 31;
    const uint32_t m = __builtin_amdgcn_alignbit(b32[4 * kRowVec * (r + 1) + c], b32[4 * kRowVec * r + c], sh) &
                       (uint32_t)low_mask(e - a);
    if (m) return a + __builtin_ctz(m);
    a += 32;
  }
  return e;
}

// datesRegex (templatize.go:67) for a segment of length L from the digit and
// dash windows plus at most four byte reads: every accepted length has one
// fixed shape (10 + {0, 6 "THH:MM", 9 "THH:MM:SS"} + {0, 1 "Z", 5 "+HHMM"}).
// Shape per length: 2 bits T-part (1: none, 2: "THH:MM", 3: "THH:MM:SS";
// 0: no date has this length) | 2 bits zone (0: none, 1: "Z", 2: "+HHMM"),
// 4 bits per L in [0, 32).
constexpr uint64_t date_shape_bits(uint32_t L) {
  return L == 10 ? 0x1 : L == 11 ? 0x5 : L == 15 ? 0x9 : L == 16 ? 0x2 : L == 17 ? 0x6 : L == 21 ? 0xA
       : L == 19 ? 0x3 : L == 20 ? 0x7 : L == 24 ? 0xB : 0x0;
}
constexpr uint64_t date_shape_tab(uint32_t base) {
  uint64_t t = 0;
  for (uint32_t k = 0; k < 16; k++) t |= date_shape_bits(base + k) << (4 * k);
  return t;
}
// the part of date_win that needs no byte reads: the length has a date
// shape and the digit / dash windows fit it
__device__ __forceinline__ uint32_t date_shape(uint32_t L) {
  constexpr uint64_t kLo = date_shape_tab(0), kHi = date_shape_tab(16);
  return L >= 32 ? 0u : (uint32_t)(((L < 16 ? kLo : kHi) >> (4 * (L & 15))) & 15u);
}
__device__ __forceinline__ bool date_pre(uint64_t dg, uint64_t dash, uint32_t L) {
  const uint32_t sh = date_shape(L);
  const uint32_t tsel = sh & 3u, zsel = sh >> 2;
  if (tsel == 0) return false;
  const uint32_t tlen = tsel == 1 ? 0u : tsel == 2 ? 6u : 9u;
  uint64_t dm = 0x36Full;                                     // YYYY-MM-DD digits
  dm |= tsel >= 2 ? (3ull << 11) | (3ull << 14) : 0ull;       // THH:MM
  dm |= tsel == 3 ? 3ull << 17 : 0ull;                        // :SS
  const uint32_t z = 10 + tlen;
  dm |= zsel == 2 ? 0xFull << (z + 1) : 0ull;                 // +HHMM
  return (dg & dm) == dm && ((dash >> 4) & 1) != 0 && ((dash >> 7) & 1) != 0;
}
template <class R>
__device__ __forceinline__ bool date_win(R& rd, uint64_t dg, uint64_t dash, uint32_t s, uint32_t L) {
  if (!date_pre(dg, dash, L)) return false;
  const uint32_t sh = date_shape(L);
  const uint32_t tsel = sh & 3u, zsel = sh >> 2;
  const uint32_t tlen = tsel == 1 ? 0u : tsel == 2 ? 6u : 9u;
  // bytes 10-13 and 16-19 hold every fixed punctuation position and the zone
  const uint32_t wa = rd.word(s + 10), wb = rd.word(s + 16);
  const uint32_t c_t = wa & 0xFFu, c_c1 = (wa >> 24) & 0xFFu, c_c2 = wb & 0xFFu;
  const uint32_t c_z = tlen == 0 ? c_t : tlen == 6 ? c_c2 : wb >> 24;
  return (tlen == 0 || (c_t == 'T' && c_c1 == ':')) && (tlen != 9 || c_c2 == ':') &&
         (zsel == 0 || (zsel == 1 ? c_z == 'Z' : (c_z == '+' || c_z == '-')));
}

// emailRegex (templatize.go:70) from the class windows: exactly one '@' at p,
// local [0,p) >= 1 byte of [A-Za-z0-9._%+-], domain (p,L) all [A-Za-z0-9.-]
// whose last '.' is at domain index >= 1 and is followed by >= 2 letters.
__device__ __forceinline__ bool email_win(uint64_t at, lds_cu4* bm, uint32_t a, uint32_t L) {
  const uint64_t M = low_mask(L);
  const uint32_t p = (uint32_t)__builtin_ctzll(at);
  if (p == 0) return false;
  const WinT<1> e = load_win<2, 1>(bm, a);   // BLOC, BDOM, DOT, NAL
  const uint64_t dom = M & ~low_mask(p + 1);
  if ((e.c[0] & low_mask(p)) || (e.c[1] & dom)) return false;
  const uint64_t dots = e.c[2] & dom;
  if (!dots) return false;
  const uint32_t q = 63 - (uint32_t)__builtin_clzll(dots);
  if (q < p + 2 || L - q - 1 < 2) return false;
  return (e.c[3] & M & ~low_mask(q + 1)) == 0;
}

// has_fffd for a segment of length L <= 64 at s whose high-bit bytes are the
// set bits of hm: only the sequences are visited, each from one word read
// (UTF-8 rules as in has_fffd above).
template <class R>
__device__ __forceinline__ bool has_fffd_win(R& rd, uint64_t hm, uint32_t s, uint32_t L) {
  while (hm) {
    const uint32_t q = (uint32_t)__builtin_ctzll(hm);
    const uint32_t x = rd.word(s + q), c = x & 0xFFu;
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return true;
    if (q + need >= L) return true;
    const uint32_t b1 = (x >> 8) & 0xFFu, b2 = (x >> 16) & 0xFFu, b3 = x >> 24;
    if (b1 < lo || b1 > hi) return true;
    if (need >= 2 && (b2 < 0x80u || b2 > 0xBFu)) return true;
    if (need == 3 && (b3 < 0x80u || b3 > 0xBFu)) return true;
    if (need == 2 && (x & 0xFFFFFFu) == 0xBDBFEFu) return true;
    hm &= ~low_mask(q + need + 1);
  }
  return false;
}

// getSegmentTemplatizationString (templatize.go:242-269) from the class
// windows of a segment of length L <= 64 starting at s (reader coordinates,
// stage byte a).
constexpr uint64_t kUuidDash = (1ull << 8) | (1ull << 13) | (1ull << 18) | (1ull << 23);
constexpr uint64_t kUuidHex = ((1ull << 36) - 1) & ~kUuidDash;
template <class R>
__device__ __forceinline__ int classify_win(const Cfg& cfg, R& rd, const Win& w, lds_cu4* bm, uint32_t a, uint32_t s,
                                            uint32_t L) {
  const uint64_t M = low_mask(L);
  for (uint32_t k = 0; k < cfg.n_custom; k++) {   // custom ids first, in config order
    const UrlCustomDev& cu = reinterpret_cast<const UrlCustomDev*>(cfg.blob + cfg.h->custom_off)[k];
    if (dfa_match(cfg.blob, cfg.dfa_off(cu.dfa), rd, s, s + L)) return (int)cu.name;
  }
  if (date_win(rd, w.c[C_DG], w.c[C_DASH], s, L)) return kNameDate;
  const bool any_hi = (w.c[C_HI] & M) != 0;
  const uint64_t at = w.c[C_AT] & M;
  if (!any_hi && at && (at & (at - 1)) == 0 && email_win(at, bm, a, L)) return kNameEmail;
  const uint64_t d = w.c[C_DG] & M, d1 = d & (d >> 1), d2 = d1 & (d1 >> 2), d7 = d2 & (d2 >> 3);
  if ((L > 0 && (w.c[C_BNL] & M) == 0) || d7 || ((w.c[C_BHX] & M) == 0 && L >= 16 && (L & 1) == 0)) return kNameId;
  if (L >= 36) {
    const uint64_t hx = ~w.c[C_BHX], ds = w.c[C_DASH], sh = L - 36;
    if (((hx & kUuidHex) == kUuidHex && (ds & kUuidDash) == kUuidDash) ||
        (((hx >> sh) & kUuidHex) == kUuidHex && ((ds >> sh) & kUuidDash) == kUuidDash))
      return kNameId;
  }
  if (any_hi && has_fffd_win(rd, w.c[C_HI] & M, s, L)) return kNameId;
  return -1;
}

// datesRegex as one expression (no early exit): the length's shape, the
// digit and dash windows, and bytes 10-13 (wa) / 16-19 (wb) of the segment
__device__ __forceinline__ bool date_flat(uint64_t dg, uint64_t dash, uint32_t L, uint32_t wa, uint32_t wb) {
  const uint32_t sh = date_shape(L);
  const uint32_t tsel = sh & 3u, zsel = sh >> 2;
  const uint32_t tlen = tsel == 1 ? 0u : tsel == 2 ? 6u : 9u;
  uint64_t dm = 0x36Full;                                     // YYYY-MM-DD digits
  dm |= tsel >= 2 ? (3ull << 11) | (3ull << 14) : 0ull;       // THH:MM
  dm |= tsel == 3 ? 3ull << 17 : 0ull;                        // :SS
  dm |= zsel == 2 ? 0xFull << (11 + tlen) : 0ull;             // +HHMM
  const uint32_t c_t = wa & 0xFFu, c_c1 = (wa >> 24) & 0xFFu, c_c2 = wb & 0xFFu;
  const uint32_t c_z = tlen == 0 ? c_t : tlen == 6 ? c_c2 : wb >> 24;
  const bool zone = zsel == 0 ? true : zsel == 1 ? c_z == 'Z' : (c_z == '+') | (c_z == '-');
  return (tsel != 0) & ((dg & dm) == dm) & ((((dash >> 4) & (dash >> 7)) & 1) != 0) &
         ((tlen == 0) | ((c_t == 'T') & (c_c1 == ':'))) & ((tlen != 9) | (c_c2 == ':')) & zone;
}
// emailRegex as one expression, given that the segment holds exactly one '@'
// (at) and no byte >= 0x80; e: the BLOC, BDOM, DOT, NAL windows
__device__ __forceinline__ bool email_flat(uint64_t at, const WinT<1>& e, uint32_t L) {
  const uint64_t M = low_mask(L);
  const uint32_t p = (uint32_t)__builtin_ctzll(at | (1ull << 63));
  const uint64_t dom = M & ~low_mask(p + 1);
  const uint64_t dots = e.c[2] & dom;
  const uint32_t q = 63 - (uint32_t)__builtin_clzll(dots | 1ull);
  return (p != 0) & ((e.c[0] & low_mask(p)) == 0) & ((e.c[1] & dom) == 0) & (dots != 0) & (q >= p + 2) &
         (L >= q + 3) & ((e.c[3] & M & ~low_mask(q + 1)) == 0);
}

// classify_win for the default configuration (no custom ids), without
// branches: every predicate of getSegmentTemplatizationString is evaluated
// for every lane from its windows and the date bytes, and the first that
// holds in templatize.go's order (date, email, the ID rules) names the
// segment.  The short-circuit form compiled to nested exec-mask branches
// (about 300 scalar instructions per 64-segment step, more than its vector
// work) although nearly every branch was taken by some lane of the step.
// Only the U+FFFD walk stays a loop, entered when some lane needs it.
template <class R>
__device__ __forceinline__ int classify_spec(const Cfg& cfg, R& rd, lds_cu4* bm, uint32_t a, uint32_t s, uint32_t L) {
  const Win w = load_win6(bm, a);
  const WinT<1> e = load_win<2, 1>(bm, a);
  const uint32_t wa = rd.word(s + 10), wb = rd.word(s + 16);
  if (cfg.n_custom) return classify_win(cfg, rd, w, bm, a, s, L);
  const uint64_t M = low_mask(L);
  const bool date = date_flat(w.c[C_DG], w.c[C_DASH], L, wa, wb);
  const uint64_t hm = w.c[C_HI] & M;
  const uint64_t at = w.c[C_AT] & M;
  const bool email = (hm == 0) & (at != 0) & ((at & (at - 1)) == 0) & email_flat(at, e, L);
  const uint64_t d = w.c[C_DG] & M, d1 = d & (d >> 1), d2 = d1 & (d1 >> 2), d7 = d2 & (d2 >> 3);
  const uint64_t hx = ~w.c[C_BHX], ds = w.c[C_DASH], sh = L >= 36 ? L - 36 : 0;
  const bool uuid = (L >= 36) & ((((hx & kUuidHex) == kUuidHex) & ((ds & kUuidDash) == kUuidDash)) |
                                 ((((hx >> sh) & kUuidHex) == kUuidHex) & (((ds >> sh) & kUuidDash) == kUuidDash)));
  const bool idp = ((L > 0) & ((w.c[C_BNL] & M) == 0)) | (d7 != 0) |
                   (((w.c[C_BHX] & M) == 0) & (L >= 16) & ((L & 1) == 0)) | uuid;
  int id = date ? (int)kNameDate : email ? (int)kNameEmail : idp ? (int)kNameId : -1;
  const bool fffd = (hm != 0) & (id < 0);
  if (__ballot(fffd) != 0 && fffd && has_fffd_win(rd, hm, s, L)) id = kNameId;
  return id;
}

// Rare paths kept out of line so the hot LDS->LDS instantiation stays small:
// a group whose bytes do not fit the stage reads HBM, a tile whose output
// does not fit the LDS image writes HBM.
__device__ __noinline__ Plan plan_global(const Cfg& cfg, const uint8_t* p, uint32_t plen, uint32_t f) {
  ByteReader rd(p);
  return plan_path(cfg, rd, plen, f);
}
template <class R, class P>
__device__ __noinline__ void emit_out_of_line(const Cfg& cfg, R rd, uint32_t plen, uint32_t f, uint32_t mode,
                                              uint32_t lead, bool slow, uint32_t field, uint64_t code, P dst,
                                              uint32_t cap) {
  Put<P> put{dst, 0, cap};
  emit_path(cfg, rd, plen, f, mode, lead, slow, field, code, put);
}

// plan meta word: mode 3 | lead 1 | slow 1 | url_out 2 | field 25
__device__ __forceinline__ uint32_t pack_meta(uint32_t mode, uint32_t lead, bool slow, uint32_t oflags, uint32_t field) {
  return mode | (lead << 3) | ((uint32_t)slow << 4) | (oflags << 5) | (field << 7);
}

constexpr uint32_t kNamesLds = 512;
constexpr uint32_t kWaveOut = 4 * 1024;   // per-wave LDS image of one group's output


// Copies the arena bytes [lo, hi) the wave's 64 lanes reference (16-byte
// aligned down) into the wave's LDS slice.  Returns the aligned start (and
// the copied size in *nbytes), or ~0u when the range does not fit (lanes then
// read HBM directly).
__device__ uint32_t stage_wave(uint8_t* stage, const uint8_t* arena, uint32_t lo, uint32_t hi, uint32_t* nbytes) {
  const int lane = threadIdx.x & 63;
  lo = wave_min_u32(lo);
  hi = wave_max_u32(hi);
  *nbytes = 0;
  if (lo >= hi) return 0;   // no lane reads bytes
  const uint32_t lo16 = lo & ~15u;
  const uint32_t bytes = (hi - lo16 + 15u) & ~15u;
  if (bytes > kStage) return ~0u;
  *nbytes = bytes;
  const uint4* src = reinterpret_cast<const uint4*>(arena + lo16);
  uint4* dst = reinterpret_cast<uint4*>(stage);
  for (uint32_t x = lane; x < bytes / 16; x += kWave) dst[x] = src[x];
  wave_lds_sync();
  return lo16;
}

// Names and name table in LDS (whole workgroup, once).
struct NamesSmem {
  UrlCfgDev hdr;
  uint8_t names[kNamesLds];
  NameDev name_tab[kNameTab];
};
__device__ __forceinline__ Cfg load_cfg(const UrlKernelArgs& a, NamesSmem& ns) {
  const UrlCfgDev h = *reinterpret_cast<const UrlCfgDev*>(a.cfg);
  const uint32_t names_len = min(kNamesLds, h.total_bytes - h.bytes_off);
  for (uint32_t k = threadIdx.x; k < names_len; k += blockDim.x) ns.names[k] = a.cfg[h.bytes_off + k];
  if (threadIdx.x < min(h.n_names, kNameTab))
    ns.name_tab[threadIdx.x] = reinterpret_cast<const NameDev*>(a.cfg + h.names_off)[threadIdx.x];
  if (threadIdx.x == 0) ns.hdr = h;
  __syncthreads();
  return Cfg{a.cfg, (lds_cfg*)&ns.hdr, h.n_custom, h.n_rules, h.max_rule_nseg, h.names_off, h.n_names <= kNameTab ? 1u : 0u,
             (lds_u8*)ns.names, names_len, a.ablate,
             (const __attribute__((address_space(3))) NameDev*)ns.name_tab};
}

// diagnostics (UrlKernelArgs::dbg): wave-uniform shader clock
__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

// ---------------------------------------------------------------------------
// Software pipeline shared by K1 and K3: a wave's next group's arena bytes
// are loaded into registers (16 B x 4 per lane covers the 4 KB stage) before
// it works on the current group, and written to its LDS slice afterwards.
struct StagePf {
  uint4 v0, v1, v2, v3;
  uint32_t lo16, bytes;   // bytes == 0: nothing to stage; lo16 == ~0u: range too large (HBM reads)
};
__device__ __forceinline__ StagePf stage_issue(const uint8_t* arena, uint32_t lo, uint32_t hi) {
  const int lane = threadIdx.x & 63;
  lo = wave_min_u32(lo);
  hi = wave_max_u32(hi);
  StagePf pf;
  pf.lo16 = 0;
  pf.bytes = 0;
  if (lo >= hi) return pf;
  pf.lo16 = lo & ~15u;
  const uint32_t bytes = (hi - pf.lo16 + 15u) & ~15u;
  if (bytes > kStage) {
    pf.lo16 = ~0u;
    return pf;
  }
  pf.bytes = bytes;
  const uint4* src = reinterpret_cast<const uint4*>(arena + pf.lo16);
  const uint32_t nv = bytes / 16;
  if (lane < nv) pf.v0 = src[lane];
  if (lane + 64 < nv) pf.v1 = src[lane + 64];
  if (lane + 128 < nv) pf.v2 = src[lane + 128];
  if (lane + 192 < nv) pf.v3 = src[lane + 192];
  return pf;
}
__device__ __forceinline__ void stage_commit(const StagePf& pf, uint8_t* stage) {
  const int lane = threadIdx.x & 63;
  const uint32_t nv = pf.bytes / 16;
  uint4* dst = reinterpret_cast<uint4*>(stage);
  if (lane < nv) dst[lane] = pf.v0;
  if (lane + 64 < nv) dst[lane + 64] = pf.v1;
  if (lane + 128 < nv) dst[lane + 128] = pf.v2;
  if (lane + 192 < nv) dst[lane + 192] = pf.v3;
  wave_lds_sync();
}

// Persistent grid: every wave walks groups g = first, first + stride, ...
__device__ __forceinline__ uint32_t wave_first_group() { return blockIdx.x * kWaves + (threadIdx.x >> 6); }
__device__ __forceinline__ uint32_t wave_stride() { return gridDim.x * kWaves; }

// ---------------------------------------------------------------------------
// Output helpers shared by the plan kernel's writer and K3s.
typedef __attribute__((address_space(3))) uint32_t lds_w32;
struct PutOr {
  lds_w32* img;
  uint32_t wpos, nb;   // wpos: image offset of acc's first byte (dword aligned); nb: bytes in acc
  uint64_t acc;
  __device__ PutOr(lds_w32* im, uint32_t start) : img(im), wpos(start & ~3u), nb(start & 3u), acc(0) {}
  __device__ __forceinline__ void flush() {
    __hip_atomic_fetch_or(&img[wpos >> 2], (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    acc >>= 32;
    wpos += 4;
    nb -= 4;
  }
  __device__ __forceinline__ void byte(uint32_t c) {
    acc |= (uint64_t)(c & 0xFFu) << (8 * nb);
    if (++nb == 4) flush();
  }
  __device__ __forceinline__ void word(uint32_t x, uint32_t nv) {
    if (nv < 4) x &= (1u << (8 * nv)) - 1u;
    acc |= (uint64_t)x << (8 * nb);
    nb += nv;
    if (nb >= 4) flush();
  }
  __device__ __forceinline__ void finish() {
    if (nb) __hip_atomic_fetch_or(&img[wpos >> 2], (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
};


constexpr uint32_t kBNames = 1024;    // braced names for template ids 0..14, each after a '/'
typedef __attribute__((address_space(3))) uint16_t lds_w16;

struct BracedNames {
  __attribute__((aligned(16))) uint8_t b[kBNames + 16];
  uint16_t off[16];
  uint8_t len[16];
  uint32_t ok;
};

// "{name}" for ids 0..14 (the ids a plan code can carry), once per workgroup,
// as "/{id}/{date}/{email}/...": the byte before every name is '/' (the
// assembly copies an entry's separator with its body).
__device__ void load_braced_names(const Cfg& cfg, BracedNames& bn) {
  if (threadIdx.x == 0) {
    const uint32_t nn = min(cfg.h->n_names, 15u);
    uint32_t o = 1;
    bool ok = true;
    bn.b[0] = '/';
    for (uint32_t id = 0; id < nn; id++) {
      const uint32_t l = cfg.name(id).len + 2;
      if (o + l + 1 > kBNames || l > 255) { ok = false; break; }
      bn.off[id] = (uint16_t)o;
      bn.len[id] = (uint8_t)l;
      bn.b[o + l] = '/';
      o += l + 1;
    }
    bn.ok = ok ? 1u : 0u;
  }
  __syncthreads();
  if (bn.ok && threadIdx.x < min(cfg.h->n_names, 15u)) {
    const NameDev nm = cfg.name(threadIdx.x);
    const uint8_t* src = cfg.blob + cfg.h->bytes_off + nm.off;
    uint8_t* d = bn.b + bn.off[threadIdx.x];
    d[0] = '{';
    for (uint32_t q = 0; q < nm.len; q++) d[1 + q] = src[q];
    d[1 + nm.len] = '}';
  }
  __syncthreads();
}


__device__ __forceinline__ uint32_t lds_word(const lds_u8* L, uint32_t p) {
  const lds_u32* w = (const lds_u32*)(L + (p & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], p & 3);
}


// The columns K3s reads for one group.
struct EmitCols {
  uint32_t len, meta;
  uint64_t code;
  ose_strref pr;
  uint64_t base, gsum;
};
__device__ __forceinline__ EmitCols emit_cols(const UrlKernelArgs& a, uint32_t g, int lane) {
  EmitCols c{0, 0, 0, {0, 0}, 0, 0};
  const uint64_t i = (uint64_t)g * kWave + lane;
  if (g < a.n_groups) {
    c.base = a.group_base[g];
    c.gsum = a.group_sum[g];
  }
  if (i < a.n_spans) {
    c.len = a.plan_len[i];
    c.meta = a.plan_meta[i];
    c.code = a.plan_code[i];
    c.pr = a.path[i];
  }
  return c;
}
__device__ __forceinline__ bool emit_needs_path(uint32_t meta) {
  const uint32_t mode = meta & 7u;
  return mode == M_RULE || mode == M_DEFAULT || mode == M_ORIG;
}

// image dword k <-> global bytes [base - shift + 4k, +4); bytes outside
// [base, base + gtotal) belong to the neighbouring groups, so partial dwords
// at the ends are stored bytewise
__device__ __forceinline__ void store_image(const UrlKernelArgs& a, const lds_w32* img, uint64_t base, uint32_t shift,
                                            uint64_t gtotal) {
  const int lane = threadIdx.x & 63;
  uint8_t* gdst = a.out_arena + (base - shift);
  const uint32_t nd = (uint32_t)((shift + gtotal + 3) / 4);
  const uint64_t endb = shift + gtotal;
  for (uint32_t k = lane; k < nd; k += kWave) {
    const uint32_t w = img[k];
    const uint32_t b0 = 4 * k;
    if (b0 >= shift && b0 + 4 <= endb) {
      *reinterpret_cast<uint32_t*>(gdst + b0) = w;
    } else {
      for (uint32_t q = 0; q < 4; q++)
        if (b0 + q >= shift && b0 + q < endb) gdst[b0 + q] = (uint8_t)(w >> (8 * q));
    }
  }
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  const uint32_t incl = wave_incl_sum_u32(v);
  *total = lane_value(incl, kWave - 1);
  return incl - v;
}


// ---------------------------------------------------------------------------
// K1: plan and assemble.  Waves are independent (no workgroup barrier after
// the config load); per group: class bitmaps of the staged bytes, the segment
// list and its classification, one plan per span, then the group's template
// bytes, written from the segment list into an LDS image (over the bitmaps,
// which are dead by then) and stored to the wave's scratch region.  The
// group's place in the output arena is only known after K2, so K4 moves the
// image there; the path bytes are read from HBM once.
constexpr uint32_t kSegCap = 192;   // per-wave segment list (C2 groups hold ~118 segments, max seen 182)
// K1 stages each group through LDS-DMA into a per-wave buffer: the next
// group's copy is issued as soon as this group's assembly is done with the
// buffer, and waited for at the top of the next iteration.  3 KB covers 99.9%
// of C2/C4 groups as one contiguous range (p99 of a group's byte range is
// 2.9 KB); a wider range is gathered path by path (stage_dma), and a group
// whose paths alone overflow goes to url_plan_slow_kernel.  One 3 KB buffer +
// 12-class bitmaps + segment list per wave (39.7 KB per 4-wave workgroup) and
// <= 128 VGPRs keep four workgroups per CU; a second buffer, prefetching a
// whole group ahead, held the kernel to three (52 KB) and measured 8% slower
// (C4 plan 7.45 vs 6.84 ms, round 2).
constexpr uint32_t kPlanStage = 3 * 1024;
constexpr uint32_t kPlanBmRows = kPlanStage / 32 + 3;
struct PlanSmem {
  NamesSmem ns;
  __attribute__((aligned(16))) uint8_t stage[kWaves][kPlanStage + 16];
  __attribute__((aligned(16))) u32x4 bm[kWaves][kRowVec * kPlanBmRows];   // class bitmaps, then the output image
  uint32_t segs[kWaves][kSegCap];   // enumerated segments (start | len | owner lane)
  uint32_t cls[kWaves][kSegCap + 8];   // their classification (out_len << 8 | id + 1); 8 entries of
                                        // padding for the fold's fixed 8-entry read
  BracedNames bn;
};
constexpr uint32_t kImgCap = kRowVec * kPlanBmRows * 16;   // bytes of one wave's output image

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
struct StageDma {
  // per lane: a path at arena offset o sits at stage offset o - base (base is
  // wave-uniform for a contiguous copy, per lane for a gather); bytes == 0:
  // nothing staged; base == ~0u: the wave's paths do not fit the stage
  uint32_t base, bytes;
};
// Issues the copy of the arena bytes the wave's lanes reference into `stage` by
// LDS-DMA (global_load_lds_dwordx4: lane k's 16 bytes land at stage + 16k of
// each 1 KB piece).  When the wave's range [min lo, max hi) fits, it is copied
// whole (16-byte aligned down).  When it does not (paths spread through other
// strings of the arena: C4's routes, the span messages of an OTLP-decoded
// batch), each lane's path is gathered as its own 16-byte chunks, packed in
// lane order: slot x of the stage takes chunk x - cs(L) of owner L, the last
// lane whose exclusive chunk scan cs(L) <= x (binary search over shuffles).
// The caller waits vmcnt before reading the buffer.
__device__ __forceinline__ StageDma stage_dma(const uint8_t* arena, uint32_t lo_l, uint32_t hi_l, uint8_t* stage) {
  const int lane = threadIdx.x & 63;
  const uint32_t lo = wave_min_u32(lo_l), hi = wave_max_u32(hi_l);
  StageDma sd{0, 0};
  if (lo >= hi) return sd;
  const uint32_t lo16 = lo & ~15u;
  const uint32_t bytes = (hi - lo16 + 15u) & ~15u;
  if (bytes <= kPlanStage) {
    sd.base = lo16;
    sd.bytes = bytes;
    const uint4* src = reinterpret_cast<const uint4*>(arena + lo16) + lane;
    const uint32_t nv = bytes / 16;
#pragma unroll
    for (uint32_t k = 0; k < kPlanStage / 1024; k++)
      if (lane + 64 * k < nv)
        __builtin_amdgcn_global_load_lds((glb_void*)(src + 64 * k), (lds_void*)(stage + 1024 * k), 16, 0, 0);
    return sd;
  }
  const uint32_t nc = lo_l < hi_l ? ((hi_l + 15u) >> 4) - (lo_l >> 4) : 0u;
  uint32_t total;
  const uint32_t cs = wave_excl_scan(nc, &total);
  if (total * 16 > kPlanStage) {
    sd.base = ~0u;
    return sd;
  }
  sd.base = lo_l < hi_l ? lo_l - (16 * cs + (lo_l & 15u)) : 0u;
  sd.bytes = total * 16;
  const uint32_t ch = (lo_l >> 4) - cs;   // chunk index of slot x, lane L: x + ch(L)
#pragma unroll
  for (uint32_t k = 0; k < kPlanStage / 1024; k++) {
    const uint32_t x = lane + 64 * k;
    if (64 * k < total) {   // wave-uniform
      uint32_t o = 0;
#pragma unroll
      for (uint32_t step = 32; step; step >>= 1)
        if (__shfl(cs, (int)(o + step)) <= x) o += step;
      const uint32_t c = (uint32_t)__shfl(ch, (int)o) + x;
      if (x < total)
        __builtin_amdgcn_global_load_lds((glb_void*)(arena + 16ull * c), (lds_void*)(stage + 1024 * k), 16, 0, 0);
    }
  }
  return sd;
}
__device__ __forceinline__ void wait_dma() {
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  wave_lds_sync();
}

// number of bytes of class c in [a, e) (stage coordinates)
__device__ __forceinline__ uint32_t count_of(lds_cu4* bm, uint32_t c, uint32_t a, uint32_t e) {
  const lds_u32* b32 = (const lds_u32*)bm;
  uint32_t k = 0;
  while (a < e) {
    const uint32_t r = a >> 5, sh = a & 31;
    k += __builtin_popcount(__builtin_amdgcn_alignbit(b32[4 * kRowVec * (r + 1) + c], b32[4 * kRowVec * r + c], sh) &
                            (uint32_t)low_mask(e - a));
    a += 32;
  }
  return k;
}

// 64-bit mask of bits [lo, hi) of the 64-bit half starting at bit `base` of a
// 128-bit window (lo, hi are window coordinates)
__device__ __forceinline__ uint64_t half_mask(uint32_t lo, uint32_t hi, uint32_t base) {
  const uint32_t l = lo > base ? min(lo - base, 64u) : 0u, h = hi > base ? min(hi - base, 64u) : 0u;
  return low_mask(h) & ~low_mask(l);
}

// length of name `id`: the LDS table for the first kNameTab names, else a
// call (a global load inline would make the classify loop wait for every
// vector-memory operation in flight, the next group's stage included)
__device__ __noinline__ uint32_t name_len_global(const uint8_t* blob, uint32_t names_off, uint32_t id) {
  return reinterpret_cast<const NameDev*>(blob + names_off)[id].len;
}
__device__ __forceinline__ uint32_t name_len(const Cfg& cfg, uint32_t id) {
  if (cfg.names_tab_all || id < kNameTab) return cfg.name_tab[id].len;
  return name_len_global(cfg.blob, cfg.names_off, id);
}


// Phase 1 for a whole group through a segment list: each lane enumerates its
// span's segments into the wave's list; the wave classifies the list 64
// segments per step (about 2 steps for a C2 group, instead of one step per
// segment index of the longest path); each lane then folds its own entries.
// Entries: start 12 | len 13 | owner lane 6 before classification, then
// out_len << 8 | (id + 1) where out_len is what the segment adds to the
// template ({name} or itself).
// A path whose bytes lie in 6 bitmap rows (the common case) finds its '?' cut,
// leading '/' and segment ends in one read of those rows' slash and '?' words
// and folds its entries (<= 8) in one read; longer paths walk the rows.
// Returns false when the list would overflow or a segment is longer than 64
// bytes (the group is then planned by url_plan_slow_kernel).
// cls: where the classified entries go (== segs: in place; else segs keeps
// the enumerated entries for the fused writer).  *big_id: some segment of
// this lane's path took a name id the braced-name table does not hold.
__device__ __forceinline__ bool plan_group_list(const Cfg& cfg, lds_u32* stage32, lds_cu4* bm, uint32_t* segs,
                                                bool needs_path, uint32_t p0, uint32_t plen, uint32_t f, Plan& p,
                                                bool tm, uint64_t* tt, uint32_t* cls = nullptr,
                                                uint32_t* seg_off = nullptr, bool* big_id = nullptr) {
  if (!cls) cls = segs;
  const int lane = threadIdx.x & 63;
  uint64_t c0 = tm ? clk() : 0;
  LdsReader rd(stage32, p0);
  const lds_u32* b32 = (const lds_u32*)bm;
  uint32_t n = 0, nseg = 0;
  // window: stage bytes [32 r0, 32 r0 + 192) (6 bitmap rows, p99 of a C2
  // path is 129 bytes), the path at window bit b0 < 32
  const uint32_t r0 = p0 >> 5, b0 = p0 & 31;
  const bool win = needs_path && b0 + plen <= 192;
  uint64_t sl0 = 0, sl1 = 0, sl2 = 0;
  if (needs_path) {
    if (win) {
      uint32_t w[12];
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const uint32_t r = min(r0 + j, kPlanBmRows - 1);   // rows past the path are masked off below
        w[j] = b32[4 * kRowVec * r + C_SL];
        w[6 + j] = b32[4 * kRowVec * r + C_QM];
      }
      sl0 = w[0] | ((uint64_t)w[1] << 32);
      sl1 = w[2] | ((uint64_t)w[3] << 32);
      sl2 = w[4] | ((uint64_t)w[5] << 32);
      n = plen;
      if ((f & OSE_URL_PATH_MASK) == OSE_URL_PATH_TARGET) {   // strings.SplitN(target, "?", 2)[0]
        const uint64_t q0 = (w[6] | ((uint64_t)w[7] << 32)) & half_mask(b0, b0 + plen, 0);
        const uint64_t q1 = (w[8] | ((uint64_t)w[9] << 32)) & half_mask(b0, b0 + plen, 64);
        const uint64_t q2 = (w[10] | ((uint64_t)w[11] << 32)) & half_mask(b0, b0 + plen, 128);
        if (q0) n = (uint32_t)__builtin_ctzll(q0) - b0;
        else if (q1) n = 64 + (uint32_t)__builtin_ctzll(q1) - b0;
        else if (q2) n = 128 + (uint32_t)__builtin_ctzll(q2) - b0;
      }
      p.lead = (n > 0 && ((sl0 >> b0) & 1)) ? 1 : 0;
    } else {
      n = (f & OSE_URL_PATH_MASK) == OSE_URL_PATH_TARGET ? first_of(bm, C_QM, p0, p0 + plen) - p0 : plen;
      p.lead = (n > 0 && rd.at(0) == '/') ? 1 : 0;
    }
    if (n == p.lead) {   // "" or "/" -> "/" (processor.go:156-160)
      p.mode = M_SLASH;
      p.len = 1;
    } else {
      if (win) {
        sl0 &= half_mask(b0 + p.lead, b0 + n, 0);
        sl1 &= half_mask(b0 + p.lead, b0 + n, 64);
        sl2 &= half_mask(b0 + p.lead, b0 + n, 128);
        nseg = 1 + __builtin_popcountll(sl0) + __builtin_popcountll(sl1) + __builtin_popcountll(sl2);
      } else {
        nseg = 1 + count_of(bm, C_SL, p0 + p.lead, p0 + n);
      }
      if (cfg.n_rules && nseg <= cfg.max_rule_nseg) {   // processor.go:162-171: rules first
        const uint32_t* by_len = reinterpret_cast<const uint32_t*>(cfg.blob + cfg.h->rules_by_len_off);
        const UrlRuleDev* rules = reinterpret_cast<const UrlRuleDev*>(cfg.blob + cfg.h->rules_off);
        for (uint32_t r = by_len[nseg]; r < by_len[nseg + 1]; r++) {
          const int64_t l = attempt_rule(cfg, rules[r], rd, p.lead, n);
          if (l >= 0) {
            p.mode = M_RULE;
            p.field = r;
            p.len = p.lead + (uint32_t)l;
            nseg = 0;
            break;
          }
        }
      }
    }
  }
  const uint32_t incl = wave_incl_sum_u32(nseg);
  const uint32_t total = lane_value(incl, kWave - 1);
  if (total > kSegCap) return false;
  const uint32_t off = incl - nseg;
  if (nseg) {   // enumerate
    const uint32_t bend = p0 + n;
    uint32_t s = p0 + p.lead, k = 0;
    const uint32_t own = (uint32_t)lane << 25;   // the entry's span (the fused writer's owner lane)
    if (win) {
      const uint32_t wb = p0 - b0;   // stage coordinate of window bit 0
      for (uint64_t m = sl0; m; m &= m - 1) {
        const uint32_t e = wb + (uint32_t)__builtin_ctzll(m);
        segs[off + k++] = s | ((e - s) << 12) | own;
        s = e + 1;
      }
      for (uint64_t m = sl1; m; m &= m - 1) {
        const uint32_t e = wb + 64 + (uint32_t)__builtin_ctzll(m);
        segs[off + k++] = s | ((e - s) << 12) | own;
        s = e + 1;
      }
      for (uint64_t m = sl2; m; m &= m - 1) {
        const uint32_t e = wb + 128 + (uint32_t)__builtin_ctzll(m);
        segs[off + k++] = s | ((e - s) << 12) | own;
        s = e + 1;
      }
      segs[off + k] = s | ((bend - s) << 12) | own;
    } else {
      for (; k < nseg; k++) {
        const uint32_t e = k + 1 < nseg ? first_of(bm, C_SL, s, bend) : bend;
        segs[off + k] = s | ((e - s) << 12) | own;
        s = e + 1;
      }
    }
  }
  wave_lds_sync();
  if (tm) { const uint64_t c1 = clk(); tt[0] += c1 - c0; c0 = c1; }
  LdsReader rd0(stage32, 0);
  bool longseg = false;
  // id + 1 in 8 bits: 255 stands for every id >= 254 (such plans are `slow`
  // and re-classify their segments when emitted)
  auto put_cls = [&](uint32_t x, int id, uint32_t L) {
    // without custom ids a segment's id is a built-in name ("id", "date",
    // "email": engine.cpp's name table): its length without an LDS read
    const uint32_t nl = cfg.n_custom == 0 ? (id <= 0 ? 2u : id == 1 ? 4u : 5u)
                        : cfg.names_tab_all ? (uint32_t)cfg.name_tab[id >= 0 ? id : 0].len
                                            : (id >= 0 ? name_len(cfg, (uint32_t)id) : 0u);
    const uint32_t out = id >= 0 ? nl + 2 : L;
    cls[x] = (out << 8) | min((uint32_t)(id + 1), 255u);
  };
  for (uint32_t x0 = 0; x0 < total; x0 += kWave) {   // classify
    const uint32_t x = x0 + (uint32_t)lane;
    if (x < total) {
      const uint32_t ent = segs[x];
      const uint32_t s = ent & 0xFFFu, L = (ent >> 12) & 0x1FFFu;
      int id = -1;
      if (L <= 64)
        id = classify_spec(cfg, rd0, bm, s, s, L);
      else
        longseg = true;   // a segment longer than a 64-bit window: the group goes to url_plan_slow_kernel
      put_cls(x, id, L);
    }
  }
  wave_lds_sync();
  if (__ballot(longseg)) return false;
  if (tm) { const uint64_t c1 = clk(); tt[1] += c1 - c0; c0 = c1; }
  bool big = false;
  if (nseg) {   // fold
    uint32_t l = p.lead + nseg - 1;
    bool templated = false;
    if (nseg <= 8) {   // one read of the (at most 8) entries, folded without branches
      // (entries past the list are read from the list's padding and masked)
      uint32_t r[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) r[k] = cls[off + k];
      uint32_t any = 0, bigm = 0, code = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        const uint32_t v = k < nseg ? r[k] : 0u;
        const uint32_t id1 = v & 0xFFu;   // id + 1 (0: the segment stays)
        l += v >> 8;
        any |= id1;
        bigm |= id1 > 15 ? 1u : 0u;
        code |= (id1 <= 15 ? id1 : 0u) << (4 * k);   // 8 nibbles: the low 32 bits of the code
      }
      templated = any != 0;
      big = bigm != 0;
      p.slow = big;
      p.code = code;
    } else {
      for (uint32_t k = 0; k < nseg; k++) {
        const uint32_t r = cls[off + k];
        const int id = (int)(r & 0xFFu) - 1;
        l += r >> 8;
        if (id >= 0) {
          templated = true;
          if (k < 16 && id < 15) p.code |= (uint64_t)(id + 1) << (k * 4);
          else p.slow = true;
          big |= id >= 15;
        }
      }
    }
    if (templated) { p.mode = M_DEFAULT; p.len = l; }
    else { p.mode = M_ORIG; p.len = 1 + (n - p.lead); }   // "/" + body (processor.go:182-185)
    p.field = n < kNField ? n : kNField;
  }
  if (tm) tt[2] += clk() - c0;
  if (seg_off) *seg_off = off | (nseg << 16);
  if (big_id) *big_id = big;
  return true;
}

// the columns K1 reads per span, and what they decide before the path is read
struct PlanCols {
  uint32_t f;
  ose_strref pr;
  uint32_t kind;
  bool ok;
};
__device__ __forceinline__ PlanCols plan_cols(const UrlKernelArgs& a, uint64_t i) {
  PlanCols c{0, {0, 0}, 0, false};
  if (i < a.n_spans) {
    c.f = a.url_flags[i];
    c.kind = a.kind[i];
    c.pr = a.path[i];
    c.ok = a.res_url_ok == nullptr || a.res_url_ok[a.resource[i]];
  }
  return c;
}
// processor.go:235-259 enhanceSpan gate: 0 skip, 1 rename-to-slash, 2 template the path
__device__ __forceinline__ uint32_t plan_gate(const PlanCols& c) {
  if (!c.ok || !(c.f & OSE_URL_HAS_METHOD) || (c.kind != OSE_KIND_SERVER && c.kind != OSE_KIND_CLIENT)) return 0;
  const uint32_t tgt = c.f & OSE_URL_TGT_MASK;
  if (tgt != OSE_URL_TGT_ABSENT)
    return (tgt == OSE_URL_TGT_STR_EMPTY && (c.f & OSE_URL_NAME_EQ_METHOD)) ? 1u : 0u;   // :241-243
  return (c.f & OSE_URL_PATH_MASK) != OSE_URL_PATH_NONE ? 2u : 0u;
}

// The group's template bytes into img from the classified segment list,
// called by the whole wave.  Entry x of lane L's path writes '/' and then its
// output ({name} from the braced-name table, or the segment's own staged
// bytes) at L's output offset plus the outputs of L's earlier entries; a path
// that neither starts with '/' nor keeps its original form (processor.go:
// 182-185 "/" + body) drops the first separator.  M_SLASH / M_RENAME_SLASH
// spans are a lone '/'.  Every image byte is written exactly once, so the
// image needs no clearing.  Entries are written 64 per step, one per lane:
// the per-byte work follows the longest segment of a step, not the longest
// path of the group.
__device__ __forceinline__ void assemble_group(lds_out_u8* img, const lds_u8* L, uint32_t stage_src, uint32_t* segs,
                                               uint32_t* cls, const BracedNames& bn, uint32_t bn_src,
                                               const Plan& p, uint32_t seg_off, uint32_t local, bool builtin) {
  const int lane = threadIdx.x & 63;
  const uint32_t nseg = seg_off >> 16, off = seg_off & 0xFFFFu;
  const uint32_t pre = (p.lead || p.mode == M_ORIG) ? 1u : 0u;
  uint32_t unused;
  // bytes this lane's entries write, separators included; E0 = those of the lanes before
  const uint32_t E0 = wave_excl_scan(nseg ? p.len + 1 - pre : 0u, &unused);
  const int32_t adj = (int32_t)local - (int32_t)E0 - (int32_t)(1 - pre);
  const uint32_t pk = ((uint32_t)adj & 0xFFFFu) | (off << 16) | (pre << 24);
  if (p.len && (p.mode == M_SLASH || p.mode == M_RENAME_SLASH)) {
    img[local] = '/';
  }
  const uint32_t total = lane_value(off + nseg, kWave - 1);
  uint32_t carry = 0;
  for (uint32_t x0 = 0; x0 < total; x0 += kWave) {
    const uint32_t x = x0 + (uint32_t)lane;
    const bool v = x < total;
    const uint32_t ent = v ? segs[x] : 0u, c = v ? cls[x] : 0u;
    const uint32_t opk = (uint32_t)__shfl((int)pk, (int)(ent >> 25), kWave);
    uint32_t stot;
    const uint32_t E = carry + wave_excl_scan(v ? (c >> 8) + 1 : 0u, &stot);
    carry += stot;
    if (v) {
      const uint32_t pos = (uint32_t)(((int32_t)(opk << 16) >> 16) + (int32_t)E);
      const bool slash = x != ((opk >> 16) & 0xFFu) || (opk >> 24);
      const int id = (int)(c & 0xFFu) - 1;
      // both candidates read unconditionally (a branch on id >= 0 cost the
      // step its exec-mask bookkeeping)
      // builtin (no custom ids): "{id}" "{date}" "{email}" at 1, 6 and 13 of
      // the braced table (load_braced_names), no LDS read
      const uint32_t idc = id >= 0 ? (uint32_t)id : 0u;
      const uint32_t boff = builtin ? (idc == 0 ? 1u : idc == 1 ? 6u : 13u) : (uint32_t)bn.off[idc];
      const uint32_t blen = builtin ? (idc == 0 ? 4u : idc == 1 ? 6u : 7u) : (uint32_t)bn.len[idc];
      const uint32_t so = id >= 0 ? bn_src + boff : stage_src + (ent & 0xFFFu);   // the body's LDS byte offset
      const uint32_t n = id >= 0 ? blen : (ent >> 12) & 0x1FFFu;
      // gfx950 LDS takes misaligned 8-, 4- and 2-byte accesses: one 8-byte
      // read per 8 source bytes (reads past n stay inside the stage / name
      // table) and whole 8-byte stores, then the last 1-7 bytes once after
      // the loop: two overlapping 4- or 2-byte stores (both inside the entry)
      // or one byte.  The hardware replays each misaligned access (PMC
      // SQ_LDS_UNALIGNED_STALL, two thirds of this kernel's LDS cycles on
      // C2), yet an all-aligned form (funnel-shifted dword copies, byte and
      // short stores at the ends) measured 5 % slower on C2 and C4, and
      // reading the first 16 bytes before any store 1-3 % slower: the LDS
      // pipe (21 % busy) is not what bounds this kernel, its instruction
      // latency chains are (profiles/r6e_asm_aligned_ab.txt,
      // r6f_asm_details_ab.txt).
      if (slash) img[pos] = '/';
      lds_out_u8* dp = img + pos + 1;
      const lds_u8* sp = L + so;
      const uint32_t nf = n & ~7u, rem = n & 7u;
#if OSE_ASM_BATCH   // diagnostics A/B: the first 16 bytes read before any store
      const uint64_t u0 = *reinterpret_cast<const lds_u64u*>(sp), u1 = *reinterpret_cast<const lds_u64u*>(sp + 8);
      const uint64_t ut = *reinterpret_cast<const lds_u64u*>(sp + nf);
      if (nf > 0) *reinterpret_cast<lds_w64u*>(dp) = u0;
      if (nf > 8) *reinterpret_cast<lds_w64u*>(dp + 8) = u1;
      for (uint32_t q = 16; q < nf; q += 8)
        *reinterpret_cast<lds_w64u*>(dp + q) = *reinterpret_cast<const lds_u64u*>(sp + q);
      if (rem) {
        const uint64_t v = ut;
#else
      for (uint32_t q = 0; q < nf; q += 8)
        *reinterpret_cast<lds_w64u*>(dp + q) = *reinterpret_cast<const lds_u64u*>(sp + q);
      if (rem) {
        const uint64_t v = *reinterpret_cast<const lds_u64u*>(sp + nf);
#endif
        if (rem >= 4) {
          *reinterpret_cast<lds_w32u*>(dp + nf) = (uint32_t)v;
          *reinterpret_cast<lds_w32u*>(dp + n - 4) = (uint32_t)(v >> (8 * (rem - 4)));
        } else if (rem >= 2) {
          *reinterpret_cast<lds_w16u*>(dp + nf) = (uint16_t)v;
          *reinterpret_cast<lds_w16u*>(dp + n - 2) = (uint16_t)(v >> (8 * (rem - 2)));
        } else {
          dp[nf] = (uint8_t)v;
        }
      }
    }
  }
}

// kMode bit 0 (kModeGeneral): user templatization rules or custom ids are
// configured; without it the instance is compiled with neither (their loops
// fold away, which is what keeps the default-config kernel off scratch).
// bit 1 (kModeDiag, OSE_DIAG builds only): OSE_URL_ABLATE / per-section clocks.
constexpr int kModeGeneral = 1, kModeDiag = 2;
template <int kMode>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void url_plan_kernel(UrlKernelArgs a) {
  __shared__ PlanSmem sm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Cfg cfg = load_cfg(a, sm.ns);
  load_braced_names(cfg, sm.bn);   // workgroup barrier: before any wave may leave
  if (!(kMode & kModeGeneral)) {
    cfg.n_custom = 0;
    cfg.n_rules = 0;
    cfg.max_rule_nseg = 0;
    cfg.names_tab_all = 1;   // the built-in names only
  }
  if (!(kMode & kModeDiag)) {
    cfg.ablate = 0;
    a.ablate = 0;
    a.dbg = nullptr;
  }
  const uint32_t stride = wave_stride();
  uint32_t g = wave_first_group();
  if (g >= a.n_groups) return;
  const bool tm = (kMode & kModeDiag) && a.dbg != nullptr;
  uint64_t t0 = 0, t_stage = 0, t_bm = 0, t_plan = 0, t_emit = 0, tt[3] = {0, 0, 0};
  const bool fused_cfg = sm.bn.ok && !(a.ablate & 2);
  const lds_u8* L = (const lds_u8*)(void*)&sm;
  const uint32_t bn_src = (uint32_t)((uint8_t*)sm.bn.b - (uint8_t*)&sm);
  // this wave's scratch: a region of the workspace, or (refs) chunks of the
  // output arena taken as the wave goes
  uint64_t region = a.refs ? 0 : (uint64_t)wave_first_group() * a.scr_region;
  uint64_t scr_used = 0, scr_end = a.refs ? 0 : a.scr_region;
  bool exhausted = false;   // refs: a chunk went past the arena, the wave takes no more

  // prologue: columns of groups g and g + stride, bytes of group g
  PlanCols cur = plan_cols(a, (uint64_t)g * kWave + lane);
  PlanCols nxt = plan_cols(a, (uint64_t)(g + stride) * kWave + lane);
  PlanCols nn{};
  bool np = plan_gate(cur) == 2;
  StageDma pf = stage_dma(a.arena, np ? cur.pr.off : ~0u, np ? cur.pr.off + cur.pr.len : 0u, sm.stage[wv]);
  bool first = true;
  for (;;) {
    if (tm) t0 = clk();
    wait_dma();   // this group's bytes and the next group's columns have landed
    // the column sets move only here, after the wait: a copy of registers
    // whose loads are in flight would wait for every store issued since
    if (!first) {
      cur = nxt;
      nxt = nn;
    }
    first = false;
    uint8_t* stage = sm.stage[wv];
    lds_u32* stage32 = (lds_u32*)stage;
    const uint64_t i = (uint64_t)g * kWave + lane;
    const uint32_t g2 = g + stride;
    const bool more = g2 < a.n_groups;
    // in flight while this group is planned: the columns of the group after the next
    const bool np2 = more && plan_gate(nxt) == 2;
    nn = plan_cols(a, (uint64_t)(g2 + stride) * kWave + lane);
    if (tm) { const uint64_t t1 = clk(); t_stage += t1 - t0; t0 = t1; }

    const uint32_t gate = plan_gate(cur);
    const bool needs_path = gate == 2;
    const uint32_t lo16 = pf.base;   // per lane (a gathered stage)
    const bool staged = __ballot(lo16 == ~0u) == 0;
    if (staged && pf.bytes && !(a.ablate & 4)) {
      // rows holding path bytes; when other strings of the arena fill a good
      // part of the staged range (C4), only those rows get bitmaps
      uint32_t m0 = 0, m1 = 0, m2 = 0;
      if (needs_path && cur.pr.len) {
        const uint32_t rl = (cur.pr.off - lo16) >> 5, rh = (cur.pr.off - lo16 + cur.pr.len - 1) >> 5;
        m0 = row_bits(rl, rh, 0);
        m1 = row_bits(rl, rh, 32);
        m2 = row_bits(rl, rh, 64);
      }
      m0 = wave_or_u32(m0);
      m1 = wave_or_u32(m1);
      m2 = wave_or_u32(m2);
      build_bitmaps_rows(stage32, (lds_u4*)sm.bm[wv], m0, m1, m2, sm.segs[wv]);
      wave_lds_sync();
    }
    if (tm) { const uint64_t t1 = clk(); t_bm += t1 - t0; t0 = t1; }
    Plan p;
    uint32_t oflags = 0;
    // the list planner uses wave shuffles: called by the whole wave (lanes without a path add no segments)
    bool listed = false, big = false;
    uint32_t seg_off = 0;
    if (staged && !(a.ablate & (1024 | 2)))
      listed = plan_group_list(cfg, stage32, (lds_cu4*)sm.bm[wv], sm.segs[wv], needs_path, cur.pr.off - lo16,
                               cur.pr.len, cur.f, p, tm, tt, sm.cls[wv], &seg_off, &big);
    if (gate == 1) {
      p.mode = M_RENAME_SLASH;
      p.len = 1;
      oflags = OSE_OUT_RENAME;
    } else if (needs_path && (a.ablate & 2)) {
      p.mode = M_ORIG;
      p.len = 1 + cur.pr.len;
      p.field = cur.pr.len;
      oflags = OSE_OUT_SET_ATTR;
    }
    // wave-uniform: a group whose paths the list planner could not take (a
    // byte range over the stage, a list over kSegCap, a segment over 64
    // bytes) is planned from HBM by url_plan_slow_kernel; kept out of this
    // kernel, whose registers the fallback calls would otherwise claim
    const bool unplanned = __ballot(needs_path && !listed && !(a.ablate & 2)) != 0;
    if (needs_path && !(a.ablate & 2)) {
      oflags = OSE_OUT_SET_ATTR;                                                       // processor.go:259
      if ((cur.f & OSE_URL_NAME_EQ_METHOD) && p.len > 0) oflags |= OSE_OUT_RENAME;     // :216-225
    }
    if (unplanned) {
      if (lane == 0) a.unplanned[atomicAdd(a.unplanned_count, 1u)] = g;
    } else {
    // the group's output bytes and each lane's offset in its image: one DPP
    // scan (a 64-bit shuffle reduction would be 12 dependent LDS round trips)
    uint32_t sum32;
    const uint32_t local = wave_excl_scan(p.len, &sum32);
    const uint64_t sum = sum32;
    const uint64_t need = (sum + 15) & ~15ull;
    // wave-uniform: the group is assembled here unless a user rule matched, a
    // name id lies outside the braced table, the list planner gave up, or the
    // image does not fit LDS or the wave's scratch region
    bool fast = fused_cfg && listed && __ballot(p.mode == M_RULE || big) == 0 && sum <= kImgCap;
    if (fast && scr_used + need > scr_end) {
      if (a.refs && !exhausted) {   // a new chunk (the rest of the current one is left unused)
        // one fetch-add per chunk (a compare-and-swap loop that moved the
        // bump only by space that fits measured 12x slower on C4: 4096 waves
        // retrying one address); a chunk that ends past out_cap is used up
        // to out_cap, and the scan counts the bump only up to out_cap
        const uint64_t csz = max(a.refs_chunk, need);
        uint64_t at = 0;
        if (lane == 0) at = atomicAdd((unsigned long long*)a.bump, (unsigned long long)csz);
        at = (uint64_t)lane_value((uint32_t)at, 0) | ((uint64_t)lane_value((uint32_t)(at >> 32), 0) << 32);
        const uint64_t avail = at < a.out_cap ? min(csz, a.out_cap - at) : 0;
        if (avail >= need) {
          region = at;
          scr_used = 0;
          scr_end = avail;
        } else {
          // the arena is full for this group: hand the chunk back when no
          // wave has reserved after it (the bump still ends at this chunk),
          // so the space stays for the groups the scan places; otherwise the
          // scan counts it up to out_cap
          if (lane == 0) atomicCAS((unsigned long long*)a.bump, (unsigned long long)(at + csz), (unsigned long long)at);
          fast = false;
          exhausted = true;
        }
      } else {
        fast = false;
      }
    }
    if (i < a.n_spans) {
      a.plan_len[i] = p.len;
      a.url_out[i] = (uint8_t)oflags;
      if (!fast) {
        a.plan_meta[i] = pack_meta(p.mode, p.lead, p.slow, oflags, p.field);
        a.plan_code[i] = p.code;
      }
    }
    if (tm) { const uint64_t t1 = clk(); t_plan += t1 - t0; t0 = t1; }
    if (fast) {
      lds_u4* img4 = (lds_u4*)sm.bm[wv];
      const uint32_t n16 = (uint32_t)(need / 16);
      if (!(a.ablate & 64))   // diagnostics: OSE_URL_ABLATE 64 skips the image writes (wrong output)
        assemble_group((lds_out_u8*)sm.bm[wv], L, (uint32_t)(stage - (uint8_t*)&sm), sm.segs[wv], sm.cls[wv], sm.bn,
                       bn_src, p, seg_off, local, cfg.n_custom == 0);
      wave_lds_sync();
      uint4* dst = reinterpret_cast<uint4*>(a.scratch + region + scr_used);
      // two 1 KiB rows of the image per round: both reads in flight before
      // the stores (the image is at most kImgCap bytes, < 5 rows)
      // (two rows per round, both reads before the stores, measured 2 %
      // slower on C4: profiles/r6f_asm_details_ab.txt)
      for (uint32_t k = lane; k < n16; k += kWave) {
        const u32x4 v = img4[k];
        dst[k] = make_uint4(v.x, v.y, v.z, v.w);
      }
      if (lane == 0) {
        a.group_sum[g] = sum;
        a.group_scr[g] = region + scr_used;
      }
      // refs form: the image stays where it is, so the group's template refs
      // are known here (url_copy_kernel writes only the other groups')
      if (a.refs && i < a.n_spans) a.tmpl[i] = ose_strref{(uint32_t)(region + scr_used + local), p.len};
      scr_used += need;
    } else if (lane == 0) {
      a.group_sum[g] = sum;
      a.group_scr[g] = ~0ull;
      if (sum) a.slow_groups[atomicAdd(a.slow_count, 1u)] = g;
    }
    }
    if (tm) { const uint64_t t1 = clk(); t_emit += t1 - t0; t0 = t1; }
    if (!more) break;
    wave_lds_sync();   // every lane is done with this group's stage and bitmaps
    pf = stage_dma(a.arena, np2 ? nxt.pr.off : ~0u, np2 ? nxt.pr.off + nxt.pr.len : 0u, sm.stage[wv]);
    g = g2;
  }
  if (tm && lane == 0) {
    atomicAdd((unsigned long long*)&a.dbg[0], (unsigned long long)t_stage);
    atomicAdd((unsigned long long*)&a.dbg[1], (unsigned long long)t_bm);
    atomicAdd((unsigned long long*)&a.dbg[2], (unsigned long long)t_plan);
    atomicAdd((unsigned long long*)&a.dbg[3], 1ull);
    atomicAdd((unsigned long long*)&a.dbg[5], (unsigned long long)t_emit);
    atomicAdd((unsigned long long*)&a.dbg[13], (unsigned long long)tt[0]);
    atomicAdd((unsigned long long*)&a.dbg[14], (unsigned long long)tt[1]);
    atomicAdd((unsigned long long*)&a.dbg[15], (unsigned long long)tt[2]);
  }
}

// ---------------------------------------------------------------------------
// K2: exclusive scan of the group sums: 1024 groups per workgroup, tiles
// chained with the decoupled look-back (device_common.hpp).
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void url_scan_kernel(UrlKernelArgs a) {
  __shared__ uint64_t wsum[kScanThreads / kWave], wsum_a[kScanThreads / kWave];
  __shared__ uint64_t prefix;
  __shared__ uint32_t tile_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) tile_s = atomicAdd(a.scan_counter, 1u);
  __syncthreads();
  const uint32_t tile = tile_s;
  const uint64_t k = (uint64_t)tile * kScanThreads + tid;
  // refs mode: only the slow groups are placed by the scan, after the plan
  // waves' image chunks
  const uint64_t v = k < a.n_groups && !(a.refs && a.group_scr[k] != ~0ull) ? a.group_sum[k] : 0;
  const uint64_t sb = a.refs ? min(*a.bump, a.out_cap) : 0;   // chunks past out_cap are used up to it
  uint64_t incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += t;
  }
  if (lane == kWave - 1) wsum[wv] = incl;
  // refs: the scan-placed groups as images would take them (16-byte aligned)
  const uint64_t va = a.refs ? wave_sum_u64((v + 15) & ~15ull) : 0;
  if (a.refs && lane == 0) wsum_a[wv] = va;
  __syncthreads();
  uint64_t wbase = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / kWave; w++) {
    const uint64_t x = wsum[w];
    if (w < wv) wbase += x;
    total += x;
  }
  if (wv == 0) {
    if (a.refs && lane == 0) {   // before the tile's aggregate is published (lookback_prefix's release)
      uint64_t ta = 0;
      for (int w = 0; w < kScanThreads / kWave; w++) ta += wsum_a[w];
      if (ta) atomicAdd((unsigned long long*)a.slow_aligned, (unsigned long long)ta);
    }
    const uint64_t pfx = lookback_prefix(a.scan_status, tile, total, a.error);
    if (lane == 0) {
      prefix = pfx;
      if (tile == a.n_scan_tiles - 1) {
        const bool over = sb + pfx + total > a.out_cap;
        uint64_t used = sb + pfx + total;
        if (over && a.refs) {
          // what a retry needs: every group as a 16-byte aligned image (X,
          // with the bump's chunk tails of this call counted in), twice over
          // for the tails the retry's waves leave (a wave leaves at most one
          // chunk's tail, and chunks are an eighth of the arena over the
          // waves: the tails stay under C'/8, inside 2X), plus an image per
          // resident wave (not per wave of an oversubscribed grid beside the
          // trace stage, 16x the resident one)
          const uint64_t X = sb + __hip_atomic_load((unsigned long long*)a.slow_aligned, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
          used = 2 * X + (uint64_t)kImgCap * min(a.plan_waves, kUrlMaxWaves);
        }
        if (a.used) *a.used = used;
        if (over) atomicOr(a.error, 2u);
      }
    }
  }
  __syncthreads();
  if (k < a.n_groups) a.group_base[k] = sb + prefix + wbase + incl - v;
}

// ---------------------------------------------------------------------------
// K4: template refs of every span, and the image of every group K1 assembled
// moved from scratch to its place in the output arena.  One wave per group,
// persistent, with the next group's columns in flight while one is copied.
// Lane l of a round reads scratch chunk c = l + 64 r (16 bytes) and writes
// destination dwords 4c..4c+3: dword k covers image bytes [4k - shift, +4),
// a funnel shift of scratch dwords k-1 and k (dword 4c-1 from the lane below,
// or from lane 63 of the previous round).  Dwords the group shares with its
// neighbours are stored bytewise.
struct CopyCols {
  uint32_t len;
  uint64_t base, gsum, so;
};
__device__ __forceinline__ CopyCols copy_cols(const UrlKernelArgs& a, uint32_t g, int lane) {
  CopyCols c{0, 0, 0, ~0ull};
  const uint64_t i = (uint64_t)g * kWave + lane;
  c.base = a.group_base[g];
  c.gsum = a.group_sum[g];
  c.so = a.group_scr[g];
  if (i < a.n_spans) c.len = a.plan_len[i];
  return c;
}
// one destination round (up to 64 chunks of 16 bytes) of a group's image: v
// holds scratch chunk c = c0 + lane
__device__ __forceinline__ void copy_round(uint8_t* gdst, uint32_t shift, uint64_t endb, uint32_t c0, uint32_t nchunk,
                                           const uint4& v, uint32_t& carry) {
  const int lane = threadIdx.x & 63;
  const uint32_t c = c0 + (uint32_t)lane;
  uint32_t pw = (uint32_t)__shfl_up((int)v.w, 1, kWave);
  if (lane == 0) pw = carry;
  carry = lane_value(v.w, kWave - 1);
  const uint32_t sh = 4 - shift;
  const uint32_t w0 = shift ? __builtin_amdgcn_alignbyte(v.x, pw, sh) : v.x;
  const uint32_t w1 = shift ? __builtin_amdgcn_alignbyte(v.y, v.x, sh) : v.y;
  const uint32_t w2 = shift ? __builtin_amdgcn_alignbyte(v.z, v.y, sh) : v.z;
  const uint32_t w3 = shift ? __builtin_amdgcn_alignbyte(v.w, v.z, sh) : v.w;
  if (c < nchunk) {
    const uint64_t b0 = 16ull * c;
    if (b0 >= shift && b0 + 16 <= endb) {
      uint32_t* d = reinterpret_cast<uint32_t*>(gdst + b0);
      d[0] = w0;
      d[1] = w1;
      d[2] = w2;
      d[3] = w3;
    } else {
      const uint32_t ws[4] = {w0, w1, w2, w3};
#pragma unroll
      for (uint32_t q = 0; q < 16; q++)
        if (b0 + q >= shift && b0 + q < endb) gdst[b0 + q] = (uint8_t)(ws[q >> 2] >> (8 * (q & 3)));
    }
  }
}
// A group's copy plan: nothing to copy for K3s's groups, empty ones and an
// overflowing batch (the scan flagged it)
struct CopyJob {
  const uint4* src;
  uint8_t* gdst;
  uint32_t shift, n16, nchunk;
  uint64_t endb;
  bool on;
};
__device__ __forceinline__ CopyJob copy_job(const UrlKernelArgs& a, const CopyCols& c) {
  CopyJob j{};
  j.on = !a.refs && c.so != ~0ull && c.gsum != 0 && c.base + c.gsum <= a.out_cap;
  if (!j.on) return j;
  j.src = reinterpret_cast<const uint4*>(a.scratch + c.so);
  j.shift = (uint32_t)(c.base & 3);
  j.gdst = a.out_arena + (c.base - j.shift);
  j.endb = j.shift + c.gsum;
  j.n16 = (uint32_t)((c.gsum + 15) / 16);
  j.nchunk = (uint32_t)((j.endb + 15) / 16);
  return j;
}
__device__ __forceinline__ uint4 copy_load(const CopyJob& j, uint32_t c0) {
  const uint32_t c = c0 + (threadIdx.x & 63);
  return j.on && c < j.n16 ? j.src[c] : make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void copy_rest(const CopyJob& j, uint4 v, uint32_t& carry) {
  copy_round(j.gdst, j.shift, j.endb, 0, j.nchunk, v, carry);
  for (uint32_t c0 = kWave; c0 < j.nchunk; c0 += kWave) {
    v = copy_load(j, c0);
    copy_round(j.gdst, j.shift, j.endb, c0, j.nchunk, v, carry);
  }
}
// One group per iteration at eight waves per SIMD (62 VGPRs): on one box it
// beat the two-groups-per-iteration form below (83 VGPRs, five waves) by 3-5%
// on C4 / C5 / C2 (profiles/r2d_url_copy_ab.txt) -- more resident waves hide
// the two memory round trips per group better than the explicit pairing.
// kSize: odigostrafficmetrics' spans pass (size_device.hpp) fused in, with
// the plan lengths as the template lengths: the span columns it reads are
// loaded with the group's copy columns, so the pass adds no round trip and no
// second walk over the spans (size_span_kernel is then not launched); the
// surviving spans are counted per block into size_partials.
template <bool kSize>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kSize ? 5 : 6, 8))) void url_copy_kernel(UrlKernelArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t stride = wave_stride();
  if (!kSize && a.refs) {
    // refs form without the size pass: url_plan_kernel wrote the refs of the
    // groups it assembled; a wave looks at 64 groups' image offsets at once
    // and writes the refs of the others (their bytes are placed at the
    // scanned group base by url_emit_slow_kernel)
    for (uint64_t g0 = (uint64_t)wave_first_group() * kWave; g0 < a.n_groups; g0 += (uint64_t)stride * kWave) {
      const uint64_t gg = g0 + lane;
      const bool other = gg < a.n_groups && a.group_scr[gg] == ~0ull;
      for (uint64_t m = __ballot(other); m; m &= m - 1) {
        const uint32_t g = (uint32_t)(g0 + __builtin_ctzll(m));
        const CopyCols A = copy_cols(a, g, lane);
        uint32_t unused;
        const uint32_t la = wave_excl_scan(A.len, &unused);
        const uint64_t ia = (uint64_t)g * kWave + lane;
        if (ia < a.n_spans) a.tmpl[ia] = ose_strref{(uint32_t)(A.base + la), A.len};
      }
    }
    return;
  }
  uint32_t kept = 0;
  const bool sz_on = kSize && !sizedev::size_batch_dropped(a.sz);
  uint32_t g = wave_first_group();
  // the next group's columns are loaded while this group is worked on
  CopyCols An{0, 0, 0, ~0ull};
  sizedev::SpanCols xn{};
  if (g < a.n_groups) {
    An = copy_cols(a, g, lane);
    if (kSize && sz_on) xn = sizedev::size_span_load(a.sz, (uint64_t)g * kWave + lane, false);
  }
  for (; g < a.n_groups; g += stride) {
    const uint64_t ia = (uint64_t)g * kWave + lane;
    const CopyCols A = An;
    const sizedev::SpanCols x0 = xn;
    const bool more = g + stride < a.n_groups;
    if (more) {
      An = copy_cols(a, g + stride, lane);
      if (kSize && sz_on) xn = sizedev::size_span_load(a.sz, (uint64_t)(g + stride) * kWave + lane, false);
    }
    sizedev::SpanCols x = x0;
    uint32_t unused;
    const uint32_t la = wave_excl_scan(A.len, &unused);
    const CopyJob ja = copy_job(a, A);
    const uint4 va = copy_load(ja, 0);
    if (ia < a.n_spans && !(a.refs && A.so != ~0ull)) {
      // refs mode: a fast group's template stays in its scratch image (its
      // refs were written by url_plan_kernel)
      const uint64_t at = a.refs && A.so != ~0ull ? A.so : A.base;
      a.tmpl[ia] = ose_strref{(uint32_t)(at + la), A.len};
    }
    if (kSize && sz_on) {
      x.tl = A.len;
      kept += sizedev::size_span_finish(a.sz, x);
    }
    uint32_t carry = 0;
    if (ja.on) copy_rest(ja, va, carry);
    if (!more) break;
  }
  if (kSize) {
    __shared__ uint32_t wk[kWaves];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o, kWave);
    if (lane == 0) wk[threadIdx.x >> 6] = kept;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kWaves; w++) t += wk[w];
      a.size_partials[blockIdx.x] = t;
    }
  }
}
// K1b: the groups K1 listed as unplanned, one single-wave workgroup per
// group (persistent; exits at once when the list is empty).  Their paths are
// planned in lane subsets whose 16-byte chunks fit K1's 3 KB stage: each
// subset is gathered (stage_dma), given its row bitmaps and planned by the
// same wave-parallel list planner as K1.  A subset the list planner refuses
// (a segment over 64 bytes, more than kSegCap segments) and a single path
// over 3 KB are planned per lane (plan_path from the stage, plan_global from
// HBM): per-lane byte walks diverge across the wave, which made a lone group
// cost ~190k clocks when every lane took that route.  The plan arrays,
// url_out and the group's output sum are written; the group is listed for
// K3s, which emits it.
struct SlowPlanSmem {
  NamesSmem ns;
  __attribute__((aligned(16))) uint8_t stage[kPlanStage + 16];
  __attribute__((aligned(16))) u32x4 bm[kRowVec * kPlanBmRows];
  uint32_t segs[kSegCap];
  uint32_t cls[kSegCap + 8];   // (8 entries of padding: the fold reads 8)
};
__global__ __launch_bounds__(kWave) void url_plan_slow_kernel(UrlKernelArgs a) {
  __shared__ SlowPlanSmem sm;
  const uint32_t count = *a.unplanned_count;
  if (blockIdx.x >= count) return;
  const int lane = threadIdx.x;
  const uint64_t c0 = a.dbg ? clk() : 0;
  const Cfg cfg = load_cfg(a, sm.ns);
  uint64_t c_plan = 0;
  const uint64_t c1 = a.dbg ? clk() : 0;
  lds_u32* stage32 = (lds_u32*)sm.stage;
  uint64_t tt[3] = {0, 0, 0};
  for (uint32_t k = blockIdx.x; k < count; k += gridDim.x) {
    const uint32_t g = a.unplanned[k];
    const uint64_t i = (uint64_t)g * kWave + lane;
    const PlanCols c = plan_cols(a, i);
    const uint32_t gate = plan_gate(c);
    Plan p;
    uint32_t oflags = 0;
    if (gate == 1) {
      p.mode = M_RENAME_SLASH;
      p.len = 1;
      oflags = OSE_OUT_RENAME;
    }
    const uint32_t lo_l = c.pr.off, hi_l = c.pr.off + c.pr.len;
    const uint32_t nc = gate == 2 && c.pr.len ? ((hi_l + 15u) >> 4) - (lo_l >> 4) : 0u;
    bool todo = gate == 2;
    while (__ballot(todo)) {   // wave-uniform
      const uint64_t t = a.dbg ? clk() : 0;
      uint32_t unused;
      const uint32_t cs = wave_excl_scan(todo ? nc : 0u, &unused);
      bool take = todo && cs + nc <= kPlanStage / 16;
      const bool alone = __ballot(take) == 0;   // the first pending path alone is over 3 KB
      if (alone) {
        const int first = __builtin_ctzll(__ballot(todo));
        if (lane == first) {
          p = plan_global(cfg, a.arena + c.pr.off, c.pr.len, c.f);
          todo = false;
        }
        continue;
      }
      const StageDma sd = stage_dma(a.arena, take ? lo_l : ~0u, take ? hi_l : 0u, sm.stage);
      wait_dma();
      const uint32_t p0 = c.pr.off - sd.base;
      uint32_t m0 = 0, m1 = 0, m2 = 0;
      if (take && c.pr.len) {
        const uint32_t rl = p0 >> 5, rh = (p0 + c.pr.len - 1) >> 5;
        m0 = row_bits(rl, rh, 0);
        m1 = row_bits(rl, rh, 32);
        m2 = row_bits(rl, rh, 64);
      }
      build_bitmaps_rows(stage32, (lds_u4*)sm.bm, wave_or_u32(m0), wave_or_u32(m1), wave_or_u32(m2), sm.segs);
      wave_lds_sync();
      Plan q;
      const bool listed = plan_group_list(cfg, stage32, (lds_cu4*)sm.bm, sm.segs, take, p0, c.pr.len, c.f, q, false,
                                          tt, sm.cls);
      if (take) {
        if (listed) {
          p = q;
        } else {
          LdsReader rd(stage32, p0);
          p = plan_path(cfg, rd, c.pr.len, c.f);
        }
        todo = false;
      }
      wave_lds_sync();   // the stage and bitmaps are refilled for the next subset
      if (a.dbg) c_plan += clk() - t;
    }
    if (gate == 2) {
      oflags = OSE_OUT_SET_ATTR;                                                       // processor.go:259
      if ((c.f & OSE_URL_NAME_EQ_METHOD) && p.len > 0) oflags |= OSE_OUT_RENAME;       // :216-225
    }
    if (i < a.n_spans) {
      a.plan_len[i] = p.len;
      a.url_out[i] = (uint8_t)oflags;
      a.plan_meta[i] = pack_meta(p.mode, p.lead, p.slow, oflags, p.field);
      a.plan_code[i] = p.code;
    }
    const uint64_t sum = wave_sum_u64(p.len);
    if (lane == 0) {
      a.group_sum[g] = sum;
      a.group_scr[g] = ~0ull;
      if (sum) a.slow_groups[atomicAdd(a.slow_count, 1u)] = g;
    }
  }
  if (a.dbg) {   // diagnostics: the slowest block's clocks (config load, whole, subset planning)
    const uint64_t c2 = clk();
    if (lane == 0) {
      atomicMax((unsigned long long*)&a.dbg[8], (unsigned long long)(c1 - c0));
      atomicMax((unsigned long long*)&a.dbg[9], (unsigned long long)(c2 - c0));
      atomicMax((unsigned long long*)&a.dbg[10], (unsigned long long)c_plan);
    }
  }
}

// K3s: the groups K1 listed (user rules, plan `slow`, names outside the
// braced table, an output image or a stage larger than LDS), with the
// per-span writer (emit_path).  One wave per listed group; exits at once when
// the list is empty.
struct EmitSlowSmem {
  NamesSmem ns;
  __attribute__((aligned(16))) uint8_t stage[kWaves][kStage + 16];
  __attribute__((aligned(16))) uint32_t img[kWaves][kWaveOut / 4 + 4];
};
__global__ __launch_bounds__(kThreads) void url_emit_slow_kernel(UrlKernelArgs a) {
  __shared__ EmitSlowSmem sm;
  const uint32_t count = *a.slow_count;
  if (blockIdx.x * kWaves >= count) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const Cfg cfg = load_cfg(a, sm.ns);
  uint8_t* stage = sm.stage[wv];
  lds_u32* stage32 = (lds_u32*)stage;
  lds_w32* img = (lds_w32*)sm.img[wv];
  for (uint32_t k = wave_first_group(); k < count; k += wave_stride()) {
    const uint32_t g = a.slow_groups[k];
    const uint64_t i = (uint64_t)g * kWave + lane;
    const EmitCols c = emit_cols(a, g, lane);
    const uint64_t base = c.base, gtotal = c.gsum;
    if (base + gtotal > a.out_cap) continue;   // overflow: the scan flagged it
    const uint32_t len = c.len, meta = c.meta, mode = meta & 7u;
    uint32_t unused;
    const uint32_t local = wave_excl_scan(len, &unused);
    const bool needs_path = emit_needs_path(meta);
    const ose_strref pr = needs_path ? c.pr : ose_strref{0, 0};
    uint32_t nbytes;
    const uint32_t lo16 = stage_wave(stage, a.arena, needs_path ? pr.off : ~0u, needs_path ? pr.off + pr.len : 0u,
                                     &nbytes);
    const uint32_t shift = (uint32_t)(base & 3);
    const uint32_t img_bytes = shift + (uint32_t)gtotal;
    const bool direct = img_bytes > kWaveOut || lo16 == ~0u;   // wave-uniform
    if (!direct) {
      for (uint32_t k2 = lane; k2 < (img_bytes + 3) / 4; k2 += kWave) img[k2] = 0;
      wave_lds_sync();
    }
    if (len) {
      const uint32_t lead = (meta >> 3) & 1u, field = meta >> 7;
      const bool slow = (meta >> 4) & 1u;
      const uint32_t f = (needs_path && (mode == M_RULE || field == kNField)) ? a.url_flags[i] : 0u;
      if (!direct) {
        PutOr put(img, shift + local);
        LdsReader rd(stage32, pr.off - lo16);
        emit_path(cfg, rd, pr.len, f, mode, lead, slow, field, c.code, put);
        put.finish();
      } else if (lo16 != ~0u) {
        emit_out_of_line(cfg, LdsReader(stage32, pr.off - lo16), pr.len, f, mode, lead, slow, field, c.code,
                         a.out_arena + base + local, len);
      } else {
        emit_out_of_line(cfg, ByteReader(a.arena + pr.off), pr.len, f, mode, lead, slow, field, c.code,
                         a.out_arena + base + local, len);
      }
    }
    wave_lds_sync();
    if (!direct) store_image(a, img, base, shift, gtotal);
    wave_lds_sync();   // image and stage are reused by the next group
  }
}

// Persistent grid: as many workgroups as fit on the device at once (capped
// by the number of groups).
template <class K>
static uint32_t resident_blocks(K kernel, size_t dyn_lds) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, dyn_lds) != hipSuccess || per_cu <= 0)
    per_cu = 2;
  return (uint32_t)(cus * per_cu);
}

}  // namespace

static int url_mode(const UrlKernelArgs& a) {
  return (a.general ? kModeGeneral : 0) | ((OSE_DIAG && (a.ablate || a.dbg)) ? kModeDiag : 0);
}
template <int M>
static uint32_t plan_blocks(const UrlKernelArgs& a) {
  static const uint32_t res = resident_blocks(url_plan_kernel<M>, 0);
  // beside the trace stage (refs form: no per-wave scratch regions) the grid
  // is several times the resident one, so the dispatcher interleaves its
  // workgroups with the trace stage's instead of the plan grid holding every
  // CU's LDS until it drains (run_stages)
  const uint32_t cap = a.refs && a.plan_grid_mult > 1 ? res * a.plan_grid_mult : std::min<uint32_t>(res, kUrlMaxWaves / kWaves);
  return std::min<uint32_t>(cap, (a.n_groups + kWaves - 1) / kWaves);
}
template <int M>
static void launch_plan_mode(const UrlKernelArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(url_plan_kernel<M>, dim3(plan_blocks<M>(a)), dim3(kThreads), 0, st, a);
}
// An eighth of the arena over the plan waves, at most 256 KiB (a group
// larger than a chunk takes exactly its size): a wave leaves at most one
// chunk's tail unused at the end
uint64_t url_refs_chunk(uint64_t cap, uint32_t waves) {
  return std::min<uint64_t>(256 << 10, cap / 8 / std::max<uint32_t>(1, waves)) & ~15ull;
}
uint32_t url_plan_waves(const UrlKernelArgs& a) {
  switch (url_mode(a)) {
    case 0: return plan_blocks<0>(a) * kWaves;
#if OSE_DIAG
    case 2: return plan_blocks<2>(a) * kWaves;
    case 3: return plan_blocks<3>(a) * kWaves;
#endif
    default: return plan_blocks<1>(a) * kWaves;
  }
}
void launch_url_plan(const UrlKernelArgs& a, hipStream_t st) {
  switch (url_mode(a)) {
    case 0: launch_plan_mode<0>(a, st); break;
#if OSE_DIAG
    case 2: launch_plan_mode<2>(a, st); break;
    case 3: launch_plan_mode<3>(a, st); break;
#endif
    default: launch_plan_mode<1>(a, st); break;
  }
}
void launch_url_scan(const UrlKernelArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(url_scan_kernel, dim3(a.n_scan_tiles), dim3(kScanThreads), 0, st, a);
}
uint32_t url_copy_blocks(uint32_t n_groups) {
  // far more workgroups than fit at once (C4 sweep, profiles/r2d_url_copy_grid_sweep.txt:
  // resident grid 1.01 ms, 16384 blocks 0.93, 65536 0.92): a wave's two
  // groups are two memory round trips, and the waves waiting on them are what
  // keeps HBM busy
  return std::max<uint32_t>(1, std::min<uint32_t>(kUrlCopyMaxBlocks, (n_groups + 2 * kWaves - 1) / (2 * kWaves)));
}
void launch_url_copy(const UrlKernelArgs& a, hipStream_t st) {
  const uint32_t blocks = url_copy_blocks(a.n_groups);
  if (a.fuse_size)
    hipLaunchKernelGGL(url_copy_kernel<true>, dim3(blocks), dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL(url_copy_kernel<false>, dim3(blocks), dim3(kThreads), 0, st, a);
}
void launch_url_plan_slow(const UrlKernelArgs& a, hipStream_t st) {
  // the list length is on the device: a workgroup per group up to the resident
  // count, workgroups past the list's end exit at once
  static const uint32_t cap = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024u;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, url_plan_slow_kernel, kWave, 0) != hipSuccess || per_cu <= 0)
      per_cu = 2;
    return (uint32_t)(cus * per_cu);
  }();
  const uint32_t blocks = std::min<uint32_t>(cap, a.n_groups);
  if (blocks) hipLaunchKernelGGL(url_plan_slow_kernel, dim3(blocks), dim3(kWave), 0, st, a);
}
void launch_url_emit_slow(const UrlKernelArgs& a, hipStream_t st) {
  // the list length is on the device: a grid for every group, blocks past it exit at once
  static const uint32_t cap = resident_blocks(url_emit_slow_kernel, 0);
  const uint32_t blocks = std::min<uint32_t>(cap, (a.n_groups + kWaves - 1) / kWaves);
  hipLaunchKernelGGL(url_emit_slow_kernel, dim3(blocks), dim3(kThreads), 0, st, a);
}

}  // namespace ose
