// url_kernel.hip — odigosurltemplate on CDNA4 (gfx950).
//
// One launch templatizes a whole batch in a single pass over HBM:
//   phase 1  one thread per span decides what the reference would do
//            (processor.go:235-287 enhanceSpan/processSpan), splits the path,
//            tries the templatization rules with the same segment count in
//            config order (processor.go:149-171, templatize.go:192-237) and
//            otherwise classifies every segment (templatize.go:242-269) with
//            a streaming byte automaton that evaluates all built-in regexps
//            (noLetters, \d{7,}, UUID, hex, date, email, U+FFFD) in one read,
//            plus compiled DFAs for custom_ids / rule regexps.  It records
//            the output length and per-segment decisions in registers.
//   scan     block scan of output lengths + decoupled look-back across tiles
//            gives every span its offset in the compact output arena.
//   phase 2  each thread writes its template into an LDS image of the tile's
//            output while wave 0 resolves the look-back; the tile image is
//            then stored to HBM with coalesced stores.
// Output is byte-identical to the oracle (oracle/url.c): same template bytes,
// same compact arena layout (span order).
#include <hip/hip_runtime.h>

#include "../../include/odigos_amd.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace ose {
namespace {

constexpr int kTile = 256;
constexpr uint32_t kOutLds = 24 * 1024;   // LDS image of one tile's output

enum : uint32_t { M_NONE = 0, M_RENAME_SLASH, M_SLASH, M_RULE, M_DEFAULT, M_ORIG };

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }
__device__ __forceinline__ bool is_alpha(uint32_t c) { return (c | 0x20u) - 'a' < 26u; }
__device__ __forceinline__ bool is_hex(uint32_t c) { return is_digit(c) || (c | 0x20u) - 'a' < 6u; }

// noLettersRegex class (templatize.go:14) as a 128-bit set
__device__ __forceinline__ bool is_noletter(uint32_t c) {
  // digits and _-!@#$%^&*()=+{}[]:;"'<>,.?/\|`~
  constexpr uint64_t lo = (1ull << '!') | (1ull << '"') | (1ull << '#') | (1ull << '$') | (1ull << '%') |
                          (1ull << '&') | (1ull << '\'') | (1ull << '(') | (1ull << ')') | (1ull << '*') |
                          (1ull << '+') | (1ull << ',') | (1ull << '-') | (1ull << '.') | (1ull << '/') |
                          (0x3FFull << '0') | (1ull << ':') | (1ull << ';') | (1ull << '<') | (1ull << '=') |
                          (1ull << '>') | (1ull << '?');
  constexpr uint64_t hi = (1ull << ('@' - 64)) | (1ull << ('[' - 64)) | (1ull << ('\\' - 64)) |
                          (1ull << (']' - 64)) | (1ull << ('^' - 64)) | (1ull << ('_' - 64)) |
                          (1ull << ('`' - 64)) | (1ull << ('{' - 64)) | (1ull << ('|' - 64)) |
                          (1ull << ('}' - 64)) | (1ull << ('~' - 64));
  return c < 64 ? ((lo >> c) & 1) : (c < 128 ? ((hi >> (c - 64)) & 1) : false);
}
__device__ __forceinline__ bool is_email_local(uint32_t c) {
  return is_alpha(c) || is_digit(c) || c == '.' || c == '_' || c == '%' || c == '+' || c == '-';
}
__device__ __forceinline__ bool is_email_domain(uint32_t c) {
  return is_alpha(c) || is_digit(c) || c == '.' || c == '-';
}

// datesRegex (templatize.go:67) as a position automaton; 255 = dead.
// accepting: 10 (date), 16 (THH:MM), 19 (THH:MM:SS), 30 (Z), 35 (+hhmm)
__device__ __forceinline__ uint32_t date_step(uint32_t s, uint32_t c) {
  if (s < 10) {
    bool ok = (s == 4 || s == 7) ? c == '-' : is_digit(c);
    return ok ? s + 1 : 255;
  }
  switch (s) {
    case 10: case 16: case 19:
      if (c == 'T' && s == 10) return 11;
      if (c == ':' && s == 16) return 17;
      if (c == 'Z') return 30;
      if (c == '+' || c == '-') return 31;
      return 255;
    case 11: case 12: case 14: case 15: case 17: case 18:
      return is_digit(c) ? s + 1 : 255;
    case 13:
      return c == ':' ? 14 : 255;
    case 31: case 32: case 33: case 34:
      return is_digit(c) ? s + 1 : 255;
    default:
      return 255;
  }
}
__device__ __forceinline__ bool date_accept(uint32_t s) {
  return s == 10 || s == 16 || s == 19 || s == 30 || s == 35;
}
__device__ __forceinline__ bool uuid_char_ok(uint32_t k, uint32_t c) {
  return (k == 8 || k == 13 || k == 18 || k == 23) ? c == '-' : is_hex(c);
}

struct Cfg {
  const uint8_t* blob;
  const UrlCfgDev* h;
  __device__ const NameDev& name(uint32_t id) const {
    return reinterpret_cast<const NameDev*>(blob + h->names_off)[id];
  }
  __device__ uint32_t dfa_off(int32_t i) const {
    return reinterpret_cast<const uint32_t*>(blob + h->dfa_off)[i];
  }
};

// getSegmentTemplatizationString (templatize.go:242-269) on bytes [s, e):
// returns the name id, or -1 when the segment stays as is.
__device__ int classify_segment(const Cfg& cfg, ByteReader& rd, uint32_t s, uint32_t e) {
  const uint32_t n = e - s;
  // custom ids first, in config order
  for (uint32_t k = 0; k < cfg.h->n_custom; k++) {
    const UrlCustomDev& cu = reinterpret_cast<const UrlCustomDev*>(cfg.blob + cfg.h->custom_off)[k];
    if (dfa_match(cfg.blob, cfg.dfa_off(cu.dfa), rd, s, e)) return (int)cu.name;
  }
  bool all_nl = n > 0, all_hex = true, longnum = false, fffd = false, uuid_pre = n >= 36;
  uint32_t run = 0;
  uint32_t utf_need = 0, utf_lo = 0x80, utf_hi = 0xBF, utf_seq = 0;   // utf_seq: EF BF BD tracker
  uint32_t em = 0, local_len = 0, dom_len = 0, tail_n = 0;            // em: 0 local, 1 domain, 2 dead
  int32_t lastdot = -1;
  bool tail_ok = true;
  uint32_t ds = 0;
  for (uint32_t k = 0; k < n; k++) {
    uint32_t c = rd.at(s + k);
    all_nl &= is_noletter(c);
    all_hex &= is_hex(c);
    run = is_digit(c) ? run + 1 : 0;
    longnum |= run >= 7;
    if (k < 36) uuid_pre &= uuid_char_ok(k, c);
    ds = date_step(ds, c);
    // utf8 walk (replacementChar, templatize.go:73): sticky once found
    if (!fffd) {
      if (utf_need == 0) {
        if (c >= 0x80) {
          utf_lo = 0x80; utf_hi = 0xBF; utf_seq = c == 0xEF ? 1 : 0;
          if (c >= 0xC2 && c <= 0xDF) utf_need = 1;
          else if (c == 0xE0) { utf_need = 2; utf_lo = 0xA0; }
          else if (c >= 0xE1 && c <= 0xEC) utf_need = 2;
          else if (c == 0xED) { utf_need = 2; utf_hi = 0x9F; }
          else if (c >= 0xEE && c <= 0xEF) utf_need = 2;
          else if (c == 0xF0) { utf_need = 3; utf_lo = 0x90; }
          else if (c >= 0xF1 && c <= 0xF3) utf_need = 3;
          else if (c == 0xF4) { utf_need = 3; utf_hi = 0x8F; }
          else fffd = true;
        }
      } else {
        if (c < utf_lo || c > utf_hi) {
          fffd = true;
        } else {
          utf_seq = (utf_seq == 1 && c == 0xBF) ? 2 : (utf_seq == 2 && c == 0xBD ? 3 : 0);
          if (utf_seq == 3) fffd = true;
          utf_lo = 0x80; utf_hi = 0xBF;
          utf_need--;
        }
      }
    }
    // email (templatize.go:70)
    if (em == 0) {
      if (c == '@') em = local_len > 0 ? 1 : 2;
      else if (is_email_local(c)) local_len++;
      else em = 2;
    } else if (em == 1) {
      if (!is_email_domain(c)) em = 2;
      else {
        if (c == '.') { lastdot = (int32_t)dom_len; tail_n = 0; tail_ok = true; }
        else if (is_alpha(c)) tail_n++;
        else tail_ok = false;
        dom_len++;
      }
    }
  }
  if (utf_need) fffd = true;   // truncated sequence at the end
  if (date_accept(ds)) return kNameDate;
  if (em == 1 && lastdot >= 1 && tail_ok && tail_n >= 2) return kNameEmail;
  bool uuid = uuid_pre;
  if (!uuid && n >= 36) {
    uuid = true;
    for (uint32_t k = 0; k < 36; k++) uuid &= uuid_char_ok(k, rd.at(e - 36 + k));
  }
  bool hex = all_hex && n >= 16 && (n & 1) == 0;
  if (all_nl || longnum || uuid || hex || fffd) return kNameId;
  return -1;
}

// attemptTemplateWithRule (templatize.go:192-237): returns the output body
// length (without the leading '/') or -1.
__device__ int64_t attempt_rule(const Cfg& cfg, const UrlRuleDev& r, ByteReader& rd, uint32_t b0, uint32_t n) {
  const UrlRuleSegDev* segs = reinterpret_cast<const UrlRuleSegDev*>(cfg.blob + cfg.h->segs_off) + r.seg_first;
  const uint8_t* bytes = cfg.blob + cfg.h->bytes_off;
  uint32_t s = b0;
  int64_t len = 0;
  for (uint32_t k = 0; k < r.nseg; k++) {
    uint32_t e = s;
    while (e < n && rd.at(e) != '/') e++;
    const UrlRuleSegDev& sg = segs[k];
    uint32_t sl = e - s;
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

template <typename Put>
__device__ void emit_rule(const Cfg& cfg, const UrlRuleDev& r, ByteReader& rd, uint32_t b0, uint32_t n, Put& put) {
  const UrlRuleSegDev* segs = reinterpret_cast<const UrlRuleSegDev*>(cfg.blob + cfg.h->segs_off) + r.seg_first;
  const uint8_t* bytes = cfg.blob + cfg.h->bytes_off;
  uint32_t s = b0;
  for (uint32_t k = 0; k < r.nseg; k++) {
    uint32_t e = s;
    while (e < n && rd.at(e) != '/') e++;
    const UrlRuleSegDev& sg = segs[k];
    if (k) put('/');
    if (sg.kind == kRuleTemplate) {
      put('{');
      for (uint32_t q = 0; q < sg.text_len; q++) put(bytes[sg.text_off + q]);
      put('}');
    } else if (sg.kind == kRuleWildcard || sg.kind == kRuleRegex) {
      for (uint32_t q = s; q < e; q++) put(rd.at(q));
    } else {
      for (uint32_t q = 0; q < sg.text_len; q++) put(bytes[sg.text_off + q]);
    }
    s = e + 1;
  }
}

struct SpanPlan {
  uint32_t mode = M_NONE;
  uint32_t len = 0;        // output bytes
  uint32_t b0 = 0, n = 0;  // body start, path end (after '?' cut)
  uint32_t lead = 0;
  int32_t rule = -1;
  uint64_t code_lo = 0, code_hi = 0;   // 4-bit (name id + 1) per segment, first 32 segments
  bool slow = false;                   // more segments / names than the codes hold
};

__global__ __launch_bounds__(256) void url_template_kernel(UrlKernelArgs a) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_wsum[kTile / kWave];
  __shared__ uint32_t s_direct;
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kOutLds];

  const int tid = threadIdx.x;
  if (tid == 0) s_tile = atomicAdd(a.tile_counter, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t i = (uint64_t)tile * kTile + tid;
  const bool valid = i < a.n_spans;

  Cfg cfg{a.cfg, reinterpret_cast<const UrlCfgDev*>(a.cfg)};
  SpanPlan pl;
  uint8_t oflags = 0;
  ose_strref path{0, 0};
  if (valid) {
    uint32_t f = a.url_flags[i];
    uint32_t kind = a.kind[i];
    bool ok = a.res_url_ok == nullptr || a.res_url_ok[a.resource[i]];
    if (ok && (f & OSE_URL_HAS_METHOD) && (kind == OSE_KIND_SERVER || kind == OSE_KIND_CLIENT)) {
      uint32_t tgt = f & OSE_URL_TGT_MASK;
      uint32_t src = f & OSE_URL_PATH_MASK;
      if (tgt != OSE_URL_TGT_ABSENT) {
        if (tgt == OSE_URL_TGT_STR_EMPTY && (f & OSE_URL_NAME_EQ_METHOD)) {
          pl.mode = M_RENAME_SLASH;
          pl.len = 1;
          oflags = OSE_OUT_RENAME;
        }
      } else if (src != OSE_URL_PATH_NONE) {
        path = a.path[i];
        oflags = OSE_OUT_SET_ATTR;
      }
    }
  }
  ByteReader rd(a.arena + path.off);
  if (oflags == OSE_OUT_SET_ATTR) {
    uint32_t f = a.url_flags[i];
    uint32_t n = path.len;
    if ((f & OSE_URL_PATH_MASK) == OSE_URL_PATH_TARGET) {
      for (uint32_t k = 0; k < n; k++)
        if (rd.at(k) == '?') { n = k; break; }
    }
    pl.n = n;
    pl.lead = (n > 0 && rd.at(0) == '/') ? 1 : 0;
    pl.b0 = pl.lead;
    if (n == pl.b0) {
      pl.mode = M_SLASH;
      pl.len = 1;
    } else {
      if (cfg.h->n_rules) {
        uint32_t nseg = 1;
        for (uint32_t k = pl.b0; k < n; k++) nseg += rd.at(k) == '/';
        if (nseg <= cfg.h->max_rule_nseg) {
          const uint32_t* by_len = reinterpret_cast<const uint32_t*>(cfg.blob + cfg.h->rules_by_len_off);
          const UrlRuleDev* rules = reinterpret_cast<const UrlRuleDev*>(cfg.blob + cfg.h->rules_off);
          for (uint32_t r = by_len[nseg]; r < by_len[nseg + 1]; r++) {
            int64_t l = attempt_rule(cfg, rules[r], rd, pl.b0, n);
            if (l >= 0) {
              pl.mode = M_RULE;
              pl.rule = (int32_t)r;
              pl.len = pl.lead + (uint32_t)l;
              break;
            }
          }
        }
      }
      if (pl.mode == M_NONE) {
        uint32_t s = pl.b0, seg = 0, len = pl.lead;
        bool templated = false;
        for (;;) {
          uint32_t e = s;
          while (e < n && rd.at(e) != '/') e++;
          int id = classify_segment(cfg, rd, s, e);
          if (seg) len += 1;
          if (id >= 0) {
            templated = true;
            len += cfg.name((uint32_t)id).len + 2;
            if (seg < 32 && id < 15) {
              uint64_t code = (uint64_t)(id + 1) << ((seg & 15) * 4);
              if (seg < 16) pl.code_lo |= code; else pl.code_hi |= code;
            } else {
              pl.slow = true;
            }
          } else {
            len += e - s;
          }
          seg++;
          if (e >= n) break;
          s = e + 1;
        }
        if (templated) {
          pl.mode = M_DEFAULT;
          pl.len = len;
        } else {
          pl.mode = M_ORIG;        // "/" + body (processor.go:182-185)
          pl.len = 1 + (n - pl.b0);
        }
      }
    }
    if ((f & OSE_URL_NAME_EQ_METHOD) && pl.len > 0) oflags |= OSE_OUT_RENAME;
  }

  // ---- block exclusive scan of output lengths ----
  const int lane = tid & 63, wv = tid >> 6;
  uint32_t incl = pl.len;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    uint32_t t = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += t;
  }
  if (lane == kWave - 1) s_wsum[wv] = incl;
  __syncthreads();
  uint32_t wbase = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kTile / kWave; w++) {
    uint32_t v = s_wsum[w];
    if (w < wv) wbase += v;
    total += v;
  }
  const uint32_t local = wbase + incl - pl.len;
  const bool direct = total > kOutLds;

  // wave 0 resolves the tile prefix while all waves stage the output in LDS
  if (wv == 0) {
    uint64_t p = lookback_prefix(a.tile_status, tile, total, a.error);
    if (lane == 0) {
      s_prefix = p;
      s_direct = direct;
      if (p + total > a.out_cap) atomicOr(a.error, 2u);
      if (tile == a.n_tiles - 1 && a.used) *a.used = p + total;
    }
  }

  auto emit = [&](uint8_t* dst) {
    uint32_t w = 0;
    auto put = [&](uint32_t c) { dst[w++] = (uint8_t)c; };
    if (pl.mode == M_RENAME_SLASH || pl.mode == M_SLASH) {
      put('/');
    } else if (pl.mode == M_ORIG) {
      put('/');
      for (uint32_t k = pl.b0; k < pl.n; k++) put(rd.at(k));
    } else if (pl.mode == M_RULE) {
      if (pl.lead) put('/');
      const UrlRuleDev* rules = reinterpret_cast<const UrlRuleDev*>(cfg.blob + cfg.h->rules_off);
      emit_rule(cfg, rules[pl.rule], rd, pl.b0, pl.n, put);
    } else if (pl.mode == M_DEFAULT) {
      if (pl.lead) put('/');
      const uint8_t* bytes = cfg.blob + cfg.h->bytes_off;
      uint32_t s = pl.b0, seg = 0;
      for (;;) {
        uint32_t e = s;
        while (e < pl.n && rd.at(e) != '/') e++;
        int id;
        if (seg < 32 && !pl.slow) {
          uint64_t word = seg < 16 ? pl.code_lo : pl.code_hi;
          id = (int)((word >> ((seg & 15) * 4)) & 15) - 1;
        } else {
          id = classify_segment(cfg, rd, s, e);
        }
        if (seg) put('/');
        if (id >= 0) {
          const NameDev& nm = cfg.name((uint32_t)id);
          put('{');
          for (uint32_t q = 0; q < nm.len; q++) put(bytes[nm.off + q]);
          put('}');
        } else {
          for (uint32_t q = s; q < e; q++) put(rd.at(q));
        }
        seg++;
        if (e >= pl.n) break;
        s = e + 1;
      }
    }
  };

  if (!direct && pl.len) emit(s_out + local);
  __syncthreads();
  const uint64_t prefix = s_prefix;
  const bool overflow = prefix + total > a.out_cap;
  if (!overflow) {
    if (direct) {
      if (pl.len) emit(a.out_arena + prefix + local);
    } else {
      // coalesced copy of the tile image: 4-byte aligned body + byte edges
      uint8_t* dst = a.out_arena + prefix;
      uint32_t head = (uint32_t)((4 - ((uint64_t)dst & 3)) & 3);
      if (head > total) head = total;
      if ((uint32_t)tid < head) dst[tid] = s_out[tid];
      uint32_t body = (total - head) / 4;
      uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + head);
      for (uint32_t k = tid; k < body; k += kTile) {
        uint32_t b = head + 4 * k;
        d32[k] = (uint32_t)s_out[b] | ((uint32_t)s_out[b + 1] << 8) | ((uint32_t)s_out[b + 2] << 16) |
                 ((uint32_t)s_out[b + 3] << 24);
      }
      uint32_t tail0 = head + 4 * body;
      if ((uint32_t)tid < total - tail0) dst[tail0 + tid] = s_out[tail0 + tid];
    }
  }
  if (valid) {
    a.url_out[i] = oflags;
    a.tmpl[i] = ose_strref{(uint32_t)(prefix + local), pl.len};
  }
}

}  // namespace

void launch_url_template(const UrlKernelArgs& a, hipStream_t st) {
  uint32_t tiles = a.n_tiles;
  if (tiles == 0) return;
  hipLaunchKernelGGL(url_template_kernel, dim3(tiles), dim3(kTile), 0, st, a);
}

}  // namespace ose
