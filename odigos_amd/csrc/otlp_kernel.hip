// otlp_kernel.hip — OTLP protobuf ingest on the GPU: the
// Span messages of a serialized TracesData decoded straight into the
// columns the three stages read (what ptrace.ProtoUnmarshaler.UnmarshalTraces
// plus the shim's columnising walk produce on the CPU; collector/receivers/
// odigosebpfreceiver/traces.go:77-88, odigos_amd/csrc/columnize.cpp).
//
// One lane per span walks its payload once through 16-byte vector loads
// (ByteReader): ids, times, kind, name, status, the attributes whose keys
// the stages read (first occurrence, as pcommon.Map.Get), and the span's
// wire size as pdata's sizer computes it (gogo framing: ids, Status and
// KeyValue.value always emitted; otlp_pb.hpp / pdata.cpp ProtoSizer::span).
// Strings stay where they are: refs point into the message bytes, which are
// the arena.  A span the lane cannot finish exactly — a value that needs
// AsString or url.Parse, a nested ArrayValue / KeyValueList, a json
// span_attribute key, an id of unusual length, a group or malformed field,
// a repeated KeyValue field — is listed for the host pass (otlp_host.cpp),
// which decodes it with the host unmarshaler and writes all its columns.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "pb_device.hpp"

namespace ose {

namespace {
using namespace pbdev;
#ifndef OSE_OTHREADS
#define OSE_OTHREADS 64
#endif
// the per-record passes' workgroup size: one wave spreads a request's few
// records over more CUs (resource pass 79 -> 59 us per call against 256, r6st)
constexpr int kOThreads = OSE_OTHREADS;
#ifndef OSE_SPAN_STAGE
#define OSE_SPAN_STAGE 1
#endif
// waves per SIMD the HBM-read span kernel is compiled for: 3 (<= 168 VGPRs,
// a few spills) beats 2 (184 VGPRs) and 4 (117 spilled VGPRs), r6sv
#ifndef OSE_SPAN_WAVES
#define OSE_SPAN_WAVES 3
#endif
#ifndef OSE_SPAN_KEYS_LDS
#define OSE_SPAN_KEYS_LDS 1
#endif

// one KeyValue [s, e): key, value and its size (ProtoSizer::key_value, gogo)
__device__ OSE_PB_INL uint64_t key_value(Rd& r, uint32_t s, uint32_t e, uint32_t& ko, uint32_t& kl, Val& val) {
  const uint32_t save_i = r.i, save_end = r.end;
  r.i = s;
  r.end = e;
  uint32_t nkey = 0, nval = 0, vs = 0, vl = 0;
  ko = kl = 0;
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    uint32_t ps, pl;
    if (f == 1) {
      if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
      ko = ps; kl = pl; nkey++;
    } else if (f == 2) {
      if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
      vs = ps; vl = pl; nval++;
    } else {
      r.skip(wt);
    }
  }
  r.i = save_i;
  r.end = save_end;
  if (nkey > 1 || nval > 1) { r.bad = true; return 0; }   // field merges: host pass
  uint64_t av = 0;
  val.type = OSE_ATTR_OTHER;
  val.off = val.len = 0;
  val.v = 0;
  if (nval) av = any_value(r, vs, vs + vl, val);
  if (val.type == kNested) r.bad = true;                   // nested sizes: host pass
  return str_field(kl) + field_len(av);
}

// the key table the span decoder compares against: OtlpArgs' (HBM) or a
// workgroup's LDS copy of it
struct KeyTab {
  const OtlpKeyDev* keys;
  const uint8_t* bytes;
};
// the roles of key [o, o + l) (0 = not a key of interest)
__device__ OSE_PB_INL uint64_t key_roles(const OtlpArgs& a, const KeyTab& kt, Rd& r, uint32_t o, uint32_t l) {
  if (l >= 64 || !((a.key_lens >> l) & 1)) return 0;
  uint64_t roles = 0;
  for (uint32_t k = 0; k < a.n_keys; k++) {
    const OtlpKeyDev kd = kt.keys[k];
    if (kd.len != l) continue;
    uint32_t q = 0;
    while (q < l && r.br.at(o + q) == kt.bytes[kd.off + q]) q++;
    if (q == l) roles |= kd.roles;
  }
  return roles;
}

__device__ OSE_PB_INL bool same_bytes(Rd& r, uint32_t a0, uint32_t b0, uint32_t n) {
  for (uint32_t q = 0; q < n; q++)
    if (r.br.at(a0 + q) != r.br.at(b0 + q)) return false;
  return true;
}

// attributes of an Event / Link: sizes only (scalar values), [s, e)
__device__ OSE_PB_INL uint64_t nested_attr(Rd& r, uint32_t s, uint32_t e) {
  uint32_t ko, kl;
  Val v;
  return field_len(key_value(r, s, e, ko, kl, v));
}
}  // namespace

// span i: every byte read goes through `base` (the arena, or a wave's LDS
// copy of the arena bytes its spans cover); offsets stay arena offsets
__device__ __forceinline__ void decode_span(const OtlpArgs& a, const KeyTab& kt, uint64_t i, uint64_t ref, const uint8_t* base) {
  {
    const uint32_t s0 = (uint32_t)ref, s1 = s0 + (uint32_t)(ref >> 32);
    Rd r(base, s0, s1);
    uint64_t hi = 0, lo = 0, start = 0, end = 0;
    bool tid_nz = false, sid_nz = false, pid_nz = false;
    uint32_t ts_len = 0, name_off = 0, name_len = 0, kind = 0, flags = 0;
    uint32_t dr_attrs = 0, dr_events = 0, dr_links = 0, st_msg = 0, st_code = 0;
    uint64_t attrs_sz = 0, events_sz = 0, links_sz = 0;
    uint64_t found = 0;   // roles seen (first occurrence wins)
    Val mnew{0, 0, 0, 0}, mold{0, 0, 0, 0}, route{0, 0, 0, 0}, utmpl{0, 0, 0, 0}, upath{0, 0, 0, 0},
        target{0, 0, 0, 0};
    bool full_seen = false, host_key = false;
    uint32_t f, wt;
    while (r.more() && r.tag(f, wt)) {
      uint32_t ps, pl;
      switch (f) {
        case 1:   // trace_id
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          if (pl == 16) {
            hi = lo = 0;
            for (uint32_t k = 0; k < 8; k++) hi = hi << 8 | r.br.at(ps + k);
            for (uint32_t k = 0; k < 8; k++) lo = lo << 8 | r.br.at(ps + 8 + k);
            tid_nz = (hi | lo) != 0;
          } else if (pl == 0) {
            hi = lo = 0;
            tid_nz = false;
          } else {
            r.bad = true;
          }
          break;
        case 2:
        case 4: {   // span_id / parent_span_id
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          bool nz = false;
          if (pl == 8) {
            for (uint32_t k = 0; k < 8; k++) nz |= r.br.at(ps + k) != 0;
          } else if (pl != 0) {
            r.bad = true;
          }
          if (f == 2) sid_nz = nz; else pid_nz = nz;
          break;
        }
        case 3:
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          ts_len = pl;
          break;
        case 5:
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          name_off = ps;
          name_len = pl;
          break;
        case 6:
          if (wt != 0) { r.bad = true; break; }
          kind = (uint32_t)r.varint();
          break;
        case 7:
        case 8:
          if (wt != 1) { r.bad = true; break; }
          if (f == 7) start = r.fixed(8); else end = r.fixed(8);
          break;
        case 9: {   // attributes
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          uint32_t ko, kl;
          Val v;
          attrs_sz += field_len(key_value(r, ps, ps + pl, ko, kl, v));
          if (r.bad) break;
          const uint64_t roles = key_roles(a, kt, r, ko, kl) & ~found;
          if (!roles) break;
          found |= roles;
          if (roles & kRoleMethodNew) mnew = v;
          if (roles & kRoleMethodOld) mold = v;
          if (roles & kRoleRoute) route = v;
          if (roles & kRoleUrlTmpl) utmpl = v;
          if (roles & kRoleUrlPath) upath = v;
          if (roles & kRoleTarget) target = v;
          if (roles & kRoleFull) full_seen = true;
          if (roles & kRoleHost) host_key = true;
          for (uint32_t k = 0; k < a.n_attr_keys && k < kOtlpMaxAttrKeys; k++)
            if (roles & (kRoleAttr0 << k)) {
              const uint64_t j = (uint64_t)k * a.n_spans + i;
              uint32_t t = v.type == kAttrBytes ? OSE_ATTR_OTHER : v.type;
              a.attr_type[j] = (uint8_t)t;
              a.attr_val[j] = t == OSE_ATTR_STR ? ((uint64_t)v.off | ((uint64_t)v.len << 32)) : v.v;
            }
          break;
        }
        case 10: if (wt != 0) r.bad = true; else dr_attrs = (uint32_t)r.varint(); break;
        case 11: {   // events: time, name, attributes, dropped
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          const uint32_t save_i = r.i, save_end = r.end;
          r.i = ps;
          r.end = ps + pl;
          uint64_t t = 0, ea = 0;
          uint32_t nl = 0, dr = 0, f2, w2, qs, ql;
          while (r.more() && r.tag(f2, w2)) {
            if (f2 == 1) { if (w2 != 1) r.bad = true; else t = r.fixed(8); }
            else if (f2 == 2) { if (w2 != 2 || !r.len(qs, ql)) r.bad = true; else nl = ql; }
            else if (f2 == 3) { if (w2 != 2 || !r.len(qs, ql)) r.bad = true; else ea += nested_attr(r, qs, qs + ql); }
            else if (f2 == 4) { if (w2 != 0) r.bad = true; else dr = (uint32_t)r.varint(); }
            else r.skip(w2);
          }
          r.i = save_i;
          r.end = save_end;
          events_sz += field_len((t ? 9 : 0) + str_field(nl) + ea + varint_field(dr));
          break;
        }
        case 12: if (wt != 0) r.bad = true; else dr_events = (uint32_t)r.varint(); break;
        case 13: {   // links: trace_id, span_id, trace_state, attributes, dropped, flags
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          const uint32_t save_i = r.i, save_end = r.end;
          r.i = ps;
          r.end = ps + pl;
          uint64_t la = 0;
          uint32_t tsl = 0, dr = 0, lf = 0, f2, w2, qs, ql;
          bool lt = false, ls = false;
          while (r.more() && r.tag(f2, w2)) {
            if (f2 == 1 || f2 == 2) {
              if (w2 != 2 || !r.len(qs, ql)) { r.bad = true; break; }
              const uint32_t want = f2 == 1 ? 16 : 8;
              bool nz = false;
              if (ql == want) { for (uint32_t k = 0; k < ql; k++) nz |= r.br.at(qs + k) != 0; }
              else if (ql != 0) r.bad = true;
              if (f2 == 1) lt = nz; else ls = nz;
            } else if (f2 == 3) { if (w2 != 2 || !r.len(qs, ql)) r.bad = true; else tsl = ql; }
            else if (f2 == 4) { if (w2 != 2 || !r.len(qs, ql)) r.bad = true; else la += nested_attr(r, qs, qs + ql); }
            else if (f2 == 5) { if (w2 != 0) r.bad = true; else dr = (uint32_t)r.varint(); }
            else if (f2 == 6) { if (w2 != 5) r.bad = true; else lf = (uint32_t)r.fixed(4); }
            else r.skip(w2);
          }
          r.i = save_i;
          r.end = save_end;
          links_sz += field_len((lt ? 18 : 2) + (ls ? 10 : 2) + str_field(tsl) + la + varint_field(dr) + (lf ? 5 : 0));
          break;
        }
        case 14: if (wt != 0) r.bad = true; else dr_links = (uint32_t)r.varint(); break;
        case 15: {   // status: message (2), code (3); merges
          if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
          const uint32_t save_i = r.i, save_end = r.end;
          r.i = ps;
          r.end = ps + pl;
          uint32_t f2, w2, qs, ql;
          while (r.more() && r.tag(f2, w2)) {
            if (f2 == 2) { if (w2 != 2 || !r.len(qs, ql)) r.bad = true; else st_msg = ql; }
            else if (f2 == 3) { if (w2 != 0) r.bad = true; else st_code = (uint32_t)r.varint(); }
            else r.skip(w2);
          }
          r.i = save_i;
          r.end = save_end;
          break;
        }
        case 16: if (wt != 5) r.bad = true; else flags = (uint32_t)r.fixed(4); break;
        default:
          r.skip(wt);
      }
    }
    // the url path source and the values AsString would have to format
    const Val m = (found & kRoleMethodNew) ? mnew : mold;
    const bool has_m = (found & (kRoleMethodNew | kRoleMethodOld)) != 0;
    bool host = r.bad || host_key;
    if (found & kRoleRoute) host |= route.type != OSE_ATTR_STR;
    uint32_t uf = 0;
    ose_strref path{0, 0};
    if (has_m && !host) {
      uf |= OSE_URL_HAS_METHOD;
      if (m.type != OSE_ATTR_STR) host = true;
      else if (m.len == name_len && same_bytes(r, m.off, name_off, name_len)) uf |= OSE_URL_NAME_EQ_METHOD;
      const bool client = (int32_t)kind == OSE_KIND_CLIENT;
      const Val tv = client ? utmpl : route;
      if (found & (client ? kRoleUrlTmpl : kRoleRoute)) {
        if (tv.type != OSE_ATTR_STR) uf |= OSE_URL_TGT_NONSTR;
        else uf |= tv.len == 0 ? OSE_URL_TGT_STR_EMPTY : OSE_URL_TGT_STR;
      }
      if (found & kRoleUrlPath) {
        uf |= OSE_URL_PATH_RAW;
        if (upath.type != OSE_ATTR_STR) host = true;
        path = ose_strref{upath.off, upath.len};
      } else if (found & kRoleTarget) {
        uf |= OSE_URL_PATH_TARGET;
        if (target.type != OSE_ATTR_STR) host = true;
        path = ose_strref{target.off, target.len};
      } else if (full_seen) {
        host = true;   // net/url.Parse
      }
    }
    if (host) {
      a.host_flag[i] = 1;
      const uint32_t slot = atomicAdd(a.host_count, 1u);
      if (slot < a.host_cap) a.host_list[slot] = (uint32_t)i;
      return;
    }
    a.host_flag[i] = 0;
    for (uint32_t k = 0; k < a.n_attr_keys; k++)   // keys this span does not carry (keys past
      if (k >= kOtlpMaxAttrKeys || !(found & (kRoleAttr0 << k))) {   // kOtlpMaxAttrKeys send it to the host)
        a.attr_type[(uint64_t)k * a.n_spans + i] = OSE_ATTR_ABSENT;
        a.attr_val[(uint64_t)k * a.n_spans + i] = 0;
      }
    a.tid[2 * i] = hi;
    a.tid[2 * i + 1] = lo;
    a.start[i] = start;
    a.end[i] = end;
    const int32_t code = (int32_t)st_code;
    a.status[i] = (uint8_t)(code >= 0 && code <= 2 ? code : 3);
    const int32_t k32 = (int32_t)kind;
    a.kind[i] = (uint8_t)(k32 < 0 ? 0 : (k32 > 255 ? 255 : k32));
    a.url_flags[i] = (uint8_t)uf;
    a.path[i] = path;
    a.route[i] = (found & kRoleRoute) ? ose_strref{route.off, route.len} : ose_strref{0, 0};
    a.name_len[i] = name_len;
    if (a.attr_match)
      for (uint32_t w = 0; w < a.attr_words; w++) a.attr_match[(uint64_t)w * a.n_spans + i] = 0;
    // ProtoSizer::span (gogo): ids, Status and KeyValue.value always emitted
    const uint64_t st = str_field(st_msg) + varint_field((uint64_t)(int64_t)(int32_t)st_code);
    const uint64_t sz = (tid_nz ? 18 : 2) + (sid_nz ? 10 : 2) + str_field(ts_len) + (pid_nz ? 10 : 2) +
                        str_field(name_len) + varint_field((uint64_t)(int64_t)k32) + (start ? 9 : 0) + (end ? 9 : 0) +
                        attrs_sz + varint_field(dr_attrs) + events_sz + varint_field(dr_events) + links_sz +
                        varint_field(dr_links) + field_len(st) + (flags ? 6 : 0);
    a.span_size[i] = (uint32_t)sz;
  }
}

// one lane per span, arena bytes read from HBM through the lane's 16-byte
// reader (batches above kSpanStageMax spans)
// the key table into LDS when it fits (every attribute key is compared
// byte by byte against the keys of its length)
constexpr uint32_t kKeyLds = 128, kKeyBytesLds = 4096;
__device__ __forceinline__ KeyTab stage_keys(const OtlpArgs& a, OtlpKeyDev* s_keys, uint32_t* s_kb) {
  KeyTab kt{a.keys, a.key_bytes};
  if (!OSE_SPAN_KEYS_LDS || a.n_keys == 0 || a.n_keys > kKeyLds) return kt;
  const OtlpKeyDev last = a.keys[a.n_keys - 1];   // keys are appended in order: last.off + last.len bytes
  const uint32_t nkb = last.off + last.len;
  if (nkb > kKeyBytesLds) return kt;
  for (uint32_t k = threadIdx.x; k < a.n_keys; k += blockDim.x) s_keys[k] = a.keys[k];
  for (uint32_t c = threadIdx.x; c < (nkb + 3) / 4; c += blockDim.x) {
    const uint8_t* p = a.key_bytes + 4 * c;   // the key blob has 16 bytes of slack
    s_kb[c] = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
  }
  __syncthreads();
  return KeyTab{s_keys, reinterpret_cast<const uint8_t*>(s_kb)};
}

#if OSE_SPAN_WAVES
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(OSE_SPAN_WAVES))) void otlp_span_kernel(OtlpArgs a) {
#else
__global__ __launch_bounds__(kWave) void otlp_span_kernel(OtlpArgs a) {
#endif
  __shared__ OtlpKeyDev s_keys[kKeyLds];
  __shared__ uint32_t s_kb[kKeyBytesLds / 4];
  const KeyTab kt = stage_keys(a, s_keys, s_kb);
  const uint64_t stride = (uint64_t)gridDim.x * kWave;
  for (uint64_t i = (uint64_t)blockIdx.x * kWave + threadIdx.x; i < a.n_spans; i += stride)
    decode_span(a, kt, i, a.span_ref[i], a.pb);
}

// One wave per workgroup.  Each round the wave copies the arena bytes its 64
// spans cover (consecutive spans sit back to back in the message) into LDS
// with coalesced 16-byte loads, then every lane parses its span from there:
// the lane's ~20 dependent chunk reads become LDS round trips instead of HBM
// ones.  A round whose spans cover more than kSpanStage bytes reads the arena.
// The 24 KB per wave caps residency, so only batches that cannot fill the
// chip anyway (<= kSpanStageMax spans: a pipeline request batch) take it;
// measured in profiles/r6sx_otlp_span_kernel_ab.txt.
constexpr uint32_t kSpanStage = 24576;
constexpr uint64_t kSpanStageMax = 65536;
__global__ __launch_bounds__(kWave) void otlp_span_lds_kernel(OtlpArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 stage[kSpanStage / 16];
  __shared__ OtlpKeyDev s_keys[kKeyLds];
  __shared__ uint32_t s_kb[kKeyBytesLds / 4];
  const KeyTab kt = stage_keys(a, s_keys, s_kb);
  const uint32_t lane = threadIdx.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * kWave; i0 < a.n_spans; i0 += (uint64_t)gridDim.x * kWave) {
    const uint64_t i = i0 + lane;
    const bool live = i < a.n_spans;
    const uint64_t ref = live ? a.span_ref[i] : 0;
    const uint32_t s0 = (uint32_t)ref, s1 = s0 + (uint32_t)(ref >> 32);
    const uint32_t lo = wave_min_u32(live ? s0 : 0xFFFFFFFFu) & ~15u;
    const uint32_t hi = wave_max_u32(live ? s1 : 0u);
    // chunks [lo, hi) plus one: ByteReader::word reads up to 3 bytes past a string
    const uint32_t nchunk = ((hi + 15u) >> 4) - (lo >> 4) + 1u;
    const uint8_t* base = a.pb;
    if (nchunk <= kSpanStage / 16) {
      const uint4* src = reinterpret_cast<const uint4*>(a.pb + lo);
      for (uint32_t c = lane; c < nchunk; c += kWave) stage[c] = src[c];
      __syncthreads();
      // (integer arithmetic: the result points below the LDS array)
      base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uint64_t>(static_cast<const void*>(stage)) - lo);
    }
    if (live) decode_span(a, kt, i, ref, base);
    __syncthreads();
  }
}

// host-pass results: every column of the listed spans
__global__ __launch_bounds__(kOThreads) void otlp_fix_kernel(OtlpFixArgs a) {
  const uint32_t q = blockIdx.x * kOThreads + threadIdx.x;
  if (q >= a.n) return;
  const OtlpFix& x = a.fix[q];
  const uint64_t i = x.idx;
  a.tid[2 * i] = x.hi;
  a.tid[2 * i + 1] = x.lo;
  a.start[i] = x.start;
  a.end[i] = x.end;
  a.status[i] = x.status;
  a.kind[i] = x.kind;
  a.url_flags[i] = x.url_flags;
  a.path[i] = x.path;
  a.route[i] = x.route;
  a.name_len[i] = x.name_len;
  a.span_size[i] = x.span_size;
  if (a.attr_match)
    for (uint32_t w = 0; w < a.attr_words; w++) a.attr_match[(uint64_t)w * a.n_spans + i] = a.fix_attr[(uint64_t)q * a.attr_words + w];
  for (uint32_t k = 0; k < a.n_attr_keys; k++) {
    a.attr_type[(uint64_t)k * a.n_spans + i] = a.fix_type[(uint64_t)q * a.n_attr_keys + k];
    a.attr_val[(uint64_t)k * a.n_spans + i] = a.fix_val[(uint64_t)q * a.n_attr_keys + k];
  }
}

// ---- ScopeSpans on the GPU ------------------------------------------------------
// Pass 1, one lane per scope: the fields of its payload (otlp_pb.cpp
// pb_walk's ScopeSpans loop): InstrumentationScope (1), spans (2),
// schema_url (3), others skipped.  The scope's fixed size is
// ProtoSizer::scope_fixed: the InstrumentationScope framed (always, gogo)
// + schema_url; a merged or unusual scope message leaves it to the host.
__global__ __launch_bounds__(kOThreads) void otlp_scope_count_kernel(OtlpScopeArgs a) {
  const uint64_t q = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (q >= a.n_scopes || a.on_host[q]) return;
  const uint64_t ref = a.scope_ref[q];
  const uint32_t s0 = (uint32_t)ref, s1 = s0 + (uint32_t)(ref >> 32);
  Rd r(a.pb, s0, s1);
  uint32_t n = 0, nh = 0, flags = 0;
  uint64_t hdr = 0, schema = 0;
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    uint32_t ps, pl;
    if (f == 1 || f == 2 || f == 3) {
      if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
      if (f == 1) { hdr = (uint64_t)ps | ((uint64_t)pl << 32); nh++; }
      else if (f == 2) n++;
      else schema = (uint64_t)ps | ((uint64_t)pl << 32);
    } else {
      r.skip(wt);
    }
  }
  if (r.bad) {
    a.flags[q] = 2;
    a.count[q] = 0;
    return;
  }
  // the InstrumentationScope's pdata size (name, version: last occurrence)
  uint64_t sc = 0;
  if (nh == 1) {
    Rd h(a.pb, (uint32_t)hdr, (uint32_t)hdr + (uint32_t)(hdr >> 32));
    uint32_t name = 0, version = 0;
    uint64_t dropped = 0, attrs = 0;
    while (h.more() && h.tag(f, wt)) {
      uint32_t ps, pl;
      if (f == 1 || f == 2 || f == 3) {
        if (wt != 2 || !h.len(ps, pl)) { h.bad = true; break; }
        if (f == 1) name = pl;
        else if (f == 2) version = pl;
        else {
          uint32_t ko, kl;
          Val v;
          attrs += field_len(key_value(h, ps, ps + pl, ko, kl, v));
        }
      } else if (f == 4) {
        if (wt != 0) { h.bad = true; break; }
        dropped = (uint32_t)h.varint();
      } else {
        h.skip(wt);
      }
    }
    if (h.bad) flags = 1;
    sc = str_field(name) + str_field(version) + attrs + varint_field(dropped);
  } else if (nh > 1) {
    flags = 1;
    hdr = kOtlpScopeMulti;
  }
  a.count[q] = n;
  a.hdr[q] = hdr;
  a.schema[q] = schema;
  a.flags[q] = flags;
  a.scope_size[q] = flags ? 0u : (uint32_t)(field_len(sc) + str_field((uint32_t)(schema >> 32)));
}

// Pass 2: every scope's span refs at their place in the batch
__global__ __launch_bounds__(kOThreads) void otlp_scope_spans_kernel(OtlpScopeArgs a) {
  const uint64_t q = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (q >= a.n_scopes) return;
  uint64_t i = a.span0[q];
  const uint32_t res = a.scope_res[q];
  if (a.on_host[q]) {
    const uint64_t at = a.host_at[q];
    for (uint32_t k = 0; k < a.count[q]; k++, i++) {
      a.span_ref[i] = a.host_refs[at + k];
      a.span_res[i] = res;
      a.span_scope[i] = (uint32_t)q;
    }
    return;
  }
  const uint64_t ref = a.scope_ref[q];
  const uint32_t s0 = (uint32_t)ref, s1 = s0 + (uint32_t)(ref >> 32);
  Rd r(a.pb, s0, s1);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    uint32_t ps, pl;
    if (f == 1 || f == 2 || f == 3) {
      if (wt != 2 || !r.len(ps, pl)) break;
      if (f == 2) {
        a.span_ref[i] = (uint64_t)ps | ((uint64_t)pl << 32);
        a.span_res[i] = res;
        a.span_scope[i] = (uint32_t)q;
        i++;
      }
    } else {
      r.skip(wt);
    }
  }
}

// ---- the TracesData chain on the GPU -------------------------------------------------
// a plausible record start at q: field 1 (0x0A) whose length frames a record
// whose payload starts with a Resource or ScopeSpans tag, 4 such in a row (or
// the message end) -- the host walk's find_start (otlp_host.cpp)
__device__ bool chain_plausible(const uint8_t* pb, uint64_t n, uint32_t q) {
  uint32_t pos = q;
  for (int hops = 0; hops < 4 && pos < n; hops++) {
    Rd r(pb, pos, (uint32_t)n);
    uint32_t f, wt, ps, pl;
    if (!r.tag(f, wt) || f != 1 || wt != 2 || !r.len(ps, pl) || pl == 0) return false;
    const uint32_t b0 = r.br.at(ps);
    if (b0 != 0x0A && b0 != 0x12) return false;
    pos = r.i;
  }
  return true;
}
__global__ __launch_bounds__(kOThreads) void otlp_chain_seg_kernel(OtlpChainArgs a) {
  const uint32_t t = blockIdx.x * kOThreads + threadIdx.x;
  if (t >= a.n_seg) return;
  const uint64_t s0 = (uint64_t)t * kChainSeg, s1 = min<uint64_t>(a.n, s0 + kChainSeg);
  uint64_t c = kChainNone;
  if (t == 0) {
    c = 0;
  } else {
    ByteReader br(a.pb);
    for (uint64_t q = s0; q < s1; q++)
      if (br.at((uint32_t)q) == 0x0A && chain_plausible(a.pb, a.n, (uint32_t)q)) { c = q; break; }
  }
  a.start[t] = c;
  a.nrec[t] = 0;
  a.bad[t] = 0;
  if (c == kChainNone) return;
  Rd r(a.pb, (uint32_t)c, (uint32_t)a.n);
  uint32_t k = 0, nrec = 0;
  while (r.i < s1 && r.i < a.n) {
    const uint64_t at = r.i;
    uint32_t f, wt;
    if (!r.tag(f, wt)) break;
    const bool rec = f == 1 && wt == 2;
    if (k < kChainList) a.list[(uint64_t)t * kChainList + k] = at | ((uint64_t)rec << 63);
    k++;
    if (!r.skip(wt)) break;
    nrec += rec;
  }
  for (; k < kChainList; k++) a.list[(uint64_t)t * kChainList + k] = kChainNone;
  a.bad[t] = r.bad ? 1u : 0u;
  a.end[t] = r.i;
  a.nrec[t] = nrec;
}
__global__ __launch_bounds__(kOThreads) void otlp_chain_list_kernel(OtlpChainArgs a) {
  const uint32_t t = blockIdx.x * kOThreads + threadIdx.x;
  if (t >= a.n_seg || a.first[t] == kChainNone) return;
  const uint64_t s1 = min<uint64_t>(a.n, (uint64_t)t * kChainSeg + kChainSeg);
  Rd r(a.pb, (uint32_t)a.first[t], (uint32_t)a.n);
  uint64_t q = a.base[t];
  while (r.i < s1 && r.i < a.n) {
    uint32_t f, wt;
    if (!r.tag(f, wt)) break;
    if (f == 1 && wt == 2) {
      uint32_t ps, pl;
      if (!r.len(ps, pl)) break;
      a.res_ref[q++] = (uint64_t)ps | ((uint64_t)pl << 32);
    } else if (!r.skip(wt)) {
      break;
    }
  }
}
void launch_otlp_chain_seg(const OtlpChainArgs& a, hipStream_t st) {
  if (a.n_seg)
    hipLaunchKernelGGL(otlp_chain_seg_kernel, dim3((a.n_seg + kOThreads - 1) / kOThreads), dim3(kOThreads), 0, st, a);
}
void launch_otlp_chain_list(const OtlpChainArgs& a, hipStream_t st) {
  if (a.n_seg)
    hipLaunchKernelGGL(otlp_chain_list_kernel, dim3((a.n_seg + kOThreads - 1) / kOThreads), dim3(kOThreads), 0, st, a);
}

// ---- ResourceSpans on the GPU ------------------------------------------------------
// Pass 1, one lane per ResourceSpans (otlp_pb.cpp pb_walk's ResourceSpans
// loop): Resource (1), scope_spans (2), the deprecated
// instrumentation_library_spans (1000, read only when there is no field 2),
// schema_url (3), others skipped.  The Resource's columns come from the
// device table when its message bytes are there (one Resource field; the
// empty key stands for none); else the row is listed for the host.
__global__ __launch_bounds__(kOThreads) void otlp_res_fields_kernel(OtlpResArgs a) {
  const uint64_t r = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (r >= a.n_res) return;
  const uint64_t ref = a.res_ref[r];
  const uint32_t s0 = (uint32_t)ref, s1 = s0 + (uint32_t)(ref >> 32);
  Rd rd(a.pb, s0, s1);
  uint32_t nres = 0, nsc = 0, ndep = 0, schema = 0, ro = 0, rl = 0;
  uint32_t f, wt;
  while (rd.more() && rd.tag(f, wt)) {
    uint32_t ps, pl;
    if (f == 1 || f == 2 || f == 3 || f == 1000) {
      if (wt != 2 || !rd.len(ps, pl)) { rd.bad = true; break; }
      if (f == 1) { ro = ps; rl = pl; nres++; }
      else if (f == 2) nsc++;
      else if (f == 1000) ndep++;
      else schema = pl;
    } else {
      rd.skip(wt);
    }
  }
  uint32_t flags = 0;
  if (rd.bad) {
    a.flags[r] = 2;
    a.nscope[r] = 0;
    atomicOr(a.any_bad, 1u);
    return;
  }
  if (!nsc && ndep) flags |= 4;
  a.nscope[r] = nsc ? nsc : ndep;
  a.schema_len[r] = schema;
  bool found = false;
  if (nres <= 1) {
    uint64_t h = kResHashSeed;
    for (uint32_t q = 0; q < rl; q++) h = res_key_hash_step(h, rd.br.at(ro + q));
    for (uint32_t probe = 0, slot = (uint32_t)h & (kResSlots - 1); probe < 64; probe++, slot = (slot + 1) & (kResSlots - 1)) {
      const ResSlotDev& e = a.table[slot];
      if (!e.ready) break;
      if (e.h != h || e.klen != rl) continue;
      uint32_t q = 0;
      while (q < rl && a.keys[e.koff + q] == rd.br.at(ro + q)) q++;
      if (q < rl) continue;
      a.res_svc[r] = e.svc;
      a.res_svc_str[r] = e.svc_str;
      a.res_set[r] = e.set;
      a.res_ok[r] = (uint8_t)e.ok;
      a.attr_res[r] = e.attr_res;
      a.res_size[r] = e.rpart + (schema ? (uint32_t)field_len(schema) : 0u);
      found = true;
      break;
    }
  }
  if (!found) {
    flags |= 1;
    a.miss_list[atomicAdd(a.miss_count, 1u)] = (uint32_t)r;
  }
  a.flags[r] = flags;
}

// Pass 2: every resource's ScopeSpans refs at their place
__global__ __launch_bounds__(kOThreads) void otlp_res_scopes_kernel(OtlpResArgs a) {
  const uint64_t r = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (r >= a.n_res) return;
  const uint32_t want = (a.flags[r] & 4) ? 1000u : 2u;
  uint64_t q = a.scope0[r];
  const uint64_t ref = a.res_ref[r];
  const uint32_t s0 = (uint32_t)ref, s1 = s0 + (uint32_t)(ref >> 32);
  Rd rd(a.pb, s0, s1);
  uint32_t f, wt;
  while (rd.more() && rd.tag(f, wt)) {
    uint32_t ps, pl;
    if (f == 1 || f == 2 || f == 3 || f == 1000) {
      if (wt != 2 || !rd.len(ps, pl)) break;
      if (f == want) {
        a.scope_ref[q] = (uint64_t)ps | ((uint64_t)pl << 32);
        a.scope_res[q] = (uint32_t)r;
        q++;
      }
    } else {
      rd.skip(wt);
    }
  }
}

__global__ __launch_bounds__(kOThreads) void otlp_res_fix_kernel(OtlpResArgs a, const OtlpResFix* fix, uint32_t n) {
  const uint32_t k = blockIdx.x * kOThreads + threadIdx.x;
  if (k >= n) return;
  const OtlpResFix x = fix[k];
  const uint32_t sch = a.schema_len[x.row];
  a.res_svc[x.row] = x.svc;
  a.res_svc_str[x.row] = x.svc_str;
  a.res_set[x.row] = x.set;
  a.res_ok[x.row] = (uint8_t)x.ok;
  a.attr_res[x.row] = x.attr_res;
  a.res_size[x.row] = x.rpart + (sch ? (uint32_t)field_len(sch) : 0u);
}

__global__ __launch_bounds__(kOThreads) void otlp_set_min_kernel(const uint32_t* res_set, uint64_t n, uint32_t* first) {
  const uint64_t r = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (r < n) atomicMin(&first[res_set[r]], (uint32_t)r);
}
__global__ __launch_bounds__(kOThreads) void otlp_set_flag_kernel(const uint32_t* res_set, uint64_t n, const uint32_t* first,
                                                                  uint32_t* is_first) {
  const uint64_t r = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (r < n) is_first[r] = first[res_set[r]] == (uint32_t)r ? 1u : 0u;
}
__global__ __launch_bounds__(kOThreads) void otlp_set_apply_kernel(uint32_t* res_set, uint64_t n, const uint32_t* first,
                                                                   const uint32_t* is_first, const uint32_t* pos,
                                                                   uint32_t* list) {
  const uint64_t r = (uint64_t)blockIdx.x * kOThreads + threadIdx.x;
  if (r >= n) return;
  const uint32_t s = res_set[r];
  if (is_first[r]) list[pos[r]] = s;
  res_set[r] = pos[first[s]];
}

void launch_otlp_res_fields(const OtlpResArgs& a, hipStream_t st) {
  if (a.n_res)
    hipLaunchKernelGGL(otlp_res_fields_kernel, dim3((uint32_t)((a.n_res + kOThreads - 1) / kOThreads)), dim3(kOThreads), 0,
                       st, a);
}
void launch_otlp_res_scopes(const OtlpResArgs& a, hipStream_t st) {
  if (a.n_res)
    hipLaunchKernelGGL(otlp_res_scopes_kernel, dim3((uint32_t)((a.n_res + kOThreads - 1) / kOThreads)), dim3(kOThreads), 0,
                       st, a);
}
void launch_otlp_res_fix(const OtlpResArgs& a, const OtlpResFix* fix, uint32_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(otlp_res_fix_kernel, dim3((n + kOThreads - 1) / kOThreads), dim3(kOThreads), 0, st, a, fix, n);
}
void launch_otlp_set_first(const uint32_t* res_set, uint64_t n_res, uint32_t* first, uint32_t* is_first,
                           hipStream_t st) {
  if (!n_res) return;
  const dim3 g((uint32_t)((n_res + kOThreads - 1) / kOThreads));
  hipLaunchKernelGGL(otlp_set_min_kernel, g, dim3(kOThreads), 0, st, res_set, n_res, first);
  hipLaunchKernelGGL(otlp_set_flag_kernel, g, dim3(kOThreads), 0, st, res_set, n_res, first, is_first);
}
void launch_otlp_set_apply(uint32_t* res_set, uint64_t n_res, const uint32_t* first, const uint32_t* is_first,
                           const uint32_t* pos, uint32_t* list, hipStream_t st) {
  if (n_res)
    hipLaunchKernelGGL(otlp_set_apply_kernel, dim3((uint32_t)((n_res + kOThreads - 1) / kOThreads)), dim3(kOThreads), 0,
                       st, res_set, n_res, first, is_first, pos, list);
}

void launch_otlp_scope_count(const OtlpScopeArgs& a, hipStream_t st) {
  if (a.n_scopes)
    hipLaunchKernelGGL(otlp_scope_count_kernel, dim3((uint32_t)((a.n_scopes + kOThreads - 1) / kOThreads)),
                       dim3(kOThreads), 0, st, a);
}
void launch_otlp_scope_spans(const OtlpScopeArgs& a, hipStream_t st) {
  if (a.n_scopes)
    hipLaunchKernelGGL(otlp_scope_spans_kernel, dim3((uint32_t)((a.n_scopes + kOThreads - 1) / kOThreads)),
                       dim3(kOThreads), 0, st, a);
}

void launch_otlp_spans(const OtlpArgs& a, hipStream_t st) {
  const uint64_t blocks = std::min<uint64_t>((a.n_spans + kWave - 1) / kWave, 32768);
  if (!blocks) return;
  if (OSE_SPAN_STAGE && a.n_spans <= kSpanStageMax)
    hipLaunchKernelGGL(otlp_span_lds_kernel, dim3((uint32_t)blocks), dim3(kWave), 0, st, a);
  else
    hipLaunchKernelGGL(otlp_span_kernel, dim3((uint32_t)blocks), dim3(kWave), 0, st, a);
}
void launch_otlp_fix(const OtlpFixArgs& a, hipStream_t st) {
  const uint32_t blocks = (a.n + kOThreads - 1) / kOThreads;
  if (blocks) hipLaunchKernelGGL(otlp_fix_kernel, dim3(blocks), dim3(kOThreads), 0, st, a);
}

}  // namespace ose
