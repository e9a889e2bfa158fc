// encode_kernel.hip — the gateway's output side on the GPU:
// routing (odigosrouterconnector, collector/connectors/odigosrouterconnector/
// connector.go:147-237, routingmap.go:34-103) and the exporters' marshal step
// (ptrace.ProtoMarshaler.MarshalTraces) applied to a batch the decoder left in
// HBM, with the stages' decisions (keep, url_out, template refs) beside it.
// It is the device form of otlp_encode.cpp's two passes and writes the same
// bytes:
//   sizing   enc_span_kernel (a lane per span: its framed size, and for a
//            renamed / templated span the edit plan — where the name field
//            and the target KeyValue go), enc_scope_kernel (a lane per
//            scope), enc_res_kernel (a lane per resource: header, schema,
//            record size, and its pipelines from the Resource's k8s
//            attributes);
//   offsets  an exclusive scan per output over the records routed to it;
//   writing  enc_write_kernel, a wave per resource writing its record to
//            every output it routes to: tags and lengths, then the message
//            bytes it keeps (verbatim, or edited as planned).
// A span is copied (or edited in place) only when its bytes are already
// pdata's encoding (the decoder's pdata size equals its length, as the host
// encoder decides); headers likewise.  Anything else — and every case the
// host encoder re-marshals — sets a flag and the host encoder runs instead.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "pb_device.hpp"

namespace ose {

namespace {
using namespace pbdev;
constexpr int kEThreads = 256;
// the per-record passes' (spans, scopes, resources, write) workgroup size: one
// wave (a request's few records over more CUs; r6se / r6sg)
#ifndef OSE_ETHREADS
#define OSE_ETHREADS 64
#endif
constexpr int kERec = OSE_ETHREADS;

__device__ __forceinline__ bool eq_lit(ByteReader& br, uint32_t o, uint32_t n, const char* lit, uint32_t ln) {
  if (n != ln) return false;
  for (uint32_t q = 0; q < n; q++)
    if (br.at(o + q) != (uint8_t)lit[q]) return false;
  return true;
}

// KeyValue{key, AnyValue{string_value}} body size (otlp_encode.cpp kv_len)
__device__ __forceinline__ uint64_t kv_len(bool client, uint64_t tl) {
  return field_len(client ? 12 : 10) + field_len(field_len(tl));
}

__device__ __forceinline__ void flag(const EncArgs& a, uint32_t f) { atomicOr(a.flags, f); }
}  // namespace

// ---- sizing: spans -------------------------------------------------------------
// Enc::rewrite / plan_edit (otlp_encode.cpp) for the spans whose encoding is
// pdata's; a span that is not (span_size != its length) is re-marshaled by
// the host encoder, so it flags the call.
__global__ __launch_bounds__(kERec) void enc_span_kernel(EncArgs a) {
  const uint64_t stride = (uint64_t)gridDim.x * kERec;
  uint32_t fb = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kERec + threadIdx.x; i < a.n_spans; i += stride) {
    if (a.keep && !a.keep[i]) {
      a.span_out[i] = 0;
      continue;
    }
    const uint64_t ref = a.span_ref[i];
    const uint32_t off = (uint32_t)ref, L = (uint32_t)(ref >> 32);
    const uint32_t u = a.url_out ? a.url_out[i] : 0u;
    const bool canonical = a.span_size[i] == L;
    a.span_out[i] = (uint32_t)field_len(L);
    if (!canonical) {   // Enc::remarshal
      fb |= kEncFbSpan;
      continue;
    }
    if (!u) continue;   // verbatim
    const ose_strref t = a.tmpl[i];
    if ((uint64_t)t.off + t.len > *a.tmpl_used) {
      fb |= kEncFbTmpl;
      continue;
    }
    // plan_edit: fields ascend, so the new name takes field 5's place (or
    // goes before the first later field) and the target KeyValue replaces
    // the first one with its key or goes after the last attribute
    uint32_t name_a = L, name_b = L, attr_a = L, attr_b = L;
    int32_t kind = 0;
    bool name_set = false, attr_set = false, have_new = false, have_old = false;
    bool new_v = false, old_v = false;
    uint32_t new_o = 0, new_l = 0, old_o = 0, old_l = 0;
    uint32_t prev_f = 0;
    bool ok = true;
    Rd r(a.pb, off, off + L);
    while (r.more()) {
      const uint32_t a0 = r.i - off;
      uint32_t f, wt;
      if (!r.tag(f, wt)) break;
      if (f < prev_f) { ok = false; break; }   // out of order: re-marshaled by the host
      prev_f = f;
      uint32_t po = 0, pl = 0;
      if (f == 6 && wt == 0) {
        kind = (int32_t)r.varint();
      } else if (wt == 2) {
        if (!r.len(po, pl)) break;
      } else if (!r.skip(wt)) {
        break;
      }
      if (!name_set && f >= 5) {
        name_a = a0;
        name_b = f == 5 ? r.i - off : a0;
        name_set = true;
      }
      if (f == 9 && wt == 2) {
        Rd kv(a.pb, po, po + pl);
        uint32_t ko = 0, kl = 0, vo = 0, vl = 0;
        bool hv = false;
        while (kv.more()) {
          uint32_t kf, kwt;
          if (!kv.tag(kf, kwt)) break;
          if (kwt == 2 && (kf == 1 || kf == 2)) {
            uint32_t o, l;
            if (!kv.len(o, l)) break;
            if (kf == 1) ko = o, kl = l;
            else vo = o, vl = l, hv = true;
          } else {
            kv.skip(kwt);
          }
        }
        if (kv.bad) { ok = false; break; }
        if ((u & OSE_OUT_SET_ATTR) && !attr_set) {
          const bool client = kind == OSE_KIND_CLIENT;
          if (client ? eq_lit(r.br, ko, kl, "url.template", 12) : eq_lit(r.br, ko, kl, "http.route", 10)) {
            attr_a = a0;
            attr_b = r.i - off;
            attr_set = true;
          }
        }
        if (!have_new && eq_lit(r.br, ko, kl, "http.request.method", 19)) {
          have_new = true;
          new_v = hv, new_o = vo, new_l = vl;
        } else if (!have_old && eq_lit(r.br, ko, kl, "http.method", 11)) {
          have_old = true;
          old_v = hv, old_o = vo, old_l = vl;
        }
      } else if (f > 9 && !attr_set) {
        attr_a = attr_b = a0;
        attr_set = true;
      }
    }
    if (!ok || r.bad || r.i != off + L) {   // re-marshaled, or malformed (the host reports it)
      fb |= kEncFbSpan;
      continue;
    }
    const bool client = kind == OSE_KIND_CLIENT;
    if (!(u & OSE_OUT_RENAME)) name_a = name_b = 0;
    if (!(u & OSE_OUT_SET_ATTR)) attr_a = attr_b = L;
    uint64_t out = (uint64_t)L - (name_b - name_a) - (attr_b - attr_a);
    uint32_t meth_off = 0, meth_len = 0;
    if (u & OSE_OUT_RENAME) {
      const bool hv = have_new ? new_v : old_v;
      const uint32_t mo = have_new ? new_o : old_o, ml = have_new ? new_l : old_l;
      if ((have_new || have_old) && hv) {
        // an AnyValue{string_value} is used in place; anything else needs AsString
        bool direct = false;
        if (ml >= 2 && r.br.at(mo) == 0x0A) {
          Rd vr(a.pb, mo + 1, mo + ml);
          const uint64_t sl = vr.varint();
          direct = !vr.bad && vr.i + sl == mo + ml;
          if (direct) {
            meth_off = vr.i;
            meth_len = (uint32_t)sl;
          }
        }
        if (!direct) {
          fb |= kEncFbSpan;
          continue;
        }
      }
      out += field_len((uint64_t)meth_len + 1 + t.len);
    }
    if (u & OSE_OUT_SET_ATTR) out += field_len(kv_len(client, t.len));
    if (name_b > attr_a) {   // not the ascending order the plan assumes
      fb |= kEncFbSpan;
      continue;
    }
    a.edit[i] = EncEdit{name_a, name_b, attr_a, attr_b, meth_off, meth_len, t.off, t.len, (uint32_t)out,
                        u | (client ? 0x100u : 0u)};
    a.span_out[i] = (uint32_t)field_len(out);
  }
  if (fb) flag(a, fb);
}

// ---- sizing: scopes ------------------------------------------------------------
// Enc::size_chunk's scope loop: header (pdata always writes the
// InstrumentationScope, "0A 00" when empty), spans, schema_url; a scope whose
// spans were all dropped is removed.
__global__ __launch_bounds__(kERec) void enc_scope_kernel(EncArgs a) {
  const uint64_t s = (uint64_t)blockIdx.x * kERec + threadIdx.x;
  if (s >= a.n_scopes) return;
  const uint64_t i0 = a.scope_span0[s], i1 = s + 1 < a.n_scopes ? a.scope_span0[s + 1] : a.n_spans;
  const uint64_t h = a.scope_hdr[s];
  uint32_t fb = 0;
  if (h == kOtlpScopeMulti) fb |= kEncFbScope;   // merged scope fields: the host merges them
  uint64_t sb = field_len(h == kOtlpScopeMulti ? 0 : (uint32_t)(h >> 32)) + str_field((uint32_t)(a.scope_schema[s] >> 32));
  if (a.scope_size[s] != sb) fb |= kEncFbScope;   // not pdata's encoding: re-marshaled by the host
  bool kept_any = false;
  for (uint64_t i = i0; i < i1; i++) {
    const uint32_t so = a.span_out[i];
    kept_any |= so != 0;
    sb += so;
  }
  a.scope_body[s] = (i1 > i0 && !kept_any) ? kEncDropped : sb;
  if (fb) flag(a, fb);
}

// ---- sizing: resources and routing ---------------------------------------------
namespace {
constexpr uint64_t kFnvOff = 0xcbf29ce484222325ull, kFnvPrime = 0x100000001b3ull;
__device__ __forceinline__ uint64_t fnv_byte(uint64_t h, uint32_t c) { return (h ^ (c & 0xFFu)) * kFnvPrime; }

struct StrPart {
  uint32_t off, len;   // message bytes
};
__device__ const char* kind_name(uint32_t k) {   // NormalizeKind of the three kinds (routingmap.go:62-70)
  return k == 0 ? "deployment" : k == 1 ? "statefulset" : "daemonset";
}
__device__ __forceinline__ uint32_t kind_len(uint32_t k) { return k == 0 ? 10u : k == 1 ? 11u : 9u; }

// determineRoutingPipelines (connector.go:147-172) for one Resource payload
// [s, e): the pipelines mask, or 0 for the default pipeline; *bad when an
// attribute the key reads is not what the device decodes exactly
__device__ uint64_t route_resource(const EncArgs& a, uint32_t s, uint32_t e, bool* bad) {
  // first occurrence of each key (pcommon.Map.Get), its Str() ("" unless a
  // string): namespace, then deployment / statefulset / daemonset
  uint32_t seen = 0;
  StrPart ns{0, 0}, nm[3] = {{0, 0}, {0, 0}, {0, 0}};
  Rd r(a.pb, s, e);
  while (r.more()) {
    uint32_t f, wt;
    if (!r.tag(f, wt)) break;
    uint32_t po, pl;
    if (f == 1 && wt == 2) {
      if (!r.len(po, pl)) break;
      Rd kv(a.pb, po, po + pl);
      uint32_t ko = 0, kl = 0, vo = 0, vl = 0, nk = 0, nv = 0;
      while (kv.more()) {
        uint32_t kf, kwt;
        if (!kv.tag(kf, kwt)) break;
        if (kwt == 2 && (kf == 1 || kf == 2)) {
          uint32_t o, l;
          if (!kv.len(o, l)) break;
          if (kf == 1) ko = o, kl = l, nk++;
          else vo = o, vl = l, nv++;
        } else {
          kv.skip(kwt);
        }
      }
      if (kv.bad || nk > 1 || nv > 1) { *bad = true; return 0; }   // merged KeyValue fields
      uint32_t which = 4;
      if (eq_lit(r.br, ko, kl, "k8s.namespace.name", 18)) which = 0;
      else if (eq_lit(r.br, ko, kl, "k8s.deployment.name", 19)) which = 1;
      else if (eq_lit(r.br, ko, kl, "k8s.statefulset.name", 20)) which = 2;
      else if (eq_lit(r.br, ko, kl, "k8s.daemonset.name", 18)) which = 3;
      if (which < 4 && !((seen >> which) & 1)) {
        seen |= 1u << which;
        Val v;
        v.type = OSE_ATTR_OTHER;
        v.off = v.len = 0;
        if (nv) {
          any_value(kv, vo, vo + vl, v);
          if (kv.bad) { *bad = true; return 0; }
        }
        const StrPart sp = v.type == OSE_ATTR_STR ? StrPart{v.off, v.len} : StrPart{0, 0};
        if (which == 0) ns = sp;
        else if (which == 1) nm[0] = sp;
        else if (which == 2) nm[1] = sp;
        else nm[2] = sp;
      }
    } else if (!r.skip(wt)) {
      break;
    }
  }
  if (r.bad) { *bad = true; return 0; }
  if (!(seen & 1)) return 0;
  // the first of deployment, statefulset, daemonset present (Router::route)
  const uint32_t kn = (seen & 2) ? 0u : (seen & 4) ? 1u : (seen & 8) ? 2u : 3u;
  if (kn == 3) return 0;
  const StrPart name = kn == 0 ? nm[0] : kn == 1 ? nm[1] : nm[2];
  if (name.len == 0) return 0;   // name empty: default
  const char* kname = kind_name(kn);
  const uint32_t kl = kind_len(kn);
  // "ns/kind/name"
  uint64_t h = kFnvOff;
  for (uint32_t q = 0; q < ns.len; q++) h = fnv_byte(h, r.br.at(ns.off + q));
  h = fnv_byte(h, '/');
  for (uint32_t q = 0; q < kl; q++) h = fnv_byte(h, (uint8_t)kname[q]);
  h = fnv_byte(h, '/');
  for (uint32_t q = 0; q < name.len; q++) h = fnv_byte(h, r.br.at(name.off + q));
  const uint32_t total = ns.len + 1 + kl + 1 + name.len;
  const uint32_t mask = (1u << a.route_bits) - 1u;
  for (uint32_t slot = (uint32_t)h & mask, probes = 0; probes <= mask; slot = (slot + 1) & mask, probes++) {
    const EncRouteSlot rs = a.routes[slot];
    if (rs.klen == ~0u) return 0;
    if (rs.h != h || rs.klen != total) continue;
    const uint8_t* key = a.route_keys + rs.koff;
    bool same = true;
    uint32_t p = 0;
    for (uint32_t q = 0; q < ns.len && same; q++) same = key[p++] == r.br.at(ns.off + q);
    same = same && key[p++] == '/';
    for (uint32_t q = 0; q < kl && same; q++) same = key[p++] == (uint8_t)kname[q];
    same = same && key[p++] == '/';
    for (uint32_t q = 0; q < name.len && same; q++) same = key[p++] == r.br.at(name.off + q);
    if (same) return rs.mask;
  }
  return 0;
}
}  // namespace

// Enc::size_chunk's resource loop, and its outputs (Enc::outputs_of)
__global__ __launch_bounds__(kERec) void enc_res_kernel(EncArgs a) {
  const uint64_t rr = (uint64_t)blockIdx.x * kERec + threadIdx.x;
  if (rr >= a.n_res) return;
  const uint64_t ref = a.res_ref[rr];
  const uint32_t ro = (uint32_t)ref, rl = (uint32_t)(ref >> 32);
  uint32_t fb = 0, nres = 0, hs = 0, hl = 0;
  uint64_t schema = 0;
  {
    Rd p(a.pb, ro, ro + rl);
    while (p.more()) {
      uint32_t f, wt;
      if (!p.tag(f, wt)) break;
      if (wt == 2 && (f == 1 || f == 2 || f == 3 || f == 1000)) {
        uint32_t o, l;
        if (!p.len(o, l)) break;
        if (f == 1) nres++, hs = o, hl = l;
        else if (f == 3) schema = (uint64_t)o | ((uint64_t)l << 32);
      } else {
        p.skip(wt);
      }
    }
    if (p.bad) fb |= kEncFbRes;
  }
  if (nres > 1) fb |= kEncFbRes;   // merged Resource fields
  uint64_t body = field_len(hl) + str_field((uint32_t)(schema >> 32));
  if (a.res_size[rr] != body) fb |= kEncFbRes;   // not pdata's encoding: re-marshaled by the host
  const uint64_t s0 = a.res_scope0[rr], s1 = rr + 1 < a.n_res ? a.res_scope0[rr + 1] : a.n_scopes;
  bool had = false, any = false;
  for (uint64_t s = s0; s < s1; s++) {
    const uint64_t i0 = a.scope_span0[s], i1 = s + 1 < a.n_scopes ? a.scope_span0[s + 1] : a.n_spans;
    had |= i1 > i0;
    const uint64_t sb = a.scope_body[s];
    if (sb == kEncDropped) continue;
    body += field_len(sb);
    any = true;
  }
  const bool dropped = had && !any;   // emptied by sampling: removed
  a.res_body[rr] = dropped ? kEncDropped : body;
  a.res_rec[rr] = dropped ? 0 : field_len(body);
  a.res_hdr[rr] = nres ? ((uint64_t)hs | ((uint64_t)hl << 32)) : kEncNoHdr;
  a.res_schema[rr] = schema;
  uint64_t mask = 1;
  if (a.route_bits) {
    bool bad = false;
    const uint64_t m = nres ? route_resource(a, hs, hs + hl, &bad) : 0;
    if (bad) fb |= kEncFbRoute;
    mask = m ? m : 1ull << (a.n_out - 1);
  }
  a.res_mask[rr] = mask;
  if (fb) flag(a, fb);
}

// ---- offsets: an exclusive scan per output ------------------------------------
namespace {
// exclusive prefix over a 256-thread block (x per thread); *total gets the sum
__device__ uint64_t block_excl_u64(uint64_t x, uint64_t* total) {
  __shared__ uint64_t wsum[kEThreads / kWave];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (int w = 0; w < kEThreads / kWave; w++) {
    const uint64_t v = wsum[w];
    if (w < wv) before += v;
    all += v;
  }
  __syncthreads();
  *total = all;
  return before + incl - x;
}
__device__ __forceinline__ uint64_t rec_for(const EncArgs& a, uint64_t r, uint32_t k) {
  return r < a.n_res && ((a.res_mask[r] >> k) & 1) ? a.res_rec[r] : 0;
}
constexpr uint32_t kPer = kEncTiles / kEThreads;   // resources per thread in a tile
}  // namespace

// tile sums: bytes and records per (output, tile)
__global__ __launch_bounds__(kEThreads) void enc_scan_tiles_kernel(EncArgs a, uint32_t tiles) {
  const uint32_t t = blockIdx.x, k = blockIdx.y;
  uint64_t bytes = 0, cnt = 0;
  for (uint32_t q = 0; q < kPer; q++) {
    const uint64_t r = (uint64_t)t * kEncTiles + threadIdx.x * kPer + q;
    const uint64_t v = rec_for(a, r, k);
    bytes += v;
    cnt += v != 0;
  }
  uint64_t tb, tc;
  block_excl_u64(bytes, &tb);
  block_excl_u64(cnt, &tc);
  if (threadIdx.x == 0) {
    a.tile_sum[(uint64_t)k * tiles + t] = tb;
    a.tile_sum[(uint64_t)(a.n_out + k) * tiles + t] = tc;
  }
}
// one block per output: the tiles' exclusive prefix, and the output's totals
__global__ __launch_bounds__(kEThreads) void enc_scan_top_kernel(EncArgs a, uint32_t tiles) {
  const uint32_t k = blockIdx.x;
  uint64_t* ts = a.tile_sum + (uint64_t)k * tiles;
  const uint64_t* tc = a.tile_sum + (uint64_t)(a.n_out + k) * tiles;
  uint64_t carry = 0, count = 0;
  for (uint32_t t0 = 0; t0 < tiles; t0 += kEThreads) {
    const uint32_t t = t0 + threadIdx.x;
    const uint64_t v = t < tiles ? ts[t] : 0;
    uint64_t tot, ctot;
    const uint64_t ex = block_excl_u64(v, &tot);
    block_excl_u64(t < tiles ? tc[t] : 0, &ctot);
    if (t < tiles) ts[t] = carry + ex;
    carry += tot;
    count += ctot;
  }
  if (threadIdx.x == 0) {
    a.out_total[k] = carry;
    a.out_total[a.n_out + k] = count;
  }
}
__global__ __launch_bounds__(kEThreads) void enc_scan_apply_kernel(EncArgs a, uint32_t tiles) {
  const uint32_t t = blockIdx.x, k = blockIdx.y;
  uint64_t v[kPer], sum = 0;
  for (uint32_t q = 0; q < kPer; q++) {
    v[q] = rec_for(a, (uint64_t)t * kEncTiles + threadIdx.x * kPer + q, k);
    sum += v[q];
  }
  uint64_t tot;
  uint64_t run = a.tile_sum[(uint64_t)k * tiles + t] + block_excl_u64(sum, &tot);
  for (uint32_t q = 0; q < kPer; q++) {
    const uint64_t r = (uint64_t)t * kEncTiles + threadIdx.x * kPer + q;
    if (r < a.n_res) a.off[(uint64_t)k * a.n_res + r] = run;
    run += v[q];
  }
}

// ---- writing -----------------------------------------------------------------------
namespace {
// wave-cooperative writer of one record (positions are wave-uniform)
// Every store is checked against the record's size from the sizing pass
// (lim): a disagreement is a bug, flagged (kEncFbWrite) instead of written
// past the record.
struct WaveOut {
  uint8_t* dst;
  uint64_t pos, lim;
  int lane;
  __device__ __forceinline__ void put(uint64_t at, uint32_t b) {
    if (at < lim) dst[at] = (uint8_t)b;
  }
  // tag and varint v
  __device__ __forceinline__ void hdr(uint32_t tag, uint64_t v) {
    const uint32_t nb = 1 + sov(v);
    if ((uint32_t)lane < nb) {
      const uint32_t b = lane == 0 ? tag : (uint32_t)((v >> (7 * (lane - 1))) & 0x7F) | ((uint32_t)lane + 1 < nb ? 0x80u : 0u);
      put(pos + lane, b);
    }
    pos += nb;
  }
  __device__ __forceinline__ void byte(uint32_t c) {
    if (lane == 0) put(pos, c);
    pos += 1;
  }
  __device__ __forceinline__ void copy(const uint8_t* src, uint64_t n) {
    for (uint64_t x = (uint64_t)lane; x < n; x += kWave) put(pos + x, src[x]);
    pos += n;
  }
  __device__ __forceinline__ void lit(const char* s, uint32_t n) {
    if ((uint32_t)lane < n) put(pos + lane, (uint8_t)s[lane]);
    pos += n;
  }
};
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ uint32_t uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t lane32(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }

// Enc::write_edit
__device__ void write_edit(const EncArgs& a, WaveOut& w, const uint8_t* sp, uint32_t L, const EncEdit& e) {
  const uint32_t u = e.flags & 0xFFu;
  const bool client = (e.flags >> 8) & 1u;
  const uint8_t* T = a.tmpl_arena + e.tmpl_off;
  w.copy(sp, e.name_a);
  if (u & OSE_OUT_RENAME) {
    w.hdr(0x2A, (uint64_t)e.meth_len + 1 + e.tmpl_len);
    w.copy(a.pb + e.meth_off, e.meth_len);
    w.byte(' ');
    w.copy(T, e.tmpl_len);
  }
  w.copy(sp + e.name_b, e.attr_a - e.name_b);
  if (u & OSE_OUT_SET_ATTR) {
    const uint32_t kl = client ? 12 : 10;
    w.hdr(0x4A, kv_len(client, e.tmpl_len));
    w.hdr(0x0A, kl);
    w.lit(client ? "url.template" : "http.route", kl);
    w.hdr(0x12, field_len(e.tmpl_len));
    w.hdr(0x0A, e.tmpl_len);
    w.copy(T, e.tmpl_len);
  }
  w.copy(sp + e.attr_b, L - e.attr_b);
}

// the record of resource r at dst (Enc::write_chunk)
__device__ void write_record(const EncArgs& a, uint64_t r, uint8_t* dst, uint64_t rec) {
  WaveOut w{dst, 0, rec, (int)(threadIdx.x & 63)};
  w.hdr(0x0A, uni64(a.res_body[r]));
  const uint64_t h = uni64(a.res_hdr[r]);
  if (h == kEncNoHdr) {
    w.hdr(0x0A, 0);
  } else {
    w.hdr(0x0A, h >> 32);
    w.copy(a.pb + (uint32_t)h, h >> 32);
  }
  const uint64_t s0 = uni32(a.res_scope0[r]), s1 = r + 1 < a.n_res ? uni32(a.res_scope0[r + 1]) : a.n_scopes;
  for (uint64_t s = s0; s < s1; s++) {
    const uint64_t sb = uni64(a.scope_body[s]);
    if (sb == kEncDropped) continue;
    w.hdr(0x12, sb);
    const uint64_t sh = uni64(a.scope_hdr[s]);
    w.hdr(0x0A, sh >> 32);
    if (sh >> 32) w.copy(a.pb + (uint32_t)sh, sh >> 32);
    const uint64_t i0 = uni32(a.scope_span0[s]), i1 = s + 1 < a.n_scopes ? uni32(a.scope_span0[s + 1]) : a.n_spans;
    for (uint64_t c = i0; c < i1; c += kWave) {
      const uint64_t j = c + (uint64_t)w.lane;
      uint32_t so = 0, roff = 0, rlen = 0, u = 0;
      if (j < i1) {
        so = a.span_out[j];
        const uint64_t ref = a.span_ref[j];
        roff = (uint32_t)ref;
        rlen = (uint32_t)(ref >> 32);
        u = a.url_out ? a.url_out[j] : 0u;
      }
      uint64_t kept = __ballot(so != 0);
      while (kept) {
        const int b = __builtin_ctzll(kept);
        kept &= kept - 1;
        const uint32_t off = lane32(roff, b), L = lane32(rlen, b);
        if (lane32(u, b) == 0) {
          w.hdr(0x12, L);
          w.copy(a.pb + off, L);
        } else {
          const EncEdit* ep = a.edit + c + (uint64_t)b;
          EncEdit e;
          e.name_a = uni32(ep->name_a);
          e.name_b = uni32(ep->name_b);
          e.attr_a = uni32(ep->attr_a);
          e.attr_b = uni32(ep->attr_b);
          e.meth_off = uni32(ep->meth_off);
          e.meth_len = uni32(ep->meth_len);
          e.tmpl_off = uni32(ep->tmpl_off);
          e.tmpl_len = uni32(ep->tmpl_len);
          e.out_len = uni32(ep->out_len);
          e.flags = uni32(ep->flags);
          w.hdr(0x12, e.out_len);
          write_edit(a, w, a.pb + off, L, e);
        }
      }
    }
    const uint64_t sch = uni64(a.scope_schema[s]);
    if (sch >> 32) {
      w.hdr(0x1A, sch >> 32);
      w.copy(a.pb + (uint32_t)sch, sch >> 32);
    }
  }
  const uint64_t rs = uni64(a.res_schema[r]);
  if (rs >> 32) {
    w.hdr(0x1A, rs >> 32);
    w.copy(a.pb + (uint32_t)rs, rs >> 32);
  }
  if (w.pos != rec && w.lane == 0) atomicOr(a.flags, (uint32_t)kEncFbWrite);
}
}  // namespace

// a wave per resource (grid-stride), its record to every output it routes to
__global__ __launch_bounds__(kERec) void enc_write_kernel(EncArgs a) {
  const uint64_t waves = (uint64_t)gridDim.x * (kERec / kWave);
  for (uint64_t r = uni64((uint64_t)blockIdx.x * (kERec / kWave) + (threadIdx.x >> 6)); r < a.n_res; r += waves) {
    const uint64_t rec = uni64(a.res_rec[r]);
    if (rec == 0) continue;
    uint64_t mask = uni64(a.res_mask[r]);
    while (mask) {
      const uint32_t k = (uint32_t)__builtin_ctzll(mask);
      mask &= mask - 1;
      write_record(a, r, a.out + a.out_base[k] + uni64(a.off[(uint64_t)k * a.n_res + r]), rec);
    }
  }
}

// ---- launchers ---------------------------------------------------------------------
namespace {
// blocks of kERec threads for n threads' work, at most cap x (kEThreads / kERec) (the
// same resident thread count whatever the block size)
inline uint32_t grid_of(uint64_t n, uint32_t cap) {
  const uint64_t c = cap == ~0u ? cap : (uint64_t)cap * (kEThreads / kERec);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + kERec - 1) / kERec, c));
}
}  // namespace
void launch_enc_spans(const EncArgs& a, hipStream_t st) {
  if (a.n_spans) hipLaunchKernelGGL(enc_span_kernel, dim3(grid_of(a.n_spans, 8192)), dim3(kERec), 0, st, a);
}
void launch_enc_scopes(const EncArgs& a, hipStream_t st) {
  if (a.n_scopes) hipLaunchKernelGGL(enc_scope_kernel, dim3(grid_of(a.n_scopes, ~0u)), dim3(kERec), 0, st, a);
}
void launch_enc_resources(const EncArgs& a, hipStream_t st) {
  if (a.n_res) hipLaunchKernelGGL(enc_res_kernel, dim3(grid_of(a.n_res, ~0u)), dim3(kERec), 0, st, a);
}
void launch_enc_scan(const EncArgs& a, hipStream_t st) {
  const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (a.n_res + kEncTiles - 1) / kEncTiles);
  hipLaunchKernelGGL(enc_scan_tiles_kernel, dim3(tiles, a.n_out), dim3(kEThreads), 0, st, a, tiles);
  hipLaunchKernelGGL(enc_scan_top_kernel, dim3(a.n_out), dim3(kEThreads), 0, st, a, tiles);
  hipLaunchKernelGGL(enc_scan_apply_kernel, dim3(tiles, a.n_out), dim3(kEThreads), 0, st, a, tiles);
}
void launch_enc_write(const EncArgs& a, hipStream_t st) {
  if (a.n_res) hipLaunchKernelGGL(enc_write_kernel, dim3(grid_of(a.n_res * kWave, 16384)), dim3(kERec), 0, st, a);
}

}  // namespace ose
