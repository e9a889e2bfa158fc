// otlp_encode.cpp — the gateway's output side: the
// decisions the GPU made on a decoded OTLP batch (keep, url_out + template)
// applied to the message bytes, the resources routed to the data-stream
// pipelines as odigosrouterconnector does, and one serialized TracesData
// written per pipeline — what the exporters behind each pipeline marshal.
//
// Output bytes equal pdata's marshaler (ptrace.ProtoMarshaler, gogo-style:
// ProtoWriter in pdata.cpp) applied to the processed traces:
//   * a span whose encoding already has pdata's size (span_size, computed
//     by the decoder) and no change is copied verbatim;
//   * a renamed / templated span of that kind is edited in place: the name
//     field replaced or inserted, the target attribute's KeyValue replaced
//     (Map.PutStr on an existing key) or appended after the last attribute;
//   * any other span (an encoding pdata would not write: unknown fields,
//     unframed empty ids, non-minimal varints) is decoded and re-marshaled.
// Resource and scope headers are re-marshaled from their decoded form
// (cached by message bytes).  Resources are split over threads by span
// count; a first pass sizes every record (and writes the edited spans to a
// side buffer), a second writes each output at its final offsets.
#include "otlp_encode.hpp"

#include <strings.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string_view>
#include <thread>

#include "engine_internal.hpp"
#include "kernels.hpp"
#include "otlp_pb.hpp"
#include "taskpool.hpp"

namespace ose {

// ---- odigosrouterconnector ------------------------------------------------

std::string normalize_kind(const std::string& kind) {   // routingmap.go:62-70
  std::string low = kind;
  for (char& ch : low) ch = (char)std::tolower((unsigned char)ch);
  if (low == "deployment" || low == "statefulset" || low == "daemonset" || low == "cronjob" ||
      low == "deploymentconfig")
    return low;
  return kind;
}

namespace {
// mapstructure matches keys case-insensitively
const Json* ci_get(const Json& o, const char* key) {
  if (!o.is_obj()) return nullptr;
  for (auto& kv : o.obj)
    if (strcasecmp(kv.first.c_str(), key) == 0) return &kv.second;
  return nullptr;
}
std::string ci_str(const Json& o, const char* key) {
  const Json* v = ci_get(o, key);
  return v && v->is_str() ? v->s : std::string();
}
}  // namespace

void build_route_blob(Router& r);

std::string build_router(const Json& cfg, const std::string& signal, Router& r) {
  r = Router{};
  r.signal = signal;
  const Json* ds = ci_get(cfg, "datastreams");
  if (!ds || ds->is_null()) return "";
  if (!ds->is_arr()) return "datastreams: expected a list";
  for (const Json& d : ds->arr) {
    if (!d.is_obj()) return "datastreams: expected a map";
    const std::string name = ci_str(d, "name");
    // GetSignalsForDataStream (routingmap.go:84-103): the first three
    // distinct signals over the destinations
    std::vector<std::string> sigs;
    if (const Json* dests = ci_get(d, "destinations"); dests && dests->is_arr()) {
      for (const Json& de : dests->arr) {
        const Json* cs = ci_get(de, "configuredsignals");
        if (!cs || !cs->is_arr()) continue;
        bool full = false;
        for (const Json& s : cs->arr) {
          const std::string sig = s.is_str() ? s.s : std::string();
          if (std::find(sigs.begin(), sigs.end(), sig) == sigs.end()) sigs.push_back(sig);
          if (sigs.size() == 3) { full = true; break; }
        }
        if (full) break;
      }
    }
    if (std::find(sigs.begin(), sigs.end(), signal) == sigs.end()) continue;
    uint32_t pid;
    auto it = std::find(r.pipelines.begin(), r.pipelines.end(), name);
    if (it == r.pipelines.end()) {
      pid = (uint32_t)r.pipelines.size();
      r.pipelines.push_back(name);
    } else {
      pid = (uint32_t)(it - r.pipelines.begin());
    }
    if (const Json* srcs = ci_get(d, "sources"); srcs && srcs->is_arr()) {
      for (const Json& s : srcs->arr) {
        // routingmap.go:41: fmt.Sprintf("%s/%s/%s", ns, NormalizeKind(kind), name)
        const std::string key = ci_str(s, "namespace") + "/" + normalize_kind(ci_str(s, "kind")) + "/" +
                                ci_str(s, "name");
        auto& v = r.routes[key];
        if (std::find(v.begin(), v.end(), pid) == v.end()) v.push_back(pid);   // appendIfMissing
      }
    }
  }
  build_route_blob(r);
  return "";
}

// Router::dev_blob (encode_kernel.hip route_resource)
void build_route_blob(Router& r) {
  r.dev_blob.clear();
  r.route_bits = 0;
  r.dev_slots_bytes = 0;
  if (r.pipelines.size() > 63) return;   // the encoders refuse such a router
  uint32_t bits = 1;
  while ((size_t(1) << bits) < 2 * r.routes.size() + 2) bits++;
  const size_t slots = size_t(1) << bits;
  std::vector<EncRouteSlot> tab(slots, EncRouteSlot{0, 0, ~0u, 0});
  std::string keys;
  for (auto& kv : r.routes) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (unsigned char c : kv.first) h = (h ^ c) * 0x100000001b3ull;
    uint64_t mask = 0;
    for (uint32_t p : kv.second) mask |= 1ull << p;
    size_t s = (size_t)h & (slots - 1);
    while (tab[s].klen != ~0u) s = (s + 1) & (slots - 1);
    tab[s] = EncRouteSlot{h, (uint32_t)keys.size(), (uint32_t)kv.first.size(), mask};
    keys += kv.first;
  }
  r.route_bits = bits;
  r.dev_slots_bytes = slots * sizeof(EncRouteSlot);
  r.dev_blob.resize(r.dev_slots_bytes + keys.size() + 16, 0);
  std::memcpy(r.dev_blob.data(), tab.data(), r.dev_slots_bytes);
  std::memcpy(r.dev_blob.data() + r.dev_slots_bytes, keys.data(), keys.size());
}

const std::vector<uint32_t>* Router::route(const AttrMap& attrs, std::string* key) const {
  // connector.go:147-172.  getDynamicNameAndKind ranges over a Go map (a
  // random order); the first of deployment, statefulset, daemonset present
  // is taken here, which is the same whenever a resource carries one.
  const Value* ns = attrs.Get("k8s.namespace.name");
  if (!ns) return nullptr;
  static const char* const kKeys[3][2] = {{"k8s.deployment.name", "Deployment"},
                                          {"k8s.statefulset.name", "StatefulSet"},
                                          {"k8s.daemonset.name", "DaemonSet"}};
  std::string name, kind;
  for (auto& kk : kKeys)
    if (const Value* v = attrs.Get(kk[0])) {
      name = v->Str();
      kind = kk[1];
      break;
    }
  if (name.empty() || kind.empty()) return nullptr;
  std::string k = ns->Str() + "/" + normalize_kind(kind) + "/" + name;
  auto it = routes.find(k);
  if (it == routes.end()) return nullptr;
  if (key) *key = std::move(k);
  return &it->second;
}

// ---- the encoder ------------------------------------------------------------

namespace enc {
constexpr uint64_t kDropped = ~0ull;

inline uint32_t sov64(uint64_t x) { uint32_t n = 1; while (x >= 0x80) { x >>= 7; n++; } return n; }
inline uint64_t flen(uint64_t l) { return 1 + sov64(l) + l; }   // tag < 16
inline uint8_t* put_varint(uint8_t* w, uint64_t v) {
  while (v >= 0x80) { *w++ = (uint8_t)(v | 0x80); v >>= 7; }
  *w++ = (uint8_t)v;
  return w;
}
inline uint8_t* put_rec(uint8_t* w, uint8_t tag, const void* p, uint64_t n) {
  *w++ = tag;
  w = put_varint(w, n);
  std::memcpy(w, p, n);
  return w + n;
}

struct ResHdr {
  std::string bytes;                          // the Resource field, framed (always written)
  const std::vector<uint32_t>* route = nullptr;
  bool routed = false;                        // route found (else default)
};

// One rewritten span: the source with the name field and the target
// KeyValue replaced (a < b) or inserted (a == b) — or, in_mods, bytes
// re-marshaled into Chunk::mods at name_a.
struct Edit {
  uint32_t name_a, name_b, attr_a, attr_b;
  uint32_t meth_off, meth_len;   // the method string (in the message, or in mods)
  uint32_t tmpl_off, tmpl_len;   // the template (in the template arena)
  uint32_t out_len;
  uint8_t u, client, in_mods, meth_in_mods;
};

struct Chunk {
  size_t r0 = 0, r1 = 0;
  std::unordered_map<std::string_view, ResHdr> rcache;
  std::unordered_map<std::string_view, std::string> scache;
  std::deque<ResHdr> rown;          // merged headers (several Resource fields)
  std::deque<std::string> sown;
  std::vector<Edit> edits;          // one per rewritten span, in order
  std::string mods;                 // re-marshaled spans, AsString methods
  std::vector<uint64_t> out_bytes, out_res, cursor;
  std::string err;
};

struct Enc {
  const uint8_t* pb;
  size_t len;
  const std::vector<uint64_t>& span_ref;
  const OtlpLayout& lay;
  const EncodeDecisions& d;
  const Router* router;
  uint64_t n, R, S;
  uint32_t n_out;
  // per resource / scope results of pass 1 (the workspace's)
  std::vector<uint64_t>& res_body;
  std::vector<uint64_t>& res_schema;
  std::vector<const ResHdr*>& res_hdr;
  std::vector<uint64_t>& scope_body;
  std::vector<const std::string*>& scope_hdr;

  uint64_t scope_end(uint64_t s) const { return s + 1 < S ? lay.scope_span0[s + 1] : n; }
  uint64_t res_scope_end(uint64_t r) const { return r + 1 < R ? lay.res_scope0[r + 1] : S; }
  uint64_t res_span0(uint64_t r) const {
    const uint64_t s = lay.res_scope0[r];
    return s < S ? lay.scope_span0[s] : n;
  }
  bool kept(uint64_t i) const { return !d.keep || d.keep[i]; }
  bool rewritten(uint64_t i) const {
    return (d.url_out && d.url_out[i]) || (d.span_size && d.span_size[i] != (uint32_t)(span_ref[i] >> 32));
  }
  void outputs_of(const ResHdr* h, uint32_t* ks, uint32_t& nk) const {
    nk = 0;
    if (!router) { ks[nk++] = 0; return; }
    if (!h->routed) { ks[nk++] = n_out - 1; return; }
    for (uint32_t k : *h->route) ks[nk++] = k;
  }

  const ResHdr* resource_header(Chunk& c, const std::vector<std::pair<size_t, size_t>>& rf) {
    std::string_view key;
    if (rf.size() == 1) key = std::string_view((const char*)pb + rf[0].first, rf[0].second);
    if (rf.size() <= 1) {
      auto it = c.rcache.find(key);
      if (it != c.rcache.end()) return &it->second;
    }
    AttrMap attrs;
    uint32_t dropped = 0;
    for (auto& x : rf)
      if (!pb_resource(pb + x.first, x.second, attrs, dropped)) { c.err = "OTLP protobuf: malformed Resource"; return nullptr; }
    ResHdr h;
    std::string body;
    ProtoWriter(body).resource(attrs, dropped);
    ProtoWriter w(h.bytes);
    w.bytes(1, body.data(), body.size());
    if (router) {
      h.route = router->route(attrs);
      h.routed = h.route != nullptr;
    }
    if (rf.size() <= 1) return &c.rcache.emplace(key, std::move(h)).first->second;
    c.rown.push_back(std::move(h));
    return &c.rown.back();
  }

  const std::string* scope_header(Chunk& c, uint64_t s) {
    const uint64_t ref = lay.scope_hdr[s];
    ScopeSpans meta;
    std::string_view key;
    if (ref != OtlpLayout::kMulti) {
      key = std::string_view((const char*)pb + (uint32_t)ref, (size_t)(ref >> 32));
      auto it = c.scache.find(key);
      if (it != c.scache.end()) return &it->second;
      if (!pb_scope(pb + (uint32_t)ref, (size_t)(ref >> 32), meta)) { c.err = "OTLP protobuf: malformed InstrumentationScope"; return nullptr; }
    } else {
      const uint64_t sr = lay.scope_ref[s];
      PbReader r(pb + (uint32_t)sr, (size_t)(sr >> 32));
      uint32_t f, wt;
      while (r.more() && r.tag(f, wt)) {
        size_t o, l;
        if (f == 1 && wt == 2 && r.bytes(o, l)) {
          if (!pb_scope(pb + (uint32_t)sr + o, l, meta)) { c.err = "OTLP protobuf: malformed InstrumentationScope"; return nullptr; }
        } else if (f != 1) {
          r.skip(wt, f);
        } else {
          r.fail();
        }
      }
      if (!r.ok) { c.err = "OTLP protobuf: malformed ScopeSpans"; return nullptr; }
    }
    std::string body, out;
    ProtoWriter(body).scope(meta);
    ProtoWriter(out).bytes(1, body.data(), body.size());   // non-nullable: always written
    if (ref != OtlpLayout::kMulti) return &c.scache.emplace(key, std::move(out)).first->second;
    c.sown.push_back(std::move(out));
    return &c.sown.back();
  }

  // The processed span i: an edit plan (or bytes in c.mods) appended to
  // c.edits; false on a malformed span.
  bool rewrite(Chunk& c, uint64_t i) {
    const uint8_t* sp = pb + (uint32_t)span_ref[i];
    const size_t L = (size_t)(span_ref[i] >> 32);
    const uint8_t u = d.url_out ? d.url_out[i] : 0;
    std::string_view T;
    if (u) {
      const ose_strref t = d.tmpl[i];
      if ((uint64_t)t.off + t.len > d.tmpl_arena_len) { c.err = "template reference beyond the template arena"; return false; }
      T = std::string_view((const char*)d.tmpl_arena + t.off, t.len);
    }
    const bool canonical = !d.span_size || d.span_size[i] == (uint32_t)L;
    if (canonical) {
      int rc = plan_edit(c, sp, L, u, T);
      if (rc < 0) return false;
      if (rc > 0) return true;
    }
    return remarshal(c, sp, L, u, T);
  }

  // host.cpp Apply (processor.go:230-232, 259) on the decoded span, written to c.mods
  bool remarshal(Chunk& c, const uint8_t* sp, size_t L, uint8_t u, std::string_view T) {
    Span s;
    if (!pb_span(sp, L, s)) { c.err = "OTLP protobuf: malformed Span"; return false; }
    if (u) {
      const std::string tmpl(T);
      if (u & OSE_OUT_SET_ATTR) s.attrs.PutStr(s.kind == OSE_KIND_CLIENT ? "url.template" : "http.route", tmpl);
      if (u & OSE_OUT_RENAME) {
        const Value* m = s.attrs.Get("http.request.method");
        if (!m) m = s.attrs.Get("http.method");
        s.name = (m ? m->AsString() : std::string()) + " " + tmpl;
      }
    }
    const size_t start = c.mods.size();
    ProtoWriter(c.mods).span(s);
    Edit e{};
    e.in_mods = 1;
    e.name_a = (uint32_t)start;
    e.out_len = (uint32_t)(c.mods.size() - start);
    c.edits.push_back(e);
    return true;
  }

  // The same change on bytes already in pdata's encoding, as a plan: fields
  // ascend, so the new name takes field 5's place (or goes before the first
  // later field) and the target KeyValue replaces the first one with its key
  // (Map.PutStr) or goes after the last attribute.  1 = planned, 0 = the
  // fields are out of order (re-marshal), -1 = malformed.
  int plan_edit(Chunk& c, const uint8_t* sp, size_t L, uint8_t u, std::string_view T) {
    Edit e{};
    e.u = u;
    e.name_a = e.name_b = (uint32_t)L;
    e.attr_a = e.attr_b = (uint32_t)L;
    e.tmpl_off = (uint32_t)(T.data() - (const char*)d.tmpl_arena);
    e.tmpl_len = (uint32_t)T.size();
    int32_t kind = 0;
    bool name_set = false, attr_set = false, have_new = false, have_old = false;
    const uint8_t* mnew = nullptr; size_t mnew_len = 0;
    const uint8_t* mold = nullptr; size_t mold_len = 0;
    uint32_t prev_f = 0;
    PbReader r(sp, L);
    uint32_t f, wt;
    while (r.more()) {
      const size_t a = r.i;
      if (!r.tag(f, wt)) break;
      if (f < prev_f) return 0;
      prev_f = f;
      size_t po = 0, pl = 0;
      if (f == 6 && wt == 0) {
        kind = (int32_t)r.varint();
      } else if (wt == 2) {
        if (!r.bytes(po, pl)) break;
      } else if (!r.skip(wt, f)) {
        break;
      }
      if (!name_set && f >= 5) {   // the name's place
        e.name_a = (uint32_t)a;
        e.name_b = f == 5 ? (uint32_t)r.i : (uint32_t)a;
        name_set = true;
      }
      if (f == 9 && wt == 2) {
        // KeyValue: key (field 1), value (field 2)
        PbReader kv(sp + po, pl);
        uint32_t kf, kwt;
        size_t ko = 0, kl = 0, vo = 0, vl = 0;
        bool hv = false;
        while (kv.more() && kv.tag(kf, kwt)) {
          size_t o, l;
          if (kwt == 2 && (kf == 1 || kf == 2)) {
            if (!kv.bytes(o, l)) break;
            if (kf == 1) ko = o, kl = l;
            else vo = o, vl = l, hv = true;
          } else {
            kv.skip(kwt, kf);
          }
        }
        const char* key = (const char*)sp + po + ko;
        if ((u & OSE_OUT_SET_ATTR) && !attr_set) {
          const bool client = kind == OSE_KIND_CLIENT;
          if (client ? (kl == 12 && std::memcmp(key, "url.template", 12) == 0)
                     : (kl == 10 && std::memcmp(key, "http.route", 10) == 0)) {
            e.attr_a = (uint32_t)a;
            e.attr_b = (uint32_t)r.i;
            attr_set = true;
          }
        }
        if (!have_new && kl == 19 && std::memcmp(key, "http.request.method", 19) == 0) {
          have_new = true;
          mnew = hv ? sp + po + vo : nullptr, mnew_len = hv ? vl : 0;
        } else if (!have_old && kl == 11 && std::memcmp(key, "http.method", 11) == 0) {
          have_old = true;
          mold = hv ? sp + po + vo : nullptr, mold_len = hv ? vl : 0;
        }
      } else if (f > 9 && !attr_set) {   // after the last attribute
        e.attr_a = e.attr_b = (uint32_t)a;
        attr_set = true;
      }
    }
    if (!r.ok || r.i != L) { c.err = "OTLP protobuf: malformed Span"; return -1; }
    e.client = kind == OSE_KIND_CLIENT;
    if (!(u & OSE_OUT_RENAME)) e.name_a = e.name_b = 0;
    if (!(u & OSE_OUT_SET_ATTR)) e.attr_a = e.attr_b = (uint32_t)L;
    uint64_t out = L - (e.name_b - e.name_a) - (e.attr_b - e.attr_a);
    if (u & OSE_OUT_RENAME) {
      // the method: AnyValue{string_value} in place; anything else through pdata's AsString
      const uint8_t* mv = have_new ? mnew : mold;
      const size_t ml = have_new ? mnew_len : mold_len;
      e.meth_len = 0;
      if (have_new || have_old) {
        bool direct = false;
        if (mv && ml >= 2 && mv[0] == 0x0A) {
          PbReader vr(mv, ml);
          vr.i = 1;
          const uint64_t sl = vr.varint();
          direct = vr.ok && vr.i + sl == ml;
          if (direct) {
            e.meth_off = (uint32_t)(mv + vr.i - pb);
            e.meth_len = (uint32_t)sl;
          }
        }
        if (!direct) {
          Value v;
          if (mv && !pb_any_value(mv, ml, v)) { c.err = "OTLP protobuf: malformed AnyValue"; return -1; }
          const std::string m = v.AsString();
          e.meth_in_mods = 1;
          e.meth_off = (uint32_t)c.mods.size();
          e.meth_len = (uint32_t)m.size();
          c.mods += m;
        }
      }
      out += flen((uint64_t)e.meth_len + 1 + T.size());
    }
    if (u & OSE_OUT_SET_ATTR) out += flen(kv_len(e.client, T.size()));
    if (e.name_b > e.attr_a) return 0;   // not the ascending order the plan assumes
    e.out_len = (uint32_t)out;
    c.edits.push_back(e);
    return 1;
  }
  static uint64_t kv_len(bool client, size_t tl) {   // KeyValue{key, AnyValue{string_value}}
    return flen(client ? 12 : 10) + flen(flen(tl));
  }

  // an edited span's bytes at w
  uint8_t* write_edit(const Chunk& c, const Edit& e, const uint8_t* sp, size_t L, uint8_t* w) const {
    if (e.in_mods) {
      std::memcpy(w, c.mods.data() + e.name_a, e.out_len);
      return w + e.out_len;
    }
    const char* T = (const char*)d.tmpl_arena + e.tmpl_off;
    std::memcpy(w, sp, e.name_a);
    w += e.name_a;
    if (e.u & OSE_OUT_RENAME) {
      *w++ = 0x2A;
      w = put_varint(w, (uint64_t)e.meth_len + 1 + e.tmpl_len);
      const uint8_t* m = e.meth_in_mods ? (const uint8_t*)c.mods.data() + e.meth_off : pb + e.meth_off;
      std::memcpy(w, m, e.meth_len);
      w += e.meth_len;
      *w++ = ' ';
      std::memcpy(w, T, e.tmpl_len);
      w += e.tmpl_len;
    }
    std::memcpy(w, sp + e.name_b, e.attr_a - e.name_b);
    w += e.attr_a - e.name_b;
    if (e.u & OSE_OUT_SET_ATTR) {
      const size_t kl = e.client ? 12 : 10;
      *w++ = 0x4A;
      w = put_varint(w, kv_len(e.client, e.tmpl_len));
      *w++ = 0x0A;
      *w++ = (uint8_t)kl;
      std::memcpy(w, e.client ? "url.template" : "http.route", kl);
      w += kl;
      *w++ = 0x12;
      w = put_varint(w, flen(e.tmpl_len));
      *w++ = 0x0A;
      w = put_varint(w, e.tmpl_len);
      std::memcpy(w, T, e.tmpl_len);
      w += e.tmpl_len;
    }
    std::memcpy(w, sp + e.attr_b, L - e.attr_b);
    return w + (L - e.attr_b);
  }

  // pass 1: sizes, headers, edited spans
  void size_chunk(Chunk& c) {
    c.out_bytes.assign(n_out, 0);
    c.out_res.assign(n_out, 0);
    std::vector<std::pair<size_t, size_t>> rf;
    if (d.drop_all) {   // OSE_GROUP_BATCH, unsampled: ResourceSpans().RemoveIf(true)
      for (uint64_t r = c.r0; r < c.r1; r++) res_body[r] = kDropped;
      return;
    }
    for (uint64_t r = c.r0; r < c.r1; r++) {
      const uint64_t rr = lay.res_ref[r];
      const size_t ro = (uint32_t)rr, rl = (size_t)(rr >> 32);
      PbReader p(pb + ro, rl);
      rf.clear();
      uint64_t schema = 0;
      uint32_t f, wt;
      while (p.more() && p.tag(f, wt)) {
        size_t o, l;
        if (wt == 2 && (f == 1 || f == 2 || f == 3 || f == 1000)) {
          if (!p.bytes(o, l)) break;
          if (f == 1) rf.emplace_back(ro + o, l);
          else if (f == 3) schema = (ro + o) | ((uint64_t)l << 32);
        } else {
          p.skip(wt, f);
        }
      }
      if (!p.ok) { c.err = "OTLP protobuf: malformed ResourceSpans"; return; }
      const ResHdr* h = resource_header(c, rf);
      if (!h) return;
      res_hdr[r] = h;
      res_schema[r] = schema;
      uint64_t body = h->bytes.size() + ((schema >> 32) ? flen(schema >> 32) : 0);
      bool had = false, any = false;
      for (uint64_t s = lay.res_scope0[r]; s < res_scope_end(r); s++) {
        const std::string* sh = scope_header(c, s);
        if (!sh) return;
        scope_hdr[s] = sh;
        const uint64_t sch = lay.scope_schema[s] >> 32;
        uint64_t sb = sh->size() + (sch ? flen(sch) : 0);
        const uint64_t i0 = lay.scope_span0[s], i1 = scope_end(s);
        bool kept_any = false;
        for (uint64_t i = i0; i < i1; i++) {
          if (!kept(i)) continue;
          kept_any = true;
          uint64_t l = span_ref[i] >> 32;
          if (rewritten(i)) {
            if (!rewrite(c, i)) return;
            l = c.edits.back().out_len;
          }
          sb += flen(l);
        }
        had |= i1 > i0;
        if (i1 > i0 && !kept_any) {   // emptied by sampling: removed (host.cpp Apply)
          scope_body[s] = kDropped;
          continue;
        }
        scope_body[s] = sb;
        body += flen(sb);
        any = true;
      }
      if (had && !any) {
        res_body[r] = kDropped;
        continue;
      }
      res_body[r] = body;
      uint32_t ks[64], nk;
      outputs_of(h, ks, nk);
      for (uint32_t q = 0; q < nk; q++) {
        c.out_bytes[ks[q]] += flen(body);
        c.out_res[ks[q]]++;
      }
    }
  }

  // pass 2: the records at their final offsets
  void write_chunk(Chunk& c, std::vector<EncodedOutput>& outs) {
    size_t ei = 0;
    for (uint64_t r = c.r0; r < c.r1; r++) {
      if (res_body[r] == kDropped) continue;
      uint32_t ks[64], nk;
      outputs_of(res_hdr[r], ks, nk);
      uint8_t* const w0 = outs[ks[0]].data + c.cursor[ks[0]];
      uint8_t* w = w0;
      *w++ = 0x0A;
      w = put_varint(w, res_body[r]);
      const std::string& rh = res_hdr[r]->bytes;
      std::memcpy(w, rh.data(), rh.size());
      w += rh.size();
      for (uint64_t s = lay.res_scope0[r]; s < res_scope_end(r); s++) {
        const uint64_t i0 = lay.scope_span0[s], i1 = scope_end(s);
        if (scope_body[s] == kDropped) continue;   // no span of it kept: nothing in mods
        *w++ = 0x12;
        w = put_varint(w, scope_body[s]);
        const std::string& sh = *scope_hdr[s];
        std::memcpy(w, sh.data(), sh.size());
        w += sh.size();
        for (uint64_t i = i0; i < i1; i++) {
          if (!kept(i)) continue;
          if (rewritten(i)) {
            const Edit& ed = c.edits[ei++];
            *w++ = 0x12;
            w = put_varint(w, ed.out_len);
            w = write_edit(c, ed, pb + (uint32_t)span_ref[i], span_ref[i] >> 32, w);
          } else {
            w = put_rec(w, 0x12, pb + (uint32_t)span_ref[i], span_ref[i] >> 32);
          }
        }
        const uint64_t sch = lay.scope_schema[s];
        if (sch >> 32) w = put_rec(w, 0x1A, pb + (uint32_t)sch, sch >> 32);
      }
      const uint64_t rs = res_schema[r];
      if (rs >> 32) w = put_rec(w, 0x1A, pb + (uint32_t)rs, rs >> 32);
      const uint64_t rec = (uint64_t)(w - w0);
      c.cursor[ks[0]] += rec;
      for (uint32_t q = 1; q < nk; q++) {
        std::memcpy(outs[ks[q]].data + c.cursor[ks[q]], w0, rec);
        c.cursor[ks[q]] += rec;
      }
    }
  }
};
}  // namespace enc

struct EncodeWork {
  std::vector<enc::Chunk> ch;
  std::vector<uint64_t> res_body, res_schema, scope_body;
  std::vector<const enc::ResHdr*> res_hdr;
  std::vector<const std::string*> scope_hdr;
  std::vector<std::pair<uint8_t*, size_t>> bufs;     // free output buffers
  std::vector<std::pair<uint8_t*, size_t>> pinned;   // free pinned output buffers (the GPU encoder's)
  ~EncodeWork() {
    for (auto& b : bufs) std::free(b.first);
    for (auto& b : pinned) (void)hipHostFree(b.first);
  }
};
EncodeWork* encode_work_new() { return new EncodeWork(); }
void encode_work_free(EncodeWork* w) { delete w; }

uint8_t* encode_work_pinned(EncodeWork& w, size_t need, size_t* cap) {
  need = std::max<size_t>(need, 64);
  size_t best = w.pinned.size();
  for (size_t k = 0; k < w.pinned.size(); k++)
    if (w.pinned[k].second >= need && (best == w.pinned.size() || w.pinned[k].second < w.pinned[best].second)) best = k;
  if (best < w.pinned.size()) {
    uint8_t* p = w.pinned[best].first;
    *cap = w.pinned[best].second;
    w.pinned.erase(w.pinned.begin() + (ptrdiff_t)best);
    return p;
  }
  const size_t c = need + need / 8;
  void* p = nullptr;
  if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  *cap = c;
  return static_cast<uint8_t*>(p);
}

void otlp_out_release(OtlpOut* o) {
  if (!o) return;
  if (o->work) {
    for (auto& x : o->outs)
      if (x.data) (x.pinned ? o->work->pinned : o->work->bufs).emplace_back(x.data, x.cap);
    o->outs.clear();
    if (o->e && !o->e->closed.load()) {
      std::lock_guard<std::mutex> g(o->e->mu);
      if (o->e->enc_pool.size() < 8) {
        o->e->enc_pool.push_back(o->work);
        o->work = nullptr;
      }
    }
    delete o->work;
  }
  if (o->e) engine_unref(o->e);
  delete o;
}

void release_encode(Engine* e) {
  for (void* p : e->enc_pool) delete static_cast<EncodeWork*>(p);
  e->enc_pool.clear();
}

bool encode_traces(const uint8_t* pb, size_t len, const std::vector<uint64_t>& span_ref, const OtlpLayout& lay,
                   const EncodeDecisions& d, const Router* router, int threads, EncodeWork& w,
                   std::vector<EncodedOutput>& outs, std::string& err, double* t_ms3) {
  using namespace enc;
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  auto lap = [&](int k) {
    const auto t = clk::now();
    if (t_ms3) t_ms3[k] = std::chrono::duration<double, std::milli>(t - t0).count();
    t0 = t;
  };
  Enc e{pb, len, span_ref, lay, d, router, span_ref.size(), lay.res_ref.size(), lay.scope_ref.size(), 1,
        w.res_body, w.res_schema, w.res_hdr, w.scope_body, w.scope_hdr};
  if (router) {
    if (router->pipelines.size() > 63) { err = "router: more than 63 pipelines"; return false; }
    e.n_out = (uint32_t)router->pipelines.size() + 1;
  }
  e.res_body.assign(e.R, 0);
  e.res_schema.assign(e.R, 0);
  e.res_hdr.assign(e.R, nullptr);
  e.scope_body.assign(e.S, 0);
  e.scope_hdr.assign(e.S, nullptr);
  // chunks of about equal span counts
  int T = std::max(1, threads);
  T = (int)std::min<uint64_t>((uint64_t)T, std::max<uint64_t>(1, std::min<uint64_t>(e.R, e.n / 2048 + 1)));
  std::vector<Chunk>& ch = w.ch;
  if (ch.size() < (size_t)T) ch.resize((size_t)T);
  for (int t = 0; t < T; t++) {   // keep the capacity, drop the contents
    Chunk& c = ch[t];
    c.rcache.clear();
    c.scache.clear();
    c.rown.clear();
    c.sown.clear();
    c.mods.clear();
    c.edits.clear();
    c.err.clear();
  }
  {
    uint64_t r = 0;
    for (int t = 0; t < T; t++) {
      ch[t].r0 = r;
      const uint64_t goal = e.n * (uint64_t)(t + 1) / (uint64_t)T;
      if (t == T - 1) r = e.R;
      else while (r < e.R && e.res_span0(r) < goal) r++;
      ch[t].r1 = r;
    }
  }
  auto run = [&](auto&& fn) { parallel_run(T, [&](int t) { fn(ch[t]); }); };
  run([&](Chunk& c) { e.size_chunk(c); });
  for (int t = 0; t < T; t++)
    if (!ch[t].err.empty()) { err = ch[t].err; return false; }
  lap(0);
  outs.assign(e.n_out, EncodedOutput{});
  for (uint32_t k = 0; k < e.n_out; k++) {
    outs[k].name = router ? (k + 1 < e.n_out ? router->pipelines[k] : std::string("default")) : std::string();
    uint64_t off = 0;
    for (int t = 0; t < T; t++) {
      Chunk& c = ch[t];
      c.cursor.resize(e.n_out);
      c.cursor[k] = off;
      off += c.out_bytes[k];
      outs[k].n_resources += (uint32_t)c.out_res[k];
    }
    outs[k].len = off;
  }
  // buffers: the largest outputs take the largest free buffers
  std::vector<uint32_t> order(e.n_out);
  for (uint32_t k = 0; k < e.n_out; k++) order[k] = k;
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return outs[a].len > outs[b].len; });
  std::sort(w.bufs.begin(), w.bufs.end(), [](auto& a, auto& b) { return a.second > b.second; });
  for (uint32_t q = 0; q < e.n_out; q++) {
    EncodedOutput& x = outs[order[q]];
    const size_t need = std::max<size_t>(x.len, 64);
    if (!w.bufs.empty() && w.bufs.front().second >= need) {
      x.data = w.bufs.front().first;
      x.cap = w.bufs.front().second;
      w.bufs.erase(w.bufs.begin());
      continue;
    }
    const size_t cap = need + need / 8;
    x.data = static_cast<uint8_t*>(std::malloc(cap));
    x.cap = cap;
    if (!x.data) {
      for (auto& y : outs)
        if (y.data) w.bufs.emplace_back(y.data, y.cap);
      outs.clear();
      err = "out of host memory";
      return false;
    }
  }
  lap(1);
  run([&](Chunk& c) { e.write_chunk(c, outs); });
  lap(2);
  return true;
}

}  // namespace ose

using namespace ose;

extern "C" {

int ose_router_create(const char* cfg_json, ose_router** out) {
  if (!cfg_json || !out) return fail(OSE_EINVAL, "NULL argument");
  try {
    auto* r = new Router();
    const std::string err = build_router(parse_json(cfg_json), "TRACES", *r);   // common.TracesObservabilitySignal
    if (!err.empty()) { delete r; return fail(OSE_EINVAL, err); }
    *out = reinterpret_cast<ose_router*>(r);
    return 0;
  } catch (const std::exception& ex) {
    return fail(OSE_EINVAL, ex.what());
  }
}

void ose_router_destroy(ose_router* r) {
  LastErrorScope keep("ose_router_destroy");
  delete reinterpret_cast<Router*>(r);
}

uint32_t ose_router_pipelines(const ose_router* r) {
  return r ? (uint32_t)reinterpret_cast<const Router*>(r)->pipelines.size() : 0;
}

const char* ose_router_pipeline(const ose_router* r, uint32_t k) {
  if (!r) return nullptr;
  const auto& p = reinterpret_cast<const Router*>(r)->pipelines;
  return k < p.size() ? p[k].c_str() : nullptr;
}

uint32_t ose_otlp_out_count(const ose_otlp_out* o) {
  return o ? (uint32_t)reinterpret_cast<const OtlpOut*>(o)->outs.size() : 0;
}

int ose_otlp_out_get(const ose_otlp_out* o, uint32_t k, const char** name, const uint8_t** data, uint64_t* len,
                     uint32_t* n_resources) {
  if (!o) return fail(OSE_EINVAL, "NULL argument");
  const auto& v = reinterpret_cast<const OtlpOut*>(o)->outs;
  if (k >= v.size()) return fail(OSE_EINVAL, "output index out of range");
  if (name) *name = v[k].name.c_str();
  if (data) *data = v[k].data;
  if (len) *len = v[k].len;
  if (n_resources) *n_resources = v[k].n_resources;
  return 0;
}

void ose_otlp_out_release(ose_otlp_out* o) {
  LastErrorScope keep("ose_otlp_out_release");
  otlp_out_release(reinterpret_cast<OtlpOut*>(o));
}

// diagnostics: decisions D2H, sizing pass, buffers, writing pass (ms)
int osehost_otlp_out_timings(const ose_otlp_out* o, double* ms4) {
  if (!o || !ms4) return fail(OSE_EINVAL, "NULL argument");
  std::memcpy(ms4, reinterpret_cast<const OtlpOut*>(o)->t_ms, sizeof(double) * 4);
  return 0;
}

// diagnostics: 1 when the GPU encoder wrote the outputs; *fallback: why the
// GPU encoder handed the call to the host (kEncFb* bits, 0 when it did not run)
int osehost_otlp_out_path(const ose_otlp_out* o, uint32_t* fallback) {
  if (!o) return fail(OSE_EINVAL, "NULL argument");
  const OtlpOut* x = reinterpret_cast<const OtlpOut*>(o);
  if (fallback) *fallback = x->fallback;
  return x->gpu;
}

// Test seams (CPU).  A router for any signal (the KATs route logs and
// metrics too); the routing of one resource's attributes ({"key": value})
// as {"key": "...", "pipelines": [...]}.
int osehost_router_create_signal(const char* cfg_json, const char* signal, ose_router** out) {
  if (!cfg_json || !signal || !out) return fail(OSE_EINVAL, "NULL argument");
  try {
    auto* r = new Router();
    const std::string err = build_router(parse_json(cfg_json), signal, *r);
    if (!err.empty()) { delete r; return fail(OSE_EINVAL, err); }
    *out = reinterpret_cast<ose_router*>(r);
    return 0;
  } catch (const std::exception& ex) {
    return fail(OSE_EINVAL, ex.what());
  }
}

char* osehost_router_route(const ose_router* rr, const char* attrs_json) {
  if (!rr || !attrs_json) { fail(OSE_EINVAL, "NULL argument"); return nullptr; }
  try {
    const Router* r = reinterpret_cast<const Router*>(rr);
    const Json j = parse_json(attrs_json);
    AttrMap a;
    for (auto& kv : j.obj) {
      Value v;
      if (kv.second.is_str()) v = Value::str(kv.second.s);
      else if (kv.second.is_num()) v.type = Value::TInt, v.i = kv.second.i64();
      else if (kv.second.is_bool()) v.type = Value::TBool, v.b = kv.second.b;
      a.kv.emplace_back(kv.first, std::move(v));
    }
    std::string key;
    const std::vector<uint32_t>* p = r->route(a, &key);
    Json o = Json::object();
    o.set("key", Json::str(key));
    Json arr = Json::array();
    if (p)
      for (uint32_t k : *p) arr.push(Json::str(r->pipelines[k]));
    o.set("pipelines", std::move(arr));
    std::string s;
    dump_json(s, o);
    char* out = static_cast<char*>(std::malloc(s.size() + 1));
    std::memcpy(out, s.c_str(), s.size() + 1);
    return out;
  } catch (const std::exception& ex) {
    fail(OSE_EINVAL, ex.what());
    return nullptr;
  }
}

}  // extern "C"
