// otlp_pb.cpp — see otlp_pb.hpp.
#include "otlp_pb.hpp"

#include <cstring>

namespace ose {

// skipTraces: the unknown field whose tag was just read, groups included
bool PbReader::skip(uint32_t wt, uint32_t) {
  int depth = 0;
  for (;;) {
    switch (wt) {
      case 0: varint(); break;
      case 1: if (i + 8 > n) ok = false; else i += 8; break;
      case 2: { size_t o, l; bytes(o, l); break; }
      case 3: depth++; break;
      case 4: if (depth == 0) ok = false; else depth--; break;
      case 5: if (i + 4 > n) ok = false; else i += 4; break;
      default: ok = false;
    }
    if (!ok) return false;
    if (depth == 0) return true;
    const uint64_t t = varint();
    if (!ok) return false;
    wt = (uint32_t)(t & 7);
  }
}

namespace {
constexpr int kMaxDepth = 1000;   // nesting of ArrayValue / KeyValueList (Go's stack only bounds it)
inline bool want(PbReader& r, uint32_t wt, uint32_t expect) {
  if (wt != expect) r.fail();   // proto: wrong wireType
  return r.ok;
}
template <size_t N>
bool put_id(const uint8_t* p, size_t off, size_t len, std::array<uint8_t, N>& id) {
  if (len == 0) { id.fill(0); return true; }
  if (len != N) return false;   // data.TraceID / SpanID Unmarshal
  std::memcpy(id.data(), p + off, N);
  return true;
}
bool pb_attrs_append(const uint8_t* p, size_t off, size_t len, AttrMap& m, int depth) {
  std::string k;
  Value v;
  if (!pb_key_value(p + off, len, k, v, depth)) return false;
  m.kv.emplace_back(std::move(k), std::move(v));
  return true;
}
}  // namespace

// AnyValue fields applied onto v (oneof: the last field set wins)
bool pb_any_value(const uint8_t* p, size_t n, Value& v, int depth) {
  if (depth > kMaxDepth) return false;
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    switch (f) {
      case 1:
        if (want(r, wt, 2) && r.bytes(o, l)) { v = Value(); v.type = Value::TStr; v.s.assign((const char*)p + o, l); }
        break;
      case 2:
        if (want(r, wt, 0)) { const uint64_t x = r.varint(); v = Value(); v.type = Value::TBool; v.b = x != 0; }
        break;
      case 3:
        if (want(r, wt, 0)) { const uint64_t x = r.varint(); v = Value(); v.type = Value::TInt; v.i = (int64_t)x; }
        break;
      case 4:
        if (want(r, wt, 1)) { const uint64_t x = r.fixed64(); v = Value(); v.type = Value::TDouble; std::memcpy(&v.d, &x, 8); }
        break;
      case 5:
        if (want(r, wt, 2) && r.bytes(o, l)) {
          Value a;
          a.type = Value::TSlice;
          PbReader q(p + o, l);
          uint32_t f2, w2;
          while (q.more() && q.tag(f2, w2)) {
            size_t o2, l2;
            if (f2 == 1) {
              if (!want(q, w2, 2) || !q.bytes(o2, l2)) break;
              Value e;
              if (!pb_any_value(p + o + o2, l2, e, depth + 1)) return false;
              a.slice.push_back(std::move(e));
            } else if (!q.skip(w2, f2)) {
              break;
            }
          }
          if (!q.ok) return false;
          v = std::move(a);
        }
        break;
      case 6:
        if (want(r, wt, 2) && r.bytes(o, l)) {
          Value m;
          m.type = Value::TMap;
          PbReader q(p + o, l);
          uint32_t f2, w2;
          while (q.more() && q.tag(f2, w2)) {
            size_t o2, l2;
            if (f2 == 1) {
              if (!want(q, w2, 2) || !q.bytes(o2, l2)) break;
              std::string k;
              Value e;
              if (!pb_key_value(p + o + o2, l2, k, e, depth + 1)) return false;
              m.map.emplace_back(std::move(k), std::move(e));
            } else if (!q.skip(w2, f2)) {
              break;
            }
          }
          if (!q.ok) return false;
          v = std::move(m);
        }
        break;
      case 7:
        if (want(r, wt, 2) && r.bytes(o, l)) { v = Value(); v.type = Value::TBytes; v.s.assign((const char*)p + o, l); }
        break;
      default: r.skip(wt, f);
    }
  }
  return r.ok;
}

bool pb_key_value(const uint8_t* p, size_t n, std::string& key, Value& v, int depth) {
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    if (f == 1) {
      if (want(r, wt, 2) && r.bytes(o, l)) key.assign((const char*)p + o, l);
    } else if (f == 2) {
      if (want(r, wt, 2) && r.bytes(o, l) && !pb_any_value(p + o, l, v, depth)) return false;   // merges
    } else {
      r.skip(wt, f);
    }
  }
  return r.ok;
}

bool pb_resource(const uint8_t* p, size_t n, AttrMap& attrs, uint32_t& dropped) {
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    if (f == 1) {
      if (want(r, wt, 2) && r.bytes(o, l) && !pb_attrs_append(p, o, l, attrs, 0)) return false;
    } else if (f == 2) {
      if (want(r, wt, 0)) dropped = (uint32_t)r.varint();
    } else {
      r.skip(wt, f);
    }
  }
  return r.ok;
}

bool pb_scope(const uint8_t* p, size_t n, ScopeSpans& ss) {
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    switch (f) {
      case 1: if (want(r, wt, 2) && r.bytes(o, l)) ss.scope_name.assign((const char*)p + o, l); break;
      case 2: if (want(r, wt, 2) && r.bytes(o, l)) ss.scope_version.assign((const char*)p + o, l); break;
      case 3: if (want(r, wt, 2) && r.bytes(o, l) && !pb_attrs_append(p, o, l, ss.scope_attrs, 0)) return false; break;
      case 4: if (want(r, wt, 0)) ss.scope_dropped = (uint32_t)r.varint(); break;
      default: r.skip(wt, f);
    }
  }
  return r.ok;
}

namespace {
bool pb_status(const uint8_t* p, size_t n, Span& sp) {   // merges into the span's Status
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    if (f == 2) {
      if (want(r, wt, 2) && r.bytes(o, l)) sp.status_message.assign((const char*)p + o, l);
    } else if (f == 3) {
      if (want(r, wt, 0)) sp.status_code = (int32_t)r.varint();
    } else {
      r.skip(wt, f);
    }
  }
  return r.ok;
}
bool pb_event(const uint8_t* p, size_t n, Event& ev) {
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    switch (f) {
      case 1: if (want(r, wt, 1)) ev.time = r.fixed64(); break;
      case 2: if (want(r, wt, 2) && r.bytes(o, l)) ev.name.assign((const char*)p + o, l); break;
      case 3: if (want(r, wt, 2) && r.bytes(o, l) && !pb_attrs_append(p, o, l, ev.attrs, 0)) return false; break;
      case 4: if (want(r, wt, 0)) ev.dropped = (uint32_t)r.varint(); break;
      default: r.skip(wt, f);
    }
  }
  return r.ok;
}
bool pb_link(const uint8_t* p, size_t n, Link& lk) {
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    switch (f) {
      case 1: if (want(r, wt, 2) && r.bytes(o, l) && !put_id(p, o, l, lk.trace_id)) return false; break;
      case 2: if (want(r, wt, 2) && r.bytes(o, l) && !put_id(p, o, l, lk.span_id)) return false; break;
      case 3: if (want(r, wt, 2) && r.bytes(o, l)) lk.trace_state.assign((const char*)p + o, l); break;
      case 4: if (want(r, wt, 2) && r.bytes(o, l) && !pb_attrs_append(p, o, l, lk.attrs, 0)) return false; break;
      case 5: if (want(r, wt, 0)) lk.dropped = (uint32_t)r.varint(); break;
      case 6: if (want(r, wt, 5)) lk.flags = r.fixed32(); break;
      default: r.skip(wt, f);
    }
  }
  return r.ok;
}
}  // namespace

bool pb_span(const uint8_t* p, size_t n, Span& sp) {
  PbReader r(p, n);
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    size_t o, l;
    switch (f) {
      case 1: if (want(r, wt, 2) && r.bytes(o, l) && !put_id(p, o, l, sp.trace_id)) return false; break;
      case 2: if (want(r, wt, 2) && r.bytes(o, l) && !put_id(p, o, l, sp.span_id)) return false; break;
      case 3: if (want(r, wt, 2) && r.bytes(o, l)) sp.trace_state.assign((const char*)p + o, l); break;
      case 4: if (want(r, wt, 2) && r.bytes(o, l) && !put_id(p, o, l, sp.parent_span_id)) return false; break;
      case 5: if (want(r, wt, 2) && r.bytes(o, l)) sp.name.assign((const char*)p + o, l); break;
      case 6: if (want(r, wt, 0)) sp.kind = (int32_t)r.varint(); break;
      case 7: if (want(r, wt, 1)) sp.start = r.fixed64(); break;
      case 8: if (want(r, wt, 1)) sp.end = r.fixed64(); break;
      case 9: if (want(r, wt, 2) && r.bytes(o, l) && !pb_attrs_append(p, o, l, sp.attrs, 0)) return false; break;
      case 10: if (want(r, wt, 0)) sp.dropped_attrs = (uint32_t)r.varint(); break;
      case 11:
        if (want(r, wt, 2) && r.bytes(o, l)) {
          Event ev;
          if (!pb_event(p + o, l, ev)) return false;
          sp.events.push_back(std::move(ev));
        }
        break;
      case 12: if (want(r, wt, 0)) sp.dropped_events = (uint32_t)r.varint(); break;
      case 13:
        if (want(r, wt, 2) && r.bytes(o, l)) {
          Link lk;
          if (!pb_link(p + o, l, lk)) return false;
          sp.links.push_back(std::move(lk));
        }
        break;
      case 14: if (want(r, wt, 0)) sp.dropped_links = (uint32_t)r.varint(); break;
      case 15: if (want(r, wt, 2) && r.bytes(o, l) && !pb_status(p + o, l, sp)) return false; break;
      case 16: if (want(r, wt, 5)) sp.flags = r.fixed32(); break;
      default: r.skip(wt, f);
    }
  }
  return r.ok;
}

// ResourceSpans: resource (1), scope_spans (2), schema_url (3); the retired
// field 1000 (deprecated scope spans) takes the place of an empty
// scope_spans, as pdata's migration does
bool pb_walk(const uint8_t* p, size_t n, PbWalk& w) {
  PbReader top(p, n);
  uint32_t f, wt;
  auto bad = [&](const char* what) { w.err = std::string("OTLP protobuf: ") + what; return false; };
  while (top.more() && top.tag(f, wt)) {
    size_t ro, rl;
    if (f != 1) {
      if (!top.skip(wt, f)) break;
      continue;
    }
    if (!want(top, wt, 2) || !top.bytes(ro, rl)) break;
    const uint32_t ri = (uint32_t)w.res.size();
    w.res.emplace_back();
    PbReader r(p + ro, rl);
    std::vector<std::pair<size_t, size_t>> scopes, deprecated;
    while (r.more() && r.tag(f, wt)) {
      size_t o, l;
      if (f == 1) {
        if (want(r, wt, 2) && r.bytes(o, l) && !pb_resource(p + ro + o, l, w.res[ri].attrs, w.res[ri].dropped))
          return bad("malformed Resource");
      } else if (f == 2 || f == 1000) {
        if (want(r, wt, 2) && r.bytes(o, l)) (f == 2 ? scopes : deprecated).emplace_back(ro + o, l);
      } else if (f == 3) {
        if (want(r, wt, 2) && r.bytes(o, l)) w.res[ri].schema_url.assign((const char*)p + ro + o, l);
      } else {
        r.skip(wt, f);
      }
    }
    if (!r.ok) return bad("malformed ResourceSpans");
    if (scopes.empty()) scopes.swap(deprecated);
    for (auto& so : scopes) {
      const uint32_t si = (uint32_t)w.scopes.size();
      w.scopes.emplace_back();
      w.scopes[si].resource = ri;
      PbReader s(p + so.first, so.second);
      while (s.more() && s.tag(f, wt)) {
        size_t o, l;
        if (f == 1) {
          if (want(s, wt, 2) && s.bytes(o, l) && !pb_scope(p + so.first + o, l, w.scopes[si].meta))
            return bad("malformed InstrumentationScope");
        } else if (f == 2) {
          if (want(s, wt, 2) && s.bytes(o, l)) {
            const uint64_t off = so.first + o;
            if (off > 0xFFFFFFFFull || l > 0xFFFFFFFFull) return bad("span beyond the 4 GiB arena range");
            w.span_ref.push_back(off | ((uint64_t)l << 32));
            w.span_res.push_back(ri);
            w.span_scope.push_back(si);
          }
        } else if (f == 3) {
          if (want(s, wt, 2) && s.bytes(o, l)) w.scopes[si].meta.schema_url.assign((const char*)p + so.first + o, l);
        } else {
          s.skip(wt, f);
        }
      }
      if (!s.ok) return bad("malformed ScopeSpans");
    }
  }
  if (!top.ok) return bad("malformed TracesData");
  return true;
}

bool traces_from_protobuf(const uint8_t* p, size_t n, Traces& td, std::string& err) {
  PbWalk w;
  if (!pb_walk(p, n, w)) { err = w.err; return false; }
  td.resource_spans.clear();
  for (auto& r : w.res) {
    ResourceSpans rs;
    rs.resource_attrs = r.attrs;
    rs.resource_dropped = r.dropped;
    rs.schema_url = r.schema_url;
    td.resource_spans.push_back(std::move(rs));
  }
  std::vector<size_t> local(w.scopes.size());   // a scope's position inside its resource
  for (size_t q = 0; q < w.scopes.size(); q++) {
    auto& ss = td.resource_spans[w.scopes[q].resource].scope_spans;
    local[q] = ss.size();
    ss.push_back(w.scopes[q].meta);
  }
  for (size_t k = 0; k < w.span_ref.size(); k++) {
    const PbWalk::Scope& s = w.scopes[w.span_scope[k]];
    auto& rs = td.resource_spans[s.resource];
    const size_t idx = local[w.span_scope[k]];
    Span sp;
    if (!pb_span(p + (uint32_t)w.span_ref[k], (size_t)(w.span_ref[k] >> 32), sp)) { err = "OTLP protobuf: malformed Span"; return false; }
    rs.scope_spans[idx].spans.push_back(std::move(sp));
  }
  return true;
}

}  // namespace ose
