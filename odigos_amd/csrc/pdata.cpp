// pdata.cpp — see pdata.hpp.
#include "pdata.hpp"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <map>

namespace ose {

namespace {

// strconv.AppendFloat(f, fmt, -1, 64): shortest round-trip digits
std::string format_float(double f, bool exp) {
  char buf[64];
  auto r = exp ? std::to_chars(buf, buf + sizeof buf, f, std::chars_format::scientific)
               : std::to_chars(buf, buf + sizeof buf, f, std::chars_format::fixed);
  return std::string(buf, r.ptr);
}

// encoding/json float64 encoder / pdata float64AsString: like %g with ES6
// cutoffs (1e-6, 1e21) and the exponent cleaned (e-07 -> e-7)
std::string float64_as_string(double f) {
  if (std::isinf(f) || std::isnan(f)) {
    std::string g = std::isnan(f) ? "NaN" : (f > 0 ? "+Inf" : "-Inf");
    return "json: unsupported value: " + g;
  }
  double a = std::fabs(f);
  bool e = a != 0 && (a < 1e-6 || a >= 1e21);
  std::string s = format_float(f, e);
  if (e) {
    size_t n = s.size();
    if (n >= 4 && s[n - 4] == 'e' && s[n - 3] == '-' && s[n - 2] == '0') {
      s[n - 2] = s[n - 1];
      s.pop_back();
    }
  }
  return s;
}

const char* kB64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
std::string base64(const std::string& in) {
  std::string o;
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += kB64[(v >> 6) & 63]; o += kB64[v & 63];
  }
  if (i + 1 == in.size()) {
    uint32_t v = (uint8_t)in[i] << 16;
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += kB64[(v >> 6) & 63]; o += '=';
  }
  return o;
}
std::string unbase64(const std::string& in) {
  std::string o;
  uint32_t v = 0;
  int bits = 0;
  for (char c : in) {
    const char* p = std::strchr(kB64, c);
    if (!p || c == 0) continue;
    v = (v << 6) | (uint32_t)(p - kB64);
    bits += 6;
    if (bits >= 8) { bits -= 8; o += (char)((v >> bits) & 0xFF); }
  }
  return o;
}

// encoding/json Marshal of Value.AsRaw(): maps with sorted keys, HTML-safe
// escaping of <, >, & and U+2028/9, invalid UTF-8 -> U+FFFD.
void json_go_string(std::string& o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
      else if (c == '\n') o += "\\n";
      else if (c == '\r') o += "\\r";
      else if (c == '\t') o += "\\t";
      else if (c < 0x20 || c == '<' || c == '>' || c == '&') { o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15]; }
      else o += (char)c;
      i++;
      continue;
    }
    // decode one rune (utf8.DecodeRuneInString)
    int need = 0;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    bool ok = need > 0 && i + (size_t)need < s.size();
    if (ok) {
      for (int k = 1; k <= need; k++) {
        uint8_t b = (uint8_t)s[i + k];
        if (b < (k == 1 ? lo : 0x80) || b > (k == 1 ? hi : 0xBF)) { ok = false; break; }
      }
    }
    if (!ok) { o += "\\ufffd"; i++; continue; }
    if (need == 2 && c == 0xE2 && (uint8_t)s[i + 1] == 0x80 && ((uint8_t)s[i + 2] == 0xA8 || (uint8_t)s[i + 2] == 0xA9)) {
      o += (uint8_t)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
    } else {
      o.append(s, i, need + 1);
    }
    i += need + 1;
  }
  o += '"';
}

void json_go_value(std::string& o, const Value& v) {
  switch (v.type) {
    case Value::TEmpty: o += "null"; break;
    case Value::TStr: json_go_string(o, v.s); break;
    case Value::TInt: o += std::to_string(v.i); break;
    case Value::TDouble: o += float64_as_string(v.d); break;
    case Value::TBool: o += v.b ? "true" : "false"; break;
    case Value::TBytes: json_go_string(o, base64(v.s)); break;
    case Value::TSlice:
      o += '[';
      for (size_t k = 0; k < v.slice.size(); k++) { if (k) o += ','; json_go_value(o, v.slice[k]); }
      o += ']';
      break;
    case Value::TMap: {
      std::map<std::string, const Value*> sorted;   // AsRaw -> map[string]any; later keys win
      for (auto& kv : v.map) sorted[kv.first] = &kv.second;
      o += '{';
      bool first = true;
      for (auto& kv : sorted) {
        if (!first) o += ',';
        first = false;
        json_go_string(o, kv.first);
        o += ':';
        json_go_value(o, *kv.second);
      }
      o += '}';
      break;
    }
  }
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
template <size_t N>
void parse_id(const Json* j, std::array<uint8_t, N>& out) {
  out.fill(0);
  if (!j || !j->is_str()) return;
  const std::string& s = j->s;
  if (s.size() != 2 * N) return;
  for (size_t k = 0; k < N; k++) out[k] = (uint8_t)(hexval(s[2 * k]) * 16 + hexval(s[2 * k + 1]));
}
template <size_t N>
Json id_json(const std::array<uint8_t, N>& id) {
  static const char* hex = "0123456789abcdef";
  bool empty = std::all_of(id.begin(), id.end(), [](uint8_t b) { return b == 0; });
  if (empty) return Json::str("");
  std::string s;
  for (uint8_t b : id) { s += hex[b >> 4]; s += hex[b & 15]; }
  return Json::str(s);
}

uint64_t ju64(const Json* j) { return j ? (j->is_str() || j->is_num() ? j->u64() : 0) : 0; }
int64_t ji64(const Json* j) { return j ? (j->is_str() || j->is_num() ? j->i64() : 0) : 0; }
std::string jstr(const Json* j) { return j && j->is_str() ? j->s : std::string(); }

Value value_from_json(const Json* j);
AttrMap attrs_from_json(const Json* j) {
  AttrMap m;
  if (!j || !j->is_arr()) return m;
  for (auto& e : j->arr) m.kv.emplace_back(jstr(e.get("key")), value_from_json(e.get("value")));
  return m;
}
Value value_from_json(const Json* j) {
  Value v;
  if (!j || !j->is_obj()) return v;
  if (const Json* x = j->get("stringValue")) { v.type = Value::TStr; v.s = jstr(x); }
  else if (const Json* x = j->get("intValue")) { v.type = Value::TInt; v.i = ji64(x); }
  else if (const Json* x = j->get("doubleValue")) { v.type = Value::TDouble; v.d = x->num(); }
  else if (const Json* x = j->get("boolValue")) { v.type = Value::TBool; v.b = x->is_bool() && x->b; }
  else if (const Json* x = j->get("bytesValue")) { v.type = Value::TBytes; v.s = unbase64(jstr(x)); }
  else if (const Json* x = j->get("arrayValue")) {
    v.type = Value::TSlice;
    if (const Json* vals = x->get("values"))
      if (vals->is_arr())
        for (auto& e : vals->arr) v.slice.push_back(value_from_json(&e));
  } else if (const Json* x = j->get("kvlistValue")) {
    v.type = Value::TMap;
    v.map = attrs_from_json(x->get("values")).kv;
  }
  return v;
}
Json value_to_json(const Value& v);
Json attrs_to_json(const AttrMap& m) {
  Json a = Json::array();
  for (auto& kv : m.kv) {
    Json e = Json::object();
    e.set("key", Json::str(kv.first));
    e.set("value", value_to_json(kv.second));
    a.push(std::move(e));
  }
  return a;
}
Json value_to_json(const Value& v) {
  Json o = Json::object();
  switch (v.type) {
    case Value::TEmpty: break;
    case Value::TStr: o.set("stringValue", Json::str(v.s)); break;
    case Value::TInt: o.set("intValue", Json::str(std::to_string(v.i))); break;
    case Value::TDouble: {
      if (!std::isfinite(v.d)) {   // protobuf JSON mapping: "NaN", "Infinity", "-Infinity"
        o.set("doubleValue", Json::str(v.d != v.d ? "NaN" : v.d > 0 ? "Infinity" : "-Infinity"));
        break;
      }
      char buf[64];
      auto r = std::to_chars(buf, buf + sizeof buf, v.d);
      o.set("doubleValue", Json::number(std::string(buf, r.ptr)));
      break;
    }
    case Value::TBool: o.set("boolValue", Json::boolean(v.b)); break;
    case Value::TBytes: o.set("bytesValue", Json::str(base64(v.s))); break;
    case Value::TSlice: {
      Json vals = Json::array();
      for (auto& e : v.slice) vals.push(value_to_json(e));
      Json av = Json::object();
      av.set("values", std::move(vals));
      o.set("arrayValue", std::move(av));
      break;
    }
    case Value::TMap: {
      AttrMap m;
      m.kv = v.map;
      Json kv = Json::object();
      kv.set("values", attrs_to_json(m));
      o.set("kvlistValue", std::move(kv));
      break;
    }
  }
  return o;
}

}  // namespace

std::string Value::AsString() const {
  switch (type) {
    case TEmpty: return "";
    case TStr: return s;
    case TBool: return b ? "true" : "false";
    case TDouble: return float64_as_string(d);
    case TInt: return std::to_string(i);
    case TBytes: return base64(s);
    case TMap:
    case TSlice: {
      std::string o;
      json_go_value(o, *this);
      return o;
    }
  }
  return "";
}

Traces traces_from_json(const Json& j) {
  Traces t;
  const Json* rss = j.get("resourceSpans");
  if (!rss || !rss->is_arr()) return t;
  for (auto& rj : rss->arr) {
    ResourceSpans rs;
    if (const Json* res = rj.get("resource")) {
      rs.resource_attrs = attrs_from_json(res->get("attributes"));
      rs.resource_dropped = (uint32_t)ju64(res->get("droppedAttributesCount"));
    }
    rs.schema_url = jstr(rj.get("schemaUrl"));
    if (const Json* sss = rj.get("scopeSpans"); sss && sss->is_arr()) {
      for (auto& sj : sss->arr) {
        ScopeSpans ss;
        if (const Json* sc = sj.get("scope")) {
          ss.scope_name = jstr(sc->get("name"));
          ss.scope_version = jstr(sc->get("version"));
          ss.scope_attrs = attrs_from_json(sc->get("attributes"));
          ss.scope_dropped = (uint32_t)ju64(sc->get("droppedAttributesCount"));
        }
        ss.schema_url = jstr(sj.get("schemaUrl"));
        if (const Json* sps = sj.get("spans"); sps && sps->is_arr()) {
          for (auto& pj : sps->arr) {
            Span sp;
            parse_id(pj.get("traceId"), sp.trace_id);
            parse_id(pj.get("spanId"), sp.span_id);
            parse_id(pj.get("parentSpanId"), sp.parent_span_id);
            sp.trace_state = jstr(pj.get("traceState"));
            sp.name = jstr(pj.get("name"));
            sp.kind = (int32_t)ji64(pj.get("kind"));
            sp.start = ju64(pj.get("startTimeUnixNano"));
            sp.end = ju64(pj.get("endTimeUnixNano"));
            sp.attrs = attrs_from_json(pj.get("attributes"));
            sp.dropped_attrs = (uint32_t)ju64(pj.get("droppedAttributesCount"));
            if (const Json* evs = pj.get("events"); evs && evs->is_arr())
              for (auto& ej : evs->arr) {
                Event ev;
                ev.time = ju64(ej.get("timeUnixNano"));
                ev.name = jstr(ej.get("name"));
                ev.attrs = attrs_from_json(ej.get("attributes"));
                ev.dropped = (uint32_t)ju64(ej.get("droppedAttributesCount"));
                sp.events.push_back(std::move(ev));
              }
            sp.dropped_events = (uint32_t)ju64(pj.get("droppedEventsCount"));
            if (const Json* lks = pj.get("links"); lks && lks->is_arr())
              for (auto& lj : lks->arr) {
                Link lk;
                parse_id(lj.get("traceId"), lk.trace_id);
                parse_id(lj.get("spanId"), lk.span_id);
                lk.trace_state = jstr(lj.get("traceState"));
                lk.attrs = attrs_from_json(lj.get("attributes"));
                lk.dropped = (uint32_t)ju64(lj.get("droppedAttributesCount"));
                lk.flags = (uint32_t)ju64(lj.get("flags"));
                sp.links.push_back(std::move(lk));
              }
            sp.dropped_links = (uint32_t)ju64(pj.get("droppedLinksCount"));
            if (const Json* st = pj.get("status")) {
              sp.status_message = jstr(st->get("message"));
              sp.status_code = (int32_t)ji64(st->get("code"));
            }
            sp.flags = (uint32_t)ju64(pj.get("flags"));
            ss.spans.push_back(std::move(sp));
          }
        }
        rs.scope_spans.push_back(std::move(ss));
      }
    }
    t.resource_spans.push_back(std::move(rs));
  }
  return t;
}

Json traces_to_json(const Traces& t) {
  Json root = Json::object();
  Json rss = Json::array();
  for (auto& rs : t.resource_spans) {
    Json rj = Json::object();
    Json res = Json::object();
    res.set("attributes", attrs_to_json(rs.resource_attrs));
    if (rs.resource_dropped) res.set("droppedAttributesCount", Json::number(std::to_string(rs.resource_dropped)));
    rj.set("resource", std::move(res));
    Json sss = Json::array();
    for (auto& ss : rs.scope_spans) {
      Json sj = Json::object();
      Json sc = Json::object();
      if (!ss.scope_name.empty()) sc.set("name", Json::str(ss.scope_name));
      if (!ss.scope_version.empty()) sc.set("version", Json::str(ss.scope_version));
      if (!ss.scope_attrs.kv.empty()) sc.set("attributes", attrs_to_json(ss.scope_attrs));
      sj.set("scope", std::move(sc));
      Json sps = Json::array();
      for (auto& sp : ss.spans) {
        Json pj = Json::object();
        pj.set("traceId", id_json(sp.trace_id));
        pj.set("spanId", id_json(sp.span_id));
        if (std::any_of(sp.parent_span_id.begin(), sp.parent_span_id.end(), [](uint8_t b) { return b; }))
          pj.set("parentSpanId", id_json(sp.parent_span_id));
        if (!sp.trace_state.empty()) pj.set("traceState", Json::str(sp.trace_state));
        pj.set("name", Json::str(sp.name));
        pj.set("kind", Json::number(std::to_string(sp.kind)));
        pj.set("startTimeUnixNano", Json::str(std::to_string(sp.start)));
        pj.set("endTimeUnixNano", Json::str(std::to_string(sp.end)));
        pj.set("attributes", attrs_to_json(sp.attrs));
        Json st = Json::object();
        if (!sp.status_message.empty()) st.set("message", Json::str(sp.status_message));
        if (sp.status_code) st.set("code", Json::number(std::to_string(sp.status_code)));
        pj.set("status", std::move(st));
        sps.push(std::move(pj));
      }
      sj.set("spans", std::move(sps));
      if (!ss.schema_url.empty()) sj.set("schemaUrl", Json::str(ss.schema_url));
      sss.push(std::move(sj));
    }
    rj.set("scopeSpans", std::move(sss));
    if (!rs.schema_url.empty()) rj.set("schemaUrl", Json::str(rs.schema_url));
    rss.push(std::move(rj));
  }
  root.set("resourceSpans", std::move(rss));
  return root;
}

// ---------------- proto sizes (OTLP trace.proto) ----------------
static uint64_t str_field(const std::string& s) { return s.empty() ? 0 : field_len(s.size()); }
static uint64_t varint_field(uint64_t v) { return v ? 1 + sov(v) : 0; }

uint64_t ProtoSizer::any_value(const Value& v) const {
  switch (v.type) {
    case Value::TEmpty: return 0;
    case Value::TStr: return field_len(v.s.size());          // oneof: emitted even when ""
    case Value::TBool: return 2;
    case Value::TInt: return 1 + sov((uint64_t)v.i);
    case Value::TDouble: return 9;
    case Value::TBytes: return field_len(v.s.size());
    case Value::TSlice: {
      uint64_t l = 0;
      for (auto& e : v.slice) l += field_len(any_value(e));   // ArrayValue.values (field 1)
      return field_len(l);
    }
    case Value::TMap: {
      uint64_t l = 0;
      for (auto& kv : v.map) l += field_len(key_value(kv.first, kv.second));   // KeyValueList.values
      return field_len(l);
    }
  }
  return 0;
}
uint64_t ProtoSizer::key_value(const std::string& k, const Value& v) const {
  uint64_t av = any_value(v);
  uint64_t n = str_field(k);
  if (gogo || av) n += field_len(av);   // KeyValue.value: non-nullable in gogo
  return n;
}
uint64_t ProtoSizer::attrs(const AttrMap& m, uint32_t) const {
  uint64_t n = 0;
  for (auto& kv : m.kv) n += field_len(key_value(kv.first, kv.second));
  return n;
}
template <size_t N>
static uint64_t id_field(const std::array<uint8_t, N>& id, bool gogo) {
  bool empty = std::all_of(id.begin(), id.end(), [](uint8_t b) { return b == 0; });
  if (empty) return gogo ? 2 : 0;   // gogo customtype: tag + len 0
  return field_len(N);
}
uint64_t ProtoSizer::span(const Span& s) const {
  uint64_t n = 0;
  n += id_field(s.trace_id, gogo);            // 1 trace_id
  n += id_field(s.span_id, gogo);             // 2 span_id
  n += str_field(s.trace_state);              // 3
  n += id_field(s.parent_span_id, gogo);      // 4 parent_span_id
  n += str_field(s.name);                     // 5
  n += varint_field((uint64_t)(int64_t)s.kind);   // 6
  if (s.start) n += 9;                        // 7 fixed64
  if (s.end) n += 9;                          // 8 fixed64
  n += attrs(s.attrs, 9);                     // 9
  n += varint_field(s.dropped_attrs);         // 10
  for (auto& ev : s.events) {                 // 11
    uint64_t e = (ev.time ? 9 : 0) + str_field(ev.name) + attrs(ev.attrs, 3) + varint_field(ev.dropped);
    n += field_len(e);
  }
  n += varint_field(s.dropped_events);        // 12
  for (auto& lk : s.links) {                  // 13
    uint64_t e = id_field(lk.trace_id, gogo) + id_field(lk.span_id, gogo) + str_field(lk.trace_state) +
                 attrs(lk.attrs, 4) + varint_field(lk.dropped) + (lk.flags ? 5 : 0);
    n += field_len(e);
  }
  n += varint_field(s.dropped_links);         // 14
  uint64_t st = str_field(s.status_message) + varint_field((uint64_t)(int64_t)s.status_code);
  if (gogo || st) n += field_len(st);         // 15 status (non-nullable)
  if (s.flags) n += 6;                        // 16 fixed32: 2-byte tag + 4
  return n;
}
uint64_t ProtoSizer::scope_fixed(const ScopeSpans& ss) const {
  uint64_t sc = str_field(ss.scope_name) + str_field(ss.scope_version) + attrs(ss.scope_attrs, 3) +
                varint_field(ss.scope_dropped);
  uint64_t n = (gogo || sc) ? field_len(sc) : 0;   // 1 scope (non-nullable)
  n += str_field(ss.schema_url);                   // 3
  return n;
}
uint64_t ProtoSizer::resource_fixed(const ResourceSpans& rs) const {
  uint64_t r = attrs(rs.resource_attrs, 1) + varint_field(rs.resource_dropped);
  uint64_t n = (gogo || r) ? field_len(r) : 0;     // 1 resource (non-nullable)
  n += str_field(rs.schema_url);                   // 3
  return n;
}
uint64_t ProtoSizer::resource_spans(const ResourceSpans& rs) const {
  uint64_t n = resource_fixed(rs);
  for (auto& ss : rs.scope_spans) {
    uint64_t s = scope_fixed(ss);
    for (auto& sp : ss.spans) s += field_len(span(sp));
    n += field_len(s);                             // 2 scope_spans
  }
  return n;
}


// ---------------- protobuf encoding (the sizer's fields, written) ----------------
void ProtoWriter::varint(uint64_t v) {
  while (v >= 0x80) { o += (char)(v | 0x80); v >>= 7; }
  o += (char)v;
}
void ProtoWriter::tag(uint32_t field, uint32_t wt) { varint(((uint64_t)field << 3) | wt); }
void ProtoWriter::bytes(uint32_t field, const void* p, size_t n) {
  tag(field, 2);
  varint(n);
  o.append(static_cast<const char*>(p), n);
}
void ProtoWriter::str(uint32_t field, const std::string& s) {
  if (!s.empty()) bytes(field, s.data(), s.size());
}
namespace {
void put_fixed(std::string& o, uint64_t v, int n) {
  for (int k = 0; k < n; k++) o += (char)(v >> (8 * k));
}
template <size_t N>
void put_id(ProtoWriter& w, uint32_t field, const std::array<uint8_t, N>& id) {
  const bool empty = std::all_of(id.begin(), id.end(), [](uint8_t b) { return b == 0; });
  w.bytes(field, id.data(), empty ? 0 : N);   // gogo customtype: framed even when empty
}
}  // namespace
void ProtoWriter::any_value(const Value& v) {
  const ProtoSizer sz;
  switch (v.type) {
    case Value::TEmpty: return;
    case Value::TStr: bytes(1, v.s.data(), v.s.size()); return;   // oneof: written even when ""
    case Value::TBool: tag(2, 0); varint(v.b ? 1 : 0); return;
    case Value::TInt: tag(3, 0); varint((uint64_t)v.i); return;
    case Value::TDouble: {
      tag(4, 1);
      uint64_t bits;
      std::memcpy(&bits, &v.d, 8);
      put_fixed(o, bits, 8);
      return;
    }
    case Value::TBytes: bytes(7, v.s.data(), v.s.size()); return;
    case Value::TSlice: {
      uint64_t l = 0;
      for (auto& e : v.slice) l += field_len(sz.any_value(e));
      tag(5, 2);
      varint(l);
      for (auto& e : v.slice) {   // ArrayValue.values (field 1)
        tag(1, 2);
        varint(sz.any_value(e));
        any_value(e);
      }
      return;
    }
    case Value::TMap: {
      uint64_t l = 0;
      for (auto& kv : v.map) l += field_len(sz.key_value(kv.first, kv.second));
      tag(6, 2);
      varint(l);
      for (auto& kv : v.map) {   // KeyValueList.values (field 1)
        tag(1, 2);
        varint(sz.key_value(kv.first, kv.second));
        key_value(kv.first, kv.second);
      }
      return;
    }
  }
}
void ProtoWriter::key_value(const std::string& k, const Value& v) {
  str(1, k);
  tag(2, 2);   // KeyValue.value: non-nullable, always framed
  varint(ProtoSizer().any_value(v));
  any_value(v);
}
void ProtoWriter::attrs(const AttrMap& m, uint32_t field) {
  const ProtoSizer sz;
  for (auto& kv : m.kv) {
    tag(field, 2);
    varint(sz.key_value(kv.first, kv.second));
    key_value(kv.first, kv.second);
  }
}
void ProtoWriter::span(const Span& s) {
  put_id(*this, 1, s.trace_id);
  put_id(*this, 2, s.span_id);
  str(3, s.trace_state);
  put_id(*this, 4, s.parent_span_id);
  str(5, s.name);
  if (s.kind) { tag(6, 0); varint((uint64_t)(int64_t)s.kind); }
  if (s.start) { tag(7, 1); put_fixed(o, s.start, 8); }
  if (s.end) { tag(8, 1); put_fixed(o, s.end, 8); }
  attrs(s.attrs, 9);
  if (s.dropped_attrs) { tag(10, 0); varint(s.dropped_attrs); }
  const ProtoSizer sz;
  for (auto& ev : s.events) {
    const uint64_t e = (ev.time ? 9 : 0) + str_field(ev.name) + sz.attrs(ev.attrs, 3) + varint_field(ev.dropped);
    tag(11, 2);
    varint(e);
    if (ev.time) { tag(1, 1); put_fixed(o, ev.time, 8); }
    str(2, ev.name);
    attrs(ev.attrs, 3);
    if (ev.dropped) { tag(4, 0); varint(ev.dropped); }
  }
  if (s.dropped_events) { tag(12, 0); varint(s.dropped_events); }
  for (auto& lk : s.links) {
    const uint64_t e = id_field(lk.trace_id, true) + id_field(lk.span_id, true) + str_field(lk.trace_state) +
                       sz.attrs(lk.attrs, 4) + varint_field(lk.dropped) + (lk.flags ? 5 : 0);
    tag(13, 2);
    varint(e);
    put_id(*this, 1, lk.trace_id);
    put_id(*this, 2, lk.span_id);
    str(3, lk.trace_state);
    attrs(lk.attrs, 4);
    if (lk.dropped) { tag(5, 0); varint(lk.dropped); }
    if (lk.flags) { tag(6, 5); put_fixed(o, lk.flags, 4); }
  }
  if (s.dropped_links) { tag(14, 0); varint(s.dropped_links); }
  tag(15, 2);   // Status: non-nullable
  varint(str_field(s.status_message) + varint_field((uint64_t)(int64_t)s.status_code));
  str(2, s.status_message);
  if (s.status_code) { tag(3, 0); varint((uint64_t)(int64_t)s.status_code); }
  if (s.flags) { tag(16, 5); put_fixed(o, s.flags, 4); }
}
void ProtoWriter::resource(const AttrMap& a, uint32_t dropped) {
  attrs(a, 1);
  if (dropped) { tag(2, 0); varint(dropped); }
}
void ProtoWriter::scope(const ScopeSpans& ss) {
  str(1, ss.scope_name);
  str(2, ss.scope_version);
  attrs(ss.scope_attrs, 3);
  if (ss.scope_dropped) { tag(4, 0); varint(ss.scope_dropped); }
}

}  // namespace ose
