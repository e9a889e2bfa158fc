// pdata.hpp — the slice of go.opentelemetry.io/collector/pdata (v1.47.0)
// the three processors touch: ptrace.Traces / ResourceSpans / ScopeSpans /
// Span, pcommon.Map / Value with Get, PutStr, Str and AsString semantics,
// OTLP/JSON I/O, and the OTLP protobuf size of ResourceSpans (what
// ptrace.ProtoMarshaler.ResourceSpansSize returns, odigostrafficmetrics/
// processor.go:77).
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "json.hpp"

namespace ose {

struct Value;
using KV = std::pair<std::string, Value>;

struct Value {
  enum Type { TEmpty, TStr, TInt, TDouble, TBool, TMap, TSlice, TBytes };
  Type type = TEmpty;
  std::string s;          // Str / Bytes
  int64_t i = 0;
  double d = 0;
  bool b = false;
  std::vector<KV> map;
  std::vector<Value> slice;

  static Value str(std::string v) { Value x; x.type = TStr; x.s = std::move(v); return x; }
  // pcommon.Value.Str(): "" unless ValueTypeStr
  const std::string& Str() const { static const std::string empty; return type == TStr ? s : empty; }
  // pcommon.Value.AsString()
  std::string AsString() const;
};

// pcommon.Map: ordered, Get is a linear key scan, PutStr updates in place or
// appends.
struct AttrMap {
  std::vector<KV> kv;
  const Value* Get(std::string_view k) const {
    for (auto& e : kv)
      if (e.first == k) return &e.second;
    return nullptr;
  }
  void PutStr(std::string_view k, std::string_view v) {
    for (auto& e : kv)
      if (e.first == k) {
        if (e.second.type == Value::TStr) e.second.s.assign(v.data(), v.size());   // the string's buffer reused
        else e.second = Value::str(std::string(v));
        return;
      }
    kv.emplace_back(std::string(k), Value::str(std::string(v)));
  }
};

struct Event {
  uint64_t time = 0;
  std::string name;
  AttrMap attrs;
  uint32_t dropped = 0;
};
struct Link {
  std::array<uint8_t, 16> trace_id{};
  std::array<uint8_t, 8> span_id{};
  std::string trace_state;
  AttrMap attrs;
  uint32_t dropped = 0;
  uint32_t flags = 0;
};
struct Span {
  std::array<uint8_t, 16> trace_id{};
  std::array<uint8_t, 8> span_id{};
  std::array<uint8_t, 8> parent_span_id{};
  std::string trace_state;
  std::string name;
  int32_t kind = 0;
  uint64_t start = 0, end = 0;
  AttrMap attrs;
  uint32_t dropped_attrs = 0;
  std::vector<Event> events;
  uint32_t dropped_events = 0;
  std::vector<Link> links;
  uint32_t dropped_links = 0;
  std::string status_message;
  int32_t status_code = 0;
  uint32_t flags = 0;
};
struct ScopeSpans {
  std::string scope_name, scope_version;
  AttrMap scope_attrs;
  uint32_t scope_dropped = 0;
  std::string schema_url;
  std::vector<Span> spans;
};
struct ResourceSpans {
  AttrMap resource_attrs;
  uint32_t resource_dropped = 0;
  std::string schema_url;
  std::vector<ScopeSpans> scope_spans;
};
struct Traces {
  std::vector<ResourceSpans> resource_spans;
  size_t SpanCount() const {
    size_t n = 0;
    for (auto& r : resource_spans)
      for (auto& s : r.scope_spans) n += s.spans.size();
    return n;
  }
};

// OTLP/JSON (ids as hex strings, 64-bit ints as decimal strings or numbers)
Traces traces_from_json(const Json& j);
Json traces_to_json(const Traces& t);

// ---- protobuf sizes (OTLP trace.proto field table) ----
// gogo_always_emit = true reproduces gogoproto's non-nullable embedded
// messages and custom-typed ids (Resource, InstrumentationScope, Status,
// KeyValue.value, trace/span/parent ids are always framed, even when empty);
// false = plain proto3 (omit empty).  See DESIGN.md "Traffic size parity".
inline uint32_t sov(uint64_t x) {
  uint32_t n = 1;
  while (x >= 0x80) { x >>= 7; n++; }
  return n;
}
inline uint64_t field_len(uint64_t l) { return 1 + sov(l) + l; }   // tag (< 16) + varint len + payload
struct ProtoSizer {
  bool gogo = true;
  uint64_t any_value(const Value& v) const;
  uint64_t key_value(const std::string& k, const Value& v) const;
  uint64_t attrs(const AttrMap& m, uint32_t field) const;   // repeated KeyValue, field number < 16
  uint64_t span(const Span& s) const;                        // Span message body
  uint64_t scope_fixed(const ScopeSpans& ss) const;          // ScopeSpans body minus the spans fields
  uint64_t resource_fixed(const ResourceSpans& rs) const;    // ResourceSpans body minus scope_spans fields
  uint64_t resource_spans(const ResourceSpans& rs) const;    // full ResourceSpans body
};

// ---- protobuf encoding: what pdata's generated marshalers write ----
// (MarshalToSizedBuffer: fields in ascending number, defaults omitted,
// gogo's always-framed messages and ids as ProtoSizer counts them), so a
// message's bytes are exactly ProtoSizer{gogo=true}'s length.
struct ProtoWriter {
  std::string& o;
  explicit ProtoWriter(std::string& out) : o(out) {}
  void varint(uint64_t v);
  void tag(uint32_t field, uint32_t wt);
  void bytes(uint32_t field, const void* p, size_t n);   // LEN field, always written
  void str(uint32_t field, const std::string& s);        // omitted when empty
  void any_value(const Value& v);                        // AnyValue body
  void key_value(const std::string& k, const Value& v);  // KeyValue body
  void attrs(const AttrMap& m, uint32_t field);
  void span(const Span& s);                              // Span body
  void resource(const AttrMap& attrs, uint32_t dropped); // Resource body
  void scope(const ScopeSpans& ss);                      // InstrumentationScope body
};

}  // namespace ose
