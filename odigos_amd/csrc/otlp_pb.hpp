// otlp_pb.hpp — OTLP trace protobuf (opentelemetry/proto/trace/v1) on the
// host: the wire reader, message decoders into the pdata model, and the
// structural walk of a TracesData message that the GPU ingest starts from.
//
// Decoding follows pdata's generated unmarshalers (gogo-style): unknown
// fields are skipped; a known field with the wrong wire type, a truncated
// varint or length, and a trace / span id of a length other than 0, 16 / 8
// are errors (UnmarshalTraces rejects the request); singular scalar fields
// take the last occurrence; embedded non-nullable messages (Resource,
// InstrumentationScope, Status, KeyValue.value) merge field by field; the
// AnyValue oneof takes the last field set; repeated fields append.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "pdata.hpp"

namespace ose {

struct PbReader {
  const uint8_t* p;
  size_t n, i = 0;
  bool ok = true;
  PbReader(const uint8_t* b, size_t len) : p(b), n(len) {}
  bool more() const { return ok && i < n; }
  uint64_t varint();
  bool tag(uint32_t& field, uint32_t& wt);
  uint64_t fixed64();
  uint32_t fixed32();
  // LEN payload: offset (from p) and length
  bool bytes(size_t& off, size_t& len);
  bool skip(uint32_t wt, uint32_t field);   // unknown field (groups included)
  void fail() { ok = false; }
};

// message decoders (false + err on what the unmarshaler rejects)
bool pb_any_value(const uint8_t* p, size_t n, Value& v, int depth = 0);
bool pb_key_value(const uint8_t* p, size_t n, std::string& key, Value& v, int depth = 0);
bool pb_span(const uint8_t* p, size_t n, Span& sp);
bool pb_resource(const uint8_t* p, size_t n, AttrMap& attrs, uint32_t& dropped);
bool pb_scope(const uint8_t* p, size_t n, ScopeSpans& ss);   // InstrumentationScope fields into ss
bool traces_from_protobuf(const uint8_t* p, size_t n, Traces& td, std::string& err);

// The structure of one TracesData message: resources and scopes decoded on
// the host (their contents are few), spans located only (their payloads
// are decoded on the GPU or, for the spans it hands back, by pb_span).
struct PbWalk {
  struct Res {
    AttrMap attrs;
    uint32_t dropped = 0;
    std::string schema_url;
  };
  struct Scope {
    ScopeSpans meta;   // name, version, attributes, dropped, schema_url (no spans)
    uint32_t resource = 0;
  };
  std::vector<Res> res;
  std::vector<Scope> scopes;
  std::vector<uint64_t> span_ref;     // payload offset (low 32 bits) | length << 32
  std::vector<uint32_t> span_res, span_scope;
  std::string err;
};
bool pb_walk(const uint8_t* p, size_t n, PbWalk& w);

}  // namespace ose
