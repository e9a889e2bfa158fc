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
#include <cstring>
#include <string>
#include <vector>

#include "pdata.hpp"

namespace ose {

// The wire reader (inline: every walk and edit loop runs on it).
struct PbReader {
  const uint8_t* p;
  size_t n, i = 0;
  bool ok = true;
  PbReader(const uint8_t* b, size_t len) : p(b), n(len) {}
  bool more() const { return ok && i < n; }
  uint64_t varint() {
    if (i < n && p[i] < 0x80) return p[i++];   // one byte: tags and short lengths
    uint64_t v = 0;
    for (uint32_t shift = 0;; shift += 7) {
      if (shift >= 64 || i >= n) { ok = false; return 0; }   // ErrIntOverflow / io.ErrUnexpectedEOF
      const uint8_t b = p[i++];
      v |= (uint64_t)(b & 0x7F) << shift;
      if (b < 0x80) return v;
    }
  }
  bool tag(uint32_t& field, uint32_t& wt) {
    const uint64_t t = varint();
    if (!ok) return false;
    field = (uint32_t)(t >> 3);
    wt = (uint32_t)(t & 7);
    if ((t >> 3) == 0 || (t >> 3) > 0x1FFFFFFF || wt == 4) { ok = false; return false; }   // illegal tag / end group
    return true;
  }
  uint64_t fixed64() {
    if (i + 8 > n) { ok = false; return 0; }
    uint64_t v;
    std::memcpy(&v, p + i, 8);
    i += 8;
    return v;
  }
  uint32_t fixed32() {
    if (i + 4 > n) { ok = false; return 0; }
    uint32_t v;
    std::memcpy(&v, p + i, 4);
    i += 4;
    return v;
  }
  // LEN payload: offset (from p) and length
  bool bytes(size_t& off, size_t& len) {
    const uint64_t l = varint();
    if (!ok) return false;
    if (l > (uint64_t)INT64_MAX || l > n - i) { ok = false; return false; }   // ErrInvalidLength / EOF
    off = i;
    len = (size_t)l;
    i += (size_t)l;
    return true;
  }
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
