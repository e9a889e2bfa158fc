// otlp_encode.hpp — SoA decisions → OTLP TracesData bytes, and the
// odigosrouterconnector routing table.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/odigos_amd.h"
#include "json.hpp"
#include "pdata.hpp"

namespace ose {

// Where the structural walk found each message of one TracesData (offsets
// into the message bytes; a ref is offset | length << 32).
struct OtlpLayout {
  static constexpr uint64_t kMulti = ~0ull;   // scope_hdr: several scope fields (merged)
  std::vector<uint64_t> res_ref;       // ResourceSpans payload
  std::vector<uint32_t> res_scope0;    // first scope of each resource
  std::vector<uint64_t> scope_ref;     // ScopeSpans payload
  std::vector<uint64_t> scope_hdr;     // its InstrumentationScope message (0: none)
  std::vector<uint64_t> scope_schema;  // its schema_url (last occurrence; length 0: none)
  std::vector<uint32_t> scope_span0;   // first span of each scope
};

// odigosrouterconnector: BuildSignalRoutingMap (routingmap.go:34-57) for one
// signal, and determineRoutingPipelines (connector.go:147-172).
struct Router {
  std::string signal;
  std::vector<std::string> pipelines;                                  // output order: first appearance
  std::unordered_map<std::string, std::vector<uint32_t>> routes;       // "ns/kind/name" → pipelines
  // NULL when the resource routes to the default pipeline; *key gets the
  // routing key when one matched
  const std::vector<uint32_t>* route(const AttrMap& attrs, std::string* key = nullptr) const;
  // the routes as the GPU encoder reads them (EncRouteSlot[1 << route_bits],
  // then the key bytes; FNV-1a 64 of the key, linear probing), built with
  // the router
  std::vector<uint8_t> dev_blob;
  uint32_t route_bits = 0;
  size_t dev_slots_bytes = 0;
};
// {"datastreams": [{"name", "sources": [{"namespace", "kind", "name"}],
//   "destinations": [{"destinationname", "configuredsignals": [...]}]}]}
std::string build_router(const Json& cfg, const std::string& signal, Router& r);
std::string normalize_kind(const std::string& kind);

// The per-span decisions the encoder applies (host memory).
struct EncodeDecisions {
  const uint8_t* keep = nullptr;        // NULL: every span kept
  bool drop_all = false;                // OSE_GROUP_BATCH, the call's trace unsampled
  const uint8_t* url_out = nullptr;     // NULL: no template stage
  const ose_strref* tmpl = nullptr;
  const uint8_t* tmpl_arena = nullptr;
  uint64_t tmpl_arena_len = 0;
  const uint32_t* span_size = nullptr;  // pdata's size of each span (NULL: trust the input's encoding)
};

struct EncodedOutput {
  std::string name;
  uint8_t* data = nullptr;   // malloc'd (or pinned), from the workspace's buffers
  size_t cap = 0;
  bool pinned = false;       // hipHostMalloc'd (the GPU encoder's D2H target)
  uint64_t len = 0;
  uint32_t n_resources = 0;
};

// The encoder's grow-only state (per-thread chunks, per-resource records,
// output buffers): reused across calls so a steady stream of batches does
// not allocate or fault in fresh pages.
struct EncodeWork;
EncodeWork* encode_work_new();
void encode_work_free(EncodeWork* w);
// a pinned host buffer of at least `need` bytes from the workspace's pool
// (NULL when hipHostMalloc fails); it goes back to the pool with the output
uint8_t* encode_work_pinned(EncodeWork& w, size_t need, size_t* cap);

struct Engine;
struct OtlpOut {   // ose_otlp_out
  std::vector<EncodedOutput> outs;
  EncodeWork* work = nullptr;   // the outputs' buffers go back to it
  Engine* e = nullptr;          // whose pool the workspace returns to (NULL: freed)
  double t_ms[4] = {0, 0, 0, 0};   // decisions D2H, sizing pass, buffers, writing pass
  int gpu = 0;                     // 1: written by the GPU encoder (encode_kernel.hip)
  uint32_t fallback = 0;           // why the GPU encoder handed the call to the host (kEncFb*)
  // one request's slice of a coalesced batch (otlp_pipeline.cpp): the data
  // pointers are into the batch's outputs, which `hold` keeps alive
  std::shared_ptr<OtlpOut> hold;
};
void otlp_out_release(OtlpOut* o);

// One TracesData per output (router pipelines, then the default one; one
// output without a router).  false + err on a malformed message.  t_ms3:
// the sizing pass, buffers, writing pass.
bool encode_traces(const uint8_t* pb, size_t len, const std::vector<uint64_t>& span_ref, const OtlpLayout& lay,
                   const EncodeDecisions& d, const Router* router, int threads, EncodeWork& w,
                   std::vector<EncodedOutput>& outs, std::string& err, double* t_ms3 = nullptr);

}  // namespace ose
