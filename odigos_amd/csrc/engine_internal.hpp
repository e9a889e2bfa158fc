// engine_internal.hpp — the engine object behind the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/odigos_amd.h"
#include "config.hpp"

namespace ose {

int fail(int code, const std::string& msg);
struct Engine;
// makes the engine's device current on the calling thread (a shim's
// goroutines migrate across OS threads; HIP's current device is per thread)
int bind_device(const Engine* e);
int ensure_device();
void engine_retain(Engine* e);
// drops one reference; the last one synchronises the device and frees the engine
void engine_unref(Engine* e);
// The release entry points return nothing, so a HIP error their clean-up
// meets cannot be returned; it is taken out of the runtime's per-thread
// last-error slot (where the caller's next launch check, torch's or a
// shim's, would report it against its own work) and recorded instead:
// ose_dropped_errors() gives the count and the last one (the GPU tests fail
// on any).  An error already pending on entry is left alone.
void note_dropped_error(const char* where, hipError_t err);
struct LastErrorScope {
  const char* where;
  hipError_t prev;
  explicit LastErrorScope(const char* w) : where(w), prev(hipPeekAtLastError()) {}
  ~LastErrorScope() {
    if (prev != hipSuccess) return;
    const hipError_t now = hipGetLastError();
    if (now != hipSuccess) note_dropped_error(where, now);
  }
};
bool stream_capturing(hipStream_t st);
struct Engine;
void release_exchange_scratch(const Engine* e);   // shard_host.cpp
void release_batch_pool(Engine* e);                // batch.cpp
struct OtlpEngine;
void release_otlp(Engine* e);                      // otlp_host.cpp
void release_encode(Engine* e);                    // otlp_encode.cpp

// Device scratch for one in-flight call (look-back status words, sort
// buffers, partial records).  Engines keep a pool so concurrent callers never
// share one.
struct Workspace {
  void* dev = nullptr;
  size_t cap = 0;
  hipEvent_t pending = nullptr;   // recorded at release on the last user's stream
  bool pending_set = false;
  bool captured = false;          // taken by a hipGraph capture: never returned to the pool
  int reserve(size_t bytes);
  // exact trace_id hash table of the SAMPLE stage (trace_kernel.hip), kept
  // across calls: entries carry a generation tag, so nothing is cleared
  void* table = nullptr;
  uint64_t table_slots_cap = 0;
  uint64_t* dup_bkt = nullptr;         // bucketed duplicate detection (TraceKernelArgs::dup_bkt)
  uint32_t* dup_bkt_count = nullptr;
  uint32_t dup_bkt_bits = 0;
  uint32_t epoch = 0;
  int reserve_table(uint64_t n_spans);
  uint32_t* runs = nullptr;        // run-list path: kMaxRuns run heads per table slot
  uint32_t* run_count = nullptr;
  uint64_t runs_slots = 0;
  int reserve_runs();
  void* fold[2] = {nullptr, nullptr};   // FoldState ping-pong of rule-chunked SAMPLE passes
  uint64_t fold_cap = 0;
  int reserve_fold(uint64_t n_spans);
  uint64_t* attr_bits = nullptr;   // span_attribute bits evaluated on the GPU (attr_host.cpp)
  uint64_t attr_bits_cap = 0;
  int reserve_attr(uint64_t n_spans);
  uint64_t* ep_planes = nullptr;   // endpoint bits per rule chunk of a config with spilled route bytes
  uint64_t ep_planes_cap = 0;      // (words)
  // the caller's columns with the spilled endpoint planes substituted: the
  // SAMPLE stage's host-gated tail reads them after run_sampling returned,
  // so they live with the workspace the call holds, not on its stack
  ose_columns spill_cols{};
  // chunk-local service ids of the resources (Engine::sampling_local_svc):
  // res_svc then res_svc_str, 2 * svc_local_cap words, and the columns that
  // point at them
  uint32_t* svc_local = nullptr;
  uint64_t svc_local_cap = 0;
  ose_columns local_cols{};
  int reserve_svc_local(uint64_t n_resources);
  int reserve_ep_planes(uint64_t words);
  // SAMPLE + TEMPLATE in one call: the fast path's dup flag is copied here and
  // read by the host after the URL launches are queued (run_stages), so the
  // slow-path launches are only queued when a trace id repeats
  uint32_t* dup_host = nullptr;   // pinned
  hipEvent_t dup_ready = nullptr;
  // SAMPLE + TEMPLATE: the URL planning kernels run on a second stream
  // beside the trace stage (run_stages): fork and join events
  hipEvent_t fork = nullptr, join = nullptr;
  bool beside_url = false;   // this call's trace stage runs beside the forked URL planning
};

struct Engine {
  // Lifetime: ose_engine_destroy drops the creator's reference; every live
  // child (ose_batch, ose_otlp_batch, ose_otlp_out, ose_gbt) holds one more,
  // so the engine is freed when the last of them is released, in whatever
  // order a shim's finalizers run.  Children released after the destroy are
  // freed instead of pooled.
  std::atomic<int> refs{1};
  std::atomic<bool> closed{false};
  int device = 0;   // the HIP device current when the engine was created; every call runs there
  UrlTemplateConfig url;
  SamplingConfig sampling;
  TrafficMetricsConfig traffic;
  bool has_url = false, has_sampling = false, has_traffic = false;
  // ose_engine_set_option: alternative implementations of the OTLP legs
  // (the default path is the fast one; these select the others, for tests
  // that compare the two)
  enum : uint32_t { kOptOtlpGpuChain = 1, kOptOtlpHostResources = 2, kOptOtlpHostScopes = 4, kOptEncodeHost = 8 };
  std::atomic<uint32_t> options{0};
  bool option(uint32_t o) const { return (options.load(std::memory_order_relaxed) & o) != 0; }
  bool url_needs_resource = false;
  int64_t inverse = 1;
  uint32_t max_name = 5;

  std::vector<uint8_t> url_blob_host;
  uint8_t* url_blob_dev = nullptr;
  std::vector<uint8_t> sampling_blob_host;   // = sampling_chunks_host[0]
  uint8_t* sampling_blob_dev = nullptr;      // = sampling_chunks_dev[0]
  // the rule tables in consecutive chunks of the level-ordered rule list,
  // each within the trace stage's bounds (64 latency bits, 64 service +
  // span_attribute bits, kSampCfgLds bytes); one chunk for most configs
  std::vector<std::vector<uint8_t>> sampling_chunks_host;
  std::vector<uint8_t*> sampling_chunks_dev;
  std::vector<uint8_t> sampling_chunk_attr;   // chunk has span_attribute rules
  // trace-id exchange tables (shard_host.cpp): bit s of sampling_lat_svc =
  // service s has an http_latency rule in some chunk; on the device, the K
  // chunk table pointers then those words (ShardArgs::cfgs, ::lat_svc)
  std::vector<uint32_t> sampling_lat_svc;
  uint8_t* shard_tables_dev = nullptr;
  // which slow paths the trace stage took (ose_engine_path_counts): [0] run
  // lists, [1] the radix sort (device counters), [2] long-run passes (host)
  unsigned long long* path_count_dev = nullptr;
  std::atomic<uint64_t> long_run_passes{0};
  std::unordered_map<std::string, uint32_t> service_ids;
  uint32_t sampling_n_lat = 0, sampling_n_attr = 0;
  uint32_t sampling_n_lat_svc = 0;   // services with http_latency rules (trace_multi_kernel takes <= 64)
  bool sampling_walk_ok = false;     // every chunk has <= 128 rules (SampWalkDev, trace_multi_kernel)
  // a chunk table past kSampCfgLds (a route longer than the LDS table): the
  // trace stage and the pack then take every chunk's endpoint bits as
  // precomputed planes (spill_endpoint_planes)
  bool sampling_spill = false;
  // more interned services than one chunk's dense service tables (12 B per
  // service) fit beside its rules in the LDS budget: each chunk's tables then
  // index chunk-local ids (the services its rules name, n_services of its
  // SampCfgDev), and the trace stage translates the resources' service ids
  // for each chunk's pass (svc_translate_kernel; the trace kernels are
  // unchanged).  Map: [chunk][global id] -> local id or 0xFFFFFFFF.
  bool sampling_local_svc = false;
  std::vector<std::vector<uint32_t>> sampling_svc_map_host;
  std::vector<uint32_t*> sampling_svc_map_dev;
  uint32_t** sampling_svc_maps_dev = nullptr;   // the K map pointers on the device (ShardArgs / OwnerArgs::svc_maps)
  // span_attribute rules: all of them (attr_n_rules), the GPU-evaluated ones
  // (attr_n_dev, attr_kernel.hip) and the keys those read
  std::vector<uint8_t> attr_blob_host;
  uint8_t* attr_blob_dev = nullptr;
  uint32_t attr_n_rules = 0, attr_n_dev = 0;
  uint64_t attr_host_rules = 0;              // rules 0..63 of attr_host_words (ose_engine_info)
  std::vector<uint64_t> attr_host_words;     // the shim-evaluated rules, one bit per rule
  uint32_t attr_words = 1;                   // attr_match words per span: (attr_n_rules + 63) / 64, >= 1
  uint8_t* attr_host_mask_dev = nullptr;     // attr_host_words on the device (AttrArgs::host_mask)
  bool attr_host_rules_any() const {
    for (uint64_t w : attr_host_words)
      if (w) return true;
    return false;
  }
  std::vector<std::string> attr_keys;

  std::mutex mu;
  std::vector<Workspace*> pool, free_ws;
  std::vector<void*> batch_pool;   // released ose_batch slabs (batch.cpp)
  OtlpEngine* otlp = nullptr;      // OTLP ingest tables, built on first use (otlp_host.cpp)
  std::vector<void*> otlp_pool;    // released ose_otlp_batch objects
  std::vector<void*> enc_pool;     // encoder workspaces of released ose_otlp_out objects
  size_t batch_pool_bytes = 0;

  // ose_profile_*: (kernel name, start, stop) per launch
  bool profiling = false;
  struct Timed { const char* name; hipEvent_t a, b; };
  std::vector<Timed> timed;
  std::vector<hipEvent_t> event_pool;
  hipEvent_t take_event();
  void prof_begin(const char* name, hipStream_t st, Timed& t);
  void prof_end(Timed& t, hipStream_t st);

  ~Engine();
  Workspace* acquire_ws(hipStream_t st);
  void release_ws(Workspace* w, hipStream_t st);
  void return_unused_ws(Workspace* w);
  std::vector<hipStream_t> streams, free_streams;   // ose_process (host batches)
  hipStream_t take_stream();
  void give_stream(hipStream_t s);
  int build_sampling_tables();
  int build_attr_tables();
  size_t workspace_bytes(uint64_t n_spans, uint64_t arena_bytes) const;   // every configured stage
};

// tail != nullptr (OSE_GROUP_TRACE_ID only): queue the fast path, then hand
// back in *tail the rest of the stage (slow path if the fast path saw a
// repeated trace id, per-trace compaction); the caller queues other work on
// the stream first and calls *tail before anything that reads keep
int run_sampling(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t group_mode, const ose_rand* rnd,
                 hipStream_t st, Workspace* ws, std::function<int()>* tail = nullptr);
size_t sampling_scratch_bytes(uint64_t n_spans);
// the attr_match bits the trace stage reads for this call (attr_host.cpp)
int resolve_attr_match(Engine* e, const ose_columns* c, Workspace* ws, hipStream_t st, const uint64_t** out);
// size stage scratch at workspace byte `off` (size_host.cpp)
int run_size(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t mask, uint32_t group_mode,
             const ose_rand* rnd, hipStream_t st, Workspace* ws, size_t off);
struct SizeKernelArgs;
int prepare_size(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t mask, uint32_t group_mode,
                 const ose_rand* rnd, hipStream_t st, Workspace* ws, size_t off, SizeKernelArgs& a, bool& active);
uint32_t* size_partials_of(Workspace* ws, size_t off, uint64_t n_scopes, uint64_t n_resources);
int run_size_tail(Engine* e, const SizeKernelArgs& a, hipStream_t st);
size_t size_scratch_bytes(uint64_t n_scopes, uint64_t n_resources);
// every rule chunk's endpoint bits of the spans as planes of n words (a
// config with spilled route bytes: Engine::sampling_spill), sampling_host.cpp
int spill_endpoint_planes(Engine* e, const ose_columns* c, Workspace* ws, hipStream_t st, const uint64_t** out);
int run_stages(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t mask, uint32_t group_mode,
               const ose_rand* rnd, hipStream_t st);

}  // namespace ose
