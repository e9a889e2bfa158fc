// sampling_host.cpp — odigossampling: rule tables (built once per engine)
// and the launch sequence of the trace stage (trace_kernel.hip).
#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>
#include <cstdlib>
#include <cstring>

#include "devcfg.hpp"
#include "engine_internal.hpp"
#include "host.hpp"
#include "kernels.hpp"

namespace ose {

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {
size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
uint64_t windows_of(uint64_t n) { return std::max<uint64_t>(1, (n + 63) / 64); }
uint64_t table_slots(uint64_t n) {
  uint64_t cap = 1024;
  while (cap < 2 * n) cap <<= 1;
  return cap;
}
}  // namespace

// Interns every service name a rule compares against (latency.go:55,
// servicename.go:40, spanattribute.go:130); the shim maps resources onto
// these ids with ose_engine_service_id.  Then lays out the device tables
// (devcfg.hpp SampCfgDev): rules in level order global, service, endpoint
// (rule_engine.go:56-60), config order within a level.
namespace {
// One chunk's device tables (devcfg.hpp SampCfgDev): the rules `pick` holds
// (level, rule, global span_attribute index or -1), in the order given.
struct PickedRule {
  int level;
  const SamplingRule* r;
  int attr_index;
};
int build_sampling_blob(const std::unordered_map<std::string, uint32_t>& service_ids, const std::vector<PickedRule>& pick,
                        std::vector<uint8_t>& b, bool& has_attr, bool spill = false) {
  const uint32_t nsvc = (uint32_t)service_ids.size();
  std::vector<SampRuleDev> rules;
  std::vector<SampLatDev> lat;
  std::vector<uint32_t> svc_slot(std::max<uint32_t>(nsvc, 1), 0xFFFFFFFFu);
  std::vector<uint64_t> slot_rules;
  std::vector<uint64_t> svc_bits(std::max<uint32_t>(nsvc, 1), 0);
  std::string bytes;
  SampCfgDev h{};
  // A service_name rule is matched and satisfied iff some span's service is
  // the rule's (servicename.go:35-51): rules naming the same service share
  // one per-trace bit, so the bits count distinct services, not rules.
  std::map<std::string, uint32_t> svc_rule_bit;
  uint32_t n_svc_bits = 0, n_attr = 0;
  int attr_base = -1;
  for (const PickedRule& pr : pick) {
    if (pr.r->rtype == RuleType::ServiceName && svc_rule_bit.emplace(pr.r->service.service_name, n_svc_bits).second)
      n_svc_bits++;
    if (pr.r->rtype == RuleType::SpanAttribute) {
      if (attr_base < 0) attr_base = pr.attr_index;
      n_attr++;
    }
  }
  if (n_svc_bits + n_attr > kMaxServiceRules) return 1;
  size_t k = 0;
  for (int L = 0; L < 3; L++) {
    h.level_first[L] = (uint32_t)rules.size();
    for (; k < pick.size() && pick[k].level == L; k++) {
      const SamplingRule& r = *pick[k].r;
      SampRuleDev d{};
      switch (r.rtype) {
        case RuleType::Error:
          d.type = kSampError;
          d.fallback = r.error.fallback_sampling_ratio;
          break;
        case RuleType::HttpLatency: {
          if (lat.size() >= kMaxLatencyRules) return 1;
          d.type = kSampLatency;
          d.bit = (uint32_t)lat.size();
          d.fallback = r.latency.fallback_sampling_ratio;
          const uint32_t s = service_ids.at(r.latency.service_name);
          if (svc_slot[s] == 0xFFFFFFFFu) {
            svc_slot[s] = (uint32_t)slot_rules.size();
            slot_rules.push_back(0);
          }
          SampLatDev ld{};
          ld.slot = svc_slot[s];
          ld.route_off = (uint32_t)bytes.size();
          ld.route_len = (uint32_t)r.latency.http_route.size();
          ld.threshold = r.latency.threshold;
          // Milliseconds() >= threshold  <=>  ns >= threshold * 1e6 for threshold >= 1
          // (truncation toward zero; Validate rejects threshold <= 0)
          ld.threshold_ns = r.latency.threshold <= INT64_MAX / 1000000 ? r.latency.threshold * 1000000 : INT64_MAX;
          for (uint32_t q = 0; q < 16 && q < ld.route_len; q++) {
            ld.pre[q / 4] |= (uint32_t)(uint8_t)r.latency.http_route[q] << (8 * (q % 4));
            ld.msk[q / 4] |= 0xFFu << (8 * (q % 4));
          }
          bytes += r.latency.http_route;
          slot_rules[ld.slot] |= 1ull << d.bit;
          lat.push_back(ld);
          break;
        }
        case RuleType::ServiceName:
          d.type = kSampService;
          d.bit = svc_rule_bit.at(r.service.service_name);
          d.ratio = r.service.sampling_ratio;
          d.fallback = r.service.fallback_sampling_ratio;
          svc_bits[service_ids.at(r.service.service_name)] |= 1ull << d.bit;
          break;
        case RuleType::SpanAttribute:
          // the shim evaluates the per-span condition (attr_match column,
          // odigos_amd/csrc/span_attr.cpp); the trace stage ORs the bits per
          // trace: satisfied iff any span met it, never matched-but-unsatisfied
          // (spanattribute.go:126-320), i.e. a service_name-shaped rule
          d.type = kSampService;
          d.bit = n_svc_bits + (uint32_t)(pick[k].attr_index - attr_base);
          d.ratio = r.attr.sampling_ratio;
          d.fallback = r.attr.fallback_sampling_ratio;
          break;
      }
      rules.push_back(d);
    }
  }
  h.level_first[3] = (uint32_t)rules.size();
  h.n_rules = (uint32_t)rules.size();
  h.n_lat = (uint32_t)lat.size();
  h.n_lat_slots = (uint32_t)slot_rules.size();
  h.n_services = nsvc;
  h.n_attr = n_attr;
  h.attr_shift = n_svc_bits;
  h.attr_base = attr_base < 0 ? 0u : (uint32_t)attr_base;
  if (slot_rules.empty()) slot_rules.push_back(0);
  b.assign(sizeof(SampCfgDev), 0);
  auto put = [&](const void* p, size_t nb) {
    while (b.size() % 16) b.push_back(0);
    uint32_t off = (uint32_t)b.size();
    const uint8_t* src = static_cast<const uint8_t*>(p);
    b.insert(b.end(), src, src + nb);
    return off;
  };
  h.rules_off = put(rules.data(), rules.size() * sizeof(SampRuleDev));
  h.lat_off = put(lat.data(), lat.size() * sizeof(SampLatDev));
  h.svc_slot_off = put(svc_slot.data(), svc_slot.size() * 4);
  h.slot_rules_off = put(slot_rules.data(), slot_rules.size() * 8);
  h.svc_bits_off = put(svc_bits.data(), svc_bits.size() * 8);
  h.bytes_off = put(bytes.data(), bytes.size());
  while (b.size() % 16) b.push_back(0);
  b.resize(b.size() + 16, 0);
  h.total_bytes = (uint32_t)b.size();
  // the trace kernels copy the table into LDS: all of it, or with spill
  // (a chunk of one rule whose http_route alone does not fit) everything but
  // the route bytes past kSampCfgLds, which they read from HBM
  if (h.total_bytes > kSampCfgLds && !(spill && h.bytes_off + 16 <= kSampCfgLds)) return 1;
  std::memcpy(b.data(), &h, sizeof h);
  has_attr = n_attr > 0;
  return 0;
}
}  // namespace

// Interns every service name a rule compares against (latency.go:55,
// servicename.go:40, spanattribute.go:130); the shim maps resources onto
// these ids with ose_engine_service_id.  Then lays out the device tables
// (devcfg.hpp SampCfgDev): rules in level order global, service, endpoint
// (rule_engine.go:56-60), config order within a level.  A rule list beyond
// one table's bounds (64 latency bits, 64 service + span_attribute bits,
// kSampCfgLds bytes) is cut into consecutive chunks, each as large as fits
// (a rule whose route alone does not fit: a chunk of its own whose route
// bytes past kSampCfgLds the kernels read from HBM);
// the trace stage then runs once per chunk and carries ShouldSample's walk
// from one to the next (trace_kernel.hip decide_chunk), so every config
// Validate accepts runs (the span_attribute bits of a span stay one 64-bit
// attr_match word: at most 64 span_attribute rules, as columnize.cpp).
int Engine::build_sampling_tables() {
  service_ids.clear();
  sampling_chunks_host.clear();
  sampling_chunk_attr.clear();
  if (!has_sampling) return 0;
  for (auto& kv : intern_services(sampling)) service_ids.emplace(kv.first, kv.second);
  const std::vector<SamplingRule>* levels[3] = {&sampling.global_rules, &sampling.service_rules,
                                                &sampling.endpoint_rules};
  std::vector<PickedRule> all;
  uint32_t n_lat = 0, n_attr = 0;
  for (int L = 0; L < 3; L++)
    for (const SamplingRule& r : *levels[L]) {
      all.push_back(PickedRule{L, &r, r.rtype == RuleType::SpanAttribute ? (int)n_attr : -1});
      n_attr += r.rtype == RuleType::SpanAttribute;
      n_lat += r.rtype == RuleType::HttpLatency;
    }
  sampling_lat_svc.assign(std::max<size_t>(1, (service_ids.size() + 31) / 32), 0u);
  for (const PickedRule& pr : all)
    if (pr.r->rtype == RuleType::HttpLatency) {
      const uint32_t s = service_ids.at(pr.r->latency.service_name);
      sampling_lat_svc[s >> 5] |= 1u << (s & 31);
    }
  // greedy: extend the chunk while its tables fit (a rule that alone does not
  // fit: its route bytes or the service tables exceed kSampCfgLds).  The
  // service tables are dense over every interned id while that fits beside a
  // rule; past it (about a thousand services) each chunk indexes the
  // services its own rules name (sampling_local_svc).
  sampling_svc_map_host.clear();
  sampling_local_svc = service_ids.size() * 12 > kSampCfgLds / 2;
  // a chunk's local ids: its rules' services in first-appearance order
  auto local_ids = [&](const std::vector<PickedRule>& cur) {
    std::unordered_map<std::string, uint32_t> loc;
    for (const PickedRule& pr : cur) {
      const std::string* nm = pr.r->rtype == RuleType::HttpLatency   ? &pr.r->latency.service_name
                              : pr.r->rtype == RuleType::ServiceName ? &pr.r->service.service_name
                                                                     : nullptr;
      if (nm) loc.emplace(*nm, (uint32_t)loc.size());
    }
    return loc;
  };
  auto blob_of = [&](const std::vector<PickedRule>& cur, std::vector<uint8_t>& b, bool& a, bool spill) {
    return sampling_local_svc ? build_sampling_blob(local_ids(cur), cur, b, a, spill)
                              : build_sampling_blob(service_ids, cur, b, a, spill);
  };
  size_t k = 0;
  do {
    std::vector<PickedRule> cur;
    std::vector<uint8_t> fitted, blob;
    bool fitted_attr = false, attr = false;
    if (blob_of(cur, fitted, fitted_attr, false))
      return fail(OSE_ENOTSUP, "odigossampling service tables exceed " + std::to_string(kSampCfgLds) +
                                   " bytes (the GPU trace stage keeps them in LDS): too many distinct service names");
    for (; k < all.size(); k++) {
      cur.push_back(all[k]);
      if (blob_of(cur, blob, attr, false)) {
        cur.pop_back();
        break;
      }
      fitted.swap(blob);
      fitted_attr = attr;
    }
    if (cur.empty() && k < all.size()) {
      // one rule whose http_route alone overflows the LDS table: its own
      // chunk, the route bytes past kSampCfgLds read from HBM by the kernels
      cur.push_back(all[k]);
      if (blob_of(cur, fitted, fitted_attr, true))
        return fail(OSE_ENOTSUP, "odigossampling rule tables exceed " + std::to_string(kSampCfgLds) +
                                     " bytes before their route bytes (the GPU trace stage keeps them in LDS)");
      k++;
    }
    if (sampling_local_svc) {
      const auto loc = local_ids(cur);
      std::vector<uint32_t> map(std::max<size_t>(service_ids.size(), 1), 0xFFFFFFFFu);
      for (const auto& kv : service_ids) {
        auto it = loc.find(kv.first);
        if (it != loc.end()) map[kv.second] = it->second;
      }
      sampling_svc_map_host.push_back(std::move(map));
    }
    sampling_chunks_host.push_back(std::move(fitted));
    sampling_chunk_attr.push_back(fitted_attr ? 1 : 0);
  } while (k < all.size());
  sampling_blob_host = sampling_chunks_host[0];
  sampling_n_lat = n_lat;
  sampling_spill = false;
  for (const auto& blob : sampling_chunks_host)
    sampling_spill |= reinterpret_cast<const SampCfgDev*>(blob.data())->total_bytes > kSampCfgLds;
  sampling_n_attr = n_attr;
  return 0;
}

// Scratch of the trace stage for n spans (run_sampling layout).
size_t sampling_scratch_bytes(uint64_t n) {
  const uint64_t W = windows_of(n);
  const uint64_t N = std::max<uint64_t>(n, 1);
  const uint64_t T = (N + kSortTile - 1) / kSortTile;
  const uint64_t wtiles = (W + kScanTileItems - 1) / kScanTileItems;
  const uint64_t htiles = (256 * T + kScanTileItems - 1) / kScanTileItems;
  size_t s = 256;
  s = align_up(s + 8 * W, 256);        // win_heads
  s = align_up(s + 4 * W, 256);        // win_base
  s = align_up(s + 8 * wtiles, 256);   // scan status (windows)
  s = align_up(s + 16 * N, 256);       // rec
  s = align_up(s + 4 * N, 256) * 1;    // key
  s = align_up(s + 4 * N, 256);        // keys2
  s = align_up(s + 4 * N, 256);        // vals
  s = align_up(s + 4 * N, 256);        // keys3
  s = align_up(s + 4 * N, 256);        // vals2
  s = align_up(s + 4 * 256 * T, 256);  // hist
  s = align_up(s + 4 * 256 * T, 256);  // hist offsets
  s = align_up(s + 8 * htiles, 256);   // scan status (hist)
  s = align_up(s + 4 * (N / 64 + 1), 256);   // long runs
  s = align_up(s + 16 * (N / 64 + 1), 256);  // long-run meta
  s = align_up(s + 8 * long_piece_cap(N), 256);   // long-run pieces
  s = align_up(s + (size_t)kLongPartBytes * long_part_cap(N), 256);   // piece partials
  s = align_up(s + 8 * W, 256);        // win_first (run-list path)
  return s + 256;
}

// the workspace of a call running every configured stage (run_stages'
// layout: SAMPLE's scratch, the URL scratch after it, the size sums after
// that; scopes and resources bounded by the spans)
size_t Engine::workspace_bytes(uint64_t n_spans, uint64_t arena_bytes) const {
  size_t s = has_sampling ? align_up(sampling_scratch_bytes(n_spans), 256) : 0;
  if (has_url) s = align_up(s + url_workspace_bytes(n_spans, arena_bytes), 256);
  if (has_traffic) s += size_scratch_bytes(n_spans, n_spans);
  return s;
}

// Run lists of the run-list path (allocated the first time a batch repeats
// a trace id; sized like the exact table).
int Workspace::reserve_runs() {
  if (runs && runs_slots >= table_slots_cap) return 0;
  if (runs) HIP_TRY(hipFree(runs));
  if (run_count) HIP_TRY(hipFree(run_count));
  runs = run_count = nullptr;
  runs_slots = 0;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&runs), table_slots_cap * kMaxRuns * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&run_count), table_slots_cap * sizeof(uint32_t)));
  runs_slots = table_slots_cap;
  return 0;
}

int Workspace::reserve_table(uint64_t n_spans) {
  const uint64_t slots = table_slots(n_spans);
  if (slots <= table_slots_cap) return 0;
  if (table) HIP_TRY(hipFree(table));
  if (dup_bkt) HIP_TRY(hipFree(dup_bkt));
  if (dup_bkt_count) HIP_TRY(hipFree(dup_bkt_count));
  table = nullptr;
  dup_bkt = nullptr;
  dup_bkt_count = nullptr;
  table_slots_cap = 0;
  HIP_TRY(hipMalloc(&table, slots * sizeof(TraceSlot)));
  HIP_TRY(hipMemset(table, 0, slots * sizeof(TraceSlot)));
  // fingerprint buckets: half full (on average) at one run head per 4 spans;
  // at least 2 (the bucket is the fingerprint's top dup_bkt_bits bits)
  dup_bkt_bits = 1;
  while ((uint64_t(kDupBucketCap) / 2 << dup_bkt_bits) < n_spans / 4) dup_bkt_bits++;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dup_bkt), (size_t(kDupBucketCap) << dup_bkt_bits) * sizeof(uint64_t)));
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dup_bkt_count), (size_t(1) << dup_bkt_bits) * sizeof(uint32_t)));
  table_slots_cap = slots;
  epoch = 0;
  return 0;
}

int Workspace::reserve_fold(uint64_t n_spans) {
  if (fold_cap >= n_spans && fold[0]) return 0;
  for (void*& f : fold) {
    if (f) HIP_TRY(hipFree(f));
    f = nullptr;
  }
  fold_cap = 0;
  for (void*& f : fold) HIP_TRY(hipMalloc(&f, n_spans * sizeof(FoldState)));
  fold_cap = n_spans;
  return 0;
}

int local_service_ids(Engine* e, const ose_columns* c, Workspace* ws, hipStream_t st, uint32_t chunk,
                      const uint32_t** out);

namespace {
// LDS bytes of every chunk's table (trace_multi_kernel's copy)
uint32_t multi_cfg_bytes(const Engine* e) {
  uint32_t t = 0;
  for (const auto& h : e->sampling_chunks_host) {
    const uint32_t nb = std::min<uint32_t>(reinterpret_cast<const SampCfgDev*>(h.data())->total_bytes, kSampCfgLds);
    t += (nb + 15u) & ~15u;
  }
  return t + (uint32_t)align_up(4 * e->service_ids.size() + 4 * 64, 16) +
         (uint32_t)(e->sampling_chunks_host.size() * sizeof(SampWalkDev));
}
// trace_multi_kernel takes the call: 2..kMaxMulti chunks whose tables fit
// kMultiCfgLds together, no span_attribute rules, no spilled routes, spans
// grouped by trace id in batch order with their own route columns
bool multi_pass(const Engine* e, const ose_columns* c, uint32_t group_mode) {
  const size_t K = e->sampling_chunks_host.size();
  return K >= 2 && K <= kMaxMulti && group_mode == OSE_GROUP_TRACE_ID && c->n_spans && !e->sampling_n_attr &&
         !e->sampling_local_svc &&
         e->sampling_n_lat_svc <= 64 && e->sampling_walk_ok &&
         !e->sampling_spill && !c->route_match && !c->svc_match && multi_cfg_bytes(e) <= kMultiCfgLds;
}

// One pass of the trace stage over the rule tables of `chunk`; fold_in /
// fold_out: the FoldState before / after this chunk's rules (run_sampling)
int run_sampling_pass(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t group_mode, const ose_rand* rnd,
                      hipStream_t st, Workspace* ws, std::function<int()>* tail, uint32_t chunk,
                      const FoldState* fold_in, FoldState* fold_out, uint32_t multi = 0,
                      std::function<int()> redo = nullptr) {
  if (!e->has_sampling) return fail(OSE_EINVAL, "odigossampling is not configured on this engine");
  if (group_mode != OSE_GROUP_TRACE_ID && group_mode != OSE_GROUP_BATCH) return fail(OSE_EINVAL, "unknown group_mode");
  const uint64_t n = c->n_spans;
  if (n > 0xFFFFFFF0ull) return fail(OSE_ERANGE, "SAMPLE stage: more than 2^32-16 spans in one batch");
  const bool lat = e->sampling_n_lat > 0;
  if (n > 0) {
    if (!c->status || !c->resource || !c->res_svc || !c->res_svc_str || !o->keep)
      return fail(OSE_EINVAL, "SAMPLE stage needs status, resource, res_svc, res_svc_str and keep");
    if (!c->trace_id && (group_mode == OSE_GROUP_TRACE_ID || o->trace_keep || o->trace_level || o->trace_ratio))
      return fail(OSE_EINVAL, "SAMPLE stage needs the trace_id column");
    if (lat && (!c->start_ns || !c->end_ns || (!c->route_match && (!c->route || !c->arena))))
      return fail(OSE_EINVAL, "http_latency rules need start_ns, end_ns and route + arena (or route_match)");
  } else if (!c->res_svc_str && c->n_resources) {
    return fail(OSE_EINVAL, "SAMPLE stage needs res_svc_str");
  }
  const bool per_trace = o->trace_count || o->trace_first_span || o->trace_keep || o->trace_level || o->trace_ratio;
  if (group_mode == OSE_GROUP_TRACE_ID && n == 0) {
    if (o->trace_count) HIP_TRY(hipMemsetAsync(o->trace_count, 0, 4, st));
    return 0;
  }
  const uint64_t W = windows_of(n), N = std::max<uint64_t>(n, 1);
  const uint64_t T = (N + kSortTile - 1) / kSortTile;
  const uint32_t wtiles = (uint32_t)((W + kScanTileItems - 1) / kScanTileItems);
  const uint32_t htiles = (uint32_t)((256 * T + kScanTileItems - 1) / kScanTileItems);
  const size_t need = sampling_scratch_bytes(n);
  int rc = ws->reserve(need);
  if (rc) return rc;
  if (group_mode == OSE_GROUP_TRACE_ID) {
    rc = ws->reserve_table(n);
    if (rc) return rc;
    // generation tags: 30 bits in the exact table; the table is cleared once
    // when its tag wraps (0 is "never used")
    if (++ws->epoch >= (1u << 30)) {
      HIP_TRY(hipMemsetAsync(ws->table, 0, ws->table_slots_cap * sizeof(TraceSlot), st));
      ws->epoch = 1;
    }
  }
  uint8_t* base = static_cast<uint8_t*>(ws->dev);
  size_t off = 256;
  auto take = [&](size_t bytes) {
    uint8_t* p = base + off;
    off = align_up(off + bytes, 256);
    return p;
  };
  uint32_t* misc = reinterpret_cast<uint32_t*>(base);   // [0] dup, [2] scan counter (windows), [4] scan counter (hist), [12] long runs, [13] their pieces, [14] run-list overflow, [15] piece partials
  uint64_t* win_heads = reinterpret_cast<uint64_t*>(take(8 * W));
  uint32_t* win_base = reinterpret_cast<uint32_t*>(take(4 * W));
  uint64_t* wstatus = reinterpret_cast<uint64_t*>(take(8 * (size_t)wtiles));
  TraceRec* rec = reinterpret_cast<TraceRec*>(take(16 * N));
  uint32_t* key = reinterpret_cast<uint32_t*>(take(4 * N));
  uint32_t* k2 = reinterpret_cast<uint32_t*>(take(4 * N));
  uint32_t* v2 = reinterpret_cast<uint32_t*>(take(4 * N));
  uint32_t* k3 = reinterpret_cast<uint32_t*>(take(4 * N));
  uint32_t* v3 = reinterpret_cast<uint32_t*>(take(4 * N));
  uint32_t* hist = reinterpret_cast<uint32_t*>(take(4 * 256 * T));
  uint32_t* hoff = reinterpret_cast<uint32_t*>(take(4 * 256 * T));
  uint64_t* hstatus = reinterpret_cast<uint64_t*>(take(8 * (size_t)htiles));
  uint32_t* long_runs = reinterpret_cast<uint32_t*>(take(4 * (N / 64 + 1)));
  uint4* long_meta = reinterpret_cast<uint4*>(take(16 * (N / 64 + 1)));
  uint2* long_pieces = reinterpret_cast<uint2*>(take(8 * long_piece_cap(N)));
  uint8_t* long_part = take((size_t)kLongPartBytes * long_part_cap(N));
  uint64_t* win_first = reinterpret_cast<uint64_t*>(take(8 * W));
  if (off > need) return fail(OSE_EINVAL, "internal: trace workspace layout exceeds its bound");
  uint32_t* err = o->device_status ? o->device_status : misc + 8;
  // a later rule-chunk pass keeps the first pass's *dup (misc[0]): the batch's
  // trace-id layout is the same, so it neither registers run heads nor checks
  // buckets again
  const bool reuse_dup = chunk > 0 && group_mode == OSE_GROUP_TRACE_ID;
  if (reuse_dup)
    HIP_TRY(hipMemsetAsync(base + 4, 0, 60, st));
  else
    HIP_TRY(hipMemsetAsync(base, 0, 64, st));

  TraceKernelArgs a{};
  a.n_spans = n;
  a.n_windows = (uint32_t)W;
  a.mode = group_mode == OSE_GROUP_BATCH ? kTraceBatch : kTraceRuns;
  a.n_resources = c->n_resources;
  a.epoch = ws->epoch;
  a.tid = c->trace_id;
  a.start = c->start_ns;
  a.end = c->end_ns;
  a.status = c->status;
  a.resource = c->resource;
  a.route = c->route;
  a.arena = c->arena;
  a.res_svc = c->res_svc;
  a.res_svc_str = c->res_svc_str;
  if (e->sampling_local_svc && c->n_resources && c->res_svc && c->res_svc_str) {   // this chunk's service ids
    const uint32_t* loc = nullptr;
    const int lr = local_service_ids(e, c, ws, st, chunk, &loc);
    if (lr) return lr;
    a.res_svc = loc;
    a.res_svc_str = loc + ws->svc_local_cap;
  }
  a.cfg = e->sampling_chunks_dev[chunk];
  a.fold_in = fold_in;
  a.fold_out = fold_out;
  a.seed = rnd ? rnd->seed : 0;
  a.keep = o->keep;
  a.rec = per_trace ? rec : nullptr;
  a.win_heads = win_heads;
  a.table = static_cast<TraceSlot*>(ws->table);
  a.table_mask = ws->table_slots_cap ? ws->table_slots_cap - 1 : 0;
  a.dup = misc;
  a.error = err;
  a.batch_keep = misc + kBatchKeepWord;
  // match planes (an owner's unpacked records): this chunk's plane
  const uint64_t plane = c->match_planes > 1 ? (uint64_t)chunk * n : 0;
  // the bits in route_match / svc_match are chunk-local rule indices: with
  // more than one chunk every chunk needs its own plane (plane 0 reused for
  // chunk k > 0 would test chunk k's rules against chunk 0's bits)
  if ((c->route_match || c->svc_match) && (e->sampling_chunks_dev.size() > 1 || c->match_planes > 1) &&
      c->match_planes != e->sampling_chunks_dev.size())
    return fail(OSE_EINVAL, "cols->match_planes must equal the engine's rule chunks when route_match / svc_match are set");
  a.route_match = c->route_match ? c->route_match + plane : nullptr;
  {
    const uint64_t* am = nullptr;
    const int ar = resolve_attr_match(e, c, ws, st, &am);
    if (ar) return ar;
    a.attr_match = e->sampling_n_attr && e->sampling_chunk_attr[chunk] ? am : nullptr;
    a.attr_stride = n;
    a.attr_words = e->attr_words;
  }
  a.svc_match = c->svc_match ? c->svc_match + plane : nullptr;
#if OSE_DIAG
  if (const char* ab = getenv("OSE_TRACE_ABLATE")) a.ablate = (uint32_t)strtoul(ab, nullptr, 0);
#endif
  a.n_long = misc + 12;
  a.long_runs = a.mode == kTraceRuns && !multi ? long_runs : nullptr;
  a.long_meta = long_meta;
  a.long_pieces = long_pieces;
  a.long_part = long_part;
  if (multi) {   // every chunk in one pass (run_sampling checked the conditions)
    a.n_multi = multi;
    a.cfgs = reinterpret_cast<const uint8_t* const*>(e->shard_tables_dev);
    a.cfg_lds_bytes = multi_cfg_bytes(e);
    a.lat_gslot = reinterpret_cast<const uint32_t*>(e->shard_tables_dev + 8 * e->sampling_chunks_dev.size() +
                                                    4 * e->sampling_lat_svc.size());
    a.walks = reinterpret_cast<const SampWalkDev*>(
        e->shard_tables_dev + align_up(8 * e->sampling_chunks_dev.size() + 4 * e->sampling_lat_svc.size() +
                                           4 * e->service_ids.size() + 4 * 64, 16));
  }
  a.long_steps = kLongSteps;
  // kWinPerWave windows per wave on large batches; a small one (the drop-in's
  // 8192-span calls: 128 windows) spreads over at least ~4096 waves, one
  // window each, instead of 8 waves walking 16 windows each (112 us -> ~)
  // beside the URL planning (run_stages' fork) a wave takes kWinPerWaveBeside
  // windows: fewer, longer trace workgroups interleave better with the plan
  // grid's (C4 7.63 -> 7.47 ms, C5 3.26 -> 3.12; alone, C3, 16 stays best:
  // profiles/r5w_win_per_wave_ab.txt)
  const uint64_t wpw_cap = ws->beside_url ? kWinPerWaveBeside : kWinPerWave;
  a.win_per_wave = (uint32_t)std::min<uint64_t>(wpw_cap, std::max<uint64_t>(1, a.n_windows / 4096));
  {
    // the error bit, the endpoint bits and the service (+ span_attribute)
    // bits in one word: trace_eval_kernel's kNarrow instance (C4 trace_eval
    // 2.79 -> 2.65 ms, C3 1.41 -> 1.35 ms: profiles/r4e_narrow_ab.txt)
    const SampCfgDev* h = reinterpret_cast<const SampCfgDev*>(e->sampling_chunks_host[chunk].data());
    const uint32_t svc_bits = h->attr_shift + (a.attr_match ? h->n_attr : 0);
    a.narrow = 1 + h->n_lat + svc_bits <= 32 && h->n_lat_slots <= 32 ? 1u : 0u;
  }
#if OSE_DIAG
  if (const char* ww = getenv("OSE_WIN_PER_WAVE")) a.win_per_wave = std::max<uint32_t>(1, (uint32_t)strtoul(ww, nullptr, 0));
  if (const char* ls = getenv("OSE_LONG_STEPS")) a.long_steps = std::max<uint32_t>(1, (uint32_t)strtoul(ls, nullptr, 0));
#endif
  // duplicate detection: fingerprint buckets checked in LDS (replaced a
  // fingerprint table probed with a CAS per head: C4 trace_eval 3.02 -> 2.87
  // ms + 0.06 ms of trace_dup_check, C3 1.55 -> 1.47 + 0.03,
  // profiles/r3_dup_buckets_ab.txt)
  if (a.mode == kTraceRuns && !reuse_dup) {
    if (!ws->dup_bkt || ws->dup_bkt_bits < 1 || ws->dup_bkt_bits > 32)
      return fail(OSE_EDEVICE, "trace stage: duplicate-detection buckets missing");
    a.dup_bkt = ws->dup_bkt;
    a.dup_bkt_count = ws->dup_bkt_count;
    a.dup_bkt_bits = ws->dup_bkt_bits;
    HIP_TRY(hipMemsetAsync(a.dup_bkt_count, 0, sizeof(uint32_t) << a.dup_bkt_bits, st));
  }
  Engine::Timed tm{};
  e->prof_begin(multi ? "trace_multi_kernel" : "trace_eval_kernel", st, tm);
  launch_trace_eval(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  if (a.dup_bkt) {
    Engine::Timed td{};
    e->prof_begin("trace_dup_check", st, td);
    launch_trace_dup_check(a, st);
    HIP_TRY(hipGetLastError());
    e->prof_end(td, st);
  }
  auto long_pass = [=](uint32_t known_runs) -> int {
    e->long_run_passes.fetch_add(1, std::memory_order_relaxed);
    Engine::Timed tl{};
    e->prof_begin("trace_long_kernel", st, tl);
    launch_trace_long(a, st, known_runs);   // (trace_long_plan_kernel, then the pieces)
    HIP_TRY(hipGetLastError());
    e->prof_end(tl, st);
    return 0;
  };
  // host-gated (tail): queued only when the fast path listed long runs
  const bool gate_long = tail && group_mode == OSE_GROUP_TRACE_ID;
  if (a.long_runs && !gate_long) {
    const int lr = long_pass(0);
    if (lr) return lr;
  }

  // the rest of the stage; run_slow = false skips the slow-path launches
  // (they would all return at once: the fast path left *dup clear)
  auto rest = [=](bool run_slow) -> int {
  if (run_slow) {
    // repeated trace ids: the run-list path (every launch returns at once
    // unless the fast path set *dup), then the sort-based path, which runs
    // only when some trace overflowed the run-list path
    int rr = ws->reserve_runs();
    if (rr) return rr;
    uint32_t* overflow = misc + 14;
    TraceKernelArgs rl = a;
    rl.run_count = ws->run_count;
    rl.runs = ws->runs;
    rl.overflow = overflow;
    rl.path_count = e->path_count_dev;
    rl.win_first = win_first;
    rl.head_slot = key;
    Engine::Timed tr{};
    e->prof_begin("trace_run_list", st, tr);
    launch_trace_runs(rl, st);
    HIP_TRY(hipGetLastError());
    launch_trace_fold(rl, st);
    HIP_TRY(hipGetLastError());
    launch_trace_first_select(rl, st);
    HIP_TRY(hipGetLastError());
    e->prof_end(tr, st);
    Engine::Timed ts{};
    e->prof_begin("trace_sort_path", st, ts);
    TraceSortArgs s{};
    s.n_spans = n;
    s.n_tiles = (uint32_t)T;
    s.gate = overflow;
    s.tid = c->trace_id;
    s.table = a.table;
    s.table_mask = a.table_mask;
    s.epoch = a.epoch;
    s.key = key;
    s.error = err;
    s.path_count = e->path_count_dev;
    // (the run-list kernel already put every run head in the exact table)
    launch_trace_key(s, st);
    HIP_TRY(hipGetLastError());
    int bits = 1;
    while (bits < 32 && (n - 1) >> bits) bits++;
    const uint32_t* kin = nullptr;
    const uint32_t* vin = nullptr;
    uint32_t* kbuf[2] = {k2, k3};
    uint32_t* vbuf[2] = {v2, v3};
    int pass = 0;
    for (int shift = 0; shift < bits; shift += 8, pass++) {
      s.shift = (uint32_t)shift;
      s.keys_in = kin;
      s.vals_in = vin;
      s.keys_out = kbuf[pass & 1];
      s.vals_out = vbuf[pass & 1];
      s.hist = hist;
      s.scan_counter = misc + 4;
      s.scan_status = hstatus;
      s.scan_status_n = htiles;
      launch_sort_hist(s, st);
      HIP_TRY(hipGetLastError());
      ScanArgs sa{};
      sa.n = 256 * T;
      sa.n_tiles = htiles;
      sa.popcount = 0;
      sa.gate = overflow;
      sa.in = hist;
      sa.out = hoff;
      sa.counter = misc + 4;
      sa.status = hstatus;
      sa.error = err;
      launch_scan_u32(sa, st);
      HIP_TRY(hipGetLastError());
      TraceSortArgs s2 = s;
      s2.hist = hoff;
      launch_sort_scatter(s2, st);
      HIP_TRY(hipGetLastError());
      kin = kbuf[pass & 1];
      vin = vbuf[pass & 1];
    }
    TraceKernelArgs b = a;
    b.dup = overflow;   // perm-mode evaluation is gated on this word
    b.mode = kTracePerm;
    b.long_runs = nullptr;   // the sorted pass walks every run itself
    b.perm = vin;
    b.key = key;
    launch_trace_eval(b, st);
    HIP_TRY(hipGetLastError());
    e->prof_end(ts, st);
  }

  if (per_trace) {
    HIP_TRY(hipMemsetAsync(wstatus, 0, 8 * (size_t)wtiles, st));
    ScanArgs sa{};
    sa.n = W;
    sa.n_tiles = wtiles;
    sa.popcount = 1;
    sa.in = win_heads;
    sa.out = win_base;
    sa.total = o->trace_count;
    sa.counter = misc + 2;
    sa.status = wstatus;
    sa.error = err;
    launch_scan_u32(sa, st);
    HIP_TRY(hipGetLastError());
    TraceCompactArgs ca{};
    ca.n_windows = (uint32_t)W;
    ca.win_heads = win_heads;
    ca.win_base = win_base;
    ca.rec = rec;
    ca.trace_first_span = o->trace_first_span;
    ca.trace_keep = o->trace_keep;
    ca.trace_level = o->trace_level;
    ca.trace_ratio = o->trace_ratio;
    launch_trace_compact(ca, st);
    HIP_TRY(hipGetLastError());
  }
  return 0;
  };
  if (group_mode != OSE_GROUP_TRACE_ID) return rest(false);
  if (multi) {
    // the one-pass form decides batches without repeated trace ids; one with
    // them (*dup) is redone pass per chunk, whose slow paths handle it
    if (!ws->dup_host) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ws->dup_host), 64, hipHostMallocDefault));
    if (!ws->dup_ready) HIP_TRY(hipEventCreateWithFlags(&ws->dup_ready, hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(ws->dup_host, misc, 64, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(ws->dup_ready, st));
    auto finish = [rest, redo, ws]() -> int {
      HIP_TRY(hipEventSynchronize(ws->dup_ready));
      return ws->dup_host[0] ? redo() : rest(false);
    };
    if (!tail) return finish();
    *tail = finish;
    return 0;
  }
  if (!tail) return rest(true);
  if (!ws->dup_host) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ws->dup_host), 64, hipHostMallocDefault));
  if (!ws->dup_ready) HIP_TRY(hipEventCreateWithFlags(&ws->dup_ready, hipEventDisableTiming));
  // misc[0] = dup, misc[12] = long runs listed by the fast path
  HIP_TRY(hipMemcpyAsync(ws->dup_host, misc, 64, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipEventRecord(ws->dup_ready, st));
  const bool has_long = a.long_runs != nullptr;
  *tail = [rest, long_pass, has_long, ws]() -> int {
    HIP_TRY(hipEventSynchronize(ws->dup_ready));
    if (has_long && ws->dup_host[12]) {   // before the slow path, which rewrites every trace's keep
      const int lr = long_pass(ws->dup_host[12]);
      if (lr) return lr;
    }
    return rest(ws->dup_host[0] != 0);
  };
  return 0;
}

}  // namespace

// The trace stage: one pass per rule chunk (build_sampling_tables); with more
// than one, each pass but the last saves ShouldSample's walk per trace and
// the next resumes it (ping-pong buffers: a pass's provisional fast-path
// decisions for traces the slow path redoes never reach the state it reads).
// Each pass takes its slow paths host-gated; a later pass reuses the first pass's
// duplicate detection (run_sampling_pass).
// A chunk whose http_route bytes spill past the kernels' LDS copy of its
// table: the endpoint bits of every chunk are computed first from the tables
// in HBM (endpoint_plane_kernel), and the trace stage / the pack take them as
// route_match planes, so no kernel reads route bytes past its LDS copy.
// Chunk-local service ids of the batch's resources for rule chunk `chunk`
// (Engine::sampling_local_svc): out = res_svc, out + svc_local_cap =
// res_svc_str, both translated through the chunk's map.
int local_service_ids(Engine* e, const ose_columns* c, Workspace* ws, hipStream_t st, uint32_t chunk,
                      const uint32_t** out) {
  const uint64_t R = c->n_resources;
  int rc = ws->reserve_svc_local(std::max<uint64_t>(R, 1));
  if (rc) return rc;
  launch_svc_translate(e->sampling_svc_map_dev[chunk], (uint32_t)e->service_ids.size(), c->res_svc, c->res_svc_str,
                       ws->svc_local, ws->svc_local + ws->svc_local_cap, R, st);
  HIP_TRY(hipGetLastError());
  *out = ws->svc_local;
  return 0;
}
int Workspace::reserve_svc_local(uint64_t n_resources) {
  if (svc_local && svc_local_cap >= n_resources) return 0;
  if (svc_local) HIP_TRY(hipFree(svc_local));
  svc_local = nullptr;
  svc_local_cap = 0;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&svc_local), 2 * n_resources * sizeof(uint32_t)));
  svc_local_cap = n_resources;
  return 0;
}

int spill_endpoint_planes(Engine* e, const ose_columns* c, Workspace* ws, hipStream_t st, const uint64_t** out) {
  const uint64_t n = c->n_spans, K = e->sampling_chunks_dev.size();
  if (!c->resource || !c->res_svc || !c->route || !c->arena)
    return fail(OSE_EINVAL, "http_latency rules need resource, res_svc, route and arena");
  int rc = ws->reserve_ep_planes(n * K);
  if (rc) return rc;
  for (uint64_t k = 0; k < K; k++) {
    const uint32_t* sv = c->res_svc;
    if (e->sampling_local_svc) {
      rc = local_service_ids(e, c, ws, st, (uint32_t)k, &sv);
      if (rc) return rc;
    }
    launch_endpoint_plane(e->sampling_chunks_dev[k], c->resource, sv, c->route, c->arena, n, ws->ep_planes + k * n, st);
  }
  HIP_TRY(hipGetLastError());
  *out = ws->ep_planes;
  return 0;
}

int run_sampling(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t group_mode, const ose_rand* rnd,
                 hipStream_t st, Workspace* ws, std::function<int()>* tail) {
  const uint32_t K = (uint32_t)e->sampling_chunks_dev.size();
  if (K > 1 && c->svc_match && c->match_planes != K)
    return fail(OSE_EINVAL, "cols->match_planes must equal the engine's rule chunks when svc_match is set");
  // (a batch without route bytes has no endpoint bits to spill: the trace
  // stage refuses a missing route column)
  if (e->sampling_spill && !c->route_match && c->route && e->sampling_n_lat && c->n_spans) {
    const uint64_t* planes = nullptr;
    const int rc = spill_endpoint_planes(e, c, ws, st, &planes);
    if (rc) return rc;
    ws->spill_cols = *c;
    ws->spill_cols.route_match = planes;
    ws->spill_cols.match_planes = K;
    c = &ws->spill_cols;   // outlives this call's stack: the tails below read it later
  }
  if (K <= 1) return run_sampling_pass(e, c, o, group_mode, rnd, st, ws, tail, 0, nullptr, nullptr);
  // (one pass over the columns into partial records carrying every chunk's
  // words, decided by the owner fold, measured slower on sampling_wide:
  // 9.72 ms against 7.65, profiles/r4_owner_fold_forms.txt)
  // one pass per chunk; each pass's slow paths host-gated as in a one-table
  // call (the host waits for the pass's flags; the run-list and sort launches
  // are queued only for a batch with repeated trace ids)
  auto per_chunk = [=]() -> int {
  int rc = ws->reserve_fold(std::max<uint64_t>(c->n_spans, 1));
  if (rc) return rc;
  for (uint32_t k = 0; k < K; k++) {
    const FoldState* in = k ? static_cast<const FoldState*>(ws->fold[(k - 1) & 1]) : nullptr;
    FoldState* out = k + 1 < K ? static_cast<FoldState*>(ws->fold[k & 1]) : nullptr;
    std::function<int()> pass_tail;
    rc = run_sampling_pass(e, c, o, group_mode, rnd, st, ws, &pass_tail, k, in, out);
    if (!rc && pass_tail) rc = pass_tail();
    if (rc) return rc;
  }
  return 0;
  };
  // every chunk in one pass over the columns (trace_multi_kernel; sampling_wide
  // 5.55 -> see DESIGN §4.2); a batch with repeated trace ids falls back to the
  // passes per chunk
  if (multi_pass(e, c, group_mode))
    return run_sampling_pass(e, c, o, group_mode, rnd, st, ws, tail, 0, nullptr, nullptr, K, per_chunk);
  return per_chunk();
}

}  // namespace ose
