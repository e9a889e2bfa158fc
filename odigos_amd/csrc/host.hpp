// host.hpp — C++ mirror of the three processors' Go operator interface
// (processor.Factory -> CreateTraces -> ProcessTracesFunc) above the C ABI.
//
//   NewFactory()                     odigossamplingprocessor/factory.go:13-19,
//                                    odigosurltemplateprocessor/factory.go:19-25,
//                                    odigostrafficmetrics/factory.go:18-26
//   Factory::CreateDefaultConfig()   sampling factory.go:21-27 (empty rule lists),
//                                    urltemplate factory.go:27-29 (&Config{}),
//                                    trafficmetrics factory.go:28-32 (SamplingRatio 1.0)
//   Factory::CreateTraces()          decode + Validate, then the engine
//   TracesProcessor::ProcessTraces() columnarise -> ose_process -> apply
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/odigos_amd.h"
#include "config.hpp"
#include "pdata.hpp"
#include "columnize.hpp"
#include "span_attr.hpp"

namespace ose {

// Host-owned columnar image of one ptrace.Traces (plus output buffers).
struct HostBatch {
  Traces td;
  ose_columns cols{};
  ose_outputs outs{};
  std::vector<uint8_t> arena;               // 16-byte aligned via arena_storage
  std::vector<uint64_t> trace_id, start, end, attr_match;
  uint32_t attr_words = 1;   // attr_match words per span (word-major)
  std::vector<uint8_t> status, kind, url_flags;
  std::vector<uint32_t> resource, scope, span_size, name_len;
  std::vector<ose_strref> path, route;
  std::vector<uint32_t> res_svc, res_svc_str, res_attrset, res_size, scope_size, scope_resource;
  std::vector<uint8_t> res_url_ok;
  std::vector<uint8_t> attr_type;           // key-major [n_attr_keys * n]
  std::vector<uint64_t> attr_val;
  // outputs
  std::vector<uint8_t> keep, trace_keep, trace_level, url_out, tmpl_arena;
  std::vector<uint32_t> trace_count, trace_first_span, device_status;
  std::vector<double> trace_ratio;
  std::vector<ose_strref> tmpl;
  std::vector<int64_t> attrset_bytes, accepted;
  std::vector<uint64_t> res_bytes, tmpl_used;
  std::vector<std::vector<std::pair<std::string, std::string>>> attrsets;   // id -> attribute.Set
  void bind();   // point cols/outs at the vectors
};

enum class ProcKind { Sampling, UrlTemplate, TrafficMetrics, Pipeline };

struct Counter {   // one otel Int64Counter data point
  std::vector<std::pair<std::string, std::string>> attrs;
  int64_t value = 0;
};

class TracesProcessor {
 public:
  TracesProcessor(ProcKind k, const Json& cfg);
  ~TracesProcessor();
  const std::string& error() const { return err_; }
  ProcKind kind() const { return kind_; }
  uint32_t stages() const;
  // processTraces; returns 0 or an OSE_E* code (the hot path never fails in
  // the reference; an engine failure here is surfaced, never masked).
  // Re-entrant: receivers and groupbytrace call ConsumeTraces from several
  // goroutines.  phase_s (optional, 5 entries) accumulates the seconds spent
  // in columnarise / pinned fill / ose_process / read-back / apply.
  int ProcessTraces(Traces& td, double* phase_s = nullptr);
  // test seams: the same steps without the device
  std::unique_ptr<HostBatch> Columnarize(const Traces& td, bool keep_copy = false) const;
  void Apply(HostBatch& hb, Traces& td);
  std::string MetricsJson() const;
  void set_seed(uint64_t s) { seed_ = s; }
  uint32_t group_mode = OSE_GROUP_BATCH;   // one ConsumeTraces call = one trace (rule_engine.go)

 private:
  ProcKind kind_;
  std::string err_;
  Json cfg_json_;
  UrlTemplateConfig url_;
  SamplingConfig sampling_;
  TrafficMetricsConfig traffic_;
  bool has_url_ = false, has_sampling_ = false, has_traffic_ = false;
  ColumnizeCtx ctx_;   // the walk's view of the config (columnize.hpp)
  ose_engine* eng_ = nullptr;
  uint64_t seed_ = 0x0D16A5EEDull;
  uint64_t draws_ = 0;
  // traffic metrics state (otelcol_odigos_trace_data_size / _accepted_spans)
  std::map<std::vector<std::pair<std::string, std::string>>, int64_t> data_size_;
  int64_t accepted_spans_ = 0;
  // guards eng_ creation, the rand.Float64 stream and the traffic counters
  // (the reference's otel counters and math/rand are goroutine-safe)
  mutable std::mutex mu_;
  int ensure_engine();
  double next_uniform();
};

// Interned service ids, in the ABI-defined order (first appearance scanning
// global_rules, service_rules, endpoint_rules in config order).
std::map<std::string, uint32_t> intern_services(const SamplingConfig& c);

}  // namespace ose
