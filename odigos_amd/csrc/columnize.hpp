// columnize.hpp — what each reference function reads from pdata, per
// resource and per span: the walk a shim does to fill ose_columns.  Shared
// by the C++ host processors (host.cpp, over pdata built from OTLP/JSON) and
// the OTLP protobuf ingest (otlp_host.cpp: resources on the host, the spans
// the GPU decoder hands back for a host pass).
#pragma once
#include <string_view>
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/odigos_amd.h"
#include "config.hpp"
#include "pdata.hpp"
#include "span_attr.hpp"

namespace ose {

// resourceToWorkloadStringRepresentation (filtermatcher.go:30-84)
bool workload_key(const AttrMap& attrs, std::string& key);
// k8sWorkloadToStringRepresentation of every configured workload (:21-24)
std::set<std::string> workload_set(const MatchProperties& mp);

struct ColumnizeCtx {
  std::map<std::string, uint32_t> services;   // interned rule service names (intern_services)
  bool url_filter = false;                    // include or exclude configured
  bool has_exclude = false, has_include = false;
  std::set<std::string> excl, incl;
  std::vector<std::string> traffic_keys;      // odigostrafficmetrics res_attributes_keys
  std::vector<SpanAttrPredicate> attr_preds;  // every span_attribute rule, level order
  AttrPlan attr_plan;                         // which ones the GPU evaluates, from which key column
  std::string build(const UrlTemplateConfig* url, const SamplingConfig* sampling, const TrafficMetricsConfig* traffic);
};

// per-resource columns (service ids, include/exclude, attribute set, and the
// span_attribute rules whose service this resource is)
struct ResourceCols {
  uint32_t svc = OSE_NONE, svc_str = OSE_NONE;
  uint8_t url_ok = 1;
  std::vector<uint64_t> attr_res;   // span_attribute rules whose service this resource is (64 per word)
  std::vector<std::pair<std::string, std::string>> attrset;   // attribute.NewSet: sorted, last value wins
};
ResourceCols columnize_resource(const ColumnizeCtx& c, const AttrMap& ra);

// per-span columns; strings are returned as views (the caller places them):
// into the span's own values when they are Str, else into the owned
// conversions below (AsString of a non-Str route, a path parsed from url.full),
// so the common case copies no string.  Views are valid while the span and
// this SpanCols are.
struct SpanCols {
  uint64_t hi = 0, lo = 0, start = 0, end = 0;
  uint8_t status = 0, kind = 0, url_flags = 0;
  uint32_t span_size = 0, name_len = 0;
  std::vector<uint64_t> attr_match;           // bits of the shim-evaluated (json) rules (64 per word)
  bool has_route = false;
  std::string_view route, path;               // AsString(http.route); the url path source
  std::string route_own, path_own;            // their storage when converted
  std::vector<uint8_t> attr_type;             // per GPU key column
  std::vector<uint64_t> attr_val;             // STR values: placeholder, see attr_str
  std::vector<std::string_view> attr_str;     // STR values' bytes (per key; empty otherwise)
};
void columnize_span(const ColumnizeCtx& c, const Span& sp, const std::vector<uint64_t>& attr_res, const ProtoSizer& sizer,
                    SpanCols& out);

// ptrace.StatusCode as the status column: 0/1/2 as they are, anything else
// (not a valid code) 3 — only == OSE_STATUS_ERROR matters to the rules, and
// bit 7 of the column is reserved for the exchange's owner-side records
inline uint8_t status_column(int32_t code) { return code >= 0 && code <= 2 ? (uint8_t)code : (uint8_t)3; }

}  // namespace ose
