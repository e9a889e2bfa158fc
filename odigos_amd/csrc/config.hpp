// config.hpp — the three processors' Config structs, decoded from the
// mapstructure-shaped JSON the collector's confmap would hand to
// Factory.CreateTraces, and validated with the reference's messages.
//
//   odigossampling        odigossamplingprocessor/config.go:11-80,
//                         internal/sampling/{error,latency,servicename,spanattribute}.go
//   odigosurltemplate     odigosurltemplateprocessor/config.go:11-158
//   odigostrafficmetrics  odigostrafficmetrics/config.go:9-29, factory.go:27-32
#pragma once
#include <optional>
#include <string>
#include <vector>

#include "json.hpp"

namespace ose {

// ---------------- odigosurltemplate ----------------
struct K8sWorkload {
  std::string namespace_, kind, name;   // mapstructure: namespace, kind, name
};
struct MatchProperties {
  std::vector<K8sWorkload> k8s_workloads;   // k8s_workloads
};
struct CustomIdConfig {
  std::string regexp, template_name;        // regexp, template_name
};
struct UrlTemplateConfig {
  std::optional<MatchProperties> exclude, include;   // MatchConfig (,squash)
  std::vector<std::string> templatization_rules;      // TemplatizationConfig (,squash)
  std::vector<CustomIdConfig> custom_ids;
};

// ---------------- odigossampling ----------------
enum class RuleType { HttpLatency, Error, SpanAttribute, ServiceName };
struct HttpRouteLatencyRule {      // latency.go:12-17
  std::string http_route;
  int64_t threshold = 0;
  std::string service_name;
  double fallback_sampling_ratio = 0;
};
struct ErrorRule {                 // error.go:9-13
  double fallback_sampling_ratio = 0;
};
struct ServiceNameRule {           // servicename.go:10-14
  std::string service_name;
  double sampling_ratio = 0;
  double fallback_sampling_ratio = 0;
};
struct SpanAttributeRule {         // spanattribute.go:25-34
  std::string service_name, attribute_key, condition_type, operation, expected_value, json_path;
  double sampling_ratio = 0, fallback_sampling_ratio = 0;
};
struct SamplingRule {              // config.go:28-32
  std::string name, type;
  RuleType rtype = RuleType::Error;
  HttpRouteLatencyRule latency;
  ErrorRule error;
  ServiceNameRule service;
  SpanAttributeRule attr;
};
struct SamplingConfig {            // config.go:11-15
  std::vector<SamplingRule> global_rules, service_rules, endpoint_rules;
};

// ---------------- odigostrafficmetrics ----------------
struct TrafficMetricsConfig {      // config.go:9-18; default SamplingRatio 1.0 (factory.go:27-32)
  std::vector<std::string> res_attributes_keys;
  double sampling_ratio = 1.0;
};

// Each decode_* returns "" on success or the error the Go code would return
// (mapstructure decode error, then Validate()).
std::string decode_url_config(const Json& j, UrlTemplateConfig& out);
std::string decode_sampling_config(const Json& j, SamplingConfig& out);
std::string decode_traffic_config(const Json& j, TrafficMetricsConfig& out);

// Rule-string parsing shared by Validate and the compiled tables
// (templatize.go:97-190).
enum class SegKind { Static, Wildcard, Template, Regex };
struct RuleSegment {
  SegKind kind = SegKind::Static;
  std::string text;            // static string / template name
  std::string regexp;          // "" when absent
  bool has_regexp = false;
};
std::string parse_user_rule(const std::string& rule, std::vector<RuleSegment>& out);

}  // namespace ose
