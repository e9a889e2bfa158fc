// config.cpp — decoding + Validate() of the three processor configs.
// See config.hpp for the reference files restated here.
#include "config.hpp"

#include <cctype>

#include "regex_dfa.hpp"

namespace ose {
namespace {

// mapstructure.Decode (no WeaklyTypedInput): numbers convert between int and
// float kinds (floats truncate into ints); strings must be strings.
std::string get_str(const Json& o, const char* key, std::string& out) {
  const Json* v = o.get(key);
  if (!v || v->is_null()) return "";
  if (!v->is_str()) return std::string("'") + key + "' expected type 'string', got unconvertible type";
  out = v->s;
  return "";
}
std::string get_f64(const Json& o, const char* key, double& out) {
  const Json* v = o.get(key);
  if (!v || v->is_null()) return "";
  if (!v->is_num()) return std::string("'") + key + "' expected type 'float64', got unconvertible type";
  out = v->num();
  return "";
}
std::string get_int(const Json& o, const char* key, int64_t& out) {
  const Json* v = o.get(key);
  if (!v || v->is_null()) return "";
  if (!v->is_num()) return std::string("'") + key + "' expected type 'int', got unconvertible type";
  out = v->i64();
  return "";
}
std::string get_str_list(const Json& o, const char* key, std::vector<std::string>& out) {
  const Json* v = o.get(key);
  if (!v || v->is_null()) return "";
  if (!v->is_arr()) return std::string("'") + key + "': source data must be an array or slice";
  for (auto& e : v->arr) {
    if (!e.is_str()) return std::string("'") + key + "[]' expected type 'string'";
    out.push_back(e.s);
  }
  return "";
}

#define TRY(x) do { std::string _e = (x); if (!_e.empty()) return _e; } while (0)

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

// strings.TrimSpace (ASCII whitespace; the rule grammar is ASCII)
std::string trim_space(const std::string& s) {
  size_t a = 0, b = s.size();
  auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; };
  while (a < b && ws(s[a])) a++;
  while (b > a && ws(s[b - 1])) b--;
  return s.substr(a, b - a);
}

// validateK8sWorkload (config.go:103-118)
std::string validate_workload(const K8sWorkload& w) {
  if (w.namespace_.empty()) return "namespace is required";
  if (w.kind.empty()) return "kind is required";
  std::string lk = lower(w.kind);
  if (lk != "deployment" && lk != "statefulset" && lk != "daemonset")
    return "kind must be one of deployment, statefulset or daemonset";
  if (w.name.empty()) return "name is required";
  return "";
}

std::string decode_match(const Json& j, std::optional<MatchProperties>& out) {
  if (j.is_null()) return "";
  if (!j.is_obj()) return "expected a map for match properties";
  MatchProperties mp;
  if (const Json* wl = j.get("k8s_workloads")) {
    if (!wl->is_null()) {
      if (!wl->is_arr()) return "'k8s_workloads': source data must be an array or slice";
      for (auto& w : wl->arr) {
        K8sWorkload k;
        TRY(get_str(w, "namespace", k.namespace_));
        TRY(get_str(w, "kind", k.kind));
        TRY(get_str(w, "name", k.name));
        mp.k8s_workloads.push_back(k);
      }
    }
  }
  out = mp;
  return "";
}

}  // namespace

// parseUserInputRuleString (templatize.go:140-190), parseRuleTemplateString
// (:97-123), parseRegexPattern (:127-138)
std::string parse_user_rule(const std::string& rule, std::vector<RuleSegment>& out) {
  out.clear();
  std::vector<std::string> parts;
  size_t st = 0;
  for (size_t i = 0; i <= rule.size(); i++) {
    if (i == rule.size() || rule[i] == '/') { parts.push_back(rule.substr(st, i - st)); st = i + 1; }
  }
  if (!rule.empty() && rule[0] == '/') parts.erase(parts.begin());
  for (auto& seg : parts) {
    RuleSegment rs;
    if (seg == "*") {
      rs.kind = SegKind::Wildcard;
    } else if (seg.size() >= 2 && seg.front() == '{' && seg.back() == '}') {
      std::string body = seg.substr(1, seg.size() - 2);
      size_t colon = body.find(':');
      std::string name = trim_space(colon == std::string::npos ? body : body.substr(0, colon));
      rs.kind = SegKind::Template;
      rs.text = name.empty() ? "id" : name;
      if (colon != std::string::npos) {
        std::string rx = trim_space(body.substr(colon + 1));
        if (rx.empty()) return "invalid rule template string. regexp is empty";
        std::string err;
        if (regex_syntax_check(rx, err) != RegexStatus::Ok)
          return "invalid rule template string. regexp is invalid: " + err;
        rs.regexp = rx;
        rs.has_regexp = true;
      }
    } else if (seg.size() > 6 && seg.compare(0, 6, "regex:") == 0) {
      std::string rx = seg.substr(6);
      std::string err;
      if (regex_syntax_check(rx, err) != RegexStatus::Ok)
        return "invalid regexp pattern \"" + rx + "\": " + err;
      rs.kind = SegKind::Regex;
      rs.regexp = rx;
      rs.has_regexp = true;
    } else {
      rs.kind = SegKind::Static;
      rs.text = seg;
    }
    out.push_back(rs);
  }
  return "";
}

// Config.Validate (odigosurltemplateprocessor/config.go:133-157)
std::string decode_url_config(const Json& j, UrlTemplateConfig& out) {
  out = UrlTemplateConfig{};
  if (j.is_null()) return "";
  if (!j.is_obj()) return "expected a map for odigosurltemplate config";
  if (const Json* e = j.get("exclude")) TRY(decode_match(*e, out.exclude));
  if (const Json* i = j.get("include")) TRY(decode_match(*i, out.include));
  TRY(get_str_list(j, "templatization_rules", out.templatization_rules));
  if (const Json* c = j.get("custom_ids")) {
    if (!c->is_null()) {
      if (!c->is_arr()) return "'custom_ids': source data must be an array or slice";
      for (auto& e : c->arr) {
        CustomIdConfig ci;
        TRY(get_str(e, "regexp", ci.regexp));
        TRY(get_str(e, "template_name", ci.template_name));
        out.custom_ids.push_back(ci);
      }
    }
  }
  if (out.exclude)
    for (auto& w : out.exclude->k8s_workloads) {
      std::string e = validate_workload(w);
      if (!e.empty()) return "invalid exclude properties: invalid workload: " + e;
    }
  if (out.include)
    for (auto& w : out.include->k8s_workloads) {
      std::string e = validate_workload(w);
      if (!e.empty()) return "invalid include properties: invalid workload: " + e;
    }
  for (auto& r : out.templatization_rules) {
    std::vector<RuleSegment> segs;
    TRY(parse_user_rule(r, segs));
  }
  for (auto& c : out.custom_ids) {
    std::string err;
    if (regex_syntax_check(c.regexp, err) != RegexStatus::Ok) return "invalid custom id regexp: " + err;
  }
  return "";
}

namespace {

// per-type decode + Validate (internal/sampling/*.go)
std::string decode_rule_details(const Json& d, SamplingRule& r) {
  if (!d.is_obj()) return "'' expected a map, got '" + std::string(d.is_arr() ? "slice" : "scalar") + "'";
  if (r.type == "http_latency") {
    r.rtype = RuleType::HttpLatency;
    auto& x = r.latency;
    TRY(get_str(d, "http_route", x.http_route));
    TRY(get_int(d, "threshold", x.threshold));
    TRY(get_str(d, "service_name", x.service_name));
    TRY(get_f64(d, "fallback_sampling_ratio", x.fallback_sampling_ratio));
    // latency.go:22-40
    if (x.threshold <= 0) return "threshold must be a positive integer";
    if (x.service_name.empty()) return "service_name cannot be empty";
    if (x.http_route.empty()) return "http_route cannot be empty";
    if (x.http_route[0] != '/') return "http_route must start with '/'";
    if (x.fallback_sampling_ratio < 0 || x.fallback_sampling_ratio > 100)
      return "fallback_sampling_ratio must be between 0 and 100";
    return "";
  }
  if (r.type == "error") {
    r.rtype = RuleType::Error;
    TRY(get_f64(d, "fallback_sampling_ratio", r.error.fallback_sampling_ratio));
    // error.go:18-23
    if (r.error.fallback_sampling_ratio < 0 || r.error.fallback_sampling_ratio > 100)
      return "fallback_sampling_ratio must be between 0 and 100";
    return "";
  }
  if (r.type == "service_name") {
    r.rtype = RuleType::ServiceName;
    auto& x = r.service;
    TRY(get_str(d, "service_name", x.service_name));
    TRY(get_f64(d, "sampling_ratio", x.sampling_ratio));
    TRY(get_f64(d, "fallback_sampling_ratio", x.fallback_sampling_ratio));
    // servicename.go:18-29
    if (x.service_name.empty()) return "service name cannot be empty";
    if (x.sampling_ratio < 0 || x.sampling_ratio > 100) return "sampling ratio must be between 0 and 100";
    if (x.fallback_sampling_ratio < 0 || x.fallback_sampling_ratio > 100)
      return "fallback sampling ratio must be between 0 and 100";
    return "";
  }
  if (r.type == "span_attribute") {
    r.rtype = RuleType::SpanAttribute;
    auto& x = r.attr;
    TRY(get_str(d, "service_name", x.service_name));
    TRY(get_str(d, "attribute_key", x.attribute_key));
    TRY(get_str(d, "condition_type", x.condition_type));
    TRY(get_str(d, "operation", x.operation));
    TRY(get_str(d, "expected_value", x.expected_value));
    TRY(get_str(d, "json_path", x.json_path));
    TRY(get_f64(d, "sampling_ratio", x.sampling_ratio));
    TRY(get_f64(d, "fallback_sampling_ratio", x.fallback_sampling_ratio));
    // spanattribute.go:38-120
    if (x.sampling_ratio < 0 || x.sampling_ratio > 100) return "sampling ratio must be between 0 and 100";
    if (x.fallback_sampling_ratio < 0 || x.fallback_sampling_ratio > 100)
      return "fallback sampling ratio must be between 0 and 100";
    if (x.service_name.empty()) return "service_name cannot be empty";
    if (x.attribute_key.empty()) return "attribute_key cannot be empty";
    const std::string& op = x.operation;
    auto in = [&](std::initializer_list<const char*> l) {
      for (auto* s : l) if (op == s) return true;
      return false;
    };
    if (x.condition_type == "string") {
      if (!in({"exists", "equals", "not_equals", "contains", "not_contains", "regex"})) return "invalid string operation";
      if (op != "exists" && x.expected_value.empty()) return "expected_value required for string operations";
    } else if (x.condition_type == "number") {
      if (!in({"exists", "equals", "not_equals", "greater_than", "less_than", "greater_than_or_equal", "less_than_or_equal"}))
        return "invalid number operation";
      if (op != "exists" && x.expected_value.empty()) return "expected_value required for number operations";
    } else if (x.condition_type == "boolean") {
      if (!in({"exists", "equals"})) return "invalid boolean operation";
      if (op == "equals" && x.expected_value.empty()) return "expected_value required for boolean equals operation";
    } else if (x.condition_type == "json") {
      if (!in({"exists", "is_valid_json", "is_invalid_json", "jsonpath_exists", "contains_key", "not_contains_key", "key_equals", "key_not_equals"}))
        return "invalid json operation";
      if (op != "exists" && op != "is_valid_json" && op != "is_invalid_json" && x.json_path.empty())
        return "json_path required for json operations";
      if ((op == "key_equals" || op == "key_not_equals") && x.expected_value.empty())
        return "expected_value required for key comparison";
    } else {
      return "unsupported condition type: \"" + x.condition_type + "\"";
    }
    return "";
  }
  return "unknown rule type: " + r.type;
}

std::string decode_rules(const Json& j, const char* key, std::vector<SamplingRule>& out) {
  const Json* a = j.get(key);
  if (!a || a->is_null()) return "";
  if (!a->is_arr()) return std::string("'") + key + "': source data must be an array or slice";
  for (auto& e : a->arr) {
    SamplingRule r;
    TRY(get_str(e, "name", r.name));
    TRY(get_str(e, "type", r.type));
    out.push_back(r);
  }
  return "";
}

// Rule.Validate (config.go:34-69)
std::string validate_rule(const Json& raw, SamplingRule& r) {
  if (r.name.empty()) return "rule name cannot be empty";
  if (r.type.empty()) return "rule type cannot be empty";
  const Json* d = raw.get("rule_details");
  if (!d || d->is_null()) return "rule details cannot be nil";
  return decode_rule_details(*d, r);
}

}  // namespace

// Config.Validate (odigossamplingprocessor/config.go:17-26): endpoint, service, global
std::string decode_sampling_config(const Json& j, SamplingConfig& out) {
  out = SamplingConfig{};
  if (j.is_null()) return "";
  if (!j.is_obj()) return "expected a map for odigossampling config";
  TRY(decode_rules(j, "global_rules", out.global_rules));
  TRY(decode_rules(j, "service_rules", out.service_rules));
  TRY(decode_rules(j, "endpoint_rules", out.endpoint_rules));
  struct L { const char* key; std::vector<SamplingRule>* v; } order[] = {
      {"endpoint_rules", &out.endpoint_rules}, {"service_rules", &out.service_rules}, {"global_rules", &out.global_rules}};
  for (auto& l : order) {
    const Json* a = j.get(l.key);
    for (size_t i = 0; i < l.v->size(); i++) TRY(validate_rule(a->arr[i], (*l.v)[i]));
  }
  return "";
}

// Config.Validate (odigostrafficmetrics/config.go:23-29)
std::string decode_traffic_config(const Json& j, TrafficMetricsConfig& out) {
  out = TrafficMetricsConfig{};
  if (j.is_null()) return "";
  if (!j.is_obj()) return "expected a map for odigostrafficmetrics config";
  TRY(get_str_list(j, "res_attributes_keys", out.res_attributes_keys));
  TRY(get_f64(j, "sampling_ratio", out.sampling_ratio));
  if (out.sampling_ratio < 0 || out.sampling_ratio > 1) return "sampling_ratio must be between 0.0 and 1.0";
  return "";
}

}  // namespace ose
