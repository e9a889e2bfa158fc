// columnize.cpp — see columnize.hpp.
#include "columnize.hpp"

#include <algorithm>
#include <cstring>

#include "host.hpp"
#include "urlparse.hpp"

namespace ose {

bool workload_key(const AttrMap& attrs, std::string& key) {
  const Value* ns = attrs.Get("k8s.namespace.name");
  if (!ns || ns->type != Value::TStr) return false;
  struct { const char* attr; const char* kind; } order[] = {
      {"k8s.deployment.name", "deployment"}, {"k8s.statefulset.name", "statefulset"}, {"k8s.daemonset.name", "daemonset"}};
  for (auto& o : order) {
    const Value* v = attrs.Get(o.attr);
    if (!v) continue;
    if (v->type != Value::TStr) return false;
    key = ns->s + "/" + o.kind + "/" + v->s;
    return true;
  }
  return false;
}

std::set<std::string> workload_set(const MatchProperties& mp) {
  std::set<std::string> s;
  for (auto& w : mp.k8s_workloads) {
    std::string k = w.kind;
    for (auto& c : k) c = (char)std::tolower((unsigned char)c);
    s.insert(w.namespace_ + "/" + k + "/" + w.name);
  }
  return s;
}

std::string ColumnizeCtx::build(const UrlTemplateConfig* url, const SamplingConfig* sampling,
                                const TrafficMetricsConfig* traffic) {
  if (url) {
    has_exclude = url->exclude.has_value();
    has_include = url->include.has_value();
    url_filter = has_exclude || has_include;
    if (has_exclude) excl = workload_set(*url->exclude);
    if (has_include) incl = workload_set(*url->include);
  }
  if (traffic) traffic_keys = traffic->res_attributes_keys;
  if (sampling) {
    services = intern_services(*sampling);
    for (auto* lvl : {&sampling->global_rules, &sampling->service_rules, &sampling->endpoint_rules})
      for (auto& r : *lvl)
        if (r.rtype == RuleType::SpanAttribute) {
          attr_preds.emplace_back();
          std::string e = attr_preds.back().compile(r.attr);
          if (!e.empty()) return e;
        }
    attr_plan = plan_attr_rules(*sampling);
  }
  return "";
}

ResourceCols columnize_resource(const ColumnizeCtx& c, const AttrMap& ra) {
  ResourceCols r;
  // service ids (latency.go:51-56 AsString; servicename.go:38-42 Str)
  const Value* sv = ra.Get("service.name");
  if (sv) {
    const std::string as = sv->AsString();
    // span_attribute rules whose service this resource is (spanattribute.go:130-132)
    r.attr_res.assign((c.attr_preds.size() + 63) / 64, 0);
    for (size_t k = 0; k < c.attr_preds.size(); k++)
      if (c.attr_preds[k].service() == as) r.attr_res[k / 64] |= 1ull << (k % 64);
    auto it = c.services.find(as);
    if (it != c.services.end()) {
      r.svc = it->second;
      if (sv->type == Value::TStr) r.svc_str = it->second;
    }
  }
  // include/exclude (odigosurltemplateprocessor/processor.go:76-85)
  if (c.url_filter) {
    std::string key;
    const bool has_key = workload_key(ra, key);
    if (c.has_exclude && has_key && c.excl.count(key)) r.url_ok = 0;
    if (c.has_include && !(has_key && c.incl.count(key))) r.url_ok = 0;
  }
  // attributeSetFromResource (odigostrafficmetrics/processor.go:60-69)
  std::map<std::string, std::string> set;
  for (auto& k : c.traffic_keys)
    if (const Value* v = ra.Get(k)) set[k] = v->Str();
  r.attrset.assign(set.begin(), set.end());
  return r;
}

void columnize_span(const ColumnizeCtx& c, const Span& sp, const std::vector<uint64_t>& attr_res, const ProtoSizer& sizer,
                    SpanCols& o) {
  o.hi = o.lo = 0;
  for (int k = 0; k < 8; k++) { o.hi = o.hi << 8 | sp.trace_id[k]; o.lo = o.lo << 8 | sp.trace_id[8 + k]; }
  o.start = sp.start;
  o.end = sp.end;
  o.status = status_column(sp.status_code);
  o.kind = (uint8_t)std::min<int32_t>(std::max<int32_t>(sp.kind, 0), 255);
  o.span_size = (uint32_t)sizer.span(sp);
  o.name_len = (uint32_t)sp.name.size();
  // span_attribute: the "json" conditions here, the others from the key columns on the GPU
  const size_t W = std::max<size_t>(1, (c.attr_preds.size() + 63) / 64);
  o.attr_match.assign(W, 0);
  for (size_t w = 0; w < attr_res.size() && w < c.attr_plan.host_mask.size(); w++)
    for (uint64_t m = attr_res[w] & c.attr_plan.host_mask[w]; m; m &= m - 1) {
      const size_t k = 64 * w + (size_t)__builtin_ctzll(m);
      if (const Value* av = sp.attrs.Get(c.attr_preds[k].key()))
        if (c.attr_preds[k].eval(*av)) o.attr_match[w] |= 1ull << (k % 64);
    }
  const size_t nk = c.attr_plan.keys.size();
  o.attr_type.assign(nk, OSE_ATTR_ABSENT);
  o.attr_val.assign(nk, 0);
  o.attr_str.assign(nk, std::string_view());
  for (size_t k = 0; k < nk; k++) {
    const Value* av = sp.attrs.Get(c.attr_plan.keys[k]);
    if (!av) continue;
    switch (av->type) {
      case Value::TStr: o.attr_type[k] = OSE_ATTR_STR; o.attr_str[k] = av->s; break;
      case Value::TInt: o.attr_type[k] = OSE_ATTR_INT; o.attr_val[k] = (uint64_t)av->i; break;
      case Value::TDouble: o.attr_type[k] = OSE_ATTR_DOUBLE; std::memcpy(&o.attr_val[k], &av->d, 8); break;
      case Value::TBool: o.attr_type[k] = OSE_ATTR_BOOL; o.attr_val[k] = av->b ? 1 : 0; break;
      default: o.attr_type[k] = OSE_ATTR_OTHER; break;
    }
  }
  // the keys the processors read, picked up in one pass over the span's
  // attributes (each the first of its key, as pcommon.Map.Get finds it)
  const Value *route = nullptr, *method = nullptr, *method_old = nullptr, *url_tmpl = nullptr, *url_path = nullptr,
              *target = nullptr, *url_full = nullptr, *http_url = nullptr;
  auto first = [](const Value*& slot, const Value& v) {
    if (!slot) slot = &v;
  };
  for (auto& e : sp.attrs.kv) {
    const std::string& k = e.first;
    switch (k.size()) {
      case 8:
        if (k == "url.path") first(url_path, e.second);
        else if (k == "url.full") first(url_full, e.second);
        else if (k == "http.url") first(http_url, e.second);
        break;
      case 10:
        if (k == "http.route") first(route, e.second);
        break;
      case 11:
        if (k == "http.method") first(method_old, e.second);
        else if (k == "http.target") first(target, e.second);
        break;
      case 12:
        if (k == "url.template") first(url_tmpl, e.second);
        break;
      case 19:
        if (k == "http.request.method") first(method, e.second);
        break;
      default:
        break;
    }
  }
  // sampling: AsString(http.route) (latency.go:64-68)
  o.has_route = route != nullptr;
  if (route && route->type == Value::TStr) {
    o.route = route->s;
  } else {
    o.route_own = route ? route->AsString() : std::string();
    o.route = o.route_own;
  }
  auto as_view = [&](const Value* v) -> std::string_view {
    if (v->type == Value::TStr) return v->s;
    o.path_own = v->AsString();
    return o.path_own;
  };
  // urltemplate (processor.go:98-147, 235-287)
  uint8_t f = 0;
  o.path = std::string_view();
  const Value* m = method ? method : method_old;
  if (m) {
    f |= OSE_URL_HAS_METHOD;
    if (m->type == Value::TStr ? sp.name == m->s : sp.name == m->AsString()) f |= OSE_URL_NAME_EQ_METHOD;
    if (const Value* tv = sp.kind == OSE_KIND_CLIENT ? url_tmpl : route) {
      if (tv->type != Value::TStr) f |= OSE_URL_TGT_NONSTR;
      else f |= tv->s.empty() ? OSE_URL_TGT_STR_EMPTY : OSE_URL_TGT_STR;
    }
    if (const Value* p = url_path) {
      f |= OSE_URL_PATH_RAW;
      o.path = as_view(p);
    } else if (const Value* p = target) {
      f |= OSE_URL_PATH_TARGET;
      o.path = as_view(p);
    } else {
      const Value* fu = url_full ? url_full : http_url;
      std::string path;
      if (fu && go_url_parse_path(fu->AsString(), path)) {
        f |= OSE_URL_PATH_RAW;
        o.path_own = std::move(path);
        o.path = o.path_own;
      }
    }
  }
  o.url_flags = f;
}

}  // namespace ose
