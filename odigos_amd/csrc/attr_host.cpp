// attr_host.cpp — span_attribute rules on the GPU: the rule table (built
// once per engine from the decoded config) and the launch that turns the
// attr_type / attr_val columns into the attr_match bits the trace stage and
// the exchange pack read.
#include <cstring>

#include "blob.hpp"
#include "engine_internal.hpp"
#include "kernels.hpp"
#include "span_attr.hpp"

namespace ose {

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {
uint32_t op_code(const std::string& cond, const std::string& op) {
  if (op == "exists") return kAttrOpExists;
  if (cond == "string") {
    if (op == "equals") return kAttrOpEq;
    if (op == "not_equals") return kAttrOpNe;
    if (op == "contains") return kAttrOpContains;
    if (op == "not_contains") return kAttrOpNotContains;
    if (op == "regex") return kAttrOpRegex;
  } else if (cond == "number") {
    if (op == "equals") return kAttrOpEq;
    if (op == "not_equals") return kAttrOpNe;
    if (op == "greater_than") return kAttrOpGt;
    if (op == "less_than") return kAttrOpLt;
    if (op == "greater_than_or_equal") return kAttrOpGe;
    if (op == "less_than_or_equal") return kAttrOpLe;
  } else if (cond == "boolean") {
    if (op == "equals") return kAttrOpEq;
  }
  return kAttrOpNever;   // spanattribute.go's switch has no case: never satisfied
}
}  // namespace

// Rules in level order (their attr_match bit = index among span_attribute
// rules); only the string / number / boolean ones get an entry.
int Engine::build_attr_tables() {
  attr_keys.clear();
  attr_host_rules = 0;
  attr_host_words.clear();
  attr_words = 1;
  attr_n_rules = attr_n_dev = 0;
  if (!has_sampling) return 0;
  const AttrPlan plan = plan_attr_rules(sampling);
  attr_keys = plan.keys;
  attr_host_words = plan.host_mask;
  attr_host_rules = attr_host_words.empty() ? 0 : attr_host_words[0];
  attr_n_rules = (uint32_t)plan.rule_key.size();
  attr_words = std::max<uint32_t>(1, (attr_n_rules + 63) / 64);
  Blob bl;
  AttrCfgDev h{};
  bl.put(&h, 1);
  std::vector<AttrRuleDev> rules;
  std::string bytes;
  std::vector<std::pair<size_t, Dfa>> dfas;   // rule index -> compiled regexp
  size_t k = 0;
  for (auto* lvl : {&sampling.global_rules, &sampling.service_rules, &sampling.endpoint_rules})
    for (auto& r : *lvl) {
      if (r.rtype != RuleType::SpanAttribute) continue;
      const int key = plan.rule_key[k];
      const uint32_t bit = (uint32_t)k++;
      if (key < 0) continue;
      const SpanAttributeRule& x = r.attr;
      AttrRuleDev d{};
      d.bit = bit;
      d.key = (uint32_t)key;
      d.svc = service_ids.at(x.service_name);
      d.cond = x.condition_type == "string" ? kAttrCondStr : x.condition_type == "number" ? kAttrCondNum : kAttrCondBool;
      d.op = op_code(x.condition_type, x.operation);
      d.exp_off = (uint32_t)bytes.size();
      d.exp_len = (uint32_t)x.expected_value.size();
      bytes += x.expected_value;
      if (d.cond == kAttrCondNum) {
        double v = 0;
        d.num_ok = go_parse_float(x.expected_value, v) ? 1 : 0;   // strconv.ParseFloat (:185-188)
        d.num = v;
      }
      if (d.cond == kAttrCondBool) {
        bool b = false;
        d.bool_ok = go_parse_bool(x.expected_value, b) ? 1 : 0;   // strconv.ParseBool (:229-232)
        d.bool_val = b ? 1 : 0;
      }
      if (d.cond == kAttrCondStr && d.op == kAttrOpRegex) {
        Dfa dfa;
        std::string err;
        const RegexStatus st = compile_dfa(x.expected_value, dfa, err);
        if (st == RegexStatus::Ok) dfas.emplace_back(rules.size(), std::move(dfa));
        else if (st != RegexStatus::Syntax)   // Syntax: regexp.Compile fails, the span is skipped (:171-174)
          return fail(OSE_ENOTSUP, "span_attribute regex not supported by the DFA compiler: " + err);
      }
      rules.push_back(d);
    }
  attr_n_dev = (uint32_t)rules.size();
  if (rules.empty()) return 0;
  h.n_rules = attr_n_dev;
  h.n_keys = (uint32_t)attr_keys.size();
  h.rules_off = bl.put(rules.data(), rules.size());
  h.bytes_off = bl.put(bytes.data(), bytes.size());
  for (auto& rd : dfas) {
    const uint32_t off = put_dfa(bl, rd.second);
    if (bl.overflow) break;
    bl.at<AttrRuleDev>(h.rules_off)[rd.first].dfa_off = off;
  }
  bl.align();
  if (bl.overflow) return fail(OSE_ENOTSUP, "span_attribute device tables exceed 4 GiB (the regex rules' DFAs together)");
  // expected-value offsets are relative to the bytes section
  for (size_t q = 0; q < rules.size(); q++) bl.at<AttrRuleDev>(h.rules_off)[q].exp_off += h.bytes_off;
  bl.align();
  bl.b.resize(bl.b.size() + 16, 0);
  h.total_bytes = (uint32_t)bl.b.size();
  std::memcpy(bl.b.data(), &h, sizeof h);
  attr_blob_host = std::move(bl.b);
  return 0;
}

int Workspace::reserve_attr(uint64_t n) {
  if (attr_bits && attr_bits_cap >= n) return 0;
  if (captured) return fail(OSE_ENOMEM, "attribute workspace too small inside a hipGraph capture: call ose_reserve first");
  if (attr_bits) HIP_TRY(hipFree(attr_bits));
  attr_bits = nullptr;
  attr_bits_cap = 0;
  const uint64_t want = std::max<uint64_t>(n, 1 << 16);   // (n = spans x attr_match words)
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&attr_bits), want * 8));
  attr_bits_cap = want;
  return 0;
}

int Workspace::reserve_ep_planes(uint64_t words) {
  if (ep_planes && ep_planes_cap >= words) return 0;
  if (captured) return fail(OSE_ENOMEM, "endpoint-plane workspace too small inside a hipGraph capture");
  if (ep_planes) HIP_TRY(hipFree(ep_planes));
  ep_planes = nullptr;
  ep_planes_cap = 0;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ep_planes), std::max<uint64_t>(words, 1) * 8));
  ep_planes_cap = std::max<uint64_t>(words, 1);
  return 0;
}

// The attr_match bits for this call: evaluated here from attr_type /
// attr_val when the caller passes them (ORed with the shim's bits of the
// "json" rules), else the caller's attr_match as is.  Either way
// e->attr_words words per span, word-major (ose_columns.attr_match_words).
int resolve_attr_match(Engine* e, const ose_columns* c, Workspace* ws, hipStream_t st, const uint64_t** out) {
  *out = nullptr;
  if (!e->attr_n_rules) return 0;
  const uint64_t n = c->n_spans;
  if (c->svc_match) {   // owner side: the record carries the bits
    *out = c->attr_match;
    return 0;
  }
  const uint32_t W = e->attr_words;
  const bool gpu_eval = c->attr_type && c->attr_val && e->attr_n_dev;
  const bool reads_cols = c->attr_match && (!gpu_eval || e->attr_host_rules_any());   // attr_match is read
  if (reads_cols && std::max<uint32_t>(1, c->attr_match_words) != W)
    return fail(OSE_EINVAL, "attr_match carries " + std::to_string(std::max<uint32_t>(1, c->attr_match_words)) +
                                " words per span; the engine's " + std::to_string(e->attr_n_rules) +
                                " span_attribute rules need " + std::to_string(W) + " (ose_columns.attr_match_words)");
  if (gpu_eval) {
    if (c->n_attr_keys < e->attr_keys.size())
      return fail(OSE_EINVAL, "attr_type / attr_val carry fewer keys than the engine's span_attribute rules read");
    if (e->attr_host_rules_any() && !c->attr_match)
      return fail(OSE_EINVAL, "span_attribute rules with json conditions need the attr_match column");
    if (!c->resource || !c->res_svc) return fail(OSE_EINVAL, "span_attribute rules need resource and res_svc");
    int rc = ws->reserve_attr(n * W);
    if (rc) return rc;
    AttrArgs a{};
    a.n_spans = n;
    a.words = W;
    a.type = c->attr_type;
    a.val = c->attr_val;
    a.arena = c->arena;
    a.resource = c->resource;
    a.res_svc = c->res_svc;
    a.host_bits = e->attr_host_rules_any() ? c->attr_match : nullptr;
    a.host_mask = reinterpret_cast<const uint64_t*>(e->attr_host_mask_dev);
    a.cfg = e->attr_blob_dev;
    a.out = ws->attr_bits;
    Engine::Timed tm{};
    e->prof_begin("attr_eval_kernel", st, tm);
    launch_attr_eval(a, st);
    HIP_TRY(hipGetLastError());
    e->prof_end(tm, st);
    *out = ws->attr_bits;
    return 0;
  }
  if (!c->attr_match && n) return fail(OSE_EINVAL, "span_attribute rules need the attr_match column (or attr_type / attr_val)");
  *out = c->attr_match;
  return 0;
}

}  // namespace ose

using namespace ose;

extern "C" int ose_engine_attr_key(const ose_engine* eng, uint32_t k, const char** key, uint32_t* len) {
  if (!eng || !key || !len) return fail(OSE_EINVAL, "NULL argument");
  const Engine* e = reinterpret_cast<const Engine*>(eng);
  if (k >= e->attr_keys.size()) return fail(OSE_EINVAL, "attribute key index out of range");
  *key = e->attr_keys[k].data();
  *len = (uint32_t)e->attr_keys[k].size();
  return 0;
}
