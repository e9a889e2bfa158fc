// span_attr.hpp — the per-span predicate of odigossampling's span_attribute
// rule (internal/sampling/spanattribute.go:126-320), evaluated by the host
// columniser into the attr_match column; the GPU trace stage ORs the bits
// per trace (a rule is satisfied iff one span of a resource with the rule's
// AsString(service.name) meets the condition; it is never matched-but-
// unsatisfied, spanattribute.go:319).
//
// Third-party semantics restated here (parity pinned by the reference's
// spanattribute_test.go cases, tests/golden/span_attribute_kats.json):
//   encoding/json  Unmarshal validity (RFC 8259; numbers must fit float64),
//                  Marshal of nested values (sorted keys, HTML escaping)
//   strconv        ParseFloat, ParseBool, FormatFloat(v, 'f', -1, 64)
//   regexp         regex_dfa.hpp's HostRegexp (full DFA, lazy DFA past its caps)
//   PaesslerAG/jsonpath v0.1.1  Get: $, .key, ['key'], ["key"], [index]
//                  (pinned by the KATs); the ambiguous selectors *, [*],
//                  [a,b], [a:b:c], ..  return the match list (parity
//                  unpinned: the library is not in the reference); filters
//                  [?(..)] and scripts [(..)] evaluate a gval expression
//                  subset (literals, @ / $ paths, ! - * / % + - < <= > >=
//                  == != =~ && ||, parentheses), restated from gval's
//                  published grammar (parity unpinned, see span_attr.cpp)
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "config.hpp"
#include "pdata.hpp"
#include "regex_dfa.hpp"

namespace ose {

struct JsonExpr;   // a filter / script expression (span_attr.cpp)

// One selector of a PaesslerAG/jsonpath path: plain (Key, Index) or
// ambiguous (Wild `*` / `[*]`, Union `[a,b]`, Slice `[a:b:c]`, Descend `..`
// followed by its selector, Filter `[?(expr)]`, Script `[(expr)]`)
struct JsonPathStep {
  enum Kind { Key, Index, Wild, Union, Slice, Descend, Filter, Script } kind = Key;
  std::shared_ptr<const JsonExpr> expr;   // Filter / Script
  std::string key;
  long long index = 0;
  std::vector<JsonPathStep> items;   // Union: Key / Index items; Descend: the selector after `..`
  bool has_lo = false, has_hi = false;
  long long lo = 0, hi = 0, step = 1;   // Slice
};

class SpanAttrPredicate {
 public:
  // "" on success, else the reason the engine cannot run this rule
  std::string compile(const SpanAttributeRule& r);
  const std::string& service() const { return service_; }
  const std::string& key() const { return key_; }
  // the condition on the span's attribute value (found = the key exists)
  bool eval(const Value& attr) const;

 private:
  std::string service_, key_, cond_, op_, expected_;
  bool re_ok_ = false;
  HostRegexp re_;
  bool num_ok_ = false;
  double num_ = 0;
  bool bool_ok_ = false, bool_ = false;
  std::vector<JsonPathStep> path_;
};

// Which span_attribute rules the engine evaluates on the GPU, and from which
// attr_type / attr_val column (include/odigos_amd.h): every rule with a
// string / number / boolean condition; "json" conditions stay with the shim.
struct AttrPlan {
  std::vector<std::string> keys;   // distinct attribute_key of the GPU rules, level order
  std::vector<int> rule_key;       // per span_attribute rule (level order): key column, -1 = shim
  std::vector<uint64_t> host_mask; // attr_match bits the shim still computes ((rules + 63) / 64 words)
  bool host(size_t k) const { return k / 64 < host_mask.size() && ((host_mask[k / 64] >> (k % 64)) & 1); }
};
AttrPlan plan_attr_rules(const SamplingConfig& c);

// helpers exposed for tests
bool go_parse_float(const std::string& s, double& out);
bool go_parse_bool(const std::string& s, bool& out);
std::string go_format_float_f(double v);

}  // namespace ose
