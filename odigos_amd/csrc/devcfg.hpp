// devcfg.hpp — layouts of the compiled, read-only tables the kernels read
// from HBM (built once per engine by engine.cpp, see ose_engine_create).
#pragma once
#include <cstdint>

namespace ose {

// One compiled regexp (regex_dfa.hpp) inside a blob.  All offsets are byte
// offsets from the blob base, 16-byte aligned.
struct DfaDev {
  uint32_t nclasses, nstates, start, match;
  uint32_t hi_n;        // number of non-ASCII ranges
  uint32_t hi_off;      // uint32 triplets {lo, hi, cls}
  uint32_t trans_off;   // [nstates][nclasses]: uint16, or uint32 when wide
  uint32_t acc_off;     // uint8  [nstates]
  uint32_t wide;        // more than 65535 states: uint32 state ids
  uint8_t ascii[128];   // class of runes 0..127
};

// odigosurltemplate tables.
enum : uint32_t { kRuleStatic = 0, kRuleWildcard = 1, kRuleTemplate = 2, kRuleRegex = 3 };
struct UrlRuleSegDev {
  uint32_t kind;
  uint32_t text_off, text_len;   // static text or template name (in bytes section)
  int32_t dfa;                   // index into dfa table, -1 = none
};
struct UrlRuleDev {
  uint32_t nseg;
  uint32_t seg_first;            // index into rule segment table
};
struct UrlCustomDev {
  int32_t dfa;
  uint32_t name;                 // index into name table
};
struct NameDev {
  uint32_t off, len;             // in bytes section
};

// Name table order: 0 "id", 1 "date", 2 "email", 3.. custom-id names.
enum : uint32_t { kNameId = 0, kNameDate = 1, kNameEmail = 2, kNameCustom0 = 3 };

struct UrlCfgDev {
  uint32_t n_custom, n_rules, n_names, n_dfa;
  uint32_t max_rule_nseg;        // 0 when there are no rules
  uint32_t max_name_len;
  uint32_t rules_by_len_off;     // uint32 [max_rule_nseg + 2]: first rule index for nseg (rules sorted by nseg, config order within)
  uint32_t rules_off;            // UrlRuleDev[n_rules]
  uint32_t segs_off;             // UrlRuleSegDev[]
  uint32_t custom_off;           // UrlCustomDev[n_custom]
  uint32_t names_off;            // NameDev[n_names]
  uint32_t dfa_off;              // uint32 [n_dfa] byte offsets of DfaDev
  uint32_t bytes_off;            // raw text bytes
  uint32_t total_bytes;
};

}  // namespace ose

namespace ose {

// odigossampling tables (sampling_host.cpp builds them from the decoded
// Config; trace_kernel.hip reads them).  Rules are stored in level order
// global, service, endpoint (rule_engine.go:56-60), config order inside a
// level (evaluateLevel is an order-sensitive fold, rule_engine.go:89-115).
enum : uint32_t { kSampError = 0, kSampLatency = 1, kSampService = 2 };
constexpr uint32_t kMaxLatencyRules = 64;   // bits of the per-trace latency masks
constexpr uint32_t kMaxServiceRules = 64;   // bits of the per-trace service mask
constexpr uint32_t kSampCfgLds = 12288;     // the trace kernel keeps the whole table blob in LDS
struct SampRuleDev {
  uint32_t type;
  uint32_t bit;          // latency: latency-rule index; service: service-rule index
  double ratio;          // service_name sampling_ratio
  double fallback;       // fallback_sampling_ratio
};
struct SampLatDev {      // one http_latency rule (latency.go:12-17)
  uint32_t slot;         // latency-service slot of its service_name
  uint32_t route_off, route_len;   // http_route prefix bytes (bytes section)
  uint32_t _pad;
  int64_t threshold;     // ms
  int64_t threshold_ns;  // threshold * 1e6, or INT64_MAX when that overflows (never satisfied)
  uint32_t pre[4];       // first 16 prefix bytes, little-endian dwords, zero-padded
  uint32_t msk[4];       // byte mask of the prefix within those 16 bytes
};
// trace_multi_kernel's flush: each rule chunk's rules by what matches them
// (a chunk of at most 128 rules), so a trace's walk visits only its matched
// rules — an unmatched rule leaves evaluateLevel's state as it is
struct SampWalkDev {
  uint64_t err[2];          // the error rules (always matched), by rule index
  uint64_t svc[64][2];      // the service rules of each service bit
  uint8_t lat_rule[64];     // the rule of each latency bit
};
struct SampCfgDev {
  uint32_t n_rules;
  uint32_t level_first[4];   // rules of level L: [level_first[L], level_first[L+1])
  uint32_t n_lat;            // http_latency rules
  uint32_t n_lat_slots;      // distinct service names among them
  uint32_t n_services;       // interned service ids (res_svc values >= this are "no rule service")
  uint32_t n_attr;           // span_attribute rules: their bits follow the service-rule bits
  uint32_t attr_shift;       // = number of service_name rule bits
  uint32_t attr_base;        // attr_match bit of this table's first span_attribute rule (rule chunks)
  uint32_t rules_off;        // SampRuleDev[n_rules]
  uint32_t lat_off;          // SampLatDev[n_lat]
  uint32_t svc_slot_off;     // uint32 [n_services]: latency slot of each service, or ~0
  uint32_t slot_rules_off;   // uint64 [n_lat_slots]: latency rules of each slot
  uint32_t svc_bits_off;     // uint64 [n_services]: service rules naming each service
  uint32_t bytes_off;
  uint32_t total_bytes;
};

}  // namespace ose

namespace ose {

// span_attribute rules evaluated on the GPU (attr_kernel.hip; the rule
// semantics of internal/sampling/spanattribute.go:136-230).  One entry per
// rule with a string / number / boolean condition, in level order; `bit` is
// the rule's attr_match bit, `key` its attr_type / attr_val column.
enum : uint32_t { kAttrCondStr = 0, kAttrCondNum = 1, kAttrCondBool = 2 };
enum : uint32_t {
  kAttrOpNever = 0,   // an operation the condition type has no case for
  kAttrOpExists, kAttrOpEq, kAttrOpNe, kAttrOpContains, kAttrOpNotContains, kAttrOpRegex,
  kAttrOpGt, kAttrOpLt, kAttrOpGe, kAttrOpLe
};
struct AttrRuleDev {
  uint32_t bit, key, svc, cond, op;
  uint32_t exp_off, exp_len;   // expected_value bytes (string conditions), bytes section
  uint32_t dfa_off;            // regex: DfaDev byte offset; 0 = regexp.Compile failed (never matches)
  uint32_t num_ok;             // strconv.ParseFloat(expected_value) succeeded
  uint32_t bool_ok, bool_val;  // strconv.ParseBool(expected_value)
  uint32_t _pad;
  double num;
};
struct AttrCfgDev {
  uint32_t n_rules;
  uint32_t n_keys;
  uint32_t rules_off;          // AttrRuleDev[n_rules]
  uint32_t bytes_off;
  uint32_t total_bytes;
  uint32_t _pad[3];
};

}  // namespace ose
