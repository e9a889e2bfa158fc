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
  uint32_t trans_off;   // uint16 [nstates][nclasses]
  uint32_t acc_off;     // uint8  [nstates]
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
constexpr uint32_t kMaxRuleLen = 64;   // rules longer than this never match (paths split into > 64 segments are not rule-eligible... see engine.cpp)

struct UrlCfgDev {
  uint32_t n_custom, n_rules, n_names, n_dfa;
  uint32_t max_rule_nseg;        // 0 when there are no rules
  uint32_t max_name_len;
  uint32_t rules_by_len_off;     // uint32 [kMaxRuleLen + 2]: first rule index for nseg (rules sorted by nseg, config order within)
  uint32_t rules_off;            // UrlRuleDev[n_rules]
  uint32_t segs_off;             // UrlRuleSegDev[]
  uint32_t custom_off;           // UrlCustomDev[n_custom]
  uint32_t names_off;            // NameDev[n_names]
  uint32_t dfa_off;              // uint32 [n_dfa] byte offsets of DfaDev
  uint32_t bytes_off;            // raw text bytes
  uint32_t total_bytes;
};

}  // namespace ose
