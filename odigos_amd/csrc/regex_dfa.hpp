// regex_dfa.hpp — compiles a Go regexp (RE2 syntax, regexp.Compile = Perl
// flags) into a DFA that answers regexp.MatchString (unanchored search) over
// UTF-8 input, for evaluation inside HIP kernels.
//
// Used for odigosurltemplate custom_ids and templatization-rule regexps
// (templatize.go:97-138, 211-220, 246-249; processor.go:45-60) and the
// span_attribute "regex" operation (spanattribute.go:170-177).
//
// Construction: parse -> Thompson NFA -> subset construction over rune
// equivalence classes, with the empty-width assertions (^ $ \A \z \b \B,
// multi-line variants) resolved from a per-state "previous rune type" and the
// class of the next rune, exactly as regexp.EmptyOpContext does.  Invalid
// UTF-8 bytes are runes U+FFFD of width 1 (unicode/utf8.DecodeRune).
// \p{..} / \P{..} (Go 1.25 names: categories, aliases, scripts, Any, ASCII,
// Assigned, Cn, LC; loose matching), \Q..\E and (?i) simple case folding of
// any rune use unicode_tables.cpp (generated from ICU 70: Unicode 14.0.0
// data; the reference's Go 1.25 has 15.0.0: the code points assigned in 15.0
// are parity unpinned).
// The device tables are bounded: a DFA above kMaxStates (about two million
// states) or kMaxTableBytes of transitions is TooLarge for the kernels.  On
// the host (span_attribute json filters, the shim's predicates) HostRegexp
// takes any such pattern with a lazy DFA (the subset construction run on
// demand over the input, its state cache bounded and flushed as RE2's is):
// linear in the input, like Go's regexp, and never refused for its size.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace ose {

enum class RegexStatus { Ok, Syntax, Unsupported, TooLarge };

// Go regexp.Compile acceptance (syntax only).
RegexStatus regex_syntax_check(const std::string& pattern, std::string& err);

struct Dfa {
  // state ids: uint16 on the device up to 65535 states, uint32 beyond
  // (DfaDev::wide); the cap bounds the subset construction's time and the
  // table (kMaxTableBytes), with room for the states one more row can add
  // (at most 256 classes) after the last check (compile_dfa)
  static constexpr uint32_t kMaxStates = (1u << 21) - 256;
  static constexpr uint64_t kMaxTableBytes = 256ull << 20;
  uint8_t ascii_class[128];               // class of runes 0..127
  std::vector<uint32_t> hi_lo, hi_hi;     // non-ASCII rune ranges [lo,hi] ...
  std::vector<uint8_t> hi_cls;            // ... and their class (sorted by lo)
  uint32_t nclasses = 0;
  uint32_t nstates = 0;
  uint32_t start = 0;
  uint32_t match = 0;                     // absorbing "matched" state
  std::vector<uint32_t> trans;            // [nstates][nclasses]
  std::vector<uint8_t> accept_end;        // state accepts at end of text
};

// max_states / max_table_bytes lower the caps (never above Dfa's).
RegexStatus compile_dfa(const std::string& pattern, Dfa& out, std::string& err,
                        uint32_t max_states = Dfa::kMaxStates, uint64_t max_table_bytes = Dfa::kMaxTableBytes);

// Host-side evaluation of a compiled DFA (used by the engine's self-check
// and unit tests; the kernels implement the same loop).
bool dfa_match(const Dfa& d, const uint8_t* s, size_t n);

// regexp.MatchString by a lazily built DFA whose transition cache holds at
// most max_cache_bytes (dropped whole when full).  match() is thread-safe
// (one mutex: the cache is shared).  Any number of rune classes.
class LazyDfa {
 public:
  LazyDfa();
  ~LazyDfa();
  RegexStatus compile(const std::string& pattern, std::string& err, uint64_t max_cache_bytes = 4ull << 20);
  bool match(const uint8_t* s, size_t n) const;
  uint64_t cache_flushes() const;   // for tests
 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// Host matcher: the full DFA when it stays within (max_states,
// max_table_bytes), else a LazyDfa with a max_table_bytes cache.  Returns
// Syntax / Unsupported as compile_dfa does; never TooLarge.
class HostRegexp {
 public:
  RegexStatus compile(const std::string& pattern, std::string& err, uint32_t max_states = 16384,
                      uint64_t max_table_bytes = 4ull << 20);
  bool match(const uint8_t* s, size_t n) const;
  bool lazy() const { return lazy_ != nullptr; }
 private:
  Dfa dfa_{};
  bool full_ = false;
  std::shared_ptr<LazyDfa> lazy_;
};

}  // namespace ose
