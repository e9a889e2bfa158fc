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
// Unsupported (rejected, never approximated): DFAs above kMaxStates (about
// two million states) or kMaxTableBytes of transitions.
#pragma once
#include <cstdint>
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

RegexStatus compile_dfa(const std::string& pattern, Dfa& out, std::string& err);

// Host-side evaluation of a compiled DFA (used by the engine's self-check
// and unit tests; the kernels implement the same loop).
bool dfa_match(const Dfa& d, const uint8_t* s, size_t n);

}  // namespace ose
