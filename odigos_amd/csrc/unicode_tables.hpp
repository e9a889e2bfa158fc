// unicode_tables.hpp — Unicode data for the DFA compiler's \p{..} classes
// and (?i) folding (regex_dfa.cpp); the tables are generated
// (tools/gen_unicode_tables.py -> unicode_tables.cpp).
#pragma once
#include <cstdint>

namespace ose {
struct UniTable {
  const char* name;
  const uint32_t* ranges;   // n inclusive {lo, hi} pairs, ascending
  uint32_t n;
};
extern const UniTable kUniCategories[];   // two-letter general categories (Cn excluded)
extern const uint32_t kUniCategoriesN;
extern const UniTable kUniScripts[];      // unicode.Scripts names
extern const uint32_t kUniScriptsN;
// simple case folding: {rune, next rune of its orbit} ascending by rune; the
// orbit of a rune absent here is the rune alone
extern const uint32_t kFoldOrbit[];
extern const uint32_t kFoldOrbitN;
}  // namespace ose
