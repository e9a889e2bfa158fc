// Host check of odigos_amd/csrc/url_classes.hpp (test infrastructure): the
// class words of 32-byte rows against per-byte predicates of the character
// classes templatize.go's regexps use (noLettersRegex :14, hexEncodedRegex
// :41, longNumberAnywhereRegex :47, emailRegex :70, '/' and '?' for
// SplitN / Split in processor.go).  Every byte value at every row position,
// then random rows.  Exit status 0 = every word equal.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>

#include "../odigos_amd/csrc/url_classes.hpp"

using namespace ose::uc;

static bool in_class(uint32_t c, uint32_t cls) {
  const bool digit = c >= '0' && c <= '9';
  const bool alpha = (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
  const bool hexl = (c >= 'A' && c <= 'F') || (c >= 'a' && c <= 'f');
  const bool nolet = c < 128 && (digit || (c >= '!' && c <= '~' && !alpha));   // [\d_\-!@#$%^&*()=+{}\[\]:;"'<>,.?/\\|`~]
  const bool dom = alpha || digit || c == '.' || c == '-';
  const bool loc = dom || c == '_' || c == '%' || c == '+';
  switch (cls) {
    case BNL: return !nolet;
    case BHX: return !(digit || hexl);
    case DG: return digit;
    case AT: return c == '@';
    case HI: return c >= 0x80;
    case DASH: return c == '-';
    case SL: return c == '/';
    case QM: return c == '?';
    case BLOC: return !loc;
    case BDOM: return !dom;
    case DOT: return c == '.';
    case NAL: return !alpha;
  }
  return false;
}

static int check_row(const uint8_t* b) {
  uint32_t x[8], w[kN];
  std::memcpy(x, b, 32);
  row_classes(x, w);
  int bad = 0;
  for (uint32_t c = 0; c < kN; c++)
    for (int k = 0; k < 32; k++)
      if (((w[c] >> k) & 1u) != (in_class(b[k], c) ? 1u : 0u)) {
        if (bad++ < 8) std::printf("class %u byte %d (0x%02x): got %u\n", c, k, b[k], (w[c] >> k) & 1u);
      }
  return bad;
}

int main() {
  int bad = 0;
  uint8_t row[32];
  for (int v = 0; v < 256; v++)
    for (int pos = 0; pos < 32; pos++) {
      for (int k = 0; k < 32; k++) row[k] = (uint8_t)('a' + (k * 7 + v) % 26);
      row[pos] = (uint8_t)v;
      bad += check_row(row);
    }
  std::mt19937_64 rng(0x0D16CAFE);
  for (int it = 0; it < 200000 && !bad; it++) {
    for (int k = 0; k < 32; k++) row[k] = (uint8_t)rng();
    bad += check_row(row);
  }
  // the 8x8 transpose alone: bit 8i+b -> 8b+i
  for (int it = 0; it < 10000; it++) {
    uint64_t v = rng();
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    xpose8(lo, hi);
    const uint64_t t = lo | ((uint64_t)hi << 32);
    for (int i = 0; i < 8; i++)
      for (int b = 0; b < 8; b++)
        if (((v >> (8 * i + b)) & 1) != ((t >> (8 * b + i)) & 1)) bad++;
  }
  std::printf("%s\n", bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
