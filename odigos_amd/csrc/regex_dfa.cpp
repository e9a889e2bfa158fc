// regex_dfa.cpp — Go RE2-syntax regexp -> DFA (see regex_dfa.hpp).
#include "regex_dfa.hpp"
#include "unicode_tables.hpp"

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <set>

namespace ose {
namespace {

constexpr uint32_t kRuneMax = 0x10FFFF;
constexpr uint32_t kRuneError = 0xFFFD;

using Ranges = std::vector<std::pair<uint32_t, uint32_t>>;

// unicode/utf8.DecodeRune: invalid -> (U+FFFD, 1)
uint32_t decode(const uint8_t* s, size_t n, int& w) {
  uint8_t c = s[0];
  if (c < 0x80) { w = 1; return c; }
  int need;
  uint32_t r;
  uint8_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { need = 1; r = c & 0x1F; }
  else if (c == 0xE0) { need = 2; r = c & 0x0F; lo = 0xA0; }
  else if (c >= 0xE1 && c <= 0xEC) { need = 2; r = c & 0x0F; }
  else if (c == 0xED) { need = 2; r = c & 0x0F; hi = 0x9F; }
  else if (c >= 0xEE && c <= 0xEF) { need = 2; r = c & 0x0F; }
  else if (c == 0xF0) { need = 3; r = c & 0x07; lo = 0x90; }
  else if (c >= 0xF1 && c <= 0xF3) { need = 3; r = c & 0x07; }
  else if (c == 0xF4) { need = 3; r = c & 0x07; hi = 0x8F; }
  else { w = 1; return kRuneError; }
  if ((size_t)need >= n) { w = 1; return kRuneError; }
  for (int i = 1; i <= need; i++) {
    uint8_t b = s[i];
    if (b < (i == 1 ? lo : 0x80) || b > (i == 1 ? hi : 0xBF)) { w = 1; return kRuneError; }
    r = (r << 6) | (b & 0x3F);
  }
  w = need + 1;
  return r;
}

void normalize(Ranges& r) {
  std::sort(r.begin(), r.end());
  Ranges o;
  for (auto& x : r) {
    if (!o.empty() && x.first <= o.back().second + 1) o.back().second = std::max(o.back().second, x.second);
    else o.push_back(x);
  }
  r.swap(o);
}
Ranges negate(Ranges r) {
  normalize(r);
  Ranges o;
  uint32_t next = 0;
  for (auto& x : r) {
    if (x.first > next) o.push_back({next, x.first - 1});
    next = x.second + 1;
  }
  if (next <= kRuneMax) o.push_back({next, kRuneMax});
  return o;
}
// unicode.SimpleFold closure (regexp/syntax appendFoldedRange): every rune
// of r brings its whole simple case-folding orbit (unicode_tables.hpp).
void fold(Ranges& r) {
  normalize(r);
  // each pass adds the next rune of every member's orbit; orbits are short
  // cycles, so a few passes close the set
  for (int pass = 0; pass < 8; pass++) {
    Ranges add;
    for (uint32_t k = 0; k < kFoldOrbitN; k++) {
      const uint32_t c = kFoldOrbit[2 * k], nx = kFoldOrbit[2 * k + 1];
      auto in = [&](uint32_t x) {
        auto it = std::upper_bound(r.begin(), r.end(), std::make_pair(x, kRuneMax + 1));
        return it != r.begin() && std::prev(it)->second >= x;
      };
      if (in(c) && !in(nx)) add.push_back({nx, nx});
    }
    if (add.empty()) break;
    r.insert(r.end(), add.begin(), add.end());
    normalize(r);
  }
}

Ranges table_ranges(const UniTable& t) {
  Ranges r;
  for (uint32_t k = 0; k < t.n; k++) r.push_back({t.ranges[2 * k], t.ranges[2 * k + 1]});
  return r;
}
// TR18 loose matching (Go 1.25 regexp/syntax): case-insensitive, spaces,
// underscores and hyphens ignored
std::string loose(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == ' ' || c == '_' || c == '-') continue;
    o += (char)((c >= 'A' && c <= 'Z') ? c + 32 : c);
  }
  return o;
}
// the table of a \p{name} (Go 1.25 unicodeTable): Any, ASCII, Assigned,
// general categories (one and two letters, LC, Cn) and their long aliases,
// scripts.  false: no such class.
bool unicode_class(const std::string& name, Ranges& out) {
  static const std::pair<const char*, const char*> kAliases[] = {
      {"casedletter", "LC"}, {"closepunctuation", "Pe"}, {"combiningmark", "M"}, {"connectorpunctuation", "Pc"},
      {"control", "Cc"}, {"currencysymbol", "Sc"}, {"dashpunctuation", "Pd"}, {"decimalnumber", "Nd"},
      {"enclosingmark", "Me"}, {"finalpunctuation", "Pf"}, {"format", "Cf"}, {"initialpunctuation", "Pi"},
      {"letter", "L"}, {"letternumber", "Nl"}, {"lineseparator", "Zl"}, {"lowercaseletter", "Ll"}, {"mark", "M"},
      {"mathsymbol", "Sm"}, {"modifierletter", "Lm"}, {"modifiersymbol", "Sk"}, {"nonspacingmark", "Mn"},
      {"number", "N"}, {"openpunctuation", "Ps"}, {"other", "C"}, {"otherletter", "Lo"}, {"othernumber", "No"},
      {"otherpunctuation", "Po"}, {"othersymbol", "So"}, {"paragraphseparator", "Zp"}, {"privateuse", "Co"},
      {"punctuation", "P"}, {"separator", "Z"}, {"spaceseparator", "Zs"}, {"spacingmark", "Mc"}, {"surrogate", "Cs"},
      {"symbol", "S"}, {"titlecaseletter", "Lt"}, {"unassigned", "Cn"}, {"uppercaseletter", "Lu"}, {"cntrl", "Cc"},
      {"digit", "Nd"}, {"punct", "P"}};
  std::string key = loose(name);
  for (auto& a : kAliases)
    if (key == a.first) key = loose(a.second);
  out.clear();
  if (key == "any") { out = {{0, kRuneMax}}; return true; }
  if (key == "ascii") { out = {{0, 0x7F}}; return true; }
  auto all_assigned = [&]() {
    Ranges r;
    for (uint32_t k = 0; k < kUniCategoriesN; k++) {
      Ranges t = table_ranges(kUniCategories[k]);
      r.insert(r.end(), t.begin(), t.end());
    }
    normalize(r);
    return r;
  };
  if (key == "assigned") { out = all_assigned(); return true; }
  if (key == "cn") { out = negate(all_assigned()); return true; }
  if (key == "lc") key = "lu|ll|lt";
  bool any = false;
  for (uint32_t k = 0; k < kUniCategoriesN; k++) {
    const std::string cat = loose(kUniCategories[k].name);
    // one letter: the group (Go's unicode.C is Cc|Cf|Co|Cs: the tables have no Cn)
    const bool hit = cat == key || (key.size() == 1 && cat[0] == key[0]) ||
                     (key == "lu|ll|lt" && (cat == "lu" || cat == "ll" || cat == "lt"));
    if (!hit) continue;
    Ranges t = table_ranges(kUniCategories[k]);
    out.insert(out.end(), t.begin(), t.end());
    any = true;
  }
  if (any) { normalize(out); return true; }
  for (uint32_t k = 0; k < kUniScriptsN; k++)
    if (loose(kUniScripts[k].name) == key) {
      out = table_ranges(kUniScripts[k]);
      normalize(out);
      return true;
    }
  return false;
}

enum EmptyOp : uint8_t { kBOL = 1, kEOL = 2, kBOT = 4, kEOT = 8, kWB = 16, kNWB = 32 };

struct Node {
  enum Kind { Empty, Chars, Assert, Cat, Alt, Rep } kind = Empty;
  Ranges chars;
  uint8_t op = 0;
  std::vector<std::unique_ptr<Node>> sub;
  int min = 0, max = 0;  // max -1 = unbounded
};
using NodeP = std::unique_ptr<Node>;

struct ParseError {
  RegexStatus st;
  std::string msg;
};

class Parser {
 public:
  explicit Parser(const std::string& p) : s_(p) {}
  NodeP parse() {
    NodeP n = alt();
    if (i_ < s_.size()) throw ParseError{RegexStatus::Syntax, "unexpected ): `" + s_ + "`"};
    return n;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  bool fi_ = false, fm_ = false, fs_ = false;
  int depth_ = 0;
  Ranges uclass_;   // the set of the last \p / \P escape

  [[noreturn]] void syntax(const std::string& m) { throw ParseError{RegexStatus::Syntax, m}; }
  [[noreturn]] void unsupported(const std::string& m) { throw ParseError{RegexStatus::Unsupported, m}; }
  bool eof() const { return i_ >= s_.size(); }
  uint32_t rune(int& w) const { return decode((const uint8_t*)s_.data() + i_, s_.size() - i_, w); }

  NodeP chars(Ranges r, bool neg) {
    normalize(r);
    if (fi_) fold(r);
    if (neg) r = negate(r);
    auto n = std::make_unique<Node>();
    n->kind = Node::Chars;
    n->chars = std::move(r);
    return n;
  }
  // regexp/syntax appendGroup: under (?i) the group is folded, then negated
  void perl(Ranges& r, char k, bool neg) const {
    Ranges t;
    if (k == 'd') t = {{'0', '9'}};
    else if (k == 's') t = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}};
    else t = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
    if (fi_) fold(t);
    if (neg) t = negate(t);
    r.insert(r.end(), t.begin(), t.end());
  }
  static bool alnum(uint32_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
  static bool hexd(char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
  static uint32_t hexv(char c) { return c <= '9' ? c - '0' : ((c | 0x20) - 'a' + 10); }

  // escape after '\'; kind: 0 rune, 1 perl class (perl,neg), 2 empty op, 3 unicode class (uclass_)
  int escape(uint32_t& r, char& pk, bool& pneg, uint8_t& op, bool in_class) {
    if (eof()) syntax("trailing backslash at end of expression");
    int w;
    uint32_t c = rune(w);
    i_ += w;
    if (c < 0x80 && !alnum(c)) { r = c; return 0; }
    switch (c) {
      case 'd': case 's': case 'w': pk = (char)c; pneg = false; return 1;
      case 'D': case 'S': case 'W': pk = (char)(c + 32); pneg = true; return 1;
      case 'a': r = 7; return 0;
      case 'f': r = 12; return 0;
      case 'n': r = 10; return 0;
      case 'r': r = 13; return 0;
      case 't': r = 9; return 0;
      case 'v': r = 11; return 0;
      case 'b': if (!in_class) { op = kWB; return 2; } break;
      case 'B': if (!in_class) { op = kNWB; return 2; } break;
      case 'A': if (!in_class) { op = kBOT; return 2; } break;
      case 'z': if (!in_class) { op = kEOT; return 2; } break;
      case 'p': case 'P': {   // regexp/syntax parseUnicodeClass
        bool neg = c == 'P';
        std::string name;
        if (eof()) syntax("invalid character class range");
        if (s_[i_] == '{') {
          const size_t e = s_.find('}', i_);
          if (e == std::string::npos) syntax("invalid character class range");
          name = s_.substr(i_ + 1, e - i_ - 1);
          i_ = e + 1;
        } else {
          int w2;
          (void)rune(w2);
          name = s_.substr(i_, (size_t)w2);
          i_ += w2;
        }
        if (!name.empty() && name[0] == '^') {   // \p{^Greek} == \P{Greek}
          neg = !neg;
          name = name.substr(1);
        }
        Ranges t;
        if (!unicode_class(name, t)) syntax("invalid character class range");
        if (fi_) fold(t);   // folded, then negated (parseUnicodeClass)
        uclass_ = neg ? negate(t) : t;
        return 3;
      }
      case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        if (eof() || s_[i_] < '0' || s_[i_] > '7') break;
        [[fallthrough]];
      case '0': {
        uint32_t v = c - '0';
        for (int k = 1; k < 3 && !eof() && s_[i_] >= '0' && s_[i_] <= '7'; k++) v = v * 8 + (s_[i_++] - '0');
        r = v;
        return 0;
      }
      case 'x': {
        if (eof()) break;
        if (s_[i_] == '{') {
          size_t j = i_ + 1;
          uint32_t v = 0;
          int nd = 0;
          while (j < s_.size() && hexd(s_[j]) && v <= kRuneMax) { v = v * 16 + hexv(s_[j]); j++; nd++; }
          if (nd == 0 || j >= s_.size() || s_[j] != '}' || v > kRuneMax) break;
          i_ = j + 1;
          r = v;
          return 0;
        }
        if (i_ + 2 > s_.size() || !hexd(s_[i_]) || !hexd(s_[i_ + 1])) break;
        r = hexv(s_[i_]) * 16 + hexv(s_[i_ + 1]);
        i_ += 2;
        return 0;
      }
      default: break;
    }
    syntax("invalid escape sequence");
  }

  bool posix(Ranges& r) {  // at "[:"
    size_t j = i_ + 2;
    bool neg = false;
    if (j < s_.size() && s_[j] == '^') { neg = true; j++; }
    size_t e = s_.find(":]", j);
    if (e == std::string::npos) return false;
    std::string nm = s_.substr(j, e - j);
    Ranges t;
    if (nm == "alnum") t = {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}};
    else if (nm == "alpha") t = {{'A', 'Z'}, {'a', 'z'}};
    else if (nm == "ascii") t = {{0, 0x7F}};
    else if (nm == "blank") t = {{'\t', '\t'}, {' ', ' '}};
    else if (nm == "cntrl") t = {{0, 0x1F}, {0x7F, 0x7F}};
    else if (nm == "digit") t = {{'0', '9'}};
    else if (nm == "graph") t = {{'!', '~'}};
    else if (nm == "lower") t = {{'a', 'z'}};
    else if (nm == "print") t = {{' ', '~'}};
    else if (nm == "punct") t = {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}};
    else if (nm == "space") t = {{'\t', '\r'}, {' ', ' '}};
    else if (nm == "upper") t = {{'A', 'Z'}};
    else if (nm == "word") t = {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}, {'_', '_'}};
    else if (nm == "xdigit") t = {{'0', '9'}, {'A', 'F'}, {'a', 'f'}};
    else syntax("invalid character class range");
    if (neg) t = negate(t);
    r.insert(r.end(), t.begin(), t.end());
    i_ = e + 2;
    return true;
  }

  NodeP cls() {  // after '['
    Ranges r;
    bool neg = false;
    if (!eof() && s_[i_] == '^') { neg = true; i_++; }
    bool first = true;
    for (;;) {
      if (eof()) syntax("missing closing ]");
      if (s_[i_] == ']' && !first) { i_++; break; }
      first = false;
      if (i_ + 1 < s_.size() && s_[i_] == '[' && s_[i_ + 1] == ':' && posix(r)) continue;
      uint32_t lo, hi;
      char pk = 0;
      bool pn = false;
      uint8_t op = 0;
      if (s_[i_] == '\\') {
        i_++;
        int k = escape(lo, pk, pn, op, true);
        if (k == 1) { perl(r, pk, pn); continue; }
        if (k == 3) { r.insert(r.end(), uclass_.begin(), uclass_.end()); continue; }
      } else {
        int w;
        lo = rune(w);
        i_ += w;
      }
      hi = lo;
      if (i_ + 1 < s_.size() && s_[i_] == '-' && s_[i_ + 1] != ']') {
        i_++;
        if (s_[i_] == '\\') {
          i_++;
          int k = escape(hi, pk, pn, op, true);
          if (k != 0) syntax("invalid character class range");
        } else {
          int w;
          hi = rune(w);
          i_ += w;
        }
        if (hi < lo) syntax("invalid character class range");
      }
      r.push_back({lo, hi});
    }
    return chars(std::move(r), neg);
  }

  bool braces(int& mn, int& mx) {  // at '{'
    size_t j = i_ + 1;
    auto num = [&](int& v) {
      size_t st = j;
      long x = 0;
      while (j < s_.size() && s_[j] >= '0' && s_[j] <= '9') { if (x < 100000) x = x * 10 + (s_[j] - '0'); j++; }
      v = (int)x;
      return j > st;
    };
    if (!num(mn)) return false;
    if (j < s_.size() && s_[j] == ',') {
      j++;
      if (j < s_.size() && s_[j] == '}') mx = -1;
      else if (!num(mx)) return false;
    } else {
      mx = mn;
    }
    if (j >= s_.size() || s_[j] != '}') return false;
    i_ = j + 1;
    return true;
  }

  NodeP concat() {
    auto cat = std::make_unique<Node>();
    cat->kind = Node::Cat;
    bool last_rep = false;
    while (!eof() && s_[i_] != '|' && s_[i_] != ')') {
      char c = s_[i_];
      if (c == '*' || c == '+' || c == '?' || c == '{') {
        int mn = 0, mx = 0;
        bool is_rep = true;
        if (c == '{') {
          if (!braces(mn, mx)) is_rep = false;
          else if (mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx)) syntax("invalid repeat count");
        } else {
          i_++;
          mn = c == '+' ? 1 : 0;
          mx = c == '?' ? 1 : -1;
        }
        if (is_rep) {
          if (!eof() && s_[i_] == '?') i_++;
          if (last_rep) syntax("invalid nested repetition operator");
          if (cat->sub.empty()) syntax("missing argument to repetition operator");
          auto r = std::make_unique<Node>();
          r->kind = Node::Rep;
          r->min = mn;
          r->max = mx;
          r->sub.push_back(std::move(cat->sub.back()));
          cat->sub.back() = std::move(r);
          last_rep = true;
          continue;
        }
      }
      last_rep = false;
      if (c == '(') {
        i_++;
        bool si = fi_, sm = fm_, ss = fs_;
        bool flags_only = false;
        if (!eof() && s_[i_] == '?') {
          i_++;
          if (!eof() && (s_[i_] == 'P' || s_[i_] == '<')) {
            if (s_[i_] == 'P') i_++;
            if (eof() || s_[i_] != '<') syntax("invalid named capture");
            size_t e = s_.find('>', i_ + 1);
            if (e == std::string::npos || e == i_ + 1) syntax("invalid named capture");
            i_ = e + 1;
          } else {
            bool neg = false, any = false;
            for (;;) {
              if (eof()) syntax("missing closing )");
              char f = s_[i_++];
              if (f == 'i') { fi_ = !neg; any = true; }
              else if (f == 'm') { fm_ = !neg; any = true; }
              else if (f == 's') { fs_ = !neg; any = true; }
              else if (f == 'U') { any = true; }
              else if (f == '-') { if (neg) syntax("invalid or unsupported Perl syntax"); neg = true; any = false; }
              else if (f == ')') { if (neg && !any) syntax("invalid or unsupported Perl syntax"); flags_only = true; break; }
              else if (f == ':') { if (neg && !any) syntax("invalid or unsupported Perl syntax"); break; }
              else syntax("invalid or unsupported Perl syntax");
            }
          }
        }
        if (flags_only) continue;
        if (++depth_ > 1000) syntax("expression nests too deeply");
        NodeP sub = alt();
        depth_--;
        if (eof() || s_[i_] != ')') syntax("missing closing )");
        i_++;
        fi_ = si; fm_ = sm; fs_ = ss;
        cat->sub.push_back(std::move(sub));
        continue;
      }
      if (c == '[') { i_++; cat->sub.push_back(cls()); continue; }
      if (c == '.') {
        i_++;
        Ranges r = fs_ ? Ranges{{0, kRuneMax}} : Ranges{{0, 9}, {11, kRuneMax}};
        auto n = std::make_unique<Node>();
        n->kind = Node::Chars;
        n->chars = r;
        cat->sub.push_back(std::move(n));
        continue;
      }
      if (c == '^' || c == '$') {
        i_++;
        auto n = std::make_unique<Node>();
        n->kind = Node::Assert;
        n->op = c == '^' ? (fm_ ? kBOL : kBOT) : (fm_ ? kEOL : kEOT);
        cat->sub.push_back(std::move(n));
        continue;
      }
      uint32_t r;
      if (c == '\\' && i_ + 1 < s_.size() && s_[i_ + 1] == 'Q') {
        // \Q...\E: every rune up to \E (or the end) is a literal
        i_ += 2;
        const size_t e = s_.find("\\E", i_);
        const size_t stop = e == std::string::npos ? s_.size() : e;
        while (i_ < stop) {
          int w;
          const uint32_t lit = rune(w);
          i_ += w;
          cat->sub.push_back(chars(Ranges{{lit, lit}}, false));
        }
        if (e != std::string::npos) i_ = e + 2;
        last_rep = false;
        continue;
      }
      if (c == '\\') {
        i_++;
        char pk = 0;
        bool pn = false;
        uint8_t op = 0;
        int k = escape(r, pk, pn, op, false);
        if (k == 1) { Ranges t; perl(t, pk, pn); cat->sub.push_back(chars(t, false)); continue; }
        if (k == 3) {
          auto n = std::make_unique<Node>();
          n->kind = Node::Chars;
          n->chars = uclass_;
          cat->sub.push_back(std::move(n));
          continue;
        }
        if (k == 2) {
          auto n = std::make_unique<Node>();
          n->kind = Node::Assert;
          n->op = op;
          cat->sub.push_back(std::move(n));
          continue;
        }
      } else {
        int w;
        r = rune(w);
        i_ += w;
      }
      cat->sub.push_back(chars(Ranges{{r, r}}, false));
    }
    return cat;
  }

  NodeP alt() {
    auto a = std::make_unique<Node>();
    a->kind = Node::Alt;
    for (;;) {
      a->sub.push_back(concat());
      if (!eof() && s_[i_] == '|') { i_++; continue; }
      break;
    }
    return a;
  }
};

// ---------------- Thompson NFA ----------------
struct Inst {
  enum Op : uint8_t { Rune, Split, Empty, Match, Nop } op;
  int out = -1, out1 = -1;
  uint8_t eop = 0;
  int ranges = -1;   // index into rangesets
};

struct Nfa {
  std::vector<Inst> prog;
  std::vector<Ranges> sets;
  int start = 0;
};

struct Frag {
  int start;
  std::vector<int*> holes;  // pointers are unstable across reallocation: store (pc, which)
};
struct Hole { int pc; bool second; };
struct FragH { int start; std::vector<Hole> holes; };

class Compiler {
 public:
  Nfa nfa;
  FragH comp(const Node* n) {
    if (nfa.prog.size() > 100000) throw ParseError{RegexStatus::TooLarge, "expression too large"};
    switch (n->kind) {
      case Node::Empty: return nop();
      case Node::Chars: {
        int pc = emit(Inst::Rune);
        nfa.sets.push_back(n->chars);
        nfa.prog[pc].ranges = (int)nfa.sets.size() - 1;
        return {pc, {{pc, false}}};
      }
      case Node::Assert: {
        int pc = emit(Inst::Empty);
        nfa.prog[pc].eop = n->op;
        return {pc, {{pc, false}}};
      }
      case Node::Cat: {
        if (n->sub.empty()) return nop();
        FragH f = comp(n->sub[0].get());
        for (size_t k = 1; k < n->sub.size(); k++) {
          FragH g = comp(n->sub[k].get());
          patch(f.holes, g.start);
          f.holes = std::move(g.holes);
        }
        return f;
      }
      case Node::Alt: {
        if (n->sub.size() == 1) return comp(n->sub[0].get());
        FragH last = comp(n->sub.back().get());
        for (int k = (int)n->sub.size() - 2; k >= 0; k--) {
          FragH f = comp(n->sub[k].get());
          int sp = emit(Inst::Split);
          nfa.prog[sp].out = f.start;
          nfa.prog[sp].out1 = last.start;
          f.holes.insert(f.holes.end(), last.holes.begin(), last.holes.end());
          last = {sp, std::move(f.holes)};
        }
        return last;
      }
      case Node::Rep: {
        const Node* x = n->sub[0].get();
        FragH acc{-1, {}};
        bool have = false;
        auto append = [&](FragH g) {
          if (!have) { acc = std::move(g); have = true; return; }
          patch(acc.holes, g.start);
          acc.holes = std::move(g.holes);
        };
        for (int k = 0; k < n->min; k++) append(comp(x));
        if (n->max < 0) {
          FragH b = comp(x);
          int sp = emit(Inst::Split);
          nfa.prog[sp].out = b.start;
          patch(b.holes, sp);
          append(FragH{sp, {{sp, true}}});
        } else {
          for (int k = n->min; k < n->max; k++) {
            FragH b = comp(x);
            int sp = emit(Inst::Split);
            nfa.prog[sp].out = b.start;
            std::vector<Hole> h = b.holes;
            h.push_back({sp, true});
            append(FragH{sp, std::move(h)});
          }
        }
        if (!have) return nop();
        return acc;
      }
    }
    return nop();
  }

 private:
  int emit(Inst::Op op) {
    Inst i;
    i.op = op;
    nfa.prog.push_back(i);
    return (int)nfa.prog.size() - 1;
  }
  FragH nop() {
    int pc = emit(Inst::Nop);
    return {pc, {{pc, false}}};
  }
  void patch(const std::vector<Hole>& hs, int to) {
    for (auto& h : hs) (h.second ? nfa.prog[h.pc].out1 : nfa.prog[h.pc].out) = to;
  }
};

// rune "type" for EmptyOpContext: 0 = none (begin/end of text), 1 = '\n',
// 2 = word char, 3 = other
constexpr int kTypeBot = 0, kTypeNL = 1, kTypeWord = 2, kTypeOther = 3;

uint8_t context(int t1, int t2) {  // regexp/syntax.EmptyOpContext
  uint8_t op = kNWB;
  int b = 0;
  if (t1 == kTypeWord) b = 1;
  else if (t1 == kTypeNL) op |= kBOL;
  else if (t1 == kTypeBot) op |= kBOT | kBOL;
  if (t2 == kTypeWord) b ^= 1;
  else if (t2 == kTypeNL) op |= kEOL;
  else if (t2 == kTypeBot) op |= kEOT | kEOL;
  if (b) op ^= (kWB | kNWB);
  return op;
}

// epsilon closure of `set` under context ctx; leaves only Rune insts in set.
void closure(const Nfa& nfa, std::vector<int>& set, uint8_t ctx, std::vector<char>& seen, bool& match) {
  std::vector<int> stack(set.begin(), set.end());
  std::vector<int> visited;
  set.clear();
  while (!stack.empty()) {
    int pc = stack.back();
    stack.pop_back();
    if (pc < 0 || seen[pc]) continue;
    seen[pc] = 1;
    visited.push_back(pc);
    const Inst& in = nfa.prog[pc];
    switch (in.op) {
      case Inst::Match: match = true; break;
      case Inst::Nop: stack.push_back(in.out); break;
      case Inst::Split: stack.push_back(in.out1); stack.push_back(in.out); break;
      case Inst::Empty: if ((in.eop & ~ctx) == 0) stack.push_back(in.out); break;
      case Inst::Rune: set.push_back(pc); break;
    }
  }
  for (int pc : visited) seen[pc] = 0;
}

}  // namespace

RegexStatus regex_syntax_check(const std::string& pattern, std::string& err) {
  try {
    Parser p(pattern);
    p.parse();
    return RegexStatus::Ok;
  } catch (const ParseError& e) {
    err = "error parsing regexp: " + e.msg + ": `" + pattern + "`";
    return e.st == RegexStatus::Unsupported ? RegexStatus::Ok : e.st;   // Go accepts these
  }
}

namespace {

// The NFA and its rune equivalence classes: what the subset construction
// (compile_dfa) and the lazy DFA (LazyDfa) share.
struct Prepared {
  Nfa nfa;
  uint32_t ncls = 0;
  uint32_t ascii[128];
  std::vector<uint32_t> hi_lo, hi_hi, hi_cls;   // non-ASCII ranges, sorted
  std::vector<int> cls_type;                    // EmptyOpContext type per class
  std::vector<std::vector<uint8_t>> cls_in;     // [class][rangeset] membership
  uint32_t cls(uint32_t r) const {
    if (r < 0x80) return ascii[r];
    size_t lo = 0, hi = hi_lo.size();
    while (lo < hi) {
      size_t m = (lo + hi) / 2;
      if (r < hi_lo[m]) hi = m;
      else if (r > hi_hi[m]) lo = m + 1;
      else return hi_cls[m];
    }
    return 0;
  }
};

RegexStatus prepare(const std::string& pattern, Prepared& P, std::string& err) {
  NodeP root;
  Compiler cc;
  try {
    Parser p(pattern);
    root = p.parse();
    FragH f = cc.comp(root.get());
    Inst m;
    m.op = Inst::Match;
    cc.nfa.prog.push_back(m);
    int mpc = (int)cc.nfa.prog.size() - 1;
    for (auto& h : f.holes) (h.second ? cc.nfa.prog[h.pc].out1 : cc.nfa.prog[h.pc].out) = mpc;
    cc.nfa.start = f.start;
  } catch (const ParseError& e) {
    err = "error parsing regexp: " + e.msg + ": `" + pattern + "`";
    return e.st;
  }
  P.nfa = std::move(cc.nfa);
  const Nfa& nfa = P.nfa;

  // rune equivalence classes: boundaries of every set, plus '\n' and the word
  // chars so that each class has one EmptyOpContext type.
  std::vector<uint32_t> cuts = {0, kRuneMax + 1, '\n', '\n' + 1, '0', '9' + 1, 'A', 'Z' + 1, '_', '_' + 1, 'a', 'z' + 1, 0x80};
  for (auto& s : nfa.sets)
    for (auto& r : s) { cuts.push_back(r.first); cuts.push_back(r.second + 1); }
  std::sort(cuts.begin(), cuts.end());
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  // elementary intervals [cuts[k], cuts[k+1]) -> signature -> class
  std::map<std::vector<uint8_t>, uint32_t> sig2cls;
  std::vector<uint32_t> iv_cls;
  auto rtype = [](uint32_t r) {
    if (r == '\n') return kTypeNL;
    if ((r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_') return kTypeWord;
    return kTypeOther;
  };
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    uint32_t lo = cuts[k];
    std::vector<uint8_t> sig(nfa.sets.size() + 1);
    for (size_t si = 0; si < nfa.sets.size(); si++) {
      bool in = false;
      for (auto& r : nfa.sets[si]) if (lo >= r.first && lo <= r.second) { in = true; break; }
      sig[si] = in;
    }
    sig.back() = (uint8_t)rtype(lo);
    auto it = sig2cls.find(sig);
    uint32_t c;
    if (it == sig2cls.end()) {
      c = (uint32_t)sig2cls.size();
      sig2cls.emplace(sig, c);
      P.cls_type.push_back(rtype(lo));
    } else {
      c = it->second;
    }
    iv_cls.push_back(c);
  }
  P.ncls = (uint32_t)sig2cls.size();
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    uint32_t lo = cuts[k], hi = cuts[k + 1] - 1;
    if (lo < 0x80) {
      for (uint32_t r = lo; r <= std::min<uint32_t>(hi, 0x7F); r++) P.ascii[r] = iv_cls[k];
    } else {
      if (!P.hi_lo.empty() && P.hi_cls.back() == iv_cls[k] && P.hi_hi.back() + 1 == lo) P.hi_hi.back() = hi;
      else { P.hi_lo.push_back(lo); P.hi_hi.push_back(hi); P.hi_cls.push_back(iv_cls[k]); }
    }
  }
  // set membership per class (any interval of the class is representative)
  P.cls_in.assign(P.ncls, std::vector<uint8_t>(nfa.sets.size()));
  for (auto& kv : sig2cls)
    for (size_t si = 0; si < nfa.sets.size(); si++) P.cls_in[kv.second][si] = kv.first[si];
  return RegexStatus::Ok;
}

// DFA state = (sorted Rune-inst set before closure, type of previous rune).
// The start inst is re-injected at every position (unanchored search); MATCH
// is absorbing.
struct StateKey {
  std::vector<int> set;
  int prev;
  bool operator<(const StateKey& o) const { return prev != o.prev ? prev < o.prev : set < o.set; }
};

// One transition of the subset construction: true = the closure before the
// rune already matched (the MATCH sink), else `next` is the successor.
bool subset_step(const Prepared& P, const StateKey& cur, uint32_t c, StateKey& next, std::vector<char>& seen) {
  std::vector<int> set = cur.set;
  set.push_back(P.nfa.start);
  bool match = false;
  closure(P.nfa, set, context(cur.prev, P.cls_type[c]), seen, match);
  if (match) return true;
  next.set.clear();
  for (int pc : set) {
    const Inst& in = P.nfa.prog[pc];
    if (P.cls_in[c][in.ranges]) next.set.push_back(in.out);
  }
  std::sort(next.set.begin(), next.set.end());
  next.set.erase(std::unique(next.set.begin(), next.set.end()), next.set.end());
  next.prev = P.cls_type[c];
  return false;
}

bool subset_accepts_end(const Prepared& P, const StateKey& cur, std::vector<char>& seen) {
  std::vector<int> set = cur.set;
  set.push_back(P.nfa.start);
  bool match = false;
  closure(P.nfa, set, context(cur.prev, kTypeBot), seen, match);
  return match;
}

}  // namespace

RegexStatus compile_dfa(const std::string& pattern, Dfa& out, std::string& err, uint32_t max_states,
                        uint64_t max_table_bytes) {
  max_states = std::min(max_states, Dfa::kMaxStates);
  max_table_bytes = std::min(max_table_bytes, Dfa::kMaxTableBytes);
  Prepared P;
  const RegexStatus pst = prepare(pattern, P, err);
  if (pst != RegexStatus::Ok) return pst;
  const uint32_t ncls = P.ncls;
  if (ncls > 255) { err = "regexp needs more than 255 rune classes"; return RegexStatus::TooLarge; }
  out = Dfa{};
  out.nclasses = ncls;
  for (int r = 0; r < 128; r++) out.ascii_class[r] = (uint8_t)P.ascii[r];
  out.hi_lo = P.hi_lo;
  out.hi_hi = P.hi_hi;
  out.hi_cls.assign(P.hi_cls.begin(), P.hi_cls.end());

  std::map<StateKey, uint32_t> ids;
  std::vector<StateKey> states;
  std::vector<char> seen(P.nfa.prog.size(), 0);
  const uint32_t kMatch = 0;
  // state 0 = MATCH sink
  states.push_back(StateKey{{}, -1});
  auto intern = [&](StateKey k) -> uint32_t {
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    uint32_t id = (uint32_t)states.size();
    ids.emplace(k, id);
    states.push_back(std::move(k));
    return id;
  };
  uint32_t start = intern(StateKey{{}, kTypeBot});
  std::vector<uint32_t> trans;
  std::vector<uint8_t> acc_end;
  trans.resize(ncls);  // row for MATCH
  for (uint32_t c = 0; c < ncls; c++) trans[c] = kMatch;
  acc_end.push_back(1);
  StateKey next;
  for (uint32_t s = 1; s < states.size(); s++) {
    if (states.size() > max_states || (uint64_t)states.size() * ncls * 4 > max_table_bytes) {
      err = "regexp DFA exceeds " + std::to_string(max_states) + " states or " +
            std::to_string(max_table_bytes >> 20) + " MiB of transitions";
      return RegexStatus::TooLarge;
    }
    StateKey cur = states[s];
    std::vector<uint32_t> row(ncls);
    for (uint32_t c = 0; c < ncls; c++)
      row[c] = subset_step(P, cur, c, next, seen) ? kMatch : intern(next);
    trans.insert(trans.end(), row.begin(), row.end());
    acc_end.push_back(subset_accepts_end(P, cur, seen) ? 1 : 0);
  }
  out.nstates = (uint32_t)states.size();
  out.start = start;
  out.match = kMatch;
  out.trans = std::move(trans);
  out.accept_end = std::move(acc_end);
  return RegexStatus::Ok;
}

// ---------------- lazy DFA ----------------
struct LazyDfa::Impl {
  Prepared P;
  uint64_t max_bytes = 0;
  std::mutex mu;
  std::map<StateKey, uint32_t> ids;
  std::vector<StateKey> states;     // 0 = MATCH sink
  std::vector<uint32_t> trans;      // [state][class], kUnknown until computed
  std::vector<int8_t> acc;          // accept at end of text: -1 unknown
  std::vector<char> seen;
  uint64_t flushes = 0;
  static constexpr uint32_t kUnknown = 0xFFFFFFFFu;
  void reset() {
    ids.clear();
    states.assign(1, StateKey{{}, -1});
    trans.assign(P.ncls, 0u);
    acc.assign(1, 1);
  }
  uint32_t intern(StateKey k) {
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    const uint32_t id = (uint32_t)states.size();
    ids.emplace(k, id);
    states.push_back(std::move(k));
    trans.resize(trans.size() + P.ncls, kUnknown);
    acc.push_back(-1);
    return id;
  }
};

LazyDfa::LazyDfa() = default;
LazyDfa::~LazyDfa() = default;

RegexStatus LazyDfa::compile(const std::string& pattern, std::string& err, uint64_t max_cache_bytes) {
  auto im = std::make_unique<Impl>();
  const RegexStatus st = prepare(pattern, im->P, err);
  if (st != RegexStatus::Ok) return st;
  im->max_bytes = std::max<uint64_t>(max_cache_bytes, (uint64_t)im->P.ncls * 4 * 16);
  im->seen.assign(im->P.nfa.prog.size(), 0);
  im->reset();
  impl_ = std::move(im);
  return RegexStatus::Ok;
}

uint64_t LazyDfa::cache_flushes() const { return impl_ ? impl_->flushes : 0; }

bool LazyDfa::match(const uint8_t* s, size_t n) const {
  if (!impl_) return false;
  Impl& m = *impl_;
  std::lock_guard<std::mutex> lk(m.mu);
  const uint32_t ncls = m.P.ncls;
  uint32_t st = m.intern(StateKey{{}, kTypeBot});
  StateKey next;
  size_t i = 0;
  while (i < n) {
    int w;
    const uint32_t r = decode(s + i, n - i, w);
    i += (size_t)w;
    const uint32_t c = m.P.cls(r);
    uint32_t t = m.trans[(size_t)st * ncls + c];
    if (t == Impl::kUnknown) {
      if (subset_step(m.P, m.states[st], c, next, m.seen)) return true;   // the MATCH sink
      // the cache holds at most max_bytes of transitions: when the next state
      // would pass it, drop every state but the one being entered (RE2's
      // lazy DFA does the same); the work per input rune stays bounded by the
      // NFA's size, so the match is linear in the input
      if (m.ids.find(next) == m.ids.end() && (uint64_t)(m.states.size() + 1) * ncls * 4 > m.max_bytes) {
        m.reset();
        m.flushes++;
        st = m.intern(next);
        continue;
      }
      t = m.intern(next);
      m.trans[(size_t)st * ncls + c] = t;
    }
    if (t == 0) return true;
    st = t;
  }
  if (m.acc[st] < 0) m.acc[st] = subset_accepts_end(m.P, m.states[st], m.seen) ? 1 : 0;
  return m.acc[st] != 0;
}

// ---------------- host matcher ----------------
RegexStatus HostRegexp::compile(const std::string& pattern, std::string& err, uint32_t max_states,
                                uint64_t max_bytes) {
  full_ = false;
  lazy_.reset();
  RegexStatus st = compile_dfa(pattern, dfa_, err, max_states, max_bytes);
  if (st == RegexStatus::Ok) {
    full_ = true;
    return st;
  }
  if (st != RegexStatus::TooLarge) return st;
  auto lz = std::make_shared<LazyDfa>();
  err.clear();
  st = lz->compile(pattern, err, max_bytes);
  if (st == RegexStatus::Ok) lazy_ = std::move(lz);
  return st;
}

bool HostRegexp::match(const uint8_t* s, size_t n) const {
  if (full_) return dfa_match(dfa_, s, n);
  return lazy_ && lazy_->match(s, n);
}

bool dfa_match(const Dfa& d, const uint8_t* s, size_t n) {
  uint32_t st = d.start;
  size_t i = 0;
  while (i < n) {
    if (st == d.match) return true;
    int w;
    uint32_t r = decode(s + i, n - i, w);
    i += (size_t)w;
    uint32_t c;
    if (r < 0x80) c = d.ascii_class[r];
    else {
      size_t lo = 0, hi = d.hi_lo.size();
      c = 0;
      while (lo < hi) {
        size_t m = (lo + hi) / 2;
        if (r < d.hi_lo[m]) hi = m;
        else if (r > d.hi_hi[m]) lo = m + 1;
        else { c = d.hi_cls[m]; break; }
      }
    }
    st = d.trans[(size_t)st * d.nclasses + c];
  }
  return st == d.match || d.accept_end[st];
}

}  // namespace ose
