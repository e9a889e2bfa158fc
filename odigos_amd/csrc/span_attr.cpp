// span_attr.cpp — see span_attr.hpp.
#include "span_attr.hpp"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>

namespace ose {

// ---------------- strconv ----------------

// strconv.ParseFloat(s, 64): the whole string must be a Go float literal
// (readFloat: optional sign, decimal or "0x" mantissa — the latter needs a
// 'p' exponent — with '_' digit separators as underscoreOK allows; or
// [+-]inf / [+-]infinity / nan, case-insensitive).  Out-of-range magnitudes
// are an error (ErrRange); underflow rounds to zero silently.
bool go_parse_float(const std::string& s, double& out) {
  const size_t n = s.size();
  if (n == 0) return false;
  auto lc = [&](size_t i) { return (char)std::tolower((unsigned char)s[i]); };
  size_t i = (s[0] == '+' || s[0] == '-') ? 1 : 0;
  // special values
  std::string rest;
  for (size_t k = i; k < n; k++) rest += lc(k);
  if (rest == "inf" || rest == "infinity") {
    out = s[0] == '-' ? -HUGE_VAL : HUGE_VAL;
    return true;
  }
  if (rest == "nan") {
    if (i) return false;   // no sign on NaN
    out = std::nan("");
    return true;
  }
  const bool hex = i + 2 < n && s[i] == '0' && lc(i + 1) == 'x';
  size_t p = hex ? i + 2 : i;
  bool digits = false, dot = false, under = false;
  for (; p < n; p++) {
    const char c = lc(p);
    if (c == '_') { under = true; continue; }
    if (c == '.' && !dot) { dot = true; continue; }
    if (std::isdigit((unsigned char)c) || (hex && c >= 'a' && c <= 'f')) { digits = true; continue; }
    break;
  }
  if (!digits) return false;
  if (p < n && lc(p) == (hex ? 'p' : 'e')) {
    p++;
    if (p < n && (s[p] == '+' || s[p] == '-')) p++;
    if (p >= n || !std::isdigit((unsigned char)s[p])) return false;
    while (p < n && (std::isdigit((unsigned char)s[p]) || s[p] == '_')) under |= s[p++] == '_';
  } else if (hex) {
    return false;
  }
  if (p != n) return false;
  std::string lit;
  if (under) {
    // underscoreOK: each '_' sits between two digits (a base prefix counts as one)
    char prev = i == 0 && !hex ? '^' : '^';
    size_t q = i;
    if (hex) { prev = '0'; q = i + 2; }
    for (; q < n; q++) {
      const char c = lc(q);
      const bool dig = std::isdigit((unsigned char)c) || (hex && c >= 'a' && c <= 'f');
      if (dig) prev = '0';
      else if (c == '_') {
        if (prev != '0') return false;
        prev = '_';
      } else {
        if (prev == '_') return false;
        prev = '!';
      }
    }
    if (prev == '_') return false;
    for (char c : s)
      if (c != '_') lit += c;
  } else {
    lit = s;
  }
  errno = 0;
  char* end = nullptr;
  const double v = std::strtod(lit.c_str(), &end);
  if (end != lit.c_str() + lit.size()) return false;
  if (errno == ERANGE && std::isinf(v)) return false;
  out = v;
  return true;
}

// strconv.ParseBool
bool go_parse_bool(const std::string& s, bool& out) {
  static const char* t[] = {"1", "t", "T", "TRUE", "true", "True"};
  static const char* f[] = {"0", "f", "F", "FALSE", "false", "False"};
  for (auto* x : t)
    if (s == x) { out = true; return true; }
  for (auto* x : f)
    if (s == x) { out = false; return true; }
  return false;
}

namespace {
// shortest round-trip decimal digits of v (v finite, != 0): digits and the
// decimal exponent e such that v = 0.d1d2... * 10^e
void shortest_digits(double v, std::string& digits, int& e) {
  char buf[64];
  for (int p = 1; p <= 17; p++) {
    std::snprintf(buf, sizeof buf, "%.*e", p - 1, v);
    if (std::strtod(buf, nullptr) == v) break;
  }
  // buf = d.ddddde[+-]XX
  std::string m = buf;
  const size_t epos = m.find('e');
  const int ex = std::atoi(m.c_str() + epos + 1);
  digits.clear();
  for (size_t i = 0; i < epos; i++)
    if (std::isdigit((unsigned char)m[i])) digits += m[i];
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  e = ex + 1;
}
}  // namespace

// strconv.FormatFloat(v, 'f', -1, 64)
std::string go_format_float_f(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  std::string out = std::signbit(v) ? "-" : "";
  if (v == 0) return out + "0";
  std::string d;
  int e;
  shortest_digits(std::fabs(v), d, e);
  if (e <= 0) {
    out += "0.";
    out.append((size_t)(-e), '0');
    out += d;
  } else if ((size_t)e >= d.size()) {
    out += d;
    out.append((size_t)e - d.size(), '0');
  } else {
    out += d.substr(0, (size_t)e);
    out += '.';
    out += d.substr((size_t)e);
  }
  return out;
}

namespace {

// ---------------- encoding/json ----------------
struct JVal {
  enum T { Null, Bool, Num, Str, Arr, Obj } t = Null;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<JVal> a;
  std::map<std::string, JVal> o;   // Go unmarshals into map: last duplicate wins, Marshal sorts keys
};

struct JParser {
  const std::string& s;
  size_t p = 0;
  explicit JParser(const std::string& src) : s(src) {}
  void ws() {
    while (p < s.size() && (s[p] == ' ' || s[p] == '\t' || s[p] == '\n' || s[p] == '\r')) p++;
  }
  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if (s.compare(p, n, w) != 0) return false;
    p += n;
    return true;
  }
  static void put_utf8(std::string& o, uint32_t c) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 63)); }
    else if (c < 0x10000) { o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63)); }
    else { o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 63)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63)); }
  }
  bool hex4(uint32_t& v) {
    if (p + 4 > s.size()) return false;
    v = 0;
    for (int k = 0; k < 4; k++) {
      char c = s[p + k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    p += 4;
    return true;
  }
  bool str(std::string& o) {
    if (p >= s.size() || s[p] != '"') return false;
    p++;
    while (p < s.size()) {
      unsigned char c = (unsigned char)s[p];
      if (c == '"') { p++; return true; }
      if (c < 0x20) return false;
      if (c == '\\') {
        p++;
        if (p >= s.size()) return false;
        char e = s[p++];
        switch (e) {
          case '"': o += '"'; break;
          case '\\': o += '\\'; break;
          case '/': o += '/'; break;
          case 'b': o += '\b'; break;
          case 'f': o += '\f'; break;
          case 'n': o += '\n'; break;
          case 'r': o += '\r'; break;
          case 't': o += '\t'; break;
          case 'u': {
            uint32_t u;
            if (!hex4(u)) return false;
            if (u >= 0xD800 && u < 0xDC00) {   // surrogate pair, else U+FFFD (encoding/json)
              size_t save = p;
              uint32_t l;
              if (p + 1 < s.size() && s[p] == '\\' && s[p + 1] == 'u' && (p += 2, hex4(l)) && l >= 0xDC00 && l < 0xE000) {
                u = 0x10000 + ((u - 0xD800) << 10) + (l - 0xDC00);
              } else {
                p = save;
                u = 0xFFFD;
              }
            } else if (u >= 0xDC00 && u < 0xE000) {
              u = 0xFFFD;
            }
            put_utf8(o, u);
            break;
          }
          default: return false;
        }
        continue;
      }
      o += (char)c;   // invalid UTF-8 is kept here; Marshal replaces it
      p++;
    }
    return false;
  }
  bool num(double& v) {
    const size_t b = p;
    if (p < s.size() && s[p] == '-') p++;
    if (p >= s.size()) return false;
    if (s[p] == '0') p++;
    else if (s[p] >= '1' && s[p] <= '9') { while (p < s.size() && std::isdigit((unsigned char)s[p])) p++; }
    else return false;
    if (p < s.size() && s[p] == '.') {
      p++;
      if (p >= s.size() || !std::isdigit((unsigned char)s[p])) return false;
      while (p < s.size() && std::isdigit((unsigned char)s[p])) p++;
    }
    if (p < s.size() && (s[p] == 'e' || s[p] == 'E')) {
      p++;
      if (p < s.size() && (s[p] == '+' || s[p] == '-')) p++;
      if (p >= s.size() || !std::isdigit((unsigned char)s[p])) return false;
      while (p < s.size() && std::isdigit((unsigned char)s[p])) p++;
    }
    // float64 conversion: out of range is an UnmarshalTypeError
    return go_parse_float(s.substr(b, p - b), v);
  }
  bool value(JVal& v, int depth) {
    if (depth > 10000) return false;
    ws();
    if (p >= s.size()) return false;
    char c = s[p];
    if (c == '{') {
      p++;
      v.t = JVal::Obj;
      ws();
      if (p < s.size() && s[p] == '}') { p++; return true; }
      for (;;) {
        ws();
        std::string k;
        if (!str(k)) return false;
        ws();
        if (p >= s.size() || s[p] != ':') return false;
        p++;
        JVal x;
        if (!value(x, depth + 1)) return false;
        v.o[k] = std::move(x);
        ws();
        if (p < s.size() && s[p] == ',') { p++; continue; }
        if (p < s.size() && s[p] == '}') { p++; return true; }
        return false;
      }
    }
    if (c == '[') {
      p++;
      v.t = JVal::Arr;
      ws();
      if (p < s.size() && s[p] == ']') { p++; return true; }
      for (;;) {
        JVal x;
        if (!value(x, depth + 1)) return false;
        v.a.push_back(std::move(x));
        ws();
        if (p < s.size() && s[p] == ',') { p++; continue; }
        if (p < s.size() && s[p] == ']') { p++; return true; }
        return false;
      }
    }
    if (c == '"') { v.t = JVal::Str; return str(v.s); }
    if (lit("true")) { v.t = JVal::Bool; v.b = true; return true; }
    if (lit("false")) { v.t = JVal::Bool; v.b = false; return true; }
    if (lit("null")) { v.t = JVal::Null; return true; }
    v.t = JVal::Num;
    return num(v.n);
  }
};

// json.Unmarshal([]byte(s), &interface{}) == nil
bool json_unmarshal(const std::string& s, JVal& out) {
  JParser ps(s);
  if (!ps.value(out, 0)) return false;
  ps.ws();
  return ps.p == s.size();
}

// json.Marshal float64 (encoding/json floatEncoder)
std::string marshal_float(double f) {
  const double a = std::fabs(f);
  if (a != 0 && (a < 1e-6 || a >= 1e21)) {
    char buf[64];
    std::string d;
    int e;
    shortest_digits(a, d, e);
    // strconv 'e' with -1 precision: d[0].d[1:]e±XX, then Go trims "e-07" to "e-7"
    std::string m = d.substr(0, 1);
    if (d.size() > 1) m += "." + d.substr(1);
    int ex = e - 1;
    std::snprintf(buf, sizeof buf, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    std::string es = buf;
    if (es.size() == 4 && es[2] == '0') es.erase(2, 1);   // e-07 -> e-7
    return (f < 0 ? "-" : "") + m + es;
  }
  return go_format_float_f(f);
}

void marshal_string(const std::string& s, std::string& o) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
      else if (c == '\n') o += "\\n";
      else if (c == '\r') o += "\\r";
      else if (c == '\t') o += "\\t";
      else if (c < 0x20 || c == '<' || c == '>' || c == '&') { o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15]; }
      else o += (char)c;
      i++;
      continue;
    }
    // UTF-8 decode; invalid -> �; U+2028/2029 escaped
    uint32_t cp = 0;
    size_t n = 0;
    if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; n = 2; }
    else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; n = 3; }
    else if ((c & 0xF8) == 0xF0) { cp = c & 0x07; n = 4; }
    bool ok = n && i + n <= s.size();
    for (size_t k = 1; ok && k < n; k++) {
      unsigned char cc = (unsigned char)s[i + k];
      if ((cc & 0xC0) != 0x80) ok = false;
      cp = (cp << 6) | (cc & 63);
    }
    if (ok && ((n == 2 && cp < 0x80) || (n == 3 && (cp < 0x800 || (cp >= 0xD800 && cp < 0xE000))) ||
               (n == 4 && (cp < 0x10000 || cp > 0x10FFFF))))
      ok = false;
    if (!ok) { o += "\\ufffd"; i++; continue; }
    if (cp == 0x2028 || cp == 0x2029) { o += cp == 0x2028 ? "\\u2028" : "\\u2029"; i += n; continue; }
    o.append(s, i, n);
    i += n;
  }
  o += '"';
}

void marshal(const JVal& v, std::string& o) {
  switch (v.t) {
    case JVal::Null: o += "null"; break;
    case JVal::Bool: o += v.b ? "true" : "false"; break;
    case JVal::Num: o += marshal_float(v.n); break;
    case JVal::Str: marshal_string(v.s, o); break;
    case JVal::Arr:
      o += '[';
      for (size_t k = 0; k < v.a.size(); k++) {
        if (k) o += ',';
        marshal(v.a[k], o);
      }
      o += ']';
      break;
    case JVal::Obj: {
      o += '{';
      bool first = true;
      for (auto& kv : v.o) {   // std::map: sorted by key bytes, as Go sorts map keys
        if (!first) o += ',';
        first = false;
        marshal_string(kv.first, o);
        o += ':';
        marshal(kv.second, o);
      }
      o += '}';
      break;
    }
  }
}

}  // namespace

// ---------------- gval expressions of jsonpath filters / scripts ----------------
// PaesslerAG/jsonpath v0.1.1 evaluates `[?(expr)]` and `[(expr)]` with gval's
// full language; the engine restates the part a sampling rule can use
// (parity unpinned: neither library is in the reference):
//   literals      numbers (strconv float64), 'str' / "str", true, false, null
//   paths         @ (the current value) and $ (the document) followed by
//                 jsonpath selectors; a plain path that fails is an error,
//                 an ambiguous one yields its match list
//   operators     ! and unary -, * / %, + - (+ also joins two strings),
//                 < <= > >= (two numbers or two strings), == != (same type
//                 and value; containers by their JSON encoding), =~ (a
//                 string against a regexp: regexp.MatchString), && ||
//                 (short-circuit), parentheses
// An error anywhere (a missing key, an operator on the wrong types) makes a
// filter skip the element and a script select nothing.  A filter keeps the
// elements (array order) or member values (sorted keys) whose result is
// truthy: true, a non-zero number, a non-empty string, a container; a
// script's result selects an array index (an integral number) or an object
// key (a string).
struct JsonExpr {
  enum Op { Lit, Path, Not, Neg, Mul, Div, Mod, Add, Sub, Lt, Le, Gt, Ge, Eq, Ne, Match, And, Or } op = Lit;
  JVal lit;
  bool root = false;                    // Path: from $ (else @)
  std::vector<JsonPathStep> steps;      // Path
  std::shared_ptr<const JsonExpr> l, r;
  std::shared_ptr<HostRegexp> re;       // Match with a literal pattern
  bool re_ok = false;
};

namespace {

// Patterns met at run time (a filter's `=~` whose right side is not a
// literal): at most kDynCache per thread, the cache dropped whole when full;
// nullptr for a pattern regexp.Compile rejects (or one the parser cannot
// take).  The full DFA is capped at 4096 states / 1 MiB and the lazy DFA's
// cache at 1 MiB, so one evaluation costs O(pattern + input).
constexpr size_t kDynCache = 64;
const HostRegexp* dynamic_regexp(const std::string& pattern) {
  thread_local std::unordered_map<std::string, std::unique_ptr<HostRegexp>> cache;
  auto it = cache.find(pattern);
  if (it != cache.end()) return it->second.get();
  if (cache.size() >= kDynCache) cache.clear();
  auto re = std::make_unique<HostRegexp>();
  std::string err;
  const bool ok = re->compile(pattern, err, 4096, 1ull << 20) == RegexStatus::Ok;
  auto& slot = cache[pattern];
  if (ok) slot = std::move(re);
  return slot.get();
}

struct EV {
  bool ok = false;
  JVal v;
};

bool truthy(const EV& e) {
  if (!e.ok) return false;
  switch (e.v.t) {
    case JVal::Null: return false;
    case JVal::Bool: return e.v.b;
    case JVal::Num: return e.v.n != 0;
    case JVal::Str: return !e.v.s.empty();
    default: return true;
  }
}

void marshal(const JVal& v, std::string& o);
void select_step(const JsonPathStep& st, const JVal& v, std::vector<const JVal*>& out, const JVal& root);
bool plain_select(const JsonPathStep& st, const JVal& cur, const JVal*& out);
bool path_is_plain(const std::vector<JsonPathStep>& path);

EV eval_expr(const JsonExpr& x, const JVal& cur, const JVal& root) {
  EV r;
  auto num = [&](double d) { r.ok = true; r.v.t = JVal::Num; r.v.n = d; return r; };
  auto boolean = [&](bool b) { r.ok = true; r.v.t = JVal::Bool; r.v.b = b; return r; };
  switch (x.op) {
    case JsonExpr::Lit: r.ok = true; r.v = x.lit; return r;
    case JsonExpr::Path: {
      const JVal& base = x.root ? root : cur;
      if (path_is_plain(x.steps)) {
        const JVal* c = &base;
        for (const JsonPathStep& st : x.steps)
          if (!plain_select(st, *c, c)) return r;
        r.ok = true;
        r.v = *c;
        return r;
      }
      std::vector<const JVal*> a{&base}, b;
      for (const JsonPathStep& st : x.steps) {
        b.clear();
        for (const JVal* v : a) select_step(st, *v, b, root);
        a.swap(b);
      }
      r.ok = true;
      r.v.t = JVal::Arr;
      for (const JVal* v : a) r.v.a.push_back(*v);
      return r;
    }
    case JsonExpr::Not: return boolean(!truthy(eval_expr(*x.l, cur, root)));
    case JsonExpr::Neg: {
      EV a = eval_expr(*x.l, cur, root);
      if (!a.ok || a.v.t != JVal::Num) return r;
      return num(-a.v.n);
    }
    case JsonExpr::And: {
      if (!truthy(eval_expr(*x.l, cur, root))) return boolean(false);
      return boolean(truthy(eval_expr(*x.r, cur, root)));
    }
    case JsonExpr::Or: {
      if (truthy(eval_expr(*x.l, cur, root))) return boolean(true);
      return boolean(truthy(eval_expr(*x.r, cur, root)));
    }
    default: break;
  }
  EV a = eval_expr(*x.l, cur, root), b = eval_expr(*x.r, cur, root);
  if (!a.ok || !b.ok) return r;
  const bool nn = a.v.t == JVal::Num && b.v.t == JVal::Num, ss = a.v.t == JVal::Str && b.v.t == JVal::Str;
  switch (x.op) {
    case JsonExpr::Mul: return nn ? num(a.v.n * b.v.n) : r;
    case JsonExpr::Div: return nn ? num(a.v.n / b.v.n) : r;
    case JsonExpr::Mod: return nn ? num(std::fmod(a.v.n, b.v.n)) : r;
    case JsonExpr::Sub: return nn ? num(a.v.n - b.v.n) : r;
    case JsonExpr::Add:
      if (nn) return num(a.v.n + b.v.n);
      if (ss) {
        r.ok = true;
        r.v.t = JVal::Str;
        r.v.s = a.v.s + b.v.s;
      }
      return r;
    case JsonExpr::Lt: return nn ? boolean(a.v.n < b.v.n) : ss ? boolean(a.v.s < b.v.s) : r;
    case JsonExpr::Le: return nn ? boolean(a.v.n <= b.v.n) : ss ? boolean(a.v.s <= b.v.s) : r;
    case JsonExpr::Gt: return nn ? boolean(a.v.n > b.v.n) : ss ? boolean(a.v.s > b.v.s) : r;
    case JsonExpr::Ge: return nn ? boolean(a.v.n >= b.v.n) : ss ? boolean(a.v.s >= b.v.s) : r;
    case JsonExpr::Eq:
    case JsonExpr::Ne: {
      bool eq;
      if (a.v.t != b.v.t) eq = false;
      else if (nn) eq = a.v.n == b.v.n;
      else if (ss) eq = a.v.s == b.v.s;
      else if (a.v.t == JVal::Bool) eq = a.v.b == b.v.b;
      else if (a.v.t == JVal::Null) eq = true;
      else {
        std::string ma, mb;
        marshal(a.v, ma);
        marshal(b.v, mb);
        eq = ma == mb;
      }
      return boolean(x.op == JsonExpr::Eq ? eq : !eq);
    }
    case JsonExpr::Match: {
      if (!ss) return r;
      if (x.re) {
        if (!x.re_ok) return r;
        return boolean(x.re->match(reinterpret_cast<const uint8_t*>(a.v.s.data()), a.v.s.size()));
      }
      // a pattern taken from the span's own JSON: compiled with small caps
      // (a lazy DFA past them, so a pathological pattern costs bounded time
      // and memory per evaluation and still decides as Go's regexp would),
      // and cached per thread by pattern
      const HostRegexp* re = dynamic_regexp(b.v.s);
      if (!re) return r;   // regexp.Compile error: gval's =~ fails, the operand is an error
      return boolean(re->match(reinterpret_cast<const uint8_t*>(a.v.s.data()), a.v.s.size()));
    }
    default: return r;
  }
}

bool parse_path_steps(const std::string& p, size_t& i, std::vector<JsonPathStep>& out, bool in_expr);

// recursive descent over gval's precedence: || < && < comparisons < + - < * / % < unary
struct ExprParser {
  const std::string& p;
  size_t i;
  std::string err;
  ExprParser(const std::string& s, size_t at) : p(s), i(at) {}
  void ws() {
    while (i < p.size() && (p[i] == ' ' || p[i] == '\t')) i++;
  }
  bool eat(const char* t) {
    ws();
    const size_t n = std::strlen(t);
    if (p.compare(i, n, t) != 0) return false;
    i += n;
    return true;
  }
  using P = std::shared_ptr<JsonExpr>;
  static P bin(JsonExpr::Op op, P l, P r) {
    auto x = std::make_shared<JsonExpr>();
    x->op = op;
    x->l = l;
    x->r = r;
    return x;
  }
  P orx() {
    P l = andx();
    while (l && eat("||")) {
      P r = andx();
      if (!r) return nullptr;
      l = bin(JsonExpr::Or, l, r);
    }
    return l;
  }
  P andx() {
    P l = cmp();
    while (l && eat("&&")) {
      P r = cmp();
      if (!r) return nullptr;
      l = bin(JsonExpr::And, l, r);
    }
    return l;
  }
  P cmp() {
    P l = add();
    if (!l) return nullptr;
    static const struct { const char* t; JsonExpr::Op op; } ops[] = {
        {"==", JsonExpr::Eq}, {"!=", JsonExpr::Ne}, {"=~", JsonExpr::Match}, {"<=", JsonExpr::Le},
        {">=", JsonExpr::Ge}, {"<", JsonExpr::Lt}, {">", JsonExpr::Gt}};
    for (const auto& o : ops) {
      if (eat(o.t)) {
        P r = add();
        if (!r) return nullptr;
        P x = bin(o.op, l, r);
        if (o.op == JsonExpr::Match && r->op == JsonExpr::Lit && r->lit.t == JVal::Str) {
          x->re = std::make_shared<HostRegexp>();
          std::string e;
          const RegexStatus st = x->re->compile(r->lit.s, e);
          if (st == RegexStatus::Ok) x->re_ok = true;
          else if (st != RegexStatus::Syntax) {   // syntax Go accepts but the parser does not: refuse
            err = "regexp in a jsonpath filter: " + e;
            return nullptr;
          }
        }
        return x;
      }
    }
    return l;
  }
  P add() {
    P l = mul();
    for (;;) {
      if (!l) return nullptr;
      ws();
      if (i < p.size() && (p[i] == '+' || p[i] == '-')) {
        const JsonExpr::Op op = p[i] == '+' ? JsonExpr::Add : JsonExpr::Sub;
        i++;
        P r = mul();
        if (!r) return nullptr;
        l = bin(op, l, r);
      } else {
        return l;
      }
    }
  }
  P mul() {
    P l = unary();
    for (;;) {
      if (!l) return nullptr;
      ws();
      if (i < p.size() && (p[i] == '*' || p[i] == '/' || p[i] == '%')) {
        const JsonExpr::Op op = p[i] == '*' ? JsonExpr::Mul : p[i] == '/' ? JsonExpr::Div : JsonExpr::Mod;
        i++;
        P r = unary();
        if (!r) return nullptr;
        l = bin(op, l, r);
      } else {
        return l;
      }
    }
  }
  P unary() {
    ws();
    if (i < p.size() && p[i] == '!' && !(i + 1 < p.size() && p[i + 1] == '=')) {
      i++;
      P a = unary();
      return a ? bin(JsonExpr::Not, a, nullptr) : nullptr;
    }
    if (i < p.size() && p[i] == '-') {
      i++;
      P a = unary();
      return a ? bin(JsonExpr::Neg, a, nullptr) : nullptr;
    }
    return primary();
  }
  P primary() {
    ws();
    if (i >= p.size()) return nullptr;
    auto x = std::make_shared<JsonExpr>();
    const char c = p[i];
    if (c == '(') {
      i++;
      P e = orx();
      if (!e || !eat(")")) return nullptr;
      return e;
    }
    if (c == '@' || c == '$') {
      i++;
      x->op = JsonExpr::Path;
      x->root = c == '$';
      if (!parse_path_steps(p, i, x->steps, true)) return nullptr;
      return x;
    }
    if (c == '\'' || c == '"') {
      const size_t b = ++i;
      while (i < p.size() && p[i] != c) i++;
      if (i >= p.size()) return nullptr;
      x->lit.t = JVal::Str;
      x->lit.s = p.substr(b, i - b);
      i++;
      return x;
    }
    if (p.compare(i, 4, "true") == 0) { i += 4; x->lit.t = JVal::Bool; x->lit.b = true; return x; }
    if (p.compare(i, 5, "false") == 0) { i += 5; x->lit.t = JVal::Bool; x->lit.b = false; return x; }
    if (p.compare(i, 4, "null") == 0) { i += 4; x->lit.t = JVal::Null; return x; }
    if (std::isdigit((unsigned char)c) || c == '.') {
      const size_t b = i;
      while (i < p.size() && (std::isalnum((unsigned char)p[i]) || p[i] == '.' || p[i] == '_' ||
                              ((p[i] == '+' || p[i] == '-') && (p[i - 1] == 'e' || p[i - 1] == 'E'))))
        i++;
      x->lit.t = JVal::Num;
      if (!go_parse_float(p.substr(b, i - b), x->lit.n)) return nullptr;
      return x;
    }
    return nullptr;
  }
};

// jsonpath.Get on a plain path (Key / Index selectors only); false = an
// error (unknown key, index out of range, step on a non-container).
bool plain_select(const JsonPathStep& st, const JVal& cur, const JVal*& out) {
  if (st.kind == JsonPathStep::Index) {
    if (cur.t != JVal::Arr) return false;
    long long i = st.index;
    if (i < 0) i += (long long)cur.a.size();
    if (i < 0 || i >= (long long)cur.a.size()) return false;
    out = &cur.a[(size_t)i];
    return true;
  }
  if (cur.t != JVal::Obj) return false;
  auto it = cur.o.find(st.key);
  if (it == cur.o.end()) return false;
  out = &it->second;
  return true;
}

// The children of a container in visiting order: array order, object keys
// sorted (Go's map order is unspecified; sorted is one of its orders)
template <class F>
void visit_children(const JVal& v, F&& f) {
  if (v.t == JVal::Arr)
    for (const JVal& e : v.a) f(e);
  else if (v.t == JVal::Obj)
    for (const auto& kv : v.o) f(kv.second);
}

// One selector over one value: the matches it yields (an ambiguous path
// drops the branches a plain selector fails on instead of failing)
void select_step(const JsonPathStep& st, const JVal& v, std::vector<const JVal*>& out, const JVal& root) {
  switch (st.kind) {
    case JsonPathStep::Filter:
      visit_children(v, [&](const JVal& c) {
        if (truthy(eval_expr(*st.expr, c, root))) out.push_back(&c);
      });
      break;
    case JsonPathStep::Script: {
      const EV e = eval_expr(*st.expr, v, root);
      if (!e.ok) break;
      JsonPathStep sel;
      if (e.v.t == JVal::Num && std::floor(e.v.n) == e.v.n && std::fabs(e.v.n) < 9.0e15) {
        sel.kind = JsonPathStep::Index;
        sel.index = (long long)e.v.n;
      } else if (e.v.t == JVal::Str) {
        sel.kind = JsonPathStep::Key;
        sel.key = e.v.s;
      } else {
        break;
      }
      const JVal* r = nullptr;
      if (plain_select(sel, v, r)) out.push_back(r);
      break;
    }
    case JsonPathStep::Key:
    case JsonPathStep::Index: {
      const JVal* r = nullptr;
      if (plain_select(st, v, r)) out.push_back(r);
      break;
    }
    case JsonPathStep::Wild:
      visit_children(v, [&](const JVal& c) { out.push_back(&c); });
      break;
    case JsonPathStep::Union:
      for (const JsonPathStep& it : st.items) select_step(it, v, out, root);
      break;
    case JsonPathStep::Slice: {
      if (v.t != JVal::Arr) break;
      const long long n = (long long)v.a.size();
      long long lo = st.has_lo ? st.lo : 0, hi = st.has_hi ? st.hi : n;
      if (lo < 0) lo += n;
      if (hi < 0) hi += n;
      lo = std::max(0LL, std::min(lo, n));
      hi = std::max(0LL, std::min(hi, n));
      if (st.step > 0)
        for (long long k = lo; k < hi; k += st.step) out.push_back(&v.a[(size_t)k]);
      else if (st.step < 0)
        for (long long k = hi - 1; k >= lo; k += st.step) out.push_back(&v.a[(size_t)k]);
      break;
    }
    case JsonPathStep::Descend: {
      // `..x`: x over the value itself and every descendant, pre-order
      std::vector<const JVal*> stack{&v};
      while (!stack.empty()) {
        const JVal* cur = stack.back();
        stack.pop_back();
        select_step(st.items[0], *cur, out, root);
        std::vector<const JVal*> kids;
        visit_children(*cur, [&](const JVal& c) { kids.push_back(&c); });
        for (auto it = kids.rbegin(); it != kids.rend(); ++it) stack.push_back(*it);
      }
      break;
    }
  }
}

bool path_is_plain(const std::vector<JsonPathStep>& path) {
  for (const JsonPathStep& st : path)
    if (st.kind != JsonPathStep::Key && st.kind != JsonPathStep::Index) return false;
  return true;
}

// jsonpath.Get.  A plain path yields its value or an error (false); a path
// with an ambiguous selector never errs and yields the list of its matches
// (`holder` keeps that list).
bool jsonpath_get(const std::vector<JsonPathStep>& path, const JVal& root, const JVal*& out, JVal& holder) {
  if (path_is_plain(path)) {
    const JVal* cur = &root;
    for (const JsonPathStep& st : path)
      if (!plain_select(st, *cur, cur)) return false;
    out = cur;
    return true;
  }
  std::vector<const JVal*> cur{&root}, next;
  for (const JsonPathStep& st : path) {
    next.clear();
    for (const JVal* v : cur) select_step(st, *v, next, root);
    cur.swap(next);
  }
  holder = JVal{};
  holder.t = JVal::Arr;
  for (const JVal* v : cur) holder.a.push_back(*v);
  out = &holder;
  return true;
}

// A bracket item: 'key', "key" or an integer
bool parse_bracket_item(const std::string& p, size_t& i, JsonPathStep& out) {
  while (i < p.size() && p[i] == ' ') i++;
  if (i < p.size() && (p[i] == '\'' || p[i] == '"')) {
    const char q = p[i++];
    const size_t b = i;
    while (i < p.size() && p[i] != q) i++;
    if (i >= p.size()) return false;
    out.kind = JsonPathStep::Key;
    out.key = p.substr(b, i - b);
    i++;
  } else {
    const size_t b = i;
    if (i < p.size() && p[i] == '-') i++;
    while (i < p.size() && std::isdigit((unsigned char)p[i])) i++;
    if (i == b || (p[b] == '-' && i == b + 1)) return false;
    out.kind = JsonPathStep::Index;
    out.index = std::atoll(p.substr(b, i - b).c_str());
  }
  while (i < p.size() && p[i] == ' ') i++;
  return true;
}

bool parse_int_opt(const std::string& p, size_t& i, bool& has, long long& v) {
  while (i < p.size() && p[i] == ' ') i++;
  const size_t b = i;
  if (i < p.size() && p[i] == '-') i++;
  while (i < p.size() && std::isdigit((unsigned char)p[i])) i++;
  if (i == b) {
    has = false;
    return true;
  }
  if (p[b] == '-' && i == b + 1) return false;
  has = true;
  v = std::atoll(p.substr(b, i - b).c_str());
  while (i < p.size() && p[i] == ' ') i++;
  return true;
}

// `[...]` after the '[': *, 'k', n, unions of those, a:b:c slices
bool parse_bracket(const std::string& p, size_t& i, JsonPathStep& out) {
  while (i < p.size() && p[i] == ' ') i++;
  if (i < p.size() && (p[i] == '?' || p[i] == '(')) {   // filter [?(expr)] / script [(expr)]
    const bool filter = p[i] == '?';
    if (filter) i++;
    if (i >= p.size() || p[i] != '(') return false;
    i++;
    ExprParser ep(p, i);
    auto e = ep.orx();
    if (!e || !ep.eat(")")) return false;
    i = ep.i;
    while (i < p.size() && p[i] == ' ') i++;
    out = JsonPathStep{};
    out.kind = filter ? JsonPathStep::Filter : JsonPathStep::Script;
    out.expr = e;
    if (i >= p.size() || p[i] != ']') return false;
    i++;
    return true;
  }
  if (i < p.size() && p[i] == '*') {
    i++;
    while (i < p.size() && p[i] == ' ') i++;
    out.kind = JsonPathStep::Wild;
  } else {
    // a slice starts with an optional integer and a ':'
    size_t j = i;
    bool has_lo = false;
    long long lo = 0;
    if (parse_int_opt(p, j, has_lo, lo) && j < p.size() && p[j] == ':') {
      out = JsonPathStep{};
      out.kind = JsonPathStep::Slice;
      out.has_lo = has_lo;
      out.lo = lo;
      i = j + 1;
      if (!parse_int_opt(p, i, out.has_hi, out.hi)) return false;
      if (i < p.size() && p[i] == ':') {
        i++;
        bool has_step = false;
        if (!parse_int_opt(p, i, has_step, out.step)) return false;
        if (!has_step) out.step = 1;
      }
    } else {
      JsonPathStep first;
      if (!parse_bracket_item(p, i, first)) return false;
      if (i < p.size() && p[i] == ',') {
        out = JsonPathStep{};
        out.kind = JsonPathStep::Union;
        out.items.push_back(first);
        while (i < p.size() && p[i] == ',') {
          i++;
          JsonPathStep it;
          if (!parse_bracket_item(p, i, it)) return false;
          out.items.push_back(it);
        }
      } else {
        out = first;
      }
    }
  }
  if (i >= p.size() || p[i] != ']') return false;
  i++;
  return true;
}

// The selectors after `$` / `@`.  A whole path (in_expr false) must be
// consumed to its end; inside an expression the steps end at the first byte
// that starts no selector, and a name takes no '-' (the minus operator).
bool parse_path_steps(const std::string& p, size_t& i, std::vector<JsonPathStep>& out, bool in_expr) {
  auto name = [&](JsonPathStep& st) {
    const size_t b = i;
    while (i < p.size() && (std::isalnum((unsigned char)p[i]) || p[i] == '_' || (!in_expr && p[i] == '-'))) i++;
    if (i == b) return false;
    st.kind = JsonPathStep::Key;
    st.key = p.substr(b, i - b);
    return true;
  };
  while (i < p.size()) {
    if (in_expr && p[i] != '.' && p[i] != '[') return true;
    JsonPathStep st;
    if (p[i] == '.' && i + 1 < p.size() && p[i + 1] == '.') {
      i += 2;
      JsonPathStep sel;
      if (i < p.size() && p[i] == '*') {
        i++;
        sel.kind = JsonPathStep::Wild;
      } else if (i < p.size() && p[i] == '[') {
        i++;
        if (!parse_bracket(p, i, sel)) return false;
      } else if (!name(sel)) {
        return false;
      }
      st.kind = JsonPathStep::Descend;
      st.items.push_back(sel);
    } else if (p[i] == '.') {
      i++;
      if (i < p.size() && p[i] == '*') {
        i++;
        st.kind = JsonPathStep::Wild;
      } else if (!name(st)) {
        return false;
      }
    } else if (p[i] == '[') {
      i++;
      if (!parse_bracket(p, i, st)) return false;
    } else {
      return false;
    }
    out.push_back(std::move(st));
  }
  return true;
}

bool parse_jsonpath(const std::string& p, std::vector<JsonPathStep>& out) {
  if (p.empty() || p[0] != '$') return false;
  size_t i = 1;
  return parse_path_steps(p, i, out, false) && i == p.size();
}

}  // namespace

std::string SpanAttrPredicate::compile(const SpanAttributeRule& r) {
  service_ = r.service_name;
  key_ = r.attribute_key;
  cond_ = r.condition_type;
  op_ = r.operation;
  expected_ = r.expected_value;
  if (cond_ == "string" && op_ == "regex") {
    std::string err;
    RegexStatus st = re_.compile(expected_, err);
    if (st == RegexStatus::Ok) re_ok_ = true;
    else if (st == RegexStatus::Syntax) re_ok_ = false;   // regexp.Compile error: the span is skipped (:171-174)
    else return "span_attribute regex not supported by the DFA compiler: " + err;
  }
  if (cond_ == "number") num_ok_ = go_parse_float(expected_, num_);
  if (cond_ == "boolean") bool_ok_ = go_parse_bool(expected_, bool_);
  if (cond_ == "json" && (op_ == "contains_key" || op_ == "not_contains_key" || op_ == "key_equals" ||
                          op_ == "key_not_equals")) {
    if (!parse_jsonpath(r.json_path, path_))
      return "span_attribute json_path \"" + r.json_path +
             "\" is not a jsonpath the engine parses ($, .key, ['key'], [index], *, [a,b], [a:b:c], .., "
             "[?(expr)] and [(expr)])";
  }
  return "";
}

// One span of spanattribute.go:136-316, given that the attribute exists.
bool SpanAttrPredicate::eval(const Value& attr) const {
  if (cond_ == "string") {
    if (op_ == "exists" && attr.type == Value::TStr && !attr.s.empty()) return true;
    if (attr.type != Value::TStr) return false;
    const std::string& v = attr.s;
    if (op_ == "equals") return v == expected_;
    if (op_ == "not_equals") return v != expected_;
    if (op_ == "contains") return v.find(expected_) != std::string::npos;
    if (op_ == "not_contains") return v.find(expected_) == std::string::npos;
    if (op_ == "regex") return re_ok_ && re_.match(reinterpret_cast<const uint8_t*>(v.data()), v.size());
    return false;
  }
  if (cond_ == "number") {
    if (op_ == "exists" && (attr.type == Value::TInt || attr.type == Value::TDouble)) return true;
    if (!num_ok_) return false;
    double x;
    if (attr.type == Value::TInt) x = (double)attr.i;
    else if (attr.type == Value::TDouble) x = attr.d;
    else return false;
    if (op_ == "equals") return x == num_;
    if (op_ == "not_equals") return x != num_;
    if (op_ == "greater_than") return x > num_;
    if (op_ == "less_than") return x < num_;
    if (op_ == "greater_than_or_equal") return x >= num_;
    if (op_ == "less_than_or_equal") return x <= num_;
    return false;
  }
  if (cond_ == "boolean") {
    if (op_ == "exists" && attr.type == Value::TBool) return true;
    if (!bool_ok_ || attr.type != Value::TBool) return false;
    return op_ == "equals" && attr.b == bool_;
  }
  if (cond_ == "json") {
    if (attr.type != Value::TStr) return false;
    JVal root;
    const bool ok = json_unmarshal(attr.s, root);
    if (op_ == "is_valid_json") return ok;
    if (op_ == "is_invalid_json") return !ok;
    if (!ok) return false;
    const JVal* res = nullptr;
    JVal matches;
    const bool found = jsonpath_get(path_, root, res, matches);
    if (op_ == "contains_key") return found && res->t != JVal::Null;
    if (op_ == "not_contains_key") return !found;
    if (op_ == "key_equals" || op_ == "key_not_equals") {
      if (!found) return false;
      std::string vs;
      switch (res->t) {
        case JVal::Str: vs = res->s; break;
        case JVal::Num: vs = go_format_float_f(res->n); break;
        case JVal::Bool: vs = res->b ? "true" : "false"; break;
        case JVal::Null: vs = "null"; break;
        default: marshal(*res, vs); break;
      }
      return op_ == "key_equals" ? vs == expected_ : vs != expected_;
    }
    return false;   // "exists" / "jsonpath_exists": accepted by Validate, never satisfied (:241-315)
  }
  return false;
}

// A string "regex" rule whose DFA passes the device tables' bounds
// (Dfa::kMaxStates / kMaxTableBytes) is evaluated by the shim like a json
// rule (SpanAttrPredicate's HostRegexp takes it with a lazy DFA) instead of
// refusing the config; the answer per pattern is kept for the process.
bool regex_fits_device(const std::string& pattern) {
  static std::mutex mu;
  static std::map<std::string, bool> known;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = known.find(pattern);
    if (it != known.end()) return it->second;
  }
  Dfa d;
  std::string err;
  const bool fits = compile_dfa(pattern, d, err) != RegexStatus::TooLarge;
  std::lock_guard<std::mutex> lk(mu);
  if (known.size() > 4096) known.clear();
  known[pattern] = fits;
  return fits;
}

AttrPlan plan_attr_rules(const SamplingConfig& c) {
  AttrPlan p;
  int k = 0;
  for (auto* lvl : {&c.global_rules, &c.service_rules, &c.endpoint_rules})
    for (auto& r : *lvl) {
      if (r.rtype != RuleType::SpanAttribute) continue;
      if ((size_t)k / 64 >= p.host_mask.size()) p.host_mask.push_back(0);
      const bool host_regex = r.attr.condition_type == "string" && r.attr.operation == "regex" &&
                              !regex_fits_device(r.attr.expected_value);
      if (r.attr.condition_type == "json" || host_regex) {
        p.rule_key.push_back(-1);
        p.host_mask[k / 64] |= 1ull << (k % 64);
      } else {
        auto it = std::find(p.keys.begin(), p.keys.end(), r.attr.attribute_key);
        if (it == p.keys.end()) it = p.keys.insert(p.keys.end(), r.attr.attribute_key);
        p.rule_key.push_back((int)(it - p.keys.begin()));
      }
      k++;
    }
  return p;
}

}  // namespace ose
