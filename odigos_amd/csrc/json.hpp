// json.hpp — minimal JSON DOM used for processor configs (the mapstructure
// maps the collector's confmap hands to Factory.CreateTraces) and for the
// OTLP/JSON trace fixtures of the host layer.  Numbers keep their source
// text so int64 values (timestamps) round-trip exactly.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ose {

struct Json {
  enum Type { Null, Bool, Number, String, Array, Object };
  Type type = Null;
  bool b = false;
  std::string s;                                 // String value, or Number text
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;  // insertion order kept

  bool is_null() const { return type == Null; }
  bool is_obj() const { return type == Object; }
  bool is_arr() const { return type == Array; }
  bool is_str() const { return type == String; }
  bool is_num() const { return type == Number; }
  bool is_bool() const { return type == Bool; }

  const Json* get(const std::string& k) const {
    if (type != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  double num() const { return std::strtod(s.c_str(), nullptr); }
  int64_t i64() const {
    // integers may arrive as numbers or (OTLP/JSON) as decimal strings
    if (s.find_first_of(".eE") != std::string::npos) return (int64_t)std::strtod(s.c_str(), nullptr);
    return (int64_t)std::strtoll(s.c_str(), nullptr, 10);
  }
  uint64_t u64() const { return (uint64_t)std::strtoull(s.c_str(), nullptr, 10); }

  static Json str(std::string v) { Json j; j.type = String; j.s = std::move(v); return j; }
  static Json number(std::string text) { Json j; j.type = Number; j.s = std::move(text); return j; }
  static Json boolean(bool v) { Json j; j.type = Bool; j.b = v; return j; }
  static Json array() { Json j; j.type = Array; return j; }
  static Json object() { Json j; j.type = Object; return j; }
  Json& set(const std::string& k, Json v) {
    for (auto& kv : obj)
      if (kv.first == k) { kv.second = std::move(v); return kv.second; }
    obj.emplace_back(k, std::move(v));
    return obj.back().second;
  }
  Json& push(Json v) { arr.push_back(std::move(v)); return arr.back(); }
};

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class JsonParser {
 public:
  explicit JsonParser(const std::string& t) : t_(t) {}
  Json parse() {
    Json v = value();
    ws();
    if (i_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t i_ = 0;
  // nesting bound: the parser recurses per array / object level (deeper
  // input is refused instead of overflowing the caller's stack; Go's
  // encoding/json stops at 10000 levels, configs and OTLP/JSON stay far below)
  static constexpr int kMaxDepth = 1000;
  int depth_ = 0;
  struct Nest {
    JsonParser& p;
    explicit Nest(JsonParser& q) : p(q) {
      if (++p.depth_ > kMaxDepth) p.fail("nesting too deep");
    }
    ~Nest() { p.depth_--; }
  };
  [[noreturn]] void fail(const char* m) { throw JsonError(std::string("json: ") + m + " at offset " + std::to_string(i_)); }
  void ws() { while (i_ < t_.size() && (t_[i_] == ' ' || t_[i_] == '\n' || t_[i_] == '\r' || t_[i_] == '\t')) i_++; }
  bool lit(const char* w) {
    size_t n = std::char_traits<char>::length(w);
    if (t_.compare(i_, n, w) == 0) { i_ += n; return true; }
    return false;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  }
  uint32_t hex4() {
    if (i_ + 4 > t_.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      char c = t_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }
  std::string string_body() {
    std::string o;
    for (;;) {
      if (i_ >= t_.size()) fail("unterminated string");
      char c = t_[i_++];
      if (c == '"') return o;
      if (c != '\\') { o += c; continue; }
      if (i_ >= t_.size()) fail("bad escape");
      char e = t_[i_++];
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
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= t_.size() && t_[i_] == '\\' && t_[i_ + 1] == 'u') {
            size_t save = i_;
            i_ += 2;
            uint32_t lo = hex4();
            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else i_ = save;
          }
          put_utf8(o, cp);
          break;
        }
        case 'x': {  // extension: raw byte \xHH (lets fixtures carry invalid UTF-8)
          if (i_ + 2 > t_.size()) fail("bad \\x escape");
          o += (char)std::strtol(t_.substr(i_, 2).c_str(), nullptr, 16);
          i_ += 2;
          break;
        }
        default: fail("bad escape");
      }
    }
  }
  Json value() {
    ws();
    if (i_ >= t_.size()) fail("unexpected end");
    char c = t_[i_];
    if (c == '{') {
      Nest nest(*this);
      i_++;
      Json o = Json::object();
      ws();
      if (i_ < t_.size() && t_[i_] == '}') { i_++; return o; }
      for (;;) {
        ws();
        if (i_ >= t_.size() || t_[i_] != '"') fail("expected key");
        i_++;
        std::string k = string_body();
        ws();
        if (i_ >= t_.size() || t_[i_] != ':') fail("expected ':'");
        i_++;
        o.obj.emplace_back(std::move(k), value());
        ws();
        if (i_ < t_.size() && t_[i_] == ',') { i_++; continue; }
        if (i_ < t_.size() && t_[i_] == '}') { i_++; return o; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      Nest nest(*this);
      i_++;
      Json a = Json::array();
      ws();
      if (i_ < t_.size() && t_[i_] == ']') { i_++; return a; }
      for (;;) {
        a.arr.push_back(value());
        ws();
        if (i_ < t_.size() && t_[i_] == ',') { i_++; continue; }
        if (i_ < t_.size() && t_[i_] == ']') { i_++; return a; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') { i_++; return Json::str(string_body()); }
    if (lit("true")) return Json::boolean(true);
    if (lit("false")) return Json::boolean(false);
    if (lit("null")) return Json();
    size_t st = i_;
    if (t_[i_] == '-' || t_[i_] == '+') i_++;
    while (i_ < t_.size() && ((t_[i_] >= '0' && t_[i_] <= '9') || t_[i_] == '.' || t_[i_] == 'e' || t_[i_] == 'E' || t_[i_] == '-' || t_[i_] == '+')) i_++;
    if (st == i_) fail("unexpected character");
    return Json::number(t_.substr(st, i_ - st));
  }
};

inline Json parse_json(const std::string& t) { return JsonParser(t).parse(); }

inline void json_escape(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        // bytes >= 0x80 are emitted as \u00XX so output is ASCII and the
        // exact byte string (valid UTF-8 or not) is recovered by latin-1
        if (c < 0x20 || c >= 0x80) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
        else o += (char)c;
    }
  }
  o += '"';
}

// Serialises a DOM (strings byte-exact, see json_escape).
inline void dump_json(std::string& o, const Json& j) {
  switch (j.type) {
    case Json::Null: o += "null"; break;
    case Json::Bool: o += j.b ? "true" : "false"; break;
    case Json::Number: o += j.s; break;
    case Json::String: json_escape(o, j.s); break;
    case Json::Array:
      o += '[';
      for (size_t k = 0; k < j.arr.size(); k++) { if (k) o += ','; dump_json(o, j.arr[k]); }
      o += ']';
      break;
    case Json::Object:
      o += '{';
      for (size_t k = 0; k < j.obj.size(); k++) {
        if (k) o += ',';
        json_escape(o, j.obj[k].first);
        o += ':';
        dump_json(o, j.obj[k].second);
      }
      o += '}';
      break;
  }
}

}  // namespace ose
