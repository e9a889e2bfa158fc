// urlparse.cpp — net/url.Parse(rawURL).Path as used by
// calculateTemplatedUrlFromAttr (odigosurltemplateprocessor/processor.go:
// 196-208): returns false where url.Parse returns an error (the span is then
// left untouched), else the decoded Path.  Restates go1.25 net/url
// (Parse, parse, getScheme, parseAuthority, parseHost, validOptionalPort,
// validUserinfo, unescape, setPath, setFragment).  Host-side columnarisation
// only; parity pinned by processor_test.go:154-191 and :349-359, the rest of
// the grammar is parity unpinned.
#include "urlparse.hpp"

#include <cstring>

namespace ose {
namespace {

enum Mode { kPath, kHost, kZone, kUserPassword, kFragment };

bool ishex(char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
int unhex(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return c - 'A' + 10;
}

// shouldEscape (only the modes unescape consults)
bool should_escape(unsigned char c, Mode mode) {
  if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9')) return false;
  if (mode == kHost || mode == kZone) {
    switch (c) {
      case '!': case '$': case '&': case '\'': case '(': case ')': case '*': case '+': case ',':
      case ';': case '=': case ':': case '[': case ']': case '<': case '>': case '"':
        return false;
    }
  }
  switch (c) {
    case '-': case '_': case '.': case '~': return false;
    case '$': case '&': case '+': case ',': case '/': case ':': case ';': case '=': case '?': case '@':
      switch (mode) {
        case kPath: return c == '?';
        case kUserPassword: return c == '@' || c == '/' || c == '?' || c == ':';
        case kFragment: return false;
        default: return true;
      }
  }
  if (mode == kFragment) {
    switch (c) {
      case '!': case '(': case ')': case '*': return false;
    }
  }
  return true;
}

bool unescape(const std::string& s, Mode mode, std::string& out) {
  size_t n = 0;
  for (size_t i = 0; i < s.size();) {
    if (s[i] == '%') {
      n++;
      if (i + 2 >= s.size() || !ishex(s[i + 1]) || !ishex(s[i + 2])) return false;
      if (mode == kHost && unhex(s[i + 1]) < 8 && s.compare(i, 3, "%25") != 0) return false;
      if (mode == kZone) {
        int v = unhex(s[i + 1]) << 4 | unhex(s[i + 2]);
        if (s.compare(i, 3, "%25") != 0 && v != ' ' && should_escape((unsigned char)v, kHost)) return false;
      }
      i += 3;
    } else {
      if ((mode == kHost || mode == kZone) && (unsigned char)s[i] < 0x80 && should_escape((unsigned char)s[i], mode))
        return false;
      i++;
    }
  }
  out.clear();
  if (n == 0) { out = s; return true; }
  for (size_t i = 0; i < s.size();) {
    if (s[i] == '%') { out += (char)(unhex(s[i + 1]) << 4 | unhex(s[i + 2])); i += 3; }
    else { out += s[i]; i++; }
  }
  return true;
}

bool valid_optional_port(const std::string& p) {
  if (p.empty()) return true;
  if (p[0] != ':') return false;
  for (size_t i = 1; i < p.size(); i++)
    if (p[i] < '0' || p[i] > '9') return false;
  return true;
}

bool parse_host(const std::string& host, std::string& out) {
  if (!host.empty() && host[0] == '[') {
    size_t i = host.rfind(']');
    if (i == std::string::npos) return false;
    std::string colon_port = host.substr(i + 1);
    if (!valid_optional_port(colon_port)) return false;
    size_t zone = host.substr(0, i).find("%25");
    if (zone != std::string::npos) {
      std::string h1, h2, h3;
      if (!unescape(host.substr(0, zone), kHost, h1)) return false;
      if (!unescape(host.substr(zone, i - zone), kZone, h2)) return false;
      if (!unescape(host.substr(i), kHost, h3)) return false;
      out = h1 + h2 + h3;
      return true;
    }
  } else {
    size_t i = host.rfind(':');
    if (i != std::string::npos && !valid_optional_port(host.substr(i))) return false;
  }
  return unescape(host, kHost, out);
}

// validUserinfo: RFC 3986 userinfo characters
bool valid_userinfo(const std::string& s) {
  for (unsigned char r : s) {
    if ((r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || (r >= '0' && r <= '9')) continue;
    switch (r) {
      case '-': case '.': case '_': case ':': case '~': case '!': case '$': case '&': case '\'':
      case '(': case ')': case '*': case '+': case ',': case ';': case '=': case '%': case '@':
        continue;
      default:
        if (r >= 0x80) continue;   // validUserinfo ranges over runes; only ASCII is checked
        return false;
    }
  }
  return true;
}

bool parse_authority(const std::string& authority) {
  size_t i = authority.rfind('@');
  std::string host;
  if (!parse_host(i == std::string::npos ? authority : authority.substr(i + 1), host)) return false;
  if (i == std::string::npos) return true;
  std::string userinfo = authority.substr(0, i);
  if (!valid_userinfo(userinfo)) return false;
  std::string tmp;
  size_t c = userinfo.find(':');
  if (c == std::string::npos) return unescape(userinfo, kUserPassword, tmp);
  return unescape(userinfo.substr(0, c), kUserPassword, tmp) && unescape(userinfo.substr(c + 1), kUserPassword, tmp);
}

}  // namespace

bool go_url_parse_path(const std::string& raw, std::string& path) {
  path.clear();
  size_t hash = raw.find('#');
  std::string u = hash == std::string::npos ? raw : raw.substr(0, hash);
  std::string frag = hash == std::string::npos ? std::string() : raw.substr(hash + 1);
  // parse(u, viaRequest=false)
  for (unsigned char c : u)
    if (c < 0x20 || c == 0x7F) return false;   // invalid control character
  if (u == "*") {
    path = "*";
  } else {
    // getScheme
    std::string scheme, rest = u;
    for (size_t i = 0; i < u.size(); i++) {
      char c = u[i];
      if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) continue;
      if ((c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.') {
        if (i == 0) break;
        continue;
      }
      if (c == ':') {
        if (i == 0) return false;   // missing protocol scheme
        scheme = u.substr(0, i);
        rest = u.substr(i + 1);
      }
      break;
    }
    size_t q = rest.find('?');
    size_t qcount = 0;
    for (char c : rest) qcount += c == '?';
    if (!rest.empty() && rest.back() == '?' && qcount == 1) rest.pop_back();
    else if (q != std::string::npos) rest = rest.substr(0, q);
    if (rest.empty() || rest[0] != '/') {
      if (!scheme.empty()) {
        // opaque URL: Path stays ""
        rest.clear();
        goto fragment;
      }
      size_t slash = rest.find('/');
      std::string seg = slash == std::string::npos ? rest : rest.substr(0, slash);
      if (seg.find(':') != std::string::npos) return false;   // first path segment cannot contain colon
    }
    if ((!scheme.empty() || rest.compare(0, 3, "///") != 0) && rest.compare(0, 2, "//") == 0) {
      std::string authority = rest.substr(2);
      rest.clear();
      size_t i = authority.find('/');
      if (i != std::string::npos) { rest = authority.substr(i); authority = authority.substr(0, i); }
      if (!parse_authority(authority)) return false;
    }
    if (!unescape(rest, kPath, path)) return false;   // setPath
  }
fragment:
  if (hash != std::string::npos && !frag.empty()) {
    std::string tmp;
    if (!unescape(frag, kFragment, tmp)) return false;   // setFragment
  }
  return true;
}

}  // namespace ose
