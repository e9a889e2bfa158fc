// host_fuzz.cpp — driver for the ASan + UBSan build of the host code that
// parses untrusted input (tests/test_sanitize.py; test infrastructure, not
// part of the product library).
//
// usage: host_fuzz <mode> <file>...
//   pb        each file is one serialized TracesData: traces_from_protobuf
//             (the UnmarshalTraces restatement, otlp_pb.cpp), pb_walk, and for
//             accepted messages the OTLP/JSON form, the proto sizer and the
//             marshaler (pdata.cpp ProtoWriter) on the decoded traces
//   json      each file is OTLP/JSON: parse_json + traces_from_json
//   lines     each line of each file is "<kind>\t<text>": regex (RE2 syntax
//             check + DFA compile + a match), url (net/url.Parse path),
//             float (strconv.ParseFloat), config (processor config JSON),
//             attr (span_attribute rule JSON, then its predicate on a value)
// Prints one line per input: "<name> ok|rejected [detail]".  Any sanitizer
// report aborts the process (built with -fno-sanitize-recover=all).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

#include "../../odigos_amd/csrc/config.hpp"
#include "../../odigos_amd/csrc/json.hpp"
#include "../../odigos_amd/csrc/otlp_pb.hpp"
#include "../../odigos_amd/csrc/pdata.hpp"
#include "../../odigos_amd/csrc/regex_dfa.hpp"
#include "../../odigos_amd/csrc/span_attr.hpp"
#include "../../odigos_amd/csrc/urlparse.hpp"

using namespace ose;

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

static int run_pb(const char* name, const std::string& b) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(b.data());
  Traces td;
  std::string err;
  const bool ok = traces_from_protobuf(p, b.size(), td, err);
  PbWalk w;
  const bool wok = pb_walk(p, b.size(), w);
  if (ok) {
    std::string js;
    dump_json(js, traces_to_json(td));
    // the marshaler and the sizer over every part of the decoded traces
    std::string out;
    ProtoWriter pw(out);
    ProtoSizer sz;
    uint64_t total = 0;
    for (const auto& rs : td.resource_spans) {
      total += sz.resource_spans(rs);
      pw.resource(rs.resource_attrs, rs.resource_dropped);
      for (const auto& ss : rs.scope_spans) {
        pw.scope(ss);
        for (const auto& sp : ss.spans) pw.span(sp);
      }
    }
    printf("%s ok json=%zu pb=%zu size=%llu walk=%d\n", name, js.size(), out.size(), (unsigned long long)total,
           (int)wok);
  } else {
    printf("%s rejected walk=%d\n", name, (int)wok);
  }
  return 0;
}

static int run_json(const char* name, const std::string& b) {
  try {
    const Json j = parse_json(b);
    Traces td = traces_from_json(j);
    printf("%s ok resources=%zu\n", name, td.resource_spans.size());
  } catch (const std::exception& ex) {
    printf("%s rejected\n", name);
  }
  return 0;
}

static void run_line(const std::string& kind, const std::string& text, size_t k) {
  if (kind == "regex") {
    std::string err;
    Dfa d;
    const RegexStatus st = regex_syntax_check(text, err);
    const RegexStatus sc = compile_dfa(text, d, err);
    bool m = false;
    if (sc == RegexStatus::Ok) {
      m = dfa_match(d, reinterpret_cast<const uint8_t*>(text.data()), text.size());
      static const char* probes[] = {"", "a", "/users/123", "\xef\xbf\xbd", "\xff\xfe", "2024-01-02T03:04:05Z"};
      for (const char* s : probes) (void)dfa_match(d, reinterpret_cast<const uint8_t*>(s), strlen(s));
    }
    printf("regex %zu syntax=%d dfa=%d match=%d\n", k, (int)st, (int)sc, (int)m);
  } else if (kind == "url") {
    std::string path;
    const bool ok = go_url_parse_path(text, path);
    printf("url %zu %s %zu\n", k, ok ? "ok" : "rejected", path.size());
  } else if (kind == "float") {
    double v = 0;
    const bool ok = go_parse_float(text, v);
    bool bv = false;
    (void)go_parse_bool(text, bv);
    if (ok) (void)go_format_float_f(v);
    printf("float %zu %s\n", k, ok ? "ok" : "rejected");
  } else if (kind == "config") {
    try {
      const Json j = parse_json(text);
      UrlTemplateConfig u;
      SamplingConfig s;
      TrafficMetricsConfig t;
      const std::string e1 = decode_url_config(j, u), e2 = decode_sampling_config(j, s),
                        e3 = decode_traffic_config(j, t);
      printf("config %zu ok %d%d%d\n", k, (int)e1.empty(), (int)e2.empty(), (int)e3.empty());
    } catch (const std::exception&) {
      printf("config %zu rejected\n", k);
    }
  } else if (kind == "attr") {
    // "<rule json>\x1f<attribute value json>"
    const size_t sep = text.find('\x1f');
    try {
      const Json rj = parse_json(text.substr(0, sep));
      SamplingConfig s;
      Json wrap = parse_json("{\"global_rules\": []}");
      wrap.obj[0].second.arr.push_back(rj);
      const std::string e = decode_sampling_config(wrap, s);
      if (!e.empty() || s.global_rules.empty() || s.global_rules[0].rtype != RuleType::SpanAttribute) {
        printf("attr %zu rejected-config\n", k);
        return;
      }
      SpanAttrPredicate pred;
      const std::string ce = pred.compile(s.global_rules[0].attr);
      if (!ce.empty()) {
        printf("attr %zu refused\n", k);
        return;
      }
      Value v;
      if (sep != std::string::npos) v = Value::str(text.substr(sep + 1));
      printf("attr %zu eval=%d\n", k, (int)pred.eval(v));
    } catch (const std::exception&) {
      printf("attr %zu rejected\n", k);
    }
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: host_fuzz pb|json|lines <file>...\n");
    return 2;
  }
  const std::string mode = argv[1];
  for (int i = 2; i < argc; i++) {
    const std::string b = slurp(argv[i]);
    if (mode == "pb") run_pb(argv[i], b);
    else if (mode == "json") run_json(argv[i], b);
    else if (mode == "lines") {
      std::istringstream in(b);
      std::string line;
      size_t k = 0;
      while (std::getline(in, line)) {
        const size_t tab = line.find('\t');
        if (tab == std::string::npos) continue;
        run_line(line.substr(0, tab), line.substr(tab + 1), k++);
      }
    } else {
      fprintf(stderr, "unknown mode %s\n", mode.c_str());
      return 2;
    }
  }
  return 0;
}
