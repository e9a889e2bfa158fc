// gen_otlp.cpp — a serialized TracesData for the OTLP ingest benchmark and
// tests (bench/test infrastructure, part of libosegen): the resources,
// spans, times, statuses, kinds, paths and routes of a generated batch
// (gen_batch.cpp), written as OTLP trace.proto messages with the attributes
// an HTTP instrumentation sets, encoded as pdata's marshaler writes them
// (what a node collector's OTLP exporter sends the gateway: proto3 defaults
// omitted, ids and Status always framed); resources are encoded in parallel
// chunks (TracesData is a concatenation of ResourceSpans fields).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/odigos_amd.h"

namespace {

void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) { o += (char)(v | 0x80); v >>= 7; }
  o += (char)v;
}
void put_tag(std::string& o, uint32_t field, uint32_t wt) { put_varint(o, ((uint64_t)field << 3) | wt); }
void put_bytes(std::string& o, uint32_t field, const char* p, size_t n) {
  put_tag(o, field, 2);
  put_varint(o, n);
  o.append(p, n);
}
void put_str(std::string& o, uint32_t field, const std::string& s) { put_bytes(o, field, s.data(), s.size()); }
void put_fixed64(std::string& o, uint32_t field, uint64_t v) {
  put_tag(o, field, 1);
  char b[8];
  std::memcpy(b, &v, 8);
  o.append(b, 8);
}
void put_msg(std::string& o, uint32_t field, const std::string& m) { put_bytes(o, field, m.data(), m.size()); }
// KeyValue{key, AnyValue{string_value}} / {int_value}
void kv_str(std::string& o, uint32_t field, const char* k, const char* v, size_t vl) {
  std::string av, kv;
  put_bytes(av, 1, v, vl);
  put_bytes(kv, 1, k, std::strlen(k));
  put_msg(kv, 2, av);
  put_msg(o, field, kv);
}
void kv_int(std::string& o, uint32_t field, const char* k, int64_t v) {
  std::string av, kv;
  put_tag(av, 3, 0);
  put_varint(av, (uint64_t)v);
  put_bytes(kv, 1, k, std::strlen(k));
  put_msg(kv, 2, av);
  put_msg(o, field, kv);
}
uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
const char* kMethod[] = {"GET", "POST", "PUT", "DELETE"};

struct Res { uint64_t first, count; };

void encode_resources(const ose_columns* c, const std::vector<Res>& res, size_t r0, size_t r1, std::string& out) {
  std::string rs, sc, sp, tmp;
  for (size_t r = r0; r < r1; r++) {
    rs.clear();
    {   // Resource
      std::string resm;
      char name[32];
      const uint32_t svc = c->res_svc[r] == OSE_NONE ? 99 : c->res_svc[r];
      std::snprintf(name, sizeof name, "svc-%02u", svc);
      kv_str(resm, 1, "service.name", name, std::strlen(name));
      kv_str(resm, 1, "k8s.namespace.name", "default", 7);
      kv_str(resm, 1, "k8s.deployment.name", name, std::strlen(name));   // what k8sattributes adds
      char pod[32];
      std::snprintf(pod, sizeof pod, "pod-%u", c->res_attrset[r] % 4);
      kv_str(resm, 1, "k8s.pod.name", pod, std::strlen(pod));
      kv_str(resm, 1, "telemetry.sdk.language", "go", 2);
      put_msg(rs, 1, resm);
    }
    sc.clear();
    {   // InstrumentationScope
      std::string scm;
      put_str(scm, 1, "go.opentelemetry.io/contrib/instrumentation/net/http");
      put_str(scm, 2, "0.53.0");
      put_msg(sc, 1, scm);
    }
    for (uint64_t i = res[r].first; i < res[r].first + res[r].count; i++) {
      sp.clear();
      char id[16];
      for (int k = 0; k < 8; k++) id[k] = (char)(c->trace_id[2 * i] >> (56 - 8 * k));
      for (int k = 0; k < 8; k++) id[8 + k] = (char)(c->trace_id[2 * i + 1] >> (56 - 8 * k));
      put_bytes(sp, 1, id, 16);
      const uint64_t h = mix(i ^ c->trace_id[2 * i]);
      std::memcpy(id, &h, 8);
      put_bytes(sp, 2, id, 8);
      if (h & 3) {
        const uint64_t h2 = mix(h);
        std::memcpy(id, &h2, 8);
        put_bytes(sp, 4, id, 8);
      } else {
        put_bytes(sp, 4, id, 0);   // pdata frames an empty parent id
      }
      const uint8_t f = c->url_flags[i];
      const char* method = kMethod[h >> 62];
      if (f & OSE_URL_NAME_EQ_METHOD) {
        put_str(sp, 5, method);
      } else {
        tmp.assign("op-");
        tmp.append(std::to_string(h % 100000));
        put_str(sp, 5, tmp);
      }
      if (c->kind[i]) { put_tag(sp, 6, 0); put_varint(sp, c->kind[i]); }
      if (c->start_ns[i]) put_fixed64(sp, 7, c->start_ns[i]);
      if (c->end_ns[i]) put_fixed64(sp, 8, c->end_ns[i]);
      if (f & OSE_URL_HAS_METHOD) kv_str(sp, 9, "http.request.method", method, std::strlen(method));
      const ose_strref rt = c->route[i];
      const uint32_t tgt = f & OSE_URL_TGT_MASK;
      if (c->kind[i] == OSE_KIND_SERVER && (rt.len || tgt == OSE_URL_TGT_STR_EMPTY))
        kv_str(sp, 9, "http.route", (const char*)c->arena + rt.off, rt.len);
      if (c->kind[i] == OSE_KIND_CLIENT && tgt == OSE_URL_TGT_STR) kv_str(sp, 9, "url.template", "/t/{id}", 7);
      const ose_strref p = c->path[i];
      if ((f & OSE_URL_PATH_MASK) == OSE_URL_PATH_RAW) kv_str(sp, 9, "url.path", (const char*)c->arena + p.off, p.len);
      if ((f & OSE_URL_PATH_MASK) == OSE_URL_PATH_TARGET)
        kv_str(sp, 9, "http.target", (const char*)c->arena + p.off, p.len);
      if (f & OSE_URL_HAS_METHOD) {   // what an HTTP instrumentation adds next to them
        kv_int(sp, 9, "http.response.status_code", c->status[i] == OSE_STATUS_ERROR ? 500 : 200);
        static const char kUa[] = "Mozilla/5.0 (X11; Linux x86_64) odigos-bench/1.0";
        kv_str(sp, 9, "server.address", "api.internal.svc", 16);
        kv_str(sp, 9, "network.protocol.version", "1.1", 3);
        kv_str(sp, 9, "user_agent.original", kUa, sizeof kUa - 1);
      }
      {   // Status: non-nullable, always framed
        std::string st;
        if (c->status[i]) {
          put_tag(st, 3, 0);
          put_varint(st, c->status[i]);
        }
        put_msg(sp, 15, st);
      }
      put_msg(sc, 2, sp);
    }
    put_msg(rs, 2, sc);
    put_msg(out, 1, rs);
  }
}

}  // namespace

extern "C" {

// TracesData bytes of the batch `cols` (as osegen_columns returns it: spans
// in resource order, one scope per resource).  *len receives the size;
// free with osegen_otlp_free.
char* osegen_otlp(const ose_columns* c, int threads, uint64_t* len) {
  std::vector<Res> res(c->n_resources, Res{0, 0});
  for (uint64_t i = 0; i < c->n_spans; i++) {
    const uint32_t r = c->resource[i];
    if (res[r].count == 0) res[r].first = i;
    res[r].count++;
  }
  if (threads < 1) threads = 1;
  const size_t R = res.size();
  std::vector<std::string> parts((size_t)threads);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t]() { encode_resources(c, res, R * t / threads, R * (t + 1) / threads, parts[t]); });
  for (auto& x : th) x.join();
  uint64_t total = 0;
  for (auto& p : parts) total += p.size();
  char* out = static_cast<char*>(std::malloc(total ? total : 1));
  uint64_t off = 0;
  for (auto& p : parts) {
    std::memcpy(out + off, p.data(), p.size());
    off += p.size();
  }
  *len = total;
  return out;
}

void osegen_otlp_free(char* p) { std::free(p); }

}  // extern "C"
