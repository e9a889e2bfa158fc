// gen_batch.cpp — seeded synthetic batches in the ose_columns layout
// (bench / test infrastructure, built into libosegen.so; not product code).
//
// Workloads follow SURVEY.md §8(d):
//   url      C2: kinds 45/35/20 % server/client/internal, 80 % with a method,
//            path source 70 % url.path / 20 % http.target (half with ?query)
//            / 10 % target attribute already set (1 % empty); 1-6 segments
//            (mean 3.2) drawn from the C2 segment mix.
//   sampling C3: traces of 1-19 spans, 1-4 services (of 64) per trace, 2 %
//            error spans, lognormal durations (median 20 ms, sigma 1.5,
//            clipped to [1 us, 60 s]), http.route on 50 % of server spans
//            from 200 routes.
//   fused    C4: both mixes on every span.
//   zipf     C5: trace sizes Zipf(1.1) truncated to [1, 50000], plus the
//            high-cardinality half: http.route from 1M distinct routes and
//            paths carrying 64-bit user ids.
// Spans are grouped by trace (groupbytrace release order) unless shuffle=1,
// which permutes whole resources across the batch.
//
// Split mode (osegen_create_split): the batch one of `world` node collectors
// holds.  Trace structure (id, size, timing, services) is shared by every
// source; each ResourceSpans (one (trace, service) group) lands on the
// source hash(trace, resource) mod world, as spans of one trace reach the
// gateway through the node collectors of the services that emitted them
// (autoscaler/controllers/nodecollector/collectorconfig/traces.go:26-84).
// Concatenating the sources in rank order gives the same resources as the
// world = 1 batch of the same seed.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/odigos_amd.h"

namespace {

struct Rng {  // xoshiro256**
  uint64_t s[4];
  static uint64_t sm(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) { for (auto& v : s) v = sm(seed); }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  double unit() { return (double)(next() >> 11) * 0x1.0p-53; }
  bool chance(double p) { return unit() < p; }
  double normal() {
    double u1 = unit(), u2 = unit();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

const char* kWords[] = {"users", "orders", "items", "products", "cart", "checkout", "api", "v1", "v2", "search",
                        "accounts", "profile", "settings", "billing", "invoices", "payments", "auth", "login",
                        "logout", "session", "health", "metrics", "status", "catalog", "reviews", "comments",
                        "friends", "groups", "teams", "projects", "tasks", "files", "upload", "download",
                        "images", "thumbnails", "reports", "admin", "config", "events", "notifications",
                        "messages", "inbox", "feed", "timeline", "tags", "categories", "inventory",
                        "shipping", "returns"};
constexpr int kNWords = sizeof(kWords) / sizeof(kWords[0]);
const char* kMethods[] = {"GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"};

struct Mix {
  bool url = true, sampling = false, zipf = false, hicard = false;
  double p_route = 0.10;     // server spans carrying http.route already
};

struct Chunk {
  std::string arena;
  std::vector<uint64_t> trace_id, start, end;
  std::vector<uint8_t> status, kind, url_flags;
  std::vector<uint32_t> res_local, span_size, name_len;
  std::vector<ose_strref> path, route;
  // per resource
  std::vector<uint32_t> res_svc, res_svc_str, res_attrset, res_size, scope_size, res_first_span;
  std::vector<uint8_t> res_url_ok;
};

void gen_word(Rng& r, std::string& s) {
  // 500-word dictionary: base word + optional numeric-free suffix
  int w = (int)r.below(kNWords);
  s += kWords[w];
  uint32_t v = r.below(10);
  if (v < 9) { static const char* suf[] = {"", "list", "info", "data", "view", "item", "summary", "detail", "page"}; s += suf[v]; }
}
void gen_hex(Rng& r, std::string& s, int n, bool upper_mix) {
  static const char* lo = "0123456789abcdef";
  static const char* up = "0123456789ABCDEF";
  bool upper = upper_mix && r.chance(0.3);
  for (int i = 0; i < n; i++) s += (upper ? up : lo)[r.below(16)];
}
void gen_uuid(Rng& r, std::string& s) {
  bool deco = r.chance(0.10);
  bool pre = deco && r.chance(0.5);
  if (pre) s += "PROCESS_";
  const int g[5] = {8, 4, 4, 4, 12};
  for (int k = 0; k < 5; k++) { if (k) s += '-'; gen_hex(r, s, g[k], true); }
  if (deco && !pre) s += "_job";
}
void gen_digits(Rng& r, std::string& s, int n) { for (int i = 0; i < n; i++) s += (char)('0' + r.below(10)); }
void gen_date(Rng& r, std::string& s) {
  // the 10 accepted shapes: D, DZ, D+z, DTHM, DTHMZ, DTHM+z, DTHMS, DTHMSZ, DTHMS+z; plus a negative (day-first)
  uint32_t shape = r.below(10);
  if (shape == 9) { s += "04-12-2025T14:15:16"; return; }
  s += "2025-"; gen_digits(r, s, 2); s += '-'; gen_digits(r, s, 2);
  uint32_t t = shape / 3, z = shape % 3;
  if (t >= 1) { s += 'T'; gen_digits(r, s, 2); s += ':'; gen_digits(r, s, 2); }
  if (t >= 2) { s += ':'; gen_digits(r, s, 2); }
  if (z == 1) s += 'Z';
  if (z == 2) { s += r.chance(0.5) ? '+' : '-'; gen_digits(r, s, 4); }
}
void gen_segment(Rng& r, std::string& s) {
  uint32_t p = r.below(100);
  if (p < 45) gen_word(r, s);
  else if (p < 65) gen_digits(r, s, 1 + (int)r.below(12));
  else if (p < 75) gen_uuid(r, s);
  else if (p < 83) gen_hex(r, s, 16 + 8 * (int)r.below(3), true);
  else if (p < 87) gen_hex(r, s, 17 + 2 * (int)r.below(7), false);   // odd length: negative case
  else if (p < 91) gen_date(r, s);
  else if (p < 94) {
    static const char* dom[] = {"gmail.com", "example.io", "corp.example.co.uk", "mail.org"};
    s += "user"; gen_digits(r, s, 3); s += r.chance(0.3) ? "+tag" : ""; s += '@'; s += dom[r.below(4)];
  } else if (p < 97) {
    static const char* mixes[] = {"INC", "v", "inc_", "sb_"};
    int k = (int)r.below(4);
    s += mixes[k];
    gen_digits(r, s, k == 1 ? 4 : 4 + (int)r.below(8));
    if (k == 1) { s += '-'; gen_digits(r, s, 4); }
  } else {
    switch (r.below(4)) {
      case 0: break;                                   // empty segment ("//")
      case 1: s += "text\xEF\xBF\xBD"; break;           // U+FFFD
      case 2: s += "bad\xC3"; s += "x"; break;         // invalid UTF-8
      default: s += "caf\xC3\xA9"; break;              // valid non-ASCII
    }
  }
}

void gen_path(Rng& r, std::string& s) {
  static const double cdf[6] = {0.15, 0.35, 0.60, 0.80, 0.92, 1.0};
  double u = r.unit();
  int nseg = 1;
  while (nseg < 6 && u > cdf[nseg - 1]) nseg++;
  bool lead = !r.chance(0.02);
  if (lead) s += '/';
  for (int k = 0; k < nseg; k++) { if (k) s += '/'; gen_segment(r, s); }
  if (r.chance(0.03)) s += '/';   // trailing slash -> empty last segment
}

ose_strref add(std::string& arena, const std::string& s) {
  ose_strref ref{(uint32_t)arena.size(), (uint32_t)s.size()};
  arena += s;
  return ref;
}

// One trace (sampling/fused/zipf) or a run of independent spans (url).
// world == 0: classic batch; world >= 1: split mode, only the resources of
// source `rank` are emitted (their span contents come from a per-resource
// generator, so a skipped resource costs no draws)
void gen_chunk(uint64_t seed, uint64_t n_spans, const Mix& mx, Chunk& c, uint32_t rank = 0, uint32_t world = 0) {
  Rng r(seed);
  uint64_t trace_no = 0;
  std::string tmp;
  uint64_t made = 0;
  while (made < n_spans) {
    // trace shape
    uint64_t tsz;
    if (mx.zipf) {
      // Zipf(s=1.1) on [1, 50000] by rejection-inversion (approximate, seeded)
      double u = r.unit();
      double x = std::pow(1.0 - u * (1.0 - std::pow(50000.0, -0.1)), -1.0 / 0.1);
      tsz = std::min<uint64_t>(50000, std::max<uint64_t>(1, (uint64_t)x));
    } else if (mx.sampling) {
      tsz = 1 + r.below(19);
    } else {
      tsz = 1;
    }
    tsz = std::min<uint64_t>(tsz, n_spans - made);
    uint64_t hi = r.next(), lo = r.next();
    uint32_t nsvc = mx.sampling ? 1 + r.below(4) : 1;
    nsvc = (uint32_t)std::min<uint64_t>(nsvc, tsz);
    uint64_t base = 1700000000000000000ull + (r.next() % 100000000000000000ull);
    double dur_ms = std::exp(std::log(20.0) + 1.5 * r.normal());
    dur_ms = std::min(60000.0, std::max(0.001, dur_ms));
    uint64_t trace_dur = (uint64_t)(dur_ms * 1e6);
    // split the spans over the trace's services (one resource each)
    uint64_t left = tsz;
    trace_no++;
    for (uint32_t sv = 0; sv < nsvc; sv++) {
      uint64_t k = sv == nsvc - 1 ? left : 1 + r.below((uint32_t)std::min<uint64_t>(left - (nsvc - 1 - sv), 1u << 30)) ;
      if (k > left - (nsvc - 1 - sv)) k = left - (nsvc - 1 - sv);
      left -= k;
      Rng rres(seed ^ (trace_no * 0xD1B54A32D192ED03ull) ^ ((uint64_t)(sv + 1) * 0x8CB92BA72F3D8DD7ull));
      if (world) {
        uint64_t h = hi ^ (0x9E3779B97F4A7C15ull * (sv + 1));
        if ((uint32_t)(Rng::sm(h) % world) != rank) continue;
      }
      Rng& q_r = world ? rres : r;   // the resource's span contents
      uint32_t svc = q_r.below(64);
      uint32_t res = (uint32_t)c.res_svc.size();
      c.res_svc.push_back(svc);
      c.res_svc_str.push_back(q_r.chance(0.02) ? OSE_NONE : svc);   // 2 % service.name not a Str
      c.res_url_ok.push_back(q_r.chance(0.97) ? 1 : 0);
      c.res_attrset.push_back(svc * 4 + q_r.below(4));
      c.res_size.push_back(180 + q_r.below(240));
      c.scope_size.push_back(20 + q_r.below(40));
      c.res_first_span.push_back((uint32_t)c.kind.size());
      for (uint64_t q = 0; q < k; q++) {
        c.trace_id.push_back(hi);
        c.trace_id.push_back(lo);
        uint64_t off = trace_dur ? q_r.next() % (trace_dur + 1) : 0;
        uint64_t st = base + off;
        uint64_t en = st + (trace_dur - off) * (uint64_t)q_r.below(1000) / 1000;
        c.start.push_back(st);
        c.end.push_back(en);
        c.status.push_back(q_r.chance(0.02) ? OSE_STATUS_ERROR : (q_r.chance(0.5) ? OSE_STATUS_OK : OSE_STATUS_UNSET));
        uint32_t kp = q_r.below(100);
        uint8_t kind = kp < 45 ? OSE_KIND_SERVER : (kp < 80 ? OSE_KIND_CLIENT : OSE_KIND_INTERNAL);
        c.kind.push_back(kind);
        c.res_local.push_back(res);
        uint8_t f = 0;
        ose_strref pref{0, 0}, rref{0, 0};
        const char* method = kMethods[q_r.below(3) ? q_r.below(2) : q_r.below(7)];
        bool http = (kind == OSE_KIND_SERVER || kind == OSE_KIND_CLIENT) && q_r.chance(0.8);
        bool has_route = kind == OSE_KIND_SERVER && q_r.chance(mx.p_route);
        uint32_t nl;
        if (http) {
          f |= OSE_URL_HAS_METHOD;
          bool eq = q_r.chance(0.7);
          if (eq) f |= OSE_URL_NAME_EQ_METHOD;
          nl = eq ? (uint32_t)std::strlen(method) : 8 + q_r.below(32);
          if (has_route) {
            f |= q_r.chance(0.01) ? OSE_URL_TGT_STR_EMPTY : OSE_URL_TGT_STR;
          } else if (kind == OSE_KIND_CLIENT && q_r.chance(0.05)) {
            f |= OSE_URL_TGT_STR;
          }
          uint32_t src = q_r.below(100);
          tmp.clear();
          if (mx.hicard && q_r.chance(0.5)) {
            // C5 high-cardinality paths: 64-bit user ids (\\d{7,} -> {id})
            tmp += "/users/"; tmp += std::to_string(q_r.next()); tmp += '/'; gen_word(q_r, tmp);
            if (q_r.chance(0.5)) { tmp += "/"; tmp += std::to_string(q_r.next() >> q_r.below(40)); }
          } else {
            gen_path(q_r, tmp);
          }
          if (src < 75) {
            f |= OSE_URL_PATH_RAW;
            pref = add(c.arena, tmp);
          } else if (src < 97) {
            f |= OSE_URL_PATH_TARGET;
            if (q_r.chance(0.5)) { tmp += "?id="; gen_digits(q_r, tmp, 6); tmp += "&q=a/b"; }
            pref = add(c.arena, tmp);
          }   // else: no path source
        } else {
          nl = 8 + q_r.below(32);
        }
        if (has_route) {
          // 200 routes: /api/v{1,2}/<word>[/{id}]...; C5: 1M distinct routes
          uint32_t rid = q_r.below(mx.hicard ? 1000000 : 200);
          tmp.clear();
          tmp += "/api/v"; tmp += (char)('1' + rid % 2); tmp += '/'; tmp += kWords[rid % kNWords];
          if (rid % 3 == 0) tmp += "/{id}";
          if (rid % 5 == 0) { tmp += '/'; tmp += kWords[(rid / 7) % kNWords]; }
          if (mx.hicard) { tmp += "/r"; tmp += std::to_string(rid); }
          // http.route "" (TGT_STR_EMPTY) is an empty route string for sampling
          if ((f & OSE_URL_TGT_MASK) != OSE_URL_TGT_STR_EMPTY) rref = add(c.arena, tmp);
        }
        c.url_flags.push_back(f);
        c.path.push_back(pref);
        c.route.push_back(rref);
        c.name_len.push_back(nl);
        c.span_size.push_back(120 + pref.len + rref.len + nl + q_r.below(200));
      }
    }
    made += tsz;
  }
}

struct Gen {
  ose_columns cols{};
  std::vector<uint8_t> arena;
  std::vector<uint64_t> trace_id, start, end;
  std::vector<uint8_t> status, kind, url_flags, res_url_ok;
  std::vector<uint32_t> resource, scope, span_size, name_len, res_svc, res_svc_str, res_attrset, res_size, scope_size,
      scope_resource;
  std::vector<ose_strref> path, route;
  uint64_t arena_used = 0;
};

template <typename T>
void append(std::vector<T>& dst, const std::vector<T>& src) { dst.insert(dst.end(), src.begin(), src.end()); }


Mix mix_of(const char* workload) {
  Mix mx;
  std::string w = workload ? workload : "url";
  if (w == "sampling") { mx.url = false; mx.sampling = true; mx.p_route = 0.5; }
  else if (w == "fused") { mx.sampling = true; mx.p_route = 0.5; }
  else if (w == "zipf") { mx.sampling = true; mx.zipf = true; mx.hicard = true; mx.p_route = 0.5; }
  return mx;
}

// Concatenates the chunks in order (threads copy whole chunks: each chunk's
// arena is already in span order, path then route per span).
void assemble_ordered(Gen* g, std::vector<Chunk>& chunks, int threads) {
  const size_t K = chunks.size();
  std::vector<uint64_t> s0(K + 1, 0), r0(K + 1, 0), a0(K + 1, 0);
  for (size_t k = 0; k < K; k++) {
    s0[k + 1] = s0[k] + chunks[k].kind.size();
    r0[k + 1] = r0[k] + chunks[k].res_svc.size();
    a0[k + 1] = a0[k] + chunks[k].arena.size();
  }
  const uint64_t n = s0[K], R = r0[K];
  g->arena.assign(((a0[K] + 15) / 16) * 16 + 64, 0);
  g->trace_id.resize(2 * n);
  for (auto* v : {&g->start, &g->end}) v->resize(n);
  for (auto* v : {&g->status, &g->kind, &g->url_flags}) v->resize(n);
  for (auto* v : {&g->resource, &g->scope, &g->span_size, &g->name_len}) v->resize(n);
  g->path.resize(n);
  g->route.resize(n);
  for (auto* v : {&g->res_svc, &g->res_svc_str, &g->res_attrset, &g->res_size, &g->scope_size, &g->scope_resource})
    v->resize(R);
  g->res_url_ok.resize(R);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      for (size_t k = (size_t)t; k < K; k += (size_t)threads) {
        Chunk& c = chunks[k];
        const uint64_t sb = s0[k], rb = r0[k], ab = a0[k];
        std::memcpy(g->arena.data() + ab, c.arena.data(), c.arena.size());
        const size_t m = c.kind.size(), rr = c.res_svc.size();
        std::memcpy(&g->trace_id[2 * sb], c.trace_id.data(), 16 * m);
        std::memcpy(&g->start[sb], c.start.data(), 8 * m);
        std::memcpy(&g->end[sb], c.end.data(), 8 * m);
        std::memcpy(&g->status[sb], c.status.data(), m);
        std::memcpy(&g->kind[sb], c.kind.data(), m);
        std::memcpy(&g->url_flags[sb], c.url_flags.data(), m);
        std::memcpy(&g->span_size[sb], c.span_size.data(), 4 * m);
        std::memcpy(&g->name_len[sb], c.name_len.data(), 4 * m);
        for (size_t i = 0; i < m; i++) {
          const uint32_t res = (uint32_t)(rb + c.res_local[i]);
          g->resource[sb + i] = res;
          g->scope[sb + i] = res;   // one ScopeSpans per ResourceSpans
          ose_strref p = c.path[i], q = c.route[i];
          g->path[sb + i] = p.len ? ose_strref{(uint32_t)(ab + p.off), p.len} : ose_strref{0, 0};
          g->route[sb + i] = q.len ? ose_strref{(uint32_t)(ab + q.off), q.len} : ose_strref{0, 0};
        }
        for (size_t r = 0; r < rr; r++) {
          g->res_svc[rb + r] = c.res_svc[r];
          g->res_svc_str[rb + r] = c.res_svc_str[r];
          g->res_url_ok[rb + r] = c.res_url_ok[r];
          g->res_attrset[rb + r] = c.res_attrset[r];
          g->res_size[rb + r] = c.res_size[r];
          g->scope_size[rb + r] = c.scope_size[r];
          g->scope_resource[rb + r] = (uint32_t)(rb + r);
        }
        Chunk().arena.swap(c.arena);   // free as we go
      }
    });
  for (auto& x : th) x.join();
  g->arena_used = a0[K];
}

void* create(const char* workload, uint64_t seed, uint64_t n_spans, int threads, int shuffle, uint32_t rank,
             uint32_t world) {
  Mix mx = mix_of(workload);
  if (threads < 1) threads = 1;
  const uint64_t kChunk = 1 << 16;
  uint64_t nchunks = (n_spans + kChunk - 1) / kChunk;
  std::vector<Chunk> chunks(nchunks);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      for (uint64_t k = (uint64_t)t; k < nchunks; k += (uint64_t)threads) {
        uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (k + 1));
        gen_chunk(s, std::min(kChunk, n_spans - k * kChunk), mx, chunks[k], rank, world);
      }
    });
  for (auto& x : th) x.join();
  auto* g = new Gen();
  if (!shuffle) {
    assemble_ordered(g, chunks, threads);
    return g;
  }
  // resource permutation (shuffle) keeps each resource's spans contiguous
  std::vector<std::pair<uint64_t, uint32_t>> order;   // (chunk, local resource)
  for (uint64_t k = 0; k < nchunks; k++)
    for (uint32_t r = 0; r < chunks[k].res_svc.size(); r++) order.emplace_back(k, r);
  {
    Rng rr(seed ^ 0x5A5A5A5A5A5A5A5Aull);
    for (size_t i = order.size(); i > 1; i--) std::swap(order[i - 1], order[rr.below((uint32_t)i)]);
  }
  uint64_t total_arena = 0;
  for (auto& c : chunks) total_arena += c.arena.size();
  g->arena.reserve(((total_arena + 15) / 16) * 16 + 64);
  g->trace_id.reserve(2 * n_spans);
  for (auto* v : {&g->start, &g->end}) v->reserve(n_spans);
  for (auto& o : order) {
    Chunk& c = chunks[o.first];
    uint32_t r = o.second;
    uint32_t s0 = c.res_first_span[r];
    uint32_t s1 = r + 1 < c.res_first_span.size() ? c.res_first_span[r + 1] : (uint32_t)c.kind.size();
    uint32_t res = (uint32_t)g->res_svc.size();
    g->res_svc.push_back(c.res_svc[r]);
    g->res_svc_str.push_back(c.res_svc_str[r]);
    g->res_url_ok.push_back(c.res_url_ok[r]);
    g->res_attrset.push_back(c.res_attrset[r]);
    g->res_size.push_back(c.res_size[r]);
    g->scope_size.push_back(c.scope_size[r]);
    g->scope_resource.push_back(res);   // one ScopeSpans per ResourceSpans
    for (uint32_t i = s0; i < s1; i++) {
      g->trace_id.push_back(c.trace_id[2 * i]);
      g->trace_id.push_back(c.trace_id[2 * i + 1]);
      g->start.push_back(c.start[i]);
      g->end.push_back(c.end[i]);
      g->status.push_back(c.status[i]);
      g->kind.push_back(c.kind[i]);
      g->url_flags.push_back(c.url_flags[i]);
      g->resource.push_back(res);
      g->scope.push_back(res);   // one ScopeSpans per ResourceSpans
      g->span_size.push_back(c.span_size[i]);
      g->name_len.push_back(c.name_len[i]);
      ose_strref p = c.path[i], q = c.route[i];
      // re-pack strings so the arena is in span order (path, then route)
      ose_strref np{(uint32_t)g->arena.size(), p.len};
      g->arena.insert(g->arena.end(), c.arena.begin() + p.off, c.arena.begin() + p.off + p.len);
      ose_strref nq{(uint32_t)g->arena.size(), q.len};
      g->arena.insert(g->arena.end(), c.arena.begin() + q.off, c.arena.begin() + q.off + q.len);
      if (p.len == 0) np.off = 0;
      if (q.len == 0) nq.off = 0;
      g->path.push_back(np);
      g->route.push_back(nq);
    }
  }
  g->arena_used = g->arena.size();
  return g;
}

void* finish(Gen* g) {
  const uint64_t abytes = g->arena_used;
  g->arena.resize(((abytes + 15) / 16) * 16 + 64, 0);
  ose_columns& c = g->cols;
  c.n_spans = g->kind.size();
  c.n_resources = (uint32_t)g->res_svc.size();
  c.n_scopes = c.n_resources;
  c.n_attrsets = 256;
  c.arena_bytes = abytes;
  c.arena = g->arena.data();
  c.trace_id = g->trace_id.data();
  c.start_ns = g->start.data();
  c.end_ns = g->end.data();
  c.status = g->status.data();
  c.kind = g->kind.data();
  c.resource = g->resource.data();
  c.scope = g->scope.data();
  c.url_flags = g->url_flags.data();
  c.path = g->path.data();
  c.route = g->route.data();
  c.span_size = g->span_size.data();
  c.name_len = g->name_len.data();
  c.res_svc = g->res_svc.data();
  c.res_svc_str = g->res_svc_str.data();
  c.res_url_ok = g->res_url_ok.data();
  c.res_attrset = g->res_attrset.data();
  c.res_size = g->res_size.data();
  c.scope_size = g->scope_size.data();
  c.scope_resource = g->scope_resource.data();
  return g;
}

}  // namespace

extern "C" {

// workload: "url" | "sampling" | "fused" | "zipf"
void* osegen_create(const char* workload, uint64_t seed, uint64_t n_spans, int threads, int shuffle) {
  return finish(static_cast<Gen*>(create(workload, seed, n_spans, threads, shuffle, 0, 0)));
}

// The batch source `rank` of `world` holds when a global batch of n_spans
// spans (same seed) reaches the gateway through `world` node collectors
// (split mode above); world = 1 is the whole global batch.
void* osegen_create_split(const char* workload, uint64_t seed, uint64_t n_spans, int threads, uint32_t rank,
                          uint32_t world) {
  if (world < 1 || rank >= world) return nullptr;
  return finish(static_cast<Gen*>(create(workload, seed, n_spans, threads, 0, rank, world)));
}

const ose_columns* osegen_columns(void* g) { return &static_cast<Gen*>(g)->cols; }
uint64_t osegen_arena_alloc(void* g) { return static_cast<Gen*>(g)->arena.size(); }
void osegen_free(void* g) { delete static_cast<Gen*>(g); }

}  // extern "C"
