// otlp_host.cpp — OTLP protobuf ingest: ose_otlp_*.
//
// One call turns a serialized TracesData into device columns:
//   1. the bytes go to pinned staging and H2D (the arena: strings are
//      referenced in place) while the host walks the structure (otlp_pb.cpp
//      pb_walk: ResourceSpans / ScopeSpans headers, resource and scope
//      contents, one header per span);
//   2. per-resource and per-scope columns on the host (columnize.cpp: the
//      service ids, include/exclude, attribute sets, the fixed sizes);
//   3. otlp_span_kernel decodes every span on the GPU;
//   4. the spans it lists get the host pass: pb_span + columnize_span, their
//      strings appended after the message bytes, written by otlp_fix_kernel.
#include <algorithm>
#include <chrono>
#include <deque>
#include <shared_mutex>
#include <cstring>
#include <map>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "columnize.hpp"
#include "engine_internal.hpp"
#include "kernels.hpp"
#include "otlp_encode.hpp"
#include "otlp_pb.hpp"
#include "taskpool.hpp"

namespace ose {

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {
size_t up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

struct DevBuf {   // grow-only device (or pinned host) buffer
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool host = false;
  int need(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) { if (host) (void)hipHostFree(p); else (void)hipFree(p); }
    p = nullptr;
    cap = 0;
    const size_t want = up(std::max<size_t>(bytes + bytes / 4, 1 << 20), 1 << 16);
    if (host) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&p), want, hipHostMallocDefault));
    else HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p), want));
    cap = want;
    return 0;
  }
  ~DevBuf() {
    if (p) { if (host) (void)hipHostFree(p); else (void)hipFree(p); }
  }
};
}  // namespace

namespace {
struct CachedRes {
  uint32_t svc, svc_str, set, rpart;   // set: id in ResCache::sets
  uint8_t ok;
  uint64_t attr_res;
};

// Resource columns by message bytes, kept across calls (a gateway sees the
// same pods' resources batch after batch), and the attribute sets interned.
struct ResCache {
  static constexpr size_t kMaxEntries = size_t(1) << 16;
  std::shared_mutex mu;
  std::deque<std::string> keys;   // owned bytes the map's views point into
  std::unordered_map<std::string_view, CachedRes> map;
  std::deque<std::vector<std::pair<std::string, std::string>>> sets;   // stable addresses
  std::map<std::vector<std::pair<std::string, std::string>>, uint32_t> set_ids;
  uint32_t intern(const std::vector<std::pair<std::string, std::string>>& set) {   // under the unique lock
    auto it = set_ids.find(set);
    if (it != set_ids.end()) return it->second;
    const uint32_t id = (uint32_t)sets.size();
    sets.push_back(set);
    set_ids.emplace(set, id);
    return id;
  }
};
}  // namespace

// The engine's view for the ingest: the columniser context and the key
// table the GPU decoder matches (built once per engine).
// The device copy of the resource cache (ResCache) the GPU ResourceSpans
// pass looks resources up in (otlp_res_fields_kernel): open addressing on
// the Resource bytes' FNV-1a hash, up to 64 probes, never deleted.  A host
// mirror takes the inserts; sync() copies what changed.  Lookups in flight
// hold the lock shared, updates unique.
struct DevResTable {
  std::shared_mutex mu;
  ResSlotDev* d_slots = nullptr;
  uint8_t* d_keys = nullptr;
  std::vector<ResSlotDev> slots;
  std::vector<uint8_t> keys;
  std::vector<uint32_t> changed;   // slots filled since the last sync
  size_t keys_synced = 0;
  uint32_t n = 0;
  int ensure() {   // under the unique lock
    if (d_slots) return 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_slots), sizeof(ResSlotDev) * kResSlots));
    HIP_TRY(hipMemset(d_slots, 0, sizeof(ResSlotDev) * kResSlots));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_keys), kResKeyBytes));
    slots.assign(kResSlots, ResSlotDev{});
    return 0;
  }
  void insert(const uint8_t* key, uint32_t len, const CachedRes& cr) {   // under the unique lock
    if (!d_slots || n >= kResSlots / 2 || keys.size() + len > kResKeyBytes) return;
    uint64_t h = kResHashSeed;
    for (uint32_t q = 0; q < len; q++) h = res_key_hash_step(h, key[q]);
    uint32_t slot = (uint32_t)h & (kResSlots - 1);
    for (int probe = 0; probe < 64; probe++, slot = (slot + 1) & (kResSlots - 1)) {
      ResSlotDev& e = slots[slot];
      if (!e.ready) {
        e.h = h;
        e.koff = (uint32_t)keys.size();
        e.klen = len;
        keys.insert(keys.end(), key, key + len);
        e.svc = cr.svc;
        e.svc_str = cr.svc_str;
        e.set = cr.set;
        e.rpart = cr.rpart;
        e.attr_res = cr.attr_res;
        e.ok = cr.ok;
        e.ready = 1;
        changed.push_back(slot);
        n++;
        return;
      }
      if (e.h == h && e.klen == len && std::memcmp(keys.data() + e.koff, key, len) == 0) return;
    }
  }
  int sync(hipStream_t st) {   // under the unique lock
    if (changed.empty()) return 0;
    if (keys.size() > keys_synced)
      HIP_TRY(hipMemcpyAsync(d_keys + keys_synced, keys.data() + keys_synced, keys.size() - keys_synced,
                             hipMemcpyHostToDevice, st));
    if (changed.size() > 256) {
      HIP_TRY(hipMemcpyAsync(d_slots, slots.data(), sizeof(ResSlotDev) * kResSlots, hipMemcpyHostToDevice, st));
    } else {
      for (uint32_t k : changed)
        HIP_TRY(hipMemcpyAsync(d_slots + k, &slots[k], sizeof(ResSlotDev), hipMemcpyHostToDevice, st));
    }
    HIP_TRY(hipStreamSynchronize(st));   // the sources are the mirror, which the next insert changes
    keys_synced = keys.size();
    changed.clear();
    return 0;
  }
  ~DevResTable() {
    if (d_slots) (void)hipFree(d_slots);
    if (d_keys) (void)hipFree(d_keys);
  }
};

struct OtlpEngine {
  ColumnizeCtx ctx;
  std::vector<OtlpKeyDev> keys;
  std::string key_bytes;
  uint64_t key_lens = 0;
  uint8_t* keys_dev = nullptr;   // OtlpKeyDev[] then the bytes
  uint32_t n_attr_keys = 0;
  uint32_t attr_words = 1;   // attr_match words per span
  bool json_rules = false;
  // more than 64 shim-evaluated (json / oversize-regex) span_attribute rules:
  // the per-resource cached word cannot hold their bits, so the host pass
  // takes each span's from its resource's service id (AsString(service.name):
  // the rules whose service it is, spanattribute.go:130-132), [svc][word]
  bool wide_host_rules = false;
  std::vector<std::vector<uint64_t>> host_rules_by_svc;
  ResCache res_cache;
  DevResTable res_dev;
  std::string err;
  ~OtlpEngine() { if (keys_dev) (void)hipFree(keys_dev); }
};

struct OtlpBatchImpl {
  Engine* e = nullptr;
  ose_columns cols{};
  DevBuf arena, slab, stage, fixdev;   // device arena; device columns; pinned staging; host-pass records
  std::vector<std::vector<std::pair<std::string, std::string>>> attrsets;
  uint32_t host_spans = 0;
  double t_ms[5] = {0, 0, 0, 0, 0};   // copy-in, walk, columns upload, span kernel (+ sync), host pass
  // for ose_otlp_encode: the caller's message and where its parts are
  const uint8_t* pb = nullptr;
  size_t pb_len = 0;
  std::vector<uint64_t> span_ref;
  OtlpLayout lay;
  // with the scopes walked on the GPU, span_ref and the scopes' span0 / hdr
  // / schema are on the device until ose_otlp_encode (or the host pass)
  // brings them back
  bool layout_on_host = true;
  DevBuf sslab;   // scope-level device arrays
  DevBuf rslab, setbuf, cslab;   // resource-level device arrays; attribute-set compaction; the GPU chain walk
  uint64_t* d_res_ref = nullptr;   // the ResourceSpans refs (lay.res_ref is filled from it on demand)
  bool res_on_device = false;   // res_scope0 / scope_ref / attr_res live on the device (rslab, sslab)
  uint32_t* d_res_scope0 = nullptr;
  uint64_t* d_scope_ref = nullptr;
  uint64_t* d_attr_res = nullptr;
  uint64_t* d_span_ref = nullptr;
  uint32_t *d_span_res = nullptr, *d_span0 = nullptr;
  uint64_t *d_hdr = nullptr, *d_schema = nullptr;
  OtlpScopeArgs sargs{};   // the GPU scope walk's arrays (pass 2 reuses them)
  // the GPU encoder (encode_kernel.hip): the span refs in HBM (always), the
  // scope level there when the GPU walked it; its workspace and outputs
  uint64_t* d_spans = nullptr;
  bool scopes_dev = false;
  DevBuf eslab, eout, emisc;
  DevBuf seth;   // pinned: the resource pass's attribute-set scan words and ids (read after the scope pass's wait)
  OtlpBatchImpl() { stage.host = true; emisc.host = true; seth.host = true; }
};


namespace {
std::mutex g_otlp_mu;

OtlpEngine* otlp_engine(Engine* e, int& rc) {
  std::lock_guard<std::mutex> g(g_otlp_mu);
  rc = 0;
  if (e->otlp) return e->otlp;
  auto* o = new OtlpEngine();
  o->err = o->ctx.build(e->has_url ? &e->url : nullptr, e->has_sampling ? &e->sampling : nullptr,
                        e->has_traffic ? &e->traffic : nullptr);
  if (!o->err.empty()) { rc = fail(OSE_EINVAL, o->err); delete o; return nullptr; }
  std::map<std::string, uint64_t> roles;
  roles["http.request.method"] |= kRoleMethodNew;
  roles["http.method"] |= kRoleMethodOld;
  roles["http.route"] |= kRoleRoute;
  roles["url.template"] |= kRoleUrlTmpl;
  roles["url.path"] |= kRoleUrlPath;
  roles["http.target"] |= kRoleTarget;
  roles["url.full"] |= kRoleFull;
  roles["http.url"] |= kRoleFull;
  const AttrPlan& plan = o->ctx.attr_plan;
  // the per-resource rule word the decoder caches holds the shim-evaluated
  // rules only, one bit each; past 64 of them the host pass takes the bits
  // from the resource's service id instead (wide_host_rules)
  size_t n_host_rules = 0;
  for (int rk : plan.rule_key) n_host_rules += rk < 0;
  if (n_host_rules > 64) {
    o->wide_host_rules = true;
    o->host_rules_by_svc.assign(std::max<size_t>(o->ctx.services.size(), 1),
                                std::vector<uint64_t>(std::max<size_t>(plan.host_mask.size(), 1), 0));
    for (size_t k = 0; k < plan.rule_key.size() && k < o->ctx.attr_preds.size(); k++) {
      if (plan.rule_key[k] >= 0) continue;
      auto it = o->ctx.services.find(o->ctx.attr_preds[k].service());
      if (it != o->ctx.services.end() && it->second < o->host_rules_by_svc.size())
        o->host_rules_by_svc[it->second][k / 64] |= 1ull << (k % 64);
    }
  }
  o->attr_words = (uint32_t)std::max<size_t>(1, (plan.rule_key.size() + 63) / 64);
  o->n_attr_keys = (uint32_t)plan.keys.size();
  // key columns past kOtlpMaxAttrKeys have no role bit: a span that carries
  // such a key takes the host pass (which fills every key column), and the
  // GPU decoder writes the others ABSENT for every span it finishes
  for (size_t k = 0; k < plan.keys.size(); k++)
    roles[plan.keys[k]] |= k < kOtlpMaxAttrKeys ? kRoleAttr0 << k : (uint64_t)kRoleHost;
  for (size_t k = 0; k < plan.rule_key.size(); k++)
    if (plan.rule_key[k] < 0) {
      roles[o->ctx.attr_preds[k].key()] |= kRoleHost;
      o->json_rules = true;
    }
  for (auto& kv : roles) {
    OtlpKeyDev d{(uint32_t)kv.first.size(), (uint32_t)o->key_bytes.size(), kv.second};
    o->key_bytes += kv.first;
    o->keys.push_back(d);
    if (kv.first.size() < 64) o->key_lens |= 1ull << kv.first.size();
  }
  const size_t kb = o->keys.size() * sizeof(OtlpKeyDev);
  std::vector<uint8_t> blob(kb + o->key_bytes.size() + 16, 0);
  std::memcpy(blob.data(), o->keys.data(), kb);
  std::memcpy(blob.data() + kb, o->key_bytes.data(), o->key_bytes.size());
  if (hipMalloc(reinterpret_cast<void**>(&o->keys_dev), blob.size()) != hipSuccess ||
      hipMemcpy(o->keys_dev, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess) {
    rc = fail(OSE_EDEVICE, "OTLP ingest: key table upload failed");
    delete o;
    return nullptr;
  }
  e->otlp = o;
  return o;
}
}  // namespace

void release_otlp(Engine* e) {
  for (void* p : e->otlp_pool) delete static_cast<OtlpBatchImpl*>(p);
  e->otlp_pool.clear();
  delete e->otlp;
  e->otlp = nullptr;
}

namespace {
// memcpy over threads for large copies into pinned staging
void par_memcpy(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t kChunk = size_t(64) << 20;
  if (n < 2 * kChunk) { std::memcpy(dst, src, n); return; }
  const int T = (int)std::min<size_t>(16, n / kChunk);
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++)
    th.emplace_back([=]() { const size_t a = n * t / T, b = n * (t + 1) / T; std::memcpy(dst + a, src + a, b - a); });
  std::memcpy(dst, src, n / T);
  for (auto& x : th) x.join();
}

// The structural walk, resources split over threads.  Resource and scope
// messages repeat across a batch (one SDK, one pod), so their columns are
// cached by message bytes.
struct Walked {
  std::vector<uint64_t> span_ref;   // with gpu_scopes: the host-walked scopes' spans only
  std::vector<uint8_t> scope_on_host;
  std::vector<uint32_t> scope_count;
  std::vector<uint32_t> span_res, span_scope;
  std::vector<uint32_t> res_svc, res_svc_str, res_attrset, res_size, scope_size, scope_res;
  std::vector<uint8_t> res_ok;
  std::vector<uint64_t> attr_res;
  std::vector<std::vector<std::pair<std::string, std::string>>> sets;
  OtlpLayout lay;   // what the re-encoder needs (otlp_encode.cpp)
  std::string err;
};
struct WalkChunk {
  std::vector<uint64_t> span_ref;
  std::vector<uint32_t> span_res, span_scope;   // chunk-local indices
  std::vector<uint32_t> res_svc, res_svc_str, res_set, res_size, scope_size, scope_res;
  std::vector<uint8_t> res_ok;
  std::vector<uint64_t> attr_res;
  OtlpLayout lay;   // res_scope0 / scope_span0 chunk-local
  // GPU-walked scopes (walk with gpu_scopes): span_ref lists only the spans
  // of the scopes the host walked
  std::vector<uint8_t> scope_on_host;
  std::vector<uint32_t> scope_count;
  std::string err;
};
// ScopeSpans payloads up to this size are walked on the GPU (a lane per
// scope follows its chain of span lengths); larger ones on the host
constexpr size_t kGpuScopeBytes = size_t(64) << 10;
uint64_t sov64(uint64_t x) { uint64_t n = 1; while (x >= 0x80) { x >>= 7; n++; } return n; }
uint64_t flen(uint64_t l) { return 1 + sov64(l) + l; }

// The json (host-pass) span_attribute rules of a resource as one word: bit j
// for the j-th host rule in rule order (words: the resource's bits of every
// rule, 64 per word; ColumnizeCtx::attr_plan.host_mask marks the host rules)
uint64_t host_rule_word(const AttrPlan& p, const std::vector<uint64_t>& words) {
  uint64_t out = 0;
  uint32_t j = 0;
  for (size_t w = 0; w < p.host_mask.size(); w++)
    for (uint64_t m = p.host_mask[w]; m; m &= m - 1, j++)
      if (j < 64 && w < words.size() && ((words[w] >> __builtin_ctzll(m)) & 1)) out |= 1ull << j;
  return out;
}
// ... and back to the rule-indexed words columnize_span takes
void host_rule_words(const AttrPlan& p, uint64_t word, std::vector<uint64_t>& out) {
  out.assign(std::max<size_t>(1, p.host_mask.size()), 0);
  uint32_t j = 0;
  for (size_t w = 0; w < p.host_mask.size(); w++)
    for (uint64_t m = p.host_mask[w]; m; m &= m - 1, j++)
      if (j < 64 && ((word >> j) & 1)) out[w] |= 1ull << __builtin_ctzll(m);
}

// A resource's columns from its Resource field(s) (merged as pdata merges
// them), entered into the cache by message bytes when there is at most one
// field.  False: a malformed Resource.
bool resolve_resource(const ColumnizeCtx& ctx, ResCache& cache, const uint8_t* p,
                      const std::vector<std::pair<size_t, size_t>>& resf, ProtoSizer& sizer, CachedRes& cr) {
  AttrMap attrs;
  uint32_t dropped = 0;
  for (auto& x : resf)
    if (!pb_resource(p + x.first, x.second, attrs, dropped)) return false;
  const ResourceCols rc = columnize_resource(ctx, attrs);
  cr.svc = rc.svc;
  cr.svc_str = rc.svc_str;
  cr.ok = rc.url_ok;
  cr.attr_res = host_rule_word(ctx.attr_plan, rc.attr_res);   // <= 64 json rules (otlp_engine)
  cr.rpart = (uint32_t)flen(sizer.attrs(attrs, 1) + (dropped ? 1 + sov64(dropped) : 0));   // Resource: always emitted
  const std::string_view key = resf.size() == 1 ? std::string_view((const char*)p + resf[0].first, resf[0].second)
                                                : std::string_view();
  std::unique_lock<std::shared_mutex> g(cache.mu);
  cr.set = cache.intern(rc.attrset);
  if (resf.size() <= 1 && cache.map.size() < ResCache::kMaxEntries && !cache.map.count(key)) {
    cache.keys.emplace_back(key);
    cache.map.emplace(std::string_view(cache.keys.back()), cr);
  }
  return true;
}

// The TracesData records that start in [s, lim) (a record may run past lim:
// *end is where the last one ends), each ResourceSpans walked in full.
void walk_segment(const ColumnizeCtx& ctx, ResCache& cache, const uint8_t* p, size_t n, size_t s, size_t lim,
                  WalkChunk& c, size_t* end, bool gpu_scopes, bool chain = false) {
  std::unordered_map<std::string_view, CachedRes> rcache;   // this call's, by view into the message
  std::unordered_map<std::string_view, uint32_t> scache;
  ProtoSizer sizer;
  std::vector<std::pair<size_t, size_t>> resf, scopes, deprecated, scf;
  const size_t est = gpu_scopes ? 16 : (std::min(lim, n) - std::min(s, n)) / 128 + 16;   // spans of >= 128 bytes
  c.span_ref.reserve(est);
  c.span_res.reserve(est);
  c.span_scope.reserve(est);
  PbReader top(p, n);
  top.i = s;
  *end = s;
  // The walk is a chain of lengths: each header's address depends on the
  // last length, so without help every span costs a DRAM round trip.  The
  // segment is prefetched line by line a few KB ahead of the walk instead.
  size_t pf = s & ~size_t(63);
  auto ahead = [&](size_t pos) {
    if (gpu_scopes) return;   // the host reads headers only: no streaming of span bytes
    const size_t want = std::min(n, pos + 8192);
    for (; pf < want; pf += 64) __builtin_prefetch(p + pf, 0, 3);
  };
  uint32_t tf, twt;
  while (top.i < lim && top.more() && top.tag(tf, twt)) {
    ahead(top.i);
    size_t ro, rl;
    if (tf != 1) {
      if (!top.skip(twt, tf)) break;
      *end = top.i;
      continue;
    }
    if (twt != 2 || !top.bytes(ro, rl)) { top.fail(); break; }
    *end = top.i;
    if (gpu_scopes && top.i + 2 < n) __builtin_prefetch(p + top.i, 0, 3);   // the next record's header
    if (chain) {   // the TracesData chain only: the GPU walks each record (otlp_res_fields_kernel)
      if (ro > 0xFFFFFFFFull || rl > 0xFFFFFFFFull) { c.err = "ResourceSpans beyond the 4 GiB arena range"; return; }
      c.lay.res_ref.push_back(ro | ((uint64_t)rl << 32));
      continue;
    }
    PbReader rr(p + ro, rl);
    resf.clear();
    scopes.clear();
    deprecated.clear();
    size_t schema = 0;
    uint32_t f, wt;
    while (rr.more() && rr.tag(f, wt)) {
      size_t o, l;
      if (f == 1 || f == 2 || f == 1000 || f == 3) {
        if (wt != 2 || !rr.bytes(o, l)) { rr.fail(); break; }
        if (f == 1) resf.emplace_back(ro + o, l);
        else if (f == 3) schema = l;
        else (f == 2 ? scopes : deprecated).emplace_back(ro + o, l);
      } else {
        rr.skip(wt, f);
      }
    }
    if (!rr.ok) { c.err = "OTLP protobuf: malformed ResourceSpans"; return; }
    if (scopes.empty()) scopes.swap(deprecated);
    // the resource's columns (cached by its message bytes)
    CachedRes cr{};
    const std::string_view key = resf.size() == 1 ? std::string_view((const char*)p + resf[0].first, resf[0].second)
                                                  : std::string_view();
    auto it = resf.size() <= 1 ? rcache.find(key) : rcache.end();
    bool have = false;
    if (it != rcache.end()) {
      cr = it->second;
      have = true;
    } else if (resf.size() <= 1) {
      std::shared_lock<std::shared_mutex> g(cache.mu);
      auto ci = cache.map.find(key);
      if (ci != cache.map.end()) {
        cr = ci->second;
        have = true;
        rcache.emplace(key, cr);
      }
    }
    if (!have) {
      if (!resolve_resource(ctx, cache, p, resf, sizer, cr)) { c.err = "OTLP protobuf: malformed Resource"; return; }
      if (resf.size() <= 1) rcache.emplace(key, cr);
    }
    const uint32_t rloc = (uint32_t)c.res_svc.size();
    c.lay.res_ref.push_back(ro | ((uint64_t)rl << 32));
    c.lay.res_scope0.push_back((uint32_t)c.scope_size.size());
    c.res_svc.push_back(cr.svc);
    c.res_svc_str.push_back(cr.svc_str);
    c.res_ok.push_back(cr.ok);
    c.attr_res.push_back(cr.attr_res);
    c.res_set.push_back(cr.set);
    c.res_size.push_back(cr.rpart + (uint32_t)(schema ? flen(schema) : 0));
    for (auto& so : scopes) {
      const uint32_t sloc = (uint32_t)c.scope_size.size();
      PbReader sr(p + so.first, so.second);
      size_t sschema = 0, sschema_off = 0;
      scf.clear();
      c.lay.scope_ref.push_back(so.first | ((uint64_t)so.second << 32));
      c.lay.scope_span0.push_back((uint32_t)c.span_ref.size());
      if (gpu_scopes && so.second <= kGpuScopeBytes) {   // counted, sized and listed on the GPU
        c.scope_on_host.push_back(0);
        c.scope_count.push_back(0);
        c.scope_size.push_back(0);
        c.scope_res.push_back(rloc);
        c.lay.scope_hdr.push_back(0);
        c.lay.scope_schema.push_back(0);
        continue;
      }
      const size_t first_span = c.span_ref.size();
      while (sr.more() && sr.tag(f, wt)) {
        size_t o, l;
        if (f == 1 || f == 2 || f == 3) {
          if (wt != 2 || !sr.bytes(o, l)) { sr.fail(); break; }
          if (f == 1) {
            scf.emplace_back(so.first + o, l);
          } else if (f == 3) {
            sschema = l;
            sschema_off = so.first + o;
          } else {
            const uint64_t off = so.first + o;
            ahead(off + l);
            if (off > 0xFFFFFFFFull || l > 0xFFFFFFFFull) { c.err = "span beyond the 4 GiB arena range"; return; }
            c.span_ref.push_back(off | ((uint64_t)l << 32));
            if (!gpu_scopes) {
              c.span_res.push_back(rloc);
              c.span_scope.push_back(sloc);
            }
          }
        } else {
          sr.skip(wt, f);
        }
      }
      if (!sr.ok) { c.err = "OTLP protobuf: malformed ScopeSpans"; return; }
      uint32_t spart;
      const std::string_view sk = scf.size() == 1 ? std::string_view((const char*)p + scf[0].first, scf[0].second)
                                                  : std::string_view();
      auto si = scf.size() <= 1 ? scache.find(sk) : scache.end();
      if (si != scache.end()) {
        spart = si->second;
      } else {
        ScopeSpans meta;
        for (auto& x : scf)
          if (!pb_scope(p + x.first, x.second, meta)) { c.err = "OTLP protobuf: malformed InstrumentationScope"; return; }
        spart = (uint32_t)sizer.scope_fixed(meta);   // schema_url empty here
        if (scf.size() <= 1) scache.emplace(sk, spart);
      }
      c.scope_size.push_back(spart + (uint32_t)(sschema ? flen(sschema) : 0));
      c.scope_res.push_back(rloc);
      c.lay.scope_hdr.push_back(scf.empty() ? 0
                                : scf.size() == 1 ? (scf[0].first | ((uint64_t)scf[0].second << 32))
                                                  : OtlpLayout::kMulti);
      c.lay.scope_schema.push_back(sschema_off | ((uint64_t)sschema << 32));
      c.scope_on_host.push_back(1);
      c.scope_count.push_back((uint32_t)(c.span_ref.size() - first_span));
    }
  }
  if (!top.ok) c.err = "OTLP protobuf: malformed TracesData";
}

// A plausible record start at or after k: a TracesData field 1 (0x0A) whose
// length varint frames a record followed by 3 more such records (or the end).
size_t find_start(const uint8_t* p, size_t n, size_t k) {
  for (size_t q = k; q + 2 < n; q++) {
    if (p[q] != 0x0A) continue;
    size_t pos = q;
    int hops = 0;
    bool ok = true;
    while (hops < 4 && pos < n) {
      PbReader r(p, n);
      r.i = pos;
      uint32_t f, wt;
      size_t o, l;
      if (!r.tag(f, wt) || f != 1 || wt != 2 || !r.bytes(o, l) || l == 0 || (p[o] != 0x0A && p[o] != 0x12)) {
        ok = false;
        break;
      }
      pos = r.i;
      hops++;
    }
    if (ok) return q;
  }
  return n;
}

// The TracesData chain alone (the ResourceSpans records), split over threads
// as walk() does.
bool walk_chain(const uint8_t* p, size_t n, std::vector<uint64_t>& res_ref, std::string& err) {
  const size_t kSeg = size_t(256) << 10;
  int T = (int)std::max<size_t>(1, std::min<size_t>({(size_t)parallel_width(), n / kSeg}));
#if OSE_DIAG
  if (const char* e = getenv("OSE_WALK_THREADS")) T = std::max(1, atoi(e));
#endif
  static const ColumnizeCtx no_ctx;
  static ResCache no_cache;
  std::vector<WalkChunk> ch;
  for (int attempt = 0; attempt < 2; attempt++) {
    if (attempt) T = 1;
    std::vector<size_t> st((size_t)T + 1, n), en((size_t)T, 0);
    st[0] = 0;
    for (int t = 1; t < T; t++) st[t] = find_start(p, n, n * (size_t)t / (size_t)T);
    for (int t = T - 1; t >= 1; t--) st[t] = std::min(st[t], st[t + 1]);
    ch.assign((size_t)T, WalkChunk());
    parallel_run(T, [&](int t) { walk_segment(no_ctx, no_cache, p, n, st[t], st[t + 1], ch[t], &en[t], true, true); });
    bool exact = true;
    for (int t = 0; t < T; t++) {
      if (!ch[t].err.empty()) {
        if (t == 0 || attempt) { err = ch[t].err; return false; }
        exact = false;
      }
      if (t + 1 < T && en[t] != st[t + 1]) exact = false;
    }
    if (en[T - 1] != n && ch[T - 1].err.empty()) {
      if (attempt || T == 1) { err = "OTLP protobuf: malformed TracesData"; return false; }
      exact = false;
    }
    if (exact) break;
    if (attempt) { err = "OTLP protobuf: malformed TracesData"; return false; }
  }
  size_t total = 0;
  for (auto& c : ch) total += c.lay.res_ref.size();
  res_ref.resize(total);
  size_t o = 0;
  for (auto& c : ch) {
    std::memcpy(res_ref.data() + o, c.lay.res_ref.data(), 8 * c.lay.res_ref.size());
    o += c.lay.res_ref.size();
  }
  return true;
}

// The walk, split over threads: the records form one chain of lengths, so
// each thread starts at a speculated record start and walks up to the next
// thread's; the split is exact iff every thread ends exactly where the next
// one started (the chain from 0 is unique), else the walk runs again on one
// thread.
bool walk(const ColumnizeCtx& ctx, ResCache& cache, const uint8_t* p, size_t n, Walked& w, bool gpu_scopes = false) {
  const size_t kSeg = size_t(256) << 10;
  int T = (int)std::max<size_t>(1, std::min<size_t>({(size_t)parallel_width(), n / kSeg}));
#if OSE_DIAG
  if (const char* e = getenv("OSE_WALK_THREADS")) T = std::max(1, atoi(e));
#endif
  std::vector<WalkChunk> ch;
  for (int attempt = 0; attempt < 2; attempt++) {
    if (attempt) T = 1;
    std::vector<size_t> st((size_t)T + 1, n), en((size_t)T, 0);
    st[0] = 0;
    for (int t = 1; t < T; t++) st[t] = find_start(p, n, n * (size_t)t / (size_t)T);
    for (int t = T - 1; t >= 1; t--) st[t] = std::min(st[t], st[t + 1]);   // monotone
    ch.assign((size_t)T, WalkChunk());
    parallel_run(T, [&](int t) { walk_segment(ctx, cache, p, n, st[t], st[t + 1], ch[t], &en[t], gpu_scopes); });
    bool exact = true;
    for (int t = 0; t < T; t++) {
      if (!ch[t].err.empty()) {
        if (t == 0 || attempt) { w.err = ch[t].err; return false; }
        exact = false;   // a speculated start inside a record: redo
      }
      if (t + 1 < T && en[t] != st[t + 1]) exact = false;
    }
    if (en[T - 1] != n && ch[T - 1].err.empty()) {   // trailing bytes the segment walker did not reach
      if (attempt || T == 1) { w.err = "OTLP protobuf: malformed TracesData"; return false; }
      exact = false;
    }
    if (exact) break;
    if (attempt) { w.err = "OTLP protobuf: malformed TracesData"; return false; }
  }
  // merge: global indices, attribute sets in first-appearance order
  std::unordered_map<uint32_t, uint32_t> set_map;   // cache id -> this batch's
  {
    std::shared_lock<std::shared_mutex> g(cache.mu);
    for (auto& c : ch)
      for (uint32_t id : c.res_set)
        if (set_map.emplace(id, (uint32_t)w.sets.size()).second) w.sets.push_back(cache.sets[id]);
  }
  size_t nspan = 0, nres = 0, nscope = 0;
  for (size_t t = 0; t < ch.size(); t++) {
    nspan += ch[t].span_ref.size();
    nres += ch[t].res_svc.size();
    nscope += ch[t].scope_size.size();
  }
  w.span_ref.resize(nspan);
  if (!gpu_scopes) {
    w.span_res.resize(nspan);
    w.span_scope.resize(nspan);
  }
  w.scope_on_host.resize(nscope);
  w.scope_count.resize(nscope);
  w.res_svc.resize(nres);
  w.res_svc_str.resize(nres);
  w.res_attrset.resize(nres);
  w.res_size.resize(nres);
  w.res_ok.resize(nres);
  w.attr_res.resize(nres);
  w.scope_size.resize(nscope);
  w.scope_res.resize(nscope);
  w.lay.res_ref.resize(nres);
  w.lay.res_scope0.resize(nres);
  w.lay.scope_ref.resize(nscope);
  w.lay.scope_hdr.resize(nscope);
  w.lay.scope_schema.resize(nscope);
  w.lay.scope_span0.resize(nscope);
  std::vector<size_t> so(ch.size()), ro(ch.size()), co(ch.size());
  for (size_t t = 1; t < ch.size(); t++) {
    so[t] = so[t - 1] + ch[t - 1].span_ref.size();
    ro[t] = ro[t - 1] + ch[t - 1].res_svc.size();
    co[t] = co[t - 1] + ch[t - 1].scope_size.size();
  }
  auto place = [&](size_t t) {
    const WalkChunk& c = ch[t];
    for (size_t k = 0; k < c.span_ref.size(); k++) {
      w.span_ref[so[t] + k] = c.span_ref[k];
      if (!gpu_scopes) {
        w.span_res[so[t] + k] = (uint32_t)(ro[t] + c.span_res[k]);
        w.span_scope[so[t] + k] = (uint32_t)(co[t] + c.span_scope[k]);
      }
    }
    for (size_t k = 0; k < c.res_svc.size(); k++) {
      w.res_svc[ro[t] + k] = c.res_svc[k];
      w.res_svc_str[ro[t] + k] = c.res_svc_str[k];
      w.res_attrset[ro[t] + k] = set_map.at(c.res_set[k]);
      w.res_size[ro[t] + k] = c.res_size[k];
      w.res_ok[ro[t] + k] = c.res_ok[k];
      w.attr_res[ro[t] + k] = c.attr_res[k];
      w.lay.res_ref[ro[t] + k] = c.lay.res_ref[k];
      w.lay.res_scope0[ro[t] + k] = (uint32_t)(co[t] + c.lay.res_scope0[k]);
    }
    for (size_t k = 0; k < c.scope_size.size(); k++) {
      w.scope_size[co[t] + k] = c.scope_size[k];
      w.scope_res[co[t] + k] = (uint32_t)(ro[t] + c.scope_res[k]);
      w.lay.scope_ref[co[t] + k] = c.lay.scope_ref[k];
      w.lay.scope_hdr[co[t] + k] = c.lay.scope_hdr[k];
      w.lay.scope_schema[co[t] + k] = c.lay.scope_schema[k];
      w.lay.scope_span0[co[t] + k] = (uint32_t)(so[t] + c.lay.scope_span0[k]);   // gpu_scopes: into span_ref
      w.scope_on_host[co[t] + k] = c.scope_on_host[k];
      w.scope_count[co[t] + k] = c.scope_count[k];
    }
  };
  parallel_run((int)ch.size(), [&](int t) { place((size_t)t); });
  return true;
}
}  // namespace

namespace {
// The GPU half of the structural walk: every ScopeSpans the host did not
// walk is counted, sized and listed on the device (otlp_scope_*_kernel);
// returns the span count in *n_out, or 1 in *redo when some scope needs the
// host walk (groups or a malformed field: the caller walks on the host).
// The GPU half of the ResourceSpans level: the host walks
// the TracesData chain only (walk_chain), the device each record's fields
// (otlp_res_fields_kernel), the Resource columns from the device resource
// table; resources the table lacks are resolved on the host (pb_resource,
// columnize_resource: the same cache as the host walk), entered into the
// table, and their columns scattered in.  The attribute-set ids are then
// renumbered for the batch (ascending cache id).  *redo: a malformed record
// (the host walk reports it exactly).  Fills w.lay.res_ref and w.sets, *R,
// *S and the args of the scope listing.
// msg_in_stage: the message's H2D copy reads b->stage (a pageable caller
// buffer went through it), so the stage is reused only after that copy
int res_walk_gpu(OtlpEngine* o, OtlpBatchImpl* b, const uint8_t* pb, size_t len, hipStream_t st, Walked& w,
                 uint64_t* R_out, uint64_t* S_out, OtlpResArgs* args, bool* redo, bool msg_in_stage) {
  *redo = false;
  std::string err;
  int rc;
  // the TracesData chain: the host walk (it runs while the message's H2D
  // copy is in flight), or (engine option otlp_gpu_chain) segments walked on the GPU
  // and linked here, the host walk when the link fails.  The GPU form
  // measured slower (profiles/r3_otlp_gpu_resources.json host chain,
  // r3_otlp_gpu_chain_gpu_encode.json GPU chain: 10M spans 57.8 -> 97.4 ms of
  // walk, an 8192-span request 0.56 -> 2.06 ms of decode): it cannot
  // start before the whole message has landed, and each lane's hops through
  // its 64 KiB segment are dependent HBM reads.
  std::vector<uint64_t> seg_first;
  std::vector<uint32_t> seg_base;
  uint64_t R = 0;
  bool gpu_chain = len > 0 && b->e->option(Engine::kOptOtlpGpuChain);
  const uint32_t T = (uint32_t)((len + kChainSeg - 1) / kChainSeg);
  OtlpChainArgs ca{};
  if (gpu_chain) {
    const size_t o_end = up(8 * (size_t)T + 16), o_nrec = o_end + up(8 * (size_t)T + 16),
                 o_bad = o_nrec + up(4 * (size_t)T + 16), o_list = o_bad + up(4 * (size_t)T + 16),
                 o_first = o_list + up(8 * (size_t)T * kChainList + 16), o_base = o_first + up(8 * (size_t)T + 16),
                 o_total = o_base + up(4 * (size_t)T + 16);
    if ((rc = b->cslab.need(o_total)) || (rc = b->stage.need(o_first))) return rc;
    HIP_TRY(hipStreamSynchronize(st));   // the staging buffer (the message's H2D) is reused below
    ca.pb = b->arena.p;
    ca.n = len;
    ca.n_seg = T;
    ca.start = reinterpret_cast<uint64_t*>(b->cslab.p);
    ca.end = reinterpret_cast<uint64_t*>(b->cslab.p + o_end);
    ca.nrec = reinterpret_cast<uint32_t*>(b->cslab.p + o_nrec);
    ca.bad = reinterpret_cast<uint32_t*>(b->cslab.p + o_bad);
    ca.list = reinterpret_cast<uint64_t*>(b->cslab.p + o_list);
    ca.first = reinterpret_cast<const uint64_t*>(b->cslab.p + o_first);
    ca.base = reinterpret_cast<const uint32_t*>(b->cslab.p + o_base);
    (void)hipGetLastError();
    launch_otlp_chain_seg(ca, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(b->stage.p, b->cslab.p, o_first, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t* h_start = reinterpret_cast<const uint64_t*>(b->stage.p);
    const uint64_t* h_end = reinterpret_cast<const uint64_t*>(b->stage.p + o_end);
    const uint32_t* h_nrec = reinterpret_cast<const uint32_t*>(b->stage.p + o_nrec);
    const uint32_t* h_bad = reinterpret_cast<const uint32_t*>(b->stage.p + o_bad);
    const uint64_t* h_list = reinterpret_cast<const uint64_t*>(b->stage.p + o_list);
    // link: the true chain enters segment t at pos; the segment's walk must
    // have a field start there (its speculated start, or where a start
    // inside a record converged), and counts from it
    seg_first.assign(T, kChainNone);
    seg_base.assign(T, 0);
    uint64_t pos = 0;
    for (uint32_t t = 0; t < T && gpu_chain; t++) {
      const uint64_t s1 = std::min<uint64_t>(len, (uint64_t)t * kChainSeg + kChainSeg);
      if (pos >= s1) continue;   // a record covers the whole segment
      if (h_start[t] == kChainNone) { gpu_chain = false; break; }
      uint32_t j = 0, skipped = 0;
      while (j < kChainList && h_list[(uint64_t)t * kChainList + j] != kChainNone &&
             (h_list[(uint64_t)t * kChainList + j] & ~(1ull << 63)) != pos) {
        skipped += (uint32_t)(h_list[(uint64_t)t * kChainList + j] >> 63);
        j++;
      }
      if (j == kChainList || h_list[(uint64_t)t * kChainList + j] == kChainNone || h_bad[t]) { gpu_chain = false; break; }
      seg_first[t] = pos;
      seg_base[t] = (uint32_t)R;
      R += h_nrec[t] - skipped;
      pos = h_end[t];
    }
    if (pos != len) gpu_chain = false;   // the host walk decides (and reports a malformed message)
    if (R > 0xFFFFFFF0ull) gpu_chain = false;
  }
  if (!gpu_chain) {
    if (!walk_chain(pb, len, w.lay.res_ref, err)) return fail(OSE_EINVAL, err);
    // the staging buffer is reused below: wait for the message's H2D when it
    // came through it (a pinned caller buffer is copied from directly, and
    // the resource pass queues behind that copy on the stream)
    if (msg_in_stage) HIP_TRY(hipStreamSynchronize(st));
    R = w.lay.res_ref.size();
  }
  *R_out = R;
  const uint64_t RN = std::max<uint64_t>(R, 1);
  const uint32_t tiles = (uint32_t)((RN + kScanTileItems - 1) / kScanTileItems);
  struct Part { void** dst; size_t bytes; };
  OtlpResArgs a{};
  uint64_t* status = nullptr;
  uint32_t* words = nullptr;
  const std::vector<Part> parts = {
      {(void**)&a.res_ref, 8 * RN}, {(void**)&a.flags, 4 * RN}, {(void**)&a.nscope, 4 * RN},
      {(void**)&a.schema_len, 4 * RN}, {(void**)&a.scope0, 4 * RN}, {(void**)&a.res_svc, 4 * RN},
      {(void**)&a.res_svc_str, 4 * RN}, {(void**)&a.res_set, 4 * RN}, {(void**)&a.res_size, 4 * RN},
      {(void**)&a.res_ok, RN}, {(void**)&a.attr_res, 8 * RN}, {(void**)&a.miss_list, 4 * RN},
      {(void**)&status, 8 * (size_t)tiles + 64}, {(void**)&words, 64},
  };
  size_t total = 0;
  for (auto& p : parts) total = up(total + p.bytes + 16);
  if ((rc = b->rslab.need(total)) || (rc = b->stage.need(std::max<size_t>(8 * RN, 12 * (size_t)T) + 64))) return rc;
  size_t off = 0;
  for (auto& p : parts) {
    *p.dst = b->rslab.p + off;
    off = up(off + p.bytes + 16);
  }
  if (gpu_chain) {   // the records of the linked segments, written on the GPU
    std::memcpy(b->stage.p, seg_first.data(), 8 * (size_t)T);
    std::memcpy(b->stage.p + 8 * (size_t)T, seg_base.data(), 4 * (size_t)T);
    HIP_TRY(hipMemcpyAsync(const_cast<uint64_t*>(ca.first), b->stage.p, 8 * (size_t)T, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(const_cast<uint32_t*>(ca.base), b->stage.p + 8 * (size_t)T, 4 * (size_t)T,
                           hipMemcpyHostToDevice, st));
    ca.res_ref = const_cast<uint64_t*>(a.res_ref);
    launch_otlp_chain_list(ca, st);
    HIP_TRY(hipGetLastError());
  } else if (R) {
    std::memcpy(b->stage.p, w.lay.res_ref.data(), 8 * R);
    HIP_TRY(hipMemcpyAsync(const_cast<uint64_t*>(a.res_ref), b->stage.p, 8 * R, hipMemcpyHostToDevice, st));
  }
  b->d_res_ref = const_cast<uint64_t*>(a.res_ref);
  HIP_TRY(hipMemsetAsync(status, 0, reinterpret_cast<uint8_t*>(words) + 64 - reinterpret_cast<uint8_t*>(status), st));
  a.pb = b->arena.p;
  a.n_res = R;
  a.any_bad = words;
  a.miss_count = words + 1;
  uint32_t h[4] = {0, 0, 0, 0};
  {
    DevResTable& t = o->res_dev;
    {
      std::unique_lock<std::shared_mutex> g(t.mu);
      if ((rc = t.ensure())) return rc;
    }
    std::shared_lock<std::shared_mutex> g(t.mu);   // held until the lookups have run
    a.table = t.d_slots;
    a.keys = t.d_keys;
    (void)hipGetLastError();
    launch_otlp_res_fields(a, st);
    HIP_TRY(hipGetLastError());
    ScanArgs sa{};
    sa.n = R;
    sa.n_tiles = tiles;
    sa.in = a.nscope;
    sa.out = const_cast<uint32_t*>(a.scope0);
    sa.total = words + 2;
    sa.counter = words + 3;
    sa.status = status;
    sa.error = words + 4;
    if (R) launch_scan_u32(sa, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h, words, 12, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  if (h[0]) { *redo = true; return 0; }
  *S_out = h[2];
  // the resources the table lacks: resolved on the host
  const uint32_t nm = h[1];
  if (nm) {
    if (w.lay.res_ref.size() != R) {   // the refs the GPU chain walk wrote
      w.lay.res_ref.resize(R);
      HIP_TRY(hipMemcpy(w.lay.res_ref.data(), a.res_ref, 8 * R, hipMemcpyDeviceToHost));
    }
    std::vector<uint32_t> miss(nm);
    HIP_TRY(hipMemcpy(miss.data(), a.miss_list, 4 * (size_t)nm, hipMemcpyDeviceToHost));
    std::vector<OtlpResFix> fix(nm);
    std::vector<uint8_t> keyed(nm, 0);   // entered into the device table (one Resource field or none)
    std::vector<std::pair<size_t, size_t>> key_of(nm);
    const int T = (int)std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)parallel_width(), nm / 256));
    std::vector<std::string> errs((size_t)T);
    parallel_run(T, [&](int t) {
      ProtoSizer sizer;
      std::vector<std::pair<size_t, size_t>> resf;
      for (uint32_t k = (uint32_t)((uint64_t)nm * t / T); k < (uint32_t)((uint64_t)nm * (t + 1) / T); k++) {
        const uint32_t r = miss[k];
        const uint64_t rr = w.lay.res_ref[r];
        const size_t ro = (uint32_t)rr;
        PbReader rd(pb + ro, (size_t)(rr >> 32));
        resf.clear();
        uint32_t f, wt;
        while (rd.more() && rd.tag(f, wt)) {
          size_t fo, fl;
          if (f == 1 || f == 2 || f == 3 || f == 1000) {
            if (wt != 2 || !rd.bytes(fo, fl)) { rd.fail(); break; }
            if (f == 1) resf.emplace_back(ro + fo, fl);
          } else {
            rd.skip(wt, f);
          }
        }
        if (!rd.ok) { errs[t] = "OTLP protobuf: malformed ResourceSpans"; return; }
        CachedRes cr{};
        bool have = false;
        const std::string_view key = resf.size() == 1 ? std::string_view((const char*)pb + resf[0].first, resf[0].second)
                                                      : std::string_view();
        if (resf.size() <= 1) {
          std::shared_lock<std::shared_mutex> g(o->res_cache.mu);
          auto ci = o->res_cache.map.find(key);
          if (ci != o->res_cache.map.end()) {
            cr = ci->second;
            have = true;
          }
        }
        if (!have && !resolve_resource(o->ctx, o->res_cache, pb, resf, sizer, cr)) {
          errs[t] = "OTLP protobuf: malformed Resource";
          return;
        }
        fix[k] = OtlpResFix{r, cr.svc, cr.svc_str, cr.set, cr.rpart, cr.ok, cr.attr_res};
        if (resf.size() <= 1) {
          keyed[k] = 1;
          key_of[k] = resf.empty() ? std::pair<size_t, size_t>(0, 0) : resf[0];
        }
      }
    });
    for (auto& e : errs)
      if (!e.empty()) return fail(OSE_EINVAL, e);
    if ((rc = b->fixdev.need(sizeof(OtlpResFix) * nm)) || (rc = b->stage.need(sizeof(OtlpResFix) * nm))) return rc;
    std::memcpy(b->stage.p, fix.data(), sizeof(OtlpResFix) * nm);
    HIP_TRY(hipMemcpyAsync(b->fixdev.p, b->stage.p, sizeof(OtlpResFix) * nm, hipMemcpyHostToDevice, st));
    launch_otlp_res_fix(a, reinterpret_cast<const OtlpResFix*>(b->fixdev.p), nm, st);
    HIP_TRY(hipGetLastError());
    {   // later calls find these on the device
      DevResTable& t = o->res_dev;
      std::unique_lock<std::shared_mutex> g(t.mu);
      for (uint32_t k = 0; k < nm; k++) {
        if (!keyed[k]) continue;
        const CachedRes cr{fix[k].svc, fix[k].svc_str, fix[k].set, fix[k].rpart, (uint8_t)fix[k].ok, fix[k].attr_res};
        t.insert(pb + key_of[k].first, (uint32_t)key_of[k].second, cr);
      }
      if ((rc = t.sync(st))) return rc;
    }
  }
  // the cache's attribute-set ids -> this batch's (first appearance)
  uint32_t n_sets;
  {
    std::shared_lock<std::shared_mutex> g(o->res_cache.mu);
    n_sets = (uint32_t)o->res_cache.sets.size();
  }
  const uint64_t NS = std::max<uint64_t>(n_sets, 1);
  const size_t o_flag = up(4 * NS + 16), o_pos = o_flag + up(4 * RN + 16), o_list = o_pos + up(4 * RN + 16),
               o_stat = o_list + up(4 * RN + 16), o_words = o_stat + up(8 * (size_t)tiles + 64);
  if ((rc = b->setbuf.need(o_words + 64))) return rc;
  uint32_t* first = reinterpret_cast<uint32_t*>(b->setbuf.p);
  uint32_t* is_first = reinterpret_cast<uint32_t*>(b->setbuf.p + o_flag);
  uint32_t* pos = reinterpret_cast<uint32_t*>(b->setbuf.p + o_pos);
  uint32_t* list = reinterpret_cast<uint32_t*>(b->setbuf.p + o_list);
  uint64_t* sstat = reinterpret_cast<uint64_t*>(b->setbuf.p + o_stat);
  uint32_t* swords = reinterpret_cast<uint32_t*>(b->setbuf.p + o_words);
  HIP_TRY(hipMemsetAsync(first, 0xFF, 4 * NS, st));
  HIP_TRY(hipMemsetAsync(sstat, 0, o_words + 64 - o_stat, st));
  launch_otlp_set_first(a.res_set, R, first, is_first, st);
  HIP_TRY(hipGetLastError());
  ScanArgs ss{};
  ss.n = R;
  ss.n_tiles = tiles;
  ss.in = is_first;
  ss.out = pos;
  ss.total = swords + 1;
  ss.counter = swords + 2;
  ss.status = sstat;
  ss.error = swords;
  if (R) launch_scan_u32(ss, st);
  HIP_TRY(hipGetLastError());
  launch_otlp_set_apply(a.res_set, R, first, is_first, pos, list, st);
  HIP_TRY(hipGetLastError());
  // the scan's words and the batch's set ids come back behind the scope
  // pass, whose wait the host makes anyway (res_sets_finish)
  if ((rc = b->seth.need(4 * (RN + 2)))) return rc;
  uint32_t* hs = reinterpret_cast<uint32_t*>(b->seth.p);
  HIP_TRY(hipMemcpyAsync(hs, swords, 8, hipMemcpyDeviceToHost, st));
  if (R) HIP_TRY(hipMemcpyAsync(hs + 2, list, 4 * R, hipMemcpyDeviceToHost, st));
  *args = a;
  b->d_res_scope0 = const_cast<uint32_t*>(a.scope0);
  b->d_attr_res = a.attr_res;
  return 0;
}

// the batch's attribute sets from res_walk_gpu's copies (first appearance)
int res_sets_finish(OtlpEngine* o, OtlpBatchImpl* b, Walked& w, hipStream_t st) {
  HIP_TRY(hipStreamSynchronize(st));   // (the scope pass has waited already: returns at once)
  const uint32_t* hs = reinterpret_cast<const uint32_t*>(b->seth.p);
  if (hs[0]) return fail(OSE_EDEVICE, "OTLP ingest: attribute-set scan error");
  std::shared_lock<std::shared_mutex> g(o->res_cache.mu);
  w.sets.clear();
  for (uint32_t k = 0; k < hs[1]; k++) w.sets.push_back(o->res_cache.sets[hs[2 + k]]);
  return 0;
}

// res: the GPU ResourceSpans pass ran (res_walk_gpu): its S scopes are listed
// on the device by otlp_res_scopes_kernel, every one walked here
int scope_walk_gpu(Engine* e, OtlpBatchImpl* b, Walked& w, hipStream_t st, uint64_t* n_out, bool* redo,
                   OtlpResArgs* res = nullptr, uint64_t S_res = 0) {
  (void)e;
  const uint64_t S = res ? S_res : w.scope_size.size(), H = res ? 0 : w.span_ref.size();
  *redo = false;
  const uint32_t tiles = (uint32_t)((S + kScanTileItems - 1) / kScanTileItems);
  struct Part { void** dst; size_t bytes; const void* src; };
  uint64_t *scope_ref, *hdr, *schema, *host_at, *host_refs, *status;
  uint8_t* on_host;
  uint32_t *count, *scope_size, *flags, *span0, *scope_res, *words;
  std::vector<Part> parts = {
      {(void**)&scope_ref, 8 * S, res ? nullptr : b->lay.scope_ref.data()},
      {(void**)&hdr, 8 * S, res ? nullptr : b->lay.scope_hdr.data()},
      {(void**)&schema, 8 * S, res ? nullptr : b->lay.scope_schema.data()},
      {(void**)&host_at, 8 * S, nullptr},
      {(void**)&host_refs, 8 * H, res ? nullptr : w.span_ref.data()},
      {(void**)&on_host, S, res ? nullptr : w.scope_on_host.data()},
      {(void**)&count, 4 * S, res ? nullptr : w.scope_count.data()},
      {(void**)&scope_size, 4 * S, res ? nullptr : w.scope_size.data()},
      {(void**)&scope_res, 4 * S, res ? nullptr : w.scope_res.data()},
      // device-only
      {(void**)&flags, 4 * S, nullptr},
      {(void**)&span0, 4 * S, nullptr},
      {(void**)&status, 8 * (size_t)tiles + 64, nullptr},
      {(void**)&words, 64, nullptr},
  };
  size_t total = 0, inputs = 0;
  for (auto& p : parts) {
    total = up(total + p.bytes + 16);
    if (!res && (p.src || p.dst == (void**)&host_at)) inputs = total;
  }
  int rc;
  if ((rc = b->sslab.need(total)) || (rc = b->stage.need(inputs))) return rc;
  size_t off = 0;
  for (auto& p : parts) {
    *p.dst = b->sslab.p + off;
    if (!res && p.src && p.bytes) std::memcpy(b->stage.p + off, p.src, p.bytes);
    off = up(off + p.bytes + 16);
  }
  if (!res) {   // host_at: the host-walked scopes' offsets into host_refs (the walk's span0)
    uint64_t* ha = reinterpret_cast<uint64_t*>(b->stage.p + (reinterpret_cast<uint8_t*>(host_at) - b->sslab.p));
    for (uint64_t q = 0; q < S; q++) ha[q] = b->lay.scope_span0[q];
    HIP_TRY(hipMemcpyAsync(b->sslab.p, b->stage.p, inputs, hipMemcpyHostToDevice, st));
  } else {
    // the scopes of every resource at their place, none walked on the host
    HIP_TRY(hipMemsetAsync(on_host, 0, S, st));
    res->scope_ref = scope_ref;
    res->scope_res = scope_res;
    launch_otlp_res_scopes(*res, st);
    HIP_TRY(hipGetLastError());
    b->d_scope_ref = scope_ref;
  }
  const size_t dev0 = reinterpret_cast<uint8_t*>(flags) - b->sslab.p;
  HIP_TRY(hipMemsetAsync(flags, 0, total - dev0, st));   // flags, span0, scan status, words
  OtlpScopeArgs a{};
  a.pb = b->arena.p;
  a.n_scopes = S;
  a.scope_ref = scope_ref;
  a.on_host = on_host;
  a.scope_res = scope_res;
  a.count = count;
  a.scope_size = scope_size;
  a.hdr = hdr;
  a.schema = schema;
  a.flags = flags;
  a.span0 = span0;
  a.host_refs = host_refs;
  a.host_at = host_at;
  b->sargs = a;
  (void)hipGetLastError();
  launch_otlp_scope_count(a, st);
  HIP_TRY(hipGetLastError());
  ScanArgs sa{};
  sa.n = S;
  sa.n_tiles = tiles;
  sa.in = count;
  sa.out = span0;
  sa.total = words + 1;
  sa.counter = words + 2;
  sa.status = status;
  sa.error = words;
  if (S) launch_scan_u32(sa, st);
  HIP_TRY(hipGetLastError());
  uint32_t h[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(h, words, 8, hipMemcpyDeviceToHost, st));
  // which scopes the host must finish (flags): copied back with the counts
  std::vector<uint32_t> fl(S);
  if (S) HIP_TRY(hipMemcpyAsync(fl.data(), flags, 4 * S, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (h[0]) return fail(OSE_EDEVICE, "OTLP ingest: scope scan error");
  *n_out = h[1];
  b->d_span0 = span0;
  b->d_hdr = hdr;
  b->d_schema = schema;
  std::vector<std::pair<uint64_t, uint32_t>> patch;   // scope sizes the host computes
  ProtoSizer sizer;
  if (res) {
    bool any = false;
    for (uint64_t q = 0; q < S && !any; q++) any = fl[q] != 0;
    if (any) {   // the flagged scopes' refs
      b->lay.scope_ref.resize(S);
      HIP_TRY(hipMemcpy(b->lay.scope_ref.data(), scope_ref, 8 * S, hipMemcpyDeviceToHost));
    }
  }
  for (uint64_t q = 0; q < S; q++) {
    if (!fl[q]) continue;
    if (fl[q] & 2) { *redo = true; return 0; }
    // a merged or unusual InstrumentationScope: pb_scope over its fields
    const uint64_t sr = b->lay.scope_ref[q];
    PbReader r(b->pb + (uint32_t)sr, (size_t)(sr >> 32));
    ScopeSpans meta;
    size_t sch = 0;
    uint32_t f, wt;
    while (r.more() && r.tag(f, wt)) {
      size_t o, l;
      if ((f == 1 || f == 2 || f == 3) && wt == 2 && r.bytes(o, l)) {
        if (f == 1 && !pb_scope(b->pb + (uint32_t)sr + o, l, meta))
          return fail(OSE_EINVAL, "OTLP protobuf: malformed InstrumentationScope");
        if (f == 3) sch = l;
      } else if (f == 1 || f == 2 || f == 3) {
        return fail(OSE_EINVAL, "OTLP protobuf: malformed ScopeSpans");
      } else {
        r.skip(wt, f);
      }
    }
    if (!r.ok) return fail(OSE_EINVAL, "OTLP protobuf: malformed ScopeSpans");
    patch.emplace_back(q, (uint32_t)(sizer.scope_fixed(meta) + (sch ? flen(sch) : 0)));
  }
  for (auto& x : patch) HIP_TRY(hipMemcpyAsync(scope_size + x.first, &x.second, 4, hipMemcpyHostToDevice, st));
  if (!patch.empty()) HIP_TRY(hipStreamSynchronize(st));   // the patch sources are on this stack
  b->cols.scope_size = scope_size;
  b->cols.scope_resource = scope_res;
  // pass 2 writes into the span columns decode() allocates next
  b->layout_on_host = false;
  return 0;
}

// span refs and the scopes' span0 / header / schema refs back to the host
// (the encoder and the host pass read them there)
int layout_to_host(OtlpBatchImpl* b, hipStream_t st) {
  if (b->layout_on_host) return 0;
  const uint64_t n = b->cols.n_spans, S = b->cols.n_scopes, R = b->cols.n_resources;
  b->span_ref.resize(n);
  std::vector<uint32_t> span0(S);
  if (b->res_on_device) {   // the ResourceSpans level was walked on the GPU too
    if (b->lay.res_ref.size() != R) {
      b->lay.res_ref.resize(R);
      if (R) HIP_TRY(hipMemcpyAsync(b->lay.res_ref.data(), b->d_res_ref, 8 * R, hipMemcpyDeviceToHost, st));
    }
    b->lay.res_scope0.resize(R);
    b->lay.scope_ref.resize(S);
    b->lay.scope_hdr.resize(S);
    b->lay.scope_schema.resize(S);
    b->lay.scope_span0.resize(S);
    if (R) HIP_TRY(hipMemcpyAsync(b->lay.res_scope0.data(), b->d_res_scope0, 4 * R, hipMemcpyDeviceToHost, st));
    if (S) HIP_TRY(hipMemcpyAsync(b->lay.scope_ref.data(), b->d_scope_ref, 8 * S, hipMemcpyDeviceToHost, st));
  }
  if (n) HIP_TRY(hipMemcpyAsync(b->span_ref.data(), b->d_span_ref, 8 * n, hipMemcpyDeviceToHost, st));
  if (S) {
    HIP_TRY(hipMemcpyAsync(span0.data(), b->d_span0, 4 * S, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(b->lay.scope_hdr.data(), b->d_hdr, 8 * S, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(b->lay.scope_schema.data(), b->d_schema, 8 * S, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  for (uint64_t q = 0; q < S; q++) b->lay.scope_span0[q] = span0[q];
  b->layout_on_host = true;
  return 0;
}

int decode(Engine* e, const uint8_t* pb, size_t len, hipStream_t st, OtlpBatchImpl* b, bool host_scopes = false,
           bool host_res = false) {
  int rc;
  OtlpEngine* o = otlp_engine(e, rc);
  if (!o) return rc;
  if (len > 0xFFFFFFF0ull) return fail(OSE_ERANGE, "OTLP ingest: message beyond the 4 GiB arena range");
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  auto lap = [&](int k) {
    const auto t = clk::now();
    b->t_ms[k] = std::chrono::duration<double, std::milli>(t - t0).count();
    t0 = t;
  };
  for (double& x : b->t_ms) x = 0;
  // 1. the bytes H2D (straight from the caller's buffer when it is pinned,
  //    else through pinned staging), the walk meanwhile
  const size_t pb_cap = up(len + 16, 16);
  const size_t fix_reserve = std::max<size_t>(1 << 16, len / 8);
  if ((rc = b->arena.need(pb_cap + fix_reserve + 16))) return rc;
  hipPointerAttribute_t pa{};
  const bool pinned = len && hipPointerGetAttributes(&pa, pb) == hipSuccess && pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();   // an unregistered pointer is not an error here
  if (pinned) {
    HIP_TRY(hipMemcpyAsync(b->arena.p, pb, len, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(b->arena.p + len, 0, pb_cap - len, st));
  } else {
    if ((rc = b->stage.need(pb_cap))) return rc;
    par_memcpy(b->stage.p, pb, len);
    std::memset(b->stage.p + len, 0, pb_cap - len);
    HIP_TRY(hipMemcpyAsync(b->arena.p, b->stage.p, pb_cap, hipMemcpyHostToDevice, st));
  }
  lap(0);
  // 2. the walk: TracesData and ResourceSpans on the host, ScopeSpans up to
  //    64 KB on the GPU (engine option otlp_host_scopes: all on the host)
  //    (otlp_host_resources: ResourceSpans on the host, ScopeSpans on the
  //    GPU; without it only the TracesData chain is walked on the host)
  const bool gpu_scopes = !host_scopes && !e->option(Engine::kOptOtlpHostScopes);
  const bool gpu_res = gpu_scopes && !host_res && !e->option(Engine::kOptOtlpHostResources);
  Walked w;
  OtlpResArgs ra{};
  uint64_t R = 0, S = 0;
  if (gpu_res) {
    bool redo = false;
    if ((rc = res_walk_gpu(o, b, pb, len, st, w, &R, &S, &ra, &redo, !pinned))) return rc;
    if (redo) return decode(e, pb, len, st, b, false, true);   // a malformed record: the host walk reports it
  } else {
    if (!walk(o->ctx, o->res_cache, pb, len, w, gpu_scopes)) return fail(OSE_EINVAL, w.err);
    HIP_TRY(hipStreamSynchronize(st));   // the staging buffer is reused below
    R = w.res_svc.size();
  }
  lap(1);
  b->pb = pb;
  b->pb_len = len;
  b->lay = std::move(w.lay);
  b->layout_on_host = true;
  b->res_on_device = gpu_res;
  ose_columns& c = b->cols;
  c = ose_columns{};
  c.n_resources = (uint32_t)R;
  uint64_t n = 0;
  b->scopes_dev = false;
  if (gpu_scopes) {
    bool redo = false;
    rc = scope_walk_gpu(e, b, w, st, &n, &redo, gpu_res ? &ra : nullptr, S);
    if (gpu_res) {   // (also before an error return or a redo: no copy into seth may stay in flight)
      const int src = res_sets_finish(o, b, w, st);
      if (!rc) rc = src;
    }
    if (rc) return rc;
    if (redo) return decode(e, pb, len, st, b, true, true);   // a scope needs the host walk: all on the host
    b->scopes_dev = true;
  } else {
    n = w.span_ref.size();
    b->span_ref = std::move(w.span_ref);
  }
  if (!gpu_res) S = b->lay.scope_ref.size();
  if (n > 0xFFFFFFF0ull) return fail(OSE_ERANGE, "OTLP ingest: more than 2^32-16 spans");
  const uint32_t K = o->n_attr_keys;
  b->attrsets = std::move(w.sets);
  ProtoSizer sizer;
  // device columns: one slab
  const uint64_t N = std::max<uint64_t>(n, 1);
  struct Part { void** dst; size_t bytes; const void* src; };
  uint8_t* host_flag = nullptr;
  uint32_t* host_count = nullptr;
  uint32_t* host_list = nullptr;
  uint64_t* span_ref = nullptr;
  const ose_columns keep_scope = c;   // scope_size / scope_resource set by the GPU walk
  std::vector<Part> parts = {
      {(void**)&span_ref, 8 * N, gpu_scopes ? nullptr : b->span_ref.data()},
      {(void**)&c.resource, 4 * N, gpu_scopes ? nullptr : w.span_res.data()},
      {(void**)&c.scope, 4 * N, gpu_scopes ? nullptr : w.span_scope.data()},
  };
  if (!gpu_res) {
    parts.push_back({(void**)&c.res_svc, 4 * R, w.res_svc.data()});
    parts.push_back({(void**)&c.res_svc_str, 4 * R, w.res_svc_str.data()});
    parts.push_back({(void**)&c.res_url_ok, R, w.res_ok.data()});
    parts.push_back({(void**)&c.res_attrset, 4 * R, w.res_attrset.data()});
    parts.push_back({(void**)&c.res_size, 4 * R, w.res_size.data()});
  }
  if (!gpu_scopes) {
    parts.push_back({(void**)&c.scope_size, 4 * S, w.scope_size.data()});
    parts.push_back({(void**)&c.scope_resource, 4 * S, w.scope_res.data()});
  }
  const std::vector<Part> outs = {
      // outputs of the decoder
      {(void**)&c.trace_id, 16 * N, nullptr},
      {(void**)&c.start_ns, 8 * N, nullptr},
      {(void**)&c.end_ns, 8 * N, nullptr},
      {(void**)&c.status, N, nullptr},
      {(void**)&c.kind, N, nullptr},
      {(void**)&c.url_flags, N, nullptr},
      {(void**)&c.path, 8 * N, nullptr},
      {(void**)&c.route, 8 * N, nullptr},
      {(void**)&c.span_size, 4 * N, nullptr},
      {(void**)&c.name_len, 4 * N, nullptr},
      {(void**)&host_flag, N, nullptr},
      {(void**)&host_count, 16, nullptr},
      {(void**)&host_list, 4 * N, nullptr},
  };
  parts.insert(parts.end(), outs.begin(), outs.end());
  if (o->json_rules) parts.push_back({(void**)&c.attr_match, 8 * N * (size_t)o->attr_words, nullptr});
  if (K) {
    parts.push_back({(void**)&c.attr_type, (size_t)K * N, nullptr});
    parts.push_back({(void**)&c.attr_val, 8 * (size_t)K * N, nullptr});
  }
  size_t total = 0, inputs = 0;
  for (auto& p : parts) {
    total = up(total + p.bytes + 16);
    if (p.src) inputs = total;
  }
  if ((rc = b->slab.need(total)) || (rc = b->stage.need(inputs))) return rc;
  size_t off = 0;
  for (auto& p : parts) {
    *p.dst = b->slab.p + off;
    if (p.src && p.bytes) std::memcpy(b->stage.p + off, p.src, p.bytes);
    off = up(off + p.bytes + 16);
  }
  if (inputs) HIP_TRY(hipMemcpyAsync(b->slab.p, b->stage.p, inputs, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(host_count, 0, 16, st));
  if (gpu_res) {   // the resource columns the GPU pass wrote
    c.res_svc = ra.res_svc;
    c.res_svc_str = ra.res_svc_str;
    c.res_url_ok = ra.res_ok;
    c.res_attrset = ra.res_set;
    c.res_size = ra.res_size;
  }
  if (gpu_scopes) {
    c.scope_size = keep_scope.scope_size;
    c.scope_resource = keep_scope.scope_resource;
    // pass 2: the span refs of every scope at their place
    OtlpScopeArgs sa = b->sargs;
    sa.span_ref = span_ref;
    sa.span_res = const_cast<uint32_t*>(c.resource);
    sa.span_scope = const_cast<uint32_t*>(c.scope);
    launch_otlp_scope_spans(sa, st);
    HIP_TRY(hipGetLastError());
    b->d_span_ref = span_ref;
    b->d_span_res = const_cast<uint32_t*>(c.resource);
    b->span_ref.clear();
  }
  b->d_spans = span_ref;
  c.n_spans = n;
  c.n_resources = (uint32_t)R;
  c.n_scopes = (uint32_t)S;
  c.n_attrsets = (uint32_t)b->attrsets.size();
  c.arena = b->arena.p;
  c.arena_bytes = len;
  c.n_attr_keys = K;
  c.attr_match_words = o->attr_words;
  if (!o->ctx.url_filter) c.res_url_ok = nullptr;
  std::vector<uint64_t>& attr_res = w.attr_res;
  lap(2);
  // 3. the GPU decoder
  OtlpArgs a{};
  a.pb = b->arena.p;
  a.n_spans = n;
  a.span_ref = span_ref;
  a.keys = reinterpret_cast<const OtlpKeyDev*>(o->keys_dev);
  a.key_bytes = o->keys_dev + o->keys.size() * sizeof(OtlpKeyDev);
  a.n_keys = (uint32_t)o->keys.size();
  a.n_attr_keys = K;
  a.attr_words = o->attr_words;
  a.key_lens = o->key_lens;
  a.tid = const_cast<uint64_t*>(c.trace_id);
  a.start = const_cast<uint64_t*>(c.start_ns);
  a.end = const_cast<uint64_t*>(c.end_ns);
  a.status = const_cast<uint8_t*>(c.status);
  a.kind = const_cast<uint8_t*>(c.kind);
  a.url_flags = const_cast<uint8_t*>(c.url_flags);
  a.path = const_cast<ose_strref*>(c.path);
  a.route = const_cast<ose_strref*>(c.route);
  a.span_size = const_cast<uint32_t*>(c.span_size);
  a.name_len = const_cast<uint32_t*>(c.name_len);
  a.attr_match = const_cast<uint64_t*>(c.attr_match);
  a.attr_type = const_cast<uint8_t*>(c.attr_type);
  a.attr_val = const_cast<uint64_t*>(c.attr_val);
  a.host_flag = host_flag;
  a.host_count = host_count;
  a.host_list = host_list;
  a.host_cap = (uint32_t)N;
  (void)hipGetLastError();   // a stale error of an earlier call must not be reported as this launch's
  Engine::Timed tm{};
  e->prof_begin("otlp_span_kernel", st, tm);
  if (n) launch_otlp_spans(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  // 4. the host pass
  uint32_t cnt = 0;
  HIP_TRY(hipMemcpyAsync(&cnt, host_count, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  b->host_spans = cnt;
  lap(3);
  if (!cnt) return 0;
  std::vector<uint32_t> span_res;
  const std::vector<uint32_t>* sres = &w.span_res;
  if (gpu_res && !o->wide_host_rules) {   // the resources' span_attribute service bits from the device
    attr_res.resize(R);
    if (R) HIP_TRY(hipMemcpy(attr_res.data(), b->d_attr_res, 8 * R, hipMemcpyDeviceToHost));
  }
  std::vector<uint32_t> res_svc_h;   // wide_host_rules: the resources' service ids
  if (o->wide_host_rules) {
    if (gpu_res) {
      res_svc_h.resize(R);
      if (R) HIP_TRY(hipMemcpy(res_svc_h.data(), c.res_svc, 4 * R, hipMemcpyDeviceToHost));
    } else {
      res_svc_h = w.res_svc;
    }
  }
  if (!b->layout_on_host) {   // the spans' refs and resources from the device
    if ((rc = layout_to_host(b, st))) return rc;
    span_res.resize(n);
    HIP_TRY(hipMemcpy(span_res.data(), b->d_span_res, 4 * n, hipMemcpyDeviceToHost));
    sres = &span_res;
  }
  std::vector<uint32_t> list(cnt);
  HIP_TRY(hipMemcpy(list.data(), host_list, 4 * (size_t)cnt, hipMemcpyDeviceToHost));
  std::vector<OtlpFix> fix(cnt);
  std::vector<uint8_t> fix_type((size_t)cnt * K);
  std::vector<uint64_t> fix_val((size_t)cnt * K);
  const uint32_t AW = o->json_rules ? o->attr_words : 0;   // attr_match words the host pass writes per span
  std::vector<uint64_t> fix_attr((size_t)cnt * AW);
  std::string strs;   // appended after the message bytes
  const size_t str_base = pb_cap;
  auto put = [&](std::string_view s) {
    ose_strref r{(uint32_t)(str_base + strs.size()), (uint32_t)s.size()};
    strs += s;
    return r;
  };
  SpanCols sc;
  std::vector<uint64_t> res_words;
  for (uint32_t q = 0; q < cnt; q++) {
    const uint32_t i = list[q];
    const uint64_t ref = b->span_ref[i];
    Span sp;
    if (!pb_span(pb + (uint32_t)ref, (size_t)(ref >> 32), sp)) return fail(OSE_EINVAL, "OTLP protobuf: malformed Span");
    if (o->wide_host_rules) {
      const uint32_t sv = res_svc_h[(*sres)[i]];
      if (sv < o->host_rules_by_svc.size()) res_words = o->host_rules_by_svc[sv];
      else res_words.assign(std::max<size_t>(1, o->ctx.attr_plan.host_mask.size()), 0);
    } else {
      host_rule_words(o->ctx.attr_plan, attr_res[(*sres)[i]], res_words);
    }
    columnize_span(o->ctx, sp, res_words, sizer, sc);
    for (uint32_t w = 0; w < AW; w++) fix_attr[(size_t)q * AW + w] = w < sc.attr_match.size() ? sc.attr_match[w] : 0;
    OtlpFix& x = fix[q];
    x = OtlpFix{};
    x.idx = i;
    x.hi = sc.hi;
    x.lo = sc.lo;
    x.start = sc.start;
    x.end = sc.end;
    x.status = sc.status;
    x.kind = sc.kind;
    x.url_flags = sc.url_flags;
    x.span_size = sc.span_size;
    x.name_len = sc.name_len;
    for (uint32_t k = 0; k < K; k++) {
      uint64_t v = sc.attr_val[k];
      if (sc.attr_type[k] == OSE_ATTR_STR) {
        const ose_strref r = put(sc.attr_str[k]);
        v = (uint64_t)r.off | ((uint64_t)r.len << 32);
      }
      fix_type[(size_t)q * K + k] = sc.attr_type[k];
      fix_val[(size_t)q * K + k] = v;
    }
    x.route = sc.has_route ? put(sc.route) : ose_strref{0, 0};
    x.path = (sc.url_flags & OSE_URL_PATH_MASK) != OSE_URL_PATH_NONE ? put(sc.path) : ose_strref{0, 0};
  }
  if (str_base + strs.size() + 16 > b->arena.cap) {
    // a larger arena: the message bytes move with it
    DevBuf bigger;
    if ((rc = bigger.need(str_base + strs.size() + 16))) return rc;
    HIP_TRY(hipMemcpyAsync(bigger.p, b->arena.p, pb_cap, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::swap(b->arena.p, bigger.p);
    std::swap(b->arena.cap, bigger.cap);
    c.arena = b->arena.p;
  }
  c.arena_bytes = str_base + strs.size();
  const size_t fb = up(cnt * sizeof(OtlpFix)), tb = up((size_t)cnt * K + 16), vb = up((size_t)cnt * K * 8 + 16);
  const size_t ab = up((size_t)cnt * AW * 8 + 16), fixb = fb + tb + vb + ab;
  if ((rc = b->stage.need(fixb + strs.size() + 16))) return rc;
  DevBuf& fixdev = b->fixdev;
  if ((rc = fixdev.need(fixb))) return rc;
  std::memcpy(b->stage.p, fix.data(), cnt * sizeof(OtlpFix));
  if (K) {
    std::memcpy(b->stage.p + fb, fix_type.data(), (size_t)cnt * K);
    std::memcpy(b->stage.p + fb + tb, fix_val.data(), (size_t)cnt * K * 8);
  }
  std::memcpy(b->stage.p + fb + tb + vb, fix_attr.data(), (size_t)cnt * AW * 8);
  std::memcpy(b->stage.p + fixb, strs.data(), strs.size());
  HIP_TRY(hipMemcpyAsync(fixdev.p, b->stage.p, fixb, hipMemcpyHostToDevice, st));
  if (!strs.empty())
    HIP_TRY(hipMemcpyAsync(b->arena.p + str_base, b->stage.p + fixb, strs.size(), hipMemcpyHostToDevice, st));
  OtlpFixArgs fa{};
  fa.n = cnt;
  fa.n_attr_keys = K;
  fa.attr_words = AW;
  fa.fix_attr = reinterpret_cast<const uint64_t*>(fixdev.p + fb + tb + vb);
  fa.n_spans = n;
  fa.fix = reinterpret_cast<const OtlpFix*>(fixdev.p);
  fa.fix_type = fixdev.p + fb;
  fa.fix_val = reinterpret_cast<const uint64_t*>(fixdev.p + fb + tb);
  fa.tid = a.tid;
  fa.start = a.start;
  fa.end = a.end;
  fa.status = a.status;
  fa.kind = a.kind;
  fa.url_flags = a.url_flags;
  fa.path = a.path;
  fa.route = a.route;
  fa.span_size = a.span_size;
  fa.name_len = a.name_len;
  fa.attr_match = a.attr_match;
  fa.attr_type = a.attr_type;
  fa.attr_val = a.attr_val;
  launch_otlp_fix(fa, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));   // fixdev and the staging are reused / freed
  lap(4);
  return 0;
}
}  // namespace

// ---- the GPU encoder (encode_kernel.hip) -------------------------------------------
namespace {
// 0 with *host false: *o holds the outputs; 0 with *host true: the host
// encoder takes the call (o->fallback says why); else an error code
int encode_gpu(OtlpBatchImpl* b, const ose_outputs* outs, bool sampled, bool tmpl, const Router* router,
               hipStream_t st, OtlpOut* o, bool* host, std::vector<uint64_t>* res_off = nullptr) {
  *host = true;
  if (b->e->option(Engine::kOptEncodeHost)) return 0;   // engine option encode_host: the host encoder always
  if (router && router->pipelines.size() > 63) return 0;   // the host encoder reports it
  const uint64_t n = b->cols.n_spans, S = b->cols.n_scopes, R = b->cols.n_resources;
  if (!b->d_spans) return 0;
  const uint32_t n_out = router ? (uint32_t)router->pipelines.size() + 1 : 1;
  const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (R + kEncTiles - 1) / kEncTiles);
  // workspace
  EncArgs a{};
  const size_t blob = router ? router->dev_blob.size() : 0;
  struct Part { void** dst; size_t bytes; };
  uint64_t* flags64 = nullptr;
  uint32_t *scope_span0 = nullptr, *res_scope0 = nullptr;
  uint64_t *scope_hdr = nullptr, *scope_schema = nullptr, *res_ref = nullptr;
  uint8_t* routes = nullptr;
  uint64_t* out_base = nullptr;
  std::vector<Part> parts = {
      {(void**)&a.span_out, 4 * n},
      {(void**)&a.scope_body, 8 * S},
      {(void**)&a.res_body, 8 * R},
      {(void**)&a.res_rec, 8 * R},
      {(void**)&a.res_mask, 8 * R},
      {(void**)&a.res_hdr, 8 * R},
      {(void**)&a.res_schema, 8 * R},
      {(void**)&flags64, 8},
      {(void**)&a.tile_sum, 16 * (size_t)n_out * tiles},
      {(void**)&a.off, 8 * (size_t)n_out * R},
      {(void**)&a.out_total, 16 * (size_t)n_out},
      {(void**)&out_base, 8 * (size_t)n_out},
  };
  if (tmpl) parts.push_back({(void**)&a.edit, sizeof(EncEdit) * n});
  if (blob) parts.push_back({(void**)&routes, blob});
  // the layout arrays the decoder left on the host go up
  const bool up_scopes = !b->scopes_dev, up_res = !b->res_on_device;
  if (up_scopes) {
    parts.push_back({(void**)&scope_span0, 4 * S});
    parts.push_back({(void**)&scope_hdr, 8 * S});
    parts.push_back({(void**)&scope_schema, 8 * S});
  }
  if (up_res) {
    parts.push_back({(void**)&res_ref, 8 * R});
    parts.push_back({(void**)&res_scope0, 4 * R});
  }
  size_t total = 0;
  for (auto& p : parts) total = up(total + p.bytes + 16);
  int rc;
  if ((rc = b->eslab.need(total))) return rc;
  size_t off = 0;
  for (auto& p : parts) {
    *p.dst = b->eslab.p + off;
    off = up(off + p.bytes + 16);
  }
  // host-side uploads through pinned staging: route table, layout, offsets
  size_t hbytes = 64 + 16 * (size_t)n_out + 8 * (size_t)n_out + 16 + blob + 16;
  if (up_scopes) hbytes += 20 * S + 64;
  if (up_res) hbytes += 12 * R + 64;
  if ((rc = b->emisc.need(hbytes))) return rc;
  uint8_t* h = b->emisc.p;
  size_t ho = up(64 + 16 * (size_t)n_out, 16);   // [0, 64): flags; then the totals
  auto upload = [&](void* dst, const void* src, size_t bytes) -> int {
    if (!bytes) return 0;
    std::memcpy(h + ho, src, bytes);
    HIP_TRY(hipMemcpyAsync(dst, h + ho, bytes, hipMemcpyHostToDevice, st));
    ho = up(ho + bytes, 16);
    return 0;
  };
  if (up_scopes && (b->lay.scope_span0.size() != S || b->lay.scope_hdr.size() != S || b->lay.scope_schema.size() != S))
    return 0;
  if (up_res && (b->lay.res_ref.size() != R || b->lay.res_scope0.size() != R)) return 0;
  if (blob && (rc = upload(routes, router->dev_blob.data(), blob))) return rc;
  if (up_scopes) {
    std::vector<uint32_t> s0(b->lay.scope_span0.begin(), b->lay.scope_span0.end());
    if ((rc = upload(scope_span0, s0.data(), 4 * S)) || (rc = upload(scope_hdr, b->lay.scope_hdr.data(), 8 * S)) ||
        (rc = upload(scope_schema, b->lay.scope_schema.data(), 8 * S)))
      return rc;
  }
  if (up_res &&
      ((rc = upload(res_ref, b->lay.res_ref.data(), 8 * R)) || (rc = upload(res_scope0, b->lay.res_scope0.data(), 4 * R))))
    return rc;
  a.pb = b->arena.p;
  a.n_spans = n;
  a.n_scopes = S;
  a.n_res = R;
  a.span_ref = b->d_spans;
  a.span_size = b->cols.span_size;
  a.keep = sampled ? outs->keep : nullptr;
  if (tmpl) {
    a.url_out = outs->url_out;
    a.tmpl = outs->tmpl;
    a.tmpl_arena = outs->tmpl_arena;
    a.tmpl_used = outs->tmpl_arena_used;
  }
  a.scope_span0 = up_scopes ? scope_span0 : b->d_span0;
  a.scope_hdr = up_scopes ? scope_hdr : b->d_hdr;
  a.scope_schema = up_scopes ? scope_schema : b->d_schema;
  a.scope_size = b->cols.scope_size;
  a.res_ref = up_res ? res_ref : b->d_res_ref;
  a.res_scope0 = up_res ? res_scope0 : b->d_res_scope0;
  a.res_size = b->cols.res_size;
  a.n_out = n_out;
  a.route_bits = router ? router->route_bits : 0;
  a.routes = reinterpret_cast<const EncRouteSlot*>(routes);
  a.route_keys = routes ? routes + router->dev_slots_bytes : nullptr;
  a.flags = reinterpret_cast<uint32_t*>(flags64);
  a.out_base = out_base;
  if ((n && !a.span_size) || (S && (!a.scope_span0 || !a.scope_hdr || !a.scope_schema || !a.scope_size)) ||
      (R && (!a.res_ref || !a.res_scope0 || !a.res_size)))
    return 0;
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  // sizing pass, offsets
  HIP_TRY(hipMemsetAsync(flags64, 0, 8, st));
  launch_enc_spans(a, st);
  HIP_TRY(hipGetLastError());
  launch_enc_scopes(a, st);
  HIP_TRY(hipGetLastError());
  launch_enc_resources(a, st);
  HIP_TRY(hipGetLastError());
  launch_enc_scan(a, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(h, flags64, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(h + 64, a.out_total, 16 * (size_t)n_out, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  uint32_t fb;
  std::memcpy(&fb, h, 4);
  o->fallback = fb;
  o->t_ms[1] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  t0 = clk::now();
  if (fb) return 0;
  std::vector<uint64_t> tot(2 * (size_t)n_out);
  std::memcpy(tot.data(), h + 64, 16 * (size_t)n_out);
  std::vector<uint64_t> base(n_out);
  uint64_t all = 0;
  for (uint32_t k = 0; k < n_out; k++) {
    base[k] = all;
    all = up(all + tot[k], 16);
  }
  if ((rc = b->eout.need(all + 16))) return rc;
  a.out = b->eout.p;
  if ((rc = upload(out_base, base.data(), 8 * (size_t)n_out))) return rc;
  // host buffers (pinned, pooled with the workspace)
  o->outs.assign(n_out, EncodedOutput{});
  bool oom = false;
  for (uint32_t k = 0; k < n_out; k++) {
    EncodedOutput& x = o->outs[k];
    x.name = router ? (k + 1 < n_out ? router->pipelines[k] : std::string("default")) : std::string();
    x.len = tot[k];
    x.n_resources = (uint32_t)tot[n_out + k];
    x.data = encode_work_pinned(*o->work, x.len, &x.cap);
    x.pinned = true;
    oom |= x.data == nullptr;
  }
  if (oom) return fail(OSE_EDEVICE, "out of pinned host memory for the encoder outputs");
  o->t_ms[2] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  t0 = clk::now();
  launch_enc_write(a, st);
  HIP_TRY(hipGetLastError());
  for (uint32_t k = 0; k < n_out; k++)
    if (tot[k]) HIP_TRY(hipMemcpyAsync(o->outs[k].data, a.out + base[k], tot[k], hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(h, flags64, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  std::memcpy(&fb, h, 4);
  if (fb & kEncFbWrite) return fail(OSE_EDEVICE, "GPU encoder: a record's bytes disagree with its size");
  if (res_off) {   // each output's offset of every resource's record (the scan the writer used)
    res_off->resize((size_t)n_out * R);
    if (R) HIP_TRY(hipMemcpy(res_off->data(), a.off, 8 * (size_t)n_out * R, hipMemcpyDeviceToHost));
  }
  o->t_ms[3] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  o->gpu = 1;
  *host = false;
  return 0;
}
}  // namespace

// The GPU encoder for the OTLP pipeline (otlp_pipeline.cpp): *out holds the
// batch's outputs and res_off every output's per-resource record offsets
// (n_out x R); *gpu false when the GPU encoder declined the batch (nothing
// in *out), the caller then takes its requests one by one.
int otlp_encode_gpu_offsets(Engine* e, ose_otlp_batch* bb, const ose_outputs* outs, uint32_t stages,
                            const Router* router, hipStream_t st, OtlpOut** out, std::vector<uint64_t>& res_off,
                            bool* gpu) {
  auto* b = reinterpret_cast<OtlpBatchImpl*>(bb);
  *gpu = false;
  *out = nullptr;
  auto* o = new OtlpOut();
  o->e = e;
  engine_retain(e);
  {
    std::lock_guard<std::mutex> g(e->mu);
    if (!e->enc_pool.empty()) {
      o->work = static_cast<EncodeWork*>(e->enc_pool.back());
      e->enc_pool.pop_back();
    }
  }
  if (!o->work) o->work = encode_work_new();
  const bool sampled = stages & (OSE_STAGE_SAMPLE | OSE_STAGE_APPLY_KEEP);
  const bool tmpl = stages & OSE_STAGE_TEMPLATE;
  bool host = true;
  const int rc = encode_gpu(b, outs, sampled, tmpl, router, st, o, &host, &res_off);
  if (rc || host) {
    otlp_out_release(o);
    return rc;
  }
  *gpu = true;
  *out = o;
  return 0;
}

}  // namespace ose

using namespace ose;

extern "C" {

int ose_otlp_decode(ose_engine* eng, const void* pb, size_t len, void* hip_stream, ose_otlp_batch** out) {
  if (!eng || (!pb && len) || !out) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (int rc = bind_device(e)) return rc;
  OtlpBatchImpl* b = nullptr;
  {
    // released batches keep their (grow-only) buffers: no allocation per call
    std::lock_guard<std::mutex> g(e->mu);
    if (!e->otlp_pool.empty()) {
      b = static_cast<OtlpBatchImpl*>(e->otlp_pool.back());
      e->otlp_pool.pop_back();
    }
  }
  if (!b) b = new OtlpBatchImpl();
  b->e = e;
  const int rc = decode(e, static_cast<const uint8_t*>(pb), len, static_cast<hipStream_t>(hip_stream), b);
  if (rc) {
    (void)hipStreamSynchronize(static_cast<hipStream_t>(hip_stream));   // no copy may outlive the buffers
    delete b;
    return rc;
  }
  engine_retain(e);
  *out = reinterpret_cast<ose_otlp_batch*>(b);
  return 0;
}

// Test seam (CPU): the structural walk alone, for a pipeline config
// {"odigossampling": ..., "odigosurltemplate": ..., "odigostrafficmetrics": ...};
// the arrays as JSON, NULL on an error (osehost_last_error)
char* osehost_otlp_walk(const char* cfg_json, const uint8_t* pb, size_t len) {
  try {
    Json cfg = parse_json(cfg_json);
    UrlTemplateConfig url;
    SamplingConfig sampling;
    TrafficMetricsConfig traffic;
    std::string err;
    const Json* ju = cfg.get("odigosurltemplate");
    const Json* js = cfg.get("odigossampling");
    const Json* jt = cfg.get("odigostrafficmetrics");
    if (ju && err.empty()) err = decode_url_config(*ju, url);
    if (js && err.empty()) err = decode_sampling_config(*js, sampling);
    if (jt && err.empty()) err = decode_traffic_config(*jt, traffic);
    ColumnizeCtx ctx;
    if (err.empty()) err = ctx.build(ju ? &url : nullptr, js ? &sampling : nullptr, jt ? &traffic : nullptr);
    Walked w;
    ResCache cache;
    const bool gpu_scopes = cfg.get("gpu_scopes") != nullptr;   // the walk ose_otlp_decode runs (ScopeSpans left to the GPU)
    if (cfg.get("warm") && err.empty()) {   // diagnostics: time a walk whose resource cache is filled
      Walked w0;
      if (!walk(ctx, cache, pb, len, w0, gpu_scopes)) err = w0.err;
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (err.empty() && !walk(ctx, cache, pb, len, w, gpu_scopes)) err = w.err;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (!err.empty()) { fail(OSE_EINVAL, err); return nullptr; }
    if (cfg.get("timing_only")) {   // diagnostics: the walk's wall time only
      std::string out = "{\"walk_ms\":" + std::to_string(ms) + ",\"spans\":" + std::to_string(w.span_ref.size()) + "}";
      char* r = static_cast<char*>(std::malloc(out.size() + 1));
      std::memcpy(r, out.c_str(), out.size() + 1);
      return r;
    }
    auto arr = [](const auto& v) {
      Json a = Json::array();
      for (auto x : v) a.push(Json::number(std::to_string((uint64_t)x)));
      return a;
    };
    Json o = Json::object();
    o.set("span_ref", arr(w.span_ref));
    o.set("span_res", arr(w.span_res));
    o.set("span_scope", arr(w.span_scope));
    o.set("res_svc", arr(w.res_svc));
    o.set("res_svc_str", arr(w.res_svc_str));
    o.set("res_attrset", arr(w.res_attrset));
    o.set("res_size", arr(w.res_size));
    o.set("res_ok", arr(w.res_ok));
    o.set("scope_size", arr(w.scope_size));
    o.set("scope_res", arr(w.scope_res));
    o.set("n_sets", Json::number(std::to_string(w.sets.size())));
    std::string out;
    dump_json(out, o);
    char* r = static_cast<char*>(std::malloc(out.size() + 1));
    std::memcpy(r, out.c_str(), out.size() + 1);
    return r;
  } catch (const std::exception& ex) {
    fail(OSE_EINVAL, ex.what());
    return nullptr;
  }
}

int ose_otlp_download(const ose_otlp_batch* bb, const ose_columns* dst) {
  if (!bb || !dst) return fail(OSE_EINVAL, "NULL argument");
  const auto* b = reinterpret_cast<const OtlpBatchImpl*>(bb);
  if (int rc = bind_device(b->e)) return rc;
  const ose_columns& c = b->cols;
  const uint64_t n = c.n_spans, R = c.n_resources, S = c.n_scopes, K = c.n_attr_keys;
  struct F { const void* src; void* dst; size_t bytes; };
  const F fs[] = {
      {c.arena, (void*)dst->arena, c.arena_bytes}, {c.trace_id, (void*)dst->trace_id, 16 * n},
      {c.start_ns, (void*)dst->start_ns, 8 * n}, {c.end_ns, (void*)dst->end_ns, 8 * n},
      {c.status, (void*)dst->status, n}, {c.kind, (void*)dst->kind, n}, {c.resource, (void*)dst->resource, 4 * n},
      {c.scope, (void*)dst->scope, 4 * n}, {c.url_flags, (void*)dst->url_flags, n}, {c.path, (void*)dst->path, 8 * n},
      {c.route, (void*)dst->route, 8 * n}, {c.span_size, (void*)dst->span_size, 4 * n},
      {c.name_len, (void*)dst->name_len, 4 * n}, {c.attr_match, (void*)dst->attr_match, 8 * n * std::max<uint32_t>(1, c.attr_match_words)},
      {c.res_svc, (void*)dst->res_svc, 4 * R}, {c.res_svc_str, (void*)dst->res_svc_str, 4 * R},
      {c.res_url_ok, (void*)dst->res_url_ok, R}, {c.res_attrset, (void*)dst->res_attrset, 4 * R},
      {c.res_size, (void*)dst->res_size, 4 * R}, {c.scope_size, (void*)dst->scope_size, 4 * S},
      {c.scope_resource, (void*)dst->scope_resource, 4 * S}, {c.attr_type, (void*)dst->attr_type, K * n},
      {c.attr_val, (void*)dst->attr_val, 8 * K * n},
  };
  for (auto& f : fs)
    if (f.src && f.dst && f.bytes) HIP_TRY(hipMemcpy(f.dst, f.src, f.bytes, hipMemcpyDefault));
  return 0;
}

const ose_columns* ose_otlp_columns(const ose_otlp_batch* bb) {
  return bb ? &reinterpret_cast<const OtlpBatchImpl*>(bb)->cols : nullptr;
}

int ose_otlp_timings(const ose_otlp_batch* bb, double* ms5) {
  if (!bb || !ms5) return fail(OSE_EINVAL, "NULL argument");
  std::memcpy(ms5, reinterpret_cast<const OtlpBatchImpl*>(bb)->t_ms, sizeof(double) * 5);
  return 0;
}

uint32_t ose_otlp_host_spans(const ose_otlp_batch* bb) {
  return bb ? reinterpret_cast<const OtlpBatchImpl*>(bb)->host_spans : 0;
}

int ose_otlp_attrset(const ose_otlp_batch* bb, uint32_t k, char* json, size_t cap) {
  if (!bb || !json) return fail(OSE_EINVAL, "NULL argument");
  const auto* b = reinterpret_cast<const OtlpBatchImpl*>(bb);
  if (k >= b->attrsets.size()) return fail(OSE_EINVAL, "attribute set index out of range");
  Json o = Json::object();
  for (auto& kv : b->attrsets[k]) o.set(kv.first, Json::str(kv.second));
  std::string s;
  dump_json(s, o);
  if (s.size() + 1 > cap) return fail(OSE_ERANGE, "buffer too small");
  std::memcpy(json, s.c_str(), s.size() + 1);
  return 0;
}

namespace {
int encode_threads() { return parallel_width(); }
}  // namespace

int ose_otlp_encode(ose_engine* eng, const ose_otlp_batch* bb, const ose_outputs* outs, uint32_t stages,
                    uint32_t group_mode, const ose_router* router, void* hip_stream, ose_otlp_out** out) {
  if (!eng || !bb || !out) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  auto* b = const_cast<OtlpBatchImpl*>(reinterpret_cast<const OtlpBatchImpl*>(bb));
  if (b->e != e) return fail(OSE_EINVAL, "the batch belongs to another engine");
  if (int rc = bind_device(e)) return rc;
  const bool batch_mode = (stages & OSE_STAGE_SAMPLE) && group_mode == OSE_GROUP_BATCH;
  const bool sampled = (stages & (OSE_STAGE_SAMPLE | OSE_STAGE_APPLY_KEEP)) && !batch_mode;
  const bool tmpl = stages & OSE_STAGE_TEMPLATE;
  if ((sampled || batch_mode || tmpl) && !outs) return fail(OSE_EINVAL, "NULL outputs");
  if (sampled && !outs->keep) return fail(OSE_EINVAL, "keep is NULL");
  if (batch_mode && !outs->trace_keep) return fail(OSE_EINVAL, "trace_keep is NULL");
  if (tmpl && (!outs->url_out || !outs->tmpl || !outs->tmpl_arena || !outs->tmpl_arena_used))
    return fail(OSE_EINVAL, "template outputs are NULL");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  const auto t_start = std::chrono::steady_clock::now();
  const uint64_t n = b->cols.n_spans;
  uint32_t gpu_fallback = 0;
  if (!batch_mode) {   // the GPU encoder (OSE_GROUP_BATCH's all-or-nothing stays with the host)
    auto* o = new OtlpOut();
    o->e = e;
    engine_retain(e);   // dropped by otlp_out_release
    {
      std::lock_guard<std::mutex> g(e->mu);
      if (!e->enc_pool.empty()) {
        o->work = static_cast<EncodeWork*>(e->enc_pool.back());
        e->enc_pool.pop_back();
      }
    }
    if (!o->work) o->work = encode_work_new();
    bool host = true;
    const int rc = encode_gpu(b, outs, sampled, tmpl, reinterpret_cast<const Router*>(router), st, o, &host);
    if (rc || host) {
      gpu_fallback = o->fallback;
      otlp_out_release(o);   // pinned buffers taken before a failure go back to the work's pool
      if (rc) return rc;
    } else {
      *out = reinterpret_cast<ose_otlp_out*>(o);
      return 0;
    }
  }
  // the decisions and the decoder's span sizes, D2H into the batch's pinned staging
  const size_t o_keep = 0, o_url = up(n + 16), o_tmpl = o_url + up(n + 16), o_size = o_tmpl + up(8 * n + 16),
               o_misc = o_size + up(4 * n + 16), o_arena = o_misc + 256;
  int rc;
  if ((rc = b->stage.need(o_arena))) return rc;
  uint8_t* h = b->stage.p;
  if (n) HIP_TRY(hipMemcpyAsync(h + o_size, b->cols.span_size, 4 * n, hipMemcpyDeviceToHost, st));
  if (sampled && n) HIP_TRY(hipMemcpyAsync(h + o_keep, outs->keep, n, hipMemcpyDefault, st));
  if (batch_mode) HIP_TRY(hipMemcpyAsync(h + o_misc + 8, outs->trace_keep, 1, hipMemcpyDefault, st));
  if (tmpl) {
    if (n) HIP_TRY(hipMemcpyAsync(h + o_url, outs->url_out, n, hipMemcpyDefault, st));
    if (n) HIP_TRY(hipMemcpyAsync(h + o_tmpl, outs->tmpl, 8 * n, hipMemcpyDefault, st));
    HIP_TRY(hipMemcpyAsync(h + o_misc, outs->tmpl_arena_used, 8, hipMemcpyDefault, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  uint64_t used = 0;
  if (tmpl) {
    std::memcpy(&used, h + o_misc, 8);
    if (used > outs->tmpl_arena_cap) return fail(OSE_ERANGE, "tmpl_arena_used beyond tmpl_arena_cap");
    if (used) {
      if ((rc = b->stage.need(o_arena + used))) return rc;   // grow-only: earlier contents are lost
      h = b->stage.p;
      if (n) HIP_TRY(hipMemcpyAsync(h + o_size, b->cols.span_size, 4 * n, hipMemcpyDeviceToHost, st));
      if (sampled && n) HIP_TRY(hipMemcpyAsync(h + o_keep, outs->keep, n, hipMemcpyDefault, st));
      if (n) HIP_TRY(hipMemcpyAsync(h + o_url, outs->url_out, n, hipMemcpyDefault, st));
      if (n) HIP_TRY(hipMemcpyAsync(h + o_tmpl, outs->tmpl, 8 * n, hipMemcpyDefault, st));
      if (batch_mode) HIP_TRY(hipMemcpyAsync(h + o_misc + 8, outs->trace_keep, 1, hipMemcpyDefault, st));
      HIP_TRY(hipMemcpyAsync(h + o_arena, outs->tmpl_arena, used, hipMemcpyDefault, st));
      HIP_TRY(hipStreamSynchronize(st));
    }
  }
  EncodeDecisions d;
  d.keep = sampled ? h + o_keep : nullptr;
  d.drop_all = batch_mode && !h[o_misc + 8];
  if (tmpl) {
    d.url_out = h + o_url;
    d.tmpl = reinterpret_cast<const ose_strref*>(h + o_tmpl);
    d.tmpl_arena = h + o_arena;
    d.tmpl_arena_len = used;
  }
  d.span_size = reinterpret_cast<const uint32_t*>(h + o_size);
  if ((rc = layout_to_host(b, st))) return rc;
  auto* o = new OtlpOut();
  o->e = e;
  engine_retain(e);   // dropped by otlp_out_release
  {
    std::lock_guard<std::mutex> g(e->mu);
    if (!e->enc_pool.empty()) {
      o->work = static_cast<EncodeWork*>(e->enc_pool.back());
      e->enc_pool.pop_back();
    }
  }
  if (!o->work) o->work = encode_work_new();
  o->fallback = gpu_fallback;
  o->t_ms[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  std::string err;
  if (!encode_traces(b->pb, b->pb_len, b->span_ref, b->lay, d, reinterpret_cast<const Router*>(router),
                     encode_threads(), *o->work, o->outs, err, o->t_ms + 1)) {
    otlp_out_release(o);
    return fail(OSE_EINVAL, err);
  }
  *out = reinterpret_cast<ose_otlp_out*>(o);
  return 0;
}

// Test seam (CPU): the encoder on the host walk of `pb` with the given
// decisions (keep / url_out / tmpl NULL when absent) and span sizes
// computed on the host as the decoder would.
int osehost_otlp_encode(const uint8_t* pb, size_t len, const uint8_t* keep, int drop_all, const uint8_t* url_out,
                        const ose_strref* tmpl, const uint8_t* tmpl_arena, uint64_t tmpl_arena_len,
                        const ose_router* router, int threads, ose_otlp_out** out) {
  if ((!pb && len) || !out) return fail(OSE_EINVAL, "NULL argument");
  ColumnizeCtx ctx;
  std::string err = ctx.build(nullptr, nullptr, nullptr);
  Walked w;
  ResCache cache;
  if (err.empty() && !walk(ctx, cache, pb, len, w)) err = w.err;
  if (!err.empty()) return fail(OSE_EINVAL, err);
  std::vector<uint32_t> sizes(w.span_ref.size());
  ProtoSizer sizer;
  for (size_t i = 0; i < sizes.size(); i++) {
    Span sp;
    if (!pb_span(pb + (uint32_t)w.span_ref[i], (size_t)(w.span_ref[i] >> 32), sp))
      return fail(OSE_EINVAL, "OTLP protobuf: malformed Span");
    sizes[i] = (uint32_t)sizer.span(sp);
  }
  EncodeDecisions d;
  d.keep = keep;
  d.drop_all = drop_all != 0;
  d.url_out = url_out;
  d.tmpl = tmpl;
  d.tmpl_arena = tmpl_arena;
  d.tmpl_arena_len = tmpl_arena_len;
  d.span_size = sizes.data();
  auto* o = new OtlpOut();
  o->work = encode_work_new();
  if (!encode_traces(pb, len, w.span_ref, w.lay, d, reinterpret_cast<const Router*>(router),
                     threads > 0 ? threads : encode_threads(), *o->work, o->outs, err, o->t_ms + 1)) {
    otlp_out_release(o);
    return fail(OSE_EINVAL, err);
  }
  *out = reinterpret_cast<ose_otlp_out*>(o);
  return 0;
}

void ose_otlp_release(ose_otlp_batch* bb) {
  if (!bb) return;
  LastErrorScope keep("ose_otlp_release");
  auto* b = reinterpret_cast<OtlpBatchImpl*>(bb);
  Engine* e = b->e;
  (void)bind_device(e);
  bool pooled = false;
  if (!e->closed.load()) {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->otlp_pool.size() < 16) {
      e->otlp_pool.push_back(b);
      pooled = true;
    }
  }
  if (!pooled) delete b;
  engine_unref(e);
}

}  // extern "C"
