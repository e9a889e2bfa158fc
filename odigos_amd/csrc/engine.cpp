// engine.cpp — the C ABI (include/odigos_amd.h): config decoding/validation,
// compilation of the read-only device tables, workspaces, kernel launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/odigos_amd.h"
#include "config.hpp"
#include "devcfg.hpp"
#include "engine_internal.hpp"
#include "kernels.hpp"
#include "blob.hpp"
#include "regex_dfa.hpp"

namespace ose {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// odigosurltemplate tables: newUrlTemplateProcessor (processor.go:27-69)
// groups rules by segment count keeping config order; custom ids default
// their name to "id".
int build_url_blob(const UrlTemplateConfig& c, std::vector<uint8_t>& out, uint32_t& max_name) {
  Blob bl;
  UrlCfgDev h{};
  bl.put(&h, 1);
  std::string bytes;
  std::vector<NameDev> names;
  auto add_text = [&](const std::string& s) {
    NameDev n{(uint32_t)bytes.size(), (uint32_t)s.size()};
    bytes += s;
    return n;
  };
  names.push_back(add_text("id"));
  names.push_back(add_text("date"));
  names.push_back(add_text("email"));
  std::vector<Dfa> dfas;
  auto compile = [&](const std::string& rx, int32_t& idx) -> int {
    Dfa d;
    std::string err;
    RegexStatus st = compile_dfa(rx, d, err);
    if (st == RegexStatus::Syntax) return fail(OSE_EINVAL, err);
    if (st != RegexStatus::Ok) return fail(OSE_ENOTSUP, "regexp not supported by the DFA compiler: " + err);
    idx = (int32_t)dfas.size();
    dfas.push_back(std::move(d));
    return 0;
  };
  std::vector<UrlCustomDev> custom;
  for (auto& ci : c.custom_ids) {
    UrlCustomDev cd{};
    int rc = compile(ci.regexp, cd.dfa);
    if (rc) return rc;
    cd.name = (uint32_t)names.size();
    names.push_back(add_text(ci.template_name.empty() ? "id" : ci.template_name));
    custom.push_back(cd);
  }
  struct ParsedRule { uint32_t nseg; size_t order; std::vector<RuleSegment> segs; };
  std::vector<ParsedRule> rules;
  for (size_t k = 0; k < c.templatization_rules.size(); k++) {
    ParsedRule pr;
    std::string e = parse_user_rule(c.templatization_rules[k], pr.segs);
    if (!e.empty()) return fail(OSE_EINVAL, e);
    pr.nseg = (uint32_t)pr.segs.size();
    pr.order = k;
    rules.push_back(std::move(pr));
  }
  std::stable_sort(rules.begin(), rules.end(), [](const ParsedRule& a, const ParsedRule& b) { return a.nseg < b.nseg; });
  uint32_t longest = 0;
  for (auto& r : rules) longest = std::max(longest, r.nseg);
  // by_len[n] for n <= longest + 1 (a path with more segments than the longest rule tries none)
  std::vector<uint32_t> by_len(longest + 2, 0);
  std::vector<UrlRuleDev> rdev;
  std::vector<UrlRuleSegDev> sdev;
  uint32_t max_nseg = 0;
  for (auto& r : rules) {
    rdev.push_back(UrlRuleDev{r.nseg, (uint32_t)sdev.size()});
    max_nseg = std::max(max_nseg, r.nseg);
    for (auto& s : r.segs) {
      UrlRuleSegDev sd{};
      sd.dfa = -1;
      switch (s.kind) {
        case SegKind::Static: sd.kind = kRuleStatic; break;
        case SegKind::Wildcard: sd.kind = kRuleWildcard; break;
        case SegKind::Template: sd.kind = kRuleTemplate; break;
        case SegKind::Regex: sd.kind = kRuleRegex; break;
      }
      NameDev t = add_text(s.text);
      sd.text_off = t.off;
      sd.text_len = t.len;
      if (s.has_regexp) {
        int rc = compile(s.regexp, sd.dfa);
        if (rc) return rc;
      }
      sdev.push_back(sd);
    }
  }
  // by_len[n] = first rule with nseg >= n
  for (uint32_t n = 0; n <= longest + 1; n++) {
    uint32_t k = 0;
    while (k < rules.size() && rules[k].nseg < n) k++;
    by_len[n] = k;
  }
  max_name = 0;
  for (auto& n : names) max_name = std::max(max_name, n.len);
  h.n_custom = (uint32_t)custom.size();
  h.n_rules = (uint32_t)rdev.size();
  h.n_names = (uint32_t)names.size();
  h.n_dfa = (uint32_t)dfas.size();
  h.max_rule_nseg = max_nseg;
  h.max_name_len = max_name;
  h.rules_by_len_off = bl.put(by_len.data(), by_len.size());
  h.rules_off = bl.put(rdev.data(), rdev.size());
  h.segs_off = bl.put(sdev.data(), sdev.size());
  h.custom_off = bl.put(custom.data(), custom.size());
  h.names_off = bl.put(names.data(), names.size());
  std::vector<uint32_t> dfa_offs;
  for (auto& d : dfas) dfa_offs.push_back(put_dfa(bl, d));
  h.dfa_off = bl.put(dfa_offs.data(), dfa_offs.size());
  h.bytes_off = bl.put(bytes.data(), bytes.size());
  bl.align();
  if (bl.overflow) return fail(OSE_ENOTSUP, "odigosurltemplate device tables exceed 4 GiB (the regexps' DFAs together)");
  bl.b.resize(bl.b.size() + 16, 0);
  h.total_bytes = (uint32_t)bl.b.size();
  std::memcpy(bl.b.data(), &h, sizeof h);
  out = std::move(bl.b);
  return 0;
}

// ---------------- engine ----------------
Engine::~Engine() {
  release_exchange_scratch(this);
  release_batch_pool(this);
  release_otlp(this);
  release_encode(this);
  for (auto& t : timed) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
  for (auto s : streams) (void)hipStreamDestroy(s);
  for (auto ev : event_pool) (void)hipEventDestroy(ev);
  if (url_blob_dev) (void)hipFree(url_blob_dev);
  for (auto* d : sampling_chunks_dev)
    if (d) (void)hipFree(d);   // (sampling_blob_dev is the first)
  for (auto* d : sampling_svc_map_dev)
    if (d) (void)hipFree(d);
  if (sampling_svc_maps_dev) (void)hipFree(sampling_svc_maps_dev);
  if (shard_tables_dev) (void)hipFree(shard_tables_dev);
  if (path_count_dev) (void)hipFree(path_count_dev);
  if (attr_blob_dev) (void)hipFree(attr_blob_dev);
  if (attr_host_mask_dev) (void)hipFree(attr_host_mask_dev);
  for (auto* w : pool) {
    if (w->dev) (void)hipFree(w->dev);
    if (w->table) (void)hipFree(w->table);
    if (w->dup_bkt) (void)hipFree(w->dup_bkt);
    if (w->dup_bkt_count) (void)hipFree(w->dup_bkt_count);
    if (w->runs) (void)hipFree(w->runs);
    if (w->run_count) (void)hipFree(w->run_count);
    if (w->attr_bits) (void)hipFree(w->attr_bits);
    if (w->ep_planes) (void)hipFree(w->ep_planes);
    if (w->svc_local) (void)hipFree(w->svc_local);
    for (void* f : w->fold)
      if (f) (void)hipFree(f);
    if (w->pending) (void)hipEventDestroy(w->pending);
    if (w->dup_host) (void)hipHostFree(w->dup_host);
    if (w->dup_ready) (void)hipEventDestroy(w->dup_ready);
    if (w->fork) (void)hipEventDestroy(w->fork);
    if (w->join) (void)hipEventDestroy(w->join);
    delete w;
  }
}

hipEvent_t Engine::take_event() {
  if (!event_pool.empty()) {
    hipEvent_t ev = event_pool.back();
    event_pool.pop_back();
    return ev;
  }
  hipEvent_t ev = nullptr;
  (void)hipEventCreate(&ev);
  return ev;
}
void Engine::prof_begin(const char* name, hipStream_t st, Timed& t) {
  if (!profiling) return;
  std::lock_guard<std::mutex> g(mu);
  t.name = name;
  t.a = take_event();
  t.b = take_event();
  (void)hipEventRecord(t.a, st);
}
void Engine::prof_end(Timed& t, hipStream_t st) {
  if (!profiling || !t.a) return;
  (void)hipEventRecord(t.b, st);
  std::lock_guard<std::mutex> g(mu);
  timed.push_back(t);
}

// True while `st` is being captured into a hipGraph.
bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Stream-ordered pool: work enqueued on a workspace may still be running
// when the call returns (ose_process_device is asynchronous), so release
// records an event on the caller's stream and the next user of that
// workspace makes its own stream wait for it.  A call captured into a
// hipGraph takes a workspace out of the pool for good: the graph replays
// into it whenever it is launched, so no later call may share it (and no
// event recorded outside the capture may be waited on inside it).
Workspace* Engine::acquire_ws(hipStream_t st) {
  if (stream_capturing(st)) {
    std::lock_guard<std::mutex> g(mu);
    Workspace* w = nullptr;
    if (!free_ws.empty()) {   // the largest free one (ose_reserve sized it)
      auto it = std::max_element(free_ws.begin(), free_ws.end(),
                                 [](const Workspace* a, const Workspace* b) { return a->cap < b->cap; });
      w = *it;
      free_ws.erase(it);
    } else {
      w = new Workspace();
      pool.push_back(w);
    }
    w->captured = true;
    return w;
  }
  Workspace* w = nullptr;
  {
    std::lock_guard<std::mutex> g(mu);
    if (!free_ws.empty()) {
      w = free_ws.back();
      free_ws.pop_back();
    } else {
      w = new Workspace();
      pool.push_back(w);
    }
  }
  if (w->pending_set) (void)hipStreamWaitEvent(st, w->pending, 0);
  return w;
}
// A workspace taken for a capture that queued nothing goes back to the pool.
void Engine::return_unused_ws(Workspace* w) {
  std::lock_guard<std::mutex> g(mu);
  w->captured = false;
  free_ws.push_back(w);
}
void Engine::release_ws(Workspace* w, hipStream_t st) {
  if (w->captured) return;   // owned by the graph it was captured into
  if (!w->pending) (void)hipEventCreateWithFlags(&w->pending, hipEventDisableTiming);
  w->pending_set = w->pending && hipEventRecord(w->pending, st) == hipSuccess;
  std::lock_guard<std::mutex> g(mu);
  free_ws.push_back(w);
}
hipStream_t Engine::take_stream() {
  std::lock_guard<std::mutex> g(mu);
  if (!free_streams.empty()) {
    hipStream_t s = free_streams.back();
    free_streams.pop_back();
    return s;
  }
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams.push_back(s);
  return s;
}
void Engine::give_stream(hipStream_t s) {
  std::lock_guard<std::mutex> g(mu);
  free_streams.push_back(s);
}

int Workspace::reserve(size_t bytes) {
  if (bytes <= cap) return 0;
  if (captured) return fail(OSE_ENOMEM, "workspace too small inside a hipGraph capture: call ose_reserve first");
  if (dev) HIP_TRY(hipFree(dev));
  dev = nullptr;
  cap = 0;
  size_t want = std::max<size_t>(bytes, 1 << 20);
  HIP_TRY(hipMalloc(&dev, want));
  cap = want;
  return 0;
}

int ensure_device() {
  static int status = 1;   // 1 = unknown
  static std::mutex m;
  std::lock_guard<std::mutex> g(m);
  if (status == 1) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    status = (e == hipSuccess && n > 0) ? 0 : OSE_EDEVICE;
  }
  if (status) return fail(OSE_EDEVICE, "no HIP device visible: the odigos_amd engine runs only on an MI355X (gfx950)");
  return 0;
}

int bind_device(const Engine* e) {
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != e->device) HIP_TRY(hipSetDevice(e->device));
  return 0;
}

static std::mutex g_dropped_mu;
static uint64_t g_dropped_count = 0;
static std::string g_dropped_last;
void note_dropped_error(const char* where, hipError_t err) {
  std::lock_guard<std::mutex> g(g_dropped_mu);
  g_dropped_count++;
  g_dropped_last = std::string(where) + ": " + hipGetErrorName(err) + " (" + hipGetErrorString(err) + ")";
}

void engine_retain(Engine* e) { e->refs.fetch_add(1, std::memory_order_relaxed); }

void engine_unref(Engine* e) {
  if (e->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  LastErrorScope keep("engine_unref");
  (void)bind_device(e);
  (void)hipDeviceSynchronize();   // nothing in flight may still use the buffers freed below
  delete e;
}

int upload(const std::vector<uint8_t>& host, uint8_t** dev) {
  HIP_TRY(hipMalloc(dev, host.size()));
  HIP_TRY(hipMemcpy(*dev, host.data(), host.size(), hipMemcpyHostToDevice));
  return 0;
}

// Workspace layout for one call (byte offsets), see run_stages.
static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int run_url_back(Engine* e, const UrlKernelArgs& a, hipStream_t st);

// ws_off: the URL scratch starts this many bytes into the workspace (past a
// SAMPLE stage's scratch whose slow path is still to be queued).  front: only
// plan, plan_slow, scan and emit_slow are queued, and the arguments of the
// rest go to *front (run_url_back queues url_copy, fused with
// odigostrafficmetrics' spans pass when front->fuse_size is set).
int run_url(Engine* e, const ose_columns* c, const ose_outputs* o, hipStream_t st, Workspace* ws, size_t ws_off = 0,
            UrlKernelArgs* front = nullptr, bool refs = false, uint32_t grid_mult = 1) {
  if (!e->has_url) return fail(OSE_EINVAL, "odigosurltemplate is not configured on this engine");
  if (!c->url_flags || !c->kind || !c->path || !c->arena || !o->url_out || !o->tmpl || !o->tmpl_arena)
    return fail(OSE_EINVAL, "TEMPLATE stage needs url_flags, kind, path, arena, url_out, tmpl, tmpl_arena");
  if (e->url_needs_resource && (!c->resource || !c->res_url_ok))
    return fail(OSE_EINVAL, "include/exclude configured: resource and res_url_ok columns are required");
  if (c->res_url_ok && !c->resource) return fail(OSE_EINVAL, "res_url_ok needs the resource column");
  if (o->tmpl_arena_cap > 0xFFFFFFFFull) return fail(OSE_ERANGE, "tmpl_arena_cap exceeds the 32-bit offset range");
  uint64_t n = c->n_spans;
  const uint32_t groups = (uint32_t)((n + kUrlGroup - 1) / kUrlGroup);
  // workspace: [0,16) scan counter, slow count, error, unplanned count | [16,24) refs bump | [24,32) refs
  // slow groups aligned | scan status 8t
  // (all zeroed by one memset) | plan_len 4n | plan_meta 4n | plan_code 8n | group_sum 8g | group_base 8g | group_scr 8g |
  // slow groups 4g | unplanned groups 4g | dbg | scratch (the assembled group images)
  const uint32_t scan_tiles = (groups + kUrlScanTile - 1) / kUrlScanTile;
  const size_t off_bump = 16, off_asum = 24, off_sst = 32, zero_bytes = off_sst + 8 * (size_t)scan_tiles;
  const size_t off_len = align_up(zero_bytes, 256), off_meta = off_len + 4 * n;
  const size_t off_code = align_up(off_meta + 4 * n, 8);
  const size_t off_gsum = off_code + 8 * n, off_gbase = off_gsum + 8 * (size_t)groups;
  const size_t off_gscr = off_gbase + 8 * (size_t)groups;
  const size_t off_slow = off_gscr + 8 * (size_t)groups;
  const size_t off_unpl = off_slow + 4 * (size_t)groups;
  const size_t off_dbg = align_up(off_unpl + 4 * (size_t)groups, 256);
  const size_t off_scr = off_dbg + 256;
  const size_t scr_bytes = url_scratch_bytes(n, c->arena_bytes);
  const size_t need = off_scr + (refs ? 0 : scr_bytes);   // refs: the images go to tmpl_arena itself
  if (need > url_workspace_bytes(n, c->arena_bytes))
    return fail(OSE_EINVAL, "internal: URL workspace layout exceeds its bound");
  int rc = ws->reserve(ws_off + need);
  if (rc) return rc;
  uint8_t* base = static_cast<uint8_t*>(ws->dev) + ws_off;
  UrlKernelArgs a{};
  a.n_spans = n;
  a.n_groups = groups;
  a.arena = c->arena;
  a.url_flags = c->url_flags;
  a.kind = c->kind;
  a.resource = c->resource;
  a.res_url_ok = c->res_url_ok;   // NULL: every resource passes (no include/exclude)
  a.path = c->path;
  a.url_out = o->url_out;
  a.tmpl = o->tmpl;
  a.out_arena = o->tmpl_arena;
  a.out_cap = o->tmpl_arena_cap;
  a.cfg = e->url_blob_dev;
  a.general = (!e->url.custom_ids.empty() || !e->url.templatization_rules.empty()) ? 1u : 0u;
  a.plan_len = reinterpret_cast<uint32_t*>(base + off_len);
  a.plan_meta = reinterpret_cast<uint32_t*>(base + off_meta);
  a.plan_code = reinterpret_cast<uint64_t*>(base + off_code);
  a.group_sum = reinterpret_cast<uint64_t*>(base + off_gsum);
  a.group_base = reinterpret_cast<uint64_t*>(base + off_gbase);
  a.group_scr = reinterpret_cast<uint64_t*>(base + off_gscr);
  a.scratch = base + off_scr;
  if (refs) {
    a.refs = 1;
    a.scratch = o->tmpl_arena;
    a.bump = reinterpret_cast<uint64_t*>(base + off_bump);
    a.slow_aligned = reinterpret_cast<uint64_t*>(base + off_asum);
  }
  a.n_scan_tiles = scan_tiles;
  a.scan_counter = reinterpret_cast<uint32_t*>(base);
  a.scan_status = reinterpret_cast<uint64_t*>(base + off_sst);
  a.error = o->device_status ? o->device_status : reinterpret_cast<uint32_t*>(base + 8);
  a.slow_count = reinterpret_cast<uint32_t*>(base + 4);
  a.slow_groups = reinterpret_cast<uint32_t*>(base + off_slow);
  a.unplanned_count = reinterpret_cast<uint32_t*>(base + 12);
  a.unplanned = reinterpret_cast<uint32_t*>(base + off_unpl);
  HIP_TRY(hipMemsetAsync(base, 0, zero_bytes, st));
  a.used = o->tmpl_arena_used;
#if OSE_DIAG
  if (const char* ab = getenv("OSE_URL_ABLATE")) a.ablate = (uint32_t)strtoul(ab, nullptr, 0);   // tools/ablate_url.py
#endif
  a.plan_grid_mult = refs ? grid_mult : 1u;
  a.scr_region = (scr_bytes / std::max<uint32_t>(1, url_plan_waves(a))) & ~15ull;
  // refs: image chunks of an eighth of the arena over the plan waves (at most
  // 256 KiB; a group larger than a chunk takes exactly its size): a wave
  // leaves at most one chunk's tail unused (url_refs_chunk)
  a.plan_waves = url_plan_waves(a);
  a.refs_chunk = url_refs_chunk(o->tmpl_arena_cap, a.plan_waves);
  if (front) *front = a;
  if (n == 0) {
    if (o->tmpl_arena_used) HIP_TRY(hipMemsetAsync(o->tmpl_arena_used, 0, 8, st));
    return 0;
  }
  if (a.ablate & 512) {   // diagnostics: per-section shader clocks (tools/url_clocks.py)
    a.dbg = reinterpret_cast<uint64_t*>(base + off_dbg);
    HIP_TRY(hipMemsetAsync(a.dbg, 0, 256, st));
  }
  Engine::Timed tm{};
  e->prof_begin("url_plan_kernel", st, tm);
  launch_url_plan(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  e->prof_begin("url_plan_slow_kernel", st, tm);
  launch_url_plan_slow(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  e->prof_begin("url_scan_kernel", st, tm);
  launch_url_scan(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  // the groups url_plan_kernel did not assemble, written at their scanned
  // bases: nothing here reads SAMPLE's keep bytes or url_copy_kernel's
  // output, so it runs with the front (beside the trace stage when the
  // URL front has its own stream)
  e->prof_begin("url_emit_slow_kernel", st, tm);
  launch_url_emit_slow(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  if (front) {
    *front = a;
    return 0;
  }
  return run_url_back(e, a, st);
}

int run_url_back(Engine* e, const UrlKernelArgs& a, hipStream_t st) {
  if (a.n_spans == 0) return 0;
  Engine::Timed tm{};
  e->prof_begin("url_copy_kernel", st, tm);
  launch_url_copy(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  if (a.ablate & 512) {
    uint64_t h[16];
    uint32_t cnt[4];
    HIP_TRY(hipMemcpyAsync(h, a.dbg, sizeof h, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(cnt, a.scan_counter, sizeof cnt, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const double wp = h[3] ? (double)h[3] : 1.0, we = h[6] ? (double)h[6] : 1.0;
    (void)we;
    fprintf(stderr, "url clocks/wave: plan[stage %.0f bitmaps %.0f plan %.0f assemble+store %.0f]\n", h[0] / wp,
            h[1] / wp, h[2] / wp, h[5] / wp);
    fprintf(stderr, "url plan list clocks/wave: enumerate %.0f classify %.0f fold %.0f\n", h[13] / wp, h[14] / wp,
            h[15] / wp);
    fprintf(stderr, "url groups: %llu, slow (K3s) %u, unplanned (K1b) %u\n", (unsigned long long)((a.n_spans + 63) / 64),
            cnt[1], cnt[3]);
    fprintf(stderr, "url_plan_slow_kernel slowest block clocks: config %llu whole %llu plan_path %llu\n",
            (unsigned long long)h[8], (unsigned long long)h[9], (unsigned long long)h[10]);
  }
  return 0;
}

int run_stages(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t mask, uint32_t group_mode,
               const ose_rand* rnd, hipStream_t st) {
  if (!c || !o) return fail(OSE_EINVAL, "columns and outputs are required");
  if (mask & ~(OSE_STAGE_SAMPLE | OSE_STAGE_TEMPLATE | OSE_STAGE_SIZE | OSE_STAGE_APPLY_KEEP | OSE_STAGE_TEMPLATE_REFS |
               OSE_STAGE_APPLY_TEMPLATE))
    return fail(OSE_EINVAL, "unknown stage bit");
  if ((mask & OSE_STAGE_TEMPLATE_REFS) && !(mask & OSE_STAGE_TEMPLATE))
    return fail(OSE_EINVAL, "OSE_STAGE_TEMPLATE_REFS needs OSE_STAGE_TEMPLATE");
  if ((mask & OSE_STAGE_APPLY_KEEP) && (mask & OSE_STAGE_SAMPLE))
    return fail(OSE_EINVAL, "OSE_STAGE_APPLY_KEEP and OSE_STAGE_SAMPLE exclude each other");
  if ((mask & OSE_STAGE_APPLY_TEMPLATE) && (mask & OSE_STAGE_TEMPLATE))
    return fail(OSE_EINVAL, "OSE_STAGE_APPLY_TEMPLATE and OSE_STAGE_TEMPLATE exclude each other");
  // SAMPLE + TEMPLATE by trace id: the URL stage reads nothing SAMPLE writes,
  // so its launches are queued between SAMPLE's fast path and the rest of
  // SAMPLE, which is queued once the host has read the fast path's dup flag
  // (by then the GPU is busy with the URL kernels, and the ~12 gated
  // slow-path launches are skipped when no trace id repeats)
  // SAMPLE without TEMPLATE: the host waits for the fast path right away (an
  // idle gap of one launch latency instead of ~12 gated launches)
  // Inside a hipGraph capture the host can neither wait nor decide: the
  // trace-id stage keeps host state per call (table generations), so it is
  // refused there; every other stage is captured as plain launches.
  const bool capturing = stream_capturing(st);
  if (capturing && (mask & OSE_STAGE_SAMPLE) && group_mode == OSE_GROUP_TRACE_ID)
    return fail(OSE_ENOTSUP, "SAMPLE with OSE_GROUP_TRACE_ID cannot be captured into a hipGraph "
                             "(its trace-id tables advance a host-side generation per call)");
  Workspace* ws = e->acquire_ws(st);
  const uint64_t n = c->n_spans;
  const bool gate_on_host = (mask & OSE_STAGE_SAMPLE) && group_mode == OSE_GROUP_TRACE_ID && n > 0 && !capturing &&
                            !(OSE_DIAG && getenv("OSE_NO_DEFER_SLOW"));
  const bool defer = gate_on_host && (mask & OSE_STAGE_TEMPLATE);
  // Workspace layout, one reservation for every stage of the call (a stage
  // must not reallocate scratch an earlier stage of the same call is still
  // using on the stream):
  //   [0, 256)  SAMPLE's words (the OSE_GROUP_BATCH decision SIZE reads);
  //             its whole scratch while its slow path may still be queued
  //   url_off   the URL stage's scratch
  //   size_off  the size stage's sums (after the URL scratch: with TEMPLATE
  //             its spans pass runs inside url_copy_kernel)
  size_t need = 0;
  if (mask & OSE_STAGE_SAMPLE) need = sampling_scratch_bytes(n);
  const size_t url_off = (mask & OSE_STAGE_SAMPLE) ? align_up(defer ? sampling_scratch_bytes(n) : 256, 256) : 0;
  size_t size_off = (mask & OSE_STAGE_SAMPLE) ? 256 : 0;
  if (mask & OSE_STAGE_TEMPLATE) {
    need = std::max(need, url_off + url_workspace_bytes(n, c->arena_bytes));
    size_off = align_up(url_off + url_workspace_bytes(n, c->arena_bytes), 256);
  }
  if (mask & OSE_STAGE_SIZE) need = std::max(need, size_off + size_scratch_bytes(c->n_scopes, c->n_resources));
  int rc = ws->reserve(need);
  std::function<int()> sample_tail;
  UrlKernelArgs ua{};
  // SAMPLE + TEMPLATE (deferred slow path: the URL scratch lies past the
  // trace stage's): the URL planning kernels (plan, slow plan, scan) need
  // nothing from SAMPLE, so they run on a second stream beside the trace
  // stage; the two are latency-bound at four waves per SIMD each and fit a
  // CU together (LDS 2 x 39.7 + 2 x 29.7 KB).  The copy / size launches that
  // read the final keep bytes wait for both.
  hipStream_t ust = nullptr;
  static const bool one_stream = getenv("OSE_ONE_STREAM") != nullptr;   // per-kernel profiling: no overlap
  // (a small batch's kernels are launch-bound: a fork only adds two events
  // and a stream hand-off to each call of a request-sized batch)
  constexpr uint64_t kForkSpans = 1u << 20;
  // the plan grid beside the trace stage: 16x the resident workgroups
  // (C4 7.80 -> 7.62 ms, C5 3.49 -> 3.26; 4x: 7.88 / 3.27; alone, C2, the
  // resident grid stays: 16x there is 0.64 -> 2.0 ms, profiles/r5g_plan_grid_ab.txt)
  // The plan grid (refs form): more workgroups than fit at once, so the
  // dispatcher balances the groups' uneven cost (a persistent grid's waves
  // each take a fixed 1/4096 of the groups and the last ones finish late)
  // and, beside the trace stage, interleaves the two kernels' workgroups; a
  // wave's start costs about what a few groups do, so each wave keeps ~19
  // groups: serialised, C4 url_plan 4.30 (resident grid) -> 4.09 (2x) ->
  // 3.92 (4x) -> 3.82 (8x) -> 3.80 ms (16x, the multiplier this rule gives
  // it), C2 0.531 -> 0.520 (2x, its rule) -> 0.542 (4x) -> 0.935 (8x) -> 1.90
  // (16x) (profiles/r6s_plan_grid_serial_ab.txt)
  const uint32_t plan_groups = (uint32_t)((n + kUrlGroup - 1) / kUrlGroup);
  if (!one_stream && !rc && defer && n >= kForkSpans) {
    if (!ws->fork) (void)hipEventCreateWithFlags(&ws->fork, hipEventDisableTiming);
    if (!ws->join) (void)hipEventCreateWithFlags(&ws->join, hipEventDisableTiming);
    // (the fork stream's priority, high or low, measured no different:
    // profiles/r6u_url_stream_priority_ab.txt)
    if (ws->fork && ws->join) ust = e->take_stream();
    if (ust && (hipEventRecord(ws->fork, st) != hipSuccess || hipStreamWaitEvent(ust, ws->fork, 0) != hipSuccess)) {
      e->give_stream(ust);
      ust = nullptr;
    }
  }
  const bool tmpl = !rc && (mask & OSE_STAGE_TEMPLATE);
  ws->beside_url = ust && tmpl;
  if (ust && tmpl)
    rc = run_url(e, c, o, ust, ws, url_off, &ua, (mask & OSE_STAGE_TEMPLATE_REFS) != 0, url_plan_grid_mult(plan_groups, true));
  // gateway pipeline order: odigossampling (-24) before odigosurltemplate (1)
  if (!rc && (mask & OSE_STAGE_SAMPLE)) rc = run_sampling(e, c, o, group_mode, rnd, st, ws, gate_on_host ? &sample_tail : nullptr);
  if (sample_tail && !defer) {
    rc = sample_tail();
    sample_tail = nullptr;
  }
  if (!ust && tmpl && !rc)
    rc = run_url(e, c, o, st, ws, url_off, &ua, (mask & OSE_STAGE_TEMPLATE_REFS) != 0, url_plan_grid_mult(plan_groups));
  if (sample_tail) {
    const int trc = sample_tail();   // always drained: the host event wait must not be skipped
    if (!rc) rc = trc;
  }
  if (ust) {   // join: everything below runs on the caller's stream after both
    const hipError_t je = hipEventRecord(ws->join, ust);
    const hipError_t jw = je == hipSuccess ? hipStreamWaitEvent(st, ws->join, 0) : je;
    if (jw != hipSuccess) {   // cannot order the streams: wait for the URL work on the host
      (void)hipStreamSynchronize(ust);
      if (!rc) rc = fail(OSE_EDEVICE, std::string("URL stream join: ") + hipGetErrorString(jw));
    }
    e->give_stream(ust);
  }
  // odigostrafficmetrics runs last, on what the earlier stages left (the
  // decisions are final here: SAMPLE's tail has been queued)
  SizeKernelArgs sa{};
  bool size_on = false;
  if (!rc && (mask & OSE_STAGE_SIZE)) rc = prepare_size(e, c, o, mask, group_mode, rnd, st, ws, size_off, sa, size_on);
  if (!rc && tmpl) {
    if (size_on && n > 0 && !(OSE_DIAG && getenv("OSE_NO_FUSED_SIZE"))) {
      // the spans pass rides in url_copy_kernel (one walk over the spans)
      sa.kept_partials = size_partials_of(ws, size_off, c->n_scopes, c->n_resources);
      sa.n_kept_partials = url_copy_blocks(ua.n_groups);
      ua.fuse_size = 1;
      ua.size_partials = const_cast<uint32_t*>(sa.kept_partials);
      ua.sz = sa;
    }
    rc = run_url_back(e, ua, st);
  }
  if (!rc && size_on) rc = run_size_tail(e, sa, st);
  ws->beside_url = false;
  e->release_ws(ws, st);
  return rc;
}

}  // namespace ose

using namespace ose;

extern "C" {

const char* ose_last_error(void) { return g_last_error.c_str(); }

uint64_t ose_dropped_errors(char* last, size_t cap) {
  std::lock_guard<std::mutex> g(g_dropped_mu);
  if (last && cap) snprintf(last, cap, "%s", g_dropped_last.c_str());
  return g_dropped_count;
}

// Diagnostic, no device: the number of rule chunks build_sampling_tables
// cuts the config's odigossampling rule list into (0 without the section);
// the codes and messages of ose_engine_create's sampling checks.
extern "C" int osehost_sampling_chunks(const char* cfg_json, uint32_t* n_chunks) {
  if (!n_chunks) return fail(OSE_EINVAL, "n_chunks is NULL");
  *n_chunks = 0;
  Json root;
  try {
    root = parse_json(cfg_json ? cfg_json : "{}");
  } catch (const std::exception& ex) {
    return fail(OSE_EINVAL, ex.what());
  }
  const Json* j = root.is_obj() ? root.get("odigossampling") : nullptr;
  if (!j) return 0;
  Engine e;
  const std::string err = decode_sampling_config(*j, e.sampling);
  if (!err.empty()) return fail(OSE_EINVAL, err);
  e.has_sampling = true;
  if (const int rc = e.build_sampling_tables()) return rc;
  *n_chunks = (uint32_t)e.sampling_chunks_host.size();
  return 0;
}

int ose_engine_create(const char* cfg_json, ose_engine** out) {
  if (!out) return fail(OSE_EINVAL, "out is NULL");
  *out = nullptr;
  Json root;
  try {
    root = parse_json(cfg_json ? cfg_json : "{}");
  } catch (const std::exception& ex) {
    return fail(OSE_EINVAL, ex.what());
  }
  if (!root.is_obj()) return fail(OSE_EINVAL, "config must be a JSON object");
  auto* e = new Engine();
  std::string err;
  if (const Json* j = root.get("odigosurltemplate")) {
    err = decode_url_config(*j, e->url);
    if (!err.empty()) { delete e; return fail(OSE_EINVAL, err); }
    e->has_url = true;
    e->url_needs_resource = e->url.include.has_value() || e->url.exclude.has_value();
  }
  if (const Json* j = root.get("odigossampling")) {
    err = decode_sampling_config(*j, e->sampling);
    if (!err.empty()) { delete e; return fail(OSE_EINVAL, err); }
    e->has_sampling = true;
  }
  if (const Json* j = root.get("odigostrafficmetrics")) {
    err = decode_traffic_config(*j, e->traffic);
    if (!err.empty()) { delete e; return fail(OSE_EINVAL, err); }
    e->has_traffic = true;
    // newThroughputMeasurementProcessor (processor.go:31-36)
    e->inverse = e->traffic.sampling_ratio != 0 ? (int64_t)(1.0 / e->traffic.sampling_ratio) : 0;
  }
  if (e->has_url) {
    int rc = build_url_blob(e->url, e->url_blob_host, e->max_name);
    if (rc) { delete e; return rc; }
  }
  int rc = e->build_sampling_tables();
  if (rc) { delete e; return rc; }
  rc = e->build_attr_tables();
  if (rc) { delete e; return rc; }
  rc = ensure_device();
  if (rc) { delete e; return rc; }
  if (hipGetDevice(&e->device) != hipSuccess) { delete e; return fail(OSE_EDEVICE, "hipGetDevice failed"); }
  if (e->has_url) {
    rc = upload(e->url_blob_host, &e->url_blob_dev);
    if (rc) { delete e; return rc; }
  }
  if (e->has_sampling) {
    e->sampling_chunks_dev.assign(e->sampling_chunks_host.size(), nullptr);
    for (size_t k = 0; k < e->sampling_chunks_host.size(); k++) {
      rc = upload(e->sampling_chunks_host[k], &e->sampling_chunks_dev[k]);
      if (rc) { delete e; return rc; }
    }
    e->sampling_blob_dev = e->sampling_chunks_dev[0];
    e->sampling_svc_map_dev.assign(e->sampling_svc_map_host.size(), nullptr);
    for (size_t k = 0; k < e->sampling_svc_map_host.size(); k++) {
      const auto& m = e->sampling_svc_map_host[k];
      std::vector<uint8_t> raw(reinterpret_cast<const uint8_t*>(m.data()),
                               reinterpret_cast<const uint8_t*>(m.data()) + 4 * m.size());
      rc = upload(raw, reinterpret_cast<uint8_t**>(&e->sampling_svc_map_dev[k]));
      if (rc) { delete e; return rc; }
    }
    if (!e->sampling_svc_map_dev.empty()) {
      std::vector<uint8_t> raw(sizeof(uint32_t*) * e->sampling_svc_map_dev.size());
      std::memcpy(raw.data(), e->sampling_svc_map_dev.data(), raw.size());
      rc = upload(raw, reinterpret_cast<uint8_t**>(&e->sampling_svc_maps_dev));
      if (rc) { delete e; return rc; }
    }
    const size_t K = e->sampling_chunks_dev.size(), L = e->sampling_lat_svc.size();
    // then trace_multi_kernel's latency-service ids: [n_services] the index of
    // each service among those with http_latency rules in any chunk (or
    // 0xFFFFFFFF), [64] the service of each index
    const size_t S = e->service_ids.size();
    std::vector<uint32_t> gof(S, 0xFFFFFFFFu), gsvc(64, 0);
    uint32_t ng = 0;
    for (size_t v = 0; v < S; v++)
      if ((e->sampling_lat_svc[v >> 5] >> (v & 31)) & 1u) {
        if (ng < 64) {
          gof[v] = ng;
          gsvc[ng] = (uint32_t)v;
        }
        ng++;
      }
    e->sampling_n_lat_svc = ng;
    // then each chunk's SampWalkDev (chunks of <= 128 rules; trace_multi_kernel)
    std::vector<SampWalkDev> walks(K);
    e->sampling_walk_ok = true;
    for (size_t k = 0; k < K; k++) {
      SampWalkDev& w = walks[k];
      std::memset(&w, 0, sizeof w);
      const uint8_t* b = e->sampling_chunks_host[k].data();
      const SampCfgDev* h = reinterpret_cast<const SampCfgDev*>(b);
      if (h->n_rules > 128) e->sampling_walk_ok = false;
      const SampRuleDev* rules = reinterpret_cast<const SampRuleDev*>(b + h->rules_off);
      for (uint32_t r = 0; r < h->n_rules && r < 128; r++) {
        const uint64_t bit = 1ull << (r & 63);
        if (rules[r].type == kSampError) w.err[r >> 6] |= bit;
        else if (rules[r].type == kSampLatency) w.lat_rule[rules[r].bit & 63] = (uint8_t)r;
        else w.svc[rules[r].bit & 63][r >> 6] |= bit;
      }
    }
    const size_t wo = align_up(8 * K + 4 * L + 4 * S + 4 * 64, 16);
    std::vector<uint8_t> st(wo + K * sizeof(SampWalkDev));
    std::memcpy(st.data(), e->sampling_chunks_dev.data(), 8 * K);
    std::memcpy(st.data() + 8 * K, e->sampling_lat_svc.data(), 4 * L);
    if (S) std::memcpy(st.data() + 8 * K + 4 * L, gof.data(), 4 * S);
    std::memcpy(st.data() + 8 * K + 4 * L + 4 * S, gsvc.data(), 4 * 64);
    std::memcpy(st.data() + wo, walks.data(), K * sizeof(SampWalkDev));
    rc = upload(st, &e->shard_tables_dev);
    if (rc) { delete e; return rc; }
  }
  if (!e->attr_blob_host.empty()) {
    rc = upload(e->attr_blob_host, &e->attr_blob_dev);
    if (rc) { delete e; return rc; }
    std::vector<uint8_t> hm(8 * std::max<size_t>(e->attr_words, 1), 0);
    std::memcpy(hm.data(), e->attr_host_words.data(), 8 * std::min<size_t>(e->attr_host_words.size(), e->attr_words));
    rc = upload(hm, &e->attr_host_mask_dev);
    if (rc) { delete e; return rc; }
  }
  {
    hipError_t he = hipMalloc(reinterpret_cast<void**>(&e->path_count_dev), 64);
    if (he == hipSuccess) he = hipMemset(e->path_count_dev, 0, 64);
    if (he != hipSuccess) {
      delete e;
      return fail(OSE_EDEVICE, std::string("path counters: ") + hipGetErrorString(he));
    }
  }
  *out = reinterpret_cast<ose_engine*>(e);
  return 0;
}

uint32_t ose_engine_path_counts(ose_engine* eng, uint64_t* counts, uint32_t cap) {
  if (!eng) return 0;
  Engine* e = reinterpret_cast<Engine*>(eng);
  uint64_t c[3] = {0, 0, e->long_run_passes.load()};
  if (e->path_count_dev && bind_device(e) == 0) {
    LastErrorScope keep("ose_engine_path_counts");
    // counters the queued work has not reached yet are not counted: the
    // device is synchronised first
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(c, e->path_count_dev, 16, hipMemcpyDeviceToHost) != hipSuccess)
      c[0] = c[1] = 0;
  }
  for (uint32_t k = 0; k < 3 && k < cap && counts; k++) counts[k] = c[k];
  return 3;
}

void ose_engine_destroy(ose_engine* eng) {
  if (!eng) return;
  Engine* e = reinterpret_cast<Engine*>(eng);
  e->closed.store(true);
  engine_unref(e);
}

int ose_host_alloc(size_t bytes, void** out) {
  if (!out) return fail(OSE_EINVAL, "NULL argument");
  int rc = ensure_device();
  if (rc) return rc;
  HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return 0;
}
void ose_host_free(void* p) {
  LastErrorScope keep("ose_host_free");
  if (p) (void)hipHostFree(p);
}

int ose_set_device(int device) {
  int rc = ensure_device();
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  return 0;
}

uint32_t ose_engine_service_id(const ose_engine* eng, const char* name, size_t len) {
  if (!eng || !name) return OSE_NONE;
  const Engine* e = reinterpret_cast<const Engine*>(eng);
  auto it = e->service_ids.find(std::string(name, len));
  return it == e->service_ids.end() ? OSE_NONE : it->second;
}

int ose_engine_get_info(const ose_engine* eng, ose_engine_info* info) {
  if (!eng || !info) return fail(OSE_EINVAL, "NULL argument");
  const Engine* e = reinterpret_cast<const Engine*>(eng);
  info->stages = (e->has_sampling ? OSE_STAGE_SAMPLE : 0) | (e->has_url ? OSE_STAGE_TEMPLATE : 0) |
                 (e->has_traffic ? OSE_STAGE_SIZE : 0);
  info->max_template_name = e->max_name;
  info->inverse_sampling = e->inverse;
  info->traffic_sampling_ratio = e->traffic.sampling_ratio;
  info->n_attr_rules = e->attr_n_rules;
  info->n_attr_keys = (uint32_t)e->attr_keys.size();
  info->attr_host_rules = e->attr_host_rules;
  return 0;
}

uint32_t ose_engine_attr_host_rules(const ose_engine* eng, uint64_t* words, uint32_t cap) {
  if (!eng) return 0;
  const Engine* e = reinterpret_cast<const Engine*>(eng);
  if (!e->attr_n_rules) return 0;
  const uint32_t W = e->attr_words;
  for (uint32_t w = 0; w < W && w < cap && words; w++) words[w] = w < e->attr_host_words.size() ? e->attr_host_words[w] : 0;
  return W;
}

int ose_engine_set_option(ose_engine* eng, const char* name, int64_t value) {
  if (!eng || !name) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  static const struct { const char* name; uint32_t bit; } kOpts[] = {
      {"otlp_gpu_chain", Engine::kOptOtlpGpuChain},
      {"otlp_host_resources", Engine::kOptOtlpHostResources},
      {"otlp_host_scopes", Engine::kOptOtlpHostScopes},
      {"encode_host", Engine::kOptEncodeHost},
  };
  for (const auto& o : kOpts) {
    if (strcmp(name, o.name) != 0) continue;
    if (value) e->options.fetch_or(o.bit);
    else e->options.fetch_and(~o.bit);
    return 0;
  }
  return fail(OSE_EINVAL, std::string("unknown engine option: ") + name);
}

int ose_reserve(ose_engine* eng, uint64_t n_spans, uint64_t arena_bytes) {
  if (!eng) return fail(OSE_EINVAL, "NULL engine");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (int brc = bind_device(e)) return brc;
  Workspace* ws = e->acquire_ws(nullptr);
  int rc = ws->reserve(e->workspace_bytes(n_spans, arena_bytes));
  if (!rc && e->has_sampling) rc = ws->reserve_table(n_spans);
  if (!rc && e->attr_n_dev) rc = ws->reserve_attr(n_spans);
  if (!rc && e->sampling_chunks_dev.size() > 1) rc = ws->reserve_fold(std::max<uint64_t>(n_spans, 1));
  e->release_ws(ws, nullptr);
  return rc;
}

int ose_process_device(ose_engine* eng, const ose_columns* cols, const ose_outputs* outs, uint32_t stage_mask,
                       uint32_t group_mode, const ose_rand* rnd, void* hip_stream) {
  if (!eng) return fail(OSE_EINVAL, "NULL engine");
  if (int brc = bind_device(reinterpret_cast<Engine*>(eng))) return brc;
  return run_stages(reinterpret_cast<Engine*>(eng), cols, outs, stage_mask, group_mode, rnd,
                    static_cast<hipStream_t>(hip_stream));
}

int ose_profile_enable(ose_engine* eng, int on) {
  if (!eng) return fail(OSE_EINVAL, "NULL engine");
  reinterpret_cast<Engine*>(eng)->profiling = on != 0;
  return 0;
}

int ose_profile_read(ose_engine* eng, char* json, size_t cap) {
  if (!eng || !json) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (int brc = bind_device(e)) return brc;
  std::vector<Engine::Timed> ts;
  {
    std::lock_guard<std::mutex> g(e->mu);
    ts.swap(e->timed);
  }
  std::map<std::string, std::pair<uint64_t, double>> acc;
  for (auto& t : ts) {
    HIP_TRY(hipEventSynchronize(t.b));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, t.a, t.b));
    auto& a = acc[t.name];
    a.first++;
    a.second += ms;
  }
  {
    std::lock_guard<std::mutex> g(e->mu);
    for (auto& t : ts) { e->event_pool.push_back(t.a); e->event_pool.push_back(t.b); }
  }
  std::string s = "{";
  for (auto& kv : acc) {
    if (s.size() > 1) s += ",";
    char buf[256];
    snprintf(buf, sizeof buf, "\"%s\":{\"launches\":%llu,\"ms\":%.6f}", kv.first.c_str(),
             (unsigned long long)kv.second.first, kv.second.second);
    s += buf;
  }
  s += "}";
  if (s.size() + 1 > cap) return fail(OSE_ERANGE, "profile buffer too small");
  std::memcpy(json, s.c_str(), s.size() + 1);
  return 0;
}

int ose_device_info(char* buf, size_t cap) {
  if (!buf || cap == 0) return fail(OSE_EINVAL, "NULL buffer");
  int rc = ensure_device();
  if (rc) { snprintf(buf, cap, "no device"); return rc; }
  hipDeviceProp_t p;
  HIP_TRY(hipGetDeviceProperties(&p, 0));
  snprintf(buf, cap, "%s arch=%s CUs=%d HBM=%.1fGB", p.name, p.gcnArchName, p.multiProcessorCount,
           (double)p.totalGlobalMem / 1e9);
  return 0;
}

}  // extern "C"
