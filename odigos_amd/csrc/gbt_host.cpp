// gbt_host.cpp — the GPU-resident groupbytrace store:
// ose_gbt_*.  Restates groupbytraceprocessor (opentelemetry-collector-contrib
// v0.141.0, `collector/builder-config.yaml:73`; not in the reference tree)
// as Odigos configures it (`autoscaler/controllers/actions/sampling/
// groupbytrace.go:3-9`: wait_duration "30s"; num_traces and num_workers at
// their defaults, 1,000,000 and 1; other num_workers are taken too):
//   * ConsumeTraces splits the batch per (ResourceSpans, ScopeSpans, trace
//     id) (batchpersignal.SplitTraces) and hands each piece to the event
//     machine in that order;
//   * the first piece of an unknown trace id puts it in the ring buffer of
//     num_traces ids — evicting (dropping) the trace that slot held — and
//     arms a timer of wait_duration; later pieces append to the trace;
//   * on expiry the trace leaves the buffer and goes downstream as one
//     ptrace.Traces holding its pieces in arrival order; spans of that id
//     arriving afterwards start a new trace;
//   * num_workers W > 1: the event machine hands a trace's events to worker
//     fnv64(id) % W, each worker with a ring of num_traces / W ids, so a
//     trace is evicted by the (num_traces / W)-th trace created after it in
//     its own worker.
// Time is the caller's clock (now_ns on every call), so releases are
// deterministic.  The kernels are in gbt_kernel.hip.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "engine_internal.hpp"
#include "kernels.hpp"

namespace ose {

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {
size_t up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

struct DevMem {   // grow-only device buffer
  uint8_t* p = nullptr;
  size_t cap = 0;
  int need(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = up(std::max<size_t>(bytes + bytes / 4, 1 << 16), 1 << 16);
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p), want));
    cap = want;
    return 0;
  }
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

// Go's time.ParseDuration: [-+]?([0-9]*(\.[0-9]*)?unit)+ or "0"
bool parse_go_duration(const std::string& s, int64_t& out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '-' || s[i] == '+')) neg = s[i++] == '-';
  if (s.substr(i) == "0") { out = 0; return true; }
  if (i == s.size()) return false;
  double total = 0;
  while (i < s.size()) {
    const size_t d0 = i;
    uint64_t v = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') v = v * 10 + (uint64_t)(s[i++] - '0');
    double frac = 0, scale = 1;
    const bool int_digits = i > d0;
    bool frac_digits = false;
    if (i < s.size() && s[i] == '.') {
      i++;
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
        frac = frac * 10 + (s[i++] - '0');
        scale *= 10;
        frac_digits = true;
      }
    }
    if (!int_digits && !frac_digits) return false;
    const size_t u0 = i;
    while (i < s.size() && !(s[i] >= '0' && s[i] <= '9') && s[i] != '.') i++;
    const std::string unit = s.substr(u0, i - u0);
    double mult;
    if (unit == "ns") mult = 1;
    else if (unit == "us" || unit == "\xC2\xB5s" || unit == "\xCE\xBCs") mult = 1e3;
    else if (unit == "ms") mult = 1e6;
    else if (unit == "s") mult = 1e9;
    else if (unit == "m") mult = 60e9;
    else if (unit == "h") mult = 3600e9;
    else return false;
    total += (double)v * mult + frac / scale * mult;
  }
  if (total > 9.2e18) return false;
  out = (int64_t)std::llround(neg ? -total : total);
  return true;
}
}  // namespace

struct Gbt {
  Engine* e = nullptr;
  int64_t wait_ns = 0;
  uint64_t num_traces = 1000000;
  uint32_t W = 1;                 // num_workers
  uint64_t ring_n = 0, wcap = 0;  // ring slots (num_traces, or the pool capacity when W > 1); num_traces / W
  std::vector<uint64_t> wcnt;     // per worker: traces numbered
  std::vector<uint64_t> wrel;     // per worker: its traces with seq < rel_end (released or evicted)
  uint32_t K = 0;
  uint64_t pool_cap = 0, scope_cap = 0, arena_cap = 0;
  // device state
  DevMem table, ring, pool, scopes, arena, scratch, sortbuf, out, words, tinfo, wdev;
  uint64_t table_slots = 0;
  uint32_t epoch = 0;
  GbtPool P{};
  GbtScopes Q{};
  // host clock
  uint64_t next_seq = 0, rel_end = 0;
  uint64_t pool_begin = 0, pool_end = 0, scope_begin = 0, scope_end = 0, arena_begin = 0, arena_end = 0;
  struct Epoch {
    int64_t t;
    uint64_t seq1, pool1, scope1, arena1;
    std::vector<uint64_t> wcnt1;   // W > 1: the workers' counts after the call
  };
  std::deque<Epoch> epochs;
  uint32_t n_attrsets = 0;
  int64_t last_now = INT64_MIN;   // the clock of the last successful call
  // the last release
  ose_columns out_cols{};
  // stats: created, released traces, evicted traces, released spans, added spans
  uint64_t created = 0, released = 0, evicted = 0, released_spans = 0, added_spans = 0;

  // the persistent id table (gbt_kernel.hip): slots claimed since its last
  // rebuild (live ids and tombstones), the number of the last add
  uint64_t slots_used = 0;
  uint32_t add_gen = 0;
  bool table_valid = false;

  // one worker: the traces a ring of num_traces has evicted (W > 1: per trace, gbt_evicted)
  uint64_t evict_below() const { return W == 1 && next_seq > num_traces ? next_seq - num_traces : 0; }
  // W > 1: worker w's traces [0, this) are evicted
  uint64_t w_evicted(uint32_t w) const { return wcnt[w] > wcap ? wcnt[w] - wcap : 0; }
  uint64_t waiting() const {
    if (W == 1) return next_seq - live_lo();
    uint64_t n = 0;
    for (uint32_t w = 0; w < W; w++) n += wcnt[w] - std::max(wrel[w], w_evicted(w));
    return n;
  }
  uint64_t live_lo() const { return std::max(rel_end, evict_below()); }
  // traces whose wait is over at `now`: [.., expired_below(now)) (created by
  // the calls at least wait_duration ago; the next release hands them out)
  uint64_t expired_below(int64_t now) const {
    uint64_t b = rel_end;
    for (const Epoch& ep : epochs) {
      if (ep.t + wait_ns > now) break;
      b = std::max(b, ep.seq1);
    }
    return b;
  }
};

namespace {
// exclusive scan of n u32 (flags or lengths) with the shared look-back scan
int scan_u32(Gbt* g, const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* total, hipStream_t st) {
  if (!n) return 0;
  const uint32_t tiles = (uint32_t)((n + kScanTileItems - 1) / kScanTileItems);
  uint32_t* counter = reinterpret_cast<uint32_t*>(g->words.p) + 4;
  uint64_t* status = reinterpret_cast<uint64_t*>(g->words.p + 64);
  if ((uint64_t)tiles * 8 + 64 > g->words.cap) return fail(OSE_EDEVICE, "groupbytrace: scan status too small");
  HIP_TRY(hipMemsetAsync(counter, 0, 4, st));
  HIP_TRY(hipMemsetAsync(status, 0, (size_t)tiles * 8, st));
  ScanArgs sa{};
  sa.n = n;
  sa.n_tiles = tiles;
  sa.in = in;
  sa.out = out;
  sa.total = total;
  sa.counter = counter;
  sa.status = status;
  sa.error = reinterpret_cast<uint32_t*>(g->words.p);
  launch_scan_u32(sa, st);
  HIP_TRY(hipGetLastError());
  return 0;
}

int words_need(Gbt* g, uint64_t n) {   // error word, scan counter, totals, one gate word, scan status
  return g->words.need(64 + 8 * ((n + kScanTileItems - 1) / kScanTileItems + 256 * 4 + 16));
}

// stable LSD radix sort of m (key, value) pairs on the keys' low `bits` bits
// (the sampling stage's sort kernels: 8-bit digits, LDS histograms, look-back
// scans); *skeys / *svals: the sorted arrays (the inputs when m <= 1 or bits == 0)
int sort_pairs(Gbt* g, const uint32_t* keys, const uint32_t* vals, uint64_t m, int bits, hipStream_t st,
               const uint32_t** skeys, const uint32_t** svals) {
  *skeys = keys;
  *svals = vals;
  if (m <= 1 || !bits) return 0;
  int rc;
  const uint32_t T = (uint32_t)((m + kSortTile - 1) / kSortTile);
  const uint32_t htiles = (uint32_t)((256ull * T + kScanTileItems - 1) / kScanTileItems);
  if ((rc = g->sortbuf.need(4 * up(4 * m + 16) + 2 * up(4ull * 256 * T + 16))) || (rc = words_need(g, 256ull * T)))
    return rc;
  uint32_t* k2 = reinterpret_cast<uint32_t*>(g->sortbuf.p);
  uint32_t* k3 = k2 + up(4 * m + 16) / 4;
  uint32_t* v2 = k3 + up(4 * m + 16) / 4;
  uint32_t* v3 = v2 + up(4 * m + 16) / 4;
  uint32_t* hist = v3 + up(4 * m + 16) / 4;
  uint32_t* hoff = hist + up(4ull * 256 * T + 16) / 4;
  uint32_t* gate = reinterpret_cast<uint32_t*>(g->words.p) + 8;
  HIP_TRY(hipMemsetAsync(gate, 1, 4, st));   // open
  TraceSortArgs s{};
  s.n_spans = m;
  s.n_tiles = T;
  s.gate = gate;
  s.error = reinterpret_cast<uint32_t*>(g->words.p);
  s.key = const_cast<uint32_t*>(keys);
  const uint32_t* kin = keys;
  const uint32_t* vin = vals;
  uint32_t* kb[2] = {k2, k3};
  uint32_t* vb[2] = {v2, v3};
  int pass = 0;
  for (int shift = 0; shift < bits; shift += 8, pass++) {
    s.shift = (uint32_t)shift;
    s.keys_in = kin;
    s.vals_in = vin;
    s.keys_out = kb[pass & 1];
    s.vals_out = vb[pass & 1];
    s.hist = hist;
    s.scan_counter = reinterpret_cast<uint32_t*>(g->words.p) + 4;
    s.scan_status = reinterpret_cast<uint64_t*>(g->words.p + 64);
    s.scan_status_n = htiles;
    launch_sort_hist(s, st);
    HIP_TRY(hipGetLastError());
    ScanArgs sa{};
    sa.n = 256ull * T;
    sa.n_tiles = htiles;
    sa.gate = gate;
    sa.in = hist;
    sa.out = hoff;
    sa.counter = s.scan_counter;
    sa.status = s.scan_status;
    sa.error = s.error;
    launch_scan_u32(sa, st);
    HIP_TRY(hipGetLastError());
    TraceSortArgs s2 = s;
    s2.hist = hoff;
    launch_sort_scatter(s2, st);
    HIP_TRY(hipGetLastError());
    kin = kb[pass & 1];
    vin = vb[pass & 1];
  }
  *skeys = kin;
  *svals = vin;
  return 0;
}

GbtArgs base_args(Gbt* g) {
  GbtArgs a{};
  a.table = reinterpret_cast<GbtSlot*>(g->table.p);
  a.table_mask = g->table_slots - 1;
  a.epoch = g->epoch;
  a.n_attr_keys = g->K;
  a.attr_words = g->e->attr_words;
  a.error = reinterpret_cast<uint32_t*>(g->words.p);
  a.ring_tid = reinterpret_cast<uint64_t*>(g->ring.p);
  a.num_traces = g->num_traces;
  a.ring_n = g->ring_n;
  a.n_workers = g->W;
  a.worker_cap = g->wcap;
  if (g->W > 1) {
    a.tinfo = reinterpret_cast<uint64_t*>(g->tinfo.p);
    a.wcnt = reinterpret_cast<const uint64_t*>(g->wdev.p);
    a.wadd = reinterpret_cast<uint32_t*>(g->wdev.p + up(8ull * g->W));
    a.wstart = a.wadd + up(4ull * g->W + 16) / 4;
  }
  a.pool = g->P;
  a.pool_cap = g->pool_cap;
  a.scopes = g->Q;
  a.scope_cap = g->scope_cap;
  a.arena_ring = g->arena.p;
  a.arena_cap = g->arena_cap;
  return a;
}

// num_workers > 1: each new trace of the add gets its worker and its number
// within the worker (creation order), kept in tinfo; the workers' counts grow
int number_workers(Gbt* g, GbtArgs a, uint64_t created, hipStream_t st) {
  const uint32_t W = g->W;
  int rc, bits = 0;
  while (bits < 32 && ((uint64_t)(W - 1) >> bits)) bits++;
  HIP_TRY(hipMemsetAsync(a.wadd, 0, 4ull * W, st));
  launch_gbt_wkey(a, st);
  HIP_TRY(hipGetLastError());
  uint32_t* total = reinterpret_cast<uint32_t*>(g->words.p) + 3;
  if ((rc = scan_u32(g, a.wadd, a.wstart, W, total, st))) return rc;
  const uint32_t *skeys = nullptr, *svals = nullptr;
  if ((rc = sort_pairs(g, a.keys, a.vals, created, bits, st, &skeys, &svals))) return rc;
  a.keys = const_cast<uint32_t*>(skeys);
  a.vals = const_cast<uint32_t*>(svals);
  launch_gbt_wnum(a, created, st);
  HIP_TRY(hipGetLastError());
  std::vector<uint32_t> add(W);
  uint32_t err = 0;
  HIP_TRY(hipMemcpyAsync(add.data(), a.wadd, 4ull * W, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&err, g->words.p, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (err) return fail(OSE_EDEVICE, "groupbytrace: device error " + std::to_string(err) + " numbering the workers' traces");
  for (uint32_t w = 0; w < W; w++) g->wcnt[w] += add[w];
  return 0;
}

int gbt_add(Gbt* g, const ose_columns* c, const uint32_t* attrset_map, int64_t now, hipStream_t st) {
  if (now < g->last_now) return fail(OSE_EINVAL, "groupbytrace: now_ns went backwards");
  const uint64_t n = c->n_spans, S = c->n_scopes;
  if (!n) return 0;
  if (g->K && c->n_attr_keys != g->K) return fail(OSE_EINVAL, "groupbytrace: the batch's attribute key columns differ from the engine's");
  if (c->attr_match && std::max<uint32_t>(1, c->attr_match_words) != g->e->attr_words)
    return fail(OSE_EINVAL, "groupbytrace: attr_match_words differs from the engine's span_attribute rule words");
  if (!c->trace_id || !c->start_ns || !c->end_ns || !c->status || !c->kind || !c->scope || !c->scope_resource ||
      !c->res_svc || !c->res_attrset || (g->K && (!c->attr_type || !c->attr_val)))
    return fail(OSE_EINVAL, "groupbytrace: a required column is NULL");
  if (g->pool_end - g->pool_begin + n > g->pool_cap || g->scope_end - g->scope_begin + S > g->scope_cap)
    return fail(OSE_ERANGE, "groupbytrace: the store is full (spans waiting for wait_duration exceed its capacity)");
  int rc;
  // An added span joins its id's trace only while that trace is waiting: not
  // released, not evicted, and not past its wait_duration at `now` (contrib's
  // timer would have sent it downstream at its deadline, and later spans of
  // the id start a new trace; the expired one still goes out at the next
  // release).
  const uint64_t lo = std::max(g->live_lo(), g->expired_below(now));
  const uint64_t live = g->next_seq - lo;
  // the persistent id table: at least 4x the live traces plus the batch;
  // re-inserted from the live traces when it grows, when tombstones and live
  // ids would pass half of it, and when the epoch tag wraps
  uint64_t slots = 1024;
  while (slots < 4 * (live + n)) slots <<= 1;
  bool rebuild = !g->table_valid || g->slots_used + n > g->table_slots / 2;
  if (slots > g->table_slots || g->epoch + 1 >= (1u << 29)) {
    if ((rc = g->table.need(std::max(slots, g->table_slots) * sizeof(GbtSlot)))) return rc;
    g->table_slots = std::max(slots, g->table_slots);
    HIP_TRY(hipMemsetAsync(g->table.p, 0, g->table_slots * sizeof(GbtSlot), st));
    g->epoch = 0;
    rebuild = true;
  }
  if (rebuild) g->epoch++;
  g->add_gen = g->add_gen + 1 == 0 ? 1 : g->add_gen + 1;
  // scratch: slot_of (8n), flag, rank, strlen, stroff (4n each), the
  // attribute-set map; W > 1: the (worker, rank) pairs (4n each)
  const size_t A = c->n_attrsets;
  const size_t wpairs = g->W > 1 ? 2 * up(4 * n + 16) : 0;
  if ((rc = g->scratch.need(up(8 * n) + 4 * up(4 * n + 16) + up(4 * A + 16) + wpairs)) ||
      (rc = words_need(g, std::max<uint64_t>(n, g->W))))
    return rc;
  GbtArgs a = base_args(g);
  a.slot_of = reinterpret_cast<uint64_t*>(g->scratch.p);
  a.flag = reinterpret_cast<uint32_t*>(g->scratch.p + up(8 * n));
  a.rank = a.flag + up(4 * n + 16) / 4;
  a.strlen = a.rank + up(4 * n + 16) / 4;
  a.stroff = a.strlen + up(4 * n + 16) / 4;
  uint32_t* dmap = a.stroff + up(4 * n + 16) / 4;
  uint32_t max_set = A ? (uint32_t)A - 1 : 0;
  if (attrset_map && A) {
    HIP_TRY(hipMemcpyAsync(dmap, attrset_map, 4 * A, hipMemcpyHostToDevice, st));
    max_set = *std::max_element(attrset_map, attrset_map + A);
    a.attrset_map = dmap;
  }
  if (g->W > 1) {
    a.keys = dmap + up(4 * A + 16) / 4;
    a.vals = a.keys + up(4 * n + 16) / 4;
    // the workers' counts before the batch: its lookups and the rebuild skip evicted traces
    HIP_TRY(hipMemcpyAsync(g->wdev.p, g->wcnt.data(), 8ull * g->W, hipMemcpyHostToDevice, st));
  }
  a.cols = *c;
  a.n = n;
  a.n_scopes = S;
  a.next_seq = g->next_seq;
  a.live_lo = lo;
  a.live_hi = g->next_seq;
  a.add_gen = g->add_gen;
  a.pool_pos = g->pool_end;
  a.scope_pos = g->scope_end;
  a.arena_pos = g->arena_end;
  a.arena_room = g->arena_cap - (g->arena_end - g->arena_begin);
  HIP_TRY(hipMemsetAsync(g->words.p, 0, 16, st));   // error word, totals
  uint32_t* totals = reinterpret_cast<uint32_t*>(g->words.p) + 1;   // [0] new traces, [1] string bytes
  a.totals = totals;
  (void)hipGetLastError();
  if (rebuild) launch_gbt_rebuild(a, st);
  launch_gbt_lookup(a, st);
  launch_gbt_creator(a, st);
  HIP_TRY(hipGetLastError());
  if ((rc = scan_u32(g, a.flag, a.rank, n, totals, st))) return rc;
  if ((rc = scan_u32(g, a.strlen, a.stroff, n, totals + 1, st))) return rc;
  // every kernel from here stores nothing when the batch's strings do not
  // fit the arena ring (error bit 8): a refused add leaves the store as it was
  launch_gbt_assign(a, st);
  launch_gbt_append(a, st);
  launch_gbt_scopes(a, st);
  launch_gbt_strings(a, st);
  HIP_TRY(hipGetLastError());
  uint32_t h[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(h, g->words.p, 16, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (rebuild) g->slots_used = live;
  g->table_valid = true;
  if (h[0] & 8u) {
    g->slots_used += n;   // ids the lookups claimed stay as tombstones
    return fail(OSE_ERANGE, "groupbytrace: the string arena is full (bytes waiting for wait_duration exceed its capacity)");
  }
  if (h[0]) {
    g->table_valid = false;
    return fail(OSE_EDEVICE, "groupbytrace: device table error " + std::to_string(h[0]));
  }
  const uint64_t created = h[1], bytes = h[2];
  if (g->W > 1 && created && (rc = number_workers(g, a, created, st))) {
    g->table_valid = false;
    return rc;
  }
  g->slots_used += created;
  g->next_seq += created;
  g->created += created;
  g->added_spans += n;
  g->pool_end += n;
  g->scope_end += S;
  g->arena_end += bytes;
  g->n_attrsets = std::max<uint32_t>(g->n_attrsets, A ? max_set + 1 : 0);
  g->epochs.push_back(Gbt::Epoch{now, g->next_seq, g->pool_end, g->scope_end, g->arena_end,
                                 g->W > 1 ? g->wcnt : std::vector<uint64_t>{}});
  g->last_now = now;
  return 0;
}

int gbt_release(Gbt* g, int64_t now, hipStream_t st, uint32_t* n_traces) {
  if (now < g->last_now) return fail(OSE_EINVAL, "groupbytrace: now_ns went backwards");
  g->last_now = now;
  ose_columns& oc = g->out_cols;
  oc = ose_columns{};
  *n_traces = 0;
  // traces whose timer has fired: those created by the expired epochs
  size_t k = 0;
  uint64_t b = g->rel_end;
  while (k < g->epochs.size() && g->epochs[k].t + g->wait_ns <= now) b = std::max(b, g->epochs[k++].seq1);
  const uint64_t lo = g->live_lo();
  const uint64_t range = b > lo ? b - lo : 0;   // the seqs the release looks at
  uint64_t rel = range;                          // the traces it releases
  std::vector<uint64_t> wrel1;
  if (g->W == 1) {
    if (b > g->rel_end) {
      const uint64_t ev_hi = std::min(b, g->evict_below());
      if (ev_hi > g->rel_end) g->evicted += ev_hi - g->rel_end;   // evicted before their timer: dropped
    }
  } else if (k) {
    // worker w's traces in [rel_end, b) are its numbers [wrel, wrel1); those
    // below w_evicted were evicted before their timer: dropped
    wrel1 = g->epochs[k - 1].wcnt1;
    uint64_t ev = 0;
    for (uint32_t w = 0; w < g->W; w++) {
      const uint64_t e = std::min(wrel1[w], g->w_evicted(w));
      if (e > g->wrel[w]) ev += e - g->wrel[w];
    }
    g->evicted += ev;
    rel = range - ev;
  }
  const uint64_t window = g->pool_end - g->pool_begin;
  int rc;
  uint64_t m = 0;
  if (rel && window) {
    if ((rc = g->scratch.need(6 * up(4 * window + 16))) || (rc = words_need(g, window))) return rc;
    GbtArgs a = base_args(g);
    a.flag = reinterpret_cast<uint32_t*>(g->scratch.p);
    a.rank = a.flag + up(4 * window + 16) / 4;
    a.strlen = a.rank + up(4 * window + 16) / 4;
    a.stroff = a.strlen + up(4 * window + 16) / 4;
    a.keys = a.stroff + up(4 * window + 16) / 4;
    a.vals = a.keys + up(4 * window + 16) / 4;
    a.n = window;
    a.pool_pos = g->pool_begin;
    a.rel_lo = lo;
    a.rel_hi = b;
    uint32_t* totals = reinterpret_cast<uint32_t*>(g->words.p) + 1;
    HIP_TRY(hipMemsetAsync(g->words.p, 0, 16, st));
    if (g->W > 1) HIP_TRY(hipMemcpyAsync(g->wdev.p, g->wcnt.data(), 8ull * g->W, hipMemcpyHostToDevice, st));
    (void)hipGetLastError();
    launch_gbt_flag(a, st);
    HIP_TRY(hipGetLastError());
    if ((rc = scan_u32(g, a.flag, a.rank, window, totals, st))) return rc;
    launch_gbt_compact(a, st);
    HIP_TRY(hipGetLastError());
    uint32_t h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, g->words.p, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h[0]) return fail(OSE_EDEVICE, "groupbytrace: device error " + std::to_string(h[0]));
    m = h[1];
    // stable sort of the released spans by trace (window order = arrival order)
    int bits = 0;
    while (bits < 32 && ((range - 1) >> bits)) bits++;
    const uint32_t* order = a.vals;
    const uint32_t* skeys = a.keys;
    if ((rc = sort_pairs(g, a.keys, a.vals, m, bits, st, &skeys, &order))) return rc;
    // the released batch: fixed columns and fragment heads, then strings and fragments
    const uint64_t M = std::max<uint64_t>(m, 1), K = g->K;
    struct Part { void** dst; size_t bytes; };
    GbtOut& O = a.out;
    std::vector<Part> parts = {
        {(void**)&O.tid, 16 * M}, {(void**)&O.start, 8 * M}, {(void**)&O.end, 8 * M},
        {(void**)&O.attr_match, 8 * M * g->e->attr_words}, {(void**)&O.status, M}, {(void**)&O.kind, M},
        {(void**)&O.url_flags, M}, {(void**)&O.span_size, 4 * M}, {(void**)&O.name_len, 4 * M},
        {(void**)&O.resource, 4 * M}, {(void**)&O.scope, 4 * M}, {(void**)&O.route, 8 * M},
        {(void**)&O.path, 8 * M}, {(void**)&O.attr_type, K * M + 16}, {(void**)&O.attr_val, 8 * K * M + 16},
        {(void**)&O.res_svc, 4 * M}, {(void**)&O.res_svc_str, 4 * M}, {(void**)&O.res_attrset, 4 * M},
        {(void**)&O.res_size, 4 * M}, {(void**)&O.scope_size, 4 * M}, {(void**)&O.scope_resource, 4 * M},
        {(void**)&O.res_url_ok, M},
    };
    size_t total = 0;
    for (auto& p : parts) total = up(total + p.bytes + 16);
    const size_t arena_at = total;
    // the strings of the released spans are at most the live arena bytes
    const size_t arena_bound = g->arena_end - g->arena_begin;
    if ((rc = g->out.need(arena_at + up(arena_bound + 64)))) return rc;
    size_t off = 0;
    for (auto& p : parts) {
      *p.dst = g->out.p + off;
      off = up(off + p.bytes + 16);
    }
    O.arena = g->out.p + arena_at;
    a.n = m;
    a.order = order;
    HIP_TRY(hipMemsetAsync(g->words.p, 0, 16, st));
    launch_gbt_gather(a, st);
    HIP_TRY(hipGetLastError());
    if ((rc = scan_u32(g, a.flag, a.rank, m, totals, st))) return rc;           // fragments
    if ((rc = scan_u32(g, a.strlen, a.stroff, m, totals + 1, st))) return rc;   // string offsets
    launch_gbt_emit(a, st);
    HIP_TRY(hipGetLastError());
    uint32_t h2[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyAsync(h2, g->words.p, 12, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h2[0]) return fail(OSE_EDEVICE, "groupbytrace: device error " + std::to_string(h2[0]));
    const uint32_t F = h2[1], bytes = h2[2];
    oc.n_spans = m;
    oc.n_resources = F;
    oc.n_scopes = F;
    oc.n_attrsets = g->n_attrsets;
    oc.trace_id = O.tid;
    oc.start_ns = O.start;
    oc.end_ns = O.end;
    oc.status = O.status;
    oc.kind = O.kind;
    oc.resource = O.resource;
    oc.scope = O.scope;
    oc.url_flags = O.url_flags;
    oc.path = O.path;
    oc.route = O.route;
    oc.span_size = O.span_size;
    oc.name_len = O.name_len;
    oc.attr_match = O.attr_match;
    oc.attr_match_words = g->e->attr_words;
    oc.res_svc = O.res_svc;
    oc.res_svc_str = O.res_svc_str;
    oc.res_url_ok = O.res_url_ok;
    oc.res_attrset = O.res_attrset;
    oc.res_size = O.res_size;
    oc.scope_size = O.scope_size;
    oc.scope_resource = O.scope_resource;
    oc.arena = O.arena;
    oc.arena_bytes = bytes;
    oc.n_attr_keys = g->K;
    if (g->K) {
      oc.attr_type = O.attr_type;
      oc.attr_val = O.attr_val;
    }
  }
  *n_traces = (uint32_t)rel;   // traces with spans in the window (every released trace has >= 1)
  g->released += rel;
  g->released_spans += m;
  g->rel_end = std::max(g->rel_end, b);
  if (g->W > 1 && k) g->wrel = std::move(wrel1);
  if (k) {   // every span of an expired epoch belongs to a released or evicted trace
    const Gbt::Epoch& last = g->epochs[k - 1];
    g->pool_begin = last.pool1;
    g->scope_begin = last.scope1;
    g->arena_begin = last.arena1;
    g->epochs.erase(g->epochs.begin(), g->epochs.begin() + (long)k);
  }
  return 0;
}
}  // namespace

}  // namespace ose

using namespace ose;

extern "C" {

int ose_gbt_create(ose_engine* eng, const char* cfg_json, uint64_t span_capacity, uint64_t arena_capacity,
                   ose_gbt** out) {
  if (!eng || !cfg_json || !out) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (int rc = bind_device(e)) return rc;
  auto* g = new Gbt();
  g->e = e;
  try {
    const Json cfg = parse_json(cfg_json);
    std::string wait = "1s";   // the processor's default (contrib); Odigos sets "30s"
    if (const Json* w = cfg.get("wait_duration")) {
      if (!w->is_str()) { delete g; return fail(OSE_EINVAL, "wait_duration: expected a duration string"); }
      wait = w->s;
    }
    if (!parse_go_duration(wait, g->wait_ns)) { delete g; return fail(OSE_EINVAL, "time: invalid duration \"" + wait + "\""); }
    if (const Json* nt = cfg.get("num_traces")) g->num_traces = (uint64_t)nt->i64();
    int64_t nw = 1;
    if (const Json* w = cfg.get("num_workers")) nw = w->i64();
    if ((int64_t)g->num_traces <= 0) { delete g; return fail(OSE_EINVAL, "groupbytrace: num_traces must be positive"); }
    if (nw <= 0 || nw > (1 << 20)) { delete g; return fail(OSE_EINVAL, "groupbytrace: num_workers must be in [1, 2^20]"); }
    // each worker's ring holds num_traces / num_workers ids (contrib's
    // newRingBuffer would divide by zero below one)
    if ((uint64_t)nw > g->num_traces) { delete g; return fail(OSE_EINVAL, "groupbytrace: num_traces must be at least num_workers"); }
    g->W = (uint32_t)nw;
  } catch (const std::exception& ex) {
    delete g;
    return fail(OSE_EINVAL, ex.what());
  }
  g->K = (uint32_t)e->attr_keys.size();
  g->pool_cap = std::max<uint64_t>(span_capacity, 1024);
  g->scope_cap = g->pool_cap;
  g->arena_cap = std::max<uint64_t>(arena_capacity, 1 << 16);
  // one worker: the ring is num_traces ids (every live seq is within
  // num_traces of the newest).  W > 1: a worker's old trace can outlive
  // num_traces newer ones of other workers, but every seq not yet released
  // has its first span in the pool, so pool_cap slots cover them
  g->wcap = g->num_traces / g->W;
  g->ring_n = g->W == 1 ? g->num_traces : g->pool_cap;
  g->wcnt.assign(g->W, 0);
  g->wrel.assign(g->W, 0);
  const uint64_t C = g->pool_cap, K = g->K;
  struct Part { void** dst; size_t bytes; };
  std::vector<Part> parts = {
      {(void**)&g->P.tid, 16 * C}, {(void**)&g->P.start, 8 * C}, {(void**)&g->P.end, 8 * C},
      {(void**)&g->P.attr_match, 8 * C * g->e->attr_words}, {(void**)&g->P.seq, 8 * C}, {(void**)&g->P.origin, 8 * C},
      {(void**)&g->P.str_off, 8 * C}, {(void**)&g->P.status, C}, {(void**)&g->P.kind, C},
      {(void**)&g->P.url_flags, C}, {(void**)&g->P.span_size, 4 * C}, {(void**)&g->P.name_len, 4 * C},
      {(void**)&g->P.route, 8 * C}, {(void**)&g->P.path, 8 * C}, {(void**)&g->P.attr_type, K * C + 16},
      {(void**)&g->P.attr_val, 8 * K * C + 16},
  };
  size_t total = 0;
  for (auto& p : parts) total = up(total + p.bytes + 16);
  const uint64_t SC = g->scope_cap;
  std::vector<Part> sparts = {
      {(void**)&g->Q.res_svc, 4 * SC}, {(void**)&g->Q.res_svc_str, 4 * SC}, {(void**)&g->Q.res_attrset, 4 * SC},
      {(void**)&g->Q.res_size, 4 * SC}, {(void**)&g->Q.scope_size, 4 * SC}, {(void**)&g->Q.res_url_ok, SC},
  };
  size_t stotal = 0;
  for (auto& p : sparts) stotal = up(stotal + p.bytes + 16);
  int rc;
  if ((rc = g->pool.need(total)) || (rc = g->scopes.need(stotal)) || (rc = g->arena.need(g->arena_cap)) ||
      (rc = g->ring.need(16 * g->ring_n)) || (rc = g->words.need(1 << 16)) ||
      (g->W > 1 && ((rc = g->tinfo.need(8 * g->ring_n)) || (rc = g->wdev.need(up(8ull * g->W) + 2 * up(4ull * g->W + 16)))))) {
    delete g;
    return rc;
  }
  size_t off = 0;
  for (auto& p : parts) {
    *p.dst = g->pool.p + off;
    off = up(off + p.bytes + 16);
  }
  off = 0;
  for (auto& p : sparts) {
    *p.dst = g->scopes.p + off;
    off = up(off + p.bytes + 16);
  }
  engine_retain(e);   // dropped by ose_gbt_destroy
  *out = reinterpret_cast<ose_gbt*>(g);
  return 0;
}

void ose_gbt_destroy(ose_gbt* gg) {
  if (!gg) return;
  LastErrorScope keep("ose_gbt_destroy");
  auto* g = reinterpret_cast<Gbt*>(gg);
  Engine* e = g->e;
  (void)bind_device(e);
  delete g;
  engine_unref(e);
}

int ose_gbt_add(ose_gbt* gg, const ose_columns* cols, const uint32_t* attrset_map, int64_t now_ns, void* hip_stream) {
  if (!gg || !cols) return fail(OSE_EINVAL, "NULL argument");
  auto* g = reinterpret_cast<Gbt*>(gg);
  if (int rc = bind_device(g->e)) return rc;
  return gbt_add(g, cols, attrset_map, now_ns, static_cast<hipStream_t>(hip_stream));
}

int ose_gbt_release(ose_gbt* gg, int64_t now_ns, void* hip_stream, const ose_columns** out, uint32_t* n_traces) {
  if (!gg || !out || !n_traces) return fail(OSE_EINVAL, "NULL argument");
  auto* g = reinterpret_cast<Gbt*>(gg);
  if (int rc = bind_device(g->e)) return rc;
  const int rc = gbt_release(g, now_ns, static_cast<hipStream_t>(hip_stream), n_traces);
  *out = &g->out_cols;
  return rc;
}

int ose_gbt_stats(const ose_gbt* gg, uint64_t* out8) {
  if (!gg || !out8) return fail(OSE_EINVAL, "NULL argument");
  const auto* g = reinterpret_cast<const Gbt*>(gg);
  out8[0] = g->waiting();                         // traces waiting
  out8[1] = g->pool_end - g->pool_begin;          // spans held (waiting or released, not yet reclaimed)
  out8[2] = g->created;
  out8[3] = g->released;
  out8[4] = g->evicted;
  out8[5] = g->released_spans;
  out8[6] = g->added_spans;
  out8[7] = g->arena_end - g->arena_begin;
  return 0;
}

// copies every column of the last release whose dst pointer is non-NULL
int ose_gbt_download(const ose_gbt* gg, const ose_columns* dst) {
  if (!gg || !dst) return fail(OSE_EINVAL, "NULL argument");
  const auto* g = reinterpret_cast<const Gbt*>(gg);
  if (int rc = bind_device(g->e)) return rc;
  const ose_columns& c = g->out_cols;
  const uint64_t n = c.n_spans, R = c.n_resources, S = c.n_scopes, K = c.n_attr_keys;
  struct F { const void* src; void* dst; size_t bytes; };
  const F fs[] = {
      {c.arena, (void*)dst->arena, c.arena_bytes}, {c.trace_id, (void*)dst->trace_id, 16 * n},
      {c.start_ns, (void*)dst->start_ns, 8 * n}, {c.end_ns, (void*)dst->end_ns, 8 * n},
      {c.status, (void*)dst->status, n}, {c.kind, (void*)dst->kind, n}, {c.resource, (void*)dst->resource, 4 * n},
      {c.scope, (void*)dst->scope, 4 * n}, {c.url_flags, (void*)dst->url_flags, n}, {c.path, (void*)dst->path, 8 * n},
      {c.route, (void*)dst->route, 8 * n}, {c.span_size, (void*)dst->span_size, 4 * n},
      {c.name_len, (void*)dst->name_len, 4 * n},
      {c.attr_match, (void*)dst->attr_match, 8 * n * std::max<uint32_t>(1, c.attr_match_words)},
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

// Test seam (CPU): Go's time.ParseDuration as the store reads wait_duration
int osehost_parse_duration(const char* s, int64_t* out) {
  if (!s || !out) return fail(OSE_EINVAL, "NULL argument");
  return parse_go_duration(s, *out) ? 0 : fail(OSE_EINVAL, std::string("time: invalid duration \"") + s + "\"");
}

}  // extern "C"
