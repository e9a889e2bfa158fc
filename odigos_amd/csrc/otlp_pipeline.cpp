// otlp_pipeline.cpp — a receiver's concurrent OTLP export requests processed
// as one device batch per wave of calls (ose_otlp_pipeline_*).
//
// Each ConsumeTraces of the OTLP path (decode -> SAMPLE | TEMPLATE | SIZE ->
// route + re-encode, otlp_host.cpp) pays a chain of launches, copies and host
// waits that an 8192-span request cannot amortise: round 5 measured 0.92 ms
// per call at one caller and 33 M spans/s at eight, no faster than the CPU
// baseline.  The pipeline lets concurrent callers share that chain:
//   * a caller reserves room for its request in the open batch's pinned
//     message buffer and copies its bytes there itself (callers copy in
//     parallel); protobuf concatenation of TracesData messages is a
//     TracesData whose resource_spans are the requests' in order;
//   * the batch's first caller (its leader) waits until fewer than
//     max_running batches are on the GPU, closes the batch and runs it on
//     the slot's stream: one decode, one stage call, one encode; the other
//     callers of the batch wait for it;
//   * every output of the batch is a sequence of ResourceSpans records in
//     resource order, so request q's part of output k is the byte range from
//     the record offset of its first resource to that of the next request's
//     (the encoder's own per-output scan): a valid TracesData, byte for byte
//     what the encoder writes for that request's resources.
// At low load a batch holds one request and runs at once; under load the
// requests that arrive while batches run form the next one.
//
// Semantics against one call per request: the batch is one SAMPLE call with
// OSE_GROUP_TRACE_ID, so spans of one trace that arrive in concurrent
// requests are decided together (as groupbytrace would hand them to
// odigossampling, sampling_controller.go:193-220); the traffic gate draws
// once per batch (the leader's traffic_u); the traffic counters are summed
// per attribute set over all requests (ose_otlp_pipeline_counters).
// Requests the batch cannot take (malformed top level, larger than a batch,
// a batch the decoder or the GPU encoder declines) run alone through the
// same calls, with the same results a single call would have.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/odigos_amd.h"
#include "engine_internal.hpp"
#include "otlp_encode.hpp"

namespace ose {
int otlp_encode_gpu_offsets(Engine* e, ose_otlp_batch* bb, const ose_outputs* outs, uint32_t stages,
                            const Router* router, hipStream_t st, OtlpOut** out, std::vector<uint64_t>& res_off,
                            bool* gpu);

namespace {

#define PIPE_TRY(expr)                                                                              \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// ResourceSpans records (field 1, length-delimited) at the top level of a
// TracesData; -1 when the top level is not well-formed protobuf (the
// request then runs alone, where the decoder reports the error).
int64_t count_resource_spans(const uint8_t* p, size_t len) {
  size_t i = 0;
  int64_t n = 0;
  auto varint = [&](uint64_t& v) {
    v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (i >= len) return false;
      const uint8_t b = p[i++];
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return true;
    }
    return false;
  };
  while (i < len) {
    uint64_t tag, v;
    if (!varint(tag) || (tag >> 3) == 0) return -1;
    switch (tag & 7) {
      case 0:
        if (!varint(v)) return -1;
        break;
      case 1:
        if (len - i < 8) return -1;
        i += 8;
        break;
      case 5:
        if (len - i < 4) return -1;
        i += 4;
        break;
      case 2:
        if (!varint(v) || v > len - i) return -1;
        i += v;
        if ((tag >> 3) == 1) n++;
        break;
      default:
        return -1;   // groups: the decoder's error
    }
  }
  return n;
}

struct DBuf {   // grow-only device buffer
  uint8_t* p = nullptr;
  size_t cap = 0;
  int need(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    PIPE_TRY(hipMalloc(reinterpret_cast<void**>(&p), want));
    cap = want;
    return 0;
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

struct Req {
  const uint8_t* pb = nullptr;
  size_t len = 0;
  ose_rand rnd{0, 0.0};
  uint64_t off = 0;     // in the batch message
  uint32_t n_res = 0;   // its ResourceSpans records
  bool done = false;
  int rc = 0;
  std::string err;
  OtlpOut* out = nullptr;
};

struct Slot {
  hipStream_t st = nullptr;
  uint8_t* msg = nullptr;   // pinned, max_bytes
  DBuf keep, url, tmpl, arena, sets, misc;   // the stages' device outputs
  uint64_t* host_misc = nullptr;              // pinned: status, accepted, the attribute-set counters
  size_t host_misc_cap = 0;
  enum State { Idle, Filling, Running } state = Idle;
  std::vector<Req*> reqs;
  size_t used = 0;
  int copying = 0;
  bool closed = false;
  Req* leader = nullptr;
};

}  // namespace

struct Pipeline {
  Engine* e = nullptr;
  const Router* router = nullptr;
  uint32_t stages = 0;
  size_t max_bytes = 0;
  int max_running = 4;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::unique_ptr<Slot>> slots;
  int filling = -1;
  int running = 0;
  size_t hold = 0;   // test seam (osehost_otlp_pipeline_hold): a leader waits for this many requests
  // batching window: under load (the last batch held several requests) a
  // leader whose slot is free still waits up to window_us for requests to
  // join, until the batch holds target requests; at low load it runs at once
  uint32_t window_us = 200;
  size_t target = 8;
  size_t last_q = 0;
  std::mutex single_mu;   // requests that run alone share one slot
  std::unique_ptr<Slot> single;
  std::mutex cmu;   // counters
  std::map<std::string, int64_t> set_bytes;
  int64_t accepted = 0;
  uint64_t n_batches = 0, n_requests = 0, n_singles = 0, max_batch = 0;
  double t_ms[5] = {0, 0, 0, 0, 0};   // batches: wait (window + copies), decode + stages, encode, slices, total
};

namespace {

int slot_init(Slot& s, size_t max_bytes) {
  PIPE_TRY(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
  if (max_bytes) PIPE_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.msg), max_bytes + 16, hipHostMallocDefault));
  return 0;
}
void slot_free(Slot& s) {
  if (s.st) (void)hipStreamDestroy(s.st);
  if (s.msg) (void)hipHostFree(s.msg);
  if (s.host_misc) (void)hipHostFree(s.host_misc);
  s.st = nullptr;
  s.msg = nullptr;
  s.host_misc = nullptr;
}

// decode -> stages -> (counters) on the slot's stream; *bb is the decoded
// batch (release it), outs the outputs the encoder reads
int run_front(Pipeline* p, Slot& s, const uint8_t* pb, size_t len, const ose_rand& rnd, ose_otlp_batch** bb,
              ose_outputs& outs) {
  Engine* e = p->e;
  ose_engine* eng = reinterpret_cast<ose_engine*>(e);
  *bb = nullptr;
  int rc = ose_otlp_decode(eng, pb, len, s.st, bb);
  if (rc) return rc;
  const ose_columns* c = ose_otlp_columns(*bb);
  const uint64_t n = std::max<uint64_t>(c->n_spans, 1), sets = std::max<uint32_t>(c->n_attrsets, 1);
  // templates: at most the path bytes plus a brace pair per segment, well
  // inside the message bytes plus 64 B per span
  const uint64_t tcap = len + 64 * n;
  if ((rc = s.keep.need(n)) || (rc = s.url.need(n)) || (rc = s.tmpl.need(8 * n)) || (rc = s.arena.need(tcap)) ||
      (rc = s.sets.need(8 * sets)) || (rc = s.misc.need(64)))
    return rc;
  outs = ose_outputs{};
  outs.keep = s.keep.p;
  outs.url_out = s.url.p;
  outs.tmpl = reinterpret_cast<ose_strref*>(s.tmpl.p);
  outs.tmpl_arena = s.arena.p;
  outs.tmpl_arena_cap = tcap;
  outs.tmpl_arena_used = reinterpret_cast<uint64_t*>(s.misc.p);
  outs.accepted_spans = reinterpret_cast<int64_t*>(s.misc.p + 8);
  outs.device_status = reinterpret_cast<uint32_t*>(s.misc.p + 16);
  outs.attrset_bytes = reinterpret_cast<int64_t*>(s.sets.p);
  PIPE_TRY(hipMemsetAsync(s.misc.p, 0, 64, s.st));
  PIPE_TRY(hipMemsetAsync(s.sets.p, 0, 8 * sets, s.st));
  return ose_process_device(eng, c, &outs, p->stages, OSE_GROUP_TRACE_ID, &rnd, s.st);
}

// the device status word and the traffic counters after the stages: the
// copies are queued behind the stages (issue_counters) and read once the
// encoder has synchronised the stream (take_counters), so they cost no wait
// of their own
int issue_counters(Slot& s, ose_otlp_batch* bb) {
  const uint32_t sets = ose_otlp_columns(bb)->n_attrsets;
  const size_t need = 8 * (4 + (size_t)sets);
  if (need > s.host_misc_cap) {
    if (s.host_misc) (void)hipHostFree(s.host_misc);
    s.host_misc = nullptr;
    s.host_misc_cap = 0;
    PIPE_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.host_misc), need * 2, hipHostMallocDefault));
    s.host_misc_cap = need * 2;
  }
  PIPE_TRY(hipMemcpyAsync(s.host_misc, s.misc.p, 32, hipMemcpyDeviceToHost, s.st));
  if (sets) PIPE_TRY(hipMemcpyAsync(s.host_misc + 4, s.sets.p, 8 * (size_t)sets, hipMemcpyDeviceToHost, s.st));
  return 0;
}
int take_counters(Pipeline* p, Slot& s, ose_otlp_batch* bb) {
  PIPE_TRY(hipStreamSynchronize(s.st));   // (already synchronised by the encoder: returns at once)
  const uint32_t sets = ose_otlp_columns(bb)->n_attrsets;
  const uint32_t status = (uint32_t)s.host_misc[2];
  if (status) return fail(OSE_EDEVICE, "OTLP pipeline: device status " + std::to_string(status));
  if (!(p->stages & OSE_STAGE_SIZE)) return 0;
  std::vector<std::pair<std::string, int64_t>> add;
  char buf[4096];
  for (uint32_t k = 0; k < sets; k++) {
    const int64_t v = (int64_t)s.host_misc[4 + k];
    if (!v) continue;
    std::string key = ose_otlp_attrset(bb, k, buf, sizeof buf) == 0 ? std::string(buf) : std::string("{}");
    add.emplace_back(std::move(key), v);
  }
  std::lock_guard<std::mutex> g(p->cmu);
  p->accepted += (int64_t)s.host_misc[1];
  for (auto& kv : add) p->set_bytes[kv.first] += kv.second;
  return 0;
}

// one request through the ordinary calls (ose_otlp_encode, host fallback
// included): what a call without the pipeline returns
void run_alone(Pipeline* p, Slot& s, Req& r, const uint8_t* pb) {
  ose_otlp_batch* bb = nullptr;
  ose_outputs outs{};
  int rc = run_front(p, s, pb, r.len, r.rnd, &bb, outs);
  if (!rc) rc = issue_counters(s, bb);
  ose_otlp_out* o = nullptr;
  if (!rc)
    rc = ose_otlp_encode(reinterpret_cast<ose_engine*>(p->e), bb, &outs, p->stages, OSE_GROUP_TRACE_ID,
                         reinterpret_cast<const ose_router*>(p->router), s.st, &o);
  if (!rc) rc = take_counters(p, s, bb);
  if (rc && o) {
    ose_otlp_out_release(o);
    o = nullptr;
  }
  if (rc) r.err = ose_last_error();
  if (bb) ose_otlp_release(bb);
  r.rc = rc;
  r.out = reinterpret_cast<OtlpOut*>(o);
  std::lock_guard<std::mutex> g(p->cmu);
  p->n_singles++;
}

using pclk = std::chrono::steady_clock;
double ms_since(pclk::time_point t) { return std::chrono::duration<double, std::milli>(pclk::now() - t).count(); }

void run_batch(Pipeline* p, Slot& s) {
  const size_t Q = s.reqs.size();
  const auto t0 = pclk::now();
  auto each_alone = [&]() {
    for (Req* r : s.reqs) run_alone(p, s, *r, s.msg + r->off);
  };
  if (Q == 1) {   // one request: the ordinary calls (the host encoder stays available)
    run_alone(p, s, *s.reqs[0], s.msg);
    return;
  }
  ose_otlp_batch* bb = nullptr;
  ose_outputs outs{};
  int rc = run_front(p, s, s.msg, s.used, s.reqs[0]->rnd, &bb, outs);
  const ose_columns* c = bb ? ose_otlp_columns(bb) : nullptr;
  uint64_t R = 0;
  for (Req* r : s.reqs) R += r->n_res;
  if (rc || !c || c->n_resources != R) {   // the decoder refused the batch: find whose request it was
    if (bb) ose_otlp_release(bb);
    (void)hipStreamSynchronize(s.st);
    each_alone();
    return;
  }
  const double t_front = ms_since(t0);
  const auto t1 = pclk::now();
  OtlpOut* whole = nullptr;
  std::vector<uint64_t> off;
  bool gpu = false;
  rc = issue_counters(s, bb);
  if (!rc) rc = otlp_encode_gpu_offsets(p->e, bb, &outs, p->stages, p->router, s.st, &whole, off, &gpu);
  if (!rc && gpu) rc = take_counters(p, s, bb);
  if (rc || !gpu) {   // an error, or a batch the GPU encoder hands to the host encoder
    if (whole) otlp_out_release(whole);
    ose_otlp_release(bb);
    if (!rc) {   // (the stages' counters were not collected: the requests run again alone)
      each_alone();
      return;
    }
    const std::string err = ose_last_error();
    for (Req* r : s.reqs) {
      r->rc = rc;
      r->err = err;
    }
    return;
  }
  ose_otlp_release(bb);
  const double t_enc = ms_since(t1);
  const auto t2 = pclk::now();
  std::shared_ptr<OtlpOut> hold(whole, [](OtlpOut* o) { otlp_out_release(o); });
  const size_t n_out = whole->outs.size();
  uint64_t r0 = 0;
  for (Req* r : s.reqs) {
    const uint64_t r1 = r0 + r->n_res;
    auto* o = new OtlpOut();
    o->e = p->e;
    engine_retain(p->e);
    o->hold = hold;
    o->gpu = 1;
    o->outs.resize(n_out);
    for (size_t k = 0; k < n_out; k++) {
      const EncodedOutput& w = whole->outs[k];
      const uint64_t* ok = off.data() + k * R;
      const uint64_t lo = r0 < R ? ok[r0] : w.len, hi = r1 < R ? ok[r1] : w.len;
      EncodedOutput& x = o->outs[k];
      x.name = w.name;
      x.data = w.data + lo;
      x.len = hi - lo;
      x.cap = 0;
      // the records in the slice: resources whose record has bytes in this
      // output (from the offsets: the output bytes are pinned memory, slow
      // for the host to read)
      uint32_t nr = 0;
      for (uint64_t q = r0; q < r1; q++) nr += (q + 1 < R ? ok[q + 1] : w.len) > ok[q];
      x.n_resources = nr;
    }
    r->out = o;
    r->rc = 0;
    r0 = r1;
  }
  std::lock_guard<std::mutex> g(p->cmu);
  p->n_batches++;
  p->n_requests += Q;
  p->max_batch = std::max<uint64_t>(p->max_batch, Q);
  p->t_ms[1] += t_front;
  p->t_ms[2] += t_enc;
  p->t_ms[3] += ms_since(t2);
  p->t_ms[4] += ms_since(t0);
}

int consume(Pipeline* p, const uint8_t* pb, size_t len, const ose_rand* rnd, OtlpOut** out) {
  Req r;
  r.pb = pb;
  r.len = len;
  if (rnd) r.rnd = *rnd;
  const int64_t nres = count_resource_spans(pb, len);
  if (nres < 0 || len > p->max_bytes) {   // alone, on the shared single slot
    std::lock_guard<std::mutex> g(p->single_mu);
    run_alone(p, *p->single, r, pb);
    *out = r.out;
    return r.rc ? fail(r.rc, r.err) : 0;
  }
  r.n_res = (uint32_t)nres;
  std::unique_lock<std::mutex> lk(p->mu);
  int si = -1;
  for (;;) {
    if (p->filling < 0) {
      for (size_t k = 0; k < p->slots.size(); k++)
        if (p->slots[k]->state == Slot::Idle) {
          Slot& s = *p->slots[k];
          s.state = Slot::Filling;
          s.used = 0;
          s.closed = false;
          s.reqs.clear();
          s.leader = &r;
          p->filling = (int)k;
          break;
        }
      if (p->filling < 0) {
        p->cv.wait(lk);
        continue;
      }
    }
    Slot& s = *p->slots[p->filling];
    if (s.used + len > p->max_bytes) {   // full: the next request opens another batch
      s.closed = true;
      p->filling = -1;
      p->cv.notify_all();
      continue;
    }
    r.off = s.used;
    s.used += len;
    s.reqs.push_back(&r);
    s.copying++;
    si = p->filling;
    break;
  }
  Slot& s = *p->slots[si];
  // every caller copies its own bytes, outside the lock and in parallel (a
  // leader that deferred its copy until it knew it had company measured
  // slower: its copy then sits on the batch's critical path)
  lk.unlock();
  if (len) std::memcpy(s.msg + r.off, pb, len);
  lk.lock();
  s.copying--;
  p->cv.notify_all();
  if (s.leader == &r) {
    const auto tw = pclk::now();
    // run when fewer than max_running batches are on the GPU; requests keep
    // joining this batch until then
    p->cv.wait(lk, [&] { return p->running < p->max_running && (s.reqs.size() >= p->hold || s.closed); });
    if (p->window_us && p->last_q > 1 && !s.closed && s.reqs.size() < p->target) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(p->window_us);
      p->cv.wait_until(lk, until, [&] { return s.closed || s.reqs.size() >= p->target; });
    }
    p->last_q = s.reqs.size();
    if (p->filling == si) p->filling = -1;
    s.state = Slot::Running;
    p->running++;
    p->cv.wait(lk, [&] { return s.copying == 0; });
    const double waited = ms_since(tw);
    lk.unlock();
    {
      std::lock_guard<std::mutex> g(p->cmu);
      p->t_ms[0] += waited;
    }
    if (int brc = bind_device(p->e)) {
      for (Req* q : s.reqs) {
        q->rc = brc;
        q->err = ose_last_error();
      }
    } else {
      run_batch(p, s);
    }
    lk.lock();
    for (Req* q : s.reqs) q->done = true;
    s.reqs.clear();
    s.leader = nullptr;
    s.state = Slot::Idle;
    p->running--;
    p->cv.notify_all();
  } else {
    p->cv.wait(lk, [&] { return r.done; });
  }
  lk.unlock();
  *out = r.out;
  return r.rc ? fail(r.rc, r.err) : 0;
}

}  // namespace
}  // namespace ose

using namespace ose;

extern "C" {

int ose_otlp_pipeline_create(ose_engine* eng, const ose_router* router, uint32_t stages, uint64_t max_batch_bytes,
                             ose_otlp_pipeline** out) {
  if (!eng || !out) return fail(OSE_EINVAL, "NULL argument");
  *out = nullptr;
  if (stages & ~(OSE_STAGE_SAMPLE | OSE_STAGE_TEMPLATE | OSE_STAGE_SIZE))
    return fail(OSE_EINVAL, "the pipeline runs SAMPLE, TEMPLATE and SIZE only");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (int rc = bind_device(e)) return rc;
  auto* p = new Pipeline();
  p->e = e;
  p->router = reinterpret_cast<const Router*>(router);
  p->stages = stages;
  p->max_bytes = max_batch_bytes ? max_batch_bytes : (64ull << 20);
  for (int k = 0; k < 3; k++) {
    p->slots.emplace_back(new Slot());
    if (int rc = slot_init(*p->slots.back(), p->max_bytes)) {
      for (auto& s : p->slots) slot_free(*s);
      delete p;
      return rc;
    }
  }
  p->single.reset(new Slot());
  if (int rc = slot_init(*p->single, 0)) {
    for (auto& s : p->slots) slot_free(*s);
    delete p;
    return rc;
  }
  engine_retain(e);
  *out = reinterpret_cast<ose_otlp_pipeline*>(p);
  return 0;
}

int ose_otlp_pipeline_consume(ose_otlp_pipeline* pp, const void* pb, size_t len, const ose_rand* rnd,
                              ose_otlp_out** out) {
  if (!pp || (!pb && len) || !out) return fail(OSE_EINVAL, "NULL argument");
  *out = nullptr;
  auto* p = reinterpret_cast<Pipeline*>(pp);
  OtlpOut* o = nullptr;
  const int rc = consume(p, static_cast<const uint8_t*>(pb), len, rnd, &o);
  *out = reinterpret_cast<ose_otlp_out*>(o);
  return rc;
}

int ose_otlp_pipeline_counters(ose_otlp_pipeline* pp, char* json, size_t cap) {
  if (!pp || !json) return fail(OSE_EINVAL, "NULL argument");
  auto* p = reinterpret_cast<Pipeline*>(pp);
  std::string s;
  {
    std::lock_guard<std::mutex> g(p->cmu);
    s = "{\"accepted_spans\":" + std::to_string(p->accepted) + ",\"batches\":" + std::to_string(p->n_batches) +
        ",\"batched_requests\":" + std::to_string(p->n_requests) + ",\"alone\":" + std::to_string(p->n_singles) +
        ",\"largest_batch\":" + std::to_string(p->max_batch) + ",\"batch_ms\":{\"wait\":" + std::to_string(p->t_ms[0]) +
        ",\"decode_stages\":" + std::to_string(p->t_ms[1]) + ",\"encode\":" + std::to_string(p->t_ms[2]) +
        ",\"slices\":" + std::to_string(p->t_ms[3]) + ",\"total\":" + std::to_string(p->t_ms[4]) + "},\"data_size\":[";
    bool first = true;
    for (auto& kv : p->set_bytes) {
      s += first ? "[" : ",[";
      first = false;
      s += kv.first + "," + std::to_string(kv.second) + "]";
    }
    s += "]}";
    if (s.size() + 1 > cap) return fail(OSE_ERANGE, "buffer too small");
    p->accepted = 0;
    p->set_bytes.clear();
    p->n_batches = p->n_requests = p->n_singles = p->max_batch = 0;
    for (double& t : p->t_ms) t = 0;
  }
  std::memcpy(json, s.c_str(), s.size() + 1);
  return 0;
}

// diagnostics: how many batches may be on the GPU at once (1..8; one more
// slot fills meanwhile), the batching window and its target batch size
int osehost_otlp_pipeline_tune(ose_otlp_pipeline* pp, uint32_t max_running, uint32_t window_us, uint32_t target) {
  if (!pp || max_running < 1 || max_running > 8) return fail(OSE_EINVAL, "max_running must be in 1..8");
  auto* p = reinterpret_cast<Pipeline*>(pp);
  std::lock_guard<std::mutex> g(p->mu);
  p->window_us = window_us;
  p->target = std::max<uint32_t>(target, 1);
  while (p->slots.size() < max_running + 1) {
    p->slots.emplace_back(new Slot());
    if (int rc = slot_init(*p->slots.back(), p->max_bytes)) return rc;
  }
  p->max_running = (int)max_running;
  p->cv.notify_all();
  return 0;
}

// test seam: the next batches run only once `n` requests joined them (or
// they are full), so a test decides what one batch holds
int osehost_otlp_pipeline_hold(ose_otlp_pipeline* pp, uint32_t n) {
  if (!pp) return fail(OSE_EINVAL, "NULL argument");
  auto* p = reinterpret_cast<Pipeline*>(pp);
  std::lock_guard<std::mutex> g(p->mu);
  p->hold = n;
  p->cv.notify_all();
  return 0;
}

void ose_otlp_pipeline_destroy(ose_otlp_pipeline* pp) {
  if (!pp) return;
  LastErrorScope keep("ose_otlp_pipeline_destroy");
  auto* p = reinterpret_cast<Pipeline*>(pp);
  (void)bind_device(p->e);
  for (auto& s : p->slots) {
    if (s->st) (void)hipStreamSynchronize(s->st);
    slot_free(*s);
  }
  if (p->single) {
    if (p->single->st) (void)hipStreamSynchronize(p->single->st);
    slot_free(*p->single);
  }
  Engine* e = p->e;
  p->slots.clear();
  p->single.reset();
  delete p;
  engine_unref(e);
}

}  // extern "C"
