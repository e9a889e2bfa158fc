// batch.cpp — engine-owned pinned host staging (ose_batch_*) and the
// synchronous ose_process path used by the host processors / a cgo shim.
//
// A batch is one pinned host slab and one device slab with the same layout,
// so a call moves the data in four copies whatever the column count:
//   H2D  [counters, status]            (ADDED-to counters, status cleared)
//   H2D  [input columns ... arena]     (up to the arena bytes actually used)
//   D2H  [counters, status ... core outputs] then, after one sync,
//   D2H  tmpl_arena (the bytes the kernels wrote) and any optional outputs
// Released batches go back to a per-engine pool: ConsumeTraces calls (one per
// trace behind groupbytrace) acquire and release one each, and pinned /
// device allocations (which synchronise the device) must not sit on that
// path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/odigos_amd.h"
#include "engine_internal.hpp"

namespace ose {

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {
constexpr size_t kAlign = 256;
constexpr size_t kPoolMax = 64;                    // pooled batches per engine
constexpr size_t kPoolBytesMax = size_t(8) << 30;  // pinned bytes kept pooled per engine
size_t up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }
}  // namespace

struct Batch {
  Engine* e = nullptr;
  ose_columns cols_h{}, cols_d{};
  ose_outputs outs_h{}, outs_d{};
  ose_columns cap{};        // capacities (n_spans, n_resources, ..., arena_bytes, n_attr_keys)
  uint64_t tmpl_cap = 0;
  uint64_t used_h = 0;
  uint8_t* h = nullptr;     // pinned slab
  uint8_t* d = nullptr;     // device slab
  size_t bytes = 0;
  // regions (byte offsets into both slabs)
  size_t ctr_off = 0, ctr_end = 0;     // attrset_bytes, accepted_spans, device_status (+ used)
  size_t in_off = 0, arena_off = 0;    // input columns, then the arena
  size_t core_off = 0, core_end = 0;   // core outputs (keep .. tmpl): one D2H
  size_t tmpl_off = 0;
  struct Opt { size_t off, bytes; void** hslot; };
  std::vector<Opt> optional;           // trace_first_span, trace_level, trace_ratio, res_bytes
  struct Field { void** hs; void** ds; size_t off; };
  std::vector<Field> fields;           // every column / output of the slab layout
  // a tmpl_arena regrown past the slab (rare: see ose_process)
  uint8_t* tmpl_h_big = nullptr;
  uint8_t* tmpl_d_big = nullptr;

  ~Batch() {
    if (h) (void)hipHostFree(h);
    if (d) (void)hipFree(d);
    if (tmpl_h_big) (void)hipHostFree(tmpl_h_big);
    if (tmpl_d_big) (void)hipFree(tmpl_d_big);
  }
  bool fits(const ose_columns& x) const {
    return x.n_spans <= cap.n_spans && x.n_resources <= cap.n_resources && x.n_scopes <= cap.n_scopes &&
           x.n_attrsets <= cap.n_attrsets && x.arena_bytes <= cap.arena_bytes && x.n_attr_keys <= cap.n_attr_keys &&
           std::max<uint32_t>(1, x.attr_match_words) <= cap.attr_match_words;
  }
  int build(const ose_columns& dims);
  void set_dims(const ose_columns& dims);
};

int Batch::build(const ose_columns& dims) {
  cap = ose_columns{};
  cap.n_spans = dims.n_spans;
  cap.n_resources = dims.n_resources;
  cap.n_scopes = dims.n_scopes;
  cap.n_attrsets = dims.n_attrsets;
  cap.arena_bytes = dims.arena_bytes;
  cap.n_attr_keys = dims.n_attr_keys;
  cap.attr_match_words = std::max<uint32_t>(1, dims.attr_match_words);
  const uint64_t n = cap.n_spans, R = cap.n_resources, S = cap.n_scopes, A = cap.n_attrsets, K = cap.n_attr_keys;
  const uint64_t n1 = std::max<uint64_t>(n, 1);   // BATCH mode: one trace even with no spans
  // every template fits in 2x the input bytes + 8 per span; capped at the
  // 32-bit offset range of ose_strref (an overflow regrows it in ose_process)
  tmpl_cap = std::min<uint64_t>(2 * dims.arena_bytes + 8 * n + 4096, 0xFFFFFFF0ull);
  fields.clear();
  size_t off = 0;
  auto place = [&](void** hs, void** ds, size_t b) {
    fields.push_back(Field{hs, ds, off});
    off = up(off + b + 16);   // +16: ByteReader 16-byte loads past a column's end
    return fields.back().off;
  };
#define IN(f, b) place((void**)&cols_h.f, (void**)&cols_d.f, (size_t)(b))
#define OUT(f, b) place((void**)&outs_h.f, (void**)&outs_d.f, (size_t)(b))
  ctr_off = off;
  OUT(attrset_bytes, 8 * A);
  OUT(accepted_spans, 8);
  OUT(device_status, 16);   // [0] status, [8..15] tmpl_arena_used
  ctr_end = off;
  in_off = off;
  IN(trace_id, 16 * n);
  IN(start_ns, 8 * n);
  IN(end_ns, 8 * n);
  IN(status, n);
  IN(kind, n);
  IN(resource, 4 * n);
  IN(scope, 4 * n);
  IN(url_flags, n);
  IN(path, 8 * n);
  IN(route, 8 * n);
  IN(span_size, 4 * n);
  IN(name_len, 4 * n);   // route_match stays NULL: host batches carry route bytes
  IN(attr_match, 8 * n * cap.attr_match_words);   // word-major planes of the call's n_spans
  IN(res_svc, 4 * R);
  IN(res_svc_str, 4 * R);
  IN(res_url_ok, R);
  IN(res_attrset, 4 * R);
  IN(res_size, 4 * R);
  IN(scope_size, 4 * S);
  IN(scope_resource, 4 * S);
  if (K) {
    IN(attr_type, K * n);
    IN(attr_val, 8 * K * n);
  }
  arena_off = IN(arena, dims.arena_bytes);
  core_off = off;
  OUT(keep, n);
  OUT(trace_count, 4);
  OUT(trace_keep, n1);
  OUT(url_out, n);
  OUT(tmpl, 8 * n);
  core_end = off;
  const size_t o_first = OUT(trace_first_span, 4 * n1);
  const size_t o_level = OUT(trace_level, n1);
  const size_t o_ratio = OUT(trace_ratio, 8 * n1);
  const size_t o_res = OUT(res_bytes, 8 * R);
  tmpl_off = OUT(tmpl_arena, tmpl_cap);
#undef IN
#undef OUT
  bytes = off;
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&h), bytes, hipHostMallocDefault));
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), bytes));
  std::memset(h, 0, bytes);
  HIP_TRY(hipMemset(d, 0, bytes));
  optional = {{o_first, 4 * n1, (void**)&outs_h.trace_first_span},
              {o_level, n1, (void**)&outs_h.trace_level},
              {o_ratio, 8 * n1, (void**)&outs_h.trace_ratio},
              {o_res, 8 * R, (void**)&outs_h.res_bytes}};
  outs_h.tmpl_arena_cap = outs_d.tmpl_arena_cap = tmpl_cap;
  set_dims(dims);
  return 0;
}

// (re)binds a pooled batch to a call's dimensions: the pointers of the
// capacity layout are restored (the shim may have NULLed optional outputs)
void Batch::set_dims(const ose_columns& dims) {
  for (ose_columns* c : {&cols_h, &cols_d}) {
    c->n_spans = dims.n_spans;
    c->n_resources = dims.n_resources;
    c->n_scopes = dims.n_scopes;
    c->n_attrsets = dims.n_attrsets;
    c->arena_bytes = dims.arena_bytes;
    c->n_attr_keys = dims.n_attr_keys;
    c->attr_match_words = std::max<uint32_t>(1, dims.attr_match_words);
  }
  // every pointer back to the slab (the shim NULLs columns it does not fill)
  for (auto& f : fields) {
    *f.hs = h + f.off;
    *f.ds = d + f.off;
  }
  if (tmpl_h_big) {
    outs_h.tmpl_arena = tmpl_h_big;
    outs_d.tmpl_arena = tmpl_d_big;
  }
  // the device's tmpl_arena_used lives in device_status's slack (read back
  // with the counters); the shim reads used_h
  outs_h.tmpl_arena_used = &used_h;
  outs_d.tmpl_arena_used = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(outs_d.device_status) + 8);
  used_h = 0;
}

void release_batch_pool(Engine* e) {
  for (void* p : e->batch_pool) delete static_cast<Batch*>(p);
  e->batch_pool.clear();
  e->batch_pool_bytes = 0;
}

}  // namespace ose

using namespace ose;

extern "C" {

int ose_batch_acquire(ose_engine* eng, const ose_columns* dims, ose_batch** out) {
  if (!eng || !dims || !out) return fail(OSE_EINVAL, "NULL argument");
  int rc = ensure_device();
  if (rc) return rc;
  Engine* e = reinterpret_cast<Engine*>(eng);
  rc = bind_device(e);
  if (rc) return rc;
  {
    // smallest pooled batch that fits
    std::lock_guard<std::mutex> g(e->mu);
    size_t best = e->batch_pool.size();
    for (size_t k = 0; k < e->batch_pool.size(); k++) {
      Batch* b = static_cast<Batch*>(e->batch_pool[k]);
      if (b->fits(*dims) && (best == e->batch_pool.size() || b->bytes < static_cast<Batch*>(e->batch_pool[best])->bytes))
        best = k;
    }
    if (best < e->batch_pool.size()) {
      Batch* b = static_cast<Batch*>(e->batch_pool[best]);
      // a pooled batch far larger than the call would keep idle pinned memory busy
      if (b->cap.n_spans <= 4 * std::max<uint64_t>(dims->n_spans, 4096)) {
        e->batch_pool.erase(e->batch_pool.begin() + (long)best);
        e->batch_pool_bytes -= b->bytes;
        b->set_dims(*dims);
        engine_retain(e);
        *out = reinterpret_cast<ose_batch*>(b);
        return 0;
      }
    }
  }
  auto* b = new Batch();
  b->e = e;
  rc = b->build(*dims);
  if (rc) { delete b; return rc; }
  engine_retain(e);
  *out = reinterpret_cast<ose_batch*>(b);
  return 0;
}

ose_columns* ose_batch_columns(ose_batch* bb) { return bb ? &reinterpret_cast<Batch*>(bb)->cols_h : nullptr; }
ose_outputs* ose_batch_outputs(ose_batch* bb) { return bb ? &reinterpret_cast<Batch*>(bb)->outs_h : nullptr; }

void ose_batch_release(ose_batch* bb) {
  if (!bb) return;
  LastErrorScope keep("ose_batch_release");
  Batch* b = reinterpret_cast<Batch*>(bb);
  Engine* e = b->e;
  (void)bind_device(e);
  bool pooled = false;
  if (!e->closed.load()) {
    std::lock_guard<std::mutex> g(e->mu);
    if (!b->tmpl_h_big && e->batch_pool.size() < kPoolMax && e->batch_pool_bytes + b->bytes <= kPoolBytesMax) {
      e->batch_pool.push_back(b);
      e->batch_pool_bytes += b->bytes;
      pooled = true;
    }
  }
  if (!pooled) delete b;
  engine_unref(e);
}

int ose_process(ose_engine* eng, ose_batch* bb, uint32_t stage_mask, uint32_t group_mode, const ose_rand* rnd) {
  if (!eng || !bb) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  Batch* b = reinterpret_cast<Batch*>(bb);
  if (!b->fits(b->cols_h)) return fail(OSE_EINVAL, "batch dimensions exceed the acquired capacity");
  if (stage_mask & OSE_STAGE_TEMPLATE_REFS)
    return fail(OSE_EINVAL, "OSE_STAGE_TEMPLATE_REFS is for ose_process_device (ose_process copies the packed arena)");
  if (int brc = bind_device(e)) return brc;
  hipStream_t st = e->take_stream();
  if (!st) return fail(OSE_EDEVICE, "hipStreamCreate failed");
  struct GiveBack {
    Engine* e;
    hipStream_t s;
    ~GiveBack() { e->give_stream(s); }
  } give_back{e, st};
  // sizes the shim may have shrunk after acquire (n_spans etc. <= capacity)
  b->cols_d.n_spans = b->cols_h.n_spans;
  b->cols_d.n_resources = b->cols_h.n_resources;
  b->cols_d.n_scopes = b->cols_h.n_scopes;
  b->cols_d.n_attrsets = b->cols_h.n_attrsets;
  b->cols_d.arena_bytes = b->cols_h.arena_bytes;
  b->cols_d.n_attr_keys = b->cols_h.n_attr_keys;
  // the device view: columns / outputs the shim NULLed are absent for this call
  ose_outputs od = b->outs_d;
  ose_columns cd = b->cols_d;
  for (auto& f : b->fields) {
    if (*f.hs) continue;
    uint8_t* ds = reinterpret_cast<uint8_t*>(f.ds);
    uint8_t* cbase = reinterpret_cast<uint8_t*>(&b->cols_d);
    uint8_t* obase = reinterpret_cast<uint8_t*>(&b->outs_d);
    if (ds >= cbase && ds < cbase + sizeof(ose_columns))
      *reinterpret_cast<void**>(reinterpret_cast<uint8_t*>(&cd) + (ds - cbase)) = nullptr;
    else
      *reinterpret_cast<void**>(reinterpret_cast<uint8_t*>(&od) + (ds - obase)) = nullptr;
  }
  if (!cd.attr_type || !cd.attr_val) cd.attr_type = nullptr, cd.attr_val = nullptr, cd.n_attr_keys = 0;
  if (!od.device_status || !od.attrset_bytes || !od.accepted_spans || !od.tmpl_arena)
    return fail(OSE_EINVAL, "ose_process: device_status, attrset_bytes, accepted_spans and tmpl_arena must stay set");
  {
    // every device pointer a kernel gets lies in this batch's device memory
    auto inside = [&](const void* p) {
      const uint8_t* q = static_cast<const uint8_t*>(p);
      return !p || (q >= b->d && q < b->d + b->bytes) || (b->tmpl_d_big && q == b->tmpl_d_big);
    };
    bool ok = inside(od.tmpl_arena_used);
    for (auto& f : b->fields) {
      const uint8_t* ds = reinterpret_cast<const uint8_t*>(f.ds);
      const uint8_t* cbase = reinterpret_cast<const uint8_t*>(&b->cols_d);
      const void* p = (ds >= cbase && ds < cbase + sizeof(ose_columns))
                          ? *reinterpret_cast<void* const*>(reinterpret_cast<const uint8_t*>(&cd) + (ds - cbase))
                          : *reinterpret_cast<void* const*>(reinterpret_cast<const uint8_t*>(&od) +
                                                            (ds - reinterpret_cast<const uint8_t*>(&b->outs_d)));
      ok = ok && inside(p);
    }
    if (!ok) return fail(OSE_EINVAL, "ose_process: a device pointer of the batch lies outside its memory");
  }
  uint32_t* status_h = b->outs_h.device_status;
  uint64_t* used_h = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(status_h) + 8);
  // the counters are ADDED to on the device: keep the caller's values for a rerun
  std::vector<uint8_t> ctr_saved(b->h + b->ctr_off, b->h + b->ctr_end);
  for (int attempt = 0; attempt < 2; attempt++) {
    if (attempt) std::memcpy(b->h + b->ctr_off, ctr_saved.data(), ctr_saved.size());
    std::memset(status_h, 0, 16);
    HIP_TRY(hipMemcpyAsync(b->d + b->ctr_off, b->h + b->ctr_off, b->ctr_end - b->ctr_off, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(b->d + b->in_off, b->h + b->in_off, b->arena_off - b->in_off + b->cols_h.arena_bytes,
                           hipMemcpyHostToDevice, st));
    int rc = run_stages(e, &cd, &od, stage_mask, group_mode, rnd, st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(b->h + b->ctr_off, b->d + b->ctr_off, b->ctr_end - b->ctr_off, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(b->h + b->core_off, b->d + b->core_off, b->core_end - b->core_off, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint32_t status = status_h[0];
    const uint64_t used = *used_h;
    if (status & 1u) return fail(OSE_ETIMEDOUT, "in-kernel look-back spin timed out");
    if (status & 2u) {
      // template arena too small: a separate buffer of the exact size the
      // kernel reported, and the call runs again (counters restored first)
      if (b->tmpl_h_big) (void)hipHostFree(b->tmpl_h_big);
      if (b->tmpl_d_big) (void)hipFree(b->tmpl_d_big);
      b->tmpl_h_big = b->tmpl_d_big = nullptr;
      const uint64_t nb = used + 4096;
      HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&b->tmpl_h_big), nb, hipHostMallocDefault));
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&b->tmpl_d_big), nb));
      b->outs_h.tmpl_arena = b->tmpl_h_big;
      od.tmpl_arena = b->outs_d.tmpl_arena = b->tmpl_d_big;
      b->outs_h.tmpl_arena_cap = b->outs_d.tmpl_arena_cap = od.tmpl_arena_cap = nb;
      continue;
    }
    b->used_h = used;
    if (used) HIP_TRY(hipMemcpyAsync(b->outs_h.tmpl_arena, od.tmpl_arena, used, hipMemcpyDeviceToHost, st));
    for (auto& o : b->optional) {
      if (!*o.hslot) continue;
      const size_t fld = reinterpret_cast<uint8_t*>(o.hslot) - reinterpret_cast<uint8_t*>(&b->outs_h);
      void* dptr = *reinterpret_cast<void**>(reinterpret_cast<uint8_t*>(&od) + fld);
      if (!dptr) continue;
      size_t nbytes = o.bytes;
      if (o.hslot == (void**)&b->outs_h.res_bytes) nbytes = 8 * (size_t)b->cols_h.n_resources;
      else if (o.hslot == (void**)&b->outs_h.trace_ratio) nbytes = 8 * std::max<size_t>(b->cols_h.n_spans, 1);
      else if (o.hslot == (void**)&b->outs_h.trace_first_span) nbytes = 4 * std::max<size_t>(b->cols_h.n_spans, 1);
      else nbytes = std::max<size_t>(b->cols_h.n_spans, 1);
      HIP_TRY(hipMemcpyAsync(*o.hslot, dptr, nbytes, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  return fail(OSE_ERANGE, "template arena overflow after resize");
}

}  // extern "C"
