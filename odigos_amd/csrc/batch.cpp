// batch.cpp — engine-owned pinned host staging (ose_batch_*) and the
// synchronous ose_process path used by the host processors / a cgo shim.
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

struct Buf {
  void** host_slot;   // where the pinned pointer is published (in cols_h / outs_h)
  void** dev_slot;    // same field in cols_d / outs_d
  size_t bytes;
  bool input;
  void* h = nullptr;
  void* d = nullptr;
};

struct Batch {
  Engine* e = nullptr;
  ose_columns cols_h{}, cols_d{};
  ose_outputs outs_h{}, outs_d{};
  uint64_t used_h = 0;
  std::vector<Buf> bufs;
  ~Batch() {
    for (auto& b : bufs) {
      if (b.h) (void)hipHostFree(b.h);
      if (b.d) (void)hipFree(b.d);
    }
  }
  int alloc(Buf& b) {
    size_t n = b.bytes + 16;   // arena slack contract (ByteReader 16-byte loads)
    HIP_TRY(hipHostMalloc(&b.h, n, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&b.d, n));
    std::memset(b.h, 0, n);
    HIP_TRY(hipMemset(b.d, 0, n));
    *b.host_slot = b.h;
    *b.dev_slot = b.d;
    return 0;
  }
};

}  // namespace ose

using namespace ose;

extern "C" {

int ose_batch_acquire(ose_engine* eng, const ose_columns* dims, ose_batch** out) {
  if (!eng || !dims || !out) return fail(OSE_EINVAL, "NULL argument");
  int rc = ensure_device();
  if (rc) return rc;
  Engine* e = reinterpret_cast<Engine*>(eng);
  auto* b = new Batch();
  b->e = e;
  const uint64_t n = dims->n_spans;
  const uint64_t R = dims->n_resources, S = dims->n_scopes, A = dims->n_attrsets;
  b->cols_h.n_spans = b->cols_d.n_spans = n;
  b->cols_h.n_resources = b->cols_d.n_resources = (uint32_t)R;
  b->cols_h.n_scopes = b->cols_d.n_scopes = (uint32_t)S;
  b->cols_h.n_attrsets = b->cols_d.n_attrsets = (uint32_t)A;
  b->cols_h.arena_bytes = b->cols_d.arena_bytes = dims->arena_bytes;
#define IN(field, bytes) b->bufs.push_back(Buf{(void**)&b->cols_h.field, (void**)&b->cols_d.field, (size_t)(bytes), true})
#define OUT(field, bytes) b->bufs.push_back(Buf{(void**)&b->outs_h.field, (void**)&b->outs_d.field, (size_t)(bytes), false})
  IN(arena, dims->arena_bytes);
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
  IN(attr_match, 8 * n);
  IN(res_svc, 4 * R);
  IN(res_svc_str, 4 * R);
  IN(res_url_ok, R);
  IN(res_attrset, 4 * R);
  IN(res_size, 4 * R);
  IN(scope_size, 4 * S);
  IN(scope_resource, 4 * S);
  OUT(keep, n);
  OUT(trace_count, 4);
  OUT(trace_first_span, 4 * std::max<uint64_t>(n, 1));   // BATCH mode: one trace even with no spans
  OUT(trace_keep, 1 * std::max<uint64_t>(n, 1));
  OUT(trace_level, 1 * std::max<uint64_t>(n, 1));
  OUT(trace_ratio, 8 * std::max<uint64_t>(n, 1));
  OUT(url_out, n);
  OUT(tmpl, 8 * n);
  // every template fits in 2x the input bytes + 8 per span; capped at the
  // 32-bit offset range of ose_strref (an overflow regrows it below)
  const uint64_t tcap = std::min<uint64_t>(2 * dims->arena_bytes + 8 * n + 4096, 0xFFFFFFF0ull);
  OUT(tmpl_arena, tcap);
  OUT(attrset_bytes, 8 * A);
  OUT(accepted_spans, 8);
  OUT(res_bytes, 8 * R);
  OUT(device_status, 4);
#undef IN
#undef OUT
  b->outs_h.tmpl_arena_cap = b->outs_d.tmpl_arena_cap = tcap;
  for (auto& x : b->bufs) {
    rc = b->alloc(x);
    if (rc) { delete b; return rc; }
  }
  b->outs_h.tmpl_arena_used = &b->used_h;
  *out = reinterpret_cast<ose_batch*>(b);
  return 0;
}

ose_columns* ose_batch_columns(ose_batch* bb) { return bb ? &reinterpret_cast<Batch*>(bb)->cols_h : nullptr; }
ose_outputs* ose_batch_outputs(ose_batch* bb) { return bb ? &reinterpret_cast<Batch*>(bb)->outs_h : nullptr; }
void ose_batch_release(ose_batch* bb) { delete reinterpret_cast<Batch*>(bb); }

int ose_process(ose_engine* eng, ose_batch* bb, uint32_t stage_mask, uint32_t group_mode, const ose_rand* rnd) {
  if (!eng || !bb) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  Batch* b = reinterpret_cast<Batch*>(bb);
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
  uint64_t used_dev_slot_off = 0;
  (void)used_dev_slot_off;
  // device scalar for tmpl_arena_used lives in the device_status buffer's slack
  uint64_t* used_d = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>((void*)b->outs_d.device_status) + 8);
  b->outs_d.tmpl_arena_used = used_d;
  for (int attempt = 0; attempt < 2; attempt++) {
    for (auto& x : b->bufs) {
      if (!x.input) continue;
      size_t bytes = x.bytes;
      if ((void**)x.host_slot == (void**)&b->cols_h.arena) bytes = b->cols_h.arena_bytes;
      if (bytes) HIP_TRY(hipMemcpyAsync(x.d, x.h, bytes, hipMemcpyHostToDevice, st));
    }
    HIP_TRY(hipMemsetAsync(b->outs_d.device_status, 0, 16, st));
    if (b->outs_d.attrset_bytes && b->cols_h.n_attrsets)
      HIP_TRY(hipMemcpyAsync(b->outs_d.attrset_bytes, b->outs_h.attrset_bytes, 8 * (size_t)b->cols_h.n_attrsets,
                             hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(b->outs_d.accepted_spans, b->outs_h.accepted_spans, 8, hipMemcpyHostToDevice, st));
    int rc = run_stages(e, &b->cols_d, &b->outs_d, stage_mask, group_mode, rnd, st);
    if (rc) return rc;
    uint32_t status = 0;
    uint64_t used = 0;
    HIP_TRY(hipMemcpyAsync(&status, b->outs_d.device_status, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&used, used_d, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (status & 1u) return fail(OSE_ETIMEDOUT, "in-kernel look-back spin timed out");
    if (status & 2u) {
      // template arena too small: grow to the exact size the kernel reported and rerun
      for (auto& x : b->bufs) {
        if ((void**)x.host_slot != (void**)&b->outs_h.tmpl_arena) continue;
        if (x.h) (void)hipHostFree(x.h);
        if (x.d) (void)hipFree(x.d);
        x.h = x.d = nullptr;
        x.bytes = used + 4096;
        int rc2 = b->alloc(x);
        if (rc2) return rc2;
        b->outs_h.tmpl_arena_cap = b->outs_d.tmpl_arena_cap = x.bytes;
      }
      continue;
    }
    b->used_h = used;
    for (auto& x : b->bufs) {
      if (x.input) continue;
      size_t bytes = x.bytes;
      if ((void**)x.host_slot == (void**)&b->outs_h.tmpl_arena) bytes = used;
      if (bytes) HIP_TRY(hipMemcpyAsync(x.h, x.d, bytes, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  return fail(OSE_ERANGE, "template arena overflow after resize");
}

}  // extern "C"
