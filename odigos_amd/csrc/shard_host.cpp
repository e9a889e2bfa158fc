// shard_host.cpp — C ABI of the trace-id exchange (include/odigos_amd.h,
// ose_shard_*): bucketing spans by owner GPU, unpacking received records,
// scattering the returned decisions.  The collective itself (an all-to-all
// over RCCL/xGMI) is the caller's: these calls only touch device memory on
// the caller's stream.
#include <algorithm>

#include "engine_internal.hpp"
#include "kernels.hpp"

namespace ose {
namespace {
size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
}  // namespace
}  // namespace ose

using namespace ose;

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

extern "C" {

uint32_t ose_shard_owner(uint64_t tid_hi, uint64_t tid_lo, uint32_t n_ranks) {
  return n_ranks ? shard_owner_host(tid_hi, tid_lo, n_ranks) : 0;
}

uint32_t ose_shard_record_bytes(const ose_engine* eng) {
  const Engine* e = reinterpret_cast<const Engine*>(eng);
  if (!e || !e->has_sampling) return 0;
  return e->sampling_n_attr ? 56u : 48u;
}

int ose_shard_pack(ose_engine* eng, const ose_columns* c, uint32_t n_ranks, void* send, uint64_t* counts,
                   uint32_t* pack_pos, void* hip_stream) {
  if (!eng || !c || !send || !counts || !pack_pos) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (!e->has_sampling) return fail(OSE_EINVAL, "ose_shard_pack needs odigossampling on the engine");
  if (n_ranks == 0 || n_ranks > 64) return fail(OSE_EINVAL, "n_ranks must be in 1..64");
  const uint64_t n = c->n_spans;
  if (n > 0xFFFFFFF0ull) return fail(OSE_ERANGE, "more than 2^32-16 spans");
  if (n && (!c->trace_id || !c->status || !c->resource || !c->res_svc || !c->res_svc_str))
    return fail(OSE_EINVAL, "ose_shard_pack needs trace_id, status, resource, res_svc, res_svc_str");
  if (n && e->sampling_n_lat && (!c->start_ns || !c->end_ns || (!c->route_match && (!c->route || !c->arena))))
    return fail(OSE_EINVAL, "http_latency rules need start_ns, end_ns and route + arena (or route_match)");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipMemsetAsync(counts, 0, 8 * (size_t)n_ranks, st));
  if (n == 0) return 0;
  const uint32_t T = (uint32_t)((n + kSortTile - 1) / kSortTile);
  const uint64_t H = (uint64_t)n_ranks * T;
  const uint32_t htiles = (uint32_t)((H + kScanTileItems - 1) / kScanTileItems);
  Workspace* ws = e->acquire_ws(st);
  const size_t off_hist = 256, off_hoff = align_up(off_hist + 4 * H, 256), off_st = align_up(off_hoff + 4 * H, 256);
  int rc = ws->reserve(off_st + 8 * (size_t)htiles + 256);
  if (rc) {
    e->release_ws(ws, st);
    return rc;
  }
  uint8_t* base = static_cast<uint8_t*>(ws->dev);
  ShardArgs a{};
  a.n_spans = n;
  a.n_tiles = T;
  a.n_ranks = n_ranks;
  a.tid = c->trace_id;
  a.start = c->start_ns;
  a.end = c->end_ns;
  a.status = c->status;
  a.resource = c->resource;
  a.route = c->route;
  a.arena = c->arena;
  a.route_match = c->route_match;
  a.attr_match = e->sampling_n_attr ? c->attr_match : nullptr;
  if (n && e->sampling_n_attr && !c->attr_match) {
    e->release_ws(ws, st);
    return fail(OSE_EINVAL, "span_attribute rules need the attr_match column");
  }
  a.res_svc = c->res_svc;
  a.res_svc_str = c->res_svc_str;
  a.cfg = e->sampling_blob_dev;
  a.hist = reinterpret_cast<uint32_t*>(base + off_hist);
  a.hoff = reinterpret_cast<uint32_t*>(base + off_hoff);
  a.counts = counts;
  a.send = static_cast<uint8_t*>(send);
  a.pack_pos = pack_pos;
  a.rec_words = ose_shard_record_bytes(eng) / 8;
  uint32_t* err = reinterpret_cast<uint32_t*>(base) + 8;
  rc = 0;
  do {
    if (hipMemsetAsync(base, 0, 64, st) != hipSuccess || hipMemsetAsync(base + off_st, 0, 8 * (size_t)htiles, st) != hipSuccess) {
      rc = fail(OSE_EDEVICE, "hipMemsetAsync failed");
      break;
    }
    Engine::Timed tm{};
    e->prof_begin("shard_pack", st, tm);
    launch_shard_hist(a, st);
    ScanArgs sa{};
    sa.n = H;
    sa.n_tiles = htiles;
    sa.in = a.hist;
    sa.out = a.hoff;
    sa.counter = reinterpret_cast<uint32_t*>(base) + 2;
    sa.status = reinterpret_cast<uint64_t*>(base + off_st);
    sa.error = err;
    launch_scan_u32(sa, st);
    launch_shard_scatter(a, st);
    e->prof_end(tm, st);
    if (hipGetLastError() != hipSuccess) rc = fail(OSE_EDEVICE, "shard pack launch failed");
  } while (0);
  e->release_ws(ws, st);
  return rc;
}

int ose_shard_unpack(const void* recv, uint64_t n, uint32_t rec_bytes, uint64_t* trace_id, uint64_t* start_ns,
                     uint64_t* end_ns, uint8_t* status, uint32_t* resource, uint32_t* res_svc, uint32_t* res_svc_str,
                     uint64_t* route_match, uint64_t* attr_match, void* hip_stream) {
  if (rec_bytes != 48 && rec_bytes != 56) return fail(OSE_EINVAL, "rec_bytes must be ose_shard_record_bytes()");
  if (n && (!recv || !trace_id || !start_ns || !end_ns || !status || !resource || !res_svc || !res_svc_str ||
            !route_match || !attr_match))
    return fail(OSE_EINVAL, "NULL argument");
  UnpackArgs a{static_cast<const uint8_t*>(recv), n, trace_id, start_ns, end_ns, status, resource, res_svc, res_svc_str,
               route_match, attr_match, rec_bytes / 8};
  launch_shard_unpack(a, static_cast<hipStream_t>(hip_stream));
  HIP_TRY(hipGetLastError());
  return 0;
}

int ose_shard_scatter_keep(const uint8_t* keep_back, const uint32_t* pack_pos, uint64_t n, uint8_t* keep,
                           void* hip_stream) {
  if (n && (!keep_back || !pack_pos || !keep)) return fail(OSE_EINVAL, "NULL argument");
  launch_scatter_keep(keep_back, pack_pos, n, keep, static_cast<hipStream_t>(hip_stream));
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // extern "C"
