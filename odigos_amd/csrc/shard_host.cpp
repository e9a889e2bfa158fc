// shard_host.cpp — C ABI of the trace-id exchange (include/odigos_amd.h,
// ose_shard_*, ose_exchange_*): folding spans into per-owner partial
// records, unpacking received records, scattering the returned decisions,
// and the whole round over an RCCL communicator (ose_exchange_sample), the
// in-node replacement of the node collector's loadbalancing exporter keyed
// by trace id (autoscaler/controllers/nodecollector/collectorconfig/
// traces.go:26-84).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <vector>

#include "devcfg.hpp"
#include "engine_internal.hpp"
#include "kernels.hpp"

namespace ose {
namespace {
size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// RCCL, resolved at run time: the process's already loaded copy when there
// is one (PyTorch loads its own), else the system librccl.  Nothing links
// against it, so the library still loads where RCCL is absent.
struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};
const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    auto sym = [&](auto& fn, const char* n) { fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, n)); };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.all_reduce, "ncclAllReduce");
    sym(r.error_string, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.send && r.recv && r.group_start &&
           r.group_end && r.all_reduce;
  });
  return r;
}
int nccl_fail(const char* what, ncclResult_t rc) {
  const Rccl& r = rccl();
  return fail(OSE_EDEVICE, std::string(what) + ": " + (r.error_string ? r.error_string(rc) : "RCCL error"));
}
#define NCCL_TRY(expr)                                  \
  do {                                                  \
    ncclResult_t _r = (expr);                           \
    if (_r != ncclSuccess) return nccl_fail(#expr, _r); \
  } while (0)

// device scratch of one exchange round (per engine).  Rounds on one engine
// are serialised on the host by `mu` and on the device by `done`: the next
// round's stream waits for the event the previous round recorded at its end,
// so a round queued on another stream cannot pack into `send` while the
// previous round's transfers still read it.
struct XBuf {
  void* p = nullptr;
  size_t cap = 0;
  int need(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, std::max<size_t>(bytes, 256)) != hipSuccess) return fail(OSE_ENOMEM, "exchange scratch");
    cap = std::max<size_t>(bytes, 256);
    return 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};
struct XScratch {
  std::mutex mu;
  XBuf send, recv, pos, counts, keep_back, keep_x, cols, bkt;
  uint64_t* host_counts = nullptr;   // pinned [2 * 64]
  uint32_t* host_flag = nullptr;     // pinned: the owner fold's overflow word
  bool last_general = false;         // the last owner_decide took the general path (osehost_owner_last_general)
  hipEvent_t done = nullptr;         // recorded at the end of the last round
  bool done_set = false;
  ~XScratch() {
    for (XBuf* b : {&send, &recv, &pos, &counts, &keep_back, &keep_x, &cols, &bkt})
      if (b->p) (void)hipFree(b->p);
    if (host_counts) (void)hipHostFree(host_counts);
    if (host_flag) (void)hipHostFree(host_flag);
    if (done) (void)hipEventDestroy(done);
  }
};
std::mutex g_xs_mu;
std::vector<std::pair<const Engine*, XScratch*>> g_xs;   // engine -> scratch (few engines)
XScratch* scratch_of(const Engine* e) {
  std::lock_guard<std::mutex> g(g_xs_mu);
  for (auto& kv : g_xs)
    if (kv.first == e) return kv.second;
  auto* x = new XScratch();
  g_xs.emplace_back(e, x);
  return x;
}

// ---- transports ------------------------------------------------------------------
// What one exchange round needs of a collective library: a variable-size
// all-to-all of bytes, stream-ordered on `st` (rank r sends slen[p] bytes at
// send + soff[p] to rank p and receives rlen[p] bytes from p into
// recv + roff[p]).  The product transport is RCCL's grouped point-to-point
// over xGMI; the test transport moves the bytes between in-process ranks.
struct XTransport {
  virtual ~XTransport() = default;
  virtual int alltoallv(const uint8_t* send, const uint64_t* soff, const uint64_t* slen, uint8_t* recv,
                        const uint64_t* roff, const uint64_t* rlen, hipStream_t st) = 0;
  // node[k] = the sum over ranks of local[k] (int64), stream-ordered on `st`
  virtual int allreduce_i64(const int64_t* local, int64_t* node, uint64_t n, hipStream_t st) = 0;
  // a rank that fails in the middle of a round tells its peers (the local
  // transport unblocks them; an RCCL communicator is left to the caller)
  virtual void abort() {}
};

struct RcclTransport final : XTransport {
  ncclComm_t comm;
  int n_ranks;
  RcclTransport(ncclComm_t c, int w) : comm(c), n_ranks(w) {}
  int alltoallv(const uint8_t* send, const uint64_t* soff, const uint64_t* slen, uint8_t* recv, const uint64_t* roff,
                const uint64_t* rlen, hipStream_t st) override {
    const Rccl& r = rccl();
    ncclResult_t rc = r.group_start();
    if (rc != ncclSuccess) return nccl_fail("ncclGroupStart", rc);
    int err = 0;
    for (int p = 0; p < n_ranks && !err; p++) {
      if (slen[p] && (rc = r.send(send + soff[p], slen[p], ncclUint8, p, comm, st)) != ncclSuccess)
        err = nccl_fail("ncclSend", rc);
      if (!err && rlen[p] && (rc = r.recv(recv + roff[p], rlen[p], ncclUint8, p, comm, st)) != ncclSuccess)
        err = nccl_fail("ncclRecv", rc);
    }
    rc = r.group_end();   // the group is closed on every path, a failed enqueue included
    if (err) return err;
    if (rc != ncclSuccess) return nccl_fail("ncclGroupEnd", rc);
    return 0;
  }
  int allreduce_i64(const int64_t* local, int64_t* node, uint64_t n, hipStream_t st) override {
    NCCL_TRY(rccl().all_reduce(local, node, n, ncclInt64, ncclSum, comm, st));
    return 0;
  }
};

// In-process ranks (test transport, osehost_xgroup_*): W host threads, each
// with its own engine and stream, on one or several devices.  A phase is two
// rendezvous: every rank publishes its send buffer and an event recorded
// behind the data, then pulls its pieces with device-to-device copies queued
// behind the senders' events and records a `done` event; after the second
// rendezvous every rank's stream waits for its peers' `done`, so a send
// buffer is reused only after every copy out of it (NCCL send semantics).
struct LocalGroup {
  explicit LocalGroup(int w) : n_ranks(w), slots(w) {}
  ~LocalGroup() {
    for (auto& s : slots) {
      if (s.ready) (void)hipEventDestroy(s.ready);
      if (s.done) (void)hipEventDestroy(s.done);
    }
  }
  struct Slot {
    const uint8_t* send = nullptr;
    const uint64_t* soff = nullptr;
    const uint64_t* slen = nullptr;
    uint64_t n = 0;   // allreduce_i64: the vector length, by value (a peer may read it after this rank returned)
    hipEvent_t ready = nullptr, done = nullptr;
  };
  const int n_ranks;
  std::vector<Slot> slots;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  bool broken = false;
  int barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return fail(OSE_EDEVICE, "in-process exchange group: a peer failed");
    const uint64_t gen = generation;
    if (++arrived == n_ranks) {
      arrived = 0;
      generation++;
      cv.notify_all();
      return 0;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen || broken; })) {
      broken = true;
      cv.notify_all();
      return fail(OSE_ETIMEDOUT, "in-process exchange group: a peer never arrived");
    }
    return broken ? fail(OSE_EDEVICE, "in-process exchange group: a peer failed") : 0;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    broken = true;
    cv.notify_all();
  }
};

struct LocalTransport final : XTransport {
  LocalGroup* g;
  int rank;
  LocalTransport(LocalGroup* grp, int r) : g(grp), rank(r) {}
  void abort() override { g->abort(); }
  int alltoallv(const uint8_t* send, const uint64_t* soff, const uint64_t* slen, uint8_t* recv, const uint64_t* roff,
                const uint64_t* rlen, hipStream_t st) override {
    LocalGroup::Slot& me = g->slots[(size_t)rank];
    if (!me.ready && hipEventCreateWithFlags(&me.ready, hipEventDisableTiming) != hipSuccess)
      return fail(OSE_EDEVICE, "hipEventCreate failed");
    if (!me.done && hipEventCreateWithFlags(&me.done, hipEventDisableTiming) != hipSuccess)
      return fail(OSE_EDEVICE, "hipEventCreate failed");
    me.send = send;
    me.soff = soff;
    me.slen = slen;
    if (hipEventRecord(me.ready, st) != hipSuccess) return fail(OSE_EDEVICE, "hipEventRecord failed");
    if (int rc = g->barrier()) return rc;
    // every peer's piece in one copy launch behind the peers' events (as
    // RCCL's grouped send/recv moves them in one fused launch), not one
    // hipMemcpyAsync per peer
    int err = 0;
    PeerCopies pc{};
    uint64_t max_len = 0;
    for (int p = 0; p < g->n_ranks && !err; p++) {
      const LocalGroup::Slot& src = g->slots[(size_t)p];
      if (src.slen[rank] != rlen[p]) {
        err = fail(OSE_EINVAL, "in-process exchange: send and receive sizes disagree");
        break;
      }
      if (!rlen[p]) continue;
      if (hipStreamWaitEvent(st, src.ready, 0) != hipSuccess) {
        err = fail(OSE_EDEVICE, "hipStreamWaitEvent failed");
        break;
      }
      pc.src[pc.n] = src.send + src.soff[rank];
      pc.dst[pc.n] = recv + roff[p];
      pc.len[pc.n] = rlen[p];
      max_len = std::max(max_len, rlen[p]);
      pc.n++;
    }
    if (!err) {
      launch_peer_copies(pc, max_len, st);
      if (hipGetLastError() != hipSuccess) err = fail(OSE_EDEVICE, "in-process exchange: device copy failed");
    }
    if (!err && hipEventRecord(me.done, st) != hipSuccess) err = fail(OSE_EDEVICE, "hipEventRecord failed");
    if (err) {
      g->abort();
      return err;
    }
    if (int rc = g->barrier()) return rc;
    for (int p = 0; p < g->n_ranks; p++)
      if (slen[p] && hipStreamWaitEvent(st, g->slots[(size_t)p].done, 0) != hipSuccess)
        return fail(OSE_EDEVICE, "hipStreamWaitEvent failed");
    return 0;
  }
  // every rank publishes its vector, then adds every rank's into its own
  // node buffer (queued behind the owners' events); a second rendezvous
  // keeps each local vector alive until every peer's adds are queued behind
  // this rank's `done`
  int allreduce_i64(const int64_t* local, int64_t* node, uint64_t n, hipStream_t st) override {
    LocalGroup::Slot& me = g->slots[(size_t)rank];
    if (!me.ready && hipEventCreateWithFlags(&me.ready, hipEventDisableTiming) != hipSuccess)
      return fail(OSE_EDEVICE, "hipEventCreate failed");
    if (!me.done && hipEventCreateWithFlags(&me.done, hipEventDisableTiming) != hipSuccess)
      return fail(OSE_EDEVICE, "hipEventCreate failed");
    if (n && static_cast<const void*>(local) == static_cast<const void*>(node))
      return fail(OSE_EINVAL, "in-process all-reduce: local and node must not alias");
    me.send = reinterpret_cast<const uint8_t*>(local);
    me.soff = nullptr;
    me.slen = nullptr;
    me.n = n;
    if (hipEventRecord(me.ready, st) != hipSuccess) return fail(OSE_EDEVICE, "hipEventRecord failed");
    if (int rc = g->barrier()) return rc;
    int err = 0;
    if (n && hipMemsetAsync(node, 0, n * sizeof(int64_t), st) != hipSuccess) err = fail(OSE_EDEVICE, "hipMemsetAsync failed");
    for (int p = 0; p < g->n_ranks && !err; p++) {
      const LocalGroup::Slot& src = g->slots[(size_t)p];
      if (src.n != n) {
        err = fail(OSE_EINVAL, "in-process all-reduce: vector lengths disagree");
        break;
      }
      if (hipStreamWaitEvent(st, src.ready, 0) != hipSuccess) {
        err = fail(OSE_EDEVICE, "hipStreamWaitEvent failed");
        break;
      }
      launch_add_i64(node, reinterpret_cast<const int64_t*>(src.send), n, st);
      if (hipGetLastError() != hipSuccess) err = fail(OSE_EDEVICE, "add_i64 launch failed");
    }
    if (!err && hipEventRecord(me.done, st) != hipSuccess) err = fail(OSE_EDEVICE, "hipEventRecord failed");
    if (err) {
      g->abort();
      return err;
    }
    if (int rc = g->barrier()) return rc;
    for (int p = 0; p < g->n_ranks; p++)
      if (hipStreamWaitEvent(st, g->slots[(size_t)p].done, 0) != hipSuccess)
        return fail(OSE_EDEVICE, "hipStreamWaitEvent failed");
    return 0;
  }
};

}  // namespace

void release_exchange_scratch(const Engine* e) {
  std::lock_guard<std::mutex> g(g_xs_mu);
  for (size_t k = 0; k < g_xs.size(); k++)
    if (g_xs[k].first == e) {
      delete g_xs[k].second;
      g_xs.erase(g_xs.begin() + (long)k);
      return;
    }
}
}  // namespace ose

using namespace ose;

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace ose {
namespace {
// The owner's decisions for n received records (keep per record, recv in
// (source rank, source order)): the bucketed fold (owner_fold_kernel), or,
// when a bucket or a trace overflows it, the records unpacked into span
// columns and the general SAMPLE stage (run lists, then the sort path).
// The host waits once, for the fold's overflow word.
int owner_decide(Engine* e, XScratch* xs, const uint8_t* recvb, uint64_t n_recv, uint32_t K, uint8_t* keep,
                 uint32_t* device_status, const ose_rand* rnd, hipStream_t st) {
  if (!n_recv) return 0;
  const uint64_t RB = x_rec_bytes(K);
  const uint64_t B = std::max<uint64_t>(1, (n_recv + kOwnerAvg - 1) / kOwnerAvg);
  const size_t off_rec = align_up(64 + 4 * B, 256);
  int rc;
  if ((rc = xs->bkt.need(off_rec + 8 * kOwnerSlotWords * B * kOwnerCap))) return rc;
  if (!xs->host_flag) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&xs->host_flag), 64, hipHostMallocDefault));
  uint8_t* bb = xs->bkt.as<uint8_t>();
  OwnerArgs oa{};
  oa.recv = recvb;
  oa.n = n_recv;
  oa.words = x_rec_words(K);
  oa.n_buckets = (uint32_t)B;
  oa.overflow = reinterpret_cast<uint32_t*>(bb);
  oa.bkt_count = reinterpret_cast<uint32_t*>(bb + 64);
  oa.bkt_rec = reinterpret_cast<uint64_t*>(bb + off_rec);
  oa.cfgs = reinterpret_cast<const uint8_t* const*>(e->shard_tables_dev);
  oa.n_chunks = K;
  oa.n_global_svc = (uint32_t)e->service_ids.size();
  oa.svc_maps = e->sampling_local_svc ? e->sampling_svc_maps_dev : nullptr;
  for (const auto& blob : e->sampling_chunks_host)   // the tables the fold reads: everything before the route bytes
    oa.cfg_lds_bytes = std::max(oa.cfg_lds_bytes,
                                (reinterpret_cast<const SampCfgDev*>(blob.data())->bytes_off + 15u) & ~15u);
  oa.seed = rnd ? rnd->seed : 0;
  oa.keep = keep;
  HIP_TRY(hipMemsetAsync(bb, 0, 64 + 4 * B, st));
#if OSE_DIAG
  static uint64_t* clocks = nullptr;   // per-phase ticks (OSE_OWNER_CLOCKS), printed after the call
  if (getenv("OSE_OWNER_CLOCKS")) {
    if (!clocks) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&clocks), 64));
    HIP_TRY(hipMemsetAsync(clocks, 0, 64, st));
    oa.clocks = clocks;
  }
#endif
  Engine::Timed tf{};
  e->prof_begin("owner_fold", st, tf);
  launch_owner_bucket(oa, st);
  launch_owner_fold(oa, st);
  e->prof_end(tf, st);
  HIP_TRY(hipGetLastError());
#if OSE_DIAG
  if (oa.clocks) {
    uint64_t h[8];
    HIP_TRY(hipMemcpyAsync(h, oa.clocks, 64, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    fprintf(stderr, "owner_fold clocks (10 ns ticks summed over workgroups): load %llu group %llu sort %llu fold %llu "
            "keep %llu; records %llu buckets %llu\n", (unsigned long long)h[0], (unsigned long long)h[1],
            (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4], (unsigned long long)n_recv,
            (unsigned long long)B);
  }
#endif
  HIP_TRY(hipMemcpyAsync(xs->host_flag, oa.overflow, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  xs->last_general = *xs->host_flag != 0;
  if (!xs->last_general) return 0;
  // the general path: owner-side columns (trace_id 16, start 8, end 8, route_match 8 K, svc_match 8 K,
  // resource 4, res_svc 4, res_svc_str 4, status 1 per record)
  const uint64_t R = n_recv;
  const size_t o_tid = 0, o_st = align_up(o_tid + 16 * R, 256), o_en = align_up(o_st + 8 * R, 256),
               o_rm = align_up(o_en + 8 * R, 256), o_sm = align_up(o_rm + 8 * R * K, 256),
               o_res = align_up(o_sm + 8 * R * K, 256), o_sv = align_up(o_res + 4 * R, 256),
               o_ss = align_up(o_sv + 4 * R, 256), o_stat = align_up(o_ss + 4 * R, 256), o_end = o_stat + R + 256;
  if ((rc = xs->cols.need(o_end))) return rc;
  uint8_t* cb = xs->cols.as<uint8_t>();
  ose_columns oc{};
  oc.n_spans = n_recv;
  oc.n_resources = (uint32_t)n_recv;
  oc.match_planes = K;   // route_match / svc_match: plane k for rule chunk k
  oc.trace_id = reinterpret_cast<uint64_t*>(cb + o_tid);
  oc.start_ns = reinterpret_cast<uint64_t*>(cb + o_st);
  oc.end_ns = reinterpret_cast<uint64_t*>(cb + o_en);
  oc.route_match = reinterpret_cast<uint64_t*>(cb + o_rm);
  oc.svc_match = reinterpret_cast<uint64_t*>(cb + o_sm);
  oc.resource = reinterpret_cast<uint32_t*>(cb + o_res);
  oc.res_svc = reinterpret_cast<uint32_t*>(cb + o_sv);
  oc.res_svc_str = reinterpret_cast<uint32_t*>(cb + o_ss);
  oc.status = cb + o_stat;
  Engine::Timed tm{};
  e->prof_begin("shard_unpack", st, tm);
  rc = ose_shard_unpack(recvb, n_recv, (uint32_t)RB, const_cast<uint64_t*>(oc.trace_id), const_cast<uint64_t*>(oc.start_ns),
                        const_cast<uint64_t*>(oc.end_ns), const_cast<uint8_t*>(oc.status),
                        const_cast<uint32_t*>(oc.resource), const_cast<uint32_t*>(oc.res_svc),
                        const_cast<uint32_t*>(oc.res_svc_str), const_cast<uint64_t*>(oc.route_match),
                        const_cast<uint64_t*>(oc.svc_match), st);
  e->prof_end(tm, st);
  if (rc) return rc;
  ose_outputs ox{};
  ox.keep = keep;
  ox.device_status = device_status;
  Engine::Timed to{};
  e->prof_begin("owner_sample", st, to);
  rc = run_stages(e, &oc, &ox, OSE_STAGE_SAMPLE, OSE_GROUP_TRACE_ID, rnd, st);
  e->prof_end(to, st);
  return rc;
}

// One exchange round (ose_exchange_sample).  Everything that can fail on
// this rank alone (arguments, scratch) is checked before the first
// collective; a failure after it leaves the peers inside a collective, so
// the transport is told (abort) and the caller must treat the communicator
// as unusable, as after any NCCL error.
int exchange_round(Engine* e, const ose_columns* cols, const ose_outputs* outs, XTransport& tx, int rank, int n_ranks,
                   const ose_rand* rnd, hipStream_t st, uint64_t* stats) {
  if (n_ranks < 1 || n_ranks > 64 || rank < 0 || rank >= n_ranks) return fail(OSE_EINVAL, "rank / n_ranks out of range");
  if (cols->n_spans && !outs->keep) return fail(OSE_EINVAL, "outs->keep is required");
  if (!e->has_sampling) return fail(OSE_EINVAL, "the exchange needs odigossampling on the engine");
  if (int brc = bind_device(e)) return brc;
  XScratch* xs = scratch_of(e);
  std::lock_guard<std::mutex> g(xs->mu);
  const uint64_t n = cols->n_spans, W = (uint64_t)n_ranks;
  const uint32_t K = (uint32_t)e->sampling_chunks_dev.size();
  const uint64_t RB = x_rec_bytes(K);   // record bytes: one endpoint and one rule word per rule chunk
  int rc;
  if ((rc = xs->send.need(std::max<uint64_t>(n, 1) * RB)) || (rc = xs->pos.need(4 * std::max<uint64_t>(n, 1))) ||
      (rc = xs->counts.need(16 * W)) || (rc = xs->keep_back.need(std::max<uint64_t>(n, 1))))
    return rc;
  if (!xs->host_counts) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&xs->host_counts), 16 * 64, hipHostMallocDefault));
  if (!xs->done) HIP_TRY(hipEventCreateWithFlags(&xs->done, hipEventDisableTiming));
  if (xs->done_set) HIP_TRY(hipStreamWaitEvent(st, xs->done, 0));   // the previous round left the scratch
  uint64_t* scnt_d = xs->counts.as<uint64_t>();
  uint64_t* rcnt_d = scnt_d + W;
  // 1. partial records per owner
  rc = ose_shard_pack(reinterpret_cast<ose_engine*>(e), cols, (uint32_t)W, xs->send.p, scnt_d, xs->pos.as<uint32_t>(), st);
  if (rc) return rc;   // before any collective
  auto abort_with = [&](int code) {
    tx.abort();
    return code;
  };
  // 2. record counts, all-to-all (one u64 per peer)
  std::vector<uint64_t> c_off(W), c_len(W, 8);
  for (uint64_t p = 0; p < W; p++) c_off[p] = 8 * p;
  if ((rc = tx.alltoallv(reinterpret_cast<const uint8_t*>(scnt_d), c_off.data(), c_len.data(),
                         reinterpret_cast<uint8_t*>(rcnt_d), c_off.data(), c_len.data(), st)))
    return abort_with(rc);
  if (hipMemcpyAsync(xs->host_counts, scnt_d, 16 * W, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)   // the host needs the split sizes
    return abort_with(fail(OSE_EDEVICE, "exchange: reading the record counts failed"));
  std::vector<uint64_t> sc(xs->host_counts, xs->host_counts + W), rcv(xs->host_counts + W, xs->host_counts + 2 * W);
  std::vector<uint64_t> sd(W + 1, 0), rd(W + 1, 0);
  for (uint64_t p = 0; p < W; p++) {
    sd[p + 1] = sd[p] + sc[p];
    rd[p + 1] = rd[p] + rcv[p];
  }
  const uint64_t n_recv = rd[W];
  if (n_recv > 0xFFFFFFF0ull) return abort_with(fail(OSE_ERANGE, "more than 2^32-16 records received"));
  const uint64_t R = std::max<uint64_t>(n_recv, 1);
  if ((rc = xs->recv.need(R * RB)) || (rc = xs->keep_x.need(R))) return abort_with(rc);
  // 3. the records (variable sizes per peer)
  std::vector<uint64_t> s_off(W), s_len(W), r_off(W), r_len(W);
  for (uint64_t p = 0; p < W; p++) {
    s_off[p] = sd[p] * RB;
    s_len[p] = sc[p] * RB;
    r_off[p] = rd[p] * RB;
    r_len[p] = rcv[p] * RB;
  }
  uint8_t* recvb = xs->recv.as<uint8_t>();
  if ((rc = tx.alltoallv(xs->send.as<uint8_t>(), s_off.data(), s_len.data(), recvb, r_off.data(), r_len.data(), st)))
    return abort_with(rc);
  // 4. owner: the decisions for the received records (source-rank order)
  rc = owner_decide(e, xs, recvb, n_recv, K, xs->keep_x.as<uint8_t>(), outs->device_status, rnd, st);
  if (rc) return abort_with(rc);
  // 5. decisions back to the sources (reverse split), 6. onto the spans
  std::vector<uint64_t> kb_off(sd.begin(), sd.end() - 1), kx_off(rd.begin(), rd.end() - 1);
  if ((rc = tx.alltoallv(xs->keep_x.as<uint8_t>(), kx_off.data(), rcv.data(), xs->keep_back.as<uint8_t>(), kb_off.data(),
                         sc.data(), st)))
    return abort_with(rc);
  rc = ose_shard_scatter_keep(xs->keep_back.as<uint8_t>(), xs->pos.as<uint32_t>(), n, outs->keep, st);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(xs->done, st));
  xs->done_set = true;
  if (stats) {   // records sent, records received, spans
    stats[0] = sd[W];
    stats[1] = n_recv;
    stats[2] = n;
  }
  return 0;
}
}  // namespace
}  // namespace ose

extern "C" {

uint32_t ose_shard_owner(uint64_t tid_hi, uint64_t tid_lo, uint32_t n_ranks) {
  return n_ranks ? shard_owner_host(tid_hi, tid_lo, n_ranks) : 0;
}

uint32_t ose_shard_record_bytes(const ose_engine* eng) {
  const Engine* e = reinterpret_cast<const Engine*>(eng);
  if (!e || !e->has_sampling) return 0;
  return x_rec_bytes((uint32_t)e->sampling_chunks_dev.size());
}

int ose_shard_pack(ose_engine* eng, const ose_columns* c, uint32_t n_ranks, void* send, uint64_t* counts,
                   uint32_t* pack_pos, void* hip_stream) {
  if (!eng || !c || !send || !counts || !pack_pos) return fail(OSE_EINVAL, "NULL argument");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (!e->has_sampling) return fail(OSE_EINVAL, "ose_shard_pack needs odigossampling on the engine");
  if (int brc = bind_device(e)) return brc;
  if (n_ranks == 0 || n_ranks > 64) return fail(OSE_EINVAL, "n_ranks must be in 1..64");
  const uint64_t n = c->n_spans;
  if (n > 0xFFFFFFF0ull) return fail(OSE_ERANGE, "more than 2^32-16 spans");
  if (n && (!c->trace_id || !c->status || !c->resource || !c->res_svc || !c->res_svc_str))
    return fail(OSE_EINVAL, "ose_shard_pack needs trace_id, status, resource, res_svc, res_svc_str");
  if (n && e->sampling_n_lat && (!c->start_ns || !c->end_ns || (!c->route_match && (!c->route || !c->arena))))
    return fail(OSE_EINVAL, "http_latency rules need start_ns, end_ns and route + arena (or route_match)");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  if (n == 0) {   // (otherwise shard_counts_kernel writes every owner's count)
    HIP_TRY(hipMemsetAsync(counts, 0, 8 * (size_t)n_ranks, st));
    return 0;
  }
  const uint32_t T = (uint32_t)((n + kXChunk - 1) / kXChunk);   // packing waves
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
  a.rm_stride = c->match_planes > 1 ? n : 0;
  if (c->route_match && e->sampling_chunks_dev.size() > 1 && c->match_planes != e->sampling_chunks_dev.size()) {
    // chunk-local rule bits: one plane per chunk, never plane 0 for every chunk
    e->release_ws(ws, st);
    return fail(OSE_EINVAL, "cols->match_planes must equal the engine's rule chunks when route_match is set");
  }
  if (e->sampling_spill && !c->route_match && c->route && e->sampling_n_lat) {   // route bytes past an LDS table: planes first
    const uint64_t* planes = nullptr;
    rc = spill_endpoint_planes(e, c, ws, st, &planes);
    if (rc) {
      e->release_ws(ws, st);
      return rc;
    }
    a.route_match = planes;
    a.rm_stride = n;
  }
  if (c->route_match && c->match_planes > 1 && c->match_planes != e->sampling_chunks_dev.size()) {
    e->release_ws(ws, st);
    return fail(OSE_EINVAL, "cols->match_planes must be 1 or the engine's rule chunks");
  }
  {
    const uint64_t* am = nullptr;
    rc = resolve_attr_match(e, c, ws, st, &am);
    if (rc) {
      e->release_ws(ws, st);
      return rc;
    }
    a.attr_match = e->sampling_n_attr ? am : nullptr;
    a.attr_stride = n;
    a.attr_words = e->attr_words;
  }
  a.res_svc = c->res_svc;
  a.res_svc_str = c->res_svc_str;
  a.cfgs = reinterpret_cast<const uint8_t* const*>(e->shard_tables_dev);
  a.n_chunks = (uint32_t)e->sampling_chunks_dev.size();
  a.lat_svc = reinterpret_cast<const uint32_t*>(e->shard_tables_dev + 8 * e->sampling_chunks_dev.size());
  // records carry global service ids; chunk-local tables map them per chunk
  a.n_global_svc = (uint32_t)e->service_ids.size();
  a.svc_maps = e->sampling_local_svc ? e->sampling_svc_maps_dev : nullptr;
  {
    uint32_t lb = 0;   // the chunk tables in LDS when they fit 64 KiB (else read from HBM)
    for (const auto& blob : e->sampling_chunks_host)
      lb += (std::min<uint32_t>(reinterpret_cast<const SampCfgDev*>(blob.data())->total_bytes, kSampCfgLds) + 15u) & ~15u;
    a.cfg_lds_bytes = lb <= 65536 ? lb : 0;
  }
  a.hist = reinterpret_cast<uint32_t*>(base + off_hist);
  a.hoff = reinterpret_cast<uint32_t*>(base + off_hoff);
  a.counts = counts;
  a.send = static_cast<uint8_t*>(send);
  a.pack_pos = pack_pos;
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
    launch_shard_counts(a, st);
    launch_shard_scatter(a, st);
    e->prof_end(tm, st);
    if (hipGetLastError() != hipSuccess) rc = fail(OSE_EDEVICE, "shard pack launch failed");
  } while (0);
  e->release_ws(ws, st);
  return rc;
}

int ose_shard_unpack(const void* recv, uint64_t n, uint32_t rec_bytes, uint64_t* trace_id, uint64_t* start_ns,
                     uint64_t* end_ns, uint8_t* status, uint32_t* resource, uint32_t* res_svc, uint32_t* res_svc_str,
                     uint64_t* route_match, uint64_t* svc_match, void* hip_stream) {
  if (rec_bytes < x_rec_bytes(1) || (rec_bytes - 8 * kXFixedWords) % 16)
    return fail(OSE_EINVAL, "rec_bytes must be ose_shard_record_bytes()");
  const uint32_t K = (rec_bytes - 8 * kXFixedWords) / 16;   // rule chunks: route_match / svc_match hold K planes
  if (n && (!recv || !trace_id || !start_ns || !end_ns || !status || !resource || !res_svc || !res_svc_str ||
            !route_match || !svc_match))
    return fail(OSE_EINVAL, "NULL argument");
  UnpackArgs a{static_cast<const uint8_t*>(recv), n, K, trace_id, start_ns, end_ns, status, resource, res_svc, res_svc_str,
               route_match, svc_match};
  launch_shard_unpack(a, static_cast<hipStream_t>(hip_stream));
  HIP_TRY(hipGetLastError());
  return 0;
}

int ose_shard_decide(ose_engine* eng, const void* recv, uint64_t n, uint32_t rec_bytes, uint8_t* keep,
                     uint32_t* device_status, const ose_rand* rnd, void* hip_stream) {
  if (!eng) return fail(OSE_EINVAL, "NULL engine");
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (!e->has_sampling) return fail(OSE_EINVAL, "ose_shard_decide needs odigossampling on the engine");
  const uint32_t K = (uint32_t)e->sampling_chunks_dev.size();
  if (rec_bytes != x_rec_bytes(K)) return fail(OSE_EINVAL, "rec_bytes must be ose_shard_record_bytes(eng)");
  if (n > 0xFFFFFFF0ull) return fail(OSE_ERANGE, "more than 2^32-16 records");
  if (n && (!recv || !keep)) return fail(OSE_EINVAL, "NULL argument");
  if (int brc = bind_device(e)) return brc;
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  XScratch* xs = scratch_of(e);
  std::lock_guard<std::mutex> g(xs->mu);
  if (!xs->done) HIP_TRY(hipEventCreateWithFlags(&xs->done, hipEventDisableTiming));
  if (xs->done_set) HIP_TRY(hipStreamWaitEvent(st, xs->done, 0));
  const int rc = owner_decide(e, xs, static_cast<const uint8_t*>(recv), n, K, keep, device_status, rnd, st);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(xs->done, st));
  xs->done_set = true;
  return 0;
}

int ose_shard_scatter_keep(const uint8_t* keep_back, const uint32_t* pack_pos, uint64_t n, uint8_t* keep,
                           void* hip_stream) {
  if (n && (!keep_back || !pack_pos || !keep)) return fail(OSE_EINVAL, "NULL argument");
  launch_scatter_keep(keep_back, pack_pos, n, keep, static_cast<hipStream_t>(hip_stream));
  HIP_TRY(hipGetLastError());
  return 0;
}

// ---- RCCL -----------------------------------------------------------------------
int ose_nccl_unique_id(void* id_out, size_t cap) {
  if (!id_out || cap < NCCL_UNIQUE_ID_BYTES) return fail(OSE_EINVAL, "id buffer must hold 128 bytes");
  const Rccl& r = rccl();
  if (!r.ok) return fail(OSE_ENOTSUP, "RCCL (librccl.so.1) is not available");
  ncclUniqueId id;
  NCCL_TRY(r.get_unique_id(&id));
  std::memcpy(id_out, &id, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int ose_nccl_comm_init(void** comm_out, int n_ranks, const void* id, int rank) {
  if (!comm_out || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(OSE_EINVAL, "bad argument");
  const Rccl& r = rccl();
  if (!r.ok) return fail(OSE_ENOTSUP, "RCCL (librccl.so.1) is not available");
  int rc = ensure_device();
  if (rc) return rc;
  ncclUniqueId uid;
  std::memcpy(&uid, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  NCCL_TRY(r.comm_init_rank(&comm, n_ranks, uid, rank));
  *comm_out = comm;
  return 0;
}

void ose_nccl_comm_destroy(void* comm) {
  LastErrorScope keep("ose_nccl_comm_destroy");
  if (comm && rccl().ok) (void)rccl().comm_destroy(static_cast<ncclComm_t>(comm));
}

int ose_allreduce_counters(const int64_t* local, int64_t* node, uint64_t n, void* nccl_comm, void* hip_stream) {
  if (!nccl_comm || (n && (!local || !node))) return fail(OSE_EINVAL, "NULL argument");
  const Rccl& r = rccl();
  if (!r.ok) return fail(OSE_ENOTSUP, "RCCL (librccl.so.1) is not available");
  if (!n) return 0;
  RcclTransport tx(static_cast<ncclComm_t>(nccl_comm), 0);
  return tx.allreduce_i64(local, node, n, static_cast<hipStream_t>(hip_stream));
}

int ose_exchange_sample(ose_engine* eng, const ose_columns* cols, const ose_outputs* outs, void* nccl_comm,
                        int rank, int n_ranks, const ose_rand* rnd, void* hip_stream, uint64_t* stats) {
  if (!eng || !cols || !outs || !nccl_comm) return fail(OSE_EINVAL, "NULL argument");
  const Rccl& r = rccl();
  if (!r.ok) return fail(OSE_ENOTSUP, "RCCL (librccl.so.1) is not available");
  RcclTransport tx(static_cast<ncclComm_t>(nccl_comm), n_ranks);
  return exchange_round(reinterpret_cast<Engine*>(eng), cols, outs, tx, rank, n_ranks, rnd,
                        static_cast<hipStream_t>(hip_stream), stats);
}

// ---- test seam: in-process ranks (no RCCL) ---------------------------------------
// test hook: 1 when the engine's last owner decision (ose_shard_decide or
// the round's) fell back to the general path
uint32_t osehost_owner_last_general(ose_engine* eng) {
  if (!eng) return 0;
  XScratch* xs = scratch_of(reinterpret_cast<Engine*>(eng));
  std::lock_guard<std::mutex> g(xs->mu);
  return xs->last_general ? 1u : 0u;
}

int osehost_xgroup_create(int n_ranks, void** out) {
  if (!out || n_ranks < 1 || n_ranks > 64) return fail(OSE_EINVAL, "n_ranks must be in 1..64");
  *out = new LocalGroup(n_ranks);
  return 0;
}
void osehost_xgroup_destroy(void* grp) {
  LastErrorScope keep("osehost_xgroup_destroy");
  delete static_cast<LocalGroup*>(grp);
}
int osehost_exchange_sample_local(ose_engine* eng, const ose_columns* cols, const ose_outputs* outs, void* grp,
                                  int rank, const ose_rand* rnd, void* hip_stream, uint64_t* stats) {
  if (!eng || !cols || !outs || !grp) return fail(OSE_EINVAL, "NULL argument");
  auto* g = static_cast<LocalGroup*>(grp);
  if (rank < 0 || rank >= g->n_ranks) return fail(OSE_EINVAL, "rank out of range");
  LocalTransport tx(g, rank);
  return exchange_round(reinterpret_cast<Engine*>(eng), cols, outs, tx, rank, g->n_ranks, rnd,
                        static_cast<hipStream_t>(hip_stream), stats);
}
int osehost_allreduce_counters_local(const int64_t* local, int64_t* node, uint64_t n, void* grp, int rank,
                                     void* hip_stream) {
  if (!grp || (n && (!local || !node))) return fail(OSE_EINVAL, "NULL argument");
  auto* g = static_cast<LocalGroup*>(grp);
  if (rank < 0 || rank >= g->n_ranks) return fail(OSE_EINVAL, "rank out of range");
  LocalTransport tx(g, rank);
  return tx.allreduce_i64(local, node, n, static_cast<hipStream_t>(hip_stream));
}

}  // extern "C"
