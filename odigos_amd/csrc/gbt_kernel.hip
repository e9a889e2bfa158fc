// gbt_kernel.hip — the GPU-resident groupbytrace store.
//
// Spans wait in HBM until their trace's wait_duration has passed, then
// leave as one batch in which every released trace is contiguous: the
// batch the three processors see is the sequence of per-trace calls
// groupbytrace makes, and SAMPLE with OSE_GROUP_TRACE_ID decides each trace
// as its own call would.
//
// State (gbt_host.cpp owns the buffers and the host-side clock):
//   * traces are numbered in creation order (seq, 64-bit); the ring of
//     num_traces ids (contrib's ringBuffer) is ring_tid[seq % num_traces],
//     so a trace created num_traces creations after another evicts it;
//     with num_workers W > 1 each worker has its own ring of num_traces / W
//     ids (contrib's eventMachineWorker.buffer): a trace's worker is
//     fnv64(id) % W, its number q within the worker is kept in tinfo, and
//     it is evicted by its worker's trace number q + num_traces / W;
//   * the id -> seq table persists across adds (tombstones: an id whose
//     trace is gone reclaims its own slot; the table is re-inserted from the
//     live traces only when it grows or tombstones fill half of it); the
//     batch's spans look themselves up, and ids without a live trace start
//     new traces, numbered in the order of their first span in the batch;
//   * spans go to a pool ring in arrival order (columns + a string block in
//     an arena ring), scopes to a scope ring (the fragment's resource and
//     scope columns);
//   * a release takes the traces created before now - wait_duration: a
//     contiguous seq range.  Its spans are flagged in the pool window,
//     compacted, stably sorted by seq (arrival order kept inside a trace)
//     and gathered into fresh columns, one resource and one scope per
//     fragment (a run of one trace from one scope of one added batch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"

namespace ose {

namespace {
constexpr int kGbtThreads = 256;
constexpr uint64_t kUnset = ~0ull;

// contrib's workerIndexForTraceID: FNV-1 (64-bit) over the id's 16 bytes,
// modulo the workers (ids are {hi, lo}, big-endian)
__device__ __forceinline__ uint32_t gbt_worker(uint64_t hi, uint64_t lo, uint32_t n_workers) {
  uint64_t h = 14695981039346656037ull;
#pragma unroll
  for (int b = 0; b < 16; b++) {
    h *= 1099511628211ull;
    h ^= ((b < 8 ? hi : lo) >> (56 - 8 * (b & 7))) & 0xFFu;
  }
  return (uint32_t)(h % n_workers);
}

// a trace whose worker has numbered worker_cap more traces after it: the
// last of them took its ring slot (one worker: the contiguous eviction is in
// live_lo instead)
__device__ __forceinline__ bool gbt_evicted(const GbtArgs& a, uint64_t seq) {
  if (a.n_workers <= 1) return false;
  const uint64_t t = a.tinfo[seq % a.ring_n];
  return a.wcnt[t >> 40] > (t & ((1ull << 40) - 1)) + a.worker_cap;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// The id table persists across adds.  A slot holds an id and the creation
// number of its newest trace; the trace is live for an added span iff that
// number is in [live_lo, live_hi) (not released, evicted or expired).  A
// slot whose trace is no longer live stays as a tombstone: lookups of other
// ids probe past it, and its own id takes it back (reclaim) when it comes
// again.  The host bumps the epoch and re-inserts the live traces only when
// the table grows or tombstones fill half of it, so an add costs O(batch),
// not O(traces waiting).
//
// Slots are published with the trace table's protocol (trace_kernel.hip): a
// stale-epoch slot is claimed BUSY, its fields stored with agent-scope
// stores, drained, then READY.

// rebuild: one live trace per id (an id's expired instance is outside
// [live_lo, live_hi), so each id occurs at most once; the newest wins anyway)
__device__ void gbt_put(const GbtArgs& a, uint64_t hi, uint64_t lo, uint64_t seq) {
  const uint32_t busy = (a.epoch << 2) | 1u, ready = (a.epoch << 2) | 2u;
  uint64_t h = mix64(hi ^ mix64(lo)) & a.table_mask;
  uint32_t probes = 0, spins = 0;
  for (;;) {
    GbtSlot* s = &a.table[h];
    const uint32_t st = __hip_atomic_load(&s->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((st >> 2) != a.epoch) {
      uint32_t expect = st;
      if (__hip_atomic_compare_exchange_strong(&s->state, &expect, busy, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(&s->hi, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->lo, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->first, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&s->state, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      continue;
    }
    if ((st & 3u) != 2u) {
      if (++spins > (1u << 20)) {
        atomicOr(a.error, 1u);
        return;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (__hip_atomic_load(&s->hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == hi &&
        __hip_atomic_load(&s->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == lo) {
      __hip_atomic_fetch_max(&s->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    h = (h + 1) & a.table_mask;
    if (++probes > a.table_mask) {
      atomicOr(a.error, 4u);
      return;
    }
  }
}

// lookup of an added span: the slot of its id, which holds either a live
// trace or (claimed or reclaimed for this add) kGbtUnset | add_gen with the
// smallest batch position of the id in `first`.  UINT64_MAX on failure.
__device__ uint64_t gbt_lookup(const GbtArgs& a, uint64_t hi, uint64_t lo, uint32_t pos) {
  const uint32_t busy = (a.epoch << 2) | 1u, ready = (a.epoch << 2) | 2u;
  const uint64_t mine = kGbtUnset | a.add_gen;
  uint64_t h = mix64(hi ^ mix64(lo)) & a.table_mask;
  uint32_t probes = 0, spins = 0;
  for (;;) {
    GbtSlot* s = &a.table[h];
    const uint32_t st = __hip_atomic_load(&s->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((st >> 2) != a.epoch) {   // empty: the id is not in the table
      uint32_t expect = st;
      if (__hip_atomic_compare_exchange_strong(&s->state, &expect, busy, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(&s->hi, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->lo, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->seq, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->first, pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&s->state, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return h;
      }
      continue;
    }
    if ((st & 3u) != 2u) {   // another lane is publishing or reclaiming this slot
      if (++spins > (1u << 20)) {
        atomicOr(a.error, 1u);
        return ~0ull;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (__hip_atomic_load(&s->hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != hi ||
        __hip_atomic_load(&s->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != lo) {
      h = (h + 1) & a.table_mask;   // another id (live or a tombstone)
      if (++probes > a.table_mask) {
        atomicOr(a.error, 4u);
        return ~0ull;
      }
      continue;
    }
    const uint64_t seq = __hip_atomic_load(&s->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seq == mine) {   // numbered by this add
      atomicMin(&s->first, pos);
      return h;
    }
    if (seq < kGbtUnset && seq >= a.live_lo && seq < a.live_hi && !gbt_evicted(a, seq)) return h;   // a live trace
    // the id's last trace is gone (released, evicted, expired) or an earlier
    // add failed while numbering it: the id starts a new trace in this slot
    uint32_t expect = st;
    if (__hip_atomic_compare_exchange_strong(&s->state, &expect, busy, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
      if (__hip_atomic_load(&s->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mine) {
        atomicMin(&s->first, pos);   // reclaimed by another lane between our reads
      } else {
        // first before seq, drained between them: a lane that read the state
        // as READY before this CAS may still read seq; once it sees `mine`
        // its atomicMin must land after this store, not under it
        __hip_atomic_store(&s->first, pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&s->seq, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&s->state, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return h;
    }
  }
}

// ---- add -------------------------------------------------------------------

// the live traces [live_lo, live_hi) back into a fresh epoch of the table
__global__ __launch_bounds__(kGbtThreads) void gbt_rebuild_kernel(GbtArgs a) {
  for (uint64_t s = a.live_lo + (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x; s < a.live_hi;
       s += (uint64_t)gridDim.x * kGbtThreads) {
    if (gbt_evicted(a, s)) continue;
    const uint64_t r = s % a.ring_n;
    gbt_put(a, a.ring_tid[2 * r], a.ring_tid[2 * r + 1], s);
  }
}

// every span of the batch: its table slot
__global__ __launch_bounds__(kGbtThreads) void gbt_lookup_kernel(GbtArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (i >= a.n) return;
  a.slot_of[i] = gbt_lookup(a, a.cols.trace_id[2 * i], a.cols.trace_id[2 * i + 1], (uint32_t)i);
}

// creators (the first span of each new trace) and each span's string block length
__global__ __launch_bounds__(kGbtThreads) void gbt_creator_kernel(GbtArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t h = a.slot_of[i];
  uint32_t f = 0;
  if (h != ~0ull) {
    const GbtSlot& s = a.table[h];
    f = s.seq == (kGbtUnset | a.add_gen) && s.first == (uint32_t)i;
  }
  a.flag[i] = f;
  const ose_columns& c = a.cols;
  uint32_t len = 0;
  if (c.route) len += c.route[i].len;
  if (c.path) len += c.path[i].len;
  for (uint32_t k = 0; k < a.n_attr_keys; k++)
    if (c.attr_type[(uint64_t)k * a.n + i] == OSE_ATTR_STR) len += (uint32_t)(c.attr_val[(uint64_t)k * a.n + i] >> 32);
  a.strlen[i] = len;
}

// the batch's strings do not fit the arena ring: nothing of the batch is
// stored (no trace numbered, no ring slot overwritten) and the add fails
__device__ __forceinline__ bool gbt_batch_refused(const GbtArgs& a) {
  return (uint64_t)a.totals[1] > a.arena_room;
}

// new traces numbered in first-appearance order; the ring remembers their ids
__global__ __launch_bounds__(kGbtThreads) void gbt_assign_kernel(GbtArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (gbt_batch_refused(a)) {
    if (i == 0) atomicOr(a.error, 8u);
    return;
  }
  if (i >= a.n || !a.flag[i]) return;
  const uint64_t seq = a.next_seq + a.rank[i];
  a.table[a.slot_of[i]].seq = seq;
  const uint64_t r = seq % a.ring_n;
  a.ring_tid[2 * r] = a.cols.trace_id[2 * i];
  a.ring_tid[2 * r + 1] = a.cols.trace_id[2 * i + 1];
}

// the spans into the pool ring
__global__ __launch_bounds__(kGbtThreads) void gbt_append_kernel(GbtArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (i >= a.n || gbt_batch_refused(a)) return;
  const GbtPool& P = a.pool;
  const ose_columns& c = a.cols;
  const uint64_t p = (a.pool_pos + i) % a.pool_cap;
  const uint64_t h = a.slot_of[i];
  P.seq[p] = h == ~0ull ? kUnset : a.table[h].seq;
  P.tid[2 * p] = c.trace_id[2 * i];
  P.tid[2 * p + 1] = c.trace_id[2 * i + 1];
  P.start[p] = c.start_ns[i];
  P.end[p] = c.end_ns[i];
  P.status[p] = c.status[i];
  P.kind[p] = c.kind[i];
  P.url_flags[p] = c.url_flags ? c.url_flags[i] : 0;
  P.span_size[p] = c.span_size ? c.span_size[i] : 0;
  P.name_len[p] = c.name_len ? c.name_len[i] : 0;
  for (uint32_t w = 0; w < a.attr_words; w++)
    P.attr_match[w * a.pool_cap + p] = c.attr_match ? c.attr_match[w * a.n + i] : 0;
  P.origin[p] = a.scope_pos + c.scope[i];
}

__device__ __forceinline__ void ring_copy(uint8_t* ring, uint64_t cap, uint64_t dst, const uint8_t* src, uint32_t n) {
  uint64_t q = dst % cap;
  for (uint32_t b = 0; b < n; b++) {
    ring[q] = src[b];
    if (++q == cap) q = 0;
  }
}

// the string block: route, path, then the string attribute values; refs in
// the pool are relative to the block
__global__ __launch_bounds__(kGbtThreads) void gbt_strings_kernel(GbtArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (i >= a.n || gbt_batch_refused(a)) return;
  const GbtPool& P = a.pool;
  const ose_columns& c = a.cols;
  const uint64_t p = (a.pool_pos + i) % a.pool_cap;
  const uint64_t blk = a.arena_pos + a.stroff[i];
  P.str_off[p] = blk;
  uint32_t rel = 0;
  ose_strref r{0, 0};
  if (c.route) {
    const ose_strref x = c.route[i];
    ring_copy(a.arena_ring, a.arena_cap, blk + rel, c.arena + x.off, x.len);
    r = ose_strref{rel, x.len};
    rel += x.len;
  }
  P.route[p] = r;
  r = ose_strref{0, 0};
  if (c.path) {
    const ose_strref x = c.path[i];
    ring_copy(a.arena_ring, a.arena_cap, blk + rel, c.arena + x.off, x.len);
    r = ose_strref{rel, x.len};
    rel += x.len;
  }
  P.path[p] = r;
  for (uint32_t k = 0; k < a.n_attr_keys; k++) {
    const uint8_t t = c.attr_type[(uint64_t)k * a.n + i];
    uint64_t v = c.attr_val[(uint64_t)k * a.n + i];
    if (t == OSE_ATTR_STR) {
      const uint32_t off = (uint32_t)v, len = (uint32_t)(v >> 32);
      ring_copy(a.arena_ring, a.arena_cap, blk + rel, c.arena + off, len);
      v = (uint64_t)rel | ((uint64_t)len << 32);
      rel += len;
    }
    P.attr_type[(uint64_t)k * a.pool_cap + p] = t;
    P.attr_val[(uint64_t)k * a.pool_cap + p] = v;
  }
}

// the batch's scopes into the scope ring, with their resource's columns
__global__ __launch_bounds__(kGbtThreads) void gbt_scopes_kernel(GbtArgs a) {
  const uint64_t s = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (s >= a.n_scopes || gbt_batch_refused(a)) return;
  const ose_columns& c = a.cols;
  const GbtScopes& Q = a.scopes;
  const uint64_t q = (a.scope_pos + s) % a.scope_cap;
  const uint32_t r = c.scope_resource[s];
  Q.res_svc[q] = c.res_svc[r];
  Q.res_svc_str[q] = c.res_svc_str ? c.res_svc_str[r] : c.res_svc[r];
  Q.res_url_ok[q] = c.res_url_ok ? c.res_url_ok[r] : 1;
  const uint32_t set = c.res_attrset[r];
  Q.res_attrset[q] = a.attrset_map ? a.attrset_map[set] : set;
  Q.res_size[q] = c.res_size ? c.res_size[r] : 0;
  Q.scope_size[q] = c.scope_size ? c.scope_size[s] : 0;
}

// ---- per-worker numbering (num_workers > 1), after the add's kernels -------

// the batch's new traces as (worker, creation rank) pairs, and how many each
// worker gets
__global__ __launch_bounds__(kGbtThreads) void gbt_wkey_kernel(GbtArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (i >= a.n || !a.flag[i]) return;
  const uint32_t k = a.rank[i];
  const uint32_t w = gbt_worker(a.cols.trace_id[2 * i], a.cols.trace_id[2 * i + 1], a.n_workers);
  a.keys[k] = w;
  a.vals[k] = k;
  atomicAdd(&a.wadd[w], 1u);
}

// the pairs stably sorted by worker: the j-th is its worker's
// (j - wstart[w])-th new trace, after the wcnt[w] it had
__global__ __launch_bounds__(kGbtThreads) void gbt_wnum_kernel(GbtArgs a, uint64_t created) {
  const uint64_t j = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (j >= created) return;
  const uint32_t w = a.keys[j];
  const uint64_t q = a.wcnt[w] + (j - a.wstart[w]);
  a.tinfo[(a.next_seq + a.vals[j]) % a.ring_n] = (uint64_t)w << 40 | q;
}

// ---- release ---------------------------------------------------------------

// the pool window's spans of released traces (seq in [rel_lo, rel_hi))
__global__ __launch_bounds__(kGbtThreads) void gbt_flag_kernel(GbtArgs a) {
  const uint64_t w = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (w >= a.n) return;
  const uint64_t seq = a.pool.seq[(a.pool_pos + w) % a.pool_cap];
  a.flag[w] = seq >= a.rel_lo && seq < a.rel_hi && !gbt_evicted(a, seq);
}

__global__ __launch_bounds__(kGbtThreads) void gbt_compact_kernel(GbtArgs a) {
  const uint64_t w = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (w >= a.n || !a.flag[w]) return;
  const uint32_t d = a.rank[w];
  a.keys[d] = (uint32_t)(a.pool.seq[(a.pool_pos + w) % a.pool_cap] - a.rel_lo);
  a.vals[d] = (uint32_t)w;
}

// output span j <- pool window position order[j]: fixed columns, fragment
// heads (a new trace or a new origin scope), string block lengths
__global__ __launch_bounds__(kGbtThreads) void gbt_gather_kernel(GbtArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (j >= a.n) return;
  const GbtPool& P = a.pool;
  const GbtOut& O = a.out;
  const uint64_t p = (a.pool_pos + a.order[j]) % a.pool_cap;
  O.tid[2 * j] = P.tid[2 * p];
  O.tid[2 * j + 1] = P.tid[2 * p + 1];
  O.start[j] = P.start[p];
  O.end[j] = P.end[p];
  O.status[j] = P.status[p];
  O.kind[j] = P.kind[p];
  O.url_flags[j] = P.url_flags[p];
  O.span_size[j] = P.span_size[p];
  O.name_len[j] = P.name_len[p];
  for (uint32_t w = 0; w < a.attr_words; w++) O.attr_match[w * a.n + j] = P.attr_match[w * a.pool_cap + p];
  uint32_t head = 1;
  if (j > 0) {
    const uint64_t q = (a.pool_pos + a.order[j - 1]) % a.pool_cap;
    head = P.seq[q] != P.seq[p] || P.origin[q] != P.origin[p];
  }
  a.flag[j] = head;
  uint32_t len = P.route[p].len + P.path[p].len;
  for (uint32_t k = 0; k < a.n_attr_keys; k++)
    if (P.attr_type[(uint64_t)k * a.pool_cap + p] == OSE_ATTR_STR)
      len += (uint32_t)(P.attr_val[(uint64_t)k * a.pool_cap + p] >> 32);
  a.strlen[j] = len;
}

// strings, refs, resource / scope ids and the fragment columns
__global__ __launch_bounds__(kGbtThreads) void gbt_emit_kernel(GbtArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * kGbtThreads + threadIdx.x;
  if (j >= a.n) return;
  const GbtPool& P = a.pool;
  const GbtOut& O = a.out;
  const uint64_t p = (a.pool_pos + a.order[j]) % a.pool_cap;
  const uint32_t f = a.rank[j] + a.flag[j] - 1;   // fragment index (inclusive scan - 1)
  O.resource[j] = f;
  O.scope[j] = f;
  const uint32_t base = a.stroff[j];
  const uint64_t blk = P.str_off[p];
  const uint32_t len = P.route[p].len + P.path[p].len;
  uint32_t total = len;
  for (uint32_t k = 0; k < a.n_attr_keys; k++)
    if (P.attr_type[(uint64_t)k * a.pool_cap + p] == OSE_ATTR_STR)
      total += (uint32_t)(P.attr_val[(uint64_t)k * a.pool_cap + p] >> 32);
  uint64_t q0 = blk % a.arena_cap;
  for (uint32_t b = 0; b < total; b++) {
    O.arena[base + b] = a.arena_ring[q0];
    if (++q0 == a.arena_cap) q0 = 0;
  }
  const ose_strref r = P.route[p], q = P.path[p];
  O.route[j] = ose_strref{base + r.off, r.len};
  O.path[j] = ose_strref{base + q.off, q.len};
  for (uint32_t k = 0; k < a.n_attr_keys; k++) {
    const uint8_t t = P.attr_type[(uint64_t)k * a.pool_cap + p];
    uint64_t v = P.attr_val[(uint64_t)k * a.pool_cap + p];
    if (t == OSE_ATTR_STR) v = (uint64_t)(base + (uint32_t)v) | (v & 0xFFFFFFFF00000000ull);
    O.attr_type[(uint64_t)k * a.n + j] = t;
    O.attr_val[(uint64_t)k * a.n + j] = v;
  }
  if (a.flag[j]) {
    const GbtScopes& Q = a.scopes;
    const uint64_t o = P.origin[p] % a.scope_cap;
    O.res_svc[f] = Q.res_svc[o];
    O.res_svc_str[f] = Q.res_svc_str[o];
    O.res_url_ok[f] = Q.res_url_ok[o];
    O.res_attrset[f] = Q.res_attrset[o];
    O.res_size[f] = Q.res_size[o];
    O.scope_size[f] = Q.scope_size[o];
    O.scope_resource[f] = f;
  }
}

uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kGbtThreads - 1) / kGbtThreads); }
}  // namespace

#define GBT_LAUNCH(k, n) hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kGbtThreads), 0, st, a)

void launch_gbt_rebuild(const GbtArgs& a, hipStream_t st) {
  const uint64_t n = a.live_hi - a.live_lo;
  if (!n) return;
  const uint32_t b = (uint32_t)std::min<uint64_t>(blocks_for(n), 4096);
  hipLaunchKernelGGL(gbt_rebuild_kernel, dim3(b), dim3(kGbtThreads), 0, st, a);
}
void launch_gbt_lookup(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_lookup_kernel, a.n); }
void launch_gbt_creator(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_creator_kernel, a.n); }
void launch_gbt_assign(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_assign_kernel, a.n); }
void launch_gbt_append(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_append_kernel, a.n); }
void launch_gbt_strings(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_strings_kernel, a.n); }
void launch_gbt_scopes(const GbtArgs& a, hipStream_t st) {
  if (a.n_scopes) hipLaunchKernelGGL(gbt_scopes_kernel, dim3(blocks_for(a.n_scopes)), dim3(kGbtThreads), 0, st, a);
}
void launch_gbt_flag(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_flag_kernel, a.n); }
void launch_gbt_compact(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_compact_kernel, a.n); }
void launch_gbt_gather(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_gather_kernel, a.n); }
void launch_gbt_emit(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_emit_kernel, a.n); }
void launch_gbt_wkey(const GbtArgs& a, hipStream_t st) { GBT_LAUNCH(gbt_wkey_kernel, a.n); }
void launch_gbt_wnum(const GbtArgs& a, uint64_t created, hipStream_t st) {
  if (created) hipLaunchKernelGGL(gbt_wnum_kernel, dim3(blocks_for(created)), dim3(kGbtThreads), 0, st, a, created);
}

}  // namespace ose
