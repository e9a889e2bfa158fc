// kernels.hpp — host-side launch interfaces of the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/odigos_amd.h"

// OSE_DIAG=1: the diagnostics build (python -m odigos_amd.build --variant _diag
// OSE_DIAG=1; loaded with OSE_LIB_VARIANT=_diag): ablation switches, per-section
// clocks and tuning knobs read from the environment.  The product library is
// built without it and reads no such variable.
#ifndef OSE_DIAG
#define OSE_DIAG 0
#endif

namespace ose {

// odigosurltemplate: four launches on one stream (url_kernel.hip).
//   url_plan_kernel  one wave per 64-span group: plan, output length per span
//                    and the group's template bytes, assembled in LDS and
//                    stored to the wave's scratch region
//   url_plan_slow_kernel  the groups the plan kernel could not plan from its
//                    LDS stage (byte range over the stage, segment list
//                    overflow, a segment over 64 bytes): planned per span from HBM
//   url_scan_kernel  exclusive scan of the per-group output sums
//   url_copy_kernel  one wave per group: template refs, and the group's bytes
//                    copied from scratch to their place in the output arena
//   url_emit_slow_kernel  the groups the plan kernel could not assemble (user
//                    rules, oversized groups), from the plan arrays
struct SizePart {            // one resource run's share of a 64-scope window
  uint32_t r;                 // the resource
  uint32_t ch;                // alive scopes (bits 0-29) | had spans << 30 | whole side << 31
  uint64_t v;                 // framed scope bytes
};
struct SizeKernelArgs {
  uint64_t n_spans;
  uint32_t n_scopes, n_resources, n_attrsets;
  uint32_t sampled;           // SAMPLE ran in this call: keep decides which spans survive
  uint32_t templated;         // TEMPLATE ran: url_out / tmpl grow the spans
  uint32_t remove_empty;      // OSE_GROUP_TRACE_ID sampling: emptied scopes/resources are removed
  const uint32_t* batch_keep; // OSE_GROUP_BATCH sampling: 0 empties the whole call (null otherwise)
  const uint32_t* span_size;
  const uint32_t* name_len;
  const uint32_t* scope;
  const uint32_t* scope_size;
  const uint32_t* scope_resource;
  const uint32_t* res_size;
  const uint32_t* res_attrset;
  const uint8_t* keep;
  const uint8_t* url_out;
  const uint8_t* kind;
  const ose_strref* tmpl;
  int64_t inverse;
  uint64_t* scope_body;       // [S] zeroed: body bytes | runs that added << kSumBits (size_device.hpp)
  // the fused scopes + resources pass (size_tail_kernel): per 64-scope window
  // its first and last resource run's partial sums, and whether the window
  // holds the end of a run that began in an earlier window (size_fix_kernel)
  SizePart* parts;            // [2 * n_swin], written every call
  uint32_t* fix;              // [n_swin], written every call
  uint32_t n_swin;            // ceil(n_scopes / 64)
  int64_t* attrset_bytes;     // [n_attrsets] added to
  int64_t* accepted;          // [1] added to
  uint64_t* res_bytes;        // [R] or null
  // the spans pass ran fused in url_copy_kernel: the surviving spans counted
  // per block there, summed by size_tail_kernel (null: size_span_kernel counted)
  const uint32_t* kept_partials;
  uint32_t n_kept_partials;
};

struct UrlKernelArgs {
  uint64_t n_spans;
  uint32_t n_groups;           // ceil(n_spans / kUrlGroup)
  const uint8_t* arena;
  const uint8_t* url_flags;
  const uint8_t* kind;
  const uint32_t* resource;
  const uint8_t* res_url_ok;   // may be null (no include/exclude)
  const ose_strref* path;
  uint8_t* url_out;
  ose_strref* tmpl;
  uint8_t* out_arena;
  uint64_t out_cap;
  const uint8_t* cfg;          // UrlCfgDev blob
  // workspace
  uint32_t* plan_len;          // [n_spans] output length
  uint32_t* plan_meta;         // [n_spans] mode/lead/slow/url_out/field (slow groups only)
  uint64_t* plan_code;         // [n_spans] per-segment name ids (slow groups only)
  uint8_t* scratch;            // assembled group images: wave w owns [w * scr_region, +scr_region)
  uint64_t scr_region;         // bytes per wave (multiple of 16)
  uint64_t* group_scr;         // [n_groups] scratch offset of the group's image, ~0: slow group
  uint64_t* group_sum;         // [n_groups]
  uint64_t* group_base;        // [n_groups] exclusive prefix
  uint32_t n_scan_tiles;       // ceil(n_groups / kUrlScanTile)
  uint32_t* scan_counter;      // zeroed before launch
  uint64_t* scan_status;       // [n_scan_tiles], zeroed before launch
  uint32_t* error;             // bit0 look-back timeout, bit1 output overflow
  uint64_t* used;              // bytes written (optional)
  uint32_t* slow_count;        // groups the plan kernel left to K3s (zeroed before launch)
  uint32_t* slow_groups;       // [n_groups]
  uint32_t* unplanned_count;   // groups the plan kernel left to url_plan_slow_kernel (zeroed before launch)
  uint32_t* unplanned;         // [n_groups]
  uint32_t general;            // user rules or custom ids configured (selects the general kernel instances)
  // OSE_STAGE_TEMPLATE_REFS: scratch is the caller's tmpl_arena (== out_arena),
  // the fast groups' images stay where url_plan_kernel wrote them (their refs
  // point there, url_copy_kernel copies nothing).  A plan wave takes its
  // image space in chunks of refs_chunk bytes from *bump (zeroed before the
  // launch); the scan places the slow groups from the final *bump on.
  uint32_t refs;
  uint64_t* bump;
  uint64_t refs_chunk;          // url_refs_chunk()
  uint32_t plan_waves;          // url_plan_waves()
  uint64_t* slow_aligned;       // refs: sum of the scan-placed groups' sizes rounded up to 16 (zeroed)
  uint32_t plan_grid_mult;     // refs form beside the trace stage: plan workgroups = resident x this (run_stages)
  uint32_t ablate;             // diagnostics only (OSE_URL_ABLATE): 1 skip emission, 2 skip planning, 4 skip bitmaps
  uint64_t* dbg;               // diagnostics only (ablate & 512): per-section clock sums
  // odigostrafficmetrics' spans pass fused into url_copy_kernel (TEMPLATE and
  // SIZE in one call): sz as size_span_kernel would get it, sz.tmpl unused
  // (the plan lengths are the template lengths); the kept count of block b
  // goes to size_partials[b] (launch_url_copy's grid, <= kUrlCopyMaxBlocks)
  uint32_t fuse_size;
  uint32_t* size_partials;
  SizeKernelArgs sz;
};
constexpr uint32_t kUrlCopyMaxBlocks = 65536;
uint32_t url_copy_blocks(uint32_t n_groups);
constexpr uint32_t kUrlGroup = 64;       // spans per wave group (url_kernel.hip kWave)
constexpr uint32_t kUrlScanTile = 1024;  // groups per scan workgroup (url_kernel.hip kScanThreads)
// workspace bytes the URL stage needs for n spans (engine.cpp run_url layout)
constexpr uint32_t kUrlMaxWaves = 4096;  // waves of the persistent plan grid (>= its resident waves)
constexpr uint32_t kUrlWaveSlack = 8192; // scratch bytes per wave on top of its share
// scratch for the assembled group images of a batch whose arena holds
// arena_bytes: the path bytes bound the templates but for inserted names,
// hence 1.25x plus a per-wave slack; a group that does not fit its wave's
// region is emitted by url_emit_slow_kernel instead
inline size_t url_scratch_bytes(uint64_t n, uint64_t arena_bytes) {
  const uint64_t g = (n + kUrlGroup - 1) / kUrlGroup;
  const uint64_t w = g < kUrlMaxWaves ? g : kUrlMaxWaves;
  return ((arena_bytes + n + (arena_bytes + n) / 4 + 15) & ~15ull) + w * kUrlWaveSlack;
}
inline size_t url_workspace_bytes(uint64_t n, uint64_t arena_bytes) {
  const uint64_t g = (n + kUrlGroup - 1) / kUrlGroup;
  const uint64_t t = (g + kUrlScanTile - 1) / kUrlScanTile;
  return 16 + t * 8 + 256 + n * 16 + 8 + g * 32 + 512 + 256 + url_scratch_bytes(n, arena_bytes);
}
// refs form: the plan grid in multiples of the resident one, from the batch's
// groups (engine.cpp run_stages); OSE_PLAN_GRID_OLD builds: 16 beside the
// trace stage, 1 otherwise (A/B)
#ifndef OSE_PLAN_GRID_OLD
#define OSE_PLAN_GRID_OLD 0
#endif
inline uint32_t url_plan_grid_mult(uint32_t n_groups, bool forked = false) {
  if (OSE_PLAN_GRID_OLD) return forked ? 16u : 1u;
  const uint32_t m = n_groups / (kUrlMaxWaves * 19u);
  return m < 1 ? 1u : m > 16 ? 16u : m;
}
void launch_url_plan(const UrlKernelArgs& a, hipStream_t st);
uint32_t url_plan_waves(const UrlKernelArgs& a);   // waves of the plan grid (scratch regions)
// refs form: the image chunk size for an arena of `cap` bytes over `waves`
// plan waves (0: every group image takes exactly its size)
uint64_t url_refs_chunk(uint64_t cap, uint32_t waves);
void launch_url_scan(const UrlKernelArgs& a, hipStream_t st);
void launch_url_copy(const UrlKernelArgs& a, hipStream_t st);
void launch_url_plan_slow(const UrlKernelArgs& a, hipStream_t st);
void launch_url_emit_slow(const UrlKernelArgs& a, hipStream_t st);

}  // namespace ose

namespace ose {

// odigossampling: trace grouping, per-trace reduction and the rule fold
// (trace_kernel.hip).  A "position" is an index into the evaluation order:
// the batch order itself (fast path) or the stable sort of spans by trace
// (slow path, perm != null).
struct TraceSlot {            // exact trace_id hash table entry (32 B)
  uint32_t state;             // epoch << 2 | {0 empty, 1 busy, 2 ready}
  uint32_t first;             // smallest run-head position of this trace_id
  uint64_t hi, lo;
  uint64_t _pad;
};
struct TraceRec {             // per-trace record, stored at the trace's head position
  uint32_t first_span;
  uint8_t keep, level, _p0, _p1;
  double ratio;
};
enum : uint32_t { kTraceRuns = 0, kTracePerm = 1, kTraceBatch = 2 };
// ShouldSample's walk between the passes of a rule-chunked configuration
// (sampling_host.cpp build_sampling_tables): the level being folded, its
// evaluateLevel accumulators and the min fallback of the closed levels
struct FoldState {
  double ratio;      // the open level's ratio (after kFsDone: the satisfied level's)
  double min_fb;     // min fallback over closed matched levels (kFsHaveMin)
  uint32_t level;    // the open level (after kFsDone: the satisfied level)
  uint32_t flags;    // kFs*
};
enum : uint32_t { kFsSat = 1, kFsMatched = 2, kFsFoundFb = 4, kFsHaveMin = 8, kFsDone = 16 };
struct SampWalkDev;   // devcfg.hpp
struct TraceKernelArgs {
  uint64_t n_spans;
  uint32_t n_windows;         // ceil(n_spans / 64), >= 1
  uint32_t mode;              // kTrace*
  uint32_t n_resources;
  uint32_t epoch;             // hash table generation (>= 1)
  // rule-chunked passes (both null: one pass, the whole rule list): the
  // state before this chunk's rules (null in the first pass) and after them
  // (null in the last pass, which decides), indexed by the trace's first span
  const FoldState* fold_in;
  FoldState* fold_out;
  const uint64_t* tid;
  const uint64_t* start;
  const uint64_t* end;
  const uint8_t* status;
  const uint32_t* resource;
  const ose_strref* route;
  const uint8_t* arena;
  const uint32_t* res_svc;
  const uint32_t* res_svc_str;
  const uint8_t* cfg;         // SampCfgDev blob
  uint64_t seed;
  uint8_t* keep;              // [n_spans]
  TraceRec* rec;              // [max(n,1)] or null (no per-trace outputs)
  uint64_t* win_heads;        // [n_windows] head bitmap of each window
  // slow path
  TraceSlot* table;            // exact table (slow path)
  uint64_t table_mask;
  uint32_t* dup;              // set by the fast path when a trace_id spans several runs
  // bucketed duplicate detection (kTraceRuns): a run head appends its 64-bit fingerprint to bucket fp >> (64 -
  // dup_bkt_bits); trace_dup_check_kernel looks for a repeat per bucket in LDS
  uint32_t* dup_bkt_count;    // [1 << dup_bkt_bits], zeroed before the launch
  uint64_t* dup_bkt;          // [(1 << dup_bkt_bits) * kDupBucketCap]
  uint32_t dup_bkt_bits;
  const uint32_t* perm;       // kTracePerm: position -> span
  const uint32_t* key;        // kTracePerm: span -> canonical trace (first run-head position)
  uint32_t* error;            // bit0 spin timeout, bit2 trace table full
  uint32_t* batch_keep;       // kTraceBatch: the call's decision (read by the SIZE stage)
  const uint64_t* route_match;// optional precomputed endpoint bits (ose_columns.route_match)
  const uint64_t* attr_match; // span_attribute bits (null when no such rule)
  uint64_t attr_stride;       // attr_match: word w of span i at [w * attr_stride + i]
  uint32_t attr_words;
  const uint64_t* svc_match;  // owner-side records: OR of service_name + span_attribute rule bits (replaces both)
  uint32_t ablate;            // diagnostics only (OSE_TRACE_ABLATE, tools/ablate_trace.py): skip parts
  // kTraceRuns: runs still open kLongSteps steps past their owner's windows
  // are listed here (head positions) and decided by trace_long_kernel
  uint32_t* n_long;           // [0] runs listed, [1] pieces, [3] piece partials (trace_long_plan_kernel)
  uint32_t* long_runs;        // [n_spans / 64 + 1]
  // trace_long_plan_kernel cuts each listed run into pieces of at most
  // kLongPiece spans (one workgroup each): per run {end, pieces, first
  // partial, pieces done}, per piece {run, index}, per piece of a run of
  // several a partial (kLongPartBytes)
  uint4* long_meta;           // [n_spans / 64 + 1]
  uint2* long_pieces;         // [long_piece_cap(n_spans)]
  uint8_t* long_part;         // [long_part_cap(n_spans)][kLongPartBytes]
  uint32_t long_steps;        // hand-off distance in 64-span steps (kLongSteps)
  uint32_t win_per_wave;      // 64-span windows whose run heads one wave owns (kWinPerWave)
  uint32_t narrow;            // the table's flag bits fit one word (trace_eval_kernel kNarrow)
  // every rule chunk in one pass (trace_multi_kernel): n_multi (2..kMaxMulti)
  // chunk tables, copied into cfg_lds_bytes of dynamic LDS (0: one table, a.cfg)
  const uint8_t* const* cfgs;
  uint32_t n_multi;
  uint32_t cfg_lds_bytes;     // the tables, then the latency-service ids (lat_gslot)
  const uint32_t* lat_gslot;  // [n_services] index among the latency services, [64] their service ids
  const SampWalkDev* walks;   // [n_multi] each chunk's rules by what matches them
  // run-list path (repeated trace ids, before the sort-based fallback):
  // trace_runs_kernel lists each trace's runs in its exact-table slot,
  // trace_fold_kernel folds the runs of every trace with 2..kMaxRuns runs
  uint32_t* run_count;        // [table slots] runs listed per slot
  uint32_t* runs;             // [table slots * kMaxRuns] run-head positions
  uint32_t* overflow;         // set when a trace needs the sort-based path
  unsigned long long* path_count;   // engine counters (ose_engine_path_counts): [0] += 1 per run-list pass
  uint64_t* win_first;        // [n_windows] heads that start a trace (first run only)
  uint32_t* head_slot;        // [n_spans] exact-table slot of each run head
};
constexpr uint32_t kMaxRuns = 8;          // runs per trace the run-list path folds
constexpr uint32_t kMaxFoldSpans = 4096;  // spans per trace one lane folds
constexpr uint32_t kMaxFoldSlots = 8;     // latency services per trace one lane folds
#ifndef OSE_WPW_BESIDE
#define OSE_WPW_BESIDE 64
#endif
constexpr uint32_t kWinPerWaveBeside = OSE_WPW_BESIDE;   // beside the forked URL planning (sampling_host.cpp)
constexpr uint32_t kWinPerWave = 16;   // tools/gpu_wpw.sh: C5 0.97 -> 0.83 ms, C3 2.03 -> 1.99 ms, C4 unchanged
#ifndef OSE_LONG_PIECE
#define OSE_LONG_PIECE 2048
#endif
constexpr uint32_t kLongPiece = OSE_LONG_PIECE;   // spans of a long run one wave folds
constexpr uint32_t kLongPartBytes = 1344;    // a piece's partial: m[64], e[64], f[64], ep, svc, kmask, err
inline uint64_t long_piece_cap(uint64_t n) { return n / 64 + 1 + n / kLongPiece + 1; }
inline uint64_t long_part_cap(uint64_t n) { return 2 * (n / kLongPiece) + 2; }   // pieces of runs of > kLongPiece spans
constexpr uint32_t kLongSteps = 4;   // tools/gpu_long_iter.sh: C5 16 -> 4 steps 2.75 -> 2.13 ms, C3 unchanged
void launch_trace_eval(const TraceKernelArgs& a, hipStream_t st);
// rule chunks one trace_multi_kernel pass evaluates, and their LDS budget
constexpr uint32_t kMaxMulti = 3;
constexpr uint32_t kMultiCfgLds = 24576;
constexpr uint32_t kDupBucketCap = 1024;   // fingerprints per bucket (more: the exact path decides)
void launch_trace_dup_check(const TraceKernelArgs& a, hipStream_t st);
void launch_trace_long(const TraceKernelArgs& a, hipStream_t st, uint32_t known_runs = 0);
void launch_trace_insert_exact(const TraceKernelArgs& a, hipStream_t st);   // slow path, gated on *dup
void launch_trace_runs(const TraceKernelArgs& a, hipStream_t st);           // run-list path (gated on *dup)
void launch_trace_fold(const TraceKernelArgs& a, hipStream_t st);
void launch_trace_first_select(const TraceKernelArgs& a, hipStream_t st);   // win_first -> win_heads unless *overflow

// Slow path (runs only when *dup != 0; every launch checks the flag first).
struct TraceSortArgs {
  uint64_t n_spans;
  uint32_t n_tiles;           // ceil(n / kSortTile)
  uint32_t shift;             // digit shift of this pass
  const uint32_t* gate;       // == TraceKernelArgs::dup
  const uint64_t* tid;
  const TraceSlot* table;
  uint64_t table_mask;
  uint32_t epoch;
  const uint32_t* keys_in;    // null on the first pass: keys_in = key, vals = identity
  const uint32_t* vals_in;
  uint32_t* keys_out;
  uint32_t* vals_out;
  uint32_t* hist;             // [256 * n_tiles] digit-major
  uint32_t* key;              // canonical key per span (trace_key kernel output)
  uint32_t* error;
  unsigned long long* path_count;   // [1] += 1 per call the sort path decided (gate open)
  // sort_hist_kernel zeroes the following scan's tile counter and look-back
  // status (only when the gate is open: no memset launches per closed call)
  uint32_t* scan_counter;
  uint64_t* scan_status;
  uint32_t scan_status_n;
};
constexpr uint32_t kSortTile = 4096;
void launch_trace_key(const TraceSortArgs& a, hipStream_t st);
void launch_sort_hist(const TraceSortArgs& a, hipStream_t st);
void launch_sort_scatter(const TraceSortArgs& a, hipStream_t st);

// Exclusive scan of u32 counts (or popcounts of u64 bitmaps) with the
// decoupled look-back; *total receives the sum.  gate may be null.
struct ScanArgs {
  uint64_t n;
  uint32_t n_tiles;           // ceil(n / kScanTileItems)
  uint32_t popcount;          // 1: input is u64 bitmaps
  const uint32_t* gate;
  const void* in;
  uint32_t* out;
  uint32_t* total;            // may be null
  uint32_t* counter;          // zeroed before launch
  uint64_t* status;           // [n_tiles], zeroed before launch
  uint32_t* error;
};
constexpr uint32_t kScanTileItems = 1024;
void launch_scan_u32(const ScanArgs& a, hipStream_t st);

// Dense per-trace outputs from the records (first-appearance order).
struct TraceCompactArgs {
  uint32_t n_windows;
  const uint64_t* win_heads;
  const uint32_t* win_base;
  const TraceRec* rec;
  uint32_t* trace_first_span;
  uint8_t* trace_keep;
  uint8_t* trace_level;
  double* trace_ratio;
};
void launch_trace_compact(const TraceCompactArgs& a, hipStream_t st);

// Trace-id exchange (ose_shard_*; trace_kernel.hip).
struct ShardArgs {
  uint64_t n_spans;
  uint32_t n_tiles;           // wave chunks: ceil(n / kXChunk)
  uint32_t n_ranks;           // <= 64
  const uint64_t* tid;
  const uint64_t* start;
  const uint64_t* end;
  const uint8_t* status;
  const uint32_t* resource;
  const ose_strref* route;
  const uint8_t* arena;
  const uint64_t* route_match;
  uint64_t rm_stride;         // route_match: plane k (rule chunk k) at k * rm_stride (0: one plane)
  const uint64_t* attr_match;
  uint64_t attr_stride;       // attr_match: word w of span i at [w * attr_stride + i]
  uint32_t attr_words;
  const uint32_t* res_svc;
  const uint32_t* res_svc_str;
  const uint8_t* const* cfgs;  // [n_chunks] SampCfgDev blobs (device array of the rule chunks' tables)
  uint32_t n_chunks;
  const uint32_t* lat_svc;    // bit s: service s has an http_latency rule in some chunk
  uint32_t n_global_svc;      // services the engine interned (res_svc / res_svc_str / lat_svc index them)
  const uint32_t* const* svc_maps;   // [n_chunks] global -> chunk-local service id (0xFFFFFFFF: not in the
                                     // chunk), or null when every chunk indexes global ids (dense tables)
  uint32_t cfg_lds_bytes;     // the chunk tables copied into LDS by shard_scatter_kernel (sum of their 16-aligned
                              // sizes), 0: read from HBM
  uint32_t* hist;             // [n_ranks * n_tiles] counts, then offsets (second buffer)
  uint32_t* hoff;
  uint64_t* counts;           // [n_ranks] records per owner (shard_counts_kernel)
  uint8_t* send;              // [records * x_rec_bytes(n_chunks)], records <= n
  uint32_t* pack_pos;         // [n] slot of each span's record
};
// Partial record (trace_kernel.hip "trace-id exchange"): u64 words hi, lo,
// min start, max end, {latency service 24 | flags 8}, then per rule chunk
// the endpoint bits and the rule bits of that chunk's tables.
constexpr uint32_t kXSteps = 16;                        // 64-span steps of one packing wave's chunk
constexpr uint32_t kXChunk = kXSteps * 64;              // spans per packing wave
constexpr uint32_t kXFixedWords = 5;
constexpr uint32_t kXRecBytes = 8 * (kXFixedWords + 2);   // a one-chunk config (OSE_XREC_BYTES)
constexpr uint32_t x_rec_words(uint32_t n_chunks) { return kXFixedWords + 2 * n_chunks; }
constexpr uint32_t x_rec_bytes(uint32_t n_chunks) { return 8 * x_rec_words(n_chunks); }
void launch_shard_hist(const ShardArgs& a, hipStream_t st);
void launch_shard_counts(const ShardArgs& a, hipStream_t st);
void launch_shard_scatter(const ShardArgs& a, hipStream_t st);
struct UnpackArgs {
  const uint8_t* recv;
  uint64_t n;
  uint32_t n_chunks;          // route_match / svc_match: n_chunks planes of n words
  uint64_t* tid;
  uint64_t* start;
  uint64_t* end;
  uint8_t* status;
  uint32_t* resource;
  uint32_t* res_svc;
  uint32_t* res_svc_str;
  uint64_t* route_match;
  uint64_t* svc_match;
};
void launch_shard_unpack(const UnpackArgs& a, hipStream_t st);
// Owner-side decisions straight from the received records (ose_shard_decide;
// trace_kernel.hip "owner side"): records bucketed by trace-id hash, one
// workgroup per bucket groups, orders and folds its traces in LDS.
constexpr uint32_t kOwnerCap = 256;   // records one bucket holds (a fuller bucket: the general path)
constexpr uint32_t kOwnerAvg = 80;    // records per bucket the host sizes the bucket count for
constexpr uint32_t kOwnerSlotWords = 8;   // a bucket slot: hi, lo, min start, max end, {w4 | index << 32}, chunk 0's words, 0
struct OwnerArgs {
  const uint8_t* recv;        // n records of x_rec_words(n_chunks) words, in (source rank, source order)
  uint64_t n;
  uint32_t words;
  uint32_t n_buckets;
  uint32_t* bkt_count;        // [n_buckets], zeroed before the bucket pass
  uint64_t* bkt_rec;          // [n_buckets * kOwnerCap * kOwnerSlotWords] the records' slots
  const uint8_t* const* cfgs; // [n_chunks] SampCfgDev blobs
  uint32_t n_chunks;
  const uint32_t* const* svc_maps;   // as ShardArgs::svc_maps (records carry global service ids)
  uint32_t n_global_svc;
  uint32_t cfg_lds_bytes;     // dynamic LDS: the largest chunk table without its route bytes (16-aligned)
  uint64_t seed;
  uint8_t* keep;              // [n] per record
  uint32_t* overflow;         // set: a bucket past kOwnerCap records
  uint64_t* clocks;           // OSE_DIAG builds: per-phase clocks of owner_fold_kernel (OSE_OWNER_CLOCKS), else null
};
void launch_owner_bucket(const OwnerArgs& a, hipStream_t st);
void launch_owner_fold(const OwnerArgs& a, hipStream_t st);
void launch_scatter_keep(const uint8_t* back, const uint32_t* pos, uint64_t n, uint8_t* keep, hipStream_t st);
// endpoint bits of every span under one rule chunk's tables in HBM (a chunk
// whose route bytes spill past the LDS copy): out[j] for span j
// out[r] = map[in[r]] (0xFFFFFFFF for ids >= n_global), for res_svc and res_svc_str
void launch_svc_translate(const uint32_t* map, uint32_t n_global, const uint32_t* in1, const uint32_t* in2, uint32_t* out1,
                          uint32_t* out2, uint64_t n, hipStream_t st);
void launch_endpoint_plane(const uint8_t* cfg, const uint32_t* resource, const uint32_t* res_svc, const ose_strref* route,
                           const uint8_t* arena, uint64_t n, uint64_t* out, hipStream_t st);
// the in-process transport's pieces of one phase, moved by one launch
struct PeerCopies {
  const uint8_t* src[64];
  uint8_t* dst[64];
  uint64_t len[64];
  uint32_t n;
};
void launch_peer_copies(const PeerCopies& c, uint64_t max_len, hipStream_t st);
// dst[k] += src[k] (the in-process transport's counter all-reduce)
void launch_add_i64(int64_t* dst, const int64_t* src, uint64_t n, hipStream_t st);
uint32_t shard_owner_host(uint64_t hi, uint64_t lo, uint32_t n_ranks);

// Workspace words shared between stages of one call (uint32 index into the
// first 256 bytes of the workspace; URL uses words 0-3, SAMPLE 0-15).
constexpr uint32_t kBatchKeepWord = 16;   // OSE_GROUP_BATCH decision of the SAMPLE stage

// odigostrafficmetrics (size_kernel.hip): three passes, spans -> scopes ->
// resources, each a wave-segmented reduction (the columns are in pdata
// order, so scope and resource indices are non-decreasing).
void launch_size_spans(const SizeKernelArgs& a, hipStream_t st);
// scopes and resources in one pass (size_tail_kernel: every resource whose
// scopes lie in one 64-scope window is finished there), then the resources
// whose scopes span windows (size_fix_kernel)
void launch_size_tail(const SizeKernelArgs& a, hipStream_t st);
void launch_size_fix(const SizeKernelArgs& a, hipStream_t st);

// span_attribute conditions (attr_kernel.hip): out[i] = host_bits[i] &
// host_mask | the bits of the GPU-evaluated rules the span meets.
struct AttrArgs {
  uint64_t n_spans;
  const uint8_t* type;         // [n_keys * n_spans] OSE_ATTR_*
  const uint64_t* val;         // [n_keys * n_spans]
  const uint8_t* arena;
  const uint32_t* resource;
  const uint32_t* res_svc;
  uint32_t words;              // attr_match words per span (word-major planes of n_spans)
  const uint64_t* host_bits;   // may be null
  const uint64_t* host_mask;   // [words] the shim-evaluated rules
  const uint8_t* cfg;          // AttrCfgDev blob
  uint64_t* out;
};
void launch_attr_eval(const AttrArgs& a, hipStream_t st);

// OTLP protobuf ingest (otlp_kernel.hip).  Attribute keys the decoder
// looks for, with the roles a key plays (one entry per distinct key).
enum : uint32_t {
  kRoleMethodNew = 1u << 0,   // http.request.method
  kRoleMethodOld = 1u << 1,   // http.method
  kRoleRoute = 1u << 2,       // http.route (sampling route; SERVER target)
  kRoleUrlTmpl = 1u << 3,     // url.template (CLIENT target)
  kRoleUrlPath = 1u << 4,     // url.path
  kRoleTarget = 1u << 5,      // http.target
  kRoleFull = 1u << 6,        // url.full / http.url: net/url.Parse on the host
  kRoleHost = 1u << 7,        // a json span_attribute rule's key: host pass
};
constexpr uint64_t kRoleAttr0 = 1ull << 8;   // << k: GPU attribute key column k (k < kOtlpMaxAttrKeys)
constexpr uint32_t kOtlpMaxAttrKeys = 56;
struct OtlpKeyDev {
  uint32_t len, off;
  uint64_t roles;
};
struct OtlpArgs {
  const uint8_t* pb;            // message bytes = the arena (16-byte aligned, 16 bytes of slack)
  uint64_t n_spans;
  const uint64_t* span_ref;     // payload offset | length << 32
  const OtlpKeyDev* keys;
  const uint8_t* key_bytes;
  uint32_t n_keys;
  uint32_t n_attr_keys;
  uint64_t key_lens;            // bit l: some key has length l (< 64)
  uint64_t* tid;
  uint64_t* start;
  uint64_t* end;
  uint8_t* status;
  uint8_t* kind;
  uint8_t* url_flags;
  ose_strref* path;
  ose_strref* route;
  uint32_t* span_size;
  uint32_t* name_len;
  uint64_t* attr_match;         // may be null; attr_words word-major planes of n_spans
  uint32_t attr_words;
  uint8_t* attr_type;
  uint64_t* attr_val;
  uint8_t* host_flag;           // [n_spans] 1 = the host pass writes this span
  uint32_t* host_count;         // zeroed before launch
  uint32_t* host_list;
  uint32_t host_cap;
};
// ScopeSpans walked on the GPU (the host walks TracesData and ResourceSpans
// only): pass 1 counts each scope's spans and reads its InstrumentationScope
// and schema_url; pass 2 (after a scan of the counts) writes the span refs.
constexpr uint64_t kOtlpScopeMulti = ~0ull;
struct OtlpScopeArgs {
  const uint8_t* pb;
  uint64_t n_scopes;
  const uint64_t* scope_ref;    // ScopeSpans payload off | len << 32
  const uint8_t* on_host;       // 1: the host walked this scope (counts / sizes / layout preset)
  const uint32_t* scope_res;
  uint32_t* count;              // spans per scope
  uint32_t* scope_size;         // pdata's fixed ScopeSpans size (scope + schema_url)
  uint64_t* hdr;                // the InstrumentationScope message ref, 0 none, kOtlpScopeMulti several
  uint64_t* schema;             // schema_url ref (last occurrence; length 0: none)
  uint32_t* flags;              // 1: size left to the host (merged / unusual scope message), 2: malformed
  const uint32_t* span0;        // pass 2: exclusive scan of count
  uint64_t* span_ref;
  uint32_t* span_res;
  uint32_t* span_scope;
  // pass 2 for the host-walked scopes: their refs, listed in scope order
  const uint64_t* host_refs;
  const uint64_t* host_at;      // [n_scopes] offset into host_refs (host-walked scopes)
};
// ResourceSpans on the GPU (the host walks only the TracesData chain of
// ResourceSpans records): each record's fields, its Resource's columns from
// the engine's device table of resources seen before (keyed by the Resource
// message bytes: FNV-1a 64), its ScopeSpans listed for the scope passes.
struct ResSlotDev {          // 48 B; ready != 0: filled
  uint64_t h;
  uint32_t koff, klen;       // key bytes in the table's key arena
  uint32_t svc, svc_str, set, rpart;
  uint64_t attr_res;
  uint32_t ok, ready;
};
constexpr uint32_t kResSlots = 1u << 17;
constexpr uint32_t kResKeyBytes = 16u << 20;
// FNV-1a over the bytes (the host fills the table with the same function)
inline __host__ __device__ uint64_t res_key_hash_step(uint64_t h, uint32_t b) { return (h ^ b) * 0x100000001B3ull; }
constexpr uint64_t kResHashSeed = 0xCBF29CE484222325ull;
struct OtlpResArgs {
  const uint8_t* pb;
  uint64_t n_res;
  const uint64_t* res_ref;     // ResourceSpans payload off | len << 32
  uint32_t* flags;             // 1: resource columns from the host, 2: malformed, 4: scopes are field 1000
  uint32_t* nscope;            // ScopeSpans per resource (field 2, or field 1000 when there is no field 2)
  uint32_t* schema_len;        // ResourceSpans.schema_url length (last occurrence)
  uint32_t* any_bad;           // [1] OR of flags & 2
  const uint32_t* scope0;      // pass 2: exclusive scan of nscope
  uint64_t* scope_ref;
  uint32_t* scope_res;
  // the Resource's columns
  const ResSlotDev* table;
  const uint8_t* keys;
  uint32_t* res_svc;
  uint32_t* res_svc_str;
  uint32_t* res_set;           // the resource cache's attribute-set id (batch ids after compaction)
  uint32_t* res_size;
  uint8_t* res_ok;
  uint64_t* attr_res;
  uint32_t* miss_count;        // [1]
  uint32_t* miss_list;         // [n_res]
};
// The TracesData chain on the GPU: the message split into segments of
// kChainSeg bytes; lane t speculates a record start in its segment (as the
// host walk's find_start does) and walks the top-level fields from it until
// the first field boundary at or past the next segment.  The host links the
// segments (a speculated start inside a record converges to the true chain at
// that record's end, one of the field starts listed) and otlp_chain_list
// writes the records of each linked segment from its first true field on.
constexpr uint32_t kChainSeg = 64u << 10;
constexpr uint32_t kChainList = 16;   // field starts listed per segment
constexpr uint64_t kChainNone = ~0ull;
struct OtlpChainArgs {
  const uint8_t* pb;
  uint64_t n;
  uint32_t n_seg;
  uint64_t* start;      // [n_seg] speculated start (kChainNone: none in the segment)
  uint64_t* end;        // [n_seg] where the walk stopped (first boundary >= next segment)
  uint32_t* nrec;       // [n_seg] records (field 1) walked
  uint32_t* bad;        // [n_seg] the walk met a malformed field (end = where)
  uint64_t* list;       // [n_seg * kChainList] field starts | (field 1) << 63
  // pass 2 (linked segments): walk from first[t] (kChainNone: skip), records to res_ref from base[t]
  const uint64_t* first;
  const uint32_t* base;
  uint64_t* res_ref;
};
void launch_otlp_chain_seg(const OtlpChainArgs& a, hipStream_t st);
void launch_otlp_chain_list(const OtlpChainArgs& a, hipStream_t st);
void launch_otlp_res_fields(const OtlpResArgs& a, hipStream_t st);
void launch_otlp_res_scopes(const OtlpResArgs& a, hipStream_t st);
// the host's columns of the missed resources: fix k = {row, svc, svc_str, set, rpart, ok, attr_res}
struct OtlpResFix {
  uint32_t row, svc, svc_str, set, rpart, ok;
  uint64_t attr_res;
};
void launch_otlp_res_fix(const OtlpResArgs& a, const OtlpResFix* fix, uint32_t n, hipStream_t st);
// attribute-set ids of the cache -> the batch's, in order of first appearance
// (as the host walk numbers them): each set's first resource (first[], set
// to ~0 before), the resources that are first of their set (is_first), and
// after an exclusive scan of those flags (pos) the ids and the batch's list
void launch_otlp_set_first(const uint32_t* res_set, uint64_t n_res, uint32_t* first, uint32_t* is_first,
                           hipStream_t st);
void launch_otlp_set_apply(uint32_t* res_set, uint64_t n_res, const uint32_t* first, const uint32_t* is_first,
                           const uint32_t* pos, uint32_t* list, hipStream_t st);
void launch_otlp_scope_count(const OtlpScopeArgs& a, hipStream_t st);
void launch_otlp_scope_spans(const OtlpScopeArgs& a, hipStream_t st);

// OTLP re-encode on the GPU (encode_kernel.hip): the
// sizing and writing passes of otlp_encode.cpp over the message bytes and
// the decisions, both already in HBM.  Resources are routed on the device
// (odigosrouterconnector's key from the Resource's attributes, looked up in
// an FNV-1a table of the router's keys).  What the device path does not
// write exactly as the host encoder would — a span, scope or resource whose
// encoding is not already pdata's, a method needing AsString, fields out of
// order, a merged Resource — sets a flag, and the call goes to the host
// encoder instead.
constexpr uint64_t kEncDropped = ~0ull;
constexpr uint64_t kEncNoHdr = ~0ull;            // res_hdr / scope header: absent ("0A 00")
constexpr uint32_t kEncTiles = 1024;             // resources per scan tile
enum : uint32_t {
  kEncFbSpan = 1,       // a rewritten span pdata would re-marshal, or an AsString method
  kEncFbScope = 2,      // a scope header not in pdata's encoding / merged
  kEncFbRes = 4,        // a resource header not in pdata's encoding / merged / malformed
  kEncFbTmpl = 8,       // a template reference beyond the arena (the host reports it)
  kEncFbRoute = 16,     // a routing attribute the device does not read exactly
  kEncFbWrite = 32,     // the writing pass disagreed with the sizing pass (a bug: the call fails)
};
struct EncEdit {        // one rewritten span (otlp_encode.cpp Edit)
  uint32_t name_a, name_b, attr_a, attr_b;
  uint32_t meth_off, meth_len;   // the method string in the message
  uint32_t tmpl_off, tmpl_len;   // the template in the template arena
  uint32_t out_len;              // edited span bytes
  uint32_t flags;                // url_out | client << 8
};
struct EncRouteSlot {   // router key "ns/kind/name" -> pipelines; klen == ~0: empty
  uint64_t h;
  uint32_t koff, klen;
  uint64_t mask;
};
struct EncArgs {
  const uint8_t* pb;
  uint64_t n_spans, n_scopes, n_res;
  const uint64_t* span_ref;
  const uint32_t* span_size;
  const uint8_t* keep;           // NULL: every span kept
  const uint8_t* url_out;        // NULL: no template stage
  const ose_strref* tmpl;
  const uint8_t* tmpl_arena;
  const uint64_t* tmpl_used;
  const uint32_t* scope_span0;
  const uint64_t* scope_hdr;     // InstrumentationScope ref (0: none, kOtlpScopeMulti: merged)
  const uint64_t* scope_schema;
  const uint32_t* scope_size;    // the decoder's pdata size of the scope's fixed part
  const uint64_t* res_ref;
  const uint32_t* res_scope0;
  const uint32_t* res_size;      // the decoder's pdata size of the resource's fixed part
  uint32_t n_out;                // router pipelines + 1 (default), or 1
  uint32_t route_bits;           // log2 of the route table's slots (0: no router)
  const EncRouteSlot* routes;
  const uint8_t* route_keys;
  // sizing pass
  uint32_t* span_out;            // framed bytes of span i in its scope (0: dropped)
  EncEdit* edit;
  uint64_t* scope_body;          // kEncDropped: removed
  uint64_t* res_body;
  uint64_t* res_rec;             // framed record bytes (0: dropped)
  uint64_t* res_mask;            // outputs the resource goes to
  uint64_t* res_hdr;             // Resource payload ref, kEncNoHdr: absent
  uint64_t* res_schema;          // ResourceSpans.schema_url ref (length 0: none)
  uint32_t* flags;               // [1] OR of kEncFb*
  // scans: offsets per output, then the writing pass
  uint64_t* tile_sum;            // [n_out][tiles] bytes, then [n_out][tiles] counts
  uint64_t* off;                 // [n_out][n_res]
  uint64_t* out_total;           // [n_out] bytes, then [n_out] resource counts
  const uint64_t* out_base;      // [n_out]
  uint8_t* out;
};
void launch_enc_spans(const EncArgs& a, hipStream_t st);
void launch_enc_scopes(const EncArgs& a, hipStream_t st);
void launch_enc_resources(const EncArgs& a, hipStream_t st);
void launch_enc_scan(const EncArgs& a, hipStream_t st);
void launch_enc_write(const EncArgs& a, hipStream_t st);

struct OtlpFix {
  uint64_t idx;
  uint64_t hi, lo, start, end;
  ose_strref path, route;
  uint32_t span_size, name_len;
  uint8_t status, kind, url_flags, _pad[5];
};
struct OtlpFixArgs {
  uint32_t n;
  uint32_t n_attr_keys;
  uint64_t n_spans;
  const OtlpFix* fix;
  uint32_t attr_words;          // attr_match words per span (fix_attr: [n * attr_words])
  const uint64_t* fix_attr;
  const uint8_t* fix_type;      // [n * n_attr_keys]
  const uint64_t* fix_val;
  uint64_t* tid;
  uint64_t* start;
  uint64_t* end;
  uint8_t* status;
  uint8_t* kind;
  uint8_t* url_flags;
  ose_strref* path;
  ose_strref* route;
  uint32_t* span_size;
  uint32_t* name_len;
  uint64_t* attr_match;
  uint8_t* attr_type;
  uint64_t* attr_val;
};
void launch_otlp_spans(const OtlpArgs& a, hipStream_t st);
void launch_otlp_fix(const OtlpFixArgs& a, hipStream_t st);

// ---- groupbytrace store (gbt_kernel.hip) --------------------------------------
struct GbtSlot {              // trace id -> creation number (32 B, generation-tagged)
  uint32_t state;             // epoch << 2 | {0 empty, 1 busy, 2 ready}
  uint32_t first;             // smallest batch position carrying the id (new ids)
  uint64_t hi, lo;
  uint64_t seq;               // creation number of the id's newest trace; kGbtUnset | add
                              // while add number `add` is numbering a new trace for it
};
constexpr uint64_t kGbtUnset = 0xFFFFFFFF00000000ull;
struct GbtPool {              // spans waiting for release (ring of pool_cap)
  uint64_t* tid;              // {hi, lo}
  uint64_t *start, *end, *attr_match, *seq, *origin, *str_off;
  uint8_t *status, *kind, *url_flags;
  uint32_t *span_size, *name_len;
  ose_strref *route, *path;   // relative to the span's string block
  uint8_t* attr_type;         // key-major, [key * pool_cap + p]
  uint64_t* attr_val;
};
struct GbtScopes {            // the fragment columns of each added scope (ring)
  uint32_t *res_svc, *res_svc_str, *res_attrset, *res_size, *scope_size;
  uint8_t* res_url_ok;
};
struct GbtOut {               // the released batch
  uint64_t* tid;
  uint64_t *start, *end, *attr_match;
  uint8_t *status, *kind, *url_flags;
  uint32_t *span_size, *name_len, *resource, *scope;
  ose_strref *route, *path;
  uint8_t* attr_type;
  uint64_t* attr_val;
  uint32_t *res_svc, *res_svc_str, *res_attrset, *res_size, *scope_size, *scope_resource;
  uint8_t* res_url_ok;
  uint8_t* arena;
};
struct GbtArgs {
  GbtSlot* table;
  uint64_t table_mask;
  uint32_t epoch;
  uint32_t n_attr_keys;
  uint32_t* error;
  uint64_t* ring_tid;         // [2 * ring_n]: the id of trace seq at seq % ring_n
  uint64_t num_traces;
  uint64_t ring_n;            // num_traces (one worker), else the pool capacity
  // num_workers > 1 (contrib's event machine): trace seq belongs to worker
  // fnv64(id) % n_workers, numbered q within it; tinfo[seq % ring_n] =
  // worker << 40 | q.  It is evicted once its worker has numbered more
  // than q + worker_cap traces (wcnt: the workers' counts the call sees)
  uint32_t n_workers;
  uint64_t worker_cap;
  uint64_t* tinfo;
  const uint64_t* wcnt;
  uint32_t *wadd, *wstart;    // numbering: creators per worker in the batch, their exclusive scan
  uint64_t live_lo, live_hi;  // traces an added span may join (and the rebuild range)
  uint32_t add_gen;           // number of this add (tags the ids it numbers)
  uint32_t attr_words;        // attr_match words per span (word-major: batch, pool and released planes)
  uint64_t arena_room;        // string bytes the arena ring can still take
  const uint32_t* totals;     // [0] new traces, [1] string bytes of the batch (scans)
  // add: the batch
  ose_columns cols;
  uint64_t n, n_scopes;
  uint64_t next_seq;
  uint64_t* slot_of;
  uint32_t *flag, *rank, *strlen, *stroff;
  const uint32_t* attrset_map;
  // the rings
  GbtPool pool;
  uint64_t pool_pos, pool_cap;
  GbtScopes scopes;
  uint64_t scope_pos, scope_cap;
  uint8_t* arena_ring;
  uint64_t arena_pos, arena_cap;
  // release
  uint64_t rel_lo, rel_hi;
  uint32_t *keys, *vals;
  const uint32_t* order;
  GbtOut out;
};
void launch_gbt_rebuild(const GbtArgs& a, hipStream_t st);
void launch_gbt_lookup(const GbtArgs& a, hipStream_t st);
void launch_gbt_creator(const GbtArgs& a, hipStream_t st);
void launch_gbt_assign(const GbtArgs& a, hipStream_t st);
void launch_gbt_append(const GbtArgs& a, hipStream_t st);
void launch_gbt_strings(const GbtArgs& a, hipStream_t st);
void launch_gbt_scopes(const GbtArgs& a, hipStream_t st);
void launch_gbt_flag(const GbtArgs& a, hipStream_t st);
void launch_gbt_compact(const GbtArgs& a, hipStream_t st);
void launch_gbt_gather(const GbtArgs& a, hipStream_t st);
void launch_gbt_emit(const GbtArgs& a, hipStream_t st);
void launch_gbt_wkey(const GbtArgs& a, hipStream_t st);                 // creators -> (worker, rank) pairs
void launch_gbt_wnum(const GbtArgs& a, uint64_t created, hipStream_t st);   // sorted pairs -> tinfo

}  // namespace ose
