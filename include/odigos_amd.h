/*
 * odigos_amd.h — C ABI of the MI355X span-processing engine.
 *
 * This is the drop-in boundary for the three gateway trace processors of the
 * Odigos collector (reference: damemi/odigos @ 2026-02-13):
 *
 *   odigossampling       collector/processors/odigossamplingprocessor
 *   odigosurltemplate    collector/processors/odigosurltemplateprocessor
 *   odigostrafficmetrics collector/processors/odigostrafficmetrics
 *
 * In the reference each processor is a Go processor.Factory whose
 * processorhelper.ProcessTracesFunc walks a ptrace.Traces
 * (odigossamplingprocessor/processor.go:16-21, odigosurltemplateprocessor/
 * processor.go:71-96, odigostrafficmetrics/processor.go:71-84).  A cgo shim
 * that keeps the Go Factory / Config / mapstructure tags columnarises each
 * batch into the struct-of-arrays described by ose_columns, calls
 * ose_process*, and applies the results (RemoveIf, PutStr, SetName, counter
 * Add).  See INTEGRATION.md for the shim.
 *
 * Conventions: every entry point returns 0 on success or a negative
 * errno-style code (OSE_E*); nothing throws across the ABI; the message of the
 * last failure on the calling thread is returned by ose_last_error().  All
 * entry points are re-entrant; one engine may be used from many threads
 * (each call takes its own HIP stream and workspace from a pool).
 */
#ifndef ODIGOS_AMD_H
#define ODIGOS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OSE_ABI_VERSION 4

/* ---- error codes ---------------------------------------------------- */
#define OSE_OK        0
#define OSE_EINVAL  (-22) /* bad argument / invalid config (Validate error) */
#define OSE_ENOMEM  (-12) /* host or device allocation failed               */
#define OSE_ENOTSUP (-95) /* config uses a feature the engine cannot run     */
#define OSE_EDEVICE (-5)  /* HIP runtime error, or no MI355X visible         */
#define OSE_ERANGE  (-34) /* batch exceeds a 32-bit arena/offset limit       */
#define OSE_ETIMEDOUT (-110) /* an in-kernel bounded spin gave up            */

#define OSE_NONE 0xFFFFFFFFu   /* "no value" for interned-id columns */

/* ---- OTLP enums (ptrace.SpanKind / ptrace.StatusCode values) -------- */
#define OSE_KIND_UNSPECIFIED 0
#define OSE_KIND_INTERNAL    1
#define OSE_KIND_SERVER      2
#define OSE_KIND_CLIENT      3
#define OSE_KIND_PRODUCER    4
#define OSE_KIND_CONSUMER    5
#define OSE_STATUS_UNSET 0
#define OSE_STATUS_OK    1
#define OSE_STATUS_ERROR 2

/* ---- per-span url_flags (columnarised by the shim) ------------------
 * Mirrors what odigosurltemplateprocessor/processor.go reads from the span
 * attribute map:
 *   HAS_METHOD      getHttpMethod found http.request.method or http.method
 *                   (processor.go:98-111)
 *   TGT_*           state of the target attribute (http.route for SERVER,
 *                   url.template for CLIENT) as read by enhanceSpan
 *                   (processor.go:235-252)
 *   NAME_EQ_METHOD  span.Name() == AsString(method) (updateHttpSpanName,
 *                   processor.go:214-233)
 *   PATH_*          which source calculateTemplatedUrlFromAttr uses
 *                   (processor.go:113-147, 188-212): RAW = url.path, or the
 *                   Path of url.full/http.url after net/url.Parse on the host;
 *                   TARGET = http.target, the engine cuts at the first '?';
 *                   NONE = no source, or url.Parse failed.                     */
#define OSE_URL_HAS_METHOD      0x01u
#define OSE_URL_TGT_MASK        0x06u
#define OSE_URL_TGT_ABSENT      0x00u
#define OSE_URL_TGT_STR_EMPTY   0x02u
#define OSE_URL_TGT_STR         0x04u
#define OSE_URL_TGT_NONSTR      0x06u
#define OSE_URL_NAME_EQ_METHOD  0x08u
#define OSE_URL_PATH_MASK       0x30u
#define OSE_URL_PATH_NONE       0x00u
#define OSE_URL_PATH_RAW        0x10u
#define OSE_URL_PATH_TARGET     0x20u

/* ---- per-span url_out (results) ------------------------------------ */
#define OSE_OUT_SET_ATTR 0x01u  /* attr.PutStr(target, tmpl)             */
#define OSE_OUT_RENAME   0x02u  /* span.SetName(method + " " + tmpl)     */

/* ---- stage mask ------------------------------------------------------ */
#define OSE_STAGE_SAMPLE   0x1u  /* odigossampling       */
#define OSE_STAGE_TEMPLATE 0x2u  /* odigosurltemplate    */
#define OSE_STAGE_SIZE     0x4u  /* odigostrafficmetrics */
/* keep already holds the sampling decisions (made by an earlier call, e.g.
 * on the trace's owner GPU after the trace-id exchange): SIZE honours them
 * as if SAMPLE had run in this call with group_mode OSE_GROUP_TRACE_ID.    */
#define OSE_STAGE_APPLY_KEEP 0x8u
/* With OSE_STAGE_TEMPLATE, ose_process_device only: the templates stay where
 * the GPU assembled them (64-span groups, in the order the GPU finished
 * them) instead of being packed in span order.  tmpl[i] still refers into
 * tmpl_arena and its bytes are exactly the packed form's, but the arena has
 * gaps: up to 15 bytes after each group, per assembling wave the unused
 * tail of its last space chunk (at most tmpl_arena_cap / 8 in all), and
 * chunk tails a wave left for a group image that did not fit (at most 1/7 of
 * the bytes used); *tmpl_arena_used is the end of the highest range
 * written.  It saves a read and a write of every template byte when the
 * consumer follows the refs on the device instead of copying the arena to
 * the host.  Overflow: device_status bit 2 and *tmpl_arena_used = an arena
 * size for the retry (twice the templates as 16-byte aligned group images,
 * plus one image per assembling wave, ~4.6 KiB: room for the chunk tails the
 * retry's waves leave), as the packed form reports the bytes it needs.      */
#define OSE_STAGE_TEMPLATE_REFS 0x10u
/* url_out and tmpl already hold the templating results (written by an
 * earlier call on the same batch, e.g. TEMPLATE on a second stream while the
 * trace-id exchange runs): SIZE counts the attribute each span gains and the
 * renamed span names as if TEMPLATE had run in this call (the traffic
 * processor runs after the URL processor, config_builder.go:215-229).       */
#define OSE_STAGE_APPLY_TEMPLATE 0x20u

/* ---- grouping of spans into "traces" for odigossampling --------------
 * TRACE_ID: spans sharing a 128-bit trace_id form one trace (the contract
 *   groupbytrace establishes upstream, sampling_controller.go:193-220).
 * BATCH: the whole batch is one trace, exactly as RuleEngine.ShouldSample
 *   treats one ConsumeTraces call (rule_engine.go:55-83).                   */
#define OSE_GROUP_TRACE_ID 0u
#define OSE_GROUP_BATCH    1u

/* ---- injected randomness ---------------------------------------------
 * The reference draws rand.Float64() from Go's auto-seeded global source
 * (rule_engine.go:68,79; odigostrafficmetrics/processor.go:72), which is not
 * reproducible.  The engine instead uses, per trace,
 *   u = (splitmix64(tid_hi ^ rotl64(tid_lo, 29) ^ seed) >> 11) * 2^-53
 * and keeps the trace iff u*100 < ratio; the traffic gate uses traffic_u
 * (one draw per batch = per ConsumeTraces call).                          */
typedef struct ose_rand {
  uint64_t seed;
  double traffic_u;   /* in [0,1); the traffic stage runs iff traffic_u < sampling_ratio */
} ose_rand;

typedef struct ose_strref {
  uint32_t off;   /* byte offset into the arena */
  uint32_t len;   /* byte length                */
} ose_strref;

/* ---- columnar batch ----------------------------------------------------
 * Spans are in pdata traversal order (ResourceSpans -> ScopeSpans -> Span),
 * so `resource` and `scope` are non-decreasing.  A pointer may be NULL when
 * no requested stage reads it.  For ose_process_device every pointer is a
 * device pointer; for ose_process they point into an ose_batch.            */
typedef struct ose_columns {
  uint64_t n_spans;
  uint32_t n_resources;
  uint32_t n_scopes;
  uint32_t n_attrsets;      /* traffic-metrics attribute sets (res_attrset range) */
  uint32_t attr_match_words; /* 64-bit words of attr_match per span, word-major: word w of span i at
                                attr_match[w * n_spans + i] (bits 64w..64w+63); 0 or 1: one word.
                                ose_engine_info.n_attr_rules > 64 needs (n_attr_rules + 63) / 64 */
  uint64_t arena_bytes;     /* bytes of `arena`; also sizes the TEMPLATE stage's scratch for
                               the assembled templates (an understated value is not an error:
                               the groups that do not fit take the slower per-span writer) */
  const uint8_t* arena;     /* all string bytes referenced by ose_strref columns */

  /* per span */
  const uint64_t* trace_id;   /* [2*n]: {hi, lo}: bytes 0..7 and 8..15, big-endian */
  const uint64_t* start_ns;   /* StartTimestamp */
  const uint64_t* end_ns;     /* EndTimestamp */
  const uint8_t* status;      /* Status().Code() */
  const uint8_t* kind;        /* Kind() */
  const uint32_t* resource;   /* index of the span's ResourceSpans */
  const uint32_t* scope;      /* index of the span's ScopeSpans */
  const uint8_t* url_flags;   /* OSE_URL_* */
  const ose_strref* path;     /* url path bytes per url_flags PATH_* */
  const ose_strref* route;    /* AsString(http.route) before templating; len 0 if absent */
  const uint32_t* span_size;  /* wire size of the Span message before mutation */
  const uint32_t* name_len;   /* len(span.Name()) before mutation */
  const uint64_t* route_match; /* optional: bit r = strings.HasPrefix(AsString(http.route), http_route
                                  of the r-th http_latency rule) for the rules of the span's service
                                  (latency.go:64-68, 97-100); when non-NULL the engine reads it
                                  instead of route/arena (set by ose_shard_unpack)               */
  const uint64_t* attr_match;  /* bit k = the span meets the k-th span_attribute rule (in level order;
                                  beyond 64 rules, in word k / 64: attr_match_words):
                                  its resource's AsString(service.name) is the rule's service_name and
                                  its attribute satisfies the condition (spanattribute.go:126-320).
                                  With attr_type set, only the bits of the rules the engine leaves to
                                  the shim (ose_engine_info.attr_host_rules: "json" conditions) are
                                  read (NULL when there are none); without it every bit is read   */

  /* per resource */
  const uint32_t* res_svc;      /* ose_engine_service_id(AsString(service.name)) or OSE_NONE */
  const uint32_t* res_svc_str;  /* same, only if service.name is ValueTypeStr, else OSE_NONE */
  const uint8_t* res_url_ok;    /* include/exclude PropertiesMatcher verdict (filtermatcher.go);
                                   NULL = every resource passes (no include/exclude configured) */
  const uint32_t* res_attrset;  /* interned attributeSetFromResource (processor.go:60-69) */
  const uint32_t* res_size;     /* ResourceSpans bytes excluding its scope_spans fields */

  /* per scope */
  const uint32_t* scope_size;   /* ScopeSpans bytes excluding its spans fields */
  const uint32_t* scope_resource; /* index of the scope's ResourceSpans (non-decreasing) */

  /* per span, optional (set by ose_shard_unpack on the trace's owner GPU):
   * the OR of the service_name rule bits (servicename.go:35-51, by
   * res_svc_str) and span_attribute rule bits (attr_match, shifted past the
   * service rules) of the spans a partial record folds; when non-NULL the
   * engine reads it instead of res_svc_str / attr_match                   */
  const uint64_t* svc_match;

  /* per span x attribute key, optional: the span_attribute rules with
   * string / number / boolean conditions are evaluated on the GPU from the
   * span's value of the rule's attribute_key (spanattribute.go:136-230).
   * Key k is the k-th distinct attribute_key of those rules in level order
   * (ose_engine_attr_key).  Key-major: entry [k * n_spans + i] is
   * Attributes().Get(key k) of span i (the first entry with that key):
   *   attr_type  OSE_ATTR_* (OSE_ATTR_ABSENT when the key is not found)
   *   attr_val   STR: ose_strref {off, len} into the arena (as a u64, off in
   *              the low half); INT: the int64; DOUBLE: the float64 bits;
   *              BOOL: 0 / 1; other types: 0                               */
  uint32_t n_attr_keys;
  uint32_t match_planes;   /* route_match / svc_match hold this many planes of n_spans words,
                              plane k for rule chunk k (K = (ose_shard_record_bytes - 40) / 16; what
                              ose_shard_unpack writes); 0 or 1: one plane, accepted only by
                              an engine with one rule chunk (OSE_EINVAL otherwise: the bits
                              are chunk-local rule indices)                             */
  const uint8_t* attr_type;
  const uint64_t* attr_val;
} ose_columns;

/* pcommon.ValueType of an attribute value in attr_type */
#define OSE_ATTR_ABSENT 0u
#define OSE_ATTR_STR    1u
#define OSE_ATTR_INT    2u
#define OSE_ATTR_DOUBLE 3u
#define OSE_ATTR_BOOL   4u
#define OSE_ATTR_OTHER  5u   /* map, slice, bytes, empty */

/* ---- results -----------------------------------------------------------
 * Any pointer may be NULL when its stage is not requested.                 */
typedef struct ose_outputs {
  /* odigossampling */
  uint8_t* keep;              /* [n_spans] 1 if the span's trace is sampled */
  uint32_t* trace_count;      /* [1] number of traces found (optional) */
  uint32_t* trace_first_span; /* [n_spans cap] first span of each trace (optional) */
  uint8_t* trace_keep;        /* [n_spans cap] decision per trace (optional) */
  uint8_t* trace_level;       /* [n_spans cap] 0..2 satisfied level, 3 fallback, 4 none */
  double* trace_ratio;        /* [n_spans cap] ratio drawn against (100 when level 4) */

  /* odigosurltemplate */
  uint8_t* url_out;           /* [n_spans] OSE_OUT_* */
  ose_strref* tmpl;           /* [n_spans] template (valid where url_out != 0) */
  uint8_t* tmpl_arena;        /* output bytes */
  uint64_t tmpl_arena_cap;
  uint64_t* tmpl_arena_used;  /* [1] bytes written */

  /* odigostrafficmetrics (ADDED to, so counters accumulate across calls) */
  int64_t* attrset_bytes;     /* [n_attrsets] otelcol_odigos_trace_data_size */
  int64_t* accepted_spans;    /* [1] otelcol_odigos_accepted_spans */
  uint64_t* res_bytes;        /* [n_resources] ResourceSpansSize after mutation (optional) */

  /* device-side failure bits OR-ed in by the kernels (ose_process_device
   * only; the caller zeroes it and checks after synchronising):
   * 1 = in-kernel bounded spin gave up, 2 = tmpl_arena_cap too small */
  uint32_t* device_status;
} ose_outputs;

typedef struct ose_engine ose_engine;
typedef struct ose_batch ose_batch;

/* Replaces the three processor.Factory.CreateTraces paths
 * (odigossamplingprocessor/factory.go:29-45 -> config.go:17-80 Validate;
 *  odigosurltemplateprocessor/factory.go:31-44 -> processor.go:27-69;
 *  odigostrafficmetrics/factory.go:34-47 -> processor.go:31-58).
 * cfg_json: {"odigossampling": {...}, "odigosurltemplate": {...},
 *            "odigostrafficmetrics": {...}} with the mapstructure keys of the
 * Go Config structs; absent sections are absent processors.  Validates
 * exactly as the Go Validate() does (same messages) and compiles every user
 * regexp to a DFA; a regexp the DFA compiler cannot express is OSE_ENOTSUP
 * (there is no host fallback).  Any number of sampling rules: a rule list
 * beyond one GPU rule table (64 http_latency rules, 64 service_name
 * services + span_attribute rules, 12 KiB) runs as one trace-stage pass per
 * chunk of the list with the same decisions (an http_route longer than a
 * table: a chunk of its own, its bytes past the LDS copy read from HBM);
 * more than about 500 distinct service names among the rules: each chunk
 * indexes its own rules' services (ose_shard_pack / ose_shard_decide then
 * return OSE_ENOTSUP).  OSE_ENOTSUP remains for regexps whose DFA exceeds
 * about two million states (or 256 MiB of transitions).                     */
int ose_engine_create(const char* cfg_json, ose_engine** out);
/* The engine's batches (ose_batch, ose_otlp_batch, ose_otlp_out, ose_gbt)
 * may be released before or after this call: each holds a reference, and
 * the engine is freed (after a device synchronise) when the last one goes.
 * No other call may use `eng` after it.                                     */
void ose_engine_destroy(ose_engine* eng);

/* Device selection: an engine lives on the HIP device that is current on
 * the creating thread, and every later call on it runs there whatever
 * thread makes it (a gateway with N GPUs creates one engine per GPU, each
 * after ose_set_device(k) on the creating thread).                          */
int ose_set_device(int device);

/* Interned id of a service name referenced by a sampling rule, or OSE_NONE.
 * The shim uses it to fill res_svc / res_svc_str (rule_engine callers compare
 * service.name by equality only: latency.go:55, servicename.go:40).        */
uint32_t ose_engine_service_id(const ose_engine* eng, const char* name, size_t len);

/* Static per-engine facts the shim needs (OSE_STAGE_* bitmask of configured
 * processors; max output bytes per input path byte for tmpl_arena sizing). */
typedef struct ose_engine_info {
  uint32_t stages;
  uint32_t max_template_name;   /* longest "{name}" body the templater can emit */
  int64_t inverse_sampling;     /* odigostrafficmetrics int64(1/sampling_ratio) */
  double traffic_sampling_ratio;
  uint32_t n_attr_rules;        /* span_attribute rules (attr_match bits) */
  uint32_t n_attr_keys;         /* attribute keys the GPU-evaluated ones read */
  uint64_t attr_host_rules;     /* bit k: rule k is evaluated by the shim into
                                   attr_match even when attr_type is given (rules
                                   0..63; all of them: ose_engine_attr_host_rules) */
} ose_engine_info;
int ose_engine_get_info(const ose_engine* eng, ose_engine_info* info);
/* The shim-evaluated span_attribute rules as (n_attr_rules + 63) / 64 words
 * (bit k of word w: rule 64w + k); writes min(cap, that) words and returns
 * that count (0 without span_attribute rules).                             */
uint32_t ose_engine_attr_host_rules(const ose_engine* eng, uint64_t* words, uint32_t cap);
/* How often the SAMPLE stage left its fast path since the engine was created
 * (diagnostics and tests; no reference counterpart): counts[0] = calls whose
 * batch repeated a trace id (the run-list path ran), counts[1] = calls some
 * trace of which overflowed the run lists and was decided by the radix sort
 * by trace id, counts[2] = long-run passes (traces still open 4 steps past
 * their first window).  Synchronises the engine's device.  Writes
 * min(cap, 3) counters and returns 3.                                      */
uint32_t ose_engine_path_counts(ose_engine* eng, uint64_t* counts, uint32_t cap);

/* Attribute key k (< n_attr_keys) of the attr_type / attr_val columns; the
 * bytes stay valid for the engine's lifetime.                               */
int ose_engine_attr_key(const ose_engine* eng, uint32_t k, const char** key, uint32_t* len);

/* Engine options (no reference counterpart: they select the alternative
 * implementation of an OTLP leg, for tests that check the two against each
 * other; the defaults are the fast paths).  Set before the calls they affect,
 * not while such a call is in flight.  value 0 clears, non-zero sets.
 *   "otlp_gpu_chain"       walk the TracesData chain on the GPU (ose_otlp_decode)
 *   "otlp_host_resources"  ResourceSpans on the host, ScopeSpans on the GPU
 *   "otlp_host_scopes"     ResourceSpans and ScopeSpans on the host
 *   "encode_host"          ose_otlp_encode always uses the host encoder
 * OSE_EINVAL for any other name.                                            */
int ose_engine_set_option(ose_engine* eng, const char* name, int64_t value);

/* Pinned host staging: the engine owns the memory (cgo: no Go pointers are
 * retained).  dims->n_spans, n_resources, n_scopes, n_attrsets and
 * arena_bytes size the buffers; the returned columns/outputs point into
 * pinned memory the shim fills / reads.                                     */
int ose_batch_acquire(ose_engine* eng, const ose_columns* dims, ose_batch** out);
ose_columns* ose_batch_columns(ose_batch* b);
ose_outputs* ose_batch_outputs(ose_batch* b);
void ose_batch_release(ose_batch* b);

/* Synchronous: H2D of the batch, stages in `stage_mask`, D2H of results.
 * Replaces one ProcessTracesFunc call of each selected processor, run in
 * gateway pipeline order sample -> template -> size
 * (common/pipelinegen/config_builder.go:215-229).                           */
int ose_process(ose_engine* eng, ose_batch* b, uint32_t stage_mask,
                uint32_t group_mode, const ose_rand* rnd);

/* Asynchronous on `hip_stream` (a hipStream_t, NULL = default stream):
 * columns/outputs are device pointers already resident in HBM.  This is the
 * entry point the benchmark times.  One exception to "asynchronous": with
 * SAMPLE and OSE_GROUP_TRACE_ID the calling thread waits for SAMPLE's fast
 * pass (after queueing the URL kernels when TEMPLATE is in the mask) and
 * then queues trace_long_kernel only when the fast pass listed long runs and
 * the repeated-trace-id slow path only when a trace id repeats; the call
 * still returns before the URL and SIZE kernels finish.
 * hipGraph capture: every stage except SAMPLE with OSE_GROUP_TRACE_ID can be
 * captured (that one returns OSE_ENOTSUP while the stream is capturing); a
 * captured call keeps its workspace for the graph, so call ose_reserve
 * first.                                                                    */
int ose_process_device(ose_engine* eng, const ose_columns* cols,
                       const ose_outputs* outs, uint32_t stage_mask,
                       uint32_t group_mode, const ose_rand* rnd, void* hip_stream);

/* Workspace pre-sizing for ose_process_device (so the timed call performs no
 * allocation; required before a hipGraph capture).  arena_bytes: the largest
 * ose_columns.arena_bytes the calls will pass (the TEMPLATE stage's scratch
 * is sized from it).                                                        */
int ose_reserve(ose_engine* eng, uint64_t n_spans, uint64_t arena_bytes);

/* Per-kernel device time, measured with hipEvents recorded on the stream
 * each kernel is launched on (diagnostics and bench.py; off by default).
 * ose_profile_read writes {"<kernel>": {"launches": n, "ms": total}, ...}
 * and resets the counters; it synchronises the recorded events.           */
int ose_profile_enable(ose_engine* eng, int on);
int ose_profile_read(ose_engine* eng, char* json, size_t cap);

/* ---- trace-id exchange across the GPUs of a node ----------------------
 * odigossampling needs every span of a trace on one GPU.  In the reference
 * that co-location is the node collector's loadbalancing exporter keyed by
 * trace id (autoscaler/controllers/nodecollector/collectorconfig/
 * traces.go:26-84).  Here each GPU folds its spans into partial records
 * before the exchange: one record per stretch of consecutive spans with the
 * same trace id and the same latency service (and inside one 64-span
 * step), holding that stretch's share of the rule state — the error bit,
 * the endpoint bits (strings.HasPrefix of http.route against the service's
 * http_latency rules, latency.go:64-68 — route bytes never leave the
 * source), the service_name / span_attribute bits, and the latency element
 * (a zero start seen, min start after the last zero start, max end;
 * latency.go:69-80).  The trace's owner (trace-id hash mod n_ranks) folds
 * the records in (source rank, source order), i.e. in global batch order,
 * so decisions equal the single-GPU ones.
 *
 * Record (ose_shard_record_bytes = 40 + 16 per rule chunk): u64 trace_id
 * hi, lo, min start (~0 = none), max end, {latency service id : 24
 * (0xFFFFFF = none) | flags : 8 (1 error, 2 latency element present, 4 a
 * zero start came first)}, then per rule chunk (K of them:
 * a rule list beyond one GPU table) the endpoint bits and the rule bits
 * under that chunk's tables.  A record's stretch has one latency service
 * (a service with an http_latency rule in any chunk).
 *
 * ose_shard_pack writes the records into per-owner buckets of `send`
 * (stable: source order inside a bucket), counts[n_ranks] (records per
 * owner) and pack_pos[n_spans] (the slot of each span's record);
 * ose_shard_unpack turns received records into owner-side columns for
 * ose_process_device(SAMPLE, OSE_GROUP_TRACE_ID): one span and one
 * resource per record, svc_match set (route_match and svc_match: one
 * plane of n words per rule chunk, cols.match_planes), status bit 7 marking a record whose
 * zero start came first; the keep bytes go back with the reverse split and
 * ose_shard_scatter_keep puts them on the original spans.  All pointers
 * are device pointers; calls are asynchronous on hip_stream.
 * ose_exchange_sample runs the whole round over an RCCL communicator.      */
#define OSE_XREC_BYTES 56u   /* a config of one rule chunk; 40 + 16 per chunk */
uint32_t ose_shard_record_bytes(const ose_engine* eng);   /* 40 + 16 * rule chunks, 0 without odigossampling */
uint32_t ose_shard_owner(uint64_t tid_hi, uint64_t tid_lo, uint32_t n_ranks);
int ose_shard_pack(ose_engine* eng, const ose_columns* cols, uint32_t n_ranks, void* send,
                   uint64_t* counts, uint32_t* pack_pos, void* hip_stream);
int ose_shard_unpack(const void* recv, uint64_t n, uint32_t rec_bytes, uint64_t* trace_id,
                     uint64_t* start_ns, uint64_t* end_ns, uint8_t* status, uint32_t* resource,
                     uint32_t* res_svc, uint32_t* res_svc_str, uint64_t* route_match,
                     uint64_t* svc_match, void* hip_stream);
/* The owner's decisions for n received records (recv: the records of every
 * source in source-rank order, as the all-to-all delivers them): keep[i] for
 * record i.  The records are bucketed by trace-id hash and each bucket's
 * traces are grouped, put in batch order and folded in LDS; a bucket past
 * 256 records (kOwnerCap) sends the batch
 * through ose_shard_unpack + ose_process_device(SAMPLE) instead (same
 * decisions).  device_status (optional) as ose_outputs.device_status.  The
 * calling thread waits once (the fold's overflow word).  Replaces, with
 * ose_exchange_sample, the per-trace consumer behind the loadbalancing
 * exporter (collectorconfig/traces.go:26-84).                             */
int ose_shard_decide(ose_engine* eng, const void* recv, uint64_t n, uint32_t rec_bytes, uint8_t* keep,
                     uint32_t* device_status, const ose_rand* rnd, void* hip_stream);
int ose_shard_scatter_keep(const uint8_t* keep_back, const uint32_t* pack_pos, uint64_t n,
                           uint8_t* keep, void* hip_stream);

/* RCCL (resolved at run time; OSE_ENOTSUP when librccl is absent).  The
 * communicator is the caller's ncclComm_t as void*; these helpers create one
 * for a shim that does not link RCCL itself: rank 0 calls
 * ose_nccl_unique_id, the 128 bytes reach every rank out of band, and every
 * rank calls ose_nccl_comm_init.                                           */
int ose_nccl_unique_id(void* id_out, size_t cap);
int ose_nccl_comm_init(void** comm_out, int n_ranks, const void* id, int rank);
void ose_nccl_comm_destroy(void* comm);

/* One exchange round for this rank's batch (device columns, as
 * ose_process_device): pack, all-to-all of the record counts, grouped
 * send/recv of the records over xGMI, ose_shard_decide for the traces this
 * rank owns, the reverse split of the keep bytes and
 * the scatter into outs->keep.  Every rank of the communicator calls it for
 * the same round.  The calling thread waits once (the record counts size
 * the split).  stats (optional, [3]): records sent, records received, spans.
 * Rounds on one engine are serialised, on the host and on the device (a
 * round queued on another stream waits for the previous round's transfers).
 * Errors this rank can see alone (arguments, columns, scratch) are returned
 * before the first collective.  An error after it (a transfer, the owner's
 * SAMPLE stage) leaves the peers inside a collective: as after any NCCL
 * error, the communicator must then be destroyed by every rank.            */
int ose_exchange_sample(ose_engine* eng, const ose_columns* cols, const ose_outputs* outs,
                        void* nccl_comm, int rank, int n_ranks, const ose_rand* rnd,
                        void* hip_stream, uint64_t* stats);

/* Node-wide odigostrafficmetrics counters: node[k] = sum over the ranks of
 * local[k] (int64 ncclAllReduce; the counters of processor.go:76-81 summed
 * over the node's GPUs, as a scrape would sum the gateway replicas).
 * local and node may be the same buffer for the RCCL transport (in-place
 * ncclAllReduce); the in-process test transport refuses that (OSE_EINVAL). */
int ose_allreduce_counters(const int64_t* local, int64_t* node, uint64_t n, void* nccl_comm,
                           void* hip_stream);

/* ---- OTLP protobuf ingest -----------------------------
 * Replaces ptrace.ProtoUnmarshaler.UnmarshalTraces on the receive path
 * (collector/receivers/odigosebpfreceiver/traces.go:77-88) together with the
 * shim's columnising walk: one serialized TracesData (the body of an
 * ExportTraceServiceRequest; concatenated messages merge) becomes the
 * device columns this engine's stages read, for ose_process_device.
 * The host walks the message structure (ResourceSpans / ScopeSpans headers,
 * resource and scope contents, one header per span) while the bytes go
 * H2D; the GPU decodes every span (ids, times, status, kind, name, the
 * attributes the stages read, events and links for the sizes) and computes
 * span_size as pdata's sizer does.  Spans it cannot finish exactly (a value
 * that needs AsString or net/url.Parse, nested values, json span_attribute
 * keys, unusual ids or fields) get a host pass; ose_otlp_host_spans says how
 * many.  Strings are referenced in place: the arena is the message bytes,
 * followed by the host pass's strings.  What UnmarshalTraces rejects is
 * OSE_EINVAL.  Asynchronous work is on hip_stream; the call returns when
 * the columns are complete on that stream.  res_attrset ids index the
 * attribute sets ose_otlp_attrset returns ({"key": "value", ...}).         */
typedef struct ose_otlp_batch ose_otlp_batch;
/* Pinned host memory for a receiver to read requests into: ose_otlp_decode
 * copies a pinned message straight to HBM (a pageable one goes through the
 * batch's pinned staging first).                                           */
int ose_host_alloc(size_t bytes, void** out);
void ose_host_free(void* p);
int ose_otlp_decode(ose_engine* eng, const void* pb, size_t len, void* hip_stream, ose_otlp_batch** out);
const ose_columns* ose_otlp_columns(const ose_otlp_batch* b);   /* device pointers */
uint32_t ose_otlp_host_spans(const ose_otlp_batch* b);
/* host wall time of the call's phases (ms): bytes in (copy / H2D issue),
 * structural walk, columns upload, span decoder (+ sync), host pass */
int ose_otlp_timings(const ose_otlp_batch* b, double* ms5);
int ose_otlp_attrset(const ose_otlp_batch* b, uint32_t k, char* json, size_t cap);
/* copies every column whose dst pointer is non-NULL (host or device memory) */
int ose_otlp_download(const ose_otlp_batch* b, const ose_columns* dst);
void ose_otlp_release(ose_otlp_batch* b);

/* ---- output side: routing + OTLP re-encode ------------
 * ose_router replaces odigosrouterconnector's routing table
 * (collector/connectors/odigosrouterconnector/routingmap.go:34-57
 * BuildSignalRoutingMap, for the TRACES signal).  cfg_json is the
 * connector's Config: {"datastreams": [{"name": ..., "sources":
 * [{"namespace", "kind", "name"}], "destinations": [{"destinationname",
 * "configuredsignals": ["TRACES", ...]}]}]}.  Pipelines are the data
 * streams carrying TRACES, in order of first appearance.                    */
typedef struct ose_router ose_router;
int ose_router_create(const char* cfg_json, ose_router** out);
void ose_router_destroy(ose_router* r);
uint32_t ose_router_pipelines(const ose_router* r);
const char* ose_router_pipeline(const ose_router* r, uint32_t k);   /* owned by r */

/* Replaces the end of the gateway's traces/in pipeline: the processed
 * ptrace.Traces leaving the three processors, odigosrouterconnector's
 * ConsumeTraces (connector.go:174-237: each ResourceSpans copied to every
 * pipeline its k8s workload routes to, unmatched ones to "default") and the
 * exporters' ptrace.ProtoMarshaler.MarshalTraces.  `outs` are the outputs
 * ose_process_device wrote for this batch with `stages` / `group_mode`
 * (device or host memory; read on hip_stream): keep (or trace_keep[0] with
 * OSE_GROUP_BATCH) removes spans, emptied scopes and resources, url_out /
 * tmpl rename and template the kept spans.  With a router the outputs are
 * its pipelines then "default" (ose_router_pipelines + 1 of them); without,
 * one output.  Each output is a serialized TracesData, byte for byte what
 * pdata's marshaler writes for the processed traces; n_resources == 0 means
 * the connector would not call that pipeline.  The message bytes given to
 * ose_otlp_decode must be unchanged until this call returns.              */
typedef struct ose_otlp_out ose_otlp_out;
int ose_otlp_encode(ose_engine* eng, const ose_otlp_batch* b, const ose_outputs* outs, uint32_t stages,
                    uint32_t group_mode, const ose_router* router, void* hip_stream, ose_otlp_out** out);
uint32_t ose_otlp_out_count(const ose_otlp_out* o);
int ose_otlp_out_get(const ose_otlp_out* o, uint32_t k, const char** name, const uint8_t** data, uint64_t* len,
                     uint32_t* n_resources);   /* pointers valid until release */
void ose_otlp_out_release(ose_otlp_out* o);

/* ---- the OTLP path for concurrent callers -------------------------------
 * A receiver's concurrent export requests (each a serialized TracesData)
 * processed as one device batch per wave of calls: ose_otlp_pipeline_consume
 * runs decode -> `stages` (OSE_GROUP_TRACE_ID) -> route + re-encode for its
 * request together with the requests other threads hand in meanwhile, and
 * returns this request's outputs (the form ose_otlp_encode returns: the
 * router's pipelines then "default"; release with ose_otlp_out_release).
 * Each output is byte for byte what ose_otlp_encode writes for the request's
 * resources.  Differences from one call per request: spans of one trace that
 * arrive in concurrent requests are decided together (as groupbytrace hands
 * a whole trace to odigossampling); the traffic gate draws once per batch;
 * the odigostrafficmetrics counters are kept by the pipeline, summed over
 * its requests, and read (and reset) with ose_otlp_pipeline_counters:
 * {"accepted_spans": n, "data_size": [[{attributes}, bytes], ...], plus the
 * batching statistics}.  max_batch_bytes bounds a batch's message bytes (0:
 * 64 MiB; a larger request runs alone).  The router (may be NULL) must
 * outlive the pipeline; the pipeline holds a reference on the engine.     */
typedef struct ose_otlp_pipeline ose_otlp_pipeline;
int ose_otlp_pipeline_create(ose_engine* eng, const ose_router* router, uint32_t stages, uint64_t max_batch_bytes,
                             ose_otlp_pipeline** out);
int ose_otlp_pipeline_consume(ose_otlp_pipeline* p, const void* pb, size_t len, const ose_rand* rnd,
                              ose_otlp_out** out);
int ose_otlp_pipeline_counters(ose_otlp_pipeline* p, char* json, size_t cap);
void ose_otlp_pipeline_destroy(ose_otlp_pipeline* p);

/* ---- groupbytrace, resident in HBM ----------------------
 * Replaces the groupbytrace processor the gateway runs before odigossampling
 * (opentelemetry-collector-contrib groupbytraceprocessor v0.141.0,
 * `collector/builder-config.yaml:73`; configured by
 * `autoscaler/controllers/actions/sampling/groupbytrace.go:3-9` and
 * `sampling_controller.go:193-220`).  cfg_json: {"wait_duration": "30s",
 * "num_traces": 1000000, "num_workers": 1} (the processor's keys; Go
 * durations).  Spans wait on the GPU (span_capacity spans, arena_capacity
 * bytes of their route / path / attribute strings) until wait_duration after
 * their trace's first span; ose_gbt_release then returns every trace whose
 * time has come as one device batch: each trace contiguous, its pieces (one
 * per ResourceSpans x ScopeSpans it arrived in) in arrival order as
 * resources with one scope each, traces in creation order.  Run the
 * processors on it with OSE_GROUP_TRACE_ID: each trace is decided as
 * groupbytrace's one-trace ConsumeTraces call would be.  A new trace evicts
 * (drops) the one created num_traces creations earlier if it is still
 * waiting; with num_workers W > 1, the one created num_traces / W creations
 * earlier in its own worker (worker = FNV-1 64 of the id's 16 bytes mod W, as
 * contrib's event machine shards traces; num_traces >= W, else OSE_EINVAL).
 * now_ns is the caller's clock and must not go backwards.
 * attrset_map (n_attrsets of the added batch, may be NULL = identity) maps
 * the batch's res_attrset ids to ids stable across batches.  The released
 * columns stay valid until the next release; OSE_ERANGE when the store is
 * full (more spans than the capacity within one wait_duration).            */
typedef struct ose_gbt ose_gbt;
int ose_gbt_create(ose_engine* eng, const char* cfg_json, uint64_t span_capacity, uint64_t arena_capacity,
                   ose_gbt** out);
void ose_gbt_destroy(ose_gbt* g);
int ose_gbt_add(ose_gbt* g, const ose_columns* cols_dev, const uint32_t* attrset_map, int64_t now_ns,
                void* hip_stream);
int ose_gbt_release(ose_gbt* g, int64_t now_ns, void* hip_stream, const ose_columns** out_dev,
                    uint32_t* n_traces);
/* traces waiting, spans held, traces created / released / evicted, spans
 * released / added, string bytes held */
int ose_gbt_stats(const ose_gbt* g, uint64_t* out8);
/* copies every column of the last release whose dst pointer is non-NULL */
int ose_gbt_download(const ose_gbt* g, const ose_columns* dst);

/* HIP errors met by the entry points that return nothing (ose_*_release,
 * ose_*_destroy, ose_host_free) since the library loaded: they are recorded
 * here instead of being left in the HIP runtime's per-thread last-error
 * slot.  Returns the count; `last` (may be NULL) receives the latest one as
 * "entry point: hipErrorName (text)".                                        */
uint64_t ose_dropped_errors(char* last, size_t cap);

/* Message of the last failure on this thread ("" if none). */
const char* ose_last_error(void);

/* Runtime facts for diagnostics: device name, gfx arch, CU count. */
int ose_device_info(char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* ODIGOS_AMD_H */
