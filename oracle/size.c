/*
 * size.c — CPU restatement of odigostrafficmetrics (traces).  TEST
 * INFRASTRUCTURE (see oracle.h): the checker for the HIP size stage and the
 * timed CPU baseline, never part of the product.
 *
 * Restates (paths under collector/processors/odigostrafficmetrics/):
 *   processor.go:31-58   newThroughputMeasurementProcessor (inverse = int64(1/ratio))
 *   processor.go:60-69   attributeSetFromResource (host-interned: res_attrset column)
 *   processor.go:71-84   processTraces
 * and the third-party size it calls, ptrace.ProtoMarshaler.ResourceSpansSize
 * (pdata v1.47.0), as the OTLP trace.proto wire size over the columns:
 *   ResourceSpans = res_size (resource + schema_url, host-sized)
 *                 + sum over surviving scopes of framed ScopeSpans
 *   ScopeSpans    = scope_size (scope + schema_url) + sum of framed Spans
 *   Span          = span_size (host-sized before mutation) + the growth the
 *                   odigosurltemplate stage causes: one appended KeyValue
 *                   (http.route / url.template, processor.go:259-261) and the
 *                   renamed span (processor.go:214-233).
 * The batch is the one the earlier gateway stages produced: spans of
 * dropped traces are gone, and a ScopeSpans / ResourceSpans emptied by the
 * drop is gone (host apply, odigos_amd/csrc/host.cpp TracesProcessor::Apply);
 * with OSE_GROUP_BATCH a dropped trace empties the whole call
 * (removeAllSpans, odigossamplingprocessor/processor.go:23-25).
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static uint64_t sov(uint64_t x) {
  uint64_t n = 1;
  while (x >= 0x80) { x >>= 7; n++; }
  return n;
}
static uint64_t field_len(uint64_t l) { return 1 + sov(l) + l; }   /* tag (field < 16) + varint + payload */

uint64_t orc_span_size_after(const ose_columns* c, const ose_outputs* res, uint32_t stages, uint64_t i) {
  uint64_t sz = c->span_size[i];
  if (!(stages & OSE_STAGE_TEMPLATE) || !res->url_out[i]) return sz;
  const uint64_t tl = res->tmpl[i].len;
  if (res->url_out[i] & OSE_OUT_SET_ATTR) {
    /* attr.PutStr(target, tmpl) on an absent key: one more KeyValue (field 9)
     * {key (1): target, value (2): AnyValue{string_value (1): tmpl}} */
    const uint64_t keylen = c->kind[i] == OSE_KIND_CLIENT ? 12 /* url.template */ : 10 /* http.route */;
    const uint64_t kv = field_len(keylen) + field_len(field_len(tl));
    sz += field_len(kv);
  }
  if (res->url_out[i] & OSE_OUT_RENAME) {
    /* span.SetName(method + " " + tmpl) where the old name == method (field 5) */
    const uint64_t old = c->name_len[i];
    sz += field_len(old + 1 + tl) - (old ? field_len(old) : 0);
  }
  return sz;
}

/* Work split for the threaded form: [lo, hi) of n items cut at t*n/T and
 * moved forward to the next change of key[] (scopes / resources are
 * non-decreasing), so every key belongs to exactly one part. */
static uint64_t cut(const uint32_t* key, uint64_t n, uint64_t t, uint64_t T) {
  uint64_t b = n * t / T;
  if (b == 0 || b >= n) return b >= n ? n : 0;
  while (b < n && key[b] == key[b - 1]) b++;
  return b;
}

typedef struct {
  const ose_columns* c;
  const ose_outputs* res;
  ose_outputs* o;
  uint32_t stages;
  int sampled;
  int64_t inverse;
  uint64_t lo, hi;           /* spans, then scopes, then resources */
  uint64_t* sbody;
  uint8_t* shad;
  uint64_t* skept;
  uint64_t* rbody;
  uint8_t* rhad;
  uint32_t* ralive;
  int64_t accepted;
  int64_t* attr;             /* per-thread attribute-set sums */
} SizeJob;

static void* size_spans(void* p) {
  SizeJob* j = (SizeJob*)p;
  const ose_columns* c = j->c;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint32_t s = c->scope[i];
    j->shad[s] = 1;
    if (j->sampled && !j->res->keep[i]) continue;
    j->skept[s]++;
    j->accepted++;
    j->sbody[s] += field_len(orc_span_size_after(c, j->res, j->stages, i));   /* ScopeSpans.spans (2) */
  }
  return NULL;
}
static void* size_scopes(void* p) {
  SizeJob* j = (SizeJob*)p;
  const ose_columns* c = j->c;
  for (uint64_t s = j->lo; s < j->hi; s++) {
    const uint32_t r = c->scope_resource[s];
    j->rhad[r] |= j->shad[s];
    if (!j->shad[s] || j->skept[s]) {   /* emptied scopes are removed, spanless ones stay */
      j->ralive[r]++;
      j->rbody[r] += field_len(c->scope_size[s] + j->sbody[s]);   /* ResourceSpans.scope_spans (2) */
    }
  }
  return NULL;
}
static void* size_resources(void* p) {
  SizeJob* j = (SizeJob*)p;
  const ose_columns* c = j->c;
  for (uint64_t r = j->lo; r < j->hi; r++) {
    if (j->sampled && j->rhad[r] && !j->ralive[r]) continue;   /* emptied resource removed */
    const uint64_t size = c->res_size[r] + j->rbody[r];
    if (j->o->res_bytes) j->o->res_bytes[r] = size;
    j->attr[c->res_attrset[r]] += (int64_t)size * j->inverse;
  }
  return NULL;
}

static void run_jobs(void* (*fn)(void*), SizeJob* jobs, int T) {
  pthread_t th[ORC_MAX_THREADS];
  for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
  fn(&jobs[0]);
  for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
}

int orc_size_process_mt(const ose_columns* c, const ose_outputs* res, uint32_t stages, uint32_t group_mode,
                        ose_outputs* o, int64_t inverse, double sampling_ratio, double traffic_u, int nthreads) {
  const uint64_t n = c->n_spans;
  const uint32_t R = c->n_resources, S = c->n_scopes;
  /* if p.samplingFraction != 0 && rand.Float64() < p.samplingFraction (processor.go:72) */
  if (!(sampling_ratio != 0 && traffic_u < sampling_ratio)) return 0;
  const int sampled = (stages & (OSE_STAGE_SAMPLE | OSE_STAGE_APPLY_KEEP)) != 0;
  if (o->res_bytes) memset(o->res_bytes, 0, (size_t)R * sizeof(uint64_t));
  if ((stages & OSE_STAGE_SAMPLE) && group_mode == OSE_GROUP_BATCH && !res->trace_keep[0]) return 0;   /* td emptied */
  int T = nthreads < 1 ? 1 : nthreads > ORC_MAX_THREADS ? ORC_MAX_THREADS : nthreads;
  if (n < (uint64_t)T * 4096) T = 1;
  uint64_t* sbody = (uint64_t*)calloc(S ? S : 1, sizeof(uint64_t));
  uint8_t* shad = (uint8_t*)calloc(S ? S : 1, 1);
  uint64_t* skept = (uint64_t*)calloc(S ? S : 1, sizeof(uint64_t));
  uint64_t* rbody = (uint64_t*)calloc(R ? R : 1, sizeof(uint64_t));
  uint8_t* rhad = (uint8_t*)calloc(R ? R : 1, 1);
  uint32_t* ralive = (uint32_t*)calloc(R ? R : 1, sizeof(uint32_t));
  const uint32_t A = c->n_attrsets ? c->n_attrsets : 1;
  int64_t* attr = (int64_t*)calloc((size_t)T * A, sizeof(int64_t));
  SizeJob jobs[ORC_MAX_THREADS];
  for (int t = 0; t < T; t++) {
    SizeJob j = {c, res, o, stages, sampled, inverse, cut(c->scope, n, t, T), cut(c->scope, n, t + 1, T),
                 sbody, shad, skept, rbody, rhad, ralive, 0, attr + (size_t)t * A};
    jobs[t] = j;
  }
  run_jobs(size_spans, jobs, T);
  int64_t accepted = 0;
  for (int t = 0; t < T; t++) {
    accepted += jobs[t].accepted;
    jobs[t].lo = cut(c->scope_resource, S, t, T);
    jobs[t].hi = cut(c->scope_resource, S, t + 1, T);
  }
  run_jobs(size_scopes, jobs, T);
  for (int t = 0; t < T; t++) {
    jobs[t].lo = (uint64_t)R * t / T;
    jobs[t].hi = (uint64_t)R * (t + 1) / T;
  }
  run_jobs(size_resources, jobs, T);
  for (int t = 0; t < T; t++)
    for (uint32_t a = 0; a < A; a++) o->attrset_bytes[a] += attr[(size_t)t * A + a];
  *o->accepted_spans += accepted;
  free(sbody); free(shad); free(skept); free(rbody); free(rhad); free(ralive); free(attr);
  return 0;
}

int orc_size_process(const ose_columns* c, const ose_outputs* res, uint32_t stages, uint32_t group_mode,
                     ose_outputs* o, int64_t inverse, double sampling_ratio, double traffic_u) {
  return orc_size_process_mt(c, res, stages, group_mode, o, inverse, sampling_ratio, traffic_u, 1);
}
