/*
 * sampling.c — CPU restatement of odigossamplingprocessor.  TEST
 * INFRASTRUCTURE (see oracle.h): the checker for the HIP trace stage and the
 * timed CPU baseline, never part of the product.
 *
 * Restates (paths under collector/processors/odigossamplingprocessor/):
 *   processor.go:16-25            processTraces / removeAllSpans (keep column)
 *   rule_engine.go:55-83          RuleEngine.ShouldSample
 *   rule_engine.go:89-115         evaluateLevel (order-sensitive fold)
 *   internal/sampling/error.go:29-44        ErrorRule.Evaluate
 *   internal/sampling/latency.go:44-100     HttpRouteLatencyRule.Evaluate
 *   internal/sampling/servicename.go:35-51  ServiceNameRule.Evaluate
 *
 * The rules are evaluated literally: one pass over the trace's spans per
 * rule, in batch order, with the same sentinel logic as the Go code.  The
 * only departure is rand.Float64(), replaced by the injected uniform of
 * include/odigos_amd.h so that decisions are reproducible.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

struct orc_sampling {
  int n;
  orc_rule* rules;   /* copies; route strings owned */
  orc_attr_cond* conds;   /* span_attribute rules with attr_col >= 0 */
  int* lat_index;    /* index of each http_latency rule among them (route_match bit) */
  int* attr_index;   /* index of each span_attribute rule among them (attr_match bit) */
};

orc_sampling* orc_sampling_create(const orc_rule* rules, int n_rules) {
  orc_sampling* s = (orc_sampling*)calloc(1, sizeof *s);
  s->n = n_rules;
  s->rules = (orc_rule*)calloc(n_rules > 0 ? (size_t)n_rules : 1, sizeof(orc_rule));
  s->lat_index = (int*)calloc(n_rules > 0 ? (size_t)n_rules : 1, sizeof(int));
  s->attr_index = (int*)calloc(n_rules > 0 ? (size_t)n_rules : 1, sizeof(int));
  s->conds = (orc_attr_cond*)calloc(n_rules > 0 ? (size_t)n_rules : 1, sizeof(orc_attr_cond));
  int nl = 0, na = 0;
  for (int i = 0; i < n_rules; i++) {
    s->lat_index[i] = rules[i].type == ORC_RULE_LATENCY ? nl++ : -1;
    s->attr_index[i] = rules[i].type == ORC_RULE_ATTR ? na++ : -1;
  }
  for (int i = 0; i < n_rules; i++) {
    s->rules[i] = rules[i];
    char* r = (char*)malloc(rules[i].route_len + 1);
    if (rules[i].route_len) memcpy(r, rules[i].route, rules[i].route_len);
    r[rules[i].route_len] = 0;
    s->rules[i].route = r;
    if (rules[i].type == ORC_RULE_ATTR && rules[i].attr_col >= 0 &&
        orc_attr_cond_init(&s->conds[i], rules[i].attr_cond, rules[i].attr_op, rules[i].attr_expected,
                           rules[i].attr_expected_len) != 0)
      s->rules[i].attr_col = -1;
    s->rules[i].attr_cond = s->rules[i].attr_op = s->rules[i].attr_expected = NULL;
  }
  return s;
}

void orc_sampling_free(orc_sampling* s) {
  if (!s) return;
  for (int i = 0; i < s->n; i++) {
    free((void*)s->rules[i].route);
    if (s->rules[i].type == ORC_RULE_ATTR && s->rules[i].attr_col >= 0) orc_attr_cond_free(&s->conds[i]);
  }
  free(s->conds);
  free(s->rules);
  free(s->lat_index);
  free(s->attr_index);
  free(s);
}

static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

double orc_trace_uniform(uint64_t hi, uint64_t lo, uint64_t seed) {
  uint64_t x = hi ^ ((lo << 29) | (lo >> 35)) ^ seed;
  return (double)(splitmix64(x) >> 11) * 0x1.0p-53;
}

/* One trace = a list of span indices in batch order. */
typedef struct {
  const ose_columns* c;
  const uint32_t* spans;
  uint64_t n;
  int batch_mode;   /* ServiceNameRule scans every resource of the batch */
} trace_view;

typedef struct { int matched, satisfied; double ratio; } eval_t;

static eval_t eval_error(const orc_rule* r, const trace_view* t) {
  /* error.go:29-44: matched is always true */
  for (uint64_t k = 0; k < t->n; k++)
    if (t->c->status[t->spans[k]] == OSE_STATUS_ERROR) return (eval_t){1, 1, 100.0};
  return (eval_t){1, 0, r->fallback};
}

/* time.Time.Sub on two time.Unix(0, ns) values: exact int64 difference,
 * saturated at the Duration range (time.go Sub's overflow checks). */
static int64_t go_sub_ns(int64_t t, int64_t u) {
  int64_t d;
  if (__builtin_sub_overflow(t, u, &d)) return t < u ? INT64_MIN : INT64_MAX;
  return d;
}

static eval_t eval_latency(const orc_rule* r, int lat_index, const trace_view* t) {
  const ose_columns* c = t->c;
  int service_found = 0, endpoint_found = 0;
  uint64_t min_start = 0, max_end = 0;   /* pcommon.Timestamp sentinels */
  for (uint64_t k = 0; k < t->n; k++) {
    uint32_t i = t->spans[k];
    /* AsString(service.name) != ServiceName -> skip the resource (latency.go:51-56) */
    if (c->res_svc[c->resource[i]] != r->svc || r->svc == OSE_NONE) continue;
    service_found = 1;
    if (c->route_match) {   /* precomputed HasPrefix bits (ose_columns.route_match) */
      if ((c->route_match[i] >> lat_index) & 1) endpoint_found = 1;
    } else {
      ose_strref rt = c->route ? c->route[i] : (ose_strref){0, 0};   /* AsString(http.route); absent == "" here (no column: every span absent) */
      if (rt.len >= r->route_len && memcmp(c->arena + rt.off, r->route, r->route_len) == 0)
        endpoint_found = 1;   /* strings.HasPrefix (latency.go:97-100) */
    }
    uint64_t s = c->start_ns[i], e = c->end_ns[i];
    if (min_start == 0 || s < min_start) min_start = s;
    if (max_end == 0 || e > max_end) max_end = e;
  }
  if (!service_found || !endpoint_found) return (eval_t){0, 0, 0.0};
  /* maxEnd.AsTime().Sub(minStart.AsTime()).Milliseconds() */
  int64_t ms = go_sub_ns((int64_t)max_end, (int64_t)min_start) / 1000000;
  if (ms >= r->threshold) return (eval_t){1, 1, 100.0};
  return (eval_t){1, 0, r->fallback};
}

static eval_t eval_service(const orc_rule* r, const trace_view* t) {
  const ose_columns* c = t->c;
  /* resourceAttrs service.name Str() == ServiceName (servicename.go:38-47) */
  if (r->svc != OSE_NONE) {
    if (t->batch_mode) {
      for (uint32_t q = 0; q < c->n_resources; q++)
        if (c->res_svc_str[q] == r->svc) return (eval_t){1, 1, r->ratio};
    } else {
      for (uint64_t k = 0; k < t->n; k++)
        if (c->res_svc_str[c->resource[t->spans[k]]] == r->svc) return (eval_t){1, 1, r->ratio};
    }
  }
  return (eval_t){0, 0, r->fallback};
}

/* SpanAttributeRule.Evaluate (spanattribute.go:126-320) over the per-span
 * condition bits: (true, true, ratio) as soon as one span of the trace meets
 * it, else (false, false, fallback) — never matched-but-unsatisfied. */
static eval_t eval_attr(const orc_rule* r, const orc_attr_cond* cond, int attr_index, const trace_view* t) {
  const ose_columns* c = t->c;
  if (r->attr_col >= 0 && c->attr_type && (uint32_t)r->attr_col < c->n_attr_keys) {
    /* spanattribute.go:127-135: resources whose AsString(service.name) is the
     * rule's service, then Get(AttributeKey) per span */
    const uint64_t n = c->n_spans;
    for (uint64_t k = 0; k < t->n; k++) {
      const uint32_t i = t->spans[k];
      if (r->svc == OSE_NONE || c->res_svc[c->resource[i]] != r->svc) continue;
      const uint64_t j = (uint64_t)r->attr_col * n + i;
      const uint8_t ty = c->attr_type[j];
      if (ty == OSE_ATTR_ABSENT) continue;
      if (orc_attr_cond_eval(cond, ty, c->attr_val[j], c->arena)) return (eval_t){1, 1, r->ratio};
    }
    return (eval_t){0, 0, r->fallback};
  }
  /* bit attr_index of the span's attr_match words (word-major planes, ose_columns.attr_match_words) */
  const uint64_t plane = (uint64_t)(attr_index / 64) * c->n_spans;
  for (uint64_t k = 0; k < t->n; k++)
    if ((c->attr_match[plane + t->spans[k]] >> (attr_index % 64)) & 1) return (eval_t){1, 1, r->ratio};
  return (eval_t){0, 0, r->fallback};
}

/* evaluateLevel (rule_engine.go:89-115) */
static void evaluate_level(const orc_sampling* s, int level, const trace_view* t, double* ratio, int* sat,
                           int* matched) {
  int found_fallback = 0;
  *ratio = 0;
  *sat = 0;
  *matched = 0;
  for (int k = 0; k < s->n; k++) {
    const orc_rule* r = &s->rules[k];
    if (r->level != level) continue;
    eval_t e;
    switch (r->type) {
      case ORC_RULE_ERROR: e = eval_error(r, t); break;
      case ORC_RULE_LATENCY: e = eval_latency(r, s->lat_index[k], t); break;
      case ORC_RULE_ATTR: e = eval_attr(r, &s->conds[k], s->attr_index[k], t); break;
      default: e = eval_service(r, t); break;
    }
    if (e.satisfied) {
      *sat = 1;
      *ratio = *ratio > e.ratio ? *ratio : e.ratio;   /* Go max(): ratios are never NaN (Validate) */
      *matched = 1;
    } else if (e.matched) {
      *matched = 1;
      if (!found_fallback) {
        *ratio = e.ratio;
        found_fallback = 1;
      } else {
        *ratio = *ratio < e.ratio ? *ratio : e.ratio;
      }
    }
  }
}

/* ShouldSample (rule_engine.go:55-83).  level out: 0..2 = the satisfied
 * level, 3 = min fallback over matched levels, 4 = nothing matched. */
static int should_sample(const orc_sampling* s, const trace_view* t, double u, uint8_t* level, double* ratio_out) {
  int have_min = 0;
  double min_fb = 0;
  for (int L = 0; L < 3; L++) {
    double ratio;
    int sat, matched;
    evaluate_level(s, L, t, &ratio, &sat, &matched);
    if (sat) {
      *level = (uint8_t)L;
      *ratio_out = ratio;
      return u * 100 < ratio;
    }
    if (matched && (!have_min || ratio < min_fb)) {
      min_fb = ratio;
      have_min = 1;
    }
  }
  if (have_min) {
    *level = 3;
    *ratio_out = min_fb;
    return u * 100 < min_fb;
  }
  *level = 4;
  *ratio_out = 100.0;
  return 1;
}

/* ---- grouping by trace_id (first-appearance order) ---- */
typedef struct { uint64_t hi, lo; uint32_t trace; uint32_t used; } slot_t;

static uint64_t mix(uint64_t hi, uint64_t lo) { return splitmix64(hi ^ splitmix64(lo)); }

typedef struct {
  const orc_sampling* s;
  const ose_columns* c;
  ose_outputs* o;
  const uint32_t* first;   /* trace -> offset into members */
  const uint32_t* members; /* span indices grouped by trace, batch order */
  uint32_t lo, hi;         /* trace range */
  int batch_mode;
  uint64_t seed;
  uint8_t* tkeep;
} job_t;

static void* run_traces(void* arg) {
  job_t* j = (job_t*)arg;
  const ose_columns* c = j->c;
  for (uint32_t t = j->lo; t < j->hi; t++) {
    trace_view v = {c, j->members + j->first[t], (uint64_t)(j->first[t + 1] - j->first[t]), j->batch_mode};
    uint64_t hi = 0, lo = 0;
    if (v.n) {
      hi = c->trace_id[2 * (uint64_t)v.spans[0]];
      lo = c->trace_id[2 * (uint64_t)v.spans[0] + 1];
    }
    uint8_t level;
    double ratio;
    int keep = should_sample(j->s, &v, orc_trace_uniform(hi, lo, j->seed), &level, &ratio);
    j->tkeep[t] = (uint8_t)keep;
    ose_outputs* o = j->o;
    if (o->trace_keep) o->trace_keep[t] = (uint8_t)keep;
    if (o->trace_level) o->trace_level[t] = level;
    if (o->trace_ratio) o->trace_ratio[t] = ratio;
    if (o->trace_first_span) o->trace_first_span[t] = v.n ? v.spans[0] : 0;
    if (o->keep)
      for (uint64_t k = 0; k < v.n; k++) o->keep[v.spans[k]] = (uint8_t)keep;
  }
  return NULL;
}

/* Grouping by trace_id in first-appearance order, threaded: spans are
 * partitioned by trace hash (stable, batch order inside a partition), each
 * partition groups its spans with a private table, and a trace's global
 * index is the rank of its first span among all first spans. */
typedef struct {
  const ose_columns* c;
  uint64_t lo, hi;            /* span range (passes 1, 2, 4) */
  uint32_t part, nparts;      /* partition (pass 3, 5) */
  uint64_t* counts;           /* [nparts] spans per partition in this range */
  uint64_t* offs;             /* [nparts] scatter cursors */
  uint32_t* part_spans;
  const uint64_t* part_first; /* [nparts + 1] */
  uint8_t* is_first;
  uint32_t* trace_local;      /* local trace id per span (pass 3) -> global (pass 5) */
  uint64_t nfirst;            /* pass 4: first spans in the range; then the range's base */
  uint32_t* rank_first;       /* global trace index at each first span */
  uint32_t* first;            /* [ntr + 1] offsets (pass 5 counts, pass 6 fill) */
  uint32_t* members;
  uint32_t* local_first;      /* pass 3: local trace -> first span (per partition, in part_spans space) */
} group_job;

static uint32_t part_of(uint64_t hi, uint64_t lo, uint32_t nparts) {
  return (uint32_t)((mix(hi, lo) >> 40) % nparts);
}
static void* g_count(void* p) {
  group_job* j = (group_job*)p;
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->counts[part_of(j->c->trace_id[2 * i], j->c->trace_id[2 * i + 1], j->nparts)]++;
  return NULL;
}
static void* g_scatter(void* p) {
  group_job* j = (group_job*)p;
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->part_spans[j->offs[part_of(j->c->trace_id[2 * i], j->c->trace_id[2 * i + 1], j->nparts)]++] = (uint32_t)i;
  return NULL;
}
static void* g_local(void* p) {   /* private table over one partition, batch order */
  group_job* j = (group_job*)p;
  const uint64_t a = j->part_first[j->part], b = j->part_first[j->part + 1], m = b - a;
  uint64_t cap = 16;
  while (cap < 2 * m) cap <<= 1;
  slot_t* tab = (slot_t*)calloc(cap, sizeof(slot_t));
  uint32_t nt = 0;
  for (uint64_t k = a; k < b; k++) {
    const uint32_t i = j->part_spans[k];
    const uint64_t hi = j->c->trace_id[2 * (uint64_t)i], lo = j->c->trace_id[2 * (uint64_t)i + 1];
    uint64_t h = mix(hi, lo) & (cap - 1);
    for (;;) {
      slot_t* e = &tab[h];
      if (!e->used) {
        e->used = 1;
        e->hi = hi;
        e->lo = lo;
        e->trace = nt++;
        j->is_first[i] = 1;
        j->trace_local[i] = e->trace;
        break;
      }
      if (e->hi == hi && e->lo == lo) {
        j->trace_local[i] = e->trace;
        break;
      }
      h = (h + 1) & (cap - 1);
    }
  }
  free(tab);
  /* local trace -> its first span (first occurrences are in batch order) */
  j->local_first = (uint32_t*)malloc((nt ? nt : 1) * sizeof(uint32_t));
  for (uint64_t k = a; k < b; k++) {
    const uint32_t i = j->part_spans[k];
    if (j->is_first[i]) j->local_first[j->trace_local[i]] = i;
  }
  j->nfirst = nt;
  return NULL;
}
static void* g_rank_count(void* p) {
  group_job* j = (group_job*)p;
  uint64_t c = 0;
  for (uint64_t i = j->lo; i < j->hi; i++) c += j->is_first[i];
  j->nfirst = c;
  return NULL;
}
static void* g_rank_fill(void* p) {
  group_job* j = (group_job*)p;
  uint64_t r = j->nfirst;
  for (uint64_t i = j->lo; i < j->hi; i++)
    if (j->is_first[i]) j->rank_first[i] = (uint32_t)r++;
  return NULL;
}
static void* g_globalize(void* p) {   /* per partition: global trace ids, span counts per trace */
  group_job* j = (group_job*)p;
  const uint64_t a = j->part_first[j->part], b = j->part_first[j->part + 1];
  for (uint64_t k = a; k < b; k++) {
    const uint32_t i = j->part_spans[k];
    const uint32_t g = j->rank_first[j->local_first[j->trace_local[i]]];
    j->trace_local[i] = g;
    j->first[g + 1]++;
  }
  free(j->local_first);
  return NULL;
}
static void* g_members(void* p) {   /* per partition: members in batch order (traces are disjoint) */
  group_job* j = (group_job*)p;
  const uint64_t a = j->part_first[j->part], b = j->part_first[j->part + 1];
  for (uint64_t k = a; k < b; k++) {
    const uint32_t i = j->part_spans[k];
    j->members[j->first[j->trace_local[i]]++] = i;   /* `first` holds fill cursors here */
  }
  return NULL;
}
static void run_group(void* (*fn)(void*), group_job* jobs, int T) {
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
  fn(&jobs[0]);
  for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
  free(th);
}

/* trace_of[i] = trace index (first-appearance order); first[] = offsets of
 * each trace in members[] (spans in batch order); returns the trace count */
static uint32_t group_traces(const ose_columns* c, int T, uint32_t* trace_of, uint32_t** first_out,
                             uint32_t** members_out) {
  const uint64_t n = c->n_spans;
  if (T < 1) T = 1;
  if (T > ORC_MAX_THREADS) T = ORC_MAX_THREADS;
  if (n < (uint64_t)T * 4096) T = 1;
  group_job* jobs = (group_job*)calloc((size_t)T, sizeof(group_job));
  uint64_t* counts = (uint64_t*)calloc((size_t)T * T, sizeof(uint64_t));
  uint32_t* part_spans = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  uint64_t* part_first = (uint64_t*)calloc((size_t)T + 1, sizeof(uint64_t));
  uint8_t* is_first = (uint8_t*)calloc(n ? n : 1, 1);
  uint32_t* rank_first = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  for (int t = 0; t < T; t++) {
    group_job* j = &jobs[t];
    j->c = c;
    j->lo = n * (uint64_t)t / (uint64_t)T;
    j->hi = n * (uint64_t)(t + 1) / (uint64_t)T;
    j->part = (uint32_t)t;
    j->nparts = (uint32_t)T;
    j->counts = counts + (size_t)t * T;
    j->offs = j->counts;
    j->part_spans = part_spans;
    j->part_first = part_first;
    j->is_first = is_first;
    j->trace_local = trace_of;
    j->rank_first = rank_first;
  }
  run_group(g_count, jobs, T);
  /* cursor of range t in partition p = partition start + counts of earlier ranges */
  uint64_t acc = 0;
  for (int p = 0; p < T; p++) {
    part_first[p] = acc;
    for (int t = 0; t < T; t++) {
      const uint64_t k = counts[(size_t)t * T + p];
      counts[(size_t)t * T + p] = acc;
      acc += k;
    }
  }
  part_first[T] = acc;
  run_group(g_scatter, jobs, T);
  run_group(g_local, jobs, T);
  uint64_t local_tr[ORC_MAX_THREADS];
  uint64_t ntr = 0;
  for (int t = 0; t < T; t++) { local_tr[t] = jobs[t].nfirst; ntr += jobs[t].nfirst; }
  run_group(g_rank_count, jobs, T);
  uint64_t base = 0;
  for (int t = 0; t < T; t++) { const uint64_t k = jobs[t].nfirst; jobs[t].nfirst = base; base += k; }
  run_group(g_rank_fill, jobs, T);
  uint32_t* first = (uint32_t*)calloc((size_t)ntr + 1, sizeof(uint32_t));
  uint32_t* members = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  for (int t = 0; t < T; t++) { jobs[t].first = first; jobs[t].members = members; jobs[t].nfirst = local_tr[t]; }
  run_group(g_globalize, jobs, T);
  for (uint64_t t = 0; t < ntr; t++) first[t + 1] += first[t];
  uint32_t* fill = (uint32_t*)malloc(((size_t)ntr + 1) * sizeof(uint32_t));
  memcpy(fill, first, ((size_t)ntr + 1) * sizeof(uint32_t));
  for (int t = 0; t < T; t++) jobs[t].first = fill;
  run_group(g_members, jobs, T);
  free(fill);
  free(jobs); free(counts); free(part_spans); free(part_first); free(is_first); free(rank_first);
  *first_out = first;
  *members_out = members;
  return (uint32_t)ntr;
}

int orc_sampling_process(const orc_sampling* s, const ose_columns* c, ose_outputs* o, uint32_t group_mode,
                         const ose_rand* rnd, int nthreads) {
  const uint64_t n = c->n_spans;
  if (n > 0xFFFFFFFEull) return -1;
  uint32_t* trace_of = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  uint32_t ntr = 0;
  uint32_t* first;
  uint32_t* members;
  if (group_mode == OSE_GROUP_BATCH) {
    ntr = 1;
    first = (uint32_t*)calloc(2, sizeof(uint32_t));
    first[1] = (uint32_t)n;
    members = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    for (uint64_t i = 0; i < n; i++) { trace_of[i] = 0; members[i] = (uint32_t)i; }
  } else {
    ntr = group_traces(c, nthreads, trace_of, &first, &members);
  }
  uint8_t* tkeep = (uint8_t*)malloc(ntr ? ntr : 1);

  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > ntr) nthreads = ntr ? (int)ntr : 1;
  job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job_t* j = &jobs[t];
    j->s = s;
    j->c = c;
    j->o = o;
    j->first = first;
    j->members = members;
    j->lo = (uint32_t)((uint64_t)ntr * (uint64_t)t / (uint64_t)nthreads);
    j->hi = (uint32_t)((uint64_t)ntr * (uint64_t)(t + 1) / (uint64_t)nthreads);
    j->batch_mode = group_mode == OSE_GROUP_BATCH;
    j->seed = rnd ? rnd->seed : 0;
    j->tkeep = tkeep;
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, run_traces, &jobs[t]);
  run_traces(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  if (o->trace_count) *o->trace_count = ntr;
  free(jobs);
  free(th);
  free(tkeep);
  free(members);
  free(first);
  free(trace_of);
  return 0;
}
