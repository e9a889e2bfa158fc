/*
 * oracle.h — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline; the
 * product (odigos_amd) never links or calls it.
 *
 * Each function restates a function of damemi/odigos @ 2026-02-13 (paths
 * relative to collector/processors/) over the columnar batch defined in
 * include/odigos_amd.h.  Parity is pinned by the reference's own known-answer
 * tests, transcribed as data under tests/golden/ (Go is not available, so the
 * reference cannot be run here; see DESIGN.md "Oracle").
 */
#ifndef OSE_ORACLE_H
#define OSE_ORACLE_H
#include <stdint.h>
#include <stddef.h>
#include "../include/odigos_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- regexp (Go RE2 syntax subset, backtracking; oracle-private) ----- */
typedef struct orc_re orc_re;
/* Unicode data for \p{..} and (?i) (unicode_data.c, generated): inclusive
 * {lo, hi} pairs; orc_fold_next: {rune, next rune of its simple-folding orbit} */
typedef struct { const char* name; const int* r; int n; } orc_utab;
extern const orc_utab orc_ucats[];
extern const int orc_ucats_n;
extern const orc_utab orc_uscripts[];
extern const int orc_uscripts_n;
extern const int orc_fold_next[];
extern const int orc_fold_n;
/* returns NULL and fills err on a syntax error the Go parser would reject */
orc_re* orc_re_compile(const char* pattern, char* err, size_t errcap);
/* regexp.MatchString semantics: unanchored search over the UTF-8 string */
int orc_re_match(const orc_re* re, const uint8_t* s, size_t n);
void orc_re_free(orc_re* re);

/* ---- odigosurltemplate -------------------------------------------------- */
typedef struct orc_url orc_url;
/* rules: templatization_rules strings; custom_*: custom_ids (regexp,
 * template_name).  Returns NULL + err on the errors
 * newUrlTemplateProcessor / Config.Validate return (processor.go:27-69,
 * config.go:133-157). */
orc_url* orc_url_create(const char* const* rules, int n_rules,
                        const char* const* custom_regexps,
                        const char* const* custom_names, int n_custom,
                        char* err, size_t errcap);
void orc_url_free(orc_url* u);

/* getSegmentTemplatizationString (templatize.go:242-269): writes the name
 * (without braces) into out and returns its length, or -1 if the segment is
 * not an id.  out must hold >= 256 bytes. */
int orc_url_segment_name(const orc_url* u, const uint8_t* seg, size_t n, char* out);

/* applyTemplatizationOnPath (processor.go:149-186): returns the templated
 * path length written to out (cap bytes), or -1 if cap is too small. */
long orc_url_apply_path(const orc_url* u, const uint8_t* path, size_t n,
                        uint8_t* out, size_t cap);

/* processTraces over a whole batch (processor.go:71-96 + 235-287): fills
 * outs->url_out, outs->tmpl and outs->tmpl_arena (compact, span order) and
 * *outs->tmpl_arena_used.  nthreads >= 1 splits the spans over pthreads.
 * Returns 0, or -1 if the arena capacity is exceeded. */
int orc_url_process(const orc_url* u, const ose_columns* c, ose_outputs* o,
                    int nthreads);

/* ---- odigossampling ------------------------------------------------------ */
/* One rule of the decoded config (odigossamplingprocessor/config.go:28-32
 * after decodeAndValidate).  svc is the interned id of the rule's service
 * name in first-appearance order over global, service, endpoint rules (the
 * id the shim writes into res_svc / res_svc_str). */
#define ORC_RULE_ERROR    0
#define ORC_RULE_LATENCY  1
#define ORC_RULE_SERVICE  2
#define ORC_RULE_ATTR     3   /* span_attribute (spanattribute.go:126-320): the
                                 per-span condition is restated here from the
                                 attr_type / attr_val column attr_col when the
                                 batch carries those columns and attr_col >= 0;
                                 otherwise it is bit (index among the
                                 span_attribute rules, level order) of attr_match */
typedef struct orc_rule {
  int32_t level;        /* 0 global, 1 service, 2 endpoint (rule_engine.go:56-60) */
  int32_t type;         /* ORC_RULE_* */
  uint32_t svc;         /* http_latency / service_name / span_attribute service */
  uint32_t route_len;   /* http_latency http_route */
  const char* route;
  int64_t threshold;    /* http_latency threshold (ms) */
  double ratio;         /* service_name / span_attribute sampling_ratio */
  double fallback;      /* fallback_sampling_ratio */
  /* span_attribute */
  int32_t attr_col;     /* key column of its attribute_key, -1 = from attr_match */
  uint32_t attr_expected_len;
  const char* attr_cond;       /* condition_type */
  const char* attr_op;         /* operation */
  const char* attr_expected;   /* expected_value */
} orc_rule;

/* ---- span_attribute per-span condition (oracle/span_attr.c) -------------- */
typedef struct orc_attr_cond {
  int cond;             /* 0 string, 1 number, 2 boolean */
  char op[32];
  char* expected;
  size_t expected_len;
  orc_re* re;           /* regex: NULL when regexp.Compile fails */
  int num_ok, bool_ok, bool_val;
  double num;
} orc_attr_cond;
int orc_attr_cond_init(orc_attr_cond* a, const char* cond, const char* op, const char* expected, size_t elen);
void orc_attr_cond_free(orc_attr_cond* a);
/* the condition on one span's value (attr_type / attr_val entry), given that
 * the key was found (type != OSE_ATTR_ABSENT) */
int orc_attr_cond_eval(const orc_attr_cond* a, uint8_t type, uint64_t val, const uint8_t* arena);
/* strconv.ParseFloat(s, 64) / strconv.ParseBool: 1 = ok */
int orc_go_parse_float(const char* s, size_t n, double* out);
int orc_go_parse_bool(const char* s, size_t n, int* out);
typedef struct orc_sampling orc_sampling;
orc_sampling* orc_sampling_create(const orc_rule* rules, int n_rules);
void orc_sampling_free(orc_sampling* s);
/* RuleEngine.ShouldSample per trace (rule_engine.go:55-115 and the four
 * Evaluate functions), grouping spans by trace_id in first-appearance order
 * (OSE_GROUP_TRACE_ID) or treating the batch as one trace (OSE_GROUP_BATCH);
 * fills keep, trace_* and trace_count.  rand.Float64() is the injected
 * uniform of include/odigos_amd.h. */
int orc_sampling_process(const orc_sampling* s, const ose_columns* c, ose_outputs* o,
                         uint32_t group_mode, const ose_rand* rnd, int nthreads);
/* the injected uniform for a trace whose first span has trace id {hi, lo} */
double orc_trace_uniform(uint64_t hi, uint64_t lo, uint64_t seed);

/* ---- odigostrafficmetrics -------------------------------------------------- */
/* dataSizesMetricsProcessor.processTraces (odigostrafficmetrics/
 * processor.go:71-84) on the batch as the earlier gateway stages left it:
 * `stages` says which ran (OSE_STAGE_SAMPLE: res->keep / res->trace_keep,
 * OSE_STAGE_TEMPLATE: res->url_out / res->tmpl).  When traffic_u <
 * sampling_ratio (and sampling_ratio != 0) it ADDS ResourceSpansSize(rs) *
 * inverse to o->attrset_bytes[res_attrset[rs]] for every surviving
 * ResourceSpans, writes the sizes to o->res_bytes (0 = removed) and adds
 * the surviving span count to *o->accepted_spans. */
int orc_size_process(const ose_columns* c, const ose_outputs* res, uint32_t stages, uint32_t group_mode,
                     ose_outputs* o, int64_t inverse, double sampling_ratio, double traffic_u);
/* the same with up to ORC_MAX_THREADS pthreads (spans, scopes and resources
 * cut at scope / resource boundaries; per-thread attribute-set sums) */
#define ORC_MAX_THREADS 256
int orc_size_process_mt(const ose_columns* c, const ose_outputs* res, uint32_t stages, uint32_t group_mode,
                        ose_outputs* o, int64_t inverse, double sampling_ratio, double traffic_u, int nthreads);
/* wire size of a Span body after the odigosurltemplate mutation of span i */
uint64_t orc_span_size_after(const ose_columns* c, const ose_outputs* res, uint32_t stages, uint64_t i);

#ifdef __cplusplus
}
#endif
#endif
