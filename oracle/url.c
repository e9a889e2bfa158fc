/*
 * url.c — CPU restatement of odigosurltemplateprocessor.  TEST INFRASTRUCTURE
 * (see oracle.h): the checker for the HIP templater and the timed CPU
 * baseline, never part of the product.
 *
 * Restates (paths under collector/processors/odigosurltemplateprocessor/):
 *   processor.go:27-69    newUrlTemplateProcessor (rule grouping, custom ids)
 *   processor.go:71-96    processTraces (include/exclude: res_url_ok column)
 *   processor.go:149-186  applyTemplatizationOnPath
 *   processor.go:188-212  calculateTemplatedUrlFromAttr (path source column)
 *   processor.go:214-287  updateHttpSpanName, enhanceSpan, processSpan
 *   templatize.go:10-74   built-in regexps, as hand-written byte matchers
 *   templatize.go:97-237  rule parsing and attemptTemplateWithRule
 *   templatize.go:242-290 getSegmentTemplatizationString, defaultTemplatizeURLPath
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

/* ---------------- built-in regexps (templatize.go:10-74) ----------------
 * Go regexp runs on runes; every class below is ASCII-only, so a byte >= 0x80
 * (part of a multi-byte rune or an invalid byte read as U+FFFD) never matches
 * them, and counting bytes equals counting runes for anything they accept. */

static int is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
static int is_hex(uint8_t c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
static int is_alpha(uint8_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

/* noLettersRegex `^[\d_\-!@#$%^&*()=+{}\[\]:;"'<>,.?/\\|`~]+$` (:14) */
static int is_noletter(uint8_t c) {
  if (is_digit(c)) return 1;
  switch (c) {
    case '_': case '-': case '!': case '@': case '#': case '$': case '%': case '^':
    case '&': case '*': case '(': case ')': case '=': case '+': case '{': case '}':
    case '[': case ']': case ':': case ';': case '"': case '\'': case '<': case '>':
    case ',': case '.': case '?': case '/': case '\\': case '|': case '`': case '~':
      return 1;
  }
  return 0;
}
static int re_noletters(const uint8_t* s, size_t n) {
  if (n == 0) return 0;
  for (size_t i = 0; i < n; i++) if (!is_noletter(s[i])) return 0;
  return 1;
}

/* longNumberAnywhereRegex `\d{7,}` (:48) */
static int re_longnumber(const uint8_t* s, size_t n) {
  size_t run = 0;
  for (size_t i = 0; i < n; i++) {
    run = is_digit(s[i]) ? run + 1 : 0;
    if (run >= 7) return 1;
  }
  return 0;
}

/* one 8-4-4-4-12 hex UUID at s[0..36) */
static int uuid_at(const uint8_t* s) {
  for (int i = 0; i < 36; i++) {
    if (i == 8 || i == 13 || i == 18 || i == 23) { if (s[i] != '-') return 0; }
    else if (!is_hex(s[i])) return 0;
  }
  return 1;
}
/* uuidRegex `(^UUID)|(UUID$)` (:22) */
static int re_uuid(const uint8_t* s, size_t n) {
  if (n < 36) return 0;
  return uuid_at(s) || uuid_at(s + n - 36);
}

/* hexEncodedRegex `^(?:[0-9a-fA-F]{2}){8,}$` (:43) */
static int re_hexencoded(const uint8_t* s, size_t n) {
  if (n < 16 || (n & 1)) return 0;
  for (size_t i = 0; i < n; i++) if (!is_hex(s[i])) return 0;
  return 1;
}

/* datesRegex `^\d{4}-\d{2}-\d{2}(?:T\d{2}:\d{2}(?::\d{2})?)?(?:Z|[+-]\d{4})?$` (:67)
 * Each optional group starts with a byte ('T', ':', 'Z', '+', '-') that
 * nothing after it may start with, so the greedy parse below is the only one
 * that can succeed. */
static int digits(const uint8_t* s, size_t k) {
  for (size_t i = 0; i < k; i++) if (!is_digit(s[i])) return 0;
  return 1;
}
static int re_date(const uint8_t* s, size_t n) {
  if (n < 10) return 0;
  if (!digits(s, 4) || s[4] != '-' || !digits(s + 5, 2) || s[7] != '-' || !digits(s + 8, 2)) return 0;
  size_t p = 10;
  if (p < n && s[p] == 'T') {
    if (p + 6 > n || !digits(s + p + 1, 2) || s[p + 3] != ':' || !digits(s + p + 4, 2)) return 0;
    p += 6;
    if (p < n && s[p] == ':') {
      if (p + 3 > n || !digits(s + p + 1, 2)) return 0;
      p += 3;
    }
  }
  if (p < n && s[p] == 'Z') p += 1;
  else if (p < n && (s[p] == '+' || s[p] == '-')) {
    if (p + 5 > n || !digits(s + p + 1, 4)) return 0;
    p += 5;
  }
  return p == n;
}

/* emailRegex `^[a-zA-Z0-9._%+-]+@[a-zA-Z0-9.-]+\.[a-zA-Z]{2,}$` (:70)
 * Neither class contains '@', so there is exactly one '@'.  The domain part
 * must split as X '.' Y with |X| >= 1 and Y >= 2 letters: Y has no '.', so the
 * split is at the last '.'. */
static int is_email_local(uint8_t c) {
  return is_alpha(c) || is_digit(c) || c == '.' || c == '_' || c == '%' || c == '+' || c == '-';
}
static int is_email_domain(uint8_t c) { return is_alpha(c) || is_digit(c) || c == '.' || c == '-'; }
static int re_email(const uint8_t* s, size_t n) {
  size_t at = 0;
  while (at < n && s[at] != '@') { if (!is_email_local(s[at])) return 0; at++; }
  if (at == 0 || at >= n) return 0;
  const uint8_t* d = s + at + 1;
  size_t dn = n - at - 1;
  long lastdot = -1;
  for (size_t i = 0; i < dn; i++) {
    if (!is_email_domain(d[i])) return 0;
    if (d[i] == '.') lastdot = (long)i;
  }
  if (lastdot < 1) return 0;
  size_t tail = dn - (size_t)lastdot - 1;
  if (tail < 2) return 0;
  for (size_t i = (size_t)lastdot + 1; i < dn; i++) if (!is_alpha(d[i])) return 0;
  return 1;
}

/* replacementChar `�` (:73): Go decodes invalid UTF-8 as U+FFFD (width
 * 1) and regexp/syntax keeps RuneError out of literal prefixes, so the regexp
 * matches a valid EF BF BD or any byte where utf8.DecodeRune fails. */
static int re_replacement(const uint8_t* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    int need; uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return 1;
    if (i + (size_t)need >= n) return 1;       /* truncated sequence */
    for (int k = 1; k <= need; k++) {
      uint8_t b = s[i + k];
      uint8_t l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
      if (b < l || b > h) return 1;
    }
    if (need == 2 && c == 0xEF && s[i + 1] == 0xBF && s[i + 2] == 0xBD) return 1;
    i += (size_t)need + 1;
  }
  return 0;
}

/* ---------------- processor state ---------------- */
enum { SEG_STATIC = 0, SEG_WILDCARD = 1, SEG_TEMPLATE = 2, SEG_REGEX = 3 };
typedef struct {
  int kind;
  char* text;        /* static string or template name */
  size_t textlen;
  orc_re* re;        /* template regexp or regex: segment; may be NULL */
} rule_seg;
typedef struct { int nseg; rule_seg* segs; } rule_t;
typedef struct { orc_re* re; char* name; } custom_t;

struct orc_url {
  rule_t* rules; int nrules;   /* in config order */
  custom_t* custom; int ncustom;
};

static char* dupn(const char* s, size_t n) {
  char* d = (char*)malloc(n + 1);
  memcpy(d, s, n); d[n] = 0; return d;
}
static void trim(const char** s, size_t* n) {   /* strings.TrimSpace (ASCII + common unicode not needed here) */
  while (*n && (**s == ' ' || **s == '\t' || **s == '\n' || **s == '\r' || **s == '\v' || **s == '\f')) { (*s)++; (*n)--; }
  while (*n && ((*s)[*n - 1] == ' ' || (*s)[*n - 1] == '\t' || (*s)[*n - 1] == '\n' || (*s)[*n - 1] == '\r' || (*s)[*n - 1] == '\v' || (*s)[*n - 1] == '\f')) (*n)--;
}

static orc_re* compile_n(const char* s, size_t n, char* err, size_t errcap) {
  char* z = dupn(s, n);
  orc_re* re = orc_re_compile(z, err, errcap);
  free(z);
  return re;
}

/* parseUserInputRuleString (templatize.go:140-190) with
 * parseRuleTemplateString (:97-123) and parseRegexPattern (:127-138). */
static int parse_rule(const char* rule, rule_t* out, char* err, size_t errcap) {
  size_t n = strlen(rule);
  const char* p = rule;
  size_t start = 0;
  if (n > 0 && rule[0] == '/') start = 1;
  /* strings.Split(rule, "/") then drop the first element if rule starts with "/" */
  int nseg = 1;
  for (size_t i = 0; i < n; i++) if (rule[i] == '/') nseg++;
  if (start) nseg--;
  out->nseg = nseg;
  out->segs = (rule_seg*)calloc((size_t)(nseg > 0 ? nseg : 1), sizeof(rule_seg));
  size_t pos = start;
  for (int si = 0; si < nseg; si++) {
    size_t e = pos;
    while (e < n && p[e] != '/') e++;
    const char* seg = p + pos;
    size_t sl = e - pos;
    rule_seg* rs = &out->segs[si];
    if (sl == 1 && seg[0] == '*') {
      rs->kind = SEG_WILDCARD;
    } else if (sl >= 2 && seg[0] == '{' && seg[sl - 1] == '}') {
      const char* body = seg + 1;
      size_t bl = sl - 2;
      const char* colon = memchr(body, ':', bl);
      const char* name = body;
      size_t nl = colon ? (size_t)(colon - body) : bl;
      trim(&name, &nl);
      rs->kind = SEG_TEMPLATE;
      if (nl == 0) { rs->text = dupn("id", 2); rs->textlen = 2; }
      else { rs->text = dupn(name, nl); rs->textlen = nl; }
      if (colon) {
        const char* rx = colon + 1;
        size_t rl = (size_t)(body + bl - rx);
        trim(&rx, &rl);
        if (rl == 0) { snprintf(err, errcap, "invalid rule template string. regexp is empty"); return -1; }
        char e2[256] = {0};
        rs->re = compile_n(rx, rl, e2, sizeof e2);
        if (!rs->re) { snprintf(err, errcap, "invalid rule template string. regexp is invalid: %s", e2); return -1; }
      }
    } else if (sl > 6 && memcmp(seg, "regex:", 6) == 0) {
      char e2[256] = {0};
      rs->kind = SEG_REGEX;
      rs->re = compile_n(seg + 6, sl - 6, e2, sizeof e2);
      if (!rs->re) { snprintf(err, errcap, "invalid regexp pattern: %s", e2); return -1; }
    } else {
      rs->kind = SEG_STATIC;
      rs->text = dupn(seg, sl);
      rs->textlen = sl;
    }
    pos = e + 1;
  }
  return 0;
}

void orc_url_free(orc_url* u) {
  if (!u) return;
  for (int i = 0; i < u->nrules; i++) {
    for (int k = 0; k < u->rules[i].nseg; k++) { free(u->rules[i].segs[k].text); orc_re_free(u->rules[i].segs[k].re); }
    free(u->rules[i].segs);
  }
  free(u->rules);
  for (int i = 0; i < u->ncustom; i++) { orc_re_free(u->custom[i].re); free(u->custom[i].name); }
  free(u->custom);
  free(u);
}

orc_url* orc_url_create(const char* const* rules, int n_rules,
                        const char* const* custom_regexps,
                        const char* const* custom_names, int n_custom,
                        char* err, size_t errcap) {
  if (err && errcap) err[0] = 0;
  orc_url* u = (orc_url*)calloc(1, sizeof(orc_url));
  u->rules = (rule_t*)calloc((size_t)(n_rules > 0 ? n_rules : 1), sizeof(rule_t));
  for (int i = 0; i < n_rules; i++) {
    u->nrules = i + 1;
    if (parse_rule(rules[i], &u->rules[i], err, errcap) != 0) { orc_url_free(u); return NULL; }
  }
  u->custom = (custom_t*)calloc((size_t)(n_custom > 0 ? n_custom : 1), sizeof(custom_t));
  for (int i = 0; i < n_custom; i++) {
    char e2[256] = {0};
    u->custom[i].re = orc_re_compile(custom_regexps[i], e2, sizeof e2);
    u->ncustom = i + 1;
    if (!u->custom[i].re) { snprintf(err, errcap, "invalid custom id regex: %s", e2); orc_url_free(u); return NULL; }
    const char* nm = custom_names && custom_names[i] && custom_names[i][0] ? custom_names[i] : "id";
    u->custom[i].name = dupn(nm, strlen(nm));
  }
  return u;
}

/* getSegmentTemplatizationString (templatize.go:242-269) */
int orc_url_segment_name(const orc_url* u, const uint8_t* s, size_t n, char* out) {
  for (int i = 0; i < u->ncustom; i++) {
    if (orc_re_match(u->custom[i].re, s, n)) {
      size_t l = strlen(u->custom[i].name);
      memcpy(out, u->custom[i].name, l);
      return (int)l;
    }
  }
  if (re_date(s, n)) { memcpy(out, "date", 4); return 4; }
  if (re_email(s, n)) { memcpy(out, "email", 5); return 5; }
  if (re_noletters(s, n) || re_longnumber(s, n) || re_uuid(s, n) || re_hexencoded(s, n) || re_replacement(s, n)) {
    memcpy(out, "id", 2);
    return 2;
  }
  return -1;
}

typedef struct { uint8_t* p; size_t n, cap; int overflow; } sbuf;
static void put(sbuf* b, const void* s, size_t n) {
  if (b->n + n > b->cap) { b->overflow = 1; return; }
  memcpy(b->p + b->n, s, n); b->n += n;
}

/* attemptTemplateWithRule (templatize.go:192-237) */
static int attempt_rule(const rule_t* r, const uint8_t* const* seg, const size_t* segl, sbuf* out) {
  for (int i = 0; i < r->nseg; i++) {
    const rule_seg* rs = &r->segs[i];
    if (rs->kind == SEG_WILDCARD) continue;
    if (rs->kind == SEG_STATIC && rs->textlen != 0 &&
        (rs->textlen != segl[i] || memcmp(rs->text, seg[i], segl[i]) != 0)) return 0;
    if (rs->re && !orc_re_match(rs->re, seg[i], segl[i])) return 0;
  }
  for (int i = 0; i < r->nseg; i++) {
    const rule_seg* rs = &r->segs[i];
    if (i > 0) put(out, "/", 1);
    if (rs->kind == SEG_TEMPLATE) { put(out, "{", 1); put(out, rs->text, rs->textlen); put(out, "}", 1); }
    else if (rs->kind == SEG_WILDCARD || rs->kind == SEG_REGEX) put(out, seg[i], segl[i]);
    else put(out, rs->text, rs->textlen);
  }
  return 1;
}

/* applyTemplatizationOnPath (processor.go:149-186) */
long orc_url_apply_path(const orc_url* u, const uint8_t* path, size_t n, uint8_t* outp, size_t cap) {
  sbuf out = {outp, 0, cap, 0};
  int lead = n > 0 && path[0] == '/';
  /* path = "/" + path when no leading slash; segments = Split(path, "/")[1:] */
  const uint8_t* body = lead ? path + 1 : path;
  size_t bn = lead ? n - 1 : n;
  size_t nseg = 1;
  for (size_t i = 0; i < bn; i++) if (body[i] == '/') nseg++;
  if (nseg == 1 && bn == 0) { put(&out, "/", 1); return out.overflow ? -1 : (long)out.n; }
  const uint8_t** seg = (const uint8_t**)malloc(sizeof(*seg) * nseg);
  size_t* segl = (size_t*)malloc(sizeof(*segl) * nseg);
  size_t k = 0, st = 0;
  for (size_t i = 0; i <= bn; i++) {
    if (i == bn || body[i] == '/') { seg[k] = body + st; segl[k] = i - st; k++; st = i + 1; }
  }
  for (int r = 0; r < u->nrules; r++) {
    if ((size_t)u->rules[r].nseg != nseg) continue;
    size_t mark = out.n;
    if (lead) put(&out, "/", 1);
    if (attempt_rule(&u->rules[r], seg, segl, &out)) goto done;
    out.n = mark;
  }
  {
    /* defaultTemplatizeURLPath (templatize.go:272-290) */
    int templated = 0;
    char name[256];
    if (lead) put(&out, "/", 1);
    for (size_t i = 0; i < nseg; i++) {
      if (i > 0) put(&out, "/", 1);
      int nl = orc_url_segment_name(u, seg[i], segl[i], name);
      if (nl >= 0) { put(&out, "{", 1); put(&out, name, (size_t)nl); put(&out, "}", 1); templated = 1; }
      else put(&out, seg[i], segl[i]);
    }
    if (!templated) {
      /* returns the (slash-prefixed) original path */
      out.n = 0;
      put(&out, "/", 1);
      put(&out, body, bn);
    }
  }
done:
  free(seg); free(segl);
  return out.overflow ? -1 : (long)out.n;
}

/* processSpan/enhanceSpan/updateHttpSpanName (processor.go:214-287) for one
 * span; returns url_out flags and writes the template into out. */
static uint8_t process_span(const orc_url* u, const ose_columns* c, uint64_t i, sbuf* out, uint32_t* tlen) {
  *tlen = 0;
  if (c->res_url_ok && !c->res_url_ok[c->resource[i]]) return 0;       /* processor.go:76-85 */
  uint8_t f = c->url_flags[i];
  if (!(f & OSE_URL_HAS_METHOD)) return 0;                              /* :266-270 */
  uint8_t kind = c->kind[i];
  if (kind != OSE_KIND_SERVER && kind != OSE_KIND_CLIENT) return 0;     /* :272-285 */
  uint8_t tgt = f & OSE_URL_TGT_MASK;
  if (tgt != OSE_URL_TGT_ABSENT) {                                      /* :239-251 */
    if (tgt == OSE_URL_TGT_STR_EMPTY && (f & OSE_URL_NAME_EQ_METHOD)) {
      size_t m = out->n;
      put(out, "/", 1);
      *tlen = (uint32_t)(out->n - m);
      return OSE_OUT_RENAME;
    }
    return 0;
  }
  uint8_t src = f & OSE_URL_PATH_MASK;
  if (src == OSE_URL_PATH_NONE) return 0;                               /* :253-256 */
  const uint8_t* p = c->arena + c->path[i].off;
  size_t n = c->path[i].len;
  if (src == OSE_URL_PATH_TARGET) {                                     /* :124-129 */
    const uint8_t* q = memchr(p, '?', n);
    if (q) n = (size_t)(q - p);
  }
  size_t m = out->n;
  long l = orc_url_apply_path(u, p, n, out->p + out->n, out->cap - out->n);
  if (l < 0) { out->overflow = 1; return 0; }
  out->n += (size_t)l;
  *tlen = (uint32_t)(out->n - m);
  uint8_t r = OSE_OUT_SET_ATTR;                                        /* :259-261 */
  if ((f & OSE_URL_NAME_EQ_METHOD) && l > 0) r |= OSE_OUT_RENAME;       /* :216-225 */
  return r;
}

typedef struct {
  const orc_url* u; const ose_columns* c; ose_outputs* o;
  uint64_t lo, hi;
  uint8_t* buf; size_t cap, used; int overflow;
} job_t;

static void* run_chunk(void* arg) {
  job_t* j = (job_t*)arg;
  sbuf out = {j->buf, 0, j->cap, 0};
  for (uint64_t i = j->lo; i < j->hi; i++) {
    uint32_t tl;
    size_t start = out.n;
    uint8_t r = process_span(j->u, j->c, i, &out, &tl);
    j->o->url_out[i] = r;
    j->o->tmpl[i].off = (uint32_t)start;   /* chunk-relative; rebased below */
    j->o->tmpl[i].len = r ? tl : 0;
    if (out.overflow) break;
  }
  j->used = out.n; j->overflow = out.overflow;
  return NULL;
}

int orc_url_process(const orc_url* u, const ose_columns* c, ose_outputs* o, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  uint64_t n = c->n_spans;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job_t* j = &jobs[t];
    j->u = u; j->c = c; j->o = o;
    j->lo = n * (uint64_t)t / (uint64_t)nthreads;
    j->hi = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
    uint64_t in_bytes = 0;
    for (uint64_t i = j->lo; i < j->hi; i++) in_bytes += c->path ? c->path[i].len : 0;
    /* generous private capacity; rebased into the shared arena afterwards */
    j->cap = (size_t)(in_bytes * 2 + (j->hi - j->lo) * 64 + 4096);
    j->buf = (uint8_t*)malloc(j->cap);
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, run_chunk, &jobs[t]);
  run_chunk(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  int rc = 0;
  uint64_t base = 0;
  for (int t = 0; t < nthreads; t++) {
    job_t* j = &jobs[t];
    if (j->overflow || base + j->used > o->tmpl_arena_cap) { rc = -1; }
    else {
      memcpy(o->tmpl_arena + base, j->buf, j->used);
      for (uint64_t i = j->lo; i < j->hi; i++) o->tmpl[i].off += (uint32_t)base;
      base += j->used;
    }
    free(j->buf);
  }
  if (o->tmpl_arena_used) *o->tmpl_arena_used = base;
  free(jobs); free(th);
  return rc;
}
