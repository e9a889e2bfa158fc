/*
 * regex.c — oracle-private restatement of Go regexp.MatchString for the
 * RE2 syntax subset used by odigosurltemplate (custom_ids, templatization
 * rule regexps; templatize.go:97-138, processor.go:45-60) and by the
 * span_attribute "regex" operation (spanattribute.go:170-177).
 * TEST INFRASTRUCTURE (see oracle.h).
 *
 * Third-party algorithm restated: Go stdlib regexp + regexp/syntax (go 1.25,
 * collector go.mod): Perl flags (ClassNL|OneLine|PerlX|UnicodeGroups), UTF-8
 * decoding with invalid bytes read as U+FFFD width 1, EmptyOpContext for
 * ^ $ \A \z \b \B, ASCII-only \d \s \w and [[:class:]].
 *
 * Algorithm (deliberately different from the product's DFA compiler):
 * parse -> instruction program -> backtracking with a visited bitmap
 * (RE2 "BitState"), tried from every rune boundary.
 * \p{..} / \P{..} (Go 1.25 names, loose matching) and (?i) on any rune
 * use the oracle's own generated Unicode data (unicode_data.c: Unicode
 * 13.0.0 categories; Go 1.25 uses 15.0.0, so later code points are parity
 * unpinned); \Q..\E quotes literals.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define RUNE_MAX 0x10FFFF
#define RUNE_ERR 0xFFFD

/* ---------- UTF-8 (Go unicode/utf8 DecodeRune semantics) ---------- */
static int decode_rune(const uint8_t* s, size_t n, int* width) {
  uint8_t c = s[0];
  if (c < 0x80) { *width = 1; return c; }
  int need; int r; uint8_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { need = 1; r = c & 0x1F; }
  else if (c == 0xE0) { need = 2; r = c & 0x0F; lo = 0xA0; }
  else if (c >= 0xE1 && c <= 0xEC) { need = 2; r = c & 0x0F; }
  else if (c == 0xED) { need = 2; r = c & 0x0F; hi = 0x9F; }
  else if (c >= 0xEE && c <= 0xEF) { need = 2; r = c & 0x0F; }
  else if (c == 0xF0) { need = 3; r = c & 0x07; lo = 0x90; }
  else if (c >= 0xF1 && c <= 0xF3) { need = 3; r = c & 0x07; }
  else if (c == 0xF4) { need = 3; r = c & 0x07; hi = 0x8F; }
  else { *width = 1; return RUNE_ERR; }
  if ((size_t)need >= n) { *width = 1; return RUNE_ERR; }
  for (int i = 1; i <= need; i++) {
    uint8_t b = s[i];
    uint8_t l = (i == 1) ? lo : 0x80, h = (i == 1) ? hi : 0xBF;
    if (b < l || b > h) { *width = 1; return RUNE_ERR; }
    r = (r << 6) | (b & 0x3F);
  }
  *width = need + 1;
  return r;
}

/* ---------- program ---------- */
enum { I_RUNE, I_ANY, I_ANYNL, I_SPLIT, I_JMP, I_EMPTY, I_MATCH, I_NOP };
enum { E_BOL = 1, E_EOL = 2, E_BOT = 4, E_EOT = 8, E_WB = 16, E_NWB = 32 };

typedef struct { int lo, hi; } rng;
typedef struct {
  int op;
  int x, y;           /* SPLIT targets; JMP x; next = x for RUNE/EMPTY */
  int empty;          /* I_EMPTY condition */
  int cls;            /* I_RUNE: class index */
} inst;
typedef struct { rng* r; int n, cap; } rclass;   /* sorted, merged ranges (fold applied) */

struct orc_re {
  inst* prog; int nprog, capprog;
  rclass* cls; int ncls, capcls;
  int start;
};

/* ---------- AST ---------- */
enum { N_EMPTY, N_LIT, N_CLASS, N_ANY, N_ANYNL, N_ASSERT, N_CAT, N_ALT, N_REP };
typedef struct node node;
struct node {
  int type;
  int cls;        /* N_LIT/N_CLASS: class index in re->cls */
  int assert_op;
  node** kids; int nkids, capkids;
  int min, max;   /* N_REP; max -1 = unbounded */
};

typedef struct {
  const char* p; const char* end;
  orc_re* re;
  char* err; size_t errcap;
  int flag_i, flag_m, flag_s;
  int depth;
  int unsupported;
} parser;

static void set_err(parser* ps, const char* msg) {
  if (ps->err && ps->err[0] == 0) snprintf(ps->err, ps->errcap, "%s", msg);
}

static node* mk(int type) {
  node* n = (node*)calloc(1, sizeof(node));
  n->type = type; n->cls = -1;
  return n;
}
static void addkid(node* n, node* k) {
  if (n->nkids == n->capkids) {
    n->capkids = n->capkids ? n->capkids * 2 : 4;
    n->kids = (node**)realloc(n->kids, sizeof(node*) * n->capkids);
  }
  n->kids[n->nkids++] = k;
}
static void free_node(node* n) {
  if (!n) return;
  for (int i = 0; i < n->nkids; i++) free_node(n->kids[i]);
  free(n->kids); free(n);
}

/* ---------- classes ---------- */
static int new_class(orc_re* re) {
  if (re->ncls == re->capcls) {
    re->capcls = re->capcls ? re->capcls * 2 : 8;
    re->cls = (rclass*)realloc(re->cls, sizeof(rclass) * re->capcls);
  }
  memset(&re->cls[re->ncls], 0, sizeof(rclass));
  return re->ncls++;
}
static void cls_add(rclass* c, int lo, int hi) {
  if (c->n == c->cap) { c->cap = c->cap ? c->cap * 2 : 8; c->r = (rng*)realloc(c->r, sizeof(rng) * c->cap); }
  c->r[c->n].lo = lo; c->r[c->n].hi = hi; c->n++;
}
static int rng_cmp(const void* a, const void* b) {
  const rng* x = (const rng*)a; const rng* y = (const rng*)b;
  return x->lo != y->lo ? (x->lo < y->lo ? -1 : 1) : (x->hi < y->hi ? -1 : x->hi > y->hi);
}
static void cls_norm(rclass* c) {
  if (c->n == 0) return;
  qsort(c->r, c->n, sizeof(rng), rng_cmp);
  int w = 0;
  for (int i = 1; i < c->n; i++) {
    if (c->r[i].lo <= c->r[w].hi + 1) { if (c->r[i].hi > c->r[w].hi) c->r[w].hi = c->r[i].hi; }
    else c->r[++w] = c->r[i];
  }
  c->n = w + 1;
}
static void cls_negate(rclass* c) {
  cls_norm(c);
  rclass o = {0, 0, 0};
  int next = 0;
  for (int i = 0; i < c->n; i++) {
    if (c->r[i].lo > next) cls_add(&o, next, c->r[i].lo - 1);
    next = c->r[i].hi + 1;
  }
  if (next <= RUNE_MAX) cls_add(&o, next, RUNE_MAX);
  free(c->r); *c = o;
}
static int cls_has(const rclass* c, int r);
static int peek_rune(parser* ps, int* w);
/* unicode.SimpleFold closure: every member brings its whole orbit
 * (orc_fold_next lists each orbit as a cycle; repeated passes close it). */
static void cls_fold(rclass* c) {
  cls_norm(c);
  for (int pass = 0; pass < 8; pass++) {
    int added = 0;
    for (int k = 0; k < orc_fold_n; k++) {
      int r = orc_fold_next[2 * k], nx = orc_fold_next[2 * k + 1];
      if (cls_has(c, r) && !cls_has(c, nx)) { cls_add(c, nx, nx); added = 1; }
    }
    if (!added) break;
    cls_norm(c);
  }
}
static int cls_has(const rclass* c, int r) {
  int lo = 0, hi = c->n - 1;
  while (lo <= hi) {
    int m = (lo + hi) / 2;
    if (r < c->r[m].lo) hi = m - 1; else if (r > c->r[m].hi) lo = m + 1; else return 1;
  }
  return 0;
}

static void add_perl(rclass* c, char k) {
  switch (k) {
    case 'd': cls_add(c, '0', '9'); break;
    case 's': cls_add(c, '\t', '\n'); cls_add(c, '\f', '\r'); cls_add(c, ' ', ' '); break;
    case 'w': cls_add(c, '0', '9'); cls_add(c, 'A', 'Z'); cls_add(c, '_', '_'); cls_add(c, 'a', 'z'); break;
  }
}
/* regexp/syntax appendGroup: under (?i) a negated group is folded first,
 * then negated (so (?i)[\W] excludes U+212A and U+017F) */
static void add_perl_neg(rclass* c, char k, int fold) {
  rclass t = {0, 0, 0};
  add_perl(&t, k);
  if (fold) cls_fold(&t);
  cls_negate(&t);
  for (int i = 0; i < t.n; i++) cls_add(c, t.r[i].lo, t.r[i].hi);
  free(t.r);
}

/* Go 1.25 regexp/syntax unicodeTable: names compared loosely (case, ' ',
 * '_' and '-' ignored); Any, ASCII, Assigned, Cn, LC, one-letter groups,
 * two-letter categories with their long aliases, scripts. */
static void loose_name(const char* s, size_t n, char* out, size_t cap) {
  size_t k = 0;
  for (size_t i = 0; i < n && k + 1 < cap; i++) {
    char c = s[i];
    if (c == ' ' || c == '_' || c == '-') continue;
    out[k++] = (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c;
  }
  out[k] = 0;
}
static void add_tab(rclass* t, const orc_utab* u) {
  for (int i = 0; i < u->n; i++) cls_add(t, u->r[2 * i], u->r[2 * i + 1]);
}
static int unicode_named(rclass* t, const char* name, size_t len) {
  static const char* const alias[][2] = {
    {"letter", "l"}, {"casedletter", "lc"}, {"uppercaseletter", "lu"}, {"lowercaseletter", "ll"},
    {"titlecaseletter", "lt"}, {"modifierletter", "lm"}, {"otherletter", "lo"}, {"mark", "m"},
    {"combiningmark", "m"}, {"nonspacingmark", "mn"}, {"spacingmark", "mc"}, {"enclosingmark", "me"},
    {"number", "n"}, {"decimalnumber", "nd"}, {"digit", "nd"}, {"letternumber", "nl"}, {"othernumber", "no"},
    {"punctuation", "p"}, {"punct", "p"}, {"connectorpunctuation", "pc"}, {"dashpunctuation", "pd"},
    {"openpunctuation", "ps"}, {"closepunctuation", "pe"}, {"initialpunctuation", "pi"},
    {"finalpunctuation", "pf"}, {"otherpunctuation", "po"}, {"symbol", "s"}, {"mathsymbol", "sm"},
    {"currencysymbol", "sc"}, {"modifiersymbol", "sk"}, {"othersymbol", "so"}, {"separator", "z"},
    {"spaceseparator", "zs"}, {"lineseparator", "zl"}, {"paragraphseparator", "zp"}, {"other", "c"},
    {"control", "cc"}, {"cntrl", "cc"}, {"format", "cf"}, {"surrogate", "cs"}, {"privateuse", "co"},
    {"unassigned", "cn"}};
  char key[64], nm[64];
  loose_name(name, len, key, sizeof key);
  for (size_t i = 0; i < sizeof alias / sizeof alias[0]; i++)
    if (strcmp(key, alias[i][0]) == 0) { snprintf(key, sizeof key, "%s", alias[i][1]); break; }
  if (strcmp(key, "any") == 0) { cls_add(t, 0, RUNE_MAX); return 1; }
  if (strcmp(key, "ascii") == 0) { cls_add(t, 0, 0x7F); return 1; }
  if (strcmp(key, "assigned") == 0 || strcmp(key, "cn") == 0) {
    rclass a = {0, 0, 0};
    for (int i = 0; i < orc_ucats_n; i++) add_tab(&a, &orc_ucats[i]);
    if (key[0] == 'c') cls_negate(&a);
    for (int i = 0; i < a.n; i++) cls_add(t, a.r[i].lo, a.r[i].hi);
    free(a.r);
    return 1;
  }
  int hit = 0;
  for (int i = 0; i < orc_ucats_n; i++) {
    loose_name(orc_ucats[i].name, strlen(orc_ucats[i].name), nm, sizeof nm);
    int in = strcmp(nm, key) == 0 || (key[0] && !key[1] && nm[0] == key[0]) ||
             (strcmp(key, "lc") == 0 && (!strcmp(nm, "lu") || !strcmp(nm, "ll") || !strcmp(nm, "lt")));
    if (in) { add_tab(t, &orc_ucats[i]); hit = 1; }
  }
  if (hit) return 1;
  for (int i = 0; i < orc_uscripts_n; i++) {
    loose_name(orc_uscripts[i].name, strlen(orc_uscripts[i].name), nm, sizeof nm);
    if (strcmp(nm, key) == 0) { add_tab(t, &orc_uscripts[i]); return 1; }
  }
  return 0;
}
/* \p / \P after the letter: the (folded under (?i), then signed) set into
 * out; -1 on a bad name (regexp/syntax parseUnicodeClass) */
static int parse_uclass(parser* ps, int upper, rclass* out) {
  int neg = upper;
  const char* nm; size_t len;
  if (ps->p >= ps->end) { set_err(ps, "invalid character class range"); return -1; }
  if (*ps->p == '{') {
    const char* e = memchr(ps->p, '}', (size_t)(ps->end - ps->p));
    if (!e) { set_err(ps, "invalid character class range"); return -1; }
    nm = ps->p + 1; len = (size_t)(e - nm);
    ps->p = e + 1;
  } else {
    int w; peek_rune(ps, &w);
    nm = ps->p; len = (size_t)w;
    ps->p += w;
  }
  if (len && nm[0] == '^') { neg = !neg; nm++; len--; }
  rclass t = {0, 0, 0};
  if (!unicode_named(&t, nm, len)) { free(t.r); set_err(ps, "invalid character class range"); return -1; }
  cls_norm(&t);
  if (ps->flag_i) cls_fold(&t);
  if (neg) cls_negate(&t);
  *out = t;
  return 0;
}

static int posix_class(rclass* c, const char* name, size_t len, int neg) {
  rclass t = {0, 0, 0};
#define IS(s) (len == sizeof(s) - 1 && memcmp(name, s, len) == 0)
  if (IS("alnum")) { cls_add(&t, '0', '9'); cls_add(&t, 'A', 'Z'); cls_add(&t, 'a', 'z'); }
  else if (IS("alpha")) { cls_add(&t, 'A', 'Z'); cls_add(&t, 'a', 'z'); }
  else if (IS("ascii")) { cls_add(&t, 0, 0x7F); }
  else if (IS("blank")) { cls_add(&t, '\t', '\t'); cls_add(&t, ' ', ' '); }
  else if (IS("cntrl")) { cls_add(&t, 0, 0x1F); cls_add(&t, 0x7F, 0x7F); }
  else if (IS("digit")) { cls_add(&t, '0', '9'); }
  else if (IS("graph")) { cls_add(&t, '!', '~'); }
  else if (IS("lower")) { cls_add(&t, 'a', 'z'); }
  else if (IS("print")) { cls_add(&t, ' ', '~'); }
  else if (IS("punct")) { cls_add(&t, '!', '/'); cls_add(&t, ':', '@'); cls_add(&t, '[', '`'); cls_add(&t, '{', '~'); }
  else if (IS("space")) { cls_add(&t, '\t', '\r'); cls_add(&t, ' ', ' '); }
  else if (IS("upper")) { cls_add(&t, 'A', 'Z'); }
  else if (IS("word")) { cls_add(&t, '0', '9'); cls_add(&t, 'A', 'Z'); cls_add(&t, 'a', 'z'); cls_add(&t, '_', '_'); }
  else if (IS("xdigit")) { cls_add(&t, '0', '9'); cls_add(&t, 'A', 'F'); cls_add(&t, 'a', 'f'); }
  else { free(t.r); return 0; }
#undef IS
  if (neg) cls_negate(&t);
  for (int i = 0; i < t.n; i++) cls_add(c, t.r[i].lo, t.r[i].hi);
  free(t.r);
  return 1;
}

/* ---------- parser ---------- */
static int peek_rune(parser* ps, int* w) {
  return decode_rune((const uint8_t*)ps->p, (size_t)(ps->end - ps->p), w);
}
static int is_hexd(int c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
static int hexv(int c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }
static int is_alnum_c(int c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

/* Parses one escape after '\'.  Returns rune >= 0, or -2 for a perl class
 * (kind in *perl, negated in *neg), -3 for an empty-width op (*op), -1 on error. */
static int parse_escape(parser* ps, char* perl, int* neg, int* op, int in_class) {
  if (ps->p >= ps->end) { set_err(ps, "trailing backslash at end of expression"); return -1; }
  int w; int c = peek_rune(ps, &w);
  ps->p += w;
  if (c < 0x80 && !is_alnum_c(c)) return c;
  switch (c) {
    case 'd': case 's': case 'w': *perl = (char)c; *neg = 0; return -2;
    case 'D': case 'S': case 'W': *perl = (char)(c + 32); *neg = 1; return -2;
    case 'a': return 7; case 'f': return 12; case 'n': return 10;
    case 'r': return 13; case 't': return 9; case 'v': return 11;
    case 'b': if (in_class) break; *op = E_WB; return -3;
    case 'B': if (in_class) break; *op = E_NWB; return -3;
    case 'A': if (in_class) break; *op = E_BOT; return -3;
    case 'z': if (in_class) break; *op = E_EOT; return -3;
    case 'p': case 'P': return c == 'P' ? -5 : -4;   /* unicode class: the caller parses the name */
    case 'C': ps->unsupported = 1; set_err(ps, "unsupported escape"); return -1;
    case '1': case '2': case '3': case '4': case '5': case '6': case '7':
      if (ps->p >= ps->end || *ps->p < '0' || *ps->p > '7') break;
      /* fallthrough */
    case '0': {
      int r = c - '0';
      for (int i = 1; i < 3; i++) {
        if (ps->p >= ps->end || *ps->p < '0' || *ps->p > '7') break;
        r = r * 8 + (*ps->p - '0'); ps->p++;
      }
      return r;
    }
    case 'x': {
      if (ps->p >= ps->end) break;
      if (*ps->p == '{') {
        ps->p++;
        int r = 0, nd = 0;
        while (ps->p < ps->end && is_hexd((unsigned char)*ps->p)) { r = r * 16 + hexv((unsigned char)*ps->p); ps->p++; nd++; if (r > RUNE_MAX) break; }
        if (nd == 0 || ps->p >= ps->end || *ps->p != '}' || r > RUNE_MAX) break;
        ps->p++;
        return r;
      }
      if (ps->end - ps->p < 2 || !is_hexd((unsigned char)ps->p[0]) || !is_hexd((unsigned char)ps->p[1])) break;
      int r = hexv((unsigned char)ps->p[0]) * 16 + hexv((unsigned char)ps->p[1]);
      ps->p += 2;
      return r;
    }
    default: break;
  }
  set_err(ps, "invalid escape sequence");
  return -1;
}

static node* class_node(parser* ps, rclass* tmp, int negate) {
  orc_re* re = ps->re;
  int ci = new_class(re);
  rclass* c = &re->cls[ci];
  *c = *tmp;
  cls_norm(c);
  if (ps->flag_i) cls_fold(c);
  if (negate) cls_negate(c);
  node* n = mk(N_CLASS);
  n->cls = ci;
  return n;
}

static node* parse_class(parser* ps) {  /* after '[' */
  rclass t = {0, 0, 0};
  int negate = 0;
  if (ps->p < ps->end && *ps->p == '^') { negate = 1; ps->p++; }
  int first = 1;
  for (;;) {
    if (ps->p >= ps->end) { set_err(ps, "missing closing ]"); free(t.r); return NULL; }
    if (*ps->p == ']' && !first) { ps->p++; break; }
    first = 0;
    if (ps->p + 1 < ps->end && ps->p[0] == '[' && ps->p[1] == ':') {
      const char* q = ps->p + 2;
      int neg = 0;
      if (q < ps->end && *q == '^') { neg = 1; q++; }
      const char* nm = q;
      while (q + 1 < ps->end && !(q[0] == ':' && q[1] == ']')) q++;
      if (q + 1 < ps->end) {
        if (!posix_class(&t, nm, (size_t)(q - nm), neg)) { set_err(ps, "invalid character class range"); free(t.r); return NULL; }
        ps->p = q + 2;
        continue;
      }
    }
    int lo;
    if (*ps->p == '\\') {
      ps->p++;
      char perl = 0; int neg = 0, op = 0;
      lo = parse_escape(ps, &perl, &neg, &op, 1);
      if (lo == -2) { if (neg) add_perl_neg(&t, perl, ps->flag_i); else add_perl(&t, perl); continue; }
      if (lo == -4 || lo == -5) {
        rclass u;
        if (parse_uclass(ps, lo == -5, &u) < 0) { free(t.r); return NULL; }
        for (int i = 0; i < u.n; i++) cls_add(&t, u.r[i].lo, u.r[i].hi);
        free(u.r);
        continue;
      }
      if (lo < 0) { free(t.r); return NULL; }
    } else {
      int w; lo = peek_rune(ps, &w); ps->p += w;
    }
    int hi = lo;
    if (ps->p + 1 < ps->end && *ps->p == '-' && ps->p[1] != ']') {
      ps->p++;
      if (*ps->p == '\\') {
        ps->p++;
        char perl = 0; int neg = 0, op = 0;
        hi = parse_escape(ps, &perl, &neg, &op, 1);
        if (hi < 0) { if (hi == -2) set_err(ps, "invalid character class range"); free(t.r); return NULL; }
      } else {
        int w; hi = peek_rune(ps, &w); ps->p += w;
      }
      if (hi < lo) { set_err(ps, "invalid character class range"); free(t.r); return NULL; }
    }
    cls_add(&t, lo, hi);
  }
  return class_node(ps, &t, negate);
}

static node* parse_alt(parser* ps);

static node* lit_node(parser* ps, int r) {
  rclass t = {0, 0, 0};
  cls_add(&t, r, r);
  node* n = class_node(ps, &t, 0);
  n->type = N_LIT;
  return n;
}

static int parse_int(parser* ps, int* v) {
  const char* s = ps->p;
  if (s >= ps->end || *s < '0' || *s > '9') return 0;
  long x = 0;
  while (s < ps->end && *s >= '0' && *s <= '9') { if (x < 100000) x = x * 10 + (*s - '0'); s++; }
  *v = (int)x; ps->p = s; return 1;
}

/* {n}, {n,}, {n,m}: returns 1 and advances when the text is a repeat op */
static int parse_repeat_braces(parser* ps, int* mn, int* mx) {
  const char* save = ps->p;
  ps->p++;  /* '{' */
  int a, b = -1;
  if (!parse_int(ps, &a)) { ps->p = save; return 0; }
  if (ps->p < ps->end && *ps->p == ',') {
    ps->p++;
    if (ps->p < ps->end && *ps->p == '}') b = -1;
    else if (!parse_int(ps, &b)) { ps->p = save; return 0; }
  } else b = a;
  if (ps->p >= ps->end || *ps->p != '}') { ps->p = save; return 0; }
  ps->p++;
  *mn = a; *mx = b;
  return 1;
}

static node* parse_concat(parser* ps) {
  node* cat = mk(N_CAT);
  int last_was_repeat = 0;
  while (ps->p < ps->end && *ps->p != '|' && *ps->p != ')') {
    char c = *ps->p;
    if (c == '*' || c == '+' || c == '?' || c == '{') {
      int mn, mx;
      const char* opstart = ps->p;
      if (c == '{') {
        if (!parse_repeat_braces(ps, &mn, &mx)) goto literal;
        if (mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx)) { set_err(ps, "invalid repeat count"); free_node(cat); return NULL; }
      } else {
        ps->p++;
        mn = c == '+' ? 1 : 0; mx = c == '?' ? 1 : -1;
      }
      if (ps->p < ps->end && *ps->p == '?') ps->p++;  /* non-greedy: same language */
      if (last_was_repeat) { set_err(ps, "invalid nested repetition operator"); free_node(cat); return NULL; }
      if (cat->nkids == 0) { set_err(ps, "missing argument to repetition operator"); free_node(cat); return NULL; }
      (void)opstart;
      node* r = mk(N_REP);
      r->min = mn; r->max = mx;
      addkid(r, cat->kids[cat->nkids - 1]);
      cat->kids[cat->nkids - 1] = r;
      last_was_repeat = 1;
      continue;
    }
  literal:
    last_was_repeat = 0;
    if (c == '(') {
      ps->p++;
      int save_i = ps->flag_i, save_m = ps->flag_m, save_s = ps->flag_s;
      if (ps->p < ps->end && *ps->p == '?') {
        ps->p++;
        if (ps->p < ps->end && (*ps->p == 'P' || *ps->p == '<')) {
          if (*ps->p == 'P') ps->p++;
          if (ps->p >= ps->end || *ps->p != '<') { set_err(ps, "invalid named capture"); free_node(cat); return NULL; }
          const char* q = ps->p + 1;
          while (q < ps->end && *q != '>') q++;
          if (q >= ps->end || q == ps->p + 1) { set_err(ps, "invalid named capture"); free_node(cat); return NULL; }
          ps->p = q + 1;
        } else {
          int neg = 0, any = 0;
          for (;;) {
            if (ps->p >= ps->end) { set_err(ps, "missing closing )"); free_node(cat); return NULL; }
            char f = *ps->p++;
            if (f == 'i') { ps->flag_i = !neg; any = 1; }
            else if (f == 'm') { ps->flag_m = !neg; any = 1; }
            else if (f == 's') { ps->flag_s = !neg; any = 1; }
            else if (f == 'U') { any = 1; }
            else if (f == '-') { if (neg) { set_err(ps, "invalid or unsupported Perl syntax"); free_node(cat); return NULL; } neg = 1; any = 0; }
            else if (f == ')') {
              if (neg && !any) { set_err(ps, "invalid or unsupported Perl syntax"); free_node(cat); return NULL; }
              goto flags_only;  /* flags persist to end of enclosing group */
            } else if (f == ':') {
              if (neg && !any) { set_err(ps, "invalid or unsupported Perl syntax"); free_node(cat); return NULL; }
              break;
            } else { set_err(ps, "invalid or unsupported Perl syntax"); free_node(cat); return NULL; }
          }
        }
      }
      {
        ps->depth++;
        if (ps->depth > 1000) { set_err(ps, "expression nests too deeply"); free_node(cat); return NULL; }
        node* sub = parse_alt(ps);
        ps->depth--;
        if (!sub) { free_node(cat); return NULL; }
        if (ps->p >= ps->end || *ps->p != ')') { set_err(ps, "missing closing )"); free_node(sub); free_node(cat); return NULL; }
        ps->p++;
        ps->flag_i = save_i; ps->flag_m = save_m; ps->flag_s = save_s;
        addkid(cat, sub);
      }
      continue;
    flags_only:
      continue;
    }
    if (c == '[') { ps->p++; node* n = parse_class(ps); if (!n) { free_node(cat); return NULL; } addkid(cat, n); continue; }
    if (c == '.') { ps->p++; addkid(cat, mk(ps->flag_s ? N_ANY : N_ANYNL)); continue; }
    if (c == '^') { ps->p++; node* n = mk(N_ASSERT); n->assert_op = ps->flag_m ? E_BOL : E_BOT; addkid(cat, n); continue; }
    if (c == '$') { ps->p++; node* n = mk(N_ASSERT); n->assert_op = ps->flag_m ? E_EOL : E_EOT; addkid(cat, n); continue; }
    if (c == '\\' && ps->p + 1 < ps->end && ps->p[1] == 'Q') {   /* \Q...\E: literals up to \E or the end */
      ps->p += 2;
      const char* e = ps->p;
      while (e + 1 < ps->end && !(e[0] == '\\' && e[1] == 'E')) e++;
      if (!(e + 1 < ps->end)) e = ps->end;
      while (ps->p < e) { int w; int r = peek_rune(ps, &w); ps->p += w; addkid(cat, lit_node(ps, r)); }
      if (e < ps->end) ps->p = e + 2;
      continue;
    }
    if (c == '\\') {
      ps->p++;
      char perl = 0; int neg = 0, op = 0;
      int r = parse_escape(ps, &perl, &neg, &op, 0);
      if (r == -1) { free_node(cat); return NULL; }
      if (r == -4 || r == -5) {
        rclass u;
        if (parse_uclass(ps, r == -5, &u) < 0) { free_node(cat); return NULL; }
        int ci = new_class(ps->re);
        ps->re->cls[ci] = u;
        node* n = mk(N_CLASS);
        n->cls = ci;
        addkid(cat, n);
        continue;
      }
      if (r == -2) {
        rclass t = {0, 0, 0};
        add_perl(&t, perl);
        addkid(cat, class_node(ps, &t, neg));
        continue;
      }
      if (r == -3) { node* n = mk(N_ASSERT); n->assert_op = op; addkid(cat, n); continue; }
      addkid(cat, lit_node(ps, r));
      continue;
    }
    {
      int w; int r = peek_rune(ps, &w); ps->p += w;
      addkid(cat, lit_node(ps, r));
    }
  }
  return cat;
}

static node* parse_alt(parser* ps) {
  node* alt = mk(N_ALT);
  for (;;) {
    node* c = parse_concat(ps);
    if (!c) { free_node(alt); return NULL; }
    addkid(alt, c);
    if (ps->p < ps->end && *ps->p == '|') { ps->p++; continue; }
    break;
  }
  return alt;
}

/* ---------- compile AST -> program ---------- */
static int emit(orc_re* re, int op) {
  if (re->nprog == re->capprog) {
    re->capprog = re->capprog ? re->capprog * 2 : 64;
    re->prog = (inst*)realloc(re->prog, sizeof(inst) * re->capprog);
  }
  inst* i = &re->prog[re->nprog];
  memset(i, 0, sizeof(*i));
  i->op = op; i->x = i->y = -1; i->cls = -1;
  return re->nprog++;
}

/* compiles n; returns entry pc; *hole receives the list of pcs whose .x must
 * be patched to the continuation (kept as a simple array). */
typedef struct { int* pc; int n, cap; } holes;
static void hpush(holes* h, int pc) {
  if (h->n == h->cap) { h->cap = h->cap ? h->cap * 2 : 8; h->pc = (int*)realloc(h->pc, sizeof(int) * h->cap); }
  h->pc[h->n++] = pc;
}
/* hole encoding: pc*2 + (0 -> patch x, 1 -> patch y) */
static void patch(orc_re* re, holes* h, int to) {
  for (int i = 0; i < h->n; i++) {
    int pc = h->pc[i] >> 1;
    if (h->pc[i] & 1) re->prog[pc].y = to; else re->prog[pc].x = to;
  }
  h->n = 0;
}
static void happend(holes* dst, holes* src) {
  for (int i = 0; i < src->n; i++) hpush(dst, src->pc[i]);
  src->n = 0;
}

static int too_big(orc_re* re) { return re->nprog > 200000; }

static int comp(orc_re* re, node* n, holes* out) {
  switch (n->type) {
    case N_EMPTY: { int pc = emit(re, I_NOP); hpush(out, pc * 2); return pc; }
    case N_LIT: case N_CLASS: { int pc = emit(re, I_RUNE); re->prog[pc].cls = n->cls; hpush(out, pc * 2); return pc; }
    case N_ANY: { int pc = emit(re, I_ANY); hpush(out, pc * 2); return pc; }
    case N_ANYNL: { int pc = emit(re, I_ANYNL); hpush(out, pc * 2); return pc; }
    case N_ASSERT: { int pc = emit(re, I_EMPTY); re->prog[pc].empty = n->assert_op; hpush(out, pc * 2); return pc; }
    case N_CAT: {
      if (n->nkids == 0) { int pc = emit(re, I_NOP); hpush(out, pc * 2); return pc; }
      holes h = {0, 0, 0};
      int entry = comp(re, n->kids[0], &h);
      for (int i = 1; i < n->nkids; i++) {
        holes h2 = {0, 0, 0};
        int e = comp(re, n->kids[i], &h2);
        patch(re, &h, e);
        happend(&h, &h2);
        free(h2.pc);
        if (too_big(re)) break;
      }
      happend(out, &h);
      free(h.pc);
      return entry;
    }
    case N_ALT: {
      if (n->nkids == 1) return comp(re, n->kids[0], out);
      int entry = -1, prev_split = -1;
      for (int i = 0; i < n->nkids; i++) {
        int e;
        if (i < n->nkids - 1) {
          int sp = emit(re, I_SPLIT);
          holes h = {0, 0, 0};
          e = comp(re, n->kids[i], &h);
          re->prog[sp].x = e;
          happend(out, &h); free(h.pc);
          if (prev_split >= 0) re->prog[prev_split].y = sp; else entry = sp;
          prev_split = sp;
        } else {
          holes h = {0, 0, 0};
          e = comp(re, n->kids[i], &h);
          happend(out, &h); free(h.pc);
          if (prev_split >= 0) re->prog[prev_split].y = e; else entry = e;
        }
      }
      return entry;
    }
    case N_REP: {
      node* k = n->kids[0];
      int mn = n->min, mx = n->max;
      /* x{n,m} = x^n (x?)^(m-n); x{n,} = x^n x* */
      int entry = -1;
      holes cur = {0, 0, 0};
      int have = 0;
      for (int i = 0; i < mn; i++) {
        holes h = {0, 0, 0};
        int e = comp(re, k, &h);
        if (have) patch(re, &cur, e); else entry = e;
        have = 1;
        happend(&cur, &h); free(h.pc);
        if (too_big(re)) break;
      }
      if (mx < 0) {
        int sp = emit(re, I_SPLIT);
        holes h = {0, 0, 0};
        int e = comp(re, k, &h);
        re->prog[sp].x = e;
        patch(re, &h, sp);
        free(h.pc);
        if (have) patch(re, &cur, sp); else entry = sp;
        hpush(&cur, sp * 2 + 1);
      } else {
        for (int i = mn; i < mx; i++) {
          int sp = emit(re, I_SPLIT);
          holes h = {0, 0, 0};
          int e = comp(re, k, &h);
          re->prog[sp].x = e;
          if (have) patch(re, &cur, sp); else entry = sp;
          have = 1;
          hpush(&cur, sp * 2 + 1);
          happend(&cur, &h); free(h.pc);
          if (too_big(re)) break;
        }
        if (!have && mx == 0) { int pc = emit(re, I_NOP); entry = pc; hpush(&cur, pc * 2); }
      }
      happend(out, &cur); free(cur.pc);
      return entry;
    }
  }
  return -1;
}

orc_re* orc_re_compile(const char* pattern, char* err, size_t errcap) {
  if (err && errcap) err[0] = 0;
  orc_re* re = (orc_re*)calloc(1, sizeof(orc_re));
  parser ps;
  memset(&ps, 0, sizeof(ps));
  ps.p = pattern; ps.end = pattern + strlen(pattern);
  ps.re = re; ps.err = err; ps.errcap = errcap;
  node* root = parse_alt(&ps);
  if (root && ps.p < ps.end) { set_err(&ps, "unexpected )"); free_node(root); root = NULL; }
  if (!root) { orc_re_free(re); return NULL; }
  holes h = {0, 0, 0};
  int entry = comp(re, root, &h);
  int m = emit(re, I_MATCH);
  patch(re, &h, m);
  free(h.pc);
  free_node(root);
  if (too_big(re)) { if (err) snprintf(err, errcap, "expression too large"); orc_re_free(re); return NULL; }
  re->start = entry;
  return re;
}

void orc_re_free(orc_re* re) {
  if (!re) return;
  for (int i = 0; i < re->ncls; i++) free(re->cls[i].r);
  free(re->cls); free(re->prog); free(re);
}

/* ---------- matching ---------- */
static int is_word(int r) { return r >= 0 && r < 0x80 && (is_alnum_c(r) || r == '_'); }

static int context_at(const uint8_t* s, size_t n, size_t pos) {
  int r1 = -1, r2 = -1;
  if (pos > 0) r1 = s[pos - 1] < 0x80 ? s[pos - 1] : 0x80;   /* non-ASCII: neither word nor \n */
  if (pos < n) r2 = s[pos] < 0x80 ? s[pos] : 0x80;
  int op = E_NWB, b = 0;
  if (is_word(r1)) b = 1; else if (r1 == '\n') op |= E_BOL; else if (r1 < 0) op |= E_BOT | E_BOL;
  if (is_word(r2)) b ^= 1; else if (r2 == '\n') op |= E_EOL; else if (r2 < 0) op |= E_EOT | E_EOL;
  if (b) op ^= (E_WB | E_NWB);
  return op;
}

typedef struct { int pc; size_t pos; } job;

int orc_re_match(const orc_re* re, const uint8_t* s, size_t n) {
  size_t nbits = (size_t)re->nprog * (n + 1);
  size_t words = (nbits + 63) / 64;
  uint64_t stackbuf[512];
  uint64_t* visited = words <= 512 ? stackbuf : (uint64_t*)calloc(words, 8);
  if (words <= 512) memset(visited, 0, words * 8);
  size_t cap = 256, top = 0;
  job* stk = (job*)malloc(sizeof(job) * cap);
  int found = 0;
  size_t start = 0;
  for (;;) {
    top = 0;
    stk[top].pc = re->start; stk[top].pos = start; top++;
    while (top > 0 && !found) {
      job j = stk[--top];
      for (;;) {
        size_t bit = (size_t)j.pc * (n + 1) + j.pos;
        if (visited[bit >> 6] & (1ull << (bit & 63))) break;
        visited[bit >> 6] |= 1ull << (bit & 63);
        const inst* in = &re->prog[j.pc];
        if (in->op == I_MATCH) { found = 1; break; }
        if (in->op == I_NOP) { j.pc = in->x; continue; }
        if (in->op == I_JMP) { j.pc = in->x; continue; }
        if (in->op == I_SPLIT) {
          if (top == cap) { cap *= 2; stk = (job*)realloc(stk, sizeof(job) * cap); }
          stk[top].pc = in->y; stk[top].pos = j.pos; top++;
          j.pc = in->x; continue;
        }
        if (in->op == I_EMPTY) {
          int ctx = context_at(s, n, j.pos);
          if ((in->empty & ~ctx) != 0) break;
          j.pc = in->x; continue;
        }
        if (j.pos >= n) break;
        int w; int r = decode_rune(s + j.pos, n - j.pos, &w);
        int ok;
        if (in->op == I_ANY) ok = 1;
        else if (in->op == I_ANYNL) ok = r != '\n';
        else ok = cls_has(&re->cls[in->cls], r);
        if (!ok) break;
        j.pc = in->x; j.pos += (size_t)w;
      }
    }
    if (found || start >= n) break;
    int w; decode_rune(s + start, n - start, &w);
    start += (size_t)w;
  }
  free(stk);
  if (visited != stackbuf) free(visited);
  return found;
}
