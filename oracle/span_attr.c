/*
 * span_attr.c — CPU restatement of the per-span condition of odigossampling's
 * span_attribute rule for string / number / boolean conditions.  TEST
 * INFRASTRUCTURE (see oracle.h): the checker for attr_kernel.hip, written
 * apart from the product's odigos_amd/csrc/span_attr.cpp so the GPU result
 * is not compared with itself.
 *
 * Restates collector/processors/odigossamplingprocessor/internal/sampling/
 *   spanattribute.go:136-178   string: exists / equals / not_equals /
 *                              contains / not_contains / regex
 *   spanattribute.go:179-221   number: exists and the six comparisons on
 *                              float64(attr.Int()) or attr.Double()
 *   spanattribute.go:222-235   boolean: exists / equals
 * and the Go standard library pieces they call:
 *   strconv.ParseFloat(s, 64)  readFloat's syntax (sign, "0x" mantissa with a
 *                              mandatory 'p' exponent, '_' separators checked
 *                              by underscoreOK, inf / infinity / nan), value
 *                              by correctly rounded conversion, ErrRange on
 *                              overflow only
 *   strconv.ParseBool          1 t T TRUE true True / 0 f F FALSE false False
 *   strings.Contains           byte substring ("" is in every string)
 *   regexp.MatchString         oracle/regex.c (backtracking; oracle-private)
 */
#include <errno.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int lower(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

static size_t prefix_ci(const char* s, size_t n, const char* w) {
  size_t k = 0;
  while (k < n && w[k] && lower((unsigned char)s[k]) == w[k]) k++;
  return k;
}

/* underscoreOK (strconv/atoi.go): '_' only between digits, or between a
 * base prefix and a digit */
static int underscore_ok(const char* s, size_t n) {
  size_t i = 0;
  char saw = '^';
  int hex = 0;
  if (n >= 1 && (s[0] == '-' || s[0] == '+')) { s++; n--; }
  if (n >= 2 && s[0] == '0' && (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
    i = 2;
    saw = '0';
    hex = lower(s[1]) == 'x';
  }
  for (; i < n; i++) {
    int c = (unsigned char)s[i];
    if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { saw = '0'; continue; }
    if (c == '_') {
      if (saw != '0') return 0;
      saw = '_';
      continue;
    }
    if (saw == '_') return 0;
    saw = '!';
  }
  return saw != '_';
}

int orc_go_parse_float(const char* s, size_t n, double* out) {
  if (n == 0) return 0;
  /* special(): [+-]inf / [+-]infinity, nan (no sign) */
  {
    size_t i = 0;
    int neg = 0;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i < n && lower((unsigned char)s[i]) == 'i') {
      size_t k = prefix_ci(s + i, n - i, "infinity");
      if (k > 3 && k < 8) k = 3;
      if ((k == 3 || k == 8) && i + k == n) { *out = neg ? -INFINITY : INFINITY; return 1; }
      if (k == 3 || k == 8) return 0;
    }
    if (i == 0 && lower((unsigned char)s[0]) == 'n') {
      if (prefix_ci(s, n, "nan") == 3 && n == 3) { *out = NAN; return 1; }
      return 0;
    }
  }
  /* readFloat syntax */
  size_t i = 0;
  int underscores = 0, hex = 0, sawdot = 0, sawdigits = 0;
  if (s[i] == '+' || s[i] == '-') i++;
  if (i + 2 < n && s[i] == '0' && lower((unsigned char)s[i + 1]) == 'x') { hex = 1; i += 2; }
  for (; i < n; i++) {
    int c = (unsigned char)s[i];
    if (c == '_') { underscores = 1; continue; }
    if (c == '.') {
      if (sawdot) break;
      sawdot = 1;
      continue;
    }
    if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { sawdigits = 1; continue; }
    break;
  }
  if (!sawdigits) return 0;
  if (i < n && lower((unsigned char)s[i]) == (hex ? 'p' : 'e')) {
    i++;
    if (i >= n) return 0;
    if (s[i] == '+' || s[i] == '-') i++;
    if (i >= n || s[i] < '0' || s[i] > '9') return 0;
    for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); i++)
      if (s[i] == '_') underscores = 1;
  } else if (hex) {
    return 0;   /* a hexadecimal mantissa requires a 'p' exponent */
  }
  if (i != n) return 0;
  if (underscores && !underscore_ok(s, n)) return 0;
  /* value: the literal without separators, correctly rounded by strtod */
  char stack[256];
  char* buf = n < sizeof stack ? stack : (char*)malloc(n + 1);
  size_t m = 0;
  for (size_t k = 0; k < n; k++)
    if (s[k] != '_') buf[m++] = s[k];
  buf[m] = 0;
  errno = 0;
  char* end = NULL;
  double v = strtod(buf, &end);
  int ok = end == buf + m && !(errno == ERANGE && isinf(v));
  if (buf != stack) free(buf);
  if (!ok) return 0;
  *out = v;
  return 1;
}

int orc_go_parse_bool(const char* s, size_t n, int* out) {
  static const char* t[] = {"1", "t", "T", "TRUE", "true", "True"};
  static const char* f[] = {"0", "f", "F", "FALSE", "false", "False"};
  for (int k = 0; k < 6; k++) {
    if (strlen(t[k]) == n && memcmp(s, t[k], n) == 0) { *out = 1; return 1; }
    if (strlen(f[k]) == n && memcmp(s, f[k], n) == 0) { *out = 0; return 1; }
  }
  return 0;
}

static int contains(const uint8_t* s, size_t n, const char* e, size_t m) {
  if (m == 0) return 1;
  for (size_t i = 0; i + m <= n; i++)
    if (memcmp(s + i, e, m) == 0) return 1;
  return 0;
}

int orc_attr_cond_init(orc_attr_cond* a, const char* cond, const char* op, const char* expected, size_t elen) {
  memset(a, 0, sizeof *a);
  a->cond = strcmp(cond, "string") == 0 ? 0 : strcmp(cond, "number") == 0 ? 1 : strcmp(cond, "boolean") == 0 ? 2 : -1;
  if (a->cond < 0) return -1;
  strncpy(a->op, op, sizeof a->op - 1);
  a->expected = (char*)malloc(elen + 1);
  memcpy(a->expected, expected, elen);
  a->expected[elen] = 0;
  a->expected_len = elen;
  if (a->cond == 0 && strcmp(op, "regex") == 0) {
    char err[256];
    a->re = orc_re_compile(a->expected, err, sizeof err);   /* NULL: regexp.Compile error */
  }
  if (a->cond == 1) a->num_ok = orc_go_parse_float(expected, elen, &a->num);
  if (a->cond == 2) a->bool_ok = orc_go_parse_bool(expected, elen, &a->bool_val);
  return 0;
}

void orc_attr_cond_free(orc_attr_cond* a) {
  free(a->expected);
  if (a->re) orc_re_free(a->re);
  memset(a, 0, sizeof *a);
}

int orc_attr_cond_eval(const orc_attr_cond* a, uint8_t type, uint64_t val, const uint8_t* arena) {
  const char* op = a->op;
  if (a->cond == 0) {
    const uint8_t* s = arena + (uint32_t)val;
    const size_t n = (uint32_t)(val >> 32);
    if (strcmp(op, "exists") == 0) return type == OSE_ATTR_STR && n != 0;
    if (type != OSE_ATTR_STR) return 0;
    if (strcmp(op, "equals") == 0) return n == a->expected_len && memcmp(s, a->expected, n) == 0;
    if (strcmp(op, "not_equals") == 0) return !(n == a->expected_len && memcmp(s, a->expected, n) == 0);
    if (strcmp(op, "contains") == 0) return contains(s, n, a->expected, a->expected_len);
    if (strcmp(op, "not_contains") == 0) return !contains(s, n, a->expected, a->expected_len);
    if (strcmp(op, "regex") == 0) return a->re && orc_re_match(a->re, s, n);
    return 0;
  }
  if (a->cond == 1) {
    const int num = type == OSE_ATTR_INT || type == OSE_ATTR_DOUBLE;
    if (strcmp(op, "exists") == 0) return num;
    if (!a->num_ok || !num) return 0;
    double x;
    if (type == OSE_ATTR_INT) x = (double)(int64_t)val;
    else memcpy(&x, &val, 8);
    if (strcmp(op, "equals") == 0) return x == a->num;
    if (strcmp(op, "not_equals") == 0) return x != a->num;
    if (strcmp(op, "greater_than") == 0) return x > a->num;
    if (strcmp(op, "less_than") == 0) return x < a->num;
    if (strcmp(op, "greater_than_or_equal") == 0) return x >= a->num;
    if (strcmp(op, "less_than_or_equal") == 0) return x <= a->num;
    return 0;
  }
  if (strcmp(op, "exists") == 0) return type == OSE_ATTR_BOOL;
  if (!a->bool_ok || type != OSE_ATTR_BOOL) return 0;
  return strcmp(op, "equals") == 0 && (val != 0) == (a->bool_val != 0);
}
