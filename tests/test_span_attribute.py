"""odigossampling span_attribute rules.

The per-span condition (internal/sampling/spanattribute.go:126-320): string,
number and boolean conditions run on the GPU (attr_kernel.hip) from the
attr_type / attr_val columns the host columniser fills; "json" conditions
run in the host columniser (odigos_amd/csrc/span_attr.cpp) into attr_match.
The oracle restates the string / number / boolean condition on its own
(oracle/span_attr.c, with oracle/regex.c), so the GPU path is not compared
with the product's host predicate.  The trace stage and the oracle OR the
bits per trace as service-shaped rules.

* KATs: the 20 cases of spanattribute_test.go, transcribed as data
  (tests/golden/span_attribute_kats.json) — CPU through host columniser +
  oracle, GPU through the HIP trace stage and the ConsumeTraces path.
* Edge cases of the Go library semantics the predicate restates
  (strconv.ParseFloat / ParseBool / FormatFloat, encoding/json validity and
  Marshal, jsonpath Get) through osehost_span_attr_eval.  These follow the
  published behaviour of the Go standard library; the reference's tests do
  not cover them, so they are "parity unpinned" beyond the KATs.
* Trace-level composition: the condition must hold on one span of a
  resource whose AsString(service.name) equals the rule's service.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

from odigos_amd import host, native
from tests.oracle_lib import SamplingOracle, lib as orc_lib

GOLD = json.loads((Path(__file__).parent / "golden" / "span_attribute_kats.json").read_text())
TID = "4bf92f3577b34da6a3ce929d0e0e4736"
SEED = 0x0D16A5EE
BASE = 1739000000000000000


def _rule(c):
    d = dict(c["rule"])
    return {"name": c["test"], "type": "span_attribute", "rule_details": d}


def build_trace(service, attrs, extra=()):
    """buildTrace (spanattribute_test.go:12-29): one resource, one span."""
    rs = [host.resource_spans({"service.name": service} if service is not None else {},
                              [host.span(name="span", trace_id=TID, span_id="00f067aa0ba902b7", start=BASE,
                                         end=BASE + 5_000_000, attributes=attrs)])]
    rs += list(extra)
    return host.traces(*rs)


def _expect(e):
    matched, satisfied, ratio = e
    assert matched == satisfied  # the rule is never matched-but-unsatisfied (spanattribute.go:319)
    return (0, ratio) if satisfied else (4, 100.0)


def _u():
    hi, lo = int(TID[:16], 16), int(TID[16:], 16)
    return orc_lib().orc_trace_uniform(hi, lo, SEED)


def _read(addr, ctype, n=1):
    return [C.cast(addr, C.POINTER(ctype))[i] for i in range(n)]


def _oracle(cfg, td):
    proc = host.Processor("odigossampling", cfg)
    proc.configure(SEED, native.GROUP_BATCH)
    hb = proc.columnarize(td)
    assert SamplingOracle(cfg).process(hb.cols, hb.outs, native.GROUP_BATCH, SEED) == 0
    o = hb.outs
    return (_read(o.trace_level, C.c_uint8)[0], _read(o.trace_ratio, C.c_double)[0],
            _read(o.trace_keep, C.c_uint8)[0], _read(o.keep, C.c_uint8, hb.cols.n_spans))


def test_fixture_count():
    assert len(GOLD["cases"]) == 20


@pytest.mark.parametrize("c", GOLD["cases"], ids=[c["test"] for c in GOLD["cases"]])
def test_kat_oracle(c):
    cfg = {"global_rules": [_rule(c)]}
    lvl, ratio = _expect(c["expect"])
    got_l, got_r, tk, keep = _oracle(cfg, build_trace(c["service"], c["attrs"]))
    assert (got_l, got_r) == (lvl, ratio)
    assert tk == (lvl == 4 or _u() * 100 < ratio)
    assert all(k == tk for k in keep)


# ---- the per-span predicate: Go library semantics -------------------------

def _eval(rule, value):
    L = native.lib()
    r = L.osehost_span_attr_eval(json.dumps(rule).encode(), host.dumps(value).encode())
    if r < 0:
        raise RuntimeError(L.osehost_last_error().decode())
    return bool(r)


def _r(cond, op, exp="", path=""):
    return {"service_name": "s", "attribute_key": "k", "condition_type": cond, "operation": op,
            "expected_value": exp, "json_path": path}


S = lambda s: {"stringValue": s}  # noqa: E731
I = lambda i: {"intValue": str(i)}  # noqa: E731
D = host.attr_value  # noqa: E731  (doubles; non-finite ones as the protobuf JSON strings)
B = lambda b: {"boolValue": b}  # noqa: E731

PRED_CASES = [
    # string (spanattribute.go:143-178): type must be Str; exists needs non-empty
    (_r("string", "exists"), S(""), False),
    (_r("string", "exists"), I(5), False),
    (_r("string", "equals", "5"), I(5), False),
    (_r("string", "not_equals", "x"), I(5), False),
    (_r("string", "not_equals", "x"), S(""), True),
    (_r("string", "contains", "od"), S("prod"), True),
    (_r("string", "not_contains", "od"), S("prod"), False),
    (_r("string", "regex", "ab+c"), S("xxabbbcx"), True),       # MatchString is unanchored
    (_r("string", "regex", "^ab+c$"), S("xxabbbcx"), False),
    (_r("string", "regex", "a("), S("a("), False),              # compile error -> continue
    # number (179-223): Int or Double; expected parsed by ParseFloat
    (_r("number", "exists"), I(0), True),
    (_r("number", "exists"), D(0.0), True),
    (_r("number", "exists"), S("5"), False),
    (_r("number", "equals", "5"), S("5"), False),
    (_r("number", "equals", "1e2"), I(100), True),
    (_r("number", "equals", "+100"), I(100), True),
    (_r("number", "equals", ".5"), D(0.5), True),
    (_r("number", "equals", " 5"), I(5), False),                # ParseFloat rejects spaces
    (_r("number", "equals", "5x"), I(5), False),
    (_r("number", "greater_than", "-Inf"), I(-(2 ** 62)), True),
    (_r("number", "less_than", "+inf"), D(1e308), True),
    (_r("number", "less_than", "Infinity"), D(1e308), True),
    (_r("number", "equals", "NaN"), D(1.0), False),
    (_r("number", "not_equals", "nan"), D(1.0), True),
    (_r("number", "not_equals", "5"), I(5), False),
    (_r("number", "equals", "9007199254740993"), I(9007199254740992), True),   # float64(int) rounding
    (_r("number", "greater_than_or_equal", "1e400"), D(1e308), False),         # out of range -> err -> continue
    (_r("number", "less_than", "0.1"), D(0.09999999999999999), True),
    # boolean (224-236): ParseBool
    (_r("boolean", "exists"), B(False), True),
    (_r("boolean", "exists"), S("true"), False),
    (_r("boolean", "equals", "T"), B(True), True),
    (_r("boolean", "equals", "1"), B(True), True),
    (_r("boolean", "equals", "TRUE"), B(True), True),
    (_r("boolean", "equals", "True"), B(True), True),
    (_r("boolean", "equals", "tRUE"), B(True), False),
    (_r("boolean", "equals", "yes"), B(True), False),
    (_r("boolean", "equals", "0"), B(False), True),
    (_r("boolean", "equals", "F"), B(True), False),
    (_r("boolean", "equals", "true"), S("true"), False),
    # json validity (237-252): encoding/json Unmarshal
    (_r("json", "is_valid_json"), S(""), False),
    (_r("json", "is_valid_json"), S(" {} \n"), True),
    (_r("json", "is_valid_json"), S("{}x"), False),
    (_r("json", "is_valid_json"), S("[1,2,]"), False),
    (_r("json", "is_valid_json"), S("01"), False),
    (_r("json", "is_valid_json"), S("1e400"), False),           # does not fit float64
    (_r("json", "is_valid_json"), S("-0.0e-5"), True),
    (_r("json", "is_valid_json"), S('"\\ud800"'), True),        # lone surrogate decodes to U+FFFD
    (_r("json", "is_valid_json"), S('"\\x41"'), False),
    (_r("json", "is_valid_json"), S("'a'"), False),
    (_r("json", "is_valid_json"), S("nul"), False),
    (_r("json", "is_valid_json"), S('{"a":1,"a":2}'), True),
    (_r("json", "is_valid_json"), I(5), False),                 # JSON conditions need a Str attribute
    (_r("json", "is_invalid_json"), I(5), False),
    (_r("json", "is_invalid_json"), S("{"), True),
    (_r("json", "exists", path="$"), S("{}"), False),           # no case in the switch
    # jsonpath Get + key comparisons (253-313)
    (_r("json", "contains_key", path="$.a"), S('{"a":null}'), False),          # res == nil
    (_r("json", "not_contains_key", path="$.a"), S('{"a":null}'), False),      # err == nil
    (_r("json", "contains_key", path="$.a.b"), S('{"a":{"b":0}}'), True),
    (_r("json", "contains_key", path="$['a']['b']"), S('{"a":{"b":0}}'), True),
    (_r("json", "contains_key", path="$.a[1]"), S('{"a":[5,6]}'), True),
    (_r("json", "contains_key", path="$.a[2]"), S('{"a":[5,6]}'), False),
    (_r("json", "not_contains_key", path="$.a[2]"), S('{"a":[5,6]}'), True),
    (_r("json", "contains_key", path="$"), S("5"), True),
    (_r("json", "not_contains_key", path="$.a"), S("[1]"), True),
    (_r("json", "contains_key", path="$.a"), S("{"), False),
    (_r("json", "key_equals", "2", "$.a"), S('{"a":1,"a":2}'), True),          # last duplicate wins
    (_r("json", "key_equals", "null", "$.a"), S('{"a":null}'), True),
    (_r("json", "key_equals", "true", "$.a"), S('{"a":true}'), True),
    (_r("json", "key_equals", "0.1", "$.a"), S('{"a":0.1}'), True),
    (_r("json", "key_equals", "123", "$.a"), S('{"a":123.0}'), True),
    (_r("json", "key_equals", "-0", "$.a"), S('{"a":-0}'), True),
    (_r("json", "key_equals", "1000000000000000000000", "$.a"), S('{"a":1e21}'), True),
    (_r("json", "key_equals", "0.000001", "$.a"), S('{"a":1e-6}'), True),
    (_r("json", "key_equals", "x", "$.a"), S('{"a":"x"}'), True),
    (_r("json", "key_equals", '{"a":"\\u003c","b":1}', "$.o"), S('{"o":{"b":1,"a":"<"}}'), True),
    (_r("json", "key_equals", '[1,"x",null,true,{}]', "$.o"), S('{"o":[1,"x",null,true,{}]}'), True),
    (_r("json", "key_equals", "[1e+21,1e-7,0.5]", "$.o"), S('{"o":[1e21,1e-7,0.5]}'), True),
    (_r("json", "key_equals", '["\\u0026\\u003e"]', "$.o"), S('{"o":["&>"]}'), True),
    (_r("json", "key_equals", "x", "$.b"), S('{"a":"x"}'), False),             # Get error -> continue
    (_r("json", "key_not_equals", "x", "$.b"), S('{"a":"x"}'), False),
    (_r("json", "key_not_equals", "y", "$.a"), S('{"a":"x"}'), True),
    # ambiguous selectors: Get returns the match list and never errs (parity
    # unpinned: PaesslerAG/jsonpath is not in the reference; object members
    # are visited in sorted key order)
    (_r("json", "contains_key", path="$..a"), S('{"x":{"a":1}}'), True),
    (_r("json", "contains_key", path="$..a"), S('{"x":1}'), True),            # an empty list is not nil
    (_r("json", "not_contains_key", path="$.x[*]"), S('{"a":1}'), False),     # no error
    (_r("json", "key_equals", "[1,2]", "$.a[*]"), S('{"a":[1,2]}'), True),
    (_r("json", "key_equals", "[2,1]", "$.a[1,0]"), S('{"a":[1,2]}'), True),
    (_r("json", "key_equals", '["x"]', "$['b',1]"), S('{"b":"x"}'), True),     # the index finds no array
    (_r("json", "key_equals", "[5,6]", "$.a[0:2]"), S('{"a":[5,6,7]}'), True),
    (_r("json", "key_equals", "[7]", "$.a[-1:]"), S('{"a":[5,6,7]}'), True),
    (_r("json", "key_equals", "[7,6,5]", "$.a[::-1]"), S('{"a":[5,6,7]}'), True),
    (_r("json", "key_equals", "[5,7]", "$.a[0:3:2]"), S('{"a":[5,6,7]}'), True),
    (_r("json", "key_equals", '["x","y"]', "$.*"), S('{"b":"y","a":"x"}'), True),
    (_r("json", "key_equals", "[1,3]", "$..a"), S('{"a":1,"b":{"a":3}}'), True),
    (_r("json", "key_equals", "[]", "$..q"), S('{"a":1}'), True),
    (_r("json", "key_equals", "[1,3]", "$..a"), S('[{"a":1},{"a":3}]'), True),
    # filters [?(expr)] and scripts [(expr)]: a gval expression subset
    # (parity unpinned: gval and PaesslerAG/jsonpath are not in the reference)
    (_r("json", "key_equals", '[{"b":1}]', "$.a[?(@.b==1)]"), S('{"a":[{"b":1},{"b":2},{"c":1}]}'), True),
    (_r("json", "key_equals", "[2,3]", "$.a[?(@ > 1)]"), S('{"a":[1,2,3]}'), True),
    (_r("json", "key_equals", '["x"]', "$.a[?(@.n >= 2 && @.n < 3)].s"),
     S('{"a":[{"n":1,"s":"w"},{"n":2,"s":"x"},{"n":3,"s":"y"}]}'), True),
    (_r("json", "key_equals", '["w","y"]', "$.a[?(@.n == 1 || @.n > 2)].s"),
     S('{"a":[{"n":1,"s":"w"},{"n":2,"s":"x"},{"n":3,"s":"y"}]}'), True),
    (_r("json", "key_equals", '[{"k":"v"}]', "$.a[?(@.k)]"), S('{"a":[{"k":"v"},{"j":1},{"k":""}]}'), True),
    (_r("json", "key_equals", '[{"j":1}]', "$.a[?(!@.k)]"), S('{"a":[{"k":"v"},{"j":1}]}'), True),
    (_r("json", "key_equals", '["prod-1"]', "$.e[?(@ =~ '^prod-')]"), S('{"e":["dev","prod-1"]}'), True),
    (_r("json", "key_equals", "[3]", "$.a[?(@ * 2 - 1 == 5)]"), S('{"a":[1,2,3]}'), True),
    (_r("json", "key_equals", '["ab"]', "$.a[?(@ + 'b' == 'abb')]"), S('{"a":["ab","b"]}'), True),
    (_r("json", "key_equals", "[1]", "$.a[?(@.x == $.want)].y"), S('{"want":"q","a":[{"x":"q","y":1},{"x":"r","y":2}]}'), True),
    (_r("json", "key_equals", "[2]", "$.o[?(@ > 1)]"), S('{"o":{"p":1,"q":2}}'), True),     # member values, sorted keys
    (_r("json", "key_equals", "[]", "$.a[?(@.b == 'x')]"), S('{"a":[{"b":1}]}'), True),     # mixed types: not equal
    (_r("json", "contains_key", path="$.a[?(@.b==9)]"), S('{"a":[{"b":1}]}'), True),       # an empty list is not nil
    (_r("json", "key_equals", "[7]", "$.a[(1+1)]"), S('{"a":[5,6,7]}'), True),              # script: an index
    (_r("json", "key_equals", "[5]", "$[(@.k)]"), S('{"k":"z","z":5}'), True),               # script: a key
    (_r("json", "key_equals", "[]", "$.a[(9)]"), S('{"a":[5]}'), True),
]


@pytest.mark.parametrize("rule,value,want", PRED_CASES,
                         ids=[f'{i}-{r["condition_type"]}-{r["operation"]}' for i, (r, _, _) in enumerate(PRED_CASES)])
def test_predicate(rule, value, want):
    assert _eval(rule, value) == want


def test_unsupported_jsonpath_rejected_at_creation():
    # paths the engine cannot parse are refused at creation instead of guessed
    for path in ("$.a[?(@.b==)]", "$[(@.length-1]", "$.a[?(@.b ~ 1)]", "$.a[", "a.b"):
        cfg = {"global_rules": [{"name": "j", "type": "span_attribute",
                                 "rule_details": dict(_r("json", "contains_key", path=path), sampling_ratio=1.0)}]}
        with pytest.raises((ValueError, RuntimeError)):
            host.Processor("odigossampling", cfg)


# ---- trace-level composition -----------------------------------------------

def _cfg(*rules):
    return {"global_rules": [{"name": f"r{i}", "type": "span_attribute",
                              "rule_details": dict(d, sampling_ratio=r, fallback_sampling_ratio=1.0)}
                             for i, (d, r) in enumerate(rules)]}


def _span(attrs, k):
    return host.span(name=f"s{k}", trace_id=TID, span_id="%016x" % (k + 1), start=BASE + k, end=BASE + k + 10,
                     attributes=attrs)


def _trace(*resources):
    return host.traces(*[host.resource_spans(res, [_span(a, i * 10 + j) for j, a in enumerate(sp)])
                         for i, (res, sp) in enumerate(resources)])


ENV = {"service_name": "svc", "attribute_key": "env", "condition_type": "string", "operation": "equals",
       "expected_value": "prod"}

COMPOSE = [
    # attribute on a span of another service: not satisfied
    ("other-service", _cfg((ENV, 30.0)), _trace(({"service.name": "other"}, [{"env": "prod"}])), 4, 100.0),
    # one matching span among many, in the second resource
    ("one-of-many", _cfg((ENV, 30.0)),
     _trace(({"service.name": "svc"}, [{"env": "dev"}, {}]), ({"service.name": "svc"}, [{}, {"env": "prod"}])), 0, 30.0),
    # resource without service.name is skipped
    ("no-service", _cfg((ENV, 30.0)), _trace(({}, [{"env": "prod"}])), 4, 100.0),
    # AsString of a non-string service.name (int 7 -> "7")
    ("int-service", _cfg((dict(ENV, service_name="7"), 30.0)), _trace(({"service.name": 7}, [{"env": "prod"}])), 0, 30.0),
    # two global rules satisfied: evaluateLevel keeps the maximum ratio (rule_engine.go:99-102)
    ("two-rules", _cfg((ENV, 30.0), (dict(ENV, attribute_key="tier", expected_value="gold"), 12.0)),
     _trace(({"service.name": "svc"}, [{"env": "prod"}, {"tier": "gold"}])), 0, 30.0),
    # attribute key on the resource, not the span: not seen
    ("resource-attr", _cfg((ENV, 30.0)), _trace(({"service.name": "svc", "env": "prod"}, [{}])), 4, 100.0),
]


@pytest.mark.parametrize("name,cfg,td,lvl,ratio", COMPOSE, ids=[c[0] for c in COMPOSE])
def test_compose_oracle(name, cfg, td, lvl, ratio):
    got_l, got_r, _, _ = _oracle(cfg, td)
    assert (got_l, got_r) == (lvl, ratio)


def test_mixed_with_service_rules():
    # span_attribute and service_name rules share the 64 per-trace service bits
    cfg = {"global_rules": [{"name": "a", "type": "span_attribute", "rule_details": dict(ENV, sampling_ratio=40.0)}],
           "service_rules": [{"name": "s", "type": "service_name",
                              "rule_details": {"service_name": "svc", "sampling_ratio": 20.0}}]}
    l, r, _, _ = _oracle(cfg, _trace(({"service.name": "svc"}, [{"env": "prod"}])))
    assert (l, r) == (0, 40.0)
    l, r, _, _ = _oracle(cfg, _trace(({"service.name": "svc"}, [{"env": "dev"}])))
    assert (l, r) == (1, 20.0)


def test_rule_count_past_64():
    # Validate (config.go:17-80) bounds no rule count: 65 and 150 span_attribute
    # rules are accepted, in rule chunks of at most 64 service-shaped bits,
    # their bits in (rules + 63) / 64 attr_match words (no device needed)
    import ctypes as C
    import json
    for k in (65, 150):
        rules = [{"name": f"a{i}", "type": "span_attribute", "rule_details": dict(ENV, expected_value=str(i),
                                                                                sampling_ratio=1.0)} for i in range(k)]
        n = C.c_uint32()
        assert native.lib().osehost_sampling_chunks(json.dumps({"odigossampling": {"global_rules": rules}}).encode(),
                                                    C.byref(n)) == 0
        assert n.value == (k + 63) // 64


# ---- strconv.ParseFloat: product (span_attr.cpp) vs oracle (span_attr.c) ----

FLOATS = ["5", "+5", "-5", ".5", "5.", "+.5e-3", "1e2", "1E+2", "1e", "e1", "", " 5", "5 ", "1_000", "1__0", "_1",
          "1_", "1_0.0_1", "1._5", "1_.5", "1e1_0", "0x1p-2", "0x1.8", "0x1.8p1", "0X1P+0", "0x_1p0", "0x1_0p0",
          "0x", "0xp1", "0x.8p1", "0x1p", "inf", "+Inf", "-INFINITY", "infinit", "infx", "nan", "NaN", "+nan",
          "-nan", "1e400", "-1e400", "1e-400", "4.9e-324", "0x1p-1074", "0x1p1024", "0x1.fffffffffffffp1023",
          "9007199254740993", "0.1", "00012", "1.2.3", "--1", "+-1", "1e+", "1e-_1", "0b101", "0o17", "1f"]


@pytest.mark.parametrize("s", FLOATS)
def test_parse_float_product_vs_oracle(s):
    v = C.c_double()
    ok = orc_lib().orc_go_parse_float(s.encode(), len(s), C.byref(v))
    if not ok:
        # ParseFloat error: the rule never holds (spanattribute.go:185-188)
        for op in ("equals", "not_equals", "less_than", "greater_than"):
            assert not _eval(_r("number", op, s), D(1.0)), (s, op)
        return
    x = v.value
    if x != x:   # NaN: == never holds, != always
        assert not _eval(_r("number", "equals", s), D(1.0)) and _eval(_r("number", "not_equals", s), D(1.0))
        return
    val = D(x)
    assert _eval(_r("number", "equals", s), val), s
    assert not _eval(_r("number", "not_equals", s), val), s


# ---- random differential: GPU kernel vs oracle restatement ---------------------

def _random_attr_case(seed, n_traces=60, n_rules=None):
    """Rules over three keys (string / number / bool conditions, every
    operation, regexps, unparsable expectations) and traces whose spans carry
    those keys with every value type."""
    import random
    rng = random.Random(seed)
    svcs = ["svc-a", "svc-b", "svc-c"]
    str_rules = [("equals", "prod"), ("not_equals", "prod"), ("contains", "ro"), ("not_contains", "x"),
                 ("exists", ""), ("regex", "^p[a-z]+d$"), ("regex", "(a|b)+c"), ("regex", "a("), ("regex", "é+"),
                 ("contains", ""), ("equals", "")]
    num_rules = [("equals", "5"), ("not_equals", "5"), ("greater_than", "2.5"), ("less_than", "-1e3"),
                 ("greater_than_or_equal", "0x1p3"), ("less_than_or_equal", "1_000"), ("exists", ""),
                 ("equals", "bogus"), ("equals", "NaN"), ("not_equals", "nan"), ("greater_than", "-Inf")]
    bool_rules = [("equals", "true"), ("equals", "F"), ("exists", ""), ("equals", "yes")]
    rules = []
    for k in range(n_rules or rng.randint(4, 14)):
        cond = rng.choice(["string", "number", "boolean"])
        op, exp = rng.choice({"string": str_rules, "number": num_rules, "boolean": bool_rules}[cond])
        while n_rules and exp == "" and op != "exists":   # (a long list would almost surely draw one Validate rejects)
            op, exp = rng.choice({"string": str_rules, "number": num_rules, "boolean": bool_rules}[cond])
        key = rng.choice(["env", "code", "flag"])
        rules.append({"name": f"a{k}", "type": "span_attribute",
                      "rule_details": {"service_name": rng.choice(svcs), "attribute_key": key,
                                       "condition_type": cond, "operation": op, "expected_value": exp,
                                       "sampling_ratio": float(rng.choice([0, 10, 35, 50, 100])),
                                       "fallback_sampling_ratio": float(rng.choice([0, 5, 20]))}})
    levels = {"global_rules": [], "service_rules": [], "endpoint_rules": []}
    for r in rules:
        levels[rng.choice(list(levels))].append(r)

    def value():
        t = rng.randrange(7)
        if t == 0:
            return rng.choice(["prod", "pod", "", "dev", "prxd", "abbc", "ééé", "xprodx", "p\u00e9d"])
        if t == 1:
            return rng.choice([5, -5, 0, 8, 1000, 1001, -1000, 2 ** 62, -(2 ** 53) - 1])
        if t == 2:
            return rng.choice([5.0, 2.5, 2.5000001, -1e3, float("nan"), float("inf"), -0.0, 8.0, 1e300])
        if t == 3:
            return rng.choice([True, False])
        if t == 4:
            return {"arrayValue": {"values": [{"intValue": "1"}]}}
        if t == 5:
            return {"bytesValue": "AAE="}
        return None

    rs = []
    for tr in range(n_traces):
        tid = "%032x" % rng.getrandbits(128)
        for _ in range(rng.randint(1, 3)):
            spans = []
            for j in range(rng.randint(1, 4)):
                attrs = {}
                for key in ("env", "code", "flag"):
                    if rng.random() < 0.6:
                        v = value()
                        if v is not None:
                            attrs[key] = v
                spans.append(host.span(name="s", trace_id=tid, span_id="%016x" % rng.getrandbits(64),
                                       start=BASE, end=BASE + 10, attributes=attrs))
            res = {"service.name": rng.choice(svcs + ["other"])} if rng.random() < 0.95 else {}
            rs.append(host.resource_spans(res, spans))
    rng.shuffle(rs)
    return levels, host.traces(*rs)


@pytest.mark.parametrize("seed", range(6))
def test_random_oracle_vs_host_predicate(seed):
    """The oracle's restatement from the columns equals the product's host
    predicate (span_attr.cpp, the legacy attr_match path) on every trace."""
    cfg, td = _random_attr_case(seed)
    proc = host.Processor("odigossampling", cfg)
    hb = proc.columnarize(td)
    n = hb.cols.n_spans
    from odigos_amd.batch import HostOutputs
    a = HostOutputs(hb.cols)
    assert SamplingOracle(cfg).process(hb.cols, a.outs, native.GROUP_TRACE_ID, SEED) == 0
    # the same rules with every bit from attr_match computed by the host predicate
    bits = np.zeros(max(n, 1), dtype=np.uint64)
    k = 0
    for lvl in ("global_rules", "service_rules", "endpoint_rules"):
        for r in cfg[lvl]:
            d = r["rule_details"]
            i = 0
            for rs in td["resourceSpans"]:
                svc = host.find_attr({"attributes": rs["resource"]["attributes"]}, "service.name")
                for sc in rs["scopeSpans"]:
                    for sp in sc["spans"]:
                        av = host.find_attr(sp, d["attribute_key"])
                        if svc is not None and host.as_string(svc) == d["service_name"] and av is not None \
                                and _eval(d, av):
                            bits[i] |= np.uint64(1 << k)
                        i += 1
            k += 1
    cols = hb.cols
    saved = (cols.attr_type, cols.attr_val, cols.attr_match)
    cols.attr_type = cols.attr_val = None
    cols.attr_match = bits.ctypes.data
    b = HostOutputs(hb.cols)
    try:
        assert SamplingOracle(cfg).process(cols, b.outs, native.GROUP_TRACE_ID, SEED) == 0
    finally:
        cols.attr_type, cols.attr_val, cols.attr_match = saved
    np.testing.assert_array_equal(a.view("keep", np.uint8)[:n], b.view("keep", np.uint8)[:n])
    t = int(a.view("trace_count", np.uint32)[0])
    np.testing.assert_array_equal(a.view("trace_level", np.uint8)[:t], b.view("trace_level", np.uint8)[:t])
    np.testing.assert_array_equal(a.view("trace_ratio", np.float64)[:t], b.view("trace_ratio", np.float64)[:t])


@pytest.mark.parametrize("seed", range(3))
def test_random_past_64_rules_host_words(seed):
    """More than 64 span_attribute rules: the oracle from the key columns
    equals the oracle from attr_match words (bits 64.. in word 1, built here
    from the host predicate), and the columniser's attr_match carries two
    word-major words per span."""
    cfg, td = _random_attr_case(seed, n_traces=80, n_rules=90)
    proc = host.Processor("odigossampling", cfg)
    hb = proc.columnarize(td)
    n = hb.cols.n_spans
    assert hb.cols.attr_match_words == 2
    from odigos_amd.batch import HostOutputs
    a = HostOutputs(hb.cols)
    assert SamplingOracle(cfg).process(hb.cols, a.outs, native.GROUP_TRACE_ID, SEED) == 0
    bits = np.zeros((2, max(n, 1)), dtype=np.uint64)
    k = 0
    for lvl in ("global_rules", "service_rules", "endpoint_rules"):
        for r in cfg[lvl]:
            d = r["rule_details"]
            i = 0
            for rs in td["resourceSpans"]:
                svc = host.find_attr({"attributes": rs["resource"]["attributes"]}, "service.name")
                for sc in rs["scopeSpans"]:
                    for sp in sc["spans"]:
                        av = host.find_attr(sp, d["attribute_key"])
                        if svc is not None and host.as_string(svc) == d["service_name"] and av is not None \
                                and _eval(d, av):
                            bits[k // 64, i] |= np.uint64(1 << (k % 64))
                        i += 1
            k += 1
    assert bits[1].any()
    cols = hb.cols
    saved = (cols.attr_type, cols.attr_val, cols.attr_match)
    cols.attr_type = cols.attr_val = None
    cols.attr_match = bits.ctypes.data
    b = HostOutputs(hb.cols)
    try:
        assert SamplingOracle(cfg).process(cols, b.outs, native.GROUP_TRACE_ID, SEED) == 0
    finally:
        cols.attr_type, cols.attr_val, cols.attr_match = saved
    np.testing.assert_array_equal(a.view("keep", np.uint8)[:n], b.view("keep", np.uint8)[:n])
    t = int(a.view("trace_count", np.uint32)[0])
    np.testing.assert_array_equal(a.view("trace_level", np.uint8)[:t], b.view("trace_level", np.uint8)[:t])
    np.testing.assert_array_equal(a.view("trace_ratio", np.float64)[:t], b.view("trace_ratio", np.float64)[:t])


# ---- GPU --------------------------------------------------------------------

def _gpu(cfg, td):
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    proc = host.Processor("odigossampling", cfg)
    hb = proc.columnarize(td)
    eng = Engine({"odigossampling": cfg})
    db = DeviceBatch(hb.cols)
    eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_BATCH, seed=SEED)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    n = hb.cols.n_spans
    return (int(db.out_numpy("trace_level")[0]), float(db.out_numpy("trace_ratio", np.float64)[0]),
            int(db.out_numpy("trace_keep")[0]), list(db.out_numpy("keep")[:n]))


@pytest.mark.gpu
@pytest.mark.parametrize("c", GOLD["cases"], ids=[c["test"] for c in GOLD["cases"]])
def test_kat_gpu(c):
    cfg = {"global_rules": [_rule(c)]}
    lvl, ratio = _expect(c["expect"])
    got_l, got_r, tk, keep = _gpu(cfg, build_trace(c["service"], c["attrs"]))
    assert (got_l, got_r) == (lvl, ratio)
    assert tk == (lvl == 4 or _u() * 100 < ratio)
    assert all(k == tk for k in keep)


@pytest.mark.gpu
@pytest.mark.parametrize("name,cfg,td,lvl,ratio", COMPOSE, ids=[c[0] for c in COMPOSE])
def test_compose_gpu(name, cfg, td, lvl, ratio):
    got_l, got_r, _, _ = _gpu(cfg, td)
    assert (got_l, got_r) == (lvl, ratio)


@pytest.mark.gpu
def test_consume_gpu():
    # ConsumeTraces drop-in: a 0 % rule on a satisfied trace drops it
    c = dict(ENV, sampling_ratio=0.0)
    cfg = {"global_rules": [{"name": "z", "type": "span_attribute", "rule_details": c}]}
    proc = host.Processor("odigossampling", cfg)
    proc.configure(SEED, native.GROUP_BATCH)
    assert proc.consume(_trace(({"service.name": "svc"}, [{"env": "prod"}])))["resourceSpans"] == []
    out = proc.consume(_trace(({"service.name": "svc"}, [{"env": "dev"}])))
    assert len(out["resourceSpans"]) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_random_gpu_vs_oracle(seed):
    """attr_kernel.hip + the trace stage against the oracle's restatement on
    random rules and values, grouped by trace id."""
    import torch
    from odigos_amd.batch import DeviceBatch, Engine, HostOutputs
    cfg, td = _random_attr_case(seed, n_traces=400)
    proc = host.Processor("odigossampling", cfg)
    hb = proc.columnarize(td)
    n = hb.cols.n_spans
    assert hb.cols.n_attr_keys >= 1
    eng = Engine({"odigossampling": cfg})
    info = eng.info()
    assert info.n_attr_keys == hb.cols.n_attr_keys and info.attr_host_rules == 0
    db = DeviceBatch(hb.cols)
    eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID, seed=SEED)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = HostOutputs(hb.cols)
    assert SamplingOracle(cfg).process(hb.cols, ho.outs, native.GROUP_TRACE_ID, SEED) == 0
    np.testing.assert_array_equal(db.out_numpy("keep", n=n), ho.view("keep", np.uint8)[:n])
    t = int(ho.view("trace_count", np.uint32)[0])
    assert int(db.out_numpy("trace_count", np.uint32)[0]) == t
    np.testing.assert_array_equal(db.out_numpy("trace_level", n=t), ho.view("trace_level", np.uint8)[:t])
    np.testing.assert_array_equal(db.out_numpy("trace_ratio", np.float64, n=t), ho.view("trace_ratio", np.float64)[:t])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_random_gpu_past_64_rules(seed):
    """90 span_attribute rules, a json one among them past bit 64: the GPU
    attr kernel writes two attr_match words, the shim's json bit comes in
    word 1, the trace stage runs the rule chunks; against the oracle."""
    import torch
    from odigos_amd.batch import DeviceBatch, Engine, HostOutputs
    cfg, td = _random_attr_case(seed, n_traces=300, n_rules=90)
    cfg["endpoint_rules"].append({"name": "j", "type": "span_attribute",
                                  "rule_details": dict(_r("json", "is_valid_json"), service_name="svc-a",
                                                       attribute_key="env", sampling_ratio=60.0)})
    proc = host.Processor("odigossampling", cfg)
    hb = proc.columnarize(td)
    n = hb.cols.n_spans
    assert hb.cols.attr_match_words == 2
    eng = Engine({"odigossampling": cfg})
    words = (C.c_uint64 * 4)()
    assert native.lib().ose_engine_attr_host_rules(eng.h, words, 4) == 2
    assert words[0] == 0 and words[1] == 1 << 26          # the json rule is span_attribute rule 90
    db = DeviceBatch(hb.cols)
    eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID, seed=SEED)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = HostOutputs(hb.cols)
    assert SamplingOracle(cfg).process(hb.cols, ho.outs, native.GROUP_TRACE_ID, SEED) == 0
    np.testing.assert_array_equal(db.out_numpy("keep")[:n], ho.view("keep", np.uint8)[:n])
    t = int(ho.view("trace_count", np.uint32)[0])
    np.testing.assert_array_equal(db.out_numpy("trace_level", n=t), ho.view("trace_level", np.uint8)[:t])
    np.testing.assert_array_equal(db.out_numpy("trace_ratio", np.float64, n=t), ho.view("trace_ratio", np.float64)[:t])


@pytest.mark.gpu
def test_json_rules_stay_on_host():
    """A json condition is the shim's (attr_host_rules); its bit and a GPU
    rule's bit combine in one trace decision."""
    import torch
    from odigos_amd.batch import DeviceBatch, Engine, HostOutputs
    cfg = {"global_rules": [
        {"name": "j", "type": "span_attribute", "rule_details": dict(_r("json", "contains_key", path="$.a"),
                                                                     service_name="svc", attribute_key="body",
                                                                     sampling_ratio=40.0)},
        {"name": "s", "type": "span_attribute", "rule_details": dict(ENV, sampling_ratio=25.0)}]}
    td = _trace(({"service.name": "svc"}, [{"body": '{"a": 1}'}, {"env": "prod"}]),
                ({"service.name": "svc"}, [{"body": "[]"}]))
    proc = host.Processor("odigossampling", cfg)
    proc.configure(SEED, native.GROUP_BATCH)
    hb = proc.columnarize(td)
    eng = Engine({"odigossampling": cfg})
    assert eng.info().attr_host_rules == 1 and eng.info().n_attr_keys == 1
    db = DeviceBatch(hb.cols)
    eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_BATCH, seed=SEED)
    torch.cuda.synchronize()
    ho = HostOutputs(hb.cols)
    assert SamplingOracle(cfg).process(hb.cols, ho.outs, native.GROUP_BATCH, SEED) == 0
    assert float(db.out_numpy("trace_ratio", np.float64)[0]) == 40.0 == float(ho.view("trace_ratio", np.float64)[0])
