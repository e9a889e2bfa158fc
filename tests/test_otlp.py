"""OTLP protobuf ingest: a serialized TracesData decoded
into the stages' columns (odigos_amd/csrc/otlp_{pb,host}.cpp, otlp_kernel.hip).

The expected columns come from the host columniser over pdata built from
the OTLP/JSON form of the same traces (the path every other test pins
against the oracle).  The protobuf bytes are produced by google.protobuf
from a descriptor of OTLP trace.proto written in tests/test_size.py, an
encoder independent of the engine.

CPU: the host unmarshaler (otlp_pb.cpp) against the JSON path, and its
rejection of malformed messages (what UnmarshalTraces rejects).
GPU: decoded columns equal the host columniser's, column by column; the
stages on decoded columns equal the oracle chain; spans needing the host
pass (url.full, non-string values, nested values, json span_attribute
keys) are counted and still exact.
"""
import ctypes as C
import json
import random

import numpy as np
import pytest

from odigos_amd import host, native
from tests.test_size import _otlp_classes, _rand_traces

SEED = 0x0D16F00D
SERVICES = ["svc-a", "svc-b", "svc-c", "svc-d"]
CFG = {
    "odigossampling": {
        "global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 40}}],
        "service_rules": [{"name": "s-a", "type": "service_name",
                           "rule_details": {"service_name": "svc-a", "sampling_ratio": 60, "fallback_sampling_ratio": 5}}],
        "endpoint_rules": [
            {"name": "lat", "type": "http_latency",
             "rule_details": {"http_route": "/api", "service_name": "svc-b", "threshold": 20, "fallback_sampling_ratio": 10}},
            {"name": "attr", "type": "span_attribute",
             "rule_details": {"service_name": "svc-c", "attribute_key": "tier", "condition_type": "string",
                              "operation": "equals", "expected_value": "gold", "sampling_ratio": 70}},
            {"name": "num", "type": "span_attribute",
             "rule_details": {"service_name": "svc-d", "attribute_key": "code", "condition_type": "number",
                              "operation": "greater_than", "expected_value": "499", "sampling_ratio": 80}},
        ],
    },
    "odigosurltemplate": {},
    "odigostrafficmetrics": {"res_attributes_keys": ["service.name", "k8s.pod.name"]},
}
CFG_JSON_RULE = json.loads(json.dumps(CFG))
CFG_JSON_RULE["odigossampling"]["endpoint_rules"].append(
    {"name": "js", "type": "span_attribute",
     "rule_details": {"service_name": "svc-a", "attribute_key": "body", "condition_type": "json",
                      "operation": "contains_key", "json_path": "$.a", "sampling_ratio": 90}})
CFG_MANY_KEYS = json.loads(json.dumps(CFG))   # 40 distinct span_attribute keys (the decoder's key roles)
CFG_MANY_KEYS["odigossampling"]["endpoint_rules"] += [
    {"name": f"k{j}", "type": "span_attribute",
     "rule_details": {"service_name": SERVICES[j % len(SERVICES)], "attribute_key": f"k{j}",
                      "condition_type": "string", "operation": "equals", "expected_value": "v",
                      "sampling_ratio": float(j)}} for j in range(40)]
# past 64 span_attribute rules (attr_match in two words): 70 string rules over
# the 40 keys, and the json rule after them (its bit in the second word)
CFG_MANY_RULES = json.loads(json.dumps(CFG_JSON_RULE))
_js = CFG_MANY_RULES["odigossampling"]["endpoint_rules"].pop()
CFG_MANY_RULES["odigossampling"]["endpoint_rules"] += [
    {"name": f"m{j}", "type": "span_attribute",
     "rule_details": {"service_name": SERVICES[j % len(SERVICES)], "attribute_key": f"k{j % 40}",
                      "condition_type": "string", "operation": "equals" if j % 2 else "contains",
                      "expected_value": "v", "sampling_ratio": float(j)}} for j in range(70)] + [_js]
# past the decoder's 56 key roles: 62 distinct string keys (keys 56.. send the
# spans that carry them to the host pass, the others are decoded ABSENT)
CFG_WIDE_KEYS = json.loads(json.dumps(CFG))
CFG_WIDE_KEYS["odigossampling"]["endpoint_rules"] += [
    {"name": f"w{j}", "type": "span_attribute",
     "rule_details": {"service_name": SERVICES[j % len(SERVICES)], "attribute_key": f"k{j}",
                      "condition_type": "string", "operation": "equals", "expected_value": "v",
                      "sampling_ratio": float(j % 100)}} for j in range(60)]
# past 64 shim-evaluated rules: 70 json rules over two keys and every
# service (their bits from the resource's service id in the host pass)
CFG_WIDE_JSON = json.loads(json.dumps(CFG_JSON_RULE))
CFG_WIDE_JSON["odigossampling"]["service_rules"] += [
    {"name": f"j{j}", "type": "span_attribute",
     "rule_details": {"service_name": SERVICES[j % len(SERVICES)], "attribute_key": "body" if j % 3 else "k1",
                      "condition_type": "json", "operation": ["is_valid_json", "is_invalid_json", "contains_key"][j % 3],
                      "json_path": "$.a", "sampling_ratio": float((j * 7) % 101), "fallback_sampling_ratio": float(j % 4)}}
    for j in range(70)]
CFG_EXCLUDE = json.loads(json.dumps(CFG))
CFG_EXCLUDE["odigosurltemplate"] = {"exclude": {"k8s_workloads": [{"namespace": "prod", "kind": "Deployment",
                                                                    "name": "api"}]}}


def _http_traces(rng: random.Random, n_traces: int, odd: float = 0.0, extra_keys: int = 0) -> dict:
    """HTTP-shaped traces; `odd` is the share of spans with values the GPU
    hands to the host pass (url.full, int routes, nested values, events with
    nested attributes)."""
    rss = []
    for t in range(n_traces):
        tid = "%032x" % rng.getrandbits(128) if rng.random() < 0.97 else ""
        for _ in range(rng.randint(1, 3)):
            svc = rng.choice(SERVICES + ["other"])
            res = {"service.name": svc, "k8s.pod.name": f"pod-{rng.randrange(4)}"}
            if rng.random() < 0.3:
                res.update({"k8s.namespace.name": "prod", "k8s.deployment.name": rng.choice(["api", "web"])})
            spans = []
            for _ in range(rng.randint(1, 5)):
                kind = rng.choice([1, 2, 2, 3, 3, 0, 4])
                method = rng.choice(["GET", "POST", "PUT"])
                a = {}
                if rng.random() < 0.9:
                    a["http.request.method" if rng.random() < 0.7 else "http.method"] = method
                r = rng.random()
                uid = rng.randrange(1, 10 ** 9)
                if r < 0.5:
                    a["url.path"] = rng.choice([f"/api/v1/users/{uid}", f"/api/items/{uid:x}a1b2c3d4e5f6a7b8",
                                                "/api/v2/orders", f"/users/x{uid}@example.com/inbox",
                                                "/2025-01-02", "/", ""])
                elif r < 0.7:
                    a["http.target"] = rng.choice([f"/api/search?q={uid}", f"/api/v1/{uid}/details?x=1", "/health"])
                elif r < 0.7 + odd:
                    a["url.full"] = f"https://example.com/api/v1/users/{uid}?x=1"
                if rng.random() < 0.5:
                    a["http.route"] = rng.choice(["/api/v1/users/{id}", "/api", "", "/health"])
                if rng.random() < odd:
                    a["http.route"] = 7                        # AsString of an int
                if kind == 3 and rng.random() < 0.3:
                    a["url.template"] = rng.choice(["", "/t/{id}", 5])
                if rng.random() < 0.3:
                    a["tier"] = rng.choice(["gold", "silver", 3, True])
                if rng.random() < 0.3:
                    a["code"] = rng.choice([200, 500, 503.5, "500"])
                if rng.random() < 0.2:
                    a["body"] = rng.choice(['{"a": 1}', "[]", "{"])
                if rng.random() < odd:
                    a["nested"] = {"arrayValue": {"values": [{"intValue": "1"}]}}
                for j in range(extra_keys):   # span_attribute keys beyond the role word's first 24
                    if rng.random() < 0.15:
                        a[f"k{j}"] = rng.choice(["v", "w", 4, True])
                name = method if rng.random() < 0.4 else rng.choice(["op", "", "GET /x"])
                start = 1739000000000000000 + rng.randrange(10 ** 9)
                sp = host.span(name=name, kind=kind, attributes=a, trace_id=tid,
                               span_id="%016x" % rng.getrandbits(64) if rng.random() < 0.95 else "",
                               start=start if rng.random() < 0.98 else 0,
                               end=start + rng.randrange(10 ** 8) if rng.random() < 0.98 else 0,
                               status=rng.choice([0, 0, 1, 2]))
                if rng.random() < 0.2:
                    sp["parentSpanId"] = "%016x" % rng.getrandbits(64)
                if rng.random() < 0.1:
                    sp["traceState"] = "k=v"
                if rng.random() < 0.1:
                    sp["flags"] = 257
                if rng.random() < 0.1:
                    sp["droppedAttributesCount"] = 3
                if rng.random() < 0.15:
                    sp["events"] = [{"timeUnixNano": str(start + 5), "name": "ev",
                                     "attributes": host.attrs({"e": 1, "f": "x"})}]
                    if rng.random() < odd * 2:
                        sp["events"][0]["attributes"].append({"key": "n", "value": {"kvlistValue": {"values": []}}})
                if rng.random() < 0.1:
                    sp["links"] = [{"traceId": "%032x" % rng.getrandbits(128), "spanId": "%016x" % rng.getrandbits(64),
                                    "traceState": "", "attributes": host.attrs({"l": 2.5}), "flags": 1}]
                if rng.random() < 0.05:
                    sp["status"]["message"] = "boom"
                spans.append(sp)
            rss.append(host.resource_spans(res, spans))
    rng.shuffle(rss)
    return host.traces(*rss)


def _varint(x: int) -> bytes:
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def to_pb(td: dict) -> bytes:
    """TracesData bytes of an OTLP/JSON dict (google.protobuf encoder)."""
    import base64
    cls = _otlp_classes()

    def av(v, m):
        k, x = next(iter(v.items())) if v else (None, None)
        if k == "stringValue":
            m.string_value = x
        elif k == "boolValue":
            m.bool_value = x
        elif k == "intValue":
            m.int_value = int(x)
        elif k == "doubleValue":
            m.double_value = float(x)
        elif k == "bytesValue":
            m.bytes_value = base64.b64decode(x)
        elif k == "arrayValue":
            m.array_value.SetInParent()
            for e in x.get("values", []):
                av(e, m.array_value.values.add())
        elif k == "kvlistValue":
            m.kvlist_value.SetInParent()
            for e in x.get("values", []):
                kv(e, m.kvlist_value.values.add())

    def kv(d, m):
        m.key = d["key"]
        m.value.SetInParent()
        av(d["value"], m.value)

    out = b""
    for rs in td["resourceSpans"]:
        m = cls["ResourceSpans"]()
        m.resource.SetInParent()
        for d in rs["resource"].get("attributes", []):
            kv(d, m.resource.attributes.add())
        m.resource.dropped_attributes_count = int(rs["resource"].get("droppedAttributesCount", 0))
        m.schema_url = rs.get("schemaUrl", "")
        for ss in rs["scopeSpans"]:
            s = m.scope_spans.add()
            sc = ss.get("scope", {})
            s.scope.SetInParent()
            if sc.get("name"):
                s.scope.name = sc["name"]
            if sc.get("version"):
                s.scope.version = sc["version"]
            for d in sc.get("attributes", []):
                kv(d, s.scope.attributes.add())
            s.scope.dropped_attributes_count = int(sc.get("droppedAttributesCount", 0))
            s.schema_url = ss.get("schemaUrl", "")
            for sp in ss["spans"]:
                p = s.spans.add()
                p.trace_id = bytes.fromhex(sp.get("traceId", ""))
                p.span_id = bytes.fromhex(sp.get("spanId", ""))
                p.parent_span_id = bytes.fromhex(sp.get("parentSpanId", ""))
                p.trace_state = sp.get("traceState", "")
                p.name = sp.get("name", "")
                p.kind = sp.get("kind", 0)
                p.start_time_unix_nano = int(sp.get("startTimeUnixNano", "0"))
                p.end_time_unix_nano = int(sp.get("endTimeUnixNano", "0"))
                for d in sp.get("attributes", []):
                    kv(d, p.attributes.add())
                p.dropped_attributes_count = int(sp.get("droppedAttributesCount", 0))
                for ev in sp.get("events", []):
                    e = p.events.add()
                    e.time_unix_nano = int(ev.get("timeUnixNano", "0"))
                    e.name = ev.get("name", "")
                    for d in ev.get("attributes", []):
                        kv(d, e.attributes.add())
                for lk in sp.get("links", []):
                    li = p.links.add()
                    li.trace_id = bytes.fromhex(lk.get("traceId", ""))
                    li.span_id = bytes.fromhex(lk.get("spanId", ""))
                    li.trace_state = lk.get("traceState", "")
                    for d in lk.get("attributes", []):
                        kv(d, li.attributes.add())
                    li.flags = int(lk.get("flags", 0))
                st = sp.get("status") or {}
                if st.get("message"):
                    p.status.message = st["message"]
                if st.get("code"):
                    p.status.code = st["code"]
                p.flags = int(sp.get("flags", 0))
        b = m.SerializeToString()
        out += b"\x0a" + _varint(len(b)) + b
    return out


def _pb_to_json(pb: bytes):
    L = native.lib()
    p = L.osehost_pb_to_json(pb, len(pb))
    if not p:
        return None
    return host.loads(native.take_bytes(p).decode("ascii"))


def _roundtrip(td):
    return host.loads(native.take_bytes(native.lib().osehost_roundtrip(host.dumps(td).encode())).decode("ascii"))


# ---- CPU: the host unmarshaler ----------------------------------------------

@pytest.mark.parametrize("seed", range(8))
def test_host_unmarshal_matches_json(seed):
    rng = random.Random(seed)
    td = _http_traces(rng, 30, odd=0.1) if seed % 2 else _rand_traces(rng, n_res=4)
    assert _pb_to_json(to_pb(td)) == _roundtrip(td)


def test_host_unmarshal_merges_and_unknown_fields():
    # two TracesData messages concatenated merge; unknown fields are skipped
    rng = random.Random(1)
    a, b = _http_traces(rng, 3), _http_traces(rng, 2)
    both = host.traces(*(a["resourceSpans"] + b["resourceSpans"]))
    assert _pb_to_json(to_pb(a) + to_pb(b)) == _roundtrip(both)
    unknown = b"\x18\x05" + b"\x22\x02hi" + b"\x29" + b"\x00" * 8   # fields 3 (varint), 4 (LEN), 5 (fixed64)
    assert _pb_to_json(unknown + to_pb(a)) == _roundtrip(a)


@pytest.mark.parametrize("bad", [
    b"\x0a\x05\x12\x03\x12",                    # truncated ScopeSpans
    b"\x08\x01",                                # resource_spans with a varint wire type
    b"\x0a\x80",                                # truncated length varint
    b"\x0a\x06\x12\x04\x12\x02\x0a\x05",        # span with a 5-byte... (truncated trace_id)
    b"\x0a\x09\x12\x07\x12\x05\x0a\x03abc",     # trace_id of length 3
    b"\x0a\x06\x12\x04\x12\x02\x30\x80",        # truncated kind varint
    b"\x0c",                                    # end group at top level
])
def test_host_unmarshal_rejects(bad):
    assert _pb_to_json(bad) is None


# ---- GPU ---------------------------------------------------------------------------

def _host_columns(cfg, td):
    proc = host.Processor("pipeline", cfg)
    return proc, proc.columnarize(td)


def _arr(addr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array((C.c_uint8 * (n * np.dtype(dtype).itemsize)).from_address(addr)).view(dtype).copy()


def _strings(arena, refs):
    return [bytes(arena[o:o + l]) for o, l in refs]


def _compare(cols, hb_cols, got):
    n, R, S, K = hb_cols.n_spans, hb_cols.n_resources, hb_cols.n_scopes, hb_cols.n_attr_keys
    assert (cols.n_spans, cols.n_resources, cols.n_scopes, cols.n_attrsets, cols.n_attr_keys) == \
        (n, R, S, hb_cols.n_attrsets, K)
    want = {
        "trace_id": (2 * n, np.uint64), "start_ns": (n, np.uint64), "end_ns": (n, np.uint64),
        "status": (n, np.uint8), "kind": (n, np.uint8), "resource": (n, np.uint32), "scope": (n, np.uint32),
        "url_flags": (n, np.uint8), "span_size": (n, np.uint32), "name_len": (n, np.uint32),
        "res_svc": (R, np.uint32), "res_svc_str": (R, np.uint32), "res_attrset": (R, np.uint32),
        "res_size": (R, np.uint32), "scope_size": (S, np.uint32), "scope_resource": (S, np.uint32),
    }
    if cols.res_url_ok:
        want["res_url_ok"] = (R, np.uint8)
    for name, (cnt, dt) in want.items():
        np.testing.assert_array_equal(got[name].view(dt)[:cnt], _arr(getattr(hb_cols, name), cnt, dt), err_msg=name)
    harena = _arr(hb_cols.arena, hb_cols.arena_bytes, np.uint8)
    garena = got["arena"]
    for name in ("route", "path"):
        g = got[name].view(np.uint32).reshape(-1, 2)[:n]
        h = _arr(getattr(hb_cols, name), 2 * n, np.uint32).reshape(-1, 2)
        if name == "path":   # refs matter where a path source is set
            m = (_arr(hb_cols.url_flags, n, np.uint8) & native.URL_PATH_MASK) != 0
            g, h = g[m], h[m]
        assert _strings(garena, g) == _strings(harena, h), name
    if K:
        gt = got["attr_type"][:K * n]
        np.testing.assert_array_equal(gt, _arr(hb_cols.attr_type, K * n, np.uint8))
        gv = got["attr_val"].view(np.uint64)[:K * n]
        hv = _arr(hb_cols.attr_val, K * n, np.uint64)
        s = gt == native.ATTR_STR
        np.testing.assert_array_equal(gv[~s], hv[~s])
        g2 = np.stack([gv[s] & 0xFFFFFFFF, gv[s] >> 32], 1)
        h2 = np.stack([hv[s] & 0xFFFFFFFF, hv[s] >> 32], 1)
        assert _strings(garena, g2) == _strings(harena, h2)
    if got.get("attr_match") is not None and hb_cols.attr_match:
        W = max(1, hb_cols.attr_match_words)
        assert max(1, cols.attr_match_words) == W
        np.testing.assert_array_equal(got["attr_match"].view(np.uint64)[:W * n],
                                      _arr(hb_cols.attr_match, W * n, np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,odd,cfg", [(0, 0.0, "base"), (1, 0.0, "base"), (2, 0.15, "base"), (3, 0.1, "json"),
                                          (4, 0.0, "exclude"), (5, 0.3, "json"), (6, 0.0, "many_keys"),
                                          (7, 0.1, "many_rules"), (8, 0.0, "wide_keys"), (9, 0.1, "wide_json")])
def test_gpu_decode_matches_host_columns(seed, odd, cfg):
    from odigos_amd.batch import Engine, OtlpBatch
    c = {"base": CFG, "json": CFG_JSON_RULE, "exclude": CFG_EXCLUDE, "many_keys": CFG_MANY_KEYS,
         "many_rules": CFG_MANY_RULES, "wide_keys": CFG_WIDE_KEYS, "wide_json": CFG_WIDE_JSON}[cfg]
    rng = random.Random(seed)
    td = _http_traces(rng, 200, odd=odd, extra_keys={"many_keys": 40, "many_rules": 40, "wide_keys": 62,
                                                     "wide_json": 4}.get(cfg, 0))
    _, hb = _host_columns(c, td)
    eng = Engine(c)
    ob = OtlpBatch(eng, to_pb(td))
    if odd == 0.0 and cfg not in ("json", "many_rules", "wide_keys", "wide_json"):
        assert ob.host_spans == 0
    else:
        assert ob.host_spans > 0
    _compare(ob.cols, hb.cols, ob.download())


@pytest.mark.gpu
def test_gpu_resource_walk_cold_warm_and_host():
    # the ResourceSpans level on the GPU (otlp_res_fields_kernel): a cold
    # engine resolves every resource on the host and enters it in the device
    # table, a second decode finds them all there; both equal the host
    # columniser and the host ResourceSpans walk (engine option otlp_host_resources)
    from odigos_amd.batch import Engine, OtlpBatch
    td = _http_traces(random.Random(31), 300, odd=0.05)
    _, hb = _host_columns(CFG, td)
    pb = to_pb(td)
    eng = Engine(CFG)
    for _ in range(2):
        ob = OtlpBatch(eng, pb)
        _compare(ob.cols, hb.cols, ob.download())
        ob.close()
    eng.set_option("otlp_host_resources", 1)
    ob = OtlpBatch(eng, pb)
    _compare(ob.cols, hb.cols, ob.download())
    eng.set_option("otlp_host_resources", 0)
    # a message of several copies (resources repeated, table hits in one call)
    td3 = {"resourceSpans": td["resourceSpans"] * 3}
    _, hb3 = _host_columns(CFG, td3)
    ob3 = OtlpBatch(Engine(CFG), to_pb(td3))
    _compare(ob3.cols, hb3.cols, ob3.download())
    # the TracesData chain walked on the GPU (engine option otlp_gpu_chain) equals the host's
    eng4 = Engine(CFG)
    eng4.set_option("otlp_gpu_chain", 1)
    ob4 = OtlpBatch(eng4, to_pb(td3))
    _compare(ob4.cols, hb3.cols, ob4.download())


@pytest.mark.gpu
def test_gpu_chain_walk_records_over_segments():
    # ResourceSpans records larger than the GPU chain walk's 64 KiB segments
    # (whole segments inside one record) between small ones, and a message
    # whose bytes end inside a record (malformed: the host walk reports it)
    from odigos_amd.batch import Engine, OtlpBatch
    rng = random.Random(41)
    td = _http_traces(rng, 120)
    rss = td["resourceSpans"]
    big = host.resource_spans({"service.name": "big", "k8s.pod.name": "pod-0"},
                              [sp for r in rss[:40] for ss in r["scopeSpans"] for sp in ss["spans"]] * 30)
    td2 = host.traces(*(rss[40:80] + [big] + rss[80:] + [big]))
    pb = to_pb(td2)
    assert len(pb) > 3 * (64 << 10)
    _, hb = _host_columns(CFG, td2)
    eng = Engine(CFG)
    eng.set_option("otlp_gpu_chain", 1)
    ob = OtlpBatch(eng, pb)
    _compare(ob.cols, hb.cols, ob.download())
    with pytest.raises(native.OseError) as ei:
        OtlpBatch(eng, pb[: len(pb) - 1000])
    assert ei.value.code == native.OSE_EINVAL


@pytest.mark.gpu
def test_gpu_decode_generic_traces():
    # the size test's generator: nested values, random keys, empty ids
    from odigos_amd.batch import Engine, OtlpBatch
    eng = Engine(CFG)
    for seed in range(6):
        td = _rand_traces(random.Random(100 + seed), n_res=6)
        _, hb = _host_columns(CFG, td)
        ob = OtlpBatch(eng, to_pb(td))
        _compare(ob.cols, hb.cols, ob.download())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["base", "json", "many_rules", "wide_keys", "wide_json"])
def test_gpu_stages_on_decoded_columns(cfg):
    """SAMPLE|TEMPLATE|SIZE on the decoded columns equals the oracle chain on
    the host columniser's batch (decisions, templates, counters); many_rules:
    71 span_attribute rules, attr_match in two words; wide_keys: 62 attribute
    keys (past the decoder's 56 key roles); wide_json: 71 json rules (past the
    64 the per-resource word holds)."""
    import torch
    from odigos_amd.batch import Engine, HostOutputs, OtlpBatch
    from tests.oracle_lib import SamplingOracle, UrlOracle, size_process
    c = {"base": CFG, "json": CFG_JSON_RULE, "many_rules": CFG_MANY_RULES, "wide_keys": CFG_WIDE_KEYS,
         "wide_json": CFG_WIDE_JSON}[cfg]
    td = _http_traces(random.Random(77), 400, odd=0.05,
                      extra_keys={"many_rules": 40, "wide_keys": 62, "wide_json": 4}.get(cfg, 0))
    _, hb = _host_columns(c, td)
    eng = Engine(c)
    ob = OtlpBatch(eng, to_pb(td))
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=SEED)
    torch.cuda.synchronize()
    cols = hb.cols
    ho = HostOutputs(cols)
    assert SamplingOracle(c["odigossampling"]).process(cols, ho.outs, native.GROUP_TRACE_ID, SEED, 4) == 0
    assert UrlOracle(c["odigosurltemplate"]).process(cols, ho.outs, 4) == 0
    assert size_process(cols, ho.outs, st, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, 4) == 0
    n, A = cols.n_spans, cols.n_attrsets
    np.testing.assert_array_equal(ob.out_numpy("keep", n=n), ho.view("keep", np.uint8)[:n])
    np.testing.assert_array_equal(ob.out_numpy("url_out", n=n), ho.view("url_out", np.uint8)[:n])
    used = ob.used()
    assert used == int(ho.used[0])
    np.testing.assert_array_equal(ob.out_numpy("tmpl_arena", n=used), ho.bufs["tmpl_arena"][:used])
    np.testing.assert_array_equal(ob.out_numpy("attrset_bytes", np.int64, n=A), ho.view("attrset_bytes", np.int64)[:A])
    assert int(ob.out_numpy("accepted_spans", np.int64, n=1)[0]) == int(ho.view("accepted_spans", np.int64)[0])
    assert set(ob.attrset(0)) <= {"service.name", "k8s.pod.name"}


@pytest.mark.gpu
def test_gpu_decode_rejects_malformed():
    from odigos_amd.batch import Engine, OtlpBatch
    eng = Engine(CFG)
    td = _http_traces(random.Random(5), 10)
    pb = to_pb(td)
    with pytest.raises(native.OseError) as ei:
        OtlpBatch(eng, pb[:-3])
    assert ei.value.code == native.OSE_EINVAL
    # an empty message decodes to an empty batch
    ob = OtlpBatch(eng, b"")
    assert ob.cols.n_spans == 0


# ---- CPU: the threaded structural walk of the ingest --------------------------------

def _walk(cfg, pb):
    L = native.lib()
    p = L.osehost_otlp_walk(json.dumps(cfg).encode(), pb, len(pb))
    if not p:
        return None
    return json.loads(native.take_bytes(p).decode("ascii"))


def _check_walk(cfg, pb):
    w = _walk(cfg, pb)
    td = _pb_to_json(pb)
    _, hb = _host_columns(cfg, td)
    c = hb.cols
    n, R, S = c.n_spans, c.n_resources, c.n_scopes
    assert len(w["span_ref"]) == n and len(w["res_svc"]) == R and len(w["scope_size"]) == S
    for name, col, cnt, dt in (("span_res", "resource", n, np.uint32), ("span_scope", "scope", n, np.uint32),
                               ("res_svc", "res_svc", R, np.uint32), ("res_svc_str", "res_svc_str", R, np.uint32),
                               ("res_attrset", "res_attrset", R, np.uint32), ("res_size", "res_size", R, np.uint32),
                               ("scope_size", "scope_size", S, np.uint32), ("scope_res", "scope_resource", S, np.uint32)):
        np.testing.assert_array_equal(np.array(w[name], dtype=dt), _arr(getattr(c, col), cnt, dt), err_msg=name)
    if cfg.get("odigosurltemplate", {}).get("exclude"):
        np.testing.assert_array_equal(np.array(w["res_ok"], dtype=np.uint8), _arr(c.res_url_ok, R, np.uint8))
    assert w["n_sets"] == c.n_attrsets
    # every span reference frames a Span payload inside the message
    refs = np.array(w["span_ref"], dtype=np.uint64)
    assert ((refs & 0xFFFFFFFF) + (refs >> 32) <= len(pb)).all()


@pytest.mark.parametrize("seed", range(4))
def test_walk_matches_host_columns(seed):
    rng = random.Random(seed)
    td = _http_traces(rng, 60, odd=0.1) if seed % 2 else _rand_traces(rng, n_res=5)
    _check_walk([CFG, CFG_EXCLUDE][seed % 2], to_pb(td))


def test_walk_threaded_generated_batch():
    # enough resources for the threaded walk (>= 1024), repeated resource and
    # scope messages (the caches)
    from odigos_amd.batch import Generator
    g = Generator("fused", seed=0x0D16F001, n_spans=30_000, threads=4)
    _check_walk(CFG_EXCLUDE, g.otlp(4))


def test_walk_rejects_malformed():
    assert _walk(CFG, b"\x0a\x05\x12\x03\x12") is None


def test_walk_gpu_scopes_resources_match():
    # the walk ose_otlp_decode runs leaves ScopeSpans to the GPU: the host
    # lists no span, and its resource columns equal the full walk's
    from odigos_amd.batch import Generator
    g = Generator("fused", seed=0x0D16F002, n_spans=30_000, threads=4)
    pb = g.otlp(4)
    full = _walk(CFG_EXCLUDE, pb)
    part = _walk(dict(CFG_EXCLUDE, gpu_scopes=True), pb)
    assert len(part["span_ref"]) == 0 and len(full["span_ref"]) == 30_000
    for k in ("res_svc", "res_svc_str", "res_attrset", "res_size", "res_ok", "n_sets"):
        assert part[k] == full[k], k
    assert len(part["scope_size"]) == len(full["scope_size"])
