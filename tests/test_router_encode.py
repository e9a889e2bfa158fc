"""The output side: odigosrouterconnector's routing and
the processed traces re-encoded as OTLP protobuf per pipeline
(odigos_amd/csrc/otlp_encode.cpp, ose_router_* / ose_otlp_encode).

CPU: the connector's own test cases (connector_test.go:10-80) and the
routing-map rules (routingmap.go) against the product's router; random
resources against the restatement in tests/otlp_gogo.py.  The encoder,
through its CPU seam, against tests/otlp_gogo.py: the Python restatement of
the processors' writes and of pdata's marshaler, byte for byte, for inputs
already in pdata's encoding (copied / edited in place) and for inputs
written by google.protobuf (empty ids and Status omitted: re-marshaled).
GPU: decode → SAMPLE|TEMPLATE|SIZE → ose_otlp_encode equals the same
restatement applied with the decisions the GPU made; on a generated batch
it equals the CPU seam fed those decisions.
"""
import ctypes as C
import json
import random

import numpy as np
import pytest

from odigos_amd import host, native
from odigos_amd.batch import Router, take_otlp_out
from tests import otlp_gogo as gg
from tests.test_otlp import CFG, SEED, _http_traces, _pb_to_json, _roundtrip, to_pb
from tests.test_size import _rand_traces

# ---- routing -------------------------------------------------------------------------

# connector_test.go:11-21's SignalRoutingMap as the data streams that build it
KAT_STREAMS = [
    {"name": "traces/B", "sources": [{"namespace": "default", "kind": "Deployment", "name": "my-app"}],
     "destinations": [{"destinationname": "d1", "configuredsignals": ["traces"]}]},
    {"name": "logs/A", "sources": [{"namespace": "default", "kind": "DaemonSet", "name": "log-agent"}],
     "destinations": [{"destinationname": "d2", "configuredsignals": ["logs"]}]},
    {"name": "logs/B", "sources": [{"namespace": "default", "kind": "daemonset", "name": "log-agent"}],
     "destinations": [{"destinationname": "d3", "configuredsignals": ["logs"]}]},
    {"name": "metrics/X", "sources": [{"namespace": "default", "kind": "StatefulSet", "name": "metricsd"}],
     "destinations": [{"destinationname": "d4", "configuredsignals": ["metrics"]}]},
]


@pytest.mark.parametrize("attrs,signal,key,pipelines", [
    ({"k8s.namespace.name": "default", "k8s.deployment.name": "my-app"}, "traces", "default/deployment/my-app",
     ["traces/B"]),
    ({"k8s.namespace.name": "default", "k8s.daemonset.name": "log-agent"}, "logs", "default/daemonset/log-agent",
     ["logs/A", "logs/B"]),
    ({"k8s.namespace.name": "default", "k8s.statefulset.name": "metricsd"}, "metrics", "default/statefulset/metricsd",
     ["metrics/X"]),
    ({"k8s.deployment.name": "my-app"}, "traces", "", []),                                   # missing namespace
    ({"k8s.namespace.name": "default"}, "traces", "", []),                                   # missing workload
    ({"k8s.namespace.name": "default", "k8s.deployment.name": "ghost"}, "traces", "", []),   # not in map
])
def test_routing_kats(attrs, signal, key, pipelines):
    r = Router({"datastreams": KAT_STREAMS}, signal=signal)
    got, k = r.route(attrs)
    assert k == key
    assert sorted(got) == sorted(pipelines)


def test_routing_map_rules():
    streams = [
        # NormalizeKind: the five workload kinds case-folded, others kept as written
        {"name": "a", "sources": [{"namespace": "ns", "kind": "DEPLOYMENT", "name": "w1"},
                                  {"namespace": "ns", "kind": "Rollout", "name": "w2"}],
         "destinations": [{"destinationname": "x", "configuredsignals": ["TRACES"]}]},
        # duplicate names across streams collapse (appendIfMissing)
        {"name": "a", "sources": [{"namespace": "ns", "kind": "Deployment", "name": "w1"}],
         "destinations": [{"destinationname": "y", "configuredsignals": ["TRACES", "TRACES"]}]},
        # only the first three distinct signals count (GetSignalsForDataStream maxSignals)
        {"name": "b", "sources": [{"namespace": "ns", "kind": "Deployment", "name": "w1"}],
         "destinations": [{"destinationname": "z", "configuredsignals": ["LOGS", "METRICS"]},
                          {"destinationname": "z2", "configuredsignals": ["PROFILES", "TRACES"]}]},
        # a stream without TRACES is not a traces pipeline
        {"name": "c", "sources": [{"namespace": "ns", "kind": "StatefulSet", "name": "db"}],
         "destinations": [{"destinationname": "w", "configuredsignals": ["LOGS"]}]},
        {"name": "d", "sources": [{"namespace": "ns", "kind": "statefulset", "name": "db"}],
         "destinations": [{"destinationname": "w", "configuredsignals": ["METRICS", "TRACES"]}]},
    ]
    r = Router({"datastreams": streams})
    assert r.pipelines == ["a", "d"]
    assert r.route({"k8s.namespace.name": "ns", "k8s.deployment.name": "w1"}) == (["a"], "ns/deployment/w1")
    assert r.route({"k8s.namespace.name": "ns", "k8s.statefulset.name": "db"}) == (["d"], "ns/statefulset/db")
    # resources only ever carry the three semconv kinds: a Rollout source never matches
    assert r.route({"k8s.namespace.name": "ns", "k8s.deployment.name": "w2"}) == ([], "")
    # Value.Str() of a non-string namespace is ""
    assert r.route({"k8s.namespace.name": 5, "k8s.deployment.name": "w1"}) == ([], "")
    assert gg.normalize_kind("DeploymentConfig") == "deploymentconfig" and gg.normalize_kind("CronJob") == "cronjob"
    assert Router({}).pipelines == [] and Router({"datastreams": None}).pipelines == []
    with pytest.raises(native.OseError):
        Router({"datastreams": 3})


def _streams(rng):
    ns = ["prod", "default", "dev"]
    wl = [("Deployment", "api"), ("Deployment", "web"), ("StatefulSet", "db"), ("DaemonSet", "agent"),
          ("deployment", "api"), ("CronJob", "batch")]
    out = []
    for k in range(rng.randint(1, 5)):
        sig = rng.sample(["TRACES", "LOGS", "METRICS"], rng.randint(1, 3))
        out.append({"name": "ds-%d" % rng.randrange(4),
                    "sources": [{"namespace": rng.choice(ns), "kind": w[0], "name": w[1]}
                                for w in rng.sample(wl, rng.randint(1, 3))],
                    "destinations": [{"destinationname": "d%d" % k, "configuredsignals": sig}]})
    return out


def _routing_attrs(rng) -> dict:
    a = {}
    if rng.random() < 0.85:
        a["k8s.namespace.name"] = rng.choice(["prod", "default", "dev", "other"])
    key = rng.choice(["k8s.deployment.name", "k8s.statefulset.name", "k8s.daemonset.name", None])
    if key:
        a[key] = rng.choice(["api", "web", "db", "agent", "batch", "x"])
    return a


def test_routing_random_matches_restatement():
    rng = random.Random(0x40D7)
    for _ in range(30):
        streams = _streams(rng)
        r = Router({"datastreams": streams})
        m = gg.build_routing_map(streams)
        assert set(r.pipelines) == {d["name"] for d in streams if "TRACES" in gg.signals_for(d)}
        for _ in range(40):
            a = _routing_attrs(rng)
            want, key = gg.route(host.attrs(a), m, "TRACES")
            got, gkey = r.route(a)
            assert (got, gkey) == (want or [], key), a


# ---- the encoder (CPU seam) ----------------------------------------------------------

def _encode_seam(pb, keep=None, url_out=None, tmpls=None, drop_all=False, router=None, threads=1):
    L = native.lib()
    keep_a = None if keep is None else np.ascontiguousarray(keep, dtype=np.uint8)
    url_a = None if url_out is None else np.ascontiguousarray(url_out, dtype=np.uint8)
    refs = arena = None
    if tmpls is not None:
        bs = [t.encode("utf-8", "surrogateescape") for t in tmpls]
        arena = np.frombuffer(b"".join(bs) + b"\0" * 16, dtype=np.uint8).copy()
        refs = np.zeros((len(bs) + 1, 2), dtype=np.uint32)
        off = 0
        for i, b in enumerate(bs):
            refs[i] = (off, len(b))
            off += len(b)
    ptr = lambda a: None if a is None else a.ctypes.data   # noqa: E731
    h = C.c_void_p()
    native.check(L.osehost_otlp_encode(pb, len(pb), ptr(keep_a), int(drop_all), ptr(url_a), ptr(refs), ptr(arena),
                                       0 if arena is None else len(arena) - 16,
                                       router.h if router is not None else None, threads, C.byref(h)))
    return take_otlp_out(L, h)


def _routable(td, rng):
    """Resources given k8s workload attributes, scopes and schema URLs the
    encoder must carry (several scopes, empty scopes, spanless resources)."""
    for rs in td["resourceSpans"]:
        rs["resource"]["attributes"] += host.attrs(_routing_attrs(rng))
        if rng.random() < 0.2:
            rs["schemaUrl"] = "https://opentelemetry.io/schemas/1.26.0"
        if rs["scopeSpans"] and rng.random() < 0.3:
            rs["scopeSpans"][0]["scope"] = {"name": "lib", "version": "1.%d" % rng.randrange(3),
                                            "attributes": host.attrs({"s": rng.randrange(3)})}
            rs["scopeSpans"][0]["schemaUrl"] = "s%d" % rng.randrange(2)
        if len(rs["scopeSpans"]) == 1 and rng.random() < 0.2:
            sp = rs["scopeSpans"][0]["spans"]
            cut = rng.randrange(len(sp) + 1)
            rs["scopeSpans"] = [{"scope": {"name": "a"}, "spans": sp[:cut]},
                                {"scope": {"name": "b"}, "spans": sp[cut:]}]
        if rng.random() < 0.05:
            rs["scopeSpans"].append({"scope": {"name": "empty"}, "spans": []})
    if td["resourceSpans"] and rng.random() < 0.5:
        td["resourceSpans"].insert(rng.randrange(len(td["resourceSpans"])),
                                   host.resource_spans({"service.name": "idle"}, scopes=[]))
    return td


def _decisions(td, rng, p_keep=0.6):
    spans = [sp for rs in td["resourceSpans"] for ss in rs["scopeSpans"] for sp in ss["spans"]]
    n = len(spans)
    keep = [1 if rng.random() < p_keep else 0 for _ in range(n)]
    url_out = [rng.choice([0, 0, 1, 2, 3]) for _ in range(n)]
    tmpls = [rng.choice(["/api/v1/users/{id}", "", "/items/{id}/x", "/é/{id}"]) if u else "" for u in url_out]
    return keep, url_out, tmpls


def _expected(td, streams, pipelines, **dec):
    applied = gg.apply(td, **dec)
    if streams is None:
        return [("", gg.marshal_traces(applied), len(applied["resourceSpans"]))]
    return [(p, gg.marshal_traces(t), len(t["resourceSpans"]))
            for p, t in gg.split_by_pipeline(applied, streams, pipelines)]


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("encoding", ["pdata", "google"])
def test_encode_matches_restatement(seed, encoding):
    rng = random.Random(seed * 7 + (encoding == "google"))
    td = _http_traces(rng, 40, odd=0.1) if seed % 3 else _rand_traces(rng, n_res=6)
    td = _routable(td, rng)
    td = _roundtrip(td)   # pdata's view of it (what both encodings decode to)
    pb = gg.marshal_traces(td) if encoding == "pdata" else to_pb(td)
    assert _pb_to_json(pb) == td
    streams = _streams(rng)
    router = Router({"datastreams": streams})
    keep, url_out, tmpls = _decisions(td, rng)
    want = _expected(td, streams, router.pipelines, keep=keep, url_out=url_out, tmpls=tmpls)
    for threads in (1, 3):
        got = _encode_seam(pb, keep, url_out, tmpls, router=router, threads=threads)
        assert [g[0] for g in got] == [w[0] for w in want]
        for g, w in zip(got, want):
            assert g[2] == w[2], g[0]
            assert g[1] == w[1], g[0]
    # no router: one output with every kept resource
    got = _encode_seam(pb, keep, url_out, tmpls)
    assert got == _expected(td, None, None, keep=keep, url_out=url_out, tmpls=tmpls)


def test_encode_identity_and_drop_all():
    rng = random.Random(11)
    td = _roundtrip(_routable(_http_traces(rng, 30), rng))
    pb = gg.marshal_traces(td)
    # nothing decided: pdata's encoding comes back unchanged
    assert _encode_seam(pb) == [("", pb, len(td["resourceSpans"]))]
    # a google.protobuf encoding comes back in pdata's
    assert _encode_seam(to_pb(td)) == [("", pb, len(td["resourceSpans"]))]
    # OSE_GROUP_BATCH, unsampled: every resource goes, spanless ones too
    r = Router({"datastreams": _streams(rng)})
    got = _encode_seam(pb, drop_all=True, router=r)
    assert all(g[1] == b"" and g[2] == 0 for g in got) and len(got) == len(r.pipelines) + 1
    # nothing kept: the resources that had spans go, spanless ones stay
    n = sum(len(ss["spans"]) for rs in td["resourceSpans"] for ss in rs["scopeSpans"])
    got = _encode_seam(pb, keep=[0] * n)
    assert got == _expected(td, None, None, keep=[0] * n)
    assert _encode_seam(b"") == [("", b"", 0)]


def test_encode_unusual_encodings():
    """Merged Resource / scope fields, schema URLs written twice, unknown
    fields: what pdata decodes them to, marshaled as pdata would."""
    rng = random.Random(5)
    td = _roundtrip(_http_traces(rng, 6))
    pb = gg.marshal_traces(td)
    # a TracesData with an unknown top-level field, then a resource whose
    # Resource and scope arrive in two fields each and a schema_url twice
    res = gg._len(1, gg.key_value({"key": "k8s.namespace.name", "value": {"stringValue": "prod"}}))
    res2 = gg._len(1, gg.key_value({"key": "k8s.deployment.name", "value": {"stringValue": "api"}}))
    sp = gg.span(td["resourceSpans"][0]["scopeSpans"][0]["spans"][0])
    ss = gg._len(1, gg._str(1, "lib")) + gg._len(2, sp) + gg._len(1, gg._str(2, "v2")) + gg._str(3, "u1") + \
        gg._str(3, "u2") + b"\x20\x07"
    rsb = gg._len(1, res) + gg._len(2, ss) + gg._len(1, res2) + gg._str(3, "x") + gg._str(3, "y")
    odd = b"\x10\x01" + gg._len(1, rsb)
    msg = pb + odd
    want_td = _pb_to_json(msg)
    assert want_td is not None
    streams = [{"name": "p", "sources": [{"namespace": "prod", "kind": "Deployment", "name": "api"}],
                "destinations": [{"destinationname": "d", "configuredsignals": ["TRACES"]}]}]
    r = Router({"datastreams": streams})
    n = sum(len(ss["spans"]) for rs in want_td["resourceSpans"] for ss in rs["scopeSpans"])
    url_out = [3] * n
    tmpls = ["/t/{id}"] * n
    got = _encode_seam(msg, url_out=url_out, tmpls=tmpls, router=r, threads=2)
    want = _expected(want_td, streams, r.pipelines, url_out=url_out, tmpls=tmpls)
    assert got == want
    assert got[0][2] >= 1   # the merged resource routes (its two Resource fields merged)


def test_encode_rejects_bad_template_reference():
    td = _roundtrip(_http_traces(random.Random(3), 2))
    pb = gg.marshal_traces(td)
    n = sum(len(ss["spans"]) for rs in td["resourceSpans"] for ss in rs["scopeSpans"])
    L = native.lib()
    url = np.ones(n, dtype=np.uint8)
    refs = np.full((n, 2), 1000, dtype=np.uint32)
    arena = np.zeros(32, dtype=np.uint8)
    h = C.c_void_p()
    rc = L.osehost_otlp_encode(pb, len(pb), None, 0, url.ctypes.data, refs.ctypes.data, arena.ctypes.data, 16, None,
                               1, C.byref(h))
    assert rc == native.OSE_EINVAL


# ---- GPU -----------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("group_mode", [native.GROUP_TRACE_ID, native.GROUP_BATCH])
def test_gpu_encode_after_stages(group_mode):
    """decode → SAMPLE|TEMPLATE|SIZE → encode + route equals the restatement
    with the decisions the GPU made (those equal the oracle's:
    test_otlp.py::test_gpu_stages_on_decoded_columns)."""
    import torch
    from odigos_amd.batch import Engine, OtlpBatch
    rng = random.Random(0xE7C0 + group_mode)
    td = _roundtrip(_routable(_http_traces(rng, 300 if group_mode == native.GROUP_TRACE_ID else 3, odd=0.05), rng))
    streams = _streams(rng)
    router = Router({"datastreams": streams})
    eng = Engine(CFG)
    for encoding in ("pdata", "google"):
        pb = gg.marshal_traces(td) if encoding == "pdata" else to_pb(td)
        ob = OtlpBatch(eng, pb)
        st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
        for seed in (SEED, SEED + 1):
            eng.process_device(ob, st, group_mode, seed=seed)
            torch.cuda.synchronize()
            n = ob.cols.n_spans
            url_out = ob.out_numpy("url_out", n=n)
            refs = ob.out_numpy("tmpl", np.uint32, n=2 * n).reshape(-1, 2)
            arena = ob.out_numpy("tmpl_arena", n=ob.used()).tobytes()
            tmpls = [arena[o:o + ln].decode("utf-8", "surrogateescape") if u else ""
                     for (o, ln), u in zip(refs, url_out)]
            if group_mode == native.GROUP_BATCH:
                tk = int(ob.out_numpy("trace_keep", n=1)[0])
                dec = {"drop_all": not tk}
            else:
                dec = {"keep": list(ob.out_numpy("keep", n=n))}
            want = _expected(td, streams, router.pipelines, url_out=list(url_out), tmpls=tmpls, **dec)
            got = ob.encode(st, group_mode, router)
            assert got == want
        ob.close()


@pytest.mark.gpu
def test_gpu_encode_generated_batch():
    """A generated C4 batch (pdata's encoding, 200k spans): the GPU path's
    outputs equal the CPU seam's with the same decisions; kept spans are the
    ones keep says, edited as url_out says."""
    import torch
    from odigos_amd.batch import Engine, Generator, OtlpBatch
    from tests.workloads import c3_sampling_config
    g = Generator("fused", seed=0x0E7C, n_spans=200_000, threads=8)
    pb = g.otlp(8)
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": ["service.name"]}}
    eng = Engine(cfg)
    ob = OtlpBatch(eng, pb)
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=SEED)
    torch.cuda.synchronize()
    n = ob.cols.n_spans
    keep = ob.out_numpy("keep", n=n)
    url_out = ob.out_numpy("url_out", n=n)
    refs = ob.out_numpy("tmpl", np.uint32, n=2 * n).reshape(-1, 2)
    arena = ob.out_numpy("tmpl_arena", n=ob.used()).tobytes()
    assert 0 < keep.sum() < n and (url_out != 0).sum() > n // 10
    got = ob.encode(st)
    assert ob.encode_path == {"gpu": True, "fallback": 0}   # written by the GPU encoder
    L = native.lib()
    arena_a = np.frombuffer(arena + b"\0" * 16, dtype=np.uint8).copy()
    refs_a = np.ascontiguousarray(refs)
    keep_a, url_a = np.ascontiguousarray(keep), np.ascontiguousarray(url_out)
    h = C.c_void_p()
    native.check(L.osehost_otlp_encode(pb, len(pb), keep_a.ctypes.data, 0, url_a.ctypes.data, refs_a.ctypes.data,
                                       arena_a.ctypes.data, len(arena), None, 4, C.byref(h)))
    want = take_otlp_out(L, h)
    assert got == want
    # spot check: the kept spans, in order, decoded
    out_td = _pb_to_json(got[0][1])
    names = [sp["name"] for rs in out_td["resourceSpans"] for ss in rs["scopeSpans"] for sp in ss["spans"]]
    assert len(names) == int(keep.sum())
    ob.close()


def test_encode_concurrent_callers():
    """Calls from several threads at once share the host task pool (each
    caller helps run the queued work): every result equals the serial one."""
    import threading
    from odigos_amd.batch import Generator
    g = Generator("fused", seed=0x7A5C, n_spans=40_000, threads=4)
    pb = g.otlp(4)
    n = g.cols.n_spans
    rng = np.random.default_rng(3)
    keep = (rng.random(n) < 0.5).astype(np.uint8)
    url = rng.choice(np.array([0, 1, 2, 3], dtype=np.uint8), n)
    tmpls = ["/a/{id}"] * n
    want = _encode_seam(pb, keep, url, tmpls, threads=8)
    errs = []

    def worker():
        try:
            for _ in range(3):
                if _encode_seam(pb, keep, url, tmpls, threads=8) != want:
                    errs.append("mismatch")
        except Exception as ex:   # noqa: BLE001
            errs.append(repr(ex))

    th = [threading.Thread(target=worker) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs


def _routable_gpu(td, rng):
    """_routable, plus routing attributes the device must read as the host
    does: a second workload key (deployment wins over statefulset, either
    wins over daemonset, whatever their order), a repeated key (the first
    occurrence counts), a namespace that is not a string (Str() is "")."""
    td = _routable(td, rng)
    for rs in td["resourceSpans"]:
        attrs = rs["resource"]["attributes"]
        x = rng.random()
        if x < 0.1:
            attrs.insert(0, host.attrs({"k8s.daemonset.name": "agent"})[0])
        elif x < 0.2:
            attrs += host.attrs({"k8s.statefulset.name": "db"})
        elif x < 0.3:
            attrs.insert(0, host.attrs({"k8s.namespace.name": 7})[0])
        elif x < 0.4:
            attrs += host.attrs({"k8s.namespace.name": "prod"})
    return td


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_encoder_writes_pdata_inputs(seed):
    """A batch in pdata's encoding is routed and written by the GPU encoder
    (encode_kernel.hip: no fallback), byte for byte what the restatement
    writes with the GPU's decisions, and what the host encoder writes
    (engine option encode_host) — with and without a router, with SAMPLE|TEMPLATE and
    with TEMPLATE alone."""
    import torch
    from odigos_amd.batch import Engine, OtlpBatch
    rng = random.Random(0x6E0C + seed)
    td = _roundtrip(_routable_gpu(_http_traces(rng, 200), rng))
    streams = _streams(rng)
    router = Router({"datastreams": streams})
    eng = Engine(CFG)
    pb = gg.marshal_traces(td)
    ob = OtlpBatch(eng, pb)
    for st in (native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE, native.STAGE_TEMPLATE):
        eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=SEED)
        torch.cuda.synchronize()
        n = ob.cols.n_spans
        url_out = ob.out_numpy("url_out", n=n)
        refs = ob.out_numpy("tmpl", np.uint32, n=2 * n).reshape(-1, 2)
        arena = ob.out_numpy("tmpl_arena", n=ob.used()).tobytes()
        tmpls = [arena[o:o + ln].decode("utf-8", "surrogateescape") if u else "" for (o, ln), u in zip(refs, url_out)]
        dec = {"keep": list(ob.out_numpy("keep", n=n))} if st & native.STAGE_SAMPLE else {}
        for r in (router, None):
            want = _expected(td, streams if r else None, router.pipelines if r else None, url_out=list(url_out),
                             tmpls=tmpls, **dec)
            got = ob.encode(st, native.GROUP_TRACE_ID, r)
            assert ob.encode_path == {"gpu": True, "fallback": 0}
            assert got == want
            eng.set_option("encode_host", 1)
            assert ob.encode(st, native.GROUP_TRACE_ID, r) == want
            assert ob.encode_path["gpu"] is False
            eng.set_option("encode_host", 0)
    ob.close()


@pytest.mark.gpu
def test_gpu_encoder_hands_other_encodings_to_the_host():
    """google.protobuf's encoding (empty ids and Status left out) is not
    pdata's: the GPU encoder flags the call and the host encoder re-marshals
    it, with the same result as the restatement."""
    import torch
    from odigos_amd.batch import Engine, OtlpBatch
    rng = random.Random(0x6E1F)
    td = _roundtrip(_routable(_http_traces(rng, 50), rng))
    eng = Engine(CFG)
    ob = OtlpBatch(eng, to_pb(td))
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE
    eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=SEED)
    torch.cuda.synchronize()
    n = ob.cols.n_spans
    url_out = ob.out_numpy("url_out", n=n)
    refs = ob.out_numpy("tmpl", np.uint32, n=2 * n).reshape(-1, 2)
    arena = ob.out_numpy("tmpl_arena", n=ob.used()).tobytes()
    tmpls = [arena[o:o + ln].decode("utf-8", "surrogateescape") if u else "" for (o, ln), u in zip(refs, url_out)]
    want = _expected(td, None, None, keep=list(ob.out_numpy("keep", n=n)), url_out=list(url_out), tmpls=tmpls)
    assert ob.encode(st) == want
    assert ob.encode_path["gpu"] is False and ob.encode_path["fallback"] != 0
    ob.close()
