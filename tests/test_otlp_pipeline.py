"""ose_otlp_pipeline: concurrent OTLP requests coalesced into one device batch
per wave of calls (odigos_amd/csrc/otlp_pipeline.cpp).

Each request's outputs from a coalesced batch must equal, byte for byte, the
outputs of the same request through the ordinary calls (ose_otlp_decode ->
ose_process_device -> ose_otlp_encode), which test_router_encode.py and
test_otlp.py check against the restatement (tests/otlp_gogo.py) and the
oracle.  The traffic counters summed over a batch equal the sums of the
requests run alone.  Requests whose traces do not cross requests decide the
same either way; a trace split over two requests of one batch is decided as
one trace, which equals the concatenated message run as one request."""
import threading

import numpy as np
import pytest

from odigos_amd import native

SEED = 0x5EED
ST = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE


def _cfg():
    from tests.workloads import c3_sampling_config
    return {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
            "odigostrafficmetrics": {"res_attributes_keys": ["service.name", "k8s.namespace.name"]}}


def _router():
    from odigos_amd.batch import Router
    streams = [{"name": "ds-a", "sources": [{"namespace": "default", "kind": "Deployment", "name": "svc-%02d" % k}
                                            for k in range(0, 12)],
                "destinations": [{"destinationname": "d1", "configuredsignals": ["TRACES"]}]},
               {"name": "ds-b", "sources": [{"namespace": "default", "kind": "Deployment", "name": "svc-%02d" % k}
                                            for k in range(8, 20)],
                "destinations": [{"destinationname": "d2", "configuredsignals": ["TRACES", "LOGS"]}]}]
    return Router({"datastreams": streams})


def _requests(n_req, spans, seed0):
    from odigos_amd.batch import Generator
    return [Generator("fused", seed=seed0 + k, n_spans=spans, threads=4).otlp(4) for k in range(n_req)]


def _alone(eng, router, pb, seed=SEED):
    """the ordinary calls for one request"""
    import torch
    from odigos_amd.batch import OtlpBatch
    ob = OtlpBatch(eng, pb)
    eng.process_device(ob, ST, native.GROUP_TRACE_ID, seed=seed)
    torch.cuda.synchronize()
    out = ob.encode(ST, native.GROUP_TRACE_ID, router)
    ob.close()
    return out


def _records(buf: bytes):
    """top-level (tag, payload) records of a TracesData"""
    out, i = [], 0
    while i < len(buf):
        tag, s = 0, 0
        while True:
            b = buf[i]
            i += 1
            tag |= (b & 0x7F) << s
            s += 7
            if not b & 0x80:
                break
        ln, s = 0, 0
        while True:
            b = buf[i]
            i += 1
            ln |= (b & 0x7F) << s
            s += 7
            if not b & 0x80:
                break
        out.append((tag, i, i + ln))
        i += ln
    return out


def _concurrently(pipe, reqs, seed=SEED):
    res, errs = [None] * len(reqs), [None] * len(reqs)

    def run(k):
        try:
            res[k] = pipe.consume(reqs[k], seed=seed)
        except Exception as ex:   # noqa: BLE001
            errs[k] = ex

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(reqs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return res, errs


@pytest.mark.gpu
@pytest.mark.parametrize("n_req", [2, 8])
def test_gpu_pipeline_batch_equals_alone(n_req):
    from odigos_amd.batch import Engine, OtlpPipeline
    eng, router = Engine(_cfg()), _router()
    reqs = _requests(n_req, 8192, 0x0D17A000 + n_req)
    want = [_alone(eng, router, pb) for pb in reqs]
    pipe = OtlpPipeline(eng, router)
    pipe.hold(n_req)   # one batch of all requests
    got, errs = _concurrently(pipe, reqs)
    assert errs == [None] * n_req
    c = pipe.counters()
    assert c["batches"] == 1 and c["batched_requests"] == n_req and c["alone"] == 0, c
    for g, w in zip(got, want):
        assert g == w
    # the batch's traffic counters equal the requests' run alone
    alone = OtlpPipeline(eng, router)
    for pb in reqs:
        alone.consume(pb, seed=SEED)
    ca = alone.counters()
    assert ca["alone"] == n_req
    assert c["accepted_spans"] == ca["accepted_spans"] > 0
    to_map = lambda cs: {str(k): v for k, v in cs["data_size"]}   # noqa: E731
    assert to_map(c) == to_map(ca) and sum(to_map(c).values()) > 0
    pipe.close()
    alone.close()


@pytest.mark.gpu
def test_gpu_pipeline_trace_split_over_requests():
    # one message cut into two requests at a ResourceSpans boundary: traces
    # with spans on both sides are decided once, in the batch; each
    # request's outputs are its byte range of the whole message's outputs
    from odigos_amd.batch import Engine, OtlpPipeline
    eng, router = Engine(_cfg()), _router()
    pb = _requests(1, 20_000, 0x0D17A100)[0]
    recs = _records(pb)
    cut = recs[len(recs) // 2 - 1][2]   # the end of a record = the next one's tag
    a, b = pb[:cut], pb[cut:]
    whole = _alone(eng, router, pb)
    pipe = OtlpPipeline(eng, router)
    pipe.hold(2)
    got, errs = _concurrently(pipe, [a, b])
    assert errs == [None, None]
    assert pipe.counters()["batches"] == 1
    for k, (name, data, nres) in enumerate(whole):
        ga, gb = got[0][k], got[1][k]
        assert ga[0] == gb[0] == name
        # the batch holds the requests in the order they reserved room
        assert data in (ga[1] + gb[1], gb[1] + ga[1])
        assert ga[2] + gb[2] == nres
    pipe.close()


@pytest.mark.gpu
def test_gpu_pipeline_bad_request_alone():
    # a malformed request in a batch: the batch's decode fails, every request
    # runs alone: the good one gets its outputs, the bad one the decoder's error
    from odigos_amd.batch import Engine, OtlpPipeline
    eng, router = Engine(_cfg()), _router()
    good = _requests(1, 8192, 0x0D17A200)[0]
    recs = _records(good)
    # well-formed at the top level (so it joins the batch), but its last
    # ResourceSpans holds a Resource field whose bytes are not protobuf
    bad = good[: recs[3][2]] + b"\x0a\x04\x0a\x02\xff\xff"
    want = _alone(eng, router, good)
    pipe = OtlpPipeline(eng, router)
    pipe.hold(2)
    got, errs = _concurrently(pipe, [good, bad])
    assert got[0] == want and errs[0] is None
    assert isinstance(errs[1], native.OseError) and errs[1].code == native.OSE_EINVAL
    pipe.close()


@pytest.mark.gpu
def test_gpu_pipeline_host_encoder_requests():
    # requests in google.protobuf's encoding: the GPU encoder declines the
    # batch, each request runs alone through the host encoder
    import random
    from odigos_amd.batch import Engine, OtlpPipeline
    from tests.test_router_encode import CFG, _http_traces, _roundtrip, _routable, to_pb
    rng = random.Random(0x0D17)
    eng, router = Engine(CFG), _router()
    reqs = [to_pb(_roundtrip(_routable(_http_traces(rng, 40), rng))) for _ in range(3)]
    want = [_alone(eng, router, pb) for pb in reqs]
    pipe = OtlpPipeline(eng, router)
    pipe.hold(3)
    got, errs = _concurrently(pipe, reqs)
    assert errs == [None] * 3
    assert got == want
    assert pipe.counters()["alone"] == 3
    pipe.close()


@pytest.mark.gpu
def test_gpu_pipeline_many_callers():
    # 16 callers x 12 requests of assorted sizes with no hold: batches form
    # from whatever arrives while others run; every result equals its
    # request run alone, and the counters add up
    from odigos_amd.batch import Engine, OtlpPipeline
    eng, router = Engine(_cfg()), _router()
    sizes = [1, 64, 1000, 4096, 8192]
    reqs = [_requests(1, sizes[k % len(sizes)], 0x0D17A300 + k)[0] for k in range(24)]
    want = [_alone(eng, router, pb) for pb in reqs]
    pipe = OtlpPipeline(eng, router, max_batch_bytes=4 << 20)
    pipe.tune(1, 500, 8)   # one batch on the GPU at a time: the others fill meanwhile
    errs = []

    def caller(c):
        try:
            for j in range(12):
                k = (c * 5 + j) % len(reqs)
                if pipe.consume(reqs[k], seed=SEED) != want[k]:
                    errs.append(("mismatch", k))
        except Exception as ex:   # noqa: BLE001
            errs.append(repr(ex))

    th = [threading.Thread(target=caller, args=(c,)) for c in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[:5]
    c = pipe.counters()
    assert c["batched_requests"] + c["alone"] == 16 * 12
    assert c["largest_batch"] > 1, c
    pipe.close()
