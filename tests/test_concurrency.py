"""Re-entrancy of the engine (include/odigos_amd.h: "one engine may be used
from many threads").  In the reference, receivers call ConsumeTraces
concurrently and groupbytrace releases traces from its own goroutine
(SURVEY.md §8b Threading), so every entry point must be safe to call from
several threads on one engine.  Also hipGraph capture of the stages that
allow it.

GPU (@gpu):
  * several threads drive ose_process_device on one engine, each on its own
    HIP stream and batch; every output matches the oracle chain;
  * several threads call ConsumeTraces (host processors -> ose_process) on
    one processor; every result matches the single-threaded one;
  * TEMPLATE | SIZE captured into a hipGraph (torch.cuda.graph) replays to
    the same outputs as eager calls; SAMPLE by trace id refuses capture.
"""
import ctypes as C
import json
import threading

import numpy as np
import pytest

from odigos_amd import native
from odigos_amd.batch import Generator, HostOutputs
from tests.oracle_lib import SamplingOracle, UrlOracle, size_process
from tests.workloads import c3_sampling_config

CFG = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
       "odigostrafficmetrics": {"res_attributes_keys": ["service.name"]}}
STAGES = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
SEED = 0x5EED


def oracle_chain(cols):
    ho = HostOutputs(cols)
    assert SamplingOracle(CFG["odigossampling"]).process(cols, ho.outs, native.GROUP_TRACE_ID, SEED, 8) == 0
    assert UrlOracle({}).process(cols, ho.outs, 8) == 0
    assert size_process(cols, ho.outs, STAGES, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, 8) == 0
    return ho


@pytest.mark.gpu
def test_gpu_concurrent_process_device():
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    eng = Engine(CFG)
    T, CALLS = 4, 3
    gens = [Generator("fused", seed=0x0D160900 + t, n_spans=150_000 + 7919 * t, shuffle=(t % 2 == 1)) for t in range(T)]
    dbs = [DeviceBatch(g.cols) for g in gens]
    errors = []

    def worker(t):
        try:
            s = torch.cuda.Stream()
            for _ in range(CALLS):
                eng.process_device(dbs[t], STAGES, native.GROUP_TRACE_ID, seed=SEED, stream=s.cuda_stream)
            s.synchronize()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for g, db in zip(gens, dbs):
        n, A = g.cols.n_spans, g.cols.n_attrsets
        ho = oracle_chain(g.cols)
        assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
        np.testing.assert_array_equal(db.out_numpy("keep", n=n), ho.view("keep", np.uint8)[:n])
        np.testing.assert_array_equal(db.out_numpy("url_out", n=n), ho.view("url_out", np.uint8)[:n])
        used = db.used()
        assert used == int(ho.used[0])
        np.testing.assert_array_equal(db.out_numpy("tmpl_arena", n=used), ho.bufs["tmpl_arena"][:used])
        np.testing.assert_array_equal(db.out_numpy("attrset_bytes", np.int64, n=A),
                                      CALLS * ho.view("attrset_bytes", np.int64)[:A])


@pytest.mark.gpu
def test_gpu_concurrent_consume_traces():
    from odigos_amd import host
    p = host.Processor("odigosurltemplate", {"templatization_rules": ["/users/{user}/orders/{order:\\d+}"]})
    paths = ["/user/1234", "/users/alice/orders/77", "/v1/items/550e8400-e29b-41d4-a716-446655440000",
             "/api/2025-01-02/x", "/files/deadbeefdeadbeef", "/a/b/c", "/mail/john@example.com/inbox"]
    tds = []
    for k in range(48):
        spans = [host.span(name="GET", kind=2, attributes={"http.request.method": "GET", "url.path": paths[(k + j) % len(paths)] + f"/{k}"})
                 for j in range(1 + k % 5)]
        tds.append(host.traces(host.resource_spans({"service.name": f"svc{k % 3}"}, spans)))
    want = [p.consume(td) for td in tds]
    got = [None] * len(tds)
    errors = []

    def worker(t):
        try:
            for k in range(t, len(tds), 6):
                got[k] = p.consume(tds[k])
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert got == want


@pytest.mark.gpu
def test_gpu_graph_capture_template_size():
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    cfg = {"odigosurltemplate": {}, "odigostrafficmetrics": {"res_attributes_keys": ["service.name"]}}
    eng = Engine(cfg)
    g = Generator("fused", seed=0x0D160910, n_spans=100_000)
    st = native.STAGE_TEMPLATE | native.STAGE_SIZE
    eager, cap = DeviceBatch(g.cols), DeviceBatch(g.cols)
    eng.reserve(g.cols.n_spans)
    eng.process_device(eager, st, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            eng.process_device(cap, st, stream=s.cuda_stream)
    torch.cuda.synchronize()
    cap.o["attrset_bytes"].zero_()
    graph.replay()
    torch.cuda.synchronize()
    n, A = g.cols.n_spans, g.cols.n_attrsets
    for name, dt, k in (("url_out", np.uint8, n), ("tmpl", np.uint64, n), ("attrset_bytes", np.int64, A)):
        np.testing.assert_array_equal(cap.out_numpy(name, dt, n=k), eager.out_numpy(name, dt, n=k))
    used = eager.used()
    assert cap.used() == used
    np.testing.assert_array_equal(cap.out_numpy("tmpl_arena", n=used), eager.out_numpy("tmpl_arena", n=used))
    # a second replay adds the counters again
    graph.replay()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cap.out_numpy("attrset_bytes", np.int64, n=A),
                                  2 * eager.out_numpy("attrset_bytes", np.int64, n=A))


@pytest.mark.gpu
def test_gpu_graph_capture_refuses_trace_id_sampling():
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    eng = Engine({"odigossampling": c3_sampling_config()})
    g = Generator("sampling", seed=0x0D160911, n_spans=10_000)
    db = DeviceBatch(g.cols)
    eng.reserve(g.cols.n_spans)
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with pytest.raises(native.OseError) as ei:
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID, stream=s.cuda_stream)
    assert ei.value.code == native.OSE_ENOTSUP
    torch.cuda.synchronize()
    # batch-mode sampling (one trace per call) has no per-call host state: it captures
    graph2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph2, stream=s):
            eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_BATCH, stream=s.cuda_stream)
    graph2.replay()
    torch.cuda.synchronize()
    ho = HostOutputs(g.cols)
    assert SamplingOracle(c3_sampling_config()).process(g.cols, ho.outs, native.GROUP_BATCH, 0, 1) == 0
    n = g.cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("keep", n=n), ho.view("keep", np.uint8)[:n])


@pytest.mark.gpu
def test_gpu_concurrent_pipeline_counters():
    """odigosurltemplate + odigostrafficmetrics from 6 threads: every output
    and the summed otel counters equal the single-threaded run's (the traffic
    counters are shared state, processor.go:76-81)."""
    from odigos_amd import host
    cfg = {"odigosurltemplate": {}, "odigostrafficmetrics": {"res_attributes_keys": ["service.name", "k8s.pod.name"]}}
    from tools.dropin_bench import batch_items
    items = batch_items(12, 700, 0x0D16C0DE)
    ref = host.Processor("pipeline", cfg)
    want = [ref.consume(td) for td in items]
    p = host.Processor("pipeline", cfg)
    got = [None] * len(items)
    errors = []

    def worker(t):
        try:
            for k in range(t, len(items), 6):
                got[k] = p.consume(items[k])
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert got == want
    key = lambda m: sorted((json.dumps(d["attributes"], sort_keys=True), d["value"]) for d in m["otelcol_odigos_trace_data_size"])
    assert key(p.metrics()) == key(ref.metrics())
    assert p.metrics()["otelcol_odigos_accepted_spans"] == ref.metrics()["otelcol_odigos_accepted_spans"]


@pytest.mark.gpu
def test_gpu_host_bench_entry():
    """osehost_bench (tools/dropin_bench.py) runs every call and times it."""
    import ctypes as C
    from odigos_amd import host
    from tools.dropin_bench import per_trace_items
    items = per_trace_items(40, 7)
    p = host.Processor("odigossampling", c3_sampling_config())
    out = (C.c_double * 12)()
    rc = native.lib().osehost_bench(p.h, host.dumps(items).encode(), 3, 4, out)
    assert rc == 0, native.lib().osehost_last_error()
    assert int(out[1]) == 120
    assert out[0] > 0 and 0 < out[8] <= out[9] <= out[10] <= out[11]
    assert out[5] > 0   # ose_process time


@pytest.mark.gpu
def test_gpu_ose_process_pinned_pool():
    """ose_process on engine-owned pinned batches (batch.cpp): outputs equal
    the oracle chain; a released batch is reused by the next acquire (the
    pool), including for a smaller batch, with the absent columns NULLed."""
    from odigos_amd.batch import Engine, PinnedBatch
    eng = Engine(CFG)
    for k, n in enumerate((120_000, 90_000, 120_000)):
        g = Generator("fused", seed=0x0D160920 + k, n_spans=n)
        g.cols.res_url_ok = None   # no include/exclude configured (fill NULLs the pinned column)
        b = PinnedBatch(eng, g.cols)
        b.fill(g.cols)
        for f in ("trace_first_span", "trace_level", "trace_ratio", "res_bytes"):
            setattr(b.outs, f, None)
        A = g.cols.n_attrsets
        np.ctypeslib.as_array((C.c_int64 * max(A, 1)).from_address(b.outs.attrset_bytes))[:] = 0
        np.ctypeslib.as_array((C.c_int64 * 1).from_address(b.outs.accepted_spans))[:] = 0
        b.process(STAGES, native.GROUP_TRACE_ID, seed=SEED)
        ho = oracle_chain(g.cols)
        keep = np.ctypeslib.as_array((C.c_uint8 * n).from_address(b.outs.keep))
        np.testing.assert_array_equal(keep, ho.view("keep", np.uint8)[:n])
        url = np.ctypeslib.as_array((C.c_uint8 * n).from_address(b.outs.url_out))
        np.testing.assert_array_equal(url, ho.view("url_out", np.uint8)[:n])
        used = int(b.outs.tmpl_arena_used[0]) if hasattr(b.outs.tmpl_arena_used, "__getitem__") else \
            int(C.cast(b.outs.tmpl_arena_used, C.POINTER(C.c_uint64))[0])
        assert used == int(ho.used[0])
        arena = np.ctypeslib.as_array((C.c_uint8 * used).from_address(b.outs.tmpl_arena))
        np.testing.assert_array_equal(arena, ho.bufs["tmpl_arena"][:used])
        ab = np.ctypeslib.as_array((C.c_int64 * A).from_address(b.outs.attrset_bytes))
        np.testing.assert_array_equal(ab, ho.view("attrset_bytes", np.int64)[:A])
        b.close()
