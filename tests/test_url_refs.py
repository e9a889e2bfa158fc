"""OSE_STAGE_TEMPLATE_REFS: the templates left where the GPU assembled them
(include/odigos_amd.h).  Parity is per span: the bytes each span's ref names
equal the oracle's template for that span (odigosurltemplateprocessor/
processor.go:150-190 via oracle/url.c), whatever the arena layout; url_out
and the template lengths are compared as in the packed form.  The spans pass
of odigostrafficmetrics (fused into url_copy_kernel) must count the same in
both forms.
"""
import ctypes as C

import numpy as np
import pytest

from odigos_amd import native
from odigos_amd.batch import DeviceBatch, Engine, Generator, HostOutputs
from tests.oracle_lib import UrlOracle, span_template_bytes
from tests.workloads import c3_sampling_config

REFS = native.STAGE_TEMPLATE | native.STAGE_TEMPLATE_REFS


def _refs_vs_oracle(g, cfg, arena_bytes=None, tmpl_cap=None):
    import torch
    eng = Engine({"odigosurltemplate": cfg})
    db = DeviceBatch(g.cols, tmpl_cap=tmpl_cap)
    if arena_bytes is not None:
        db.cols.arena_bytes = arena_bytes
    eng.process_device(db, REFS)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = HostOutputs(g.cols)
    assert UrlOracle(cfg).process(g.cols, ho.outs, nthreads=8) == 0
    ns = g.cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("url_out")[:ns], ho.view("url_out", np.uint8)[:ns])
    mask = ho.view("url_out", np.uint8)[:ns] != 0
    used = db.used()
    cap = db.outs.tmpl_arena_cap
    # the gaps: <= 15 bytes per 64-span group and the waves' last chunk tails (<= cap / 8)
    assert int(ho.used[0]) <= used <= min(cap, int(ho.used[0]) + 16 * ((ns + 63) // 64) + cap // 8)
    gt = db.out_numpy("tmpl", np.uint32)[: 2 * ns]
    gb, gl = span_template_bytes(gt, db.out_numpy("tmpl_arena")[:used], mask)
    ob, ol = span_template_bytes(ho.view("tmpl", np.uint32)[: 2 * ns], ho.bufs["tmpl_arena"][: int(ho.used[0])], mask)
    np.testing.assert_array_equal(gl, ol)
    np.testing.assert_array_equal(gb, ob)
    return gt.reshape(-1, 2)[mask], used


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 257, 100_000])
def test_gpu_refs_parity_small(n):
    refs, used = _refs_vs_oracle(Generator("url", seed=0x0D1600E0 + n, n_spans=n), {})
    assert refs.size == 0 or int((refs[:, 0] + refs[:, 1]).max()) <= used


@pytest.mark.gpu
def test_gpu_refs_parity_rules_and_custom_ids():
    # rule plans take the per-span writer: those groups are placed by the scan
    cfg = {"templatization_rules": ["/users/{user}/orders/{order:\\d+}", "/api/v1/*", "/{a}/{b}/{c}/{d}/{e}/{f}"],
           "custom_ids": [{"regexp": "^inc_\\d+$", "template_name": "incident"}, {"regexp": "(?i)^PROCESS_"}]}
    _refs_vs_oracle(Generator("url", seed=0x0D1600E8, n_spans=200_000), cfg)


@pytest.mark.gpu
def test_gpu_refs_parity_scratch_regions_overflow():
    # arena_bytes understated to 0 (it sizes only the packed form's scratch)
    _refs_vs_oracle(Generator("url", seed=0x0D1600E9, n_spans=1_000_000, threads=8), {}, arena_bytes=0)


@pytest.mark.gpu
def test_gpu_refs_parity_paths_spread_and_stretched():
    g = Generator("url", seed=0x0D1600EA, n_spans=300_000, threads=8)
    path = g.array("path").view(np.uint32).reshape(-1, 2)
    has = np.flatnonzero(path[:, 1] > 0)
    perm = np.random.default_rng(0x0D1600EA).permutation(has.size)
    path[has] = path[has][perm]
    # every 50th path stretched over 200 bytes (its group's image outgrows LDS)
    st = has[::50]
    path[st, 1] = np.minimum(200, g.cols.arena_bytes - path[st, 0]).astype(np.uint32)
    _refs_vs_oracle(g, {})


@pytest.mark.gpu
def test_gpu_refs_overflow_flagged():
    # a capacity the templates cannot fit: device_status bit 2 and the bytes needed, as in the packed form
    import torch
    g = Generator("url", seed=0x0D1600EB, n_spans=50_000)
    eng = Engine({"odigosurltemplate": {}})
    db = DeviceBatch(g.cols, tmpl_cap=4096)
    eng.process_device(db, REFS)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) & 2
    need = db.used()
    assert need > 4096
    db2 = DeviceBatch(g.cols, tmpl_cap=need)   # what the shim retries with
    eng.process_device(db2, REFS)
    torch.cuda.synchronize()
    assert int(db2.out_numpy("device_status", np.uint32)[0]) == 0


@pytest.mark.gpu
def test_gpu_refs_size_counts_equal_packed():
    # the fused spans pass (url_copy_kernel) counts the same in both forms
    import torch
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": ["service.name"]}}
    g = Generator("fused", seed=0x0D1600EC, n_spans=400_000, threads=8)
    eng = Engine(cfg)
    out = {}
    for name, extra in (("packed", 0), ("refs", native.STAGE_TEMPLATE_REFS)):
        db = DeviceBatch(g.cols)
        eng.process_device(db, native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE | extra, seed=11)
        torch.cuda.synchronize()
        assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
        ns = g.cols.n_spans
        t = db.out_numpy("tmpl", np.uint32)[: 2 * ns]
        m = db.out_numpy("url_out")[:ns] != 0
        out[name] = (db.out_numpy("keep")[:ns].copy(), db.out_numpy("attrset_bytes", np.int64).copy(),
                     db.out_numpy("accepted_spans", np.int64).copy(),
                     span_template_bytes(t, db.out_numpy("tmpl_arena")[: db.used()], m))
    a, b = out["packed"], out["refs"]
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[3][1], b[3][1])
    np.testing.assert_array_equal(a[3][0], b[3][0])


@pytest.mark.gpu
def test_gpu_refs_refused_by_host_path():
    from odigos_amd.batch import PinnedBatch
    g = Generator("url", seed=0x0D1600ED, n_spans=1000)
    eng = Engine({"odigosurltemplate": {}})
    pb = PinnedBatch(eng, g.cols)
    pb.fill(g.cols)
    with pytest.raises(native.OseError):
        pb.process(REFS)
    with pytest.raises(native.OseError):   # REFS without TEMPLATE
        eng.process_device(DeviceBatch(g.cols), native.STAGE_TEMPLATE_REFS)


@pytest.mark.gpu
def test_gpu_forked_refs_equal_packed_and_overflow_retry():
    # SAMPLE | TEMPLATE on 1M+ spans: the URL planning runs on a second stream
    # beside the trace stage, in the refs form with a plan grid 16x the
    # resident one (engine.cpp run_stages).  Its decisions, counters and
    # templates equal the packed form's, and an arena too small for the
    # larger grid's chunks reports a capacity whose retry fits.
    import torch
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": ["service.name"]}}
    g = Generator("fused", seed=0x0D1600ED, n_spans=1_200_000, threads=8)
    eng = Engine(cfg)
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    out = {}
    for name, extra in (("packed", 0), ("refs", native.STAGE_TEMPLATE_REFS)):
        db = DeviceBatch(g.cols)
        eng.process_device(db, st | extra, seed=13)
        torch.cuda.synchronize()
        assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
        ns = g.cols.n_spans
        t = db.out_numpy("tmpl", np.uint32)[: 2 * ns]
        m = db.out_numpy("url_out")[:ns] != 0
        out[name] = (db.out_numpy("keep")[:ns].copy(), db.out_numpy("url_out")[:ns].copy(),
                     db.out_numpy("attrset_bytes", np.int64).copy(), db.out_numpy("accepted_spans", np.int64).copy(),
                     span_template_bytes(t, db.out_numpy("tmpl_arena")[: db.used()], m))
    for a, b in zip(out["packed"][:4], out["refs"][:4]):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(out["packed"][4], out["refs"][4]):   # template bytes, lengths
        np.testing.assert_array_equal(a, b)
    # both forms ran forked (URL planning beside the trace stage): a fork or
    # join ordering fault would corrupt them alike, so the forked result is
    # also checked against the oracle chain on the whole batch
    from tests.oracle_lib import SamplingOracle, size_process
    ns = g.cols.n_spans
    ho = HostOutputs(g.cols)
    assert SamplingOracle(cfg["odigossampling"]).process(g.cols, ho.outs, native.GROUP_TRACE_ID, 13, 8) == 0
    assert UrlOracle(cfg["odigosurltemplate"]).process(g.cols, ho.outs, 8) == 0
    assert size_process(g.cols, ho.outs, st, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, 8) == 0
    A = g.cols.n_attrsets
    np.testing.assert_array_equal(out["refs"][0], ho.view("keep", np.uint8)[:ns])
    np.testing.assert_array_equal(out["refs"][1], ho.view("url_out", np.uint8)[:ns])
    np.testing.assert_array_equal(out["refs"][2][:A], ho.view("attrset_bytes", np.int64)[:A])
    assert int(out["refs"][3][0]) == int(ho.view("accepted_spans", np.int64)[0])
    hm = ho.view("url_out", np.uint8)[:ns] != 0
    want_t = span_template_bytes(ho.view("tmpl", np.uint32)[: 2 * ns], ho.bufs["tmpl_arena"][: int(ho.used[0])], hm)
    for a, b in zip(want_t, out["refs"][4]):
        np.testing.assert_array_equal(a, b)
    small = DeviceBatch(g.cols, tmpl_cap=1 << 16)
    eng.process_device(small, st | native.STAGE_TEMPLATE_REFS, seed=13)
    torch.cuda.synchronize()
    assert int(small.out_numpy("device_status", np.uint32)[0]) & 2
    need = small.used()
    retry = DeviceBatch(g.cols, tmpl_cap=need)
    eng.process_device(retry, st | native.STAGE_TEMPLATE_REFS, seed=13)
    torch.cuda.synchronize()
    assert int(retry.out_numpy("device_status", np.uint32)[0]) == 0
    ns = g.cols.n_spans
    t = retry.out_numpy("tmpl", np.uint32)[: 2 * ns]
    m = retry.out_numpy("url_out")[:ns] != 0
    for a, b in zip(span_template_bytes(t, retry.out_numpy("tmpl_arena")[: retry.used()], m), out["packed"][4]):
        np.testing.assert_array_equal(a, b)
