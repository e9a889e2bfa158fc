"""Object lifetimes across the C ABI (include/odigos_amd.h, ose_engine_destroy).

A cgo shim's finalizers, like Python's garbage collector on a reference
cycle, may release an engine before the batches made from it.  Every child
(ose_batch, ose_otlp_batch, ose_otlp_out, ose_gbt) holds a reference on the
engine, so each order is legal: no use after free, no HIP error met by a
release entry point (ose_dropped_errors), none left in the runtime's
last-error slot (tests/conftest.py checks both around every GPU test).
"""
import ctypes as C
import gc

import numpy as np
import pytest

from odigos_amd import native
from tests.workloads import c3_sampling_config

CFG = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
       "odigostrafficmetrics": {"res_attributes_keys": ["service.name"]}}


def test_dropped_errors_entry_point():
    L = native.lib()
    buf = C.create_string_buffer(256)
    assert L.ose_dropped_errors(buf, len(buf)) >= 0
    assert L.ose_dropped_errors(None, 0) >= 0


def _children(eng):
    """One live child of every kind, each used once."""
    from odigos_amd.batch import Generator, GroupByTrace, OtlpBatch, PinnedBatch
    import torch
    L = native.lib()
    g = Generator("fused", seed=0x0D1600A1, n_spans=4000)
    pb = PinnedBatch(eng, g.cols)
    pb.fill(g.cols)
    pb.process(native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE)
    ob = OtlpBatch(eng, g.otlp())
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=7)
    out = C.c_void_p()
    native.check(L.ose_otlp_encode(eng.h, ob.h, C.byref(ob.outs), st, native.GROUP_TRACE_ID, None, None,
                                   C.byref(out)))
    assert L.ose_otlp_out_count(out) == 1
    gbt = GroupByTrace(eng, {"wait_duration": "1s", "num_traces": 10000}, 1 << 16, 1 << 22)
    gbt.add(ob.cols, 1)
    torch.cuda.synchronize()
    return pb, ob, out, gbt


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["engine_first", "engine_middle", "engine_last"])
def test_gpu_children_released_around_engine_destroy(order):
    import torch
    from odigos_amd.batch import Engine
    L = native.lib()
    eng = Engine(CFG)
    pb, ob, out, gbt = _children(eng)
    h = eng.h
    eng.h = None   # bypass Engine.close (which releases the children first)

    def release_children(k):
        seq = [pb.close, ob.close, lambda: L.ose_otlp_out_release(out), gbt.close]
        for f in seq[k:] if k else seq:
            f()

    if order == "engine_first":
        L.ose_engine_destroy(h)
        release_children(0)
    elif order == "engine_middle":
        pb.close()
        ob.close()
        L.ose_engine_destroy(h)
        L.ose_otlp_out_release(out)
        gbt.close()
    else:
        release_children(0)
        L.ose_engine_destroy(h)
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_garbage_cycle_with_engine():
    # a reference cycle holding the engine and its children: the collector
    # clears the engine's weak child set before any finalizer runs, so the
    # engine's finalizer may run before the children's (the round-2 use-after-
    # free: a release bound a freed engine's device)
    import torch
    from odigos_amd.batch import Engine
    for _ in range(3):
        eng = Engine(CFG)
        pb, ob, out, gbt = _children(eng)
        native.lib().ose_otlp_out_release(out)
        box = {"eng": eng, "kids": [pb, ob, gbt]}
        box["self"] = box
        pb.cycle = box
        del eng, pb, ob, gbt, box
        gc.collect()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_pooled_batches_after_destroy_are_freed():
    # released while the engine is alive: pooled; the engine's destroy frees the pool
    import torch
    from odigos_amd.batch import Engine, Generator, PinnedBatch, host_array
    eng = Engine(CFG)
    g = Generator("fused", seed=0x0D1600A2, n_spans=1000)
    keeps = []
    for _ in range(3):
        b = PinnedBatch(eng, g.cols)
        b.fill(g.cols)
        b.process(native.STAGE_SAMPLE | native.STAGE_TEMPLATE)
        keeps.append(host_array(b.outs.keep, g.cols.n_spans).copy())
        b.close()
    assert all(np.array_equal(keeps[0], k) for k in keeps) and keeps[0].size == g.cols.n_spans
    eng.close()
    torch.cuda.synchronize()
