"""The drop-in pdata path at the batch size tools/dropin_bench.py measures:
8192-span ConsumeTraces calls through all three processors (GROUP_TRACE_ID)
on the GPU equal, trace for trace, the same calls decided by the CPU oracle
through the host seam (columnarize -> SamplingOracle -> UrlOracle -> size ->
apply).  Each call samples with the processor's first draw (the seed), so a
fresh processor per call makes both sides draw alike."""
import pytest

from odigos_amd import host, native
from tests.oracle_lib import SamplingOracle, UrlOracle, size_process
from tests.workloads import c3_sampling_config
from tools.dropin_bench import batch_items

PIPE = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
        "odigostrafficmetrics": {"res_attributes_keys": ["service.name", "k8s.namespace.name"]}}
STAGES = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE


def _oracle_consume(td, seed):
    ref = host.Processor("pipeline", PIPE)
    ref.configure(seed, native.GROUP_TRACE_ID)
    hb = ref.columnarize(td)
    o = hb.outs
    assert SamplingOracle(PIPE["odigossampling"]).process(hb.cols, o, native.GROUP_TRACE_ID, seed) == 0
    assert UrlOracle(PIPE["odigosurltemplate"]).process(hb.cols, o) == 0
    assert size_process(hb.cols, o, STAGES, native.GROUP_TRACE_ID, o, 1, 1.0, 0.0) == 0
    out = hb.apply()
    m = ref.metrics()
    ref.close()
    return out, m


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(3))
def test_gpu_dropin_batch_equals_oracle(k):
    td = batch_items(3, 8192, 0x0D16D002)[k]
    seed = 0x0D16B0B0 + k
    want, wm = _oracle_consume(td, seed)
    p = host.Processor("pipeline", PIPE)
    p.configure(seed, native.GROUP_TRACE_ID)
    got = p.consume(td)
    gm = p.metrics()
    p.close()
    assert got == want
    assert gm == wm
