"""odigossampling configs beyond one rule table: more than 64 http_latency
rules, more than 64 distinct service_name services, tables beyond the LDS
budget.  The engine cuts the level-ordered rule list into chunks and runs the
trace stage once per chunk, carrying ShouldSample's walk per trace
(sampling_host.cpp build_sampling_tables / run_sampling, trace_kernel.hip
decide_chunk).  The reference accepts these configs (odigossamplingprocessor
config.go:17-80 Validate has no rule-count bound; rule_engine.go:55-115
folds any number of rules).

CPU: the oracle against the pure-Python restatement on the wide configs.
GPU (@gpu): the chunked HIP path against the oracle, bit-exact on keep and
the per-trace records, through the fast path, the slow (repeated-id) path,
the long-run kernel and batch mode.
"""
import ctypes as C

import numpy as np
import pytest

from odigos_amd import native
from odigos_amd.batch import Generator
from tests.oracle_lib import intern_services, lib as orc_lib
from tests.test_sampling_random import SEED, _arr, _group, _py_eval, gpu_vs_oracle, inject_zero_starts, oracle_run
from tests.workloads import (check_interning, long_routes_config, many_services_config, wide_attr100_config,
                             wide_attr_config, wide_latency2_config, wide_latency_config, wide_latency_split_config,
                             wide_mixed_config)

CONFIGS = {"latency": wide_latency_config, "latency2": wide_latency2_config, "latency_split": wide_latency_split_config,
           "mixed": wide_mixed_config, "long_routes": long_routes_config, "many_services": many_services_config}


def _chunks(cfg):
    import json
    n = C.c_uint32()
    native.check(native.lib().osehost_sampling_chunks(json.dumps({"odigossampling": cfg}).encode(), C.byref(n)))
    return n.value


def test_chunk_counts():
    # greedy chunks of the level-ordered list (no device needed)
    from tests.workloads import c3_sampling_config
    assert _chunks(c3_sampling_config()) == 1
    assert _chunks(wide_latency_config()) == 3          # 150 latency rules: 64 + 64 + 22
    assert _chunks(wide_latency2_config()) == 2
    assert _chunks(wide_latency_split_config()) == 2
    assert _chunks(wide_attr_config()) == 2             # 64 service + attr bits fill the first
    assert _chunks(wide_mixed_config()) >= 4
    assert _chunks(long_routes_config()) >= 2           # route bytes past the 12 KiB table
    cfg = wide_latency_config()
    cfg["endpoint_rules"] = cfg["endpoint_rules"][:64]
    assert _chunks(cfg) == 1
    cfg["endpoint_rules"] = wide_latency_config()["endpoint_rules"][:65]
    assert _chunks(cfg) == 2


def test_chunk_refusals():
    import json
    n = C.c_uint32()
    L = native.lib()
    one = {"global_rules": [{"name": "l", "type": "http_latency",
                             "rule_details": {"http_route": "/" + "a" * 13000, "service_name": "s", "threshold": 5,
                                              "fallback_sampling_ratio": 1}}]}
    # a route longer than the 12 KiB LDS table: its own chunk, the bytes past
    # the table read from HBM
    assert L.osehost_sampling_chunks(json.dumps({"odigossampling": one}).encode(), C.byref(n)) == 0 and n.value == 1
    assert _chunks(_long_route_config()) == 3
    attr = {"global_rules": [{"name": f"a{j}", "type": "span_attribute",
                              "rule_details": {"service_name": "s", "attribute_key": "k", "condition_type": "string",
                                               "operation": "equals", "expected_value": "v", "sampling_ratio": 1}}
                             for j in range(64)]}
    assert L.osehost_sampling_chunks(json.dumps({"odigossampling": attr}).encode(), C.byref(n)) == 0 and n.value == 1
    # past 64 span_attribute rules: more chunks, attr_match in more words
    for k in (65, 130, 200):
        attr["global_rules"] = [dict(attr["global_rules"][0], name=f"a{j}") for j in range(k)]
        assert L.osehost_sampling_chunks(json.dumps({"odigossampling": attr}).encode(), C.byref(n)) == 0
        assert n.value == (k + 63) // 64
    assert _chunks(wide_attr100_config()) == 3        # 40 service + 24 attr bits, 64 attr, 12 attr
    # 1200 services: dense service tables (14.4 KB) no longer fit a chunk, so
    # each chunk indexes the services its rules name (no refusal); 64
    # service bits per chunk bound the count from below
    for n in (600, 1200, 5000):
        assert _chunks(many_services_config(n)) >= (n + 63) // 64


LONG_PRE = "/" + "a" * 13000


def _long_route_config():
    # C3's rules with an http_latency rule whose route alone overflows the LDS
    # rule table, between two ordinary ones (three chunks: before, the long
    # rule, after)
    from tests.workloads import c3_sampling_config
    cfg = c3_sampling_config()
    ep = cfg["endpoint_rules"]
    ep.insert(8, {"name": "long", "type": "http_latency",
                  "rule_details": {"http_route": LONG_PRE, "service_name": "svc-02", "threshold": 1,
                                   "fallback_sampling_ratio": 3}})
    return cfg


def _with_long_routes(g, seed, frac=0.05):
    """Points a fraction of the spans' routes at 13 KB strings: the long rule's
    prefix exactly, the prefix and more, one differing in its last byte, one
    differing early, one a byte short.  Returns the new arena (keep it alive)."""
    rng = np.random.default_rng(seed)
    variants = [LONG_PRE, LONG_PRE + "/x", LONG_PRE[:-1] + "b", "/b" + LONG_PRE[2:], LONG_PRE[:-1]]
    arena = g.array("arena")
    used = int(g.cols.arena_bytes)
    offs, blob = [], bytearray()
    base = (used + 15) // 16 * 16
    for v in variants:
        offs.append(base + len(blob))
        blob += v.encode()
        blob += b"\0" * ((-len(blob)) % 16)
    new = np.zeros(base + len(blob) + 32, dtype=np.uint8)
    new[:used] = arena[:used]
    new[base:base + len(blob)] = np.frombuffer(bytes(blob), dtype=np.uint8)
    route = g.array("route").view(np.uint32).reshape(-1, 2)
    pick = np.nonzero(rng.random(g.cols.n_spans) < frac)[0]
    which = rng.integers(0, len(variants), size=len(pick))
    route[pick, 0] = np.array(offs, dtype=np.uint32)[which]
    route[pick, 1] = np.array([len(v) for v in variants], dtype=np.uint32)[which]
    g.cols.arena = new.ctypes.data
    g.cols.arena_bytes = base + len(blob)
    return new


def test_long_route_oracle_vs_python():
    # the oracle against the Python restatement with the 13 KB rule and routes
    # that match it, extend it or differ past the LDS part
    cfg = _long_route_config()
    g = Generator("sampling", seed=0x0D160841, n_spans=4000)
    inject_zero_starts(g, 0.03, 7)
    keep = _with_long_routes(g, 3, frac=0.2)
    cols = g.cols
    ho = oracle_run(cols, native.GROUP_TRACE_ID, cfg=cfg)
    traces = _group(cols, False)
    svc_ids = intern_services(cfg)
    res = _arr(cols.resource, C.c_uint32, cols.n_spans)
    tid = _arr(cols.trace_id, C.c_uint64, 2 * cols.n_spans).reshape(-1, 2)
    hits = 0
    for t, spans in enumerate(traces):
        u = orc_lib().orc_trace_uniform(int(tid[spans[0], 0]), int(tid[spans[0], 1]), SEED)
        k, lvl, ratio = _py_eval(cfg, svc_ids, cols, res, spans, False, u)
        assert ho.view("trace_level", np.uint8)[t] == lvl, t
        assert ho.view("trace_ratio", np.float64)[t] == ratio, t
        hits += ratio == 3.0 or (lvl == 2 and ratio == 100.0)
    assert hits > 0
    del keep


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_route_past_the_lds_table(shuffle):
    # a 13 KB http_route (Validate accepts it): the rule's chunk keeps its
    # tables in LDS and reads the route bytes past kSampCfgLds from HBM; spans
    # carrying the exact prefix, longer routes, and routes differing only
    # past the LDS part decide as the oracle does
    cfg = _long_route_config()
    g = Generator("sampling", seed=0x0D160821 + int(shuffle), n_spans=200_000, shuffle=shuffle)
    inject_zero_starts(g, 0.01, 11)
    g.keep_arena = _with_long_routes(g, 12)
    gpu_vs_oracle(g, cfg=cfg)


@pytest.mark.gpu
def test_gpu_route_past_the_lds_table_exchange_world3():
    # the same rule through the trace-id exchange: the pack's endpoint test
    # reads the spilled route bytes from HBM too
    from tests.test_exchange import _concat_keep_oracle, _local_round
    cfg = _long_route_config()
    sources = [Generator("sampling", seed=0x0D160831, n_spans=300_000, rank=r, world=3) for r in range(3)]
    for r, g in enumerate(sources):
        inject_zero_starts(g, 0.01, 40 + r)
        g.keep_arena = _with_long_routes(g, 20 + r)
    got, _ = _local_round(sources, cfg)
    want = _concat_keep_oracle(sources, cfg)
    for gk, wk in zip(got, want):
        np.testing.assert_array_equal(gk, wk)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_wide_config_oracle_vs_python(name):
    cfg = CONFIGS[name]()
    check_interning(cfg)
    g = Generator("sampling", seed=0x0D1607A1, n_spans=2500)
    inject_zero_starts(g, 0.03, 5)
    cols = g.cols
    ho = oracle_run(cols, native.GROUP_TRACE_ID, cfg=cfg)
    traces = _group(cols, False)
    svc_ids = intern_services(cfg)
    res = _arr(cols.resource, C.c_uint32, cols.n_spans)
    tid = _arr(cols.trace_id, C.c_uint64, 2 * cols.n_spans).reshape(-1, 2)
    levels = set()
    for t, spans in enumerate(traces):
        u = orc_lib().orc_trace_uniform(int(tid[spans[0], 0]), int(tid[spans[0], 1]), SEED)
        k, lvl, ratio = _py_eval(cfg, svc_ids, cols, res, spans, False, u)
        assert ho.view("trace_level", np.uint8)[t] == lvl, t
        assert ho.view("trace_ratio", np.float64)[t] == ratio, t
        assert ho.view("trace_keep", np.uint8)[t] == int(k), t
        levels.add(lvl)
    assert len(levels) >= 2, levels


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CONFIGS))
@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_wide_config(name, shuffle):
    # contiguous traces (fast path) and resource-shuffled ones (repeated ids:
    # the run-list and sort paths redo the fast path's provisional walk)
    g = Generator("sampling", seed=0x0D1607B1 + int(shuffle), n_spans=200_000, shuffle=shuffle)
    inject_zero_starts(g, 0.01, 9)
    gpu_vs_oracle(g, cfg=CONFIGS[name]())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["latency", "latency2", "latency_split"])
@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_multi_chunk_pass(name, shuffle):
    # 2 and 3 rule chunks without span_attribute rules: every chunk in one
    # pass over the columns (trace_multi_kernel); a batch with repeated trace
    # ids is then redone pass per chunk (trace_eval_kernel, the slow paths)
    g = Generator("sampling", seed=0x0D160901 + int(shuffle), n_spans=300_000, shuffle=shuffle)
    inject_zero_starts(g, 0.01, 7)
    ran = set()
    ho = gpu_vs_oracle(g, cfg=CONFIGS[name](), kernels=ran)
    assert "trace_multi_kernel" in ran, ran
    assert ("trace_eval_kernel" in ran) == shuffle, ran
    t = int(ho.view("trace_count", np.uint32)[0])
    assert len(set(ho.view("trace_level", np.uint8)[:t].tolist())) >= 2


@pytest.mark.gpu
def test_gpu_multi_chunk_pass_many_rules():
    # a chunk of more than 128 rules (150 service_name rules sharing 4 service
    # bits, then 100 latency rules): the pass per chunk decides it
    cfg = wide_latency2_config()
    cfg["service_rules"] = [_wide_svc_rule(k) for k in range(150)]
    assert _chunks(cfg) == 2
    g = Generator("sampling", seed=0x0D160931, n_spans=200_000)
    ran = set()
    gpu_vs_oracle(g, cfg=cfg, kernels=ran)
    assert "trace_multi_kernel" not in ran and "trace_eval_kernel" in ran, ran


def _wide_svc_rule(k):
    from tests.workloads import _wide_svc
    return _wide_svc(k, k % 4)


@pytest.mark.gpu
def test_gpu_multi_chunk_pass_edges():
    # batches of one span, one step, a ragged last step and one long trace
    # followed by its owner wave (no long-run hand-off in the one-pass form)
    from tests.workloads import wide_latency_config
    for n in (1, 63, 64, 65, 1000):
        ran = set()
        gpu_vs_oracle(Generator("sampling", seed=0x0D160911 + n, n_spans=n), cfg=wide_latency_config(), kernels=ran)
        assert "trace_multi_kernel" in ran
    g = Generator("zipf", seed=0x0D160921, n_spans=200_000)
    inject_zero_starts(g, 0.01, 4)
    ran = set()
    gpu_vs_oracle(g, cfg=wide_latency_config(), kernels=ran)
    assert "trace_multi_kernel" in ran


def _attr_bits(g, rules, seed, p=0.02):
    # the shim's attr_match column for json span_attribute rules: bit k = the
    # k-th span_attribute rule in level order met by the span; past 64 rules
    # word k // 64 (word-major planes, ose_columns.attr_match_words)
    rng = np.random.default_rng(seed)
    n = g.cols.n_spans
    W = max(1, (rules + 63) // 64)
    bits = np.zeros((W, n), dtype=np.uint64)
    for k in range(rules):
        bits[k // 64] |= (rng.random(n) < p).astype(np.uint64) << np.uint64(k % 64)
    g.cols.attr_match = bits.ctypes.data
    g.cols.attr_match_words = W
    return bits   # (the caller keeps it alive)


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_wide_config_attr_bits_across_chunks(shuffle):
    # span_attribute bits 0..13 in one chunk, 14..39 in the next (attr_base)
    check_interning(wide_attr_config())
    g = Generator("sampling", seed=0x0D1607F1 + int(shuffle), n_spans=200_000, shuffle=shuffle)
    keep_alive = _attr_bits(g, 40, seed=17)
    ho = gpu_vs_oracle(g, cfg=wide_attr_config())
    t = int(ho.view("trace_count", np.uint32)[0])
    assert len(set(ho.view("trace_level", np.uint8)[:t].tolist())) >= 2
    del keep_alive


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_attr_rules_past_64(shuffle):
    # 100 span_attribute rules: attr_match in two words, the middle rule
    # chunk's bits straddling them (attr_base 24: words 0 and 1)
    check_interning(wide_attr100_config())
    g = Generator("sampling", seed=0x0D160801 + int(shuffle), n_spans=300_000, shuffle=shuffle)
    keep_alive = _attr_bits(g, 100, seed=23, p=0.01)
    ho = gpu_vs_oracle(g, cfg=wide_attr100_config())
    t = int(ho.view("trace_count", np.uint32)[0])
    assert len(set(ho.view("trace_level", np.uint8)[:t].tolist())) >= 2
    del keep_alive


@pytest.mark.gpu
def test_gpu_wide_config_long_traces():
    # Zipf trace sizes: runs past the fast pass's windows go to trace_long_kernel
    g = Generator("zipf", seed=0x0D1607C1, n_spans=400_000)
    inject_zero_starts(g, 0.01, 4)
    gpu_vs_oracle(g, cfg=wide_mixed_config(), seed=0xDEADBEEF)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 65, 5000])
def test_gpu_wide_config_batch_mode(n):
    if n == 0:
        g = Generator("sampling", seed=1, n_spans=1)
        g.cols.n_spans = 0
    else:
        g = Generator("sampling", seed=0x0D1607D1 + n, n_spans=n)
    gpu_vs_oracle(g, mode=native.GROUP_BATCH, cfg=wide_latency_config())


@pytest.mark.gpu
def test_gpu_wide_config_large():
    # 2M spans through three chunks, per-trace outputs off (the bench shape)
    g = Generator("sampling", seed=0x0D1607E1, n_spans=2_000_000, threads=8)
    gpu_vs_oracle(g, cfg=wide_latency_config(), per_trace=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["attr", "attr100", "latency", "long_routes", "mixed"])
def test_gpu_wide_config_exchange_world3(name):
    # chunked rule lists through the trace-id exchange (ose_exchange_sample's
    # round at world 3, in-process transport): a record carries one endpoint
    # and one rule word per rule chunk, the owner runs every chunk's pass on
    # its plane; traces straddle ranks, and every rank's keep equals the
    # oracle on the concatenated global batch
    from tests.test_exchange import _concat_keep_oracle, _local_round
    cfg = {"attr": wide_attr_config, "attr100": wide_attr100_config}.get(name, CONFIGS.get(name))()
    sources = [Generator("sampling", seed=0x0D160811, n_spans=600_000, rank=r, world=3) for r in range(3)]
    for r, g in enumerate(sources):
        inject_zero_starts(g, 0.01, 30 + r)
        if name in ("attr", "attr100"):
            g.attr_bits = _attr_bits(g, 40 if name == "attr" else 100, seed=50 + r, p=0.01)
    assert _chunks(cfg) >= 2
    got, stats = _local_round(sources, cfg)
    want = _concat_keep_oracle(sources, cfg)
    for gk, wk in zip(got, want):
        np.testing.assert_array_equal(gk, wk)
    assert sum(s[0] for s in stats) == sum(s[1] for s in stats) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 65, 5000])
def test_gpu_many_services_batch_mode(n):
    # one decision per call over chunk-local service ids (every resource's
    # service, spanless ones included: servicename.go:38-47)
    g = Generator("sampling", seed=0x0D160951 + n, n_spans=n)
    gpu_vs_oracle(g, native.GROUP_BATCH, cfg=many_services_config())


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_services", [(2, 1200), (3, 1200), (3, 5000)])
def test_gpu_many_services_exchange(world, n_services):
    # a config past the dense service tables (chunk-local service ids, 19+
    # rule chunks) through ose_exchange_sample's round (in-process transport):
    # records carry global service ids, the pack and the owner fold map them
    # through each chunk's table (ShardArgs / OwnerArgs::svc_maps); traces
    # straddle ranks, zero starts reset minStart, and every rank's keep equals
    # the oracle on the concatenated global batch.  The same config decides
    # at N = 1 (test_gpu_many_services_config), so no config is refused at
    # N > 1 that N = 1 runs.
    from tests.test_exchange import _concat_keep_oracle, _local_round
    cfg = many_services_config(n_services)
    sources = [Generator("sampling", seed=0x0D160961 + world, n_spans=400_000, rank=r, world=world)
               for r in range(world)]
    for r, g in enumerate(sources):
        inject_zero_starts(g, 0.01, 70 + r)
    got, stats = _local_round(sources, cfg)
    want = _concat_keep_oracle(sources, cfg)
    for gk, wk in zip(got, want):
        np.testing.assert_array_equal(gk, wk)
    assert sum(s[0] for s in stats) == sum(s[1] for s in stats) > 0


@pytest.mark.gpu
def test_gpu_many_services_owner_general_path():
    # the owner's general path (records unpacked into columns, then the SAMPLE
    # stage, which translates the records' global ids per chunk) on the same
    # records as the bucketed fold: byte-identical keep
    from tests.test_exchange import _decide_both, _owner_recvs
    sources = [Generator("sampling", seed=0x0D160971, n_spans=300_000, rank=r, world=3) for r in range(3)]
    for r, g in enumerate(sources):
        inject_zero_starts(g, 0.01, 80 + r)
    eng, recvs, rb = _owner_recvs(sources, many_services_config())
    for recv in recvs:
        fold, ref, general = _decide_both(eng, recv, rb)
        np.testing.assert_array_equal(fold, ref)
        assert not general


@pytest.mark.gpu
def test_gpu_match_planes_checked_against_chunks():
    # route_match / svc_match bits are chunk-local rule indices: an engine with
    # K > 1 chunks refuses caller planes unless match_planes == K (plane 0 read
    # for every chunk would decide chunks 1..K-1 on chunk 0's bits); with a
    # spilled route the engine builds K route planes itself, so a caller's
    # one-plane svc_match is refused rather than read past its end
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    for cfg in (_long_route_config(), wide_latency_config()):
        eng = Engine({"odigossampling": cfg})
        assert _chunks(cfg) > 1
        g = Generator("sampling", seed=0x0D160851, n_spans=5000)
        db = DeviceBatch(g.cols)
        n = g.cols.n_spans
        plane = torch.zeros(8 * n, dtype=torch.uint8, device="cuda")
        for field in ("svc_match", "route_match"):
            for planes in (0, 1):
                setattr(db.cols, field, plane.data_ptr())
                db.cols.match_planes = planes
                with pytest.raises(native.OseError) as ei:
                    eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID)
                assert ei.value.code == native.OSE_EINVAL
                setattr(db.cols, field, 0)
        db.cols.match_planes = 0
        eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID)
        torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_spilled_route_config_without_route_column():
    # a batch without an http.route column (and no route_match) is refused the
    # same way whether or not the config spills a route past the LDS table:
    # http_latency rules need the route bytes (no spill-specific failure)
    from odigos_amd.batch import DeviceBatch, Engine
    from tests.workloads import c3_sampling_config
    msgs = []
    for cfg in (c3_sampling_config(), _long_route_config()):
        g = Generator("sampling", seed=0x0D160861, n_spans=20_000)
        g.cols.route = None
        eng = Engine({"odigossampling": cfg})
        db = DeviceBatch(g.cols)
        with pytest.raises(native.OseError) as ei:
            eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID)
        assert ei.value.code == native.OSE_EINVAL
        msgs.append(str(ei.value))
    assert msgs[0] == msgs[1]
