"""odigossampling parity on seeded synthetic batches.

CPU: the C oracle (oracle/sampling.c) against an independent pure-Python
restatement of rule_engine.go / internal/sampling/*.go on small batches
(zero start timestamps, shuffled traces, fractional ratios included), and
thread-count invariance.
GPU (@gpu): the HIP trace stage against the oracle, bit-exact on keep,
trace order, level, ratio and decision, from tiny batches to the full C3
size (50M spans / ~5M traces), with contiguous traces (fast path) and
resource-shuffled traces (sort-based slow path).
"""
import numpy as np
import pytest

from odigos_amd import native
from odigos_amd.batch import Generator, HostOutputs
from tests.oracle_lib import SamplingOracle, intern_services, lib as orc_lib
from tests.workloads import c3_sampling_config, check_interning

CFG = c3_sampling_config()
SEED = 0x5EED


def test_c3_config_interning():
    check_interning(CFG)


# ---------------- independent pure-Python restatement ----------------
def _arr(addr, ctype, n):
    import ctypes as C
    return np.ctypeslib.as_array((ctype * max(n, 1)).from_address(addr))[:n]


def _py_eval(cfg, svc_ids, cols, res, spans, batch_mode, u):
    import ctypes as C
    n = cols.n_spans
    status = _arr(cols.status, C.c_uint8, n)
    start = _arr(cols.start_ns, C.c_uint64, n)
    end = _arr(cols.end_ns, C.c_uint64, n)
    route = _arr(cols.route, C.c_uint32, 2 * n).reshape(-1, 2)
    arena = _arr(cols.arena, C.c_uint8, cols.arena_bytes)
    res_svc = _arr(cols.res_svc, C.c_uint32, cols.n_resources)
    res_str = _arr(cols.res_svc_str, C.c_uint32, cols.n_resources)

    def ev(rule):
        d = rule["rule_details"]
        t = rule["type"]
        if t == "error":
            return (True, True, 100.0) if any(status[i] == 2 for i in spans) else (True, False, float(d["fallback_sampling_ratio"]))
        if t == "http_latency":
            sid = svc_ids[d["service_name"]]
            sf = ef = False
            ms_ = me = 0
            pre = d["http_route"].encode()
            for i in spans:
                if res_svc[res[i]] != sid:
                    continue
                sf = True
                o, ln = route[i]
                if bytes(arena[o:o + ln]).startswith(pre):
                    ef = True
                s, e = int(start[i]), int(end[i])
                if ms_ == 0 or s < ms_:
                    ms_ = s
                if me == 0 or e > me:
                    me = e
            if not sf or not ef:
                return (False, False, 0.0)
            a, b = me - (1 << 64) * (me >> 63), ms_ - (1 << 64) * (ms_ >> 63)
            dd = max(min(a - b, (1 << 63) - 1), -(1 << 63))
            ms = int(dd / 1_000_000) if dd >= 0 else -int(-dd // 1_000_000)
            if ms >= int(d["threshold"]):
                return (True, True, 100.0)
            return (True, False, float(d["fallback_sampling_ratio"]))
        sid = svc_ids[d["service_name"]]
        rs = range(cols.n_resources) if batch_mode else {int(res[i]) for i in spans}
        if any(res_str[r] == sid for r in rs):
            return (True, True, float(d["sampling_ratio"]))
        return (False, False, float(d["fallback_sampling_ratio"]))

    min_fb = None
    for lvl, key in enumerate(("global_rules", "service_rules", "endpoint_rules")):
        ratio, sat, matched, fb = 0.0, False, False, False
        for rule in cfg.get(key) or []:
            m, s, p = ev(rule)
            if s:
                sat, ratio, matched = True, max(ratio, p), True
            elif m:
                matched = True
                if not fb:
                    ratio, fb = p, True
                else:
                    ratio = min(ratio, p)
        if sat:
            return u * 100 < ratio, lvl, ratio
        if matched and (min_fb is None or ratio < min_fb):
            min_fb = ratio
    if min_fb is not None:
        return u * 100 < min_fb, 3, min_fb
    return True, 4, 100.0


def _group(cols, batch_mode):
    import ctypes as C
    n = cols.n_spans
    if batch_mode:
        return [list(range(n))]
    tid = _arr(cols.trace_id, C.c_uint64, 2 * n).reshape(-1, 2)
    order, groups = [], {}
    for i in range(n):
        k = (int(tid[i, 0]), int(tid[i, 1]))
        if k not in groups:
            groups[k] = []
            order.append(k)
        groups[k].append(i)
    return [groups[k] for k in order]


def oracle_run(cols, mode, seed=SEED, nthreads=8, cfg=CFG):
    ho = HostOutputs(cols)
    assert SamplingOracle(cfg).process(cols, ho.outs, mode, seed, nthreads) == 0
    return ho


def inject_zero_starts(g, frac, seed):
    st = g.array("start_ns").view(np.uint64)
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(st), size=max(1, int(len(st) * frac)), replace=False)
    st[idx] = 0


def fractional_config():
    cfg = c3_sampling_config()
    for k, r in enumerate(cfg["endpoint_rules"]):
        r["rule_details"]["fallback_sampling_ratio"] = 33.3 + k
    return cfg


@pytest.mark.parametrize("shuffle,zero,mode", [(False, False, native.GROUP_TRACE_ID), (True, True, native.GROUP_TRACE_ID),
                                               (False, True, native.GROUP_BATCH)])
def test_oracle_vs_python(shuffle, zero, mode):
    import ctypes as C
    cfg = fractional_config()
    g = Generator("sampling", seed=0x0D160103 + int(shuffle), n_spans=3000 if mode == native.GROUP_TRACE_ID else 400,
                  shuffle=shuffle)
    if zero:
        inject_zero_starts(g, 0.05, 7)
    cols = g.cols
    ho = oracle_run(cols, mode, cfg=cfg)
    traces = _group(cols, mode == native.GROUP_BATCH)
    assert int(ho.view("trace_count", np.uint32)[0]) == len(traces)
    svc_ids = intern_services(cfg)
    res = _arr(cols.resource, C.c_uint32, cols.n_spans)
    tid = _arr(cols.trace_id, C.c_uint64, 2 * cols.n_spans).reshape(-1, 2)
    keep = ho.view("keep", np.uint8)
    for t, spans in enumerate(traces):
        u = orc_lib().orc_trace_uniform(int(tid[spans[0], 0]), int(tid[spans[0], 1]), SEED)
        k, lvl, ratio = _py_eval(cfg, svc_ids, cols, res, spans, mode == native.GROUP_BATCH, u)
        assert ho.view("trace_level", np.uint8)[t] == lvl, t
        assert ho.view("trace_ratio", np.float64)[t] == ratio, t
        assert ho.view("trace_keep", np.uint8)[t] == int(k), t
        assert ho.view("trace_first_span", np.uint32)[t] == spans[0]
        assert all(keep[i] == int(k) for i in spans)


def test_oracle_thread_invariance():
    g = Generator("sampling", seed=0x0D160003, n_spans=200_000, shuffle=True)
    a = oracle_run(g.cols, native.GROUP_TRACE_ID, nthreads=1)
    b = oracle_run(g.cols, native.GROUP_TRACE_ID, nthreads=8)
    for f in ("keep", "trace_keep", "trace_level", "trace_ratio", "trace_first_span", "trace_count"):
        np.testing.assert_array_equal(a.bufs[f], b.bufs[f])


def test_oracle_levels_cover_all_outcomes():
    g = Generator("sampling", seed=0x0D160003, n_spans=300_000)
    ho = oracle_run(g.cols, native.GROUP_TRACE_ID)
    t = int(ho.view("trace_count", np.uint32)[0])
    levels = np.bincount(ho.view("trace_level", np.uint8)[:t], minlength=5)
    # every level outcome appears in the C3 mix (global error satisfied, service, endpoint, fallback)
    assert levels[0] > 0 and levels[1] > 0 and levels[2] > 0 and levels[3] > 0, levels


# ---------------- GPU parity ----------------
def gpu_vs_oracle(g, mode=native.GROUP_TRACE_ID, cfg=CFG, per_trace=True, seed=SEED, kernels=None, paths=None):
    """kernels: a set the names of the launches the call profiled are added to;
    paths: a dict that receives the engine's slow-path counts after the call"""
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    eng = Engine({"odigossampling": cfg})
    db = DeviceBatch(g.cols)
    if not per_trace:
        for f in ("trace_count", "trace_first_span", "trace_keep", "trace_level", "trace_ratio"):
            setattr(db.outs, f, None)
    if kernels is not None:
        eng.profile(True)
    eng.process_device(db, native.STAGE_SAMPLE, mode, seed=seed)
    torch.cuda.synchronize()
    if kernels is not None:
        kernels.update(eng.profile_read())
    if paths is not None:
        paths.update(eng.path_counts())
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = oracle_run(g.cols, mode, seed=seed, cfg=cfg)
    n = g.cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("keep")[:n], ho.view("keep", np.uint8)[:n])
    if per_trace:
        t = int(ho.view("trace_count", np.uint32)[0])
        assert int(db.out_numpy("trace_count", np.uint32)[0]) == t
        np.testing.assert_array_equal(db.out_numpy("trace_first_span", np.uint32)[:t], ho.view("trace_first_span", np.uint32)[:t])
        np.testing.assert_array_equal(db.out_numpy("trace_level")[:t], ho.view("trace_level", np.uint8)[:t])
        np.testing.assert_array_equal(db.out_numpy("trace_ratio", np.float64)[:t], ho.view("trace_ratio", np.float64)[:t])
        np.testing.assert_array_equal(db.out_numpy("trace_keep")[:t], ho.view("trace_keep", np.uint8)[:t])
    return ho


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 1000, 100_000])
def test_gpu_sampling_parity_small(n):
    gpu_vs_oracle(Generator("sampling", seed=0x0D160003 + n, n_spans=n))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 100, 5000, 300_000])
def test_gpu_sampling_parity_shuffled(n):
    # resources permuted across the batch: traces split into several runs (slow path)
    gpu_vs_oracle(Generator("sampling", seed=0x0D160013 + n, n_spans=n, shuffle=True))


@pytest.mark.gpu
def test_gpu_sampling_zero_start_sentinel():
    # latency.go:69-73: a zero start resets minStart (both paths)
    for shuffle in (False, True):
        g = Generator("sampling", seed=0x0D160023, n_spans=200_000, shuffle=shuffle)
        inject_zero_starts(g, 0.02, 11)
        gpu_vs_oracle(g, cfg=fractional_config())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 64, 65, 5000])
def test_gpu_sampling_batch_mode(n):
    if n == 0:
        # one call with no spans is still one (empty) trace
        g = Generator("sampling", seed=1, n_spans=1)
        g.cols.n_spans = 0
    else:
        g = Generator("sampling", seed=0x0D160033 + n, n_spans=n)
    gpu_vs_oracle(g, mode=native.GROUP_BATCH)


@pytest.mark.gpu
def test_gpu_sampling_long_traces():
    # Zipf trace sizes up to 50k spans: runs cross many 64-span windows
    gpu_vs_oracle(Generator("zipf", seed=0x0D160005, n_spans=400_000))


@pytest.mark.gpu
def test_gpu_sampling_fractional_ratios_and_seeds():
    g = Generator("sampling", seed=0x0D160043, n_spans=150_000)
    for seed in (0, 1, 0xDEADBEEF):
        gpu_vs_oracle(g, cfg=fractional_config(), seed=seed)


@pytest.mark.gpu
def test_gpu_sampling_parity_full_c3():
    # BASELINE.json configs[2]: 50M spans / ~5M traces, keep bit-exact
    g = Generator("sampling", seed=0x0D160003, n_spans=50_000_000, threads=16)
    ho = gpu_vs_oracle(g, per_trace=True)
    assert int(ho.view("trace_count", np.uint32)[0]) > 4_000_000


def long_prefix_config():
    """http_route prefixes of every length 1..24 (crossing the 16-byte window
    of the vectorised HasPrefix) over the generator's routes
    /api/v{1,2}/<word>[/{id}][/<word>]."""
    cfg = c3_sampling_config()
    routes = ["/api/v1/users/{id}", "/api/v2/orders", "/api/v1/checkout/{id}/", "/api/v2/products/{id}",
              "/api/v1/users", "/api/v2/", "/", "/api/v1/items/{id}", "/api/v2/cart/{id}/users",
              "/api/v1/search/{id}", "/api/v1/settings/{id}", "/api/v2/billing/{id}", "/api/v1/invoices/{id}/",
              "/api/v2/payments", "/api/v1/authx", "/api/v1/login/{id}/"]
    for r, route in zip(cfg["endpoint_rules"], routes):
        r["rule_details"]["http_route"] = route
        r["rule_details"]["threshold"] = 1
    return cfg


def test_long_prefix_config_oracle_vs_python():
    import ctypes as C
    cfg = long_prefix_config()
    g = Generator("sampling", seed=0x0D160203, n_spans=4000)
    cols = g.cols
    ho = oracle_run(cols, native.GROUP_TRACE_ID, cfg=cfg)
    traces = _group(cols, False)
    svc_ids = intern_services(cfg)
    res = _arr(cols.resource, C.c_uint32, cols.n_spans)
    tid = _arr(cols.trace_id, C.c_uint64, 2 * cols.n_spans).reshape(-1, 2)
    matched = 0
    for t, spans in enumerate(traces):
        u = orc_lib().orc_trace_uniform(int(tid[spans[0], 0]), int(tid[spans[0], 1]), SEED)
        k, lvl, ratio = _py_eval(cfg, svc_ids, cols, res, spans, False, u)
        assert ho.view("trace_level", np.uint8)[t] == lvl and ho.view("trace_ratio", np.float64)[t] == ratio
        matched += lvl == 2
    assert matched > 0


@pytest.mark.gpu
def test_gpu_sampling_long_prefixes():
    gpu_vs_oracle(Generator("sampling", seed=0x0D160063, n_spans=300_000), cfg=long_prefix_config())
    gpu_vs_oracle(Generator("sampling", seed=0x0D160073, n_spans=100_000, shuffle=True), cfg=long_prefix_config())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0x0D160105, 0x0D160205])
def test_gpu_sampling_long_runs_split(seed):
    # runs still open kLongSteps steps past their owner's windows are decided
    # by trace_long_kernel (a workgroup folds contiguous pieces in order):
    # zero starts reset minStart inside and across the pieces, fractional
    # ratios make the decision depend on the injected uniform
    g = Generator("zipf", seed=seed, n_spans=600_000)
    inject_zero_starts(g, 0.01, seed & 0xFF)
    gpu_vs_oracle(g, cfg=fractional_config(), seed=seed)
    gpu_vs_oracle(g, cfg=long_prefix_config())


@pytest.mark.gpu
def test_gpu_sampling_long_runs_slow_path():
    # shuffled Zipf traces: split runs send the batch down the sort-based
    # path, which must overwrite the long-run decisions of the fast pass
    paths = {}
    gpu_vs_oracle(Generator("zipf", seed=0x0D160305, n_spans=300_000, shuffle=True), paths=paths)
    # a Zipf trace of more than 4096 spans in several runs overflows the run
    # lists: the radix sort by trace id decided this batch
    assert paths["run_list"] == 1 and paths["sort"] == 1, paths


def interleave(g, period):
    """The sampling columns of the spans reordered by residue mod `period`
    (spans 0, p, 2p, ..., then 1, p+1, ...): a trace of at least `period`
    spans becomes `period` runs scattered through the batch.  resource
    stays in place (it must stay non-decreasing), so a span takes the
    resource of its new position: a different but valid batch."""
    import ctypes as C
    n = g.cols.n_spans
    order = np.concatenate([np.arange(k, n, period) for k in range(period)])   # new p <- old order[p]
    for name, ctype, w in (("trace_id", C.c_uint64, 2), ("start_ns", C.c_uint64, 1), ("end_ns", C.c_uint64, 1),
                           ("status", C.c_uint8, 1), ("route", C.c_uint32, 2)):
        a = _arr(getattr(g.cols, name), ctype, w * n).reshape(n, w)
        a[:] = a[order].copy()


@pytest.mark.gpu
@pytest.mark.parametrize("period,n", [(9, 5000), (16, 100_000), (33, 300_000)])
def test_gpu_sampling_sort_path_decides(period, n):
    # SURVEY §8 a-1 / north_star's "LDS radix sort by trace_id": traces cut
    # into more than 8 runs (traces of >= period spans) overflow the run-list path (trace_fold_kernel),
    # so the batch is decided by the stable radix sort by first run head and
    # trace_eval_kernel over the sorted permutation; keep, trace order,
    # levels and ratios equal the oracle, and the engine's counters show the
    # sort path ran
    g = Generator("sampling", seed=0x0D160503 + period, n_spans=n)
    interleave(g, period)
    paths = {}
    gpu_vs_oracle(g, paths=paths)
    assert paths["run_list"] == 1 and paths["sort"] == 1, paths


@pytest.mark.gpu
def test_gpu_sampling_run_list_without_sort():
    # a trace split into 2 runs stays on the run-list path: no sort
    g = Generator("sampling", seed=0x0D160603, n_spans=20_000)
    import ctypes as C
    n = g.cols.n_spans
    tid = _arr(g.cols.trace_id, C.c_uint64, 2 * n).reshape(n, 2)
    tid[n - 1] = tid[0]   # the first trace reappears as the batch's last span
    paths = {}
    gpu_vs_oracle(g, paths=paths)
    assert paths["run_list"] == 1 and paths["sort"] == 0, paths


@pytest.mark.gpu
def test_gpu_sampling_parity_full_c5():
    # BASELINE.json configs[4]: 50M spans, Zipf(1.1) trace sizes up to 50k
    g = Generator("zipf", seed=0x0D160005, n_spans=50_000_000, threads=16)
    gpu_vs_oracle(g, per_trace=True)


@pytest.mark.gpu
@pytest.mark.parametrize("workload,shuffle", [("fused", False), ("fused", True), ("zipf", False), ("zipf", True)])
def test_gpu_sample_and_template_one_call(workload, shuffle):
    # SAMPLE | TEMPLATE in one call queues the URL launches between SAMPLE's
    # fast path and its host-gated rest: trace_long_kernel (Zipf: runs longer
    # than the fast pass walks), the slow path (shuffled: repeated trace
    # ids) and per-trace compaction (engine.cpp run_stages).  Keep, per-trace
    # records and URL outputs must all match the oracle.
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    from tests.oracle_lib import UrlOracle
    g = Generator(workload, seed=0x0D160044, n_spans=400_000 if workload == "zipf" else 200_000, shuffle=shuffle)
    if workload == "zipf":
        inject_zero_starts(g, 0.01, 3)
    eng = Engine({"odigossampling": CFG, "odigosurltemplate": {}})
    db = DeviceBatch(g.cols)
    eng.process_device(db, native.STAGE_SAMPLE | native.STAGE_TEMPLATE, native.GROUP_TRACE_ID, seed=SEED)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = oracle_run(g.cols, native.GROUP_TRACE_ID, seed=SEED, cfg=CFG)
    n = g.cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("keep")[:n], ho.view("keep", np.uint8)[:n])
    t = int(ho.view("trace_count", np.uint32)[0])
    assert int(db.out_numpy("trace_count", np.uint32)[0]) == t
    np.testing.assert_array_equal(db.out_numpy("trace_first_span", np.uint32)[:t], ho.view("trace_first_span", np.uint32)[:t])
    np.testing.assert_array_equal(db.out_numpy("trace_keep")[:t], ho.view("trace_keep", np.uint8)[:t])
    np.testing.assert_array_equal(db.out_numpy("trace_level")[:t], ho.view("trace_level", np.uint8)[:t])
    np.testing.assert_array_equal(db.out_numpy("trace_ratio", np.float64)[:t], ho.view("trace_ratio", np.float64)[:t])
    uo = HostOutputs(g.cols)
    assert UrlOracle({}).process(g.cols, uo.outs, nthreads=8) == 0
    np.testing.assert_array_equal(db.out_numpy("url_out")[:n], uo.view("url_out", np.uint8)[:n])
    used = db.used()
    assert used == int(uo.used[0])
    np.testing.assert_array_equal(db.out_numpy("tmpl_arena")[:used], uo.bufs["tmpl_arena"][:used])


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle,n", [(False, 300_000), (True, 300_000), (False, 2_000_000), (True, 50_000)])
def test_gpu_sampling_dup_detection(shuffle, n):
    # the fast path's duplicate detection (fingerprint buckets checked in
    # LDS) at several sizes: the same decisions as the oracle, repeated trace
    # ids (shuffled resources) found
    gpu_vs_oracle(Generator("sampling", seed=0x0D1600F0 + n, n_spans=n, shuffle=shuffle))


@pytest.mark.gpu
def test_gpu_sampling_many_service_rules():
    """service_name rules naming the same service share one per-trace bit
    (the rule is matched and satisfied iff the service occurs): 130 rules
    over 20 services, more rules than the trace stage's 64 bits, decide as
    the oracle does rule by rule."""
    cfg = c3_sampling_config()
    cfg["service_rules"] = [
        {"name": f"r{k}", "type": "service_name",
         "rule_details": {"service_name": f"svc-{k % 20:02d}", "sampling_ratio": float((k * 37) % 101),
                          "fallback_sampling_ratio": float(k % 7)}}
        for k in range(130)]
    check_interning(cfg)
    gpu_vs_oracle(Generator("sampling", seed=0x0D1601A5, n_spans=200_000), cfg=cfg)
