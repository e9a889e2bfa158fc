"""Randomised parity for odigosurltemplate.

CPU: the oracle's hand-written built-in matchers (oracle/url.c) against
Python `re` running the reference's regexps (templatize.go:10-74) with Go's
end-of-text `$`, on random ASCII segments (byte-level semantics coincide for
ASCII).  GPU: the HIP templater against the oracle on seeded synthetic
batches (C2 mix), byte-exact on url_out, template refs and the output arena.
"""
import random
import re

import numpy as np
import pytest

from odigos_amd import native
from odigos_amd.batch import DeviceBatch, Engine, Generator, HostOutputs
from tests.oracle_lib import UrlOracle

NO_LETTERS = re.compile(rb"^[\d_\-!@#$%^&*()=+{}\[\]:;\"'<>,.?/\\|`~]+\Z")
UUID = re.compile(rb"(^[0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12})|"
                  rb"([0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12}\Z)")
HEX = re.compile(rb"^(?:[0-9a-fA-F]{2}){8,}\Z")
LONGNUM = re.compile(rb"[0-9]{7,}")
DATE = re.compile(rb"^[0-9]{4}-[0-9]{2}-[0-9]{2}(?:T[0-9]{2}:[0-9]{2}(?::[0-9]{2})?)?(?:Z|[+-][0-9]{4})?\Z")
EMAIL = re.compile(rb"^[a-zA-Z0-9._%+-]+@[a-zA-Z0-9.-]+\.[a-zA-Z]{2,}\Z")


def reference_name(seg: bytes):
    """getSegmentTemplatizationString (templatize.go:242-269) with Python re."""
    if DATE.search(seg):
        return "date"
    if EMAIL.search(seg):
        return "email"
    if NO_LETTERS.search(seg) or LONGNUM.search(seg) or UUID.search(seg) or HEX.search(seg):
        return "id"
    return None


def _segments(rng: random.Random, n: int):
    alpha = "0123456789abcdefABCDEFxyzT-_.@:+Z"
    out = []
    for _ in range(n):
        kind = rng.randrange(8)
        if kind == 0:
            s = "".join(rng.choice("0123456789-_.") for _ in range(rng.randrange(1, 12)))
        elif kind == 1:
            s = "".join(rng.choice("0123456789abcdefABCDEF") for _ in range(rng.randrange(12, 40)))
        elif kind == 2:
            g = ["".join(rng.choice("0123456789abcdef") for _ in range(k)) for k in (8, 4, 4, 4, 12)]
            s = "-".join(g)
            if rng.random() < 0.5:
                s = rng.choice(["x_", "", "PRE"]) + s + rng.choice(["", "_y", "Z"])
            if rng.random() < 0.3:
                i = rng.randrange(len(s))
                s = s[:i] + rng.choice("g-") + s[i + 1:]
        elif kind == 3:
            s = "2025-%02d-%02d" % (rng.randrange(100), rng.randrange(100))
            if rng.random() < 0.6:
                s += "T%02d:%02d" % (rng.randrange(100), rng.randrange(100))
                if rng.random() < 0.5:
                    s += ":%02d" % rng.randrange(100)
            s += rng.choice(["", "Z", "+0000", "-0530", "+00", "ZZ", ":"])
        elif kind == 4:
            s = "".join(rng.choice("ab.c_+%-") for _ in range(rng.randrange(0, 5))) + "@" + \
                "".join(rng.choice("ab.c-1") for _ in range(rng.randrange(0, 8))) + rng.choice(["", ".io", ".c", ".co1", "."])
        else:
            s = "".join(rng.choice(alpha) for _ in range(rng.randrange(0, 30)))
        out.append(s.encode())
    return out


def test_builtin_matchers_vs_python_re():
    rng = random.Random(0x0D160002)
    orc = UrlOracle({})
    for seg in _segments(rng, 20000):
        assert orc.segment_name(seg) == reference_name(seg), seg


def test_apply_path_shapes():
    orc = UrlOracle({})
    assert orc.apply_path(b"") == b"/"
    assert orc.apply_path(b"/") == b"/"
    assert orc.apply_path(b"//") == b"//"
    assert orc.apply_path(b"a/1") == b"a/{id}"           # no leading slash, templated
    assert orc.apply_path(b"a/b") == b"/a/b"             # no leading slash, untouched -> slash-prefixed
    assert orc.apply_path(b"/1/") == b"/{id}/"
    assert orc.apply_path(b"/x/\xc3") == b"/x/{id}"      # invalid UTF-8 -> U+FFFD -> id


def test_generator_oracle_smoke():
    g = Generator("url", seed=0x0D160002, n_spans=20000)
    ho = HostOutputs(g.cols)
    orc = UrlOracle({})
    assert orc.process(g.cols, ho.outs, nthreads=4) == 0
    out = ho.view("url_out", np.uint8)[: g.cols.n_spans]
    # the C2 mix: a large share of spans is templated, some renamed
    assert (out & native.OUT_SET_ATTR).mean() > 0.3
    assert (out & native.OUT_RENAME).mean() > 0.2
    # multi-threaded oracle == single-threaded oracle
    ho1 = HostOutputs(g.cols)
    assert orc.process(g.cols, ho1.outs, nthreads=1) == 0
    assert int(ho.used[0]) == int(ho1.used[0])
    n = int(ho.used[0])
    assert bytes(ho.bufs["tmpl_arena"][:n]) == bytes(ho1.bufs["tmpl_arena"][:n])


def run_gpu_vs_oracle(cfg, workload, seed, n, shuffle=False):
    g = Generator(workload, seed=seed, n_spans=n, shuffle=shuffle)
    eng = Engine({"odigosurltemplate": cfg})
    db = DeviceBatch(g.cols)
    eng.process_device(db, native.STAGE_TEMPLATE)
    import torch
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = HostOutputs(g.cols)
    orc = UrlOracle(cfg)
    assert orc.process(g.cols, ho.outs, nthreads=8) == 0
    ns = g.cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("url_out")[:ns], ho.view("url_out", np.uint8)[:ns])
    gt = db.out_numpy("tmpl", np.uint32)[: 2 * ns].reshape(-1, 2)
    ot = ho.view("tmpl", np.uint32)[: 2 * ns].reshape(-1, 2)
    mask = ho.view("url_out", np.uint8)[:ns] != 0
    np.testing.assert_array_equal(gt[mask], ot[mask])
    used = db.used()
    assert used == int(ho.used[0])
    np.testing.assert_array_equal(db.out_numpy("tmpl_arena")[:used], ho.bufs["tmpl_arena"][:used])
    return ns, used


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 256, 257, 100_000])
def test_gpu_url_parity_small(n):
    run_gpu_vs_oracle({}, "url", 0x0D160002 + n, n)


@pytest.mark.gpu
def test_gpu_url_parity_rules_and_custom_ids():
    cfg = {
        "templatization_rules": ["/users/{user}/orders/{order:\\d+}", "/api/v1/*", "/regex:v[12]/items/{id}",
                                 "/{a}/{b}/{c}/{d}/{e}/{f}"],
        "custom_ids": [{"regexp": "^inc_\\d+$", "template_name": "incident"}, {"regexp": "^INC\\d{4}", "template_name": "ticket"},
                       {"regexp": "(?i)^PROCESS_"}],
    }
    run_gpu_vs_oracle(cfg, "url", 0x0D160012, 200_000)


@pytest.mark.gpu
def test_gpu_url_parity_include_exclude_column():
    # res_url_ok is host-computed; an exclude list makes the kernel read it
    cfg = {"exclude": {"k8s_workloads": [{"namespace": "ns", "kind": "Deployment", "name": "x"}]}}
    run_gpu_vs_oracle(cfg, "fused", 0x0D160022, 150_000, shuffle=True)


@pytest.mark.gpu
def test_gpu_url_parity_full_c2():
    # BASELINE.json configs[1]: 10M spans, C2 mix, byte-exact against the oracle
    ns, used = run_gpu_vs_oracle({}, "url", 0x0D160002, 10_000_000)
    assert ns == 10_000_000 and used > 0


def _gpu_vs_oracle_cols(g, cfg, arena_bytes=None):
    """run_gpu_vs_oracle on prepared columns; arena_bytes overrides what the
    device batch declares (it sizes the plan kernel's scratch)."""
    import torch
    eng = Engine({"odigosurltemplate": cfg})
    db = DeviceBatch(g.cols)
    if arena_bytes is not None:
        db.cols.arena_bytes = arena_bytes
    eng.process_device(db, native.STAGE_TEMPLATE)
    torch.cuda.synchronize()
    assert int(db.out_numpy("device_status", np.uint32)[0]) == 0
    ho = HostOutputs(g.cols)
    assert UrlOracle(cfg).process(g.cols, ho.outs, nthreads=8) == 0
    ns = g.cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("url_out")[:ns], ho.view("url_out", np.uint8)[:ns])
    gt = db.out_numpy("tmpl", np.uint32)[: 2 * ns].reshape(-1, 2)
    ot = ho.view("tmpl", np.uint32)[: 2 * ns].reshape(-1, 2)
    mask = ho.view("url_out", np.uint8)[:ns] != 0
    np.testing.assert_array_equal(gt[mask], ot[mask])
    used = db.used()
    assert used == int(ho.used[0])
    np.testing.assert_array_equal(db.out_numpy("tmpl_arena")[:used], ho.bufs["tmpl_arena"][:used])
    return used


@pytest.mark.gpu
def test_gpu_url_parity_group_images_over_lds():
    # every path stretched to 200 arena bytes (overlapping its neighbours'):
    # a group's template outgrows the plan kernel's LDS image, so the group is
    # listed for url_emit_slow_kernel and url_copy_kernel leaves its bytes alone
    g = Generator("url", seed=0x0D160032, n_spans=20_000)
    path = g.array("path").view(np.uint32).reshape(-1, 2)
    has = path[:, 1] > 0
    path[has, 1] = np.minimum(200, g.cols.arena_bytes - path[has, 0]).astype(np.uint32)
    used = _gpu_vs_oracle_cols(g, {})
    assert used > 0


@pytest.mark.gpu
def test_gpu_url_parity_scratch_regions_overflow():
    # arena_bytes understated to 0: each plan wave's scratch region holds only
    # a few group images, the rest fall back to the per-span writer
    g = Generator("url", seed=0x0D160042, n_spans=2_000_000, threads=8)
    _gpu_vs_oracle_cols(g, {}, arena_bytes=0)


@pytest.mark.gpu
def test_gpu_url_parity_paths_spread_through_the_arena():
    # the path refs of a C2 batch permuted across its spans: every group's
    # paths lie anywhere in the 10 MB arena (as in an OTLP-decoded batch), so
    # url_plan_kernel stages them by the per-lane gather, and groups whose
    # chunks outgrow the stage go to url_plan_slow_kernel's subsets
    g = Generator("url", seed=0x0D160052, n_spans=300_000, threads=8)
    path = g.array("path").view(np.uint32).reshape(-1, 2)
    has = np.flatnonzero(path[:, 1] > 0)
    perm = np.random.default_rng(0x0D160052).permutation(has.size)
    path[has] = path[has][perm]
    used = _gpu_vs_oracle_cols(g, {})
    assert used > 0


def _long_rule_cfg():
    # a templatization rule of 70 segments (the reference has no limit:
    # parseUserInputRuleString, templatize.go:97-138)
    segs = ["seg%d" % k for k in range(70)]
    segs[3] = "{id}"
    segs[69] = "{last:\\d+}"
    return {"templatization_rules": ["/" + "/".join(segs), "/users/{user}"]}


def test_long_rule_accepted_at_creation():
    import ctypes as C
    import json
    h = C.c_void_p()
    rc = native.lib().ose_engine_create(json.dumps({"odigosurltemplate": _long_rule_cfg()}).encode(), C.byref(h))
    assert rc in (0, native.OSE_EDEVICE), (rc, native.last_error())
    if rc == 0:
        native.lib().ose_engine_destroy(h)


@pytest.mark.gpu
def test_gpu_url_parity_rule_longer_than_64_segments():
    import torch
    from tests.test_unicode_regex import _cols_from_paths
    rng = random.Random(0x0D1600D1)
    paths = []
    for k in range(3000):
        segs = ["seg%d" % j for j in range(70)]
        segs[3] = str(rng.randrange(10**6))
        segs[69] = str(rng.randrange(10**6)) if k % 3 else "x%d" % k
        if k % 5 == 0:
            segs = segs[: rng.randrange(60, 75)]
        paths.append(("/" + "/".join(segs)).encode())
    cols, _keep = _cols_from_paths(paths)
    cfg = _long_rule_cfg()
    eng = Engine({"odigosurltemplate": cfg})
    db = DeviceBatch(cols)
    eng.process_device(db, native.STAGE_TEMPLATE)
    torch.cuda.synchronize()
    ho = HostOutputs(cols)
    assert UrlOracle(cfg).process(cols, ho.outs, 4) == 0
    n = cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("url_out", n=n), ho.view("url_out", np.uint8)[:n])
    used = db.used()
    assert used == int(ho.used[0])
    np.testing.assert_array_equal(db.out_numpy("tmpl_arena", n=used), ho.bufs["tmpl_arena"][:used])
    assert b"{last}" in ho.bufs["tmpl_arena"][:used].tobytes()
