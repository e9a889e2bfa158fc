"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the
checker (test infrastructure; the product never loads it)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

from odigos_amd import native

import os

import numpy as np

# OSE_ORACLE_LIB: a host-tuned build of the same sources (bench.py builds one
# with -march=native on the GPU box for the CPU baseline)
ORACLE_PATH = Path(os.environ.get("OSE_ORACLE_LIB") or
                   Path(__file__).resolve().parent.parent / "oracle" / "liboracle.so")
_p = C.c_void_p
_L = None


class OrcRule(C.Structure):
    _fields_ = [("level", C.c_int32), ("type", C.c_int32), ("svc", C.c_uint32), ("route_len", C.c_uint32),
                ("route", C.c_char_p), ("threshold", C.c_int64), ("ratio", C.c_double), ("fallback", C.c_double),
                ("attr_col", C.c_int32), ("attr_expected_len", C.c_uint32), ("attr_cond", C.c_char_p),
                ("attr_op", C.c_char_p), ("attr_expected", C.c_char_p)]


def attr_key_columns(cfg: dict) -> list[str]:
    """The attr_type / attr_val key columns (include/odigos_amd.h): distinct
    attribute_key of the span_attribute rules whose condition_type is not
    "json", in level order (global, service, endpoint), config order inside."""
    keys = []
    for key in ("global_rules", "service_rules", "endpoint_rules"):
        for r in cfg.get(key) or []:
            d = r.get("rule_details") or {}
            if r["type"] == "span_attribute" and d.get("condition_type") != "json":
                if d.get("attribute_key") not in keys:
                    keys.append(d.get("attribute_key"))
    return keys


def lib():
    global _L
    if _L is None:
        L = C.CDLL(str(ORACLE_PATH))
        sig = {
            "orc_re_compile": (_p, [C.c_char_p, C.c_char_p, C.c_size_t]),
            "orc_re_match": (C.c_int, [_p, C.c_char_p, C.c_size_t]),
            "orc_re_free": (None, [_p]),
            "orc_url_create": (_p, [C.POINTER(C.c_char_p), C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                    C.c_int, C.c_char_p, C.c_size_t]),
            "orc_url_free": (None, [_p]),
            "orc_url_segment_name": (C.c_int, [_p, C.c_char_p, C.c_size_t, C.c_char_p]),
            "orc_url_apply_path": (C.c_long, [_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
            "orc_url_process": (C.c_int, [_p, C.POINTER(native.Columns), C.POINTER(native.Outputs), C.c_int]),
            "orc_sampling_create": (_p, [C.POINTER(OrcRule), C.c_int]),
            "orc_sampling_free": (None, [_p]),
            "orc_sampling_process": (C.c_int, [_p, C.POINTER(native.Columns), C.POINTER(native.Outputs), C.c_uint32,
                                               C.POINTER(native.Rand), C.c_int]),
            "orc_trace_uniform": (C.c_double, [C.c_uint64, C.c_uint64, C.c_uint64]),
            "orc_go_parse_float": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_double)]),
            "orc_go_parse_bool": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]),
            "orc_size_process": (C.c_int, [C.POINTER(native.Columns), C.POINTER(native.Outputs), C.c_uint32, C.c_uint32,
                                           C.POINTER(native.Outputs), C.c_int64, C.c_double, C.c_double]),
            "orc_size_process_mt": (C.c_int, [C.POINTER(native.Columns), C.POINTER(native.Outputs), C.c_uint32,
                                              C.c_uint32, C.POINTER(native.Outputs), C.c_int64, C.c_double, C.c_double,
                                              C.c_int]),
        }
        for name, (res, args) in sig.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                continue
            fn.restype = res
            fn.argtypes = args
        _L = L
    return _L


def _arr(strs):
    a = (C.c_char_p * max(len(strs), 1))()
    for i, s in enumerate(strs):
        a[i] = s if isinstance(s, bytes) else s.encode()
    return a


class Regex:
    def __init__(self, pattern: str):
        err = C.create_string_buffer(256)
        self.h = lib().orc_re_compile(pattern.encode(), err, 256)
        if not self.h:
            raise ValueError(err.value.decode())

    def match(self, s) -> bool:
        b = s if isinstance(s, bytes) else s.encode("utf-8", "surrogateescape")
        return bool(lib().orc_re_match(self.h, b, len(b)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_re_free(self.h)


class UrlOracle:
    """newUrlTemplateProcessor + processTraces restated (oracle/url.c)."""

    def __init__(self, cfg: dict | None = None):
        cfg = cfg or {}
        rules = cfg.get("templatization_rules", []) or []
        cids = cfg.get("custom_ids", []) or []
        err = C.create_string_buffer(512)
        self._keep = (_arr(rules), _arr([c.get("regexp", "") for c in cids]),
                      _arr([c.get("template_name", "") or "" for c in cids]))
        self.h = lib().orc_url_create(self._keep[0], len(rules), self._keep[1], self._keep[2], len(cids), err, 512)
        if not self.h:
            raise ValueError(err.value.decode())

    def segment_name(self, seg) -> str | None:
        b = seg if isinstance(seg, bytes) else seg.encode("utf-8", "surrogateescape")
        out = C.create_string_buffer(256)
        n = lib().orc_url_segment_name(self.h, b, len(b), out)
        return None if n < 0 else out.raw[:n].decode()

    def apply_path(self, path) -> bytes:
        b = path if isinstance(path, bytes) else path.encode("utf-8", "surrogateescape")
        cap = 64 + len(b) * 64
        out = C.create_string_buffer(cap)
        n = lib().orc_url_apply_path(self.h, b, len(b), out, cap)
        assert n >= 0
        return out.raw[:n]

    def process(self, cols, outs, nthreads: int = 1) -> int:
        return lib().orc_url_process(self.h, C.byref(cols), C.byref(outs), nthreads)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_url_free(self.h)


def intern_services(cfg: dict) -> dict:
    """Service-name ids in first-appearance order over global, service and
    endpoint rules (the ids the shim writes into res_svc / res_svc_str)."""
    ids = {}
    for lvl in ("global_rules", "service_rules", "endpoint_rules"):
        for r in cfg.get(lvl) or []:
            name = (r.get("rule_details") or {}).get("service_name")
            if r.get("type") in ("http_latency", "service_name", "span_attribute") and name is not None:
                ids.setdefault(name, len(ids))
    return ids


class SamplingOracle:
    """RuleEngine.ShouldSample per trace, restated (oracle/sampling.c)."""
    TYPES = {"error": 0, "http_latency": 1, "service_name": 2, "span_attribute": 3}

    def __init__(self, cfg: dict | None = None):
        cfg = cfg or {}
        self.services = intern_services(cfg)
        keys = attr_key_columns(cfg)
        rules = []
        for level, key in enumerate(("global_rules", "service_rules", "endpoint_rules")):
            for r in cfg.get(key) or []:
                d = r.get("rule_details") or {}
                if r["type"] not in self.TYPES:
                    raise ValueError(f"oracle: rule type {r['type']} not restated")
                route = (d.get("http_route") or "").encode()
                col, cond, op, exp = -1, b"", b"", b""
                if r["type"] == "span_attribute" and d.get("condition_type") != "json":
                    col = keys.index(d.get("attribute_key"))
                    cond = (d.get("condition_type") or "").encode()
                    op = (d.get("operation") or "").encode()
                    exp = (d.get("expected_value") or "").encode("utf-8", "surrogateescape")
                rules.append(OrcRule(level, self.TYPES[r["type"]], self.services.get(d.get("service_name"), native.OSE_NONE),
                                     len(route), route, int(d.get("threshold", 0)), float(d.get("sampling_ratio", 0.0)),
                                     float(d.get("fallback_sampling_ratio", 0.0)), col, len(exp), cond, op, exp))
        arr = (OrcRule * max(len(rules), 1))(*rules)
        self._keep = arr
        self.h = lib().orc_sampling_create(arr, len(rules))

    def process(self, cols, outs, group_mode: int, seed: int = 0, nthreads: int = 1) -> int:
        rnd = native.Rand(seed, 0.0)
        return lib().orc_sampling_process(self.h, C.byref(cols), C.byref(outs), group_mode, C.byref(rnd), nthreads)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_sampling_free(self.h)


def size_process(cols, res_outs, stages: int, group_mode: int, outs, inverse: int = 1, ratio: float = 1.0,
                 traffic_u: float = 0.0, nthreads: int = 1) -> int:
    """dataSizesMetricsProcessor.processTraces restated (oracle/size.c); res_outs
    holds the earlier stages' results (keep / trace_keep / url_out / tmpl)."""
    return lib().orc_size_process_mt(C.byref(cols), C.byref(res_outs), stages, group_mode, C.byref(outs), inverse,
                                     ratio, traffic_u, nthreads)


def span_template_bytes(refs: np.ndarray, arena: np.ndarray, mask: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Per-span template parity (OSE_STAGE_TEMPLATE_REFS): the bytes each
    masked span's ref {off, len} names, concatenated in span order, and the
    lengths.  Two arenas hold the same templates iff both results match,
    whatever the layout (packed or sparse)."""
    r = refs.reshape(-1, 2)[mask].astype(np.int64)
    lens = r[:, 1]
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, dtype=np.uint8), lens
    starts = np.cumsum(lens) - lens
    idx = np.repeat(r[:, 0] - starts, lens) + np.arange(total, dtype=np.int64)
    assert idx.max() < arena.size, "a template ref points past the arena"
    return arena[idx], lens


def concat_sampling_columns(sources):
    """The sampling columns of the global batch that the split-mode sources
    (node-collector shards, gen_batch.cpp) make concatenated in rank order:
    resources and arena offsets renumbered per source.  Returns (cols, keep
    alive arrays, per-source span offsets)."""
    cat = {}
    for f, dt in (("trace_id", np.uint64), ("start_ns", np.uint64), ("end_ns", np.uint64), ("status", np.uint8),
                  ("route", np.uint32)):
        cat[f] = np.concatenate([g.array(f).view(dt)[: (g.cols.n_spans * (2 if f in ("trace_id", "route") else 1))]
                                 for g in sources])
    roff = np.cumsum([0] + [g.cols.n_resources for g in sources])
    aoff = np.cumsum([0] + [g.cols.arena_bytes for g in sources])
    cat["resource"] = np.concatenate([g.array("resource").view(np.uint32)[: g.cols.n_spans] + np.uint32(roff[k])
                                      for k, g in enumerate(sources)])
    rt = cat["route"].reshape(-1, 2).copy()
    base = np.concatenate([np.full(g.cols.n_spans, aoff[k], np.uint64) for k, g in enumerate(sources)])
    rt[:, 0] = (rt[:, 0].astype(np.uint64) + base * (rt[:, 1] > 0)).astype(np.uint32)
    cat["route"] = rt.reshape(-1)
    cat["arena"] = np.concatenate([g.array("arena")[: g.cols.arena_bytes] for g in sources] + [np.zeros(64, np.uint8)])
    for f in ("res_svc", "res_svc_str"):
        cat[f] = np.concatenate([g.array(f).view(np.uint32)[: g.cols.n_resources] for g in sources])
    W = 1
    if all(getattr(g, "attr_bits", None) is not None for g in sources):   # the shim's span_attribute bits
        # word-major planes: plane w of the global batch is the sources' planes w, concatenated
        planes = [np.asarray(g.attr_bits, np.uint64).reshape(-1, g.cols.n_spans) for g in sources]
        W = planes[0].shape[0]
        cat["attr_match"] = np.concatenate([np.concatenate([p[w] for p in planes]) for w in range(W)])
    assert cat["arena"].size < 2**32
    from odigos_amd import native
    cols = native.Columns()
    cols.n_spans = sum(g.cols.n_spans for g in sources)
    cols.n_resources = int(roff[-1])
    cols.arena_bytes = int(aoff[-1])
    cols.attr_match_words = W
    for f, a in cat.items():
        setattr(cols, f, a.ctypes.data)
    offs = np.cumsum([0] + [g.cols.n_spans for g in sources])
    return cols, cat, offs


def concat_keep_oracle(sources, cfg, seed, threads=16):
    """SAMPLE on the global batch (the sources concatenated in rank order):
    each source's slice of the keep bytes."""
    from odigos_amd import native
    from odigos_amd.batch import HostOutputs
    cols, keepalive, offs = concat_sampling_columns(sources)
    ho = HostOutputs(cols)
    assert SamplingOracle(cfg).process(cols, ho.outs, native.GROUP_TRACE_ID, seed, threads) == 0
    keep = ho.view("keep", np.uint8)[: cols.n_spans]
    del keepalive
    return [keep[offs[k]: offs[k + 1]].copy() for k in range(len(sources))]


def node_parity(gens, dbs, cfg, stages, threads, calls, node_counters=None):
    """The emulated 8-GPU step against the oracle on the GLOBAL batch (the
    sources concatenated in rank order, traces straddling ranks): SAMPLE on the
    concatenation gives every rank's keep slice; TEMPLATE and SIZE run per
    rank on its own spans with that keep (what SIZE | APPLY_KEEP does after
    the exchange); the node's counters are the sums over ranks (what
    ose_allreduce_counters yields)."""
    from odigos_amd.batch import HostOutputs
    keeps = concat_keep_oracle(gens, cfg["odigossampling"], 0x5EED, threads)
    uo = UrlOracle(cfg["odigosurltemplate"]) if stages & native.STAGE_TEMPLATE else None
    res = {"keep": True, "url_out": True, "tmpl_lens": True, "tmpl_bytes_per_span": True}
    node_bytes = node_bytes_gpu = None
    node_acc = node_acc_gpu = 0
    for g, d, kp in zip(gens, dbs, keeps):
        n = g.cols.n_spans
        res["keep"] &= bool(np.array_equal(kp, d.out_numpy("keep", n=n)))
        ho = HostOutputs(g.cols)
        ho.view("keep", np.uint8)[:n] = kp
        if uo:
            assert uo.process(g.cols, ho.outs, threads) == 0
            u = d.out_numpy("url_out", n=n)
            res["url_out"] &= bool(np.array_equal(ho.view("url_out", np.uint8)[:n], u))
            m = u != 0
            gb, gl = span_template_bytes(d.out_numpy("tmpl", np.uint32, n=2 * n), d.out_numpy("tmpl_arena", n=d.used()), m)
            ob, ol = span_template_bytes(ho.view("tmpl", np.uint32)[: 2 * n], ho.bufs["tmpl_arena"][: int(ho.used[0])], m)
            res["tmpl_lens"] &= bool(np.array_equal(gl, ol))
            res["tmpl_bytes_per_span"] &= bool(gb.size == ob.size and np.array_equal(gb, ob))
        if stages & native.STAGE_SIZE:
            assert size_process(g.cols, ho.outs, stages, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, threads) == 0
            A = g.cols.n_attrsets
            ob_ = ho.view("attrset_bytes", np.int64)[:A].copy()
            gb_ = d.out_numpy("attrset_bytes", np.int64, n=A).copy()
            node_bytes = ob_ if node_bytes is None else node_bytes + ob_
            node_bytes_gpu = gb_ if node_bytes_gpu is None else node_bytes_gpu + gb_
            node_acc += int(ho.view("accepted_spans", np.int64)[0])
            node_acc_gpu += int(d.out_numpy("accepted_spans", np.int64, n=1)[0])
    if stages & native.STAGE_SIZE:
        # the device counters were ADDED to by every timed and warm-up call;
        # node_counters: what the counter all-reduce left on a rank
        res["attrset_bytes"] = bool(np.array_equal(calls * node_bytes, node_bytes_gpu))
        res["accepted_spans"] = bool(calls * node_acc == node_acc_gpu)
        if node_counters is not None:
            res["node_allreduce"] = bool(np.array_equal(calls * node_bytes, node_counters[0]) and
                                         calls * node_acc == node_counters[1])
    return res
