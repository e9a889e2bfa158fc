"""numpy restatement of the trace-id exchange (test infrastructure): owner
hash, the partial records and their stable per-owner bucketing, the owner-side
columns ose_shard_unpack writes, and an expansion of records into plain
spans for the oracle (odigos_amd/csrc/trace_kernel.hip shard_* kernels,
include/odigos_amd.h "trace-id exchange"), plus CPU ops for
odigos_amd.exchange.route_and_sample.

A partial record folds a stretch of consecutive spans with one trace id and
one latency slot (the latency service of the span's resource), inside one
64-span step, into: the error bit, the endpoint (HasPrefix) bits, the
service_name / span_attribute rule bits and the latency element (a zero
start seen, the min start after the last zero start, the max end) — the
per-trace state of odigossampling (rule_engine.go:55-115,
internal/sampling/{error,latency,servicename,spanattribute}.go).
"""
from __future__ import annotations

import numpy as np

from odigos_amd import native

NONE24 = 0xFFFFFF
INF = np.uint64(0xFFFFFFFFFFFFFFFF)
XERR, XLAT, XRESET = 1, 2, 4
STEP = 64
# a record of a one-chunk config: the fixed words, then the chunk's endpoint
# and rule words (a K-chunk config appends one (ep, svcb) pair per chunk)
XDT = np.dtype([("hi", "<u8"), ("lo", "<u8"), ("m", "<u8"), ("e", "<u8"), ("w4", "<u8"), ("ep", "<u8"),
                ("svcb", "<u8")])
REC_BYTES = XDT.itemsize   # 56


class RuleLayout:
    """The device rule tables' bit layout (sampling_host.cpp build_sampling_tables):
    interned service ids, latency slot per service, service_name rule bit per
    service, span_attribute bits after the service rules."""

    def __init__(self, cfg: dict):
        from tests.oracle_lib import intern_services
        self.ids = intern_services(cfg)
        self.nsvc = len(self.ids)
        self.slot = {}
        self.svc_bits = np.zeros(max(self.nsvc, 1), dtype=np.uint64)
        self.rule_svc = []            # service id of service_name rule bit k
        self.lat = []                 # (service id, route bytes) per latency rule bit
        self.slot_rules = {}          # slot -> bits of its latency rules
        levels = [cfg.get(k) or [] for k in ("global_rules", "service_rules", "endpoint_rules")]
        n_svc_rules = sum(r["type"] == "service_name" for lv in levels for r in lv)
        for lv in levels:
            for r in lv:
                d = r.get("rule_details") or {}
                if r["type"] == "http_latency":
                    s = self.ids[d["service_name"]]
                    self.slot.setdefault(s, len(self.slot))
                    self.slot_rules[self.slot[s]] = self.slot_rules.get(self.slot[s], 0) | (1 << len(self.lat))
                    self.lat.append((s, d["http_route"].encode()))
                elif r["type"] == "service_name":
                    s = self.ids[d["service_name"]]
                    self.svc_bits[s] |= np.uint64(1 << len(self.rule_svc))
                    self.rule_svc.append(s)
        self.attr_shift = n_svc_rules

    def slot_of(self, svc: np.ndarray) -> np.ndarray:
        out = np.full(len(svc), -1, dtype=np.int64)
        for s, k in self.slot.items():
            out[np.asarray(svc) == s] = k
        return out

    def svc_rule_bits(self, svc_str: np.ndarray) -> np.ndarray:
        s = np.asarray(svc_str, np.int64)
        ok = (s >= 0) & (s < self.nsvc)
        out = np.zeros(len(s), dtype=np.uint64)
        out[ok] = self.svc_bits[s[ok]]
        return out


M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def owners(hi: np.ndarray, lo: np.ndarray, world: int) -> np.ndarray:
    h = _splitmix(hi ^ _splitmix(lo))
    return ((h >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


def endpoint_bits(cfg: dict, res_svc_of_span, route_bytes) -> np.ndarray:
    """bit r = HasPrefix(route, http_route of the r-th latency rule) for the
    rules whose service is the span's service (interned ids)."""
    lay = RuleLayout(cfg)
    out = np.zeros(len(res_svc_of_span), dtype=np.uint64)
    for i, (s, rb) in enumerate(zip(res_svc_of_span, route_bytes)):
        for k, (ls, pre) in enumerate(lay.lat):
            if ls == s and rb.startswith(pre):
                out[i] |= np.uint64(1 << k)
    return out


def pack(tid: np.ndarray, start, end, status, svc, svc_str, ep, world: int, attr=None, *, cfg: dict):
    """-> (records in bucket order [XDT], counts[world] (records), pack_pos[n])"""
    lay = RuleLayout(cfg)
    n = len(start)
    hi, lo = np.asarray(tid[:, 0], np.uint64), np.asarray(tid[:, 1], np.uint64)
    start = np.asarray(start, np.uint64)
    end = np.asarray(end, np.uint64)
    status = np.asarray(status, np.uint8)
    svc = np.asarray(svc, np.int64)
    slot = lay.slot_of(svc)
    svcb = lay.svc_rule_bits(svc_str)
    if attr is not None:
        svcb |= np.asarray(attr, np.uint64) << np.uint64(lay.attr_shift)
    srm = np.array([lay.slot_rules.get(k, 0) for k in range(len(lay.slot))] + [0], dtype=np.uint64)
    ep = np.asarray(ep, np.uint64) & srm[slot]   # slot -1 -> the trailing 0
    idx = np.arange(n)
    head = np.ones(n, dtype=bool)
    if n > 1:
        head[1:] = (hi[1:] != hi[:-1]) | (lo[1:] != lo[:-1]) | (slot[1:] != slot[:-1])
    head |= (idx % STEP) == 0
    starts = np.flatnonzero(head)
    ends = np.append(starts[1:], n)
    recs = np.zeros(len(starts), dtype=XDT)
    for k, (a, b) in enumerate(zip(starts, ends)):
        f, m, e = 0, INF, np.uint64(0)
        if slot[a] >= 0:
            for i in range(a, b):
                if start[i] == 0:
                    f |= 3
                    m = INF
                else:
                    f |= 2
                    m = min(m, start[i])
                e = max(e, end[i])
        flags = (XERR if np.any(status[a:b] == native.STATUS_ERROR) else 0) | (XLAT if f & 2 else 0) | \
            (XRESET if f & 1 else 0)
        recs[k] = (hi[a], lo[a], m, e, (int(svc[a]) if slot[a] >= 0 else NONE24) | (flags << 24),
                   np.bitwise_or.reduce(ep[a:b]), np.bitwise_or.reduce(svcb[a:b]))
    own = owners(recs["hi"], recs["lo"], world)
    order = np.argsort(own, kind="stable")
    slot_of_rec = np.empty(len(starts), dtype=np.int64)
    slot_of_rec[order] = np.arange(len(starts))
    rec_of_span = np.repeat(np.arange(len(starts)), ends - starts)
    return recs[order], np.bincount(own, minlength=world).astype(np.int64), slot_of_rec[rec_of_span]


class HostCols:
    """Owns numpy arrays and an ose_columns view of a sampling batch whose
    resources are one per span (the shape ose_shard_unpack produces)."""

    def __init__(self, tid, start, end, status, svc, svc_str, ep, attr=None, svc_match=None):
        n = len(start)
        c = np.ascontiguousarray   # structured-record fields are strided views
        self.a = dict(trace_id=c(np.asarray(tid, np.uint64).reshape(-1)),
                      start_ns=c(start, np.uint64), end_ns=c(end, np.uint64),
                      status=c(status, np.uint8), resource=np.arange(n, dtype=np.uint32),
                      res_svc=c(svc, np.uint32), res_svc_str=c(svc_str, np.uint32),
                      route_match=c(ep, np.uint64),
                      attr_match=c(np.zeros(n, np.uint64) if attr is None else attr, np.uint64))
        if svc_match is not None:
            self.a["svc_match"] = c(svc_match, np.uint64)
        for k in list(self.a):
            if self.a[k].size == 0:
                self.a[k] = np.zeros(2, dtype=self.a[k].dtype)
        self.cols = native.Columns()
        self.cols.n_spans = n
        self.cols.n_resources = n
        for k, v in self.a.items():
            setattr(self.cols, k, v.ctypes.data)


def unpack(recv: np.ndarray) -> HostCols:
    """The owner-side columns ose_shard_unpack writes (one span per record)."""
    r = recv.view(XDT)
    flags = (r["w4"] >> np.uint64(24)).astype(np.int64) & 0xFF
    sv = (r["w4"] & np.uint64(NONE24)).astype(np.int64)
    lat = (flags & XLAT) != 0
    start = np.where(lat & (r["m"] != INF), r["m"], np.uint64(0))
    end = np.where(lat, r["e"], np.uint64(0))
    status = (np.where(flags & XERR, native.STATUS_ERROR, 0) |
              np.where(lat & ((flags & XRESET) != 0) & (r["m"] != INF), 0x80, 0)).astype(np.uint8)
    svc = np.where(lat & (sv != NONE24), sv, 0xFFFFFFFF).astype(np.uint32)
    tid = np.stack([r["hi"], r["lo"]], axis=1)
    return HostCols(tid, start, end, status, svc, np.full(len(r), 0xFFFFFFFF, np.uint32), r["ep"],
                    svc_match=r["svcb"])


def expand_for_oracle(recv: np.ndarray, cfg: dict):
    """Plain spans the oracle evaluates exactly as the owner folds the records:
    per record a main span (latency service, start = min start, end = max end,
    error status, endpoint bits, span_attribute bits), preceded by a
    zero-start span when a zero start came before the min start, plus one span
    per service_name rule bit carrying that rule's service as a Str
    service.name.  Returns (HostCols, index of each record's main span)."""
    lay = RuleLayout(cfg)
    r = recv.view(XDT)
    cols = {k: [] for k in ("hi", "lo", "start", "end", "status", "svc", "svc_str", "ep", "attr")}
    main = np.zeros(len(r), dtype=np.int64)

    def put(h, l, st, en, stat, s, ss, ep, at):
        for k, v in zip(cols, (h, l, st, en, stat, s, ss, ep, at)):
            cols[k].append(v)

    amask = (1 << 64) - 1
    for k in range(len(r)):
        h, l, m, e, w4, ep, sb = (int(x) for x in r[k])
        flags, sv = (w4 >> 24) & 0xFF, w4 & NONE24
        lat = bool(flags & XLAT)
        s = sv if lat else 0xFFFFFFFF
        if lat and (flags & XRESET) and m != int(INF):
            put(h, l, 0, 0, 1, s, 0xFFFFFFFF, 0, 0)
        st = (0 if m == int(INF) else m) if lat else 0
        main[k] = len(cols["hi"])
        put(h, l, st, e if lat else 0, 2 if flags & XERR else 1, s, 0xFFFFFFFF, ep,
            (sb >> lay.attr_shift) & amask if lay.attr_shift < 64 else 0)
        for b, rs in enumerate(lay.rule_svc):
            if (sb >> b) & 1:
                put(h, l, 0, 0, 1, 0xFFFFFFFF, rs, 0, 0)
    tid = np.stack([np.array(cols["hi"], np.uint64), np.array(cols["lo"], np.uint64)], axis=1) if cols["hi"] else \
        np.zeros((0, 2), np.uint64)
    hc = HostCols(tid, np.array(cols["start"], np.uint64), np.array(cols["end"], np.uint64),
                  np.array(cols["status"], np.uint8), np.array(cols["svc"], np.uint32),
                  np.array(cols["svc_str"], np.uint32), np.array(cols["ep"], np.uint64),
                  np.array(cols["attr"], np.uint64))
    return hc, main


class CpuOps:
    """route_and_sample ops over host tensors (gloo): the numpy pack above and,
    as the owner's SAMPLE stage, the oracle on the expanded records."""

    def __init__(self, batch: HostCols, cfg: dict, seed: int):
        import torch
        self.torch, self.b, self.cfg, self.seed = torch, batch, cfg, seed
        self.rec_bytes = REC_BYTES
        self.device = torch.device("cpu")
        self.keep = np.zeros(batch.cols.n_spans, dtype=np.uint8)
        self.records_sent = 0

    def pack(self, world):
        a = self.b.a
        n = self.b.cols.n_spans
        rec, counts, pos = pack(a["trace_id"][: 2 * n].reshape(-1, 2), a["start_ns"][:n], a["end_ns"][:n],
                                a["status"][:n], a["res_svc"][:n], a["res_svc_str"][:n], a["route_match"][:n], world,
                                a["attr_match"][:n], cfg=self.cfg)
        self.pos = pos
        self.records_sent = len(rec)
        return (self.torch.from_numpy(rec.view(np.uint8).copy()), self.torch.from_numpy(counts), pos)

    def alloc(self, nbytes):
        return self.torch.empty(nbytes, dtype=self.torch.uint8)

    def decide(self, recv, n):
        from odigos_amd.batch import HostOutputs
        from tests.oracle_lib import SamplingOracle
        hc, main = expand_for_oracle(recv.numpy()[: n * REC_BYTES].copy(), self.cfg)
        ho = HostOutputs(hc.cols)
        assert SamplingOracle(self.cfg).process(hc.cols, ho.outs, native.GROUP_TRACE_ID, self.seed, 1) == 0
        keep = ho.view("keep", np.uint8)[main] if n else np.zeros(1, np.uint8)
        return self.torch.from_numpy(np.ascontiguousarray(keep))

    def scatter(self, back, pos):
        self.keep[:] = back.numpy()[pos]


def synthetic_global_batch(world: int, m: int, seed: int, n_svc: int = 16):
    """A global batch of world*m spans whose traces straddle ranks: trace
    ids come from a pool, in short runs, so a trace's spans land on several
    ranks (the loadbalancing-less arrival the exchange exists for)."""
    rng = np.random.default_rng(seed)
    n = world * m
    pool = rng.integers(0, 2**63, size=(max(n // 6, 1), 2), dtype=np.int64).astype(np.uint64)
    runs, tids = [], []
    while sum(runs) < n:
        k = int(rng.integers(1, 8))
        runs.append(k)
        tids.append(pool[rng.integers(0, len(pool))])
    tid = np.repeat(np.array(tids), runs, axis=0)[:n]
    start = (np.uint64(1739000000000000000) + rng.integers(0, 10**9, size=n).astype(np.uint64))
    start[rng.random(n) < 0.01] = 0
    end = start + rng.integers(0, 3 * 10**9, size=n).astype(np.uint64)
    status = np.where(rng.random(n) < 0.03, 2, 1).astype(np.uint8)
    svc = rng.integers(0, n_svc, size=n).astype(np.uint32)
    # runs of one service, so records fold several spans
    svc = np.repeat(svc[::3], 3)[:n]
    svc_str = np.where(rng.random(n) < 0.05, np.uint32(native.OSE_NONE), svc).astype(np.uint32)
    ep = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64)
    return tid, start, end, status, svc, svc_str, ep
