"""numpy restatement of the trace-id exchange records (test infrastructure):
owner hash, stable per-owner bucketing, the 48/56-byte record and its unpacking
(odigos_amd/csrc/trace_kernel.hip shard_* kernels, include/odigos_amd.h
ose_shard_*), plus CPU ops for odigos_amd.exchange.route_and_sample."""
from __future__ import annotations

import ctypes as C

import numpy as np

from odigos_amd import native

NONE24 = 0xFFFFFF   # service ids no rule names travel as 24-bit NONE


def rec_layout(cfg: dict):
    """(interned service count, records carry attr_match) for a sampling config."""
    from tests.oracle_lib import intern_services
    with_attr = any(r.get("type") == "span_attribute"
                    for lvl in ("global_rules", "service_rules", "endpoint_rules") for r in cfg.get(lvl) or [])
    return len(intern_services(cfg)), with_attr


def xdt(with_attr: bool) -> np.dtype:
    f = [("hi", "<u8"), ("lo", "<u8"), ("start", "<u8"), ("end", "<u8"), ("ep", "<u8"), ("sv", "<u8")]
    return np.dtype(f + ([("attr", "<u8")] if with_attr else []))


def rec_bytes(cfg: dict) -> int:
    return xdt(rec_layout(cfg)[1]).itemsize

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
    from tests.oracle_lib import intern_services
    ids = intern_services(cfg)
    lat = []
    for lvl in ("global_rules", "service_rules", "endpoint_rules"):
        for r in cfg.get(lvl) or []:
            if r["type"] == "http_latency":
                d = r["rule_details"]
                lat.append((ids[d["service_name"]], d["http_route"].encode()))
    out = np.zeros(len(res_svc_of_span), dtype=np.uint64)
    for i, (s, rb) in enumerate(zip(res_svc_of_span, route_bytes)):
        for k, (ls, pre) in enumerate(lat):
            if ls == s and rb.startswith(pre):
                out[i] |= np.uint64(1 << k)
    return out


def pack(tid: np.ndarray, start, end, status, svc, svc_str, ep, world: int, attr=None, *, cfg: dict):
    """-> (records in bucket order, counts[world], pack_pos[n])"""
    nsvc, with_attr = rec_layout(cfg)
    hi, lo = tid[:, 0], tid[:, 1]
    own = owners(hi, lo, world)
    order = np.argsort(own, kind="stable")
    rec = np.zeros(len(hi), dtype=xdt(with_attr))
    rec["hi"], rec["lo"], rec["start"], rec["end"], rec["ep"] = hi, lo, start, end, ep
    s = np.where(np.asarray(svc, np.uint64) < nsvc, np.asarray(svc, np.uint64), NONE24)
    ss = np.where(np.asarray(svc_str, np.uint64) < nsvc, np.asarray(svc_str, np.uint64), NONE24)
    rec["sv"] = (s | (ss << np.uint64(24)) | (np.asarray(status, np.uint64) << np.uint64(48))).astype(np.uint64)
    if with_attr:
        rec["attr"] = 0 if attr is None else attr
    pos = np.empty(len(hi), dtype=np.int64)
    pos[order] = np.arange(len(hi))
    return rec[order], np.bincount(own, minlength=world).astype(np.int64), pos


class HostCols:
    """Owns numpy arrays and an ose_columns view of a sampling batch whose
    resources are one per span (the shape ose_shard_unpack produces)."""

    def __init__(self, tid, start, end, status, svc, svc_str, ep, attr=None):
        n = len(start)
        c = np.ascontiguousarray   # structured-record fields are strided views
        self.a = dict(trace_id=c(np.asarray(tid, np.uint64).reshape(-1)),
                      start_ns=c(start, np.uint64), end_ns=c(end, np.uint64),
                      status=c(status, np.uint8), resource=np.arange(n, dtype=np.uint32),
                      res_svc=c(svc, np.uint32), res_svc_str=c(svc_str, np.uint32),
                      route_match=c(ep, np.uint64),
                      attr_match=c(np.zeros(n, np.uint64) if attr is None else attr, np.uint64))
        for k in list(self.a):
            if self.a[k].size == 0:
                self.a[k] = np.zeros(2, dtype=self.a[k].dtype)
        self.cols = native.Columns()
        self.cols.n_spans = n
        self.cols.n_resources = n
        for k, v in self.a.items():
            setattr(self.cols, k, v.ctypes.data)


def unpack(recv: np.ndarray, cfg: dict) -> HostCols:
    nsvc, with_attr = rec_layout(cfg)
    r = recv.view(xdt(with_attr))
    tid = np.stack([r["hi"], r["lo"]], axis=1)
    sv = r["sv"]
    s = (sv & np.uint64(NONE24)).astype(np.uint32)
    ss = ((sv >> np.uint64(24)) & np.uint64(NONE24)).astype(np.uint32)
    s[s == NONE24] = 0xFFFFFFFF
    ss[ss == NONE24] = 0xFFFFFFFF
    status = (sv >> np.uint64(48)).astype(np.uint8)
    return HostCols(tid, r["start"], r["end"], status, s, ss, r["ep"], r["attr"] if with_attr else None)


class CpuOps:
    """route_and_sample ops over host tensors (gloo) with the oracle as the
    SAMPLE stage."""

    def __init__(self, batch: HostCols, cfg: dict, seed: int):
        import torch
        self.torch, self.b, self.cfg, self.seed = torch, batch, cfg, seed
        self.rec_bytes = rec_bytes(cfg)
        self.device = torch.device("cpu")
        self.keep = np.zeros(batch.cols.n_spans, dtype=np.uint8)

    def pack(self, world):
        a = self.b.a
        n = self.b.cols.n_spans
        rec, counts, pos = pack(a["trace_id"][: 2 * n].reshape(-1, 2), a["start_ns"][:n], a["end_ns"][:n],
                                a["status"][:n], a["res_svc"][:n], a["res_svc_str"][:n], a["route_match"][:n], world,
                                a["attr_match"][:n], cfg=self.cfg)
        self.pos = pos
        return (self.torch.from_numpy(rec.view(np.uint8).copy()), self.torch.from_numpy(counts), pos)

    def alloc(self, nbytes):
        return self.torch.empty(nbytes, dtype=self.torch.uint8)

    def unpack_sample(self, recv, n):
        from odigos_amd.batch import HostOutputs
        from tests.oracle_lib import SamplingOracle
        hc = unpack(recv.numpy()[: n * self.rec_bytes].copy(), self.cfg)
        ho = HostOutputs(hc.cols)
        assert SamplingOracle(self.cfg).process(hc.cols, ho.outs, native.GROUP_TRACE_ID, self.seed, 1) == 0
        return self.torch.from_numpy(ho.view("keep", np.uint8)[:max(n, 1)].copy())

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
    svc_str = np.where(rng.random(n) < 0.05, np.uint32(native.OSE_NONE), svc).astype(np.uint32)
    ep = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64)
    return tid, start, end, status, svc, svc_str, ep
