"""Parity of a multi-process (one rank per GPU) bench step against the CPU
oracle (test infrastructure: bench.py's parity leg at --gpus N and the gloo
tests of tests/test_dist_parity.py; never the product path).

Every rank reduces its step's outputs to digests: SHA-256 of its keep and
url_out bytes, of the per-span template lengths and of the template bytes each
span's ref names (span_template_bytes: the same whatever the arena layout),
plus its local traffic counters and the node-summed ones the counter
all-reduce left it.  Rank 0 gathers them (torch.distributed gather_object:
a few hundred bytes per rank), and runs the oracle chain itself:

* split workloads (C4: every source holds some ResourceSpans of a trace,
  gen_batch.cpp split mode): the W sources are regenerated on rank 0 from
  (seed, rank, world), SAMPLE runs on their concatenation in rank order
  (concat_keep_oracle: the decision a single gateway would make on the whole
  node batch, nodecollector/collectorconfig/traces.go:26-84 routing each
  trace's spans to one owner), TEMPLATE and SIZE per source with that keep;
  rank s's digests must equal those of the oracle's slice s, rank s's local
  counters calls x the oracle's counters of source s, and every rank's node
  counters calls x the sum over the sources (odigostrafficmetrics
  processor.go:71-84 summed over the gateway replicas);
* per-GPU workloads (independent batches, no exchange): every rank checks its
  own batch with the oracle (parity_full) and rank 0 ANDs the results.
"""
from __future__ import annotations

import hashlib

import numpy as np

from odigos_amd import native


def _h(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def output_digest(n: int, stages: int, keep=None, url_out=None, tmpl=None, tmpl_arena=None,
                  attrset_bytes=None, accepted_spans=None, node_counters=None) -> dict:
    """One rank's outputs (host numpy arrays) as digests.  tmpl: the 2n u32
    {off, len} refs; node_counters: (attrset bytes, accepted spans) as the
    node-wide all-reduce left them on this rank."""
    from tests.oracle_lib import span_template_bytes
    d = {"n": int(n)}
    if stages & native.STAGE_SAMPLE:
        d["keep"] = _h(np.asarray(keep, np.uint8)[:n])
    if stages & native.STAGE_TEMPLATE:
        u = np.asarray(url_out, np.uint8)[:n]
        d["url_out"] = _h(u)
        gb, gl = span_template_bytes(np.asarray(tmpl, np.uint32)[: 2 * n], np.asarray(tmpl_arena, np.uint8), u != 0)
        d["tmpl_lens"] = _h(gl.astype(np.int64))
        d["tmpl_bytes_per_span"] = _h(gb)
    if stages & native.STAGE_SIZE:
        d["attrset_bytes"] = np.asarray(attrset_bytes, np.int64).tolist()
        d["accepted_spans"] = int(accepted_spans)
        if node_counters is not None:
            d["node"] = (np.asarray(node_counters[0], np.int64).tolist(), int(node_counters[1]))
    return d


def oracle_digests(sources, cfg: dict, stages: int, threads: int, seed: int = 0x5EED) -> list[dict]:
    """The oracle chain over split-mode sources: SAMPLE on the concatenation,
    TEMPLATE and SIZE per source with its keep slice; one digest per source."""
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import UrlOracle, concat_keep_oracle, size_process
    keeps = concat_keep_oracle(sources, cfg["odigossampling"], seed, threads) if stages & native.STAGE_SAMPLE else None
    uo = UrlOracle(cfg["odigosurltemplate"]) if stages & native.STAGE_TEMPLATE else None
    out = []
    for k, g in enumerate(sources):
        n = g.cols.n_spans
        ho = HostOutputs(g.cols)
        if keeps is not None:
            ho.view("keep", np.uint8)[:n] = keeps[k]
        if uo:
            assert uo.process(g.cols, ho.outs, threads) == 0
        if stages & native.STAGE_SIZE:
            assert size_process(g.cols, ho.outs, stages, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, threads) == 0
        A = g.cols.n_attrsets
        used = int(ho.used[0]) if uo else 0
        out.append(output_digest(
            n, stages, keep=ho.view("keep", np.uint8)[:n],
            url_out=ho.view("url_out", np.uint8)[:n] if uo else None,
            tmpl=ho.view("tmpl", np.uint32)[: 2 * n] if uo else None,
            tmpl_arena=ho.bufs["tmpl_arena"][:used] if uo else None,
            attrset_bytes=ho.view("attrset_bytes", np.int64)[:A] if stages & native.STAGE_SIZE else None,
            accepted_spans=int(ho.view("accepted_spans", np.int64)[0]) if stages & native.STAGE_SIZE else None))
        del ho
    return out


def compare_split(got: list[dict], want: list[dict], stages: int, calls: int) -> dict:
    """Rank digests (got[s]) against the oracle's per-source digests."""
    res = {"n": all(g["n"] == w["n"] for g, w in zip(got, want)) and len(got) == len(want)}
    for key in ("keep", "url_out", "tmpl_lens", "tmpl_bytes_per_span"):
        if key in want[0]:
            res[key] = all(g.get(key) == w[key] for g, w in zip(got, want))
    if stages & native.STAGE_SIZE:
        # the device counters were ADDED to by every timed and warm-up call
        res["attrset_bytes"] = all(np.array_equal(np.asarray(g["attrset_bytes"]), calls * np.asarray(w["attrset_bytes"]))
                                   for g, w in zip(got, want))
        res["accepted_spans"] = all(g["accepted_spans"] == calls * w["accepted_spans"] for g, w in zip(got, want))
        node_b = calls * np.sum([np.asarray(w["attrset_bytes"]) for w in want], axis=0)
        node_a = calls * sum(w["accepted_spans"] for w in want)
        res["node_allreduce"] = all("node" in g and np.array_equal(np.asarray(g["node"][0]), node_b)
                                    and g["node"][1] == node_a for g in got)
    return res


def gather_to_rank0(obj, rank: int, world: int):
    import torch.distributed as dist
    objs = [None] * world if rank == 0 else None
    dist.gather_object(obj, objs, dst=0)
    return objs


def split_parity(rank: int, world: int, digest: dict, regen, cfg: dict, stages: int, calls: int, threads: int,
                 own_source=None):
    """Gathers every rank's digest on rank 0 and checks it against the oracle on
    the concatenated sources (regen(s) -> the split-mode Generator of source s;
    own_source: rank 0's own, reused).  Returns the result dict on rank 0,
    None elsewhere."""
    got = gather_to_rank0(digest, rank, world)
    if rank != 0:
        return None
    sources = [own_source if (s == 0 and own_source is not None) else regen(s) for s in range(world)]
    want = oracle_digests(sources, cfg, stages, threads)
    del sources
    return compare_split(got, want, stages, calls)


def local_parity(rank: int, world: int, res: dict):
    """Per-GPU workloads: every rank's own parity_full result, ANDed on rank 0."""
    got = gather_to_rank0({k: bool(v) for k, v in res.items()}, rank, world)
    if rank != 0:
        return None
    keys = sorted(set().union(*[g.keys() for g in got]))
    return {k: all(g.get(k, False) for g in got) for k in keys}
