"""bench.py's parity leg at --gpus N (tests/dist_parity.py) on the CPU: world
size 2 and 3 over gloo.  Each rank holds its split-mode C4 source (traces
straddle ranks, gen_batch.cpp), decides it through the numpy restatement of
the trace-id exchange (tests/exchange_emul.py: partial records routed to each
trace's owner, folded there, keep bytes sent back), templates and sizes it with
the oracle, all-reduces the traffic counters, and hands its digests to the
same gather-and-check bench.py runs after a multi-GPU step.  Rank 0 must find
every field equal to the oracle on the concatenated global batch; a single
flipped keep byte on one rank, or a wrong node counter, must fail the check."""
import os
import tempfile

import numpy as np
import pytest

from odigos_amd import native

SEED = 0x5EED
CALLS = 3   # the device counters are added to by every call (warm-up + timed)


def _emulated_rank_outputs(g, cfg, world, stages):
    """What one rank's step leaves on its GPU, restated on the CPU: keep from
    the exchange emulation, TEMPLATE and SIZE by the oracle with that keep."""
    from odigos_amd.batch import HostOutputs
    from odigos_amd.exchange import route_and_sample
    from tests.exchange_emul import CpuOps, HostCols, endpoint_bits
    from tests.oracle_lib import UrlOracle, size_process
    n = g.cols.n_spans
    scfg = cfg["odigossampling"]
    res = g.array("resource").view(np.uint32)[:n]
    rsvc = g.array("res_svc").view(np.uint32)
    rstr = g.array("res_svc_str").view(np.uint32)
    route = g.array("route").view(np.uint32).reshape(-1, 2)[:n]
    arena = g.array("arena")
    ep = endpoint_bits(scfg, rsvc[res], [bytes(arena[o:o + ln]) for o, ln in route])
    hc = HostCols(g.array("trace_id").view(np.uint64).reshape(-1, 2)[:n].copy(),
                  g.array("start_ns").view(np.uint64)[:n].copy(), g.array("end_ns").view(np.uint64)[:n].copy(),
                  g.array("status")[:n].copy(), rsvc[res].copy(), rstr[res].copy(), ep)
    ops = CpuOps(hc, scfg, SEED)
    route_and_sample(ops, world)
    ho = HostOutputs(g.cols)
    ho.view("keep", np.uint8)[:n] = ops.keep
    assert UrlOracle(cfg["odigosurltemplate"]).process(g.cols, ho.outs, 2) == 0
    assert size_process(g.cols, ho.outs, stages, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, 2) == 0
    return ho


def _rank_main(rank, world, n_total, store_file, q):
    import torch
    import torch.distributed as dist

    import bench
    from odigos_amd.batch import Generator
    from tests import dist_parity
    dist.init_process_group("gloo", init_method="file://" + store_file, rank=rank, world_size=world)
    try:
        wl = bench.WORKLOADS["fused"]
        cfg = bench._cfg(wl)
        stages = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE

        def regen(s):
            g = Generator("fused", seed=wl["seed"], n_spans=n_total, threads=2, rank=s, world=world)
            g.cols.res_url_ok = None
            return g
        g = regen(rank)
        n = g.cols.n_spans
        A = g.cols.n_attrsets
        ho = _emulated_rank_outputs(g, cfg, world, stages)
        local = np.concatenate([CALLS * ho.view("attrset_bytes", np.int64)[:A],
                                [CALLS * int(ho.view("accepted_spans", np.int64)[0])]])
        node = torch.from_numpy(local.copy())
        dist.all_reduce(node)   # ose_allreduce_counters
        node = node.numpy()
        used = int(ho.used[0])

        def digest(keep, node_ctr):
            return dist_parity.output_digest(
                n, stages, keep=keep, url_out=ho.view("url_out", np.uint8)[:n], tmpl=ho.view("tmpl", np.uint32)[: 2 * n],
                tmpl_arena=ho.bufs["tmpl_arena"][:used], attrset_bytes=local[:A], accepted_spans=int(local[A]),
                node_counters=(node_ctr[:A], int(node_ctr[A])))
        keep = ho.view("keep", np.uint8)[:n].copy()
        good = dist_parity.split_parity(rank, world, digest(keep, node), regen, cfg, stages, CALLS, 2, own_source=g)
        bad_keep = keep.copy()
        if rank == world - 1:
            bad_keep[n // 2] ^= 1
        bad = dist_parity.split_parity(rank, world, digest(bad_keep, node), regen, cfg, stages, CALLS, 2)
        bad_node = node.copy()
        if rank == 0:
            bad_node[0] += 1
        bad2 = dist_parity.split_parity(rank, world, digest(keep, bad_node), regen, cfg, stages, CALLS, 2)
        loc = dist_parity.local_parity(rank, world, {"keep": True, "url_out": rank != 1})
        q.put((rank, good, bad, bad2, loc, n))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_parity_leg_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = os.path.join(tempfile.mkdtemp(prefix="ose_gloo_"), "store")
    procs = [ctx.Process(target=_rank_main, args=(r, world, 30_000, store, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    _, good, bad, bad2, loc, _ = res[0]
    assert all(r[1] is None for r in res[1:])          # only rank 0 holds the verdict
    assert sum(r[5] for r in res) == 30_000            # the sources partition the global batch
    assert good and all(good.values()), good
    assert set(good) >= {"keep", "url_out", "tmpl_lens", "tmpl_bytes_per_span", "attrset_bytes",
                         "accepted_spans", "node_allreduce"}
    assert not bad["keep"] and bad["url_out"] and bad["node_allreduce"], bad
    assert bad2["keep"] and not bad2["node_allreduce"], bad2
    assert loc == {"keep": True, "url_out": False}
