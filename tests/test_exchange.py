"""Trace-id exchange across GPUs (odigos_amd/exchange.py).

CPU: the exchange protocol (route_and_sample) on world_size 2 and 3 over
gloo, with the numpy record emulation and the oracle as the SAMPLE stage:
every rank's keep bytes equal the oracle run on the concatenated global
batch, for traces that straddle ranks.
GPU (@gpu): the pack / unpack / scatter kernels against the numpy
emulation, and the full round on one GPU over RCCL (world 1).
"""
import os
import socket

import numpy as np
import pytest

from odigos_amd import native
from tests.exchange_emul import CpuOps, HostCols, endpoint_bits, owners, pack, rec_bytes, synthetic_global_batch, unpack
from tests.workloads import c3_sampling_config

CFG = c3_sampling_config()
SEED = 0x5EED


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_owner_hash_matches_abi():
    L = native.lib()
    rng = np.random.default_rng(3)
    tid = rng.integers(0, 2**63, size=(500, 2), dtype=np.int64).astype(np.uint64)
    for world in (1, 2, 3, 8):
        got = owners(tid[:, 0], tid[:, 1], world)
        want = [L.ose_shard_owner(int(h), int(l), world) for h, l in tid]
        assert list(got) == want


def test_pack_unpack_roundtrip():
    tid, start, end, status, svc, svc_str, ep = synthetic_global_batch(1, 2000, 5)
    rec, counts, pos = pack(tid, start, end, status, svc, svc_str, ep, 4, cfg=CFG)
    assert counts.sum() == 2000
    assert rec.itemsize == rec_bytes(CFG) == 48
    hc = unpack(rec.view(np.uint8), CFG)
    a = hc.a
    np.testing.assert_array_equal(a["start_ns"][pos], start)
    np.testing.assert_array_equal(a["trace_id"].reshape(-1, 2)[pos], tid)
    # buckets are contiguous and in batch order inside a bucket
    own = owners(tid[:, 0], tid[:, 1], 4)
    for d in range(4):
        p = pos[own == d]
        assert np.all(np.diff(p) == 1)


def _oracle_keep(glob):
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import SamplingOracle
    hc = HostCols(*glob)
    ho = HostOutputs(hc.cols)
    assert SamplingOracle(CFG).process(hc.cols, ho.outs, native.GROUP_TRACE_ID, SEED, 4) == 0
    return ho.view("keep", np.uint8)[: hc.cols.n_spans].copy()


def _rank_main(rank, world, m, port, q):
    import torch.distributed as dist
    from odigos_amd.exchange import route_and_sample
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        glob = synthetic_global_batch(world, m, 11)
        lo, hi = rank * m, (rank + 1) * m
        local = HostCols(*(x[lo:hi] for x in glob))
        ops = CpuOps(local, CFG, SEED)
        route_and_sample(ops, world)
        want = _oracle_keep(glob)[lo:hi]
        q.put((rank, bool(np.array_equal(ops.keep, want)), int((ops.keep != want).sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_protocol_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, 3000, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_straddling_traces_exist():
    glob = synthetic_global_batch(2, 3000, 11)
    tid = glob[0]
    a = {(int(h), int(l)) for h, l in tid[:3000]}
    b = {(int(h), int(l)) for h, l in tid[3000:]}
    assert len(a & b) > 50


# ---------------- GPU ----------------

def _shard_vs_emulation(cfg, with_attr):
    import ctypes as C
    import torch
    from odigos_amd.batch import DeviceBatch, Engine, Generator
    g = Generator("sampling", seed=0x0D160053, n_spans=120_000)
    n = g.cols.n_spans
    attr = None
    if with_attr:
        attr = np.random.default_rng(7).integers(0, 2**62, size=n, dtype=np.int64).astype(np.uint64)
        g.cols.attr_match = attr.ctypes.data
    eng = Engine({"odigossampling": cfg})
    db = DeviceBatch(g.cols)
    world = 3
    rb = native.lib().ose_shard_record_bytes(eng.h)
    assert rb == rec_bytes(cfg) == (56 if with_attr else 48)
    send = torch.empty(n * rb, dtype=torch.uint8, device="cuda")
    counts = torch.zeros(world, dtype=torch.int64, device="cuda")
    pos = torch.empty(n, dtype=torch.int32, device="cuda")
    L = native.lib()
    native.check(L.ose_shard_pack(eng.h, C.byref(db.cols), world, send.data_ptr(), counts.data_ptr(), pos.data_ptr(), None))
    torch.cuda.synchronize()
    tid = g.array("trace_id").view(np.uint64).reshape(-1, 2)[:n]
    res = g.array("resource").view(np.uint32)[:n]
    rsvc = g.array("res_svc").view(np.uint32)
    rstr = g.array("res_svc_str").view(np.uint32)
    route = g.array("route").view(np.uint32).reshape(-1, 2)[:n]
    arena = g.array("arena")
    rb_ = [bytes(arena[o:o + ln]) for o, ln in route]
    ep = endpoint_bits(cfg, rsvc[res], rb_)
    rec, cnt, p = pack(tid, g.array("start_ns").view(np.uint64)[:n], g.array("end_ns").view(np.uint64)[:n],
                       g.array("status")[:n], rsvc[res], rstr[res], ep, world, attr, cfg=cfg)
    np.testing.assert_array_equal(counts.cpu().numpy(), cnt)
    np.testing.assert_array_equal(pos.cpu().numpy(), p)
    np.testing.assert_array_equal(send.cpu().numpy(), rec.view(np.uint8))
    # unpack
    cols = {k: torch.empty(n * w, dtype=torch.uint8, device="cuda") for k, w in
            (("trace_id", 16), ("start_ns", 8), ("end_ns", 8), ("status", 1), ("resource", 4), ("res_svc", 4),
             ("res_svc_str", 4), ("route_match", 8), ("attr_match", 8))}
    native.check(L.ose_shard_unpack(send.data_ptr(), n, rb, *[cols[k].data_ptr() for k in
                                    ("trace_id", "start_ns", "end_ns", "status", "resource", "res_svc", "res_svc_str",
                                     "route_match", "attr_match")], None))
    torch.cuda.synchronize()
    hc = unpack(rec.view(np.uint8), cfg)
    for k in cols:
        np.testing.assert_array_equal(cols[k].cpu().numpy(), hc.a[k].view(np.uint8)[: cols[k].numel()])


@pytest.mark.gpu
def test_gpu_shard_kernels_vs_emulation():
    _shard_vs_emulation(CFG, False)


@pytest.mark.gpu
def test_gpu_shard_kernels_with_attr_bits():
    # span_attribute rules: 56-byte records carry the attr_match bits
    cfg = dict(CFG)
    cfg["global_rules"] = list(CFG.get("global_rules") or []) + [
        {"name": "attr", "type": "span_attribute",
         "rule_details": {"service_name": "svc-attr", "attribute_key": "env", "condition_type": "string",
                          "operation": "equals", "expected_value": "prod", "sampling_ratio": 50.0}}]
    _shard_vs_emulation(cfg, True)


@pytest.mark.gpu
def test_gpu_exchange_round_world1():
    # the full round on one GPU over RCCL: keep equals the direct SAMPLE stage
    import torch
    import torch.distributed as dist
    from odigos_amd.batch import DeviceBatch, Engine, Generator, HostOutputs
    from odigos_amd.exchange import DeviceExchange, route_and_sample
    from tests.oracle_lib import SamplingOracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        g = Generator("fused", seed=0x0D160064, n_spans=200_000, shuffle=True)
        eng = Engine({"odigossampling": CFG})
        db = DeviceBatch(g.cols)
        ex = DeviceExchange(eng, db, stream=torch.cuda.current_stream().cuda_stream)
        route_and_sample(ex, 1)
        torch.cuda.synchronize()
        ho = HostOutputs(g.cols)
        assert SamplingOracle(CFG).process(g.cols, ho.outs, native.GROUP_TRACE_ID, ex.seed, 8) == 0
        n = g.cols.n_spans
        np.testing.assert_array_equal(db.out_numpy("keep")[:n], ho.view("keep", np.uint8)[:n])
    finally:
        dist.destroy_process_group()
