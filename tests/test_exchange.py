"""Trace-id exchange across GPUs (odigos_amd/exchange.py).

CPU: the partial records (numpy restatement) fold to the same decisions as
the spans they replace (oracle on the expanded records vs oracle on the
spans, zero starts included); the exchange protocol (route_and_sample) on
world_size 2 and 3 over gloo, with the numpy records and the oracle as the
owner's SAMPLE stage: every rank's keep bytes equal the oracle run on the
concatenated global batch, for traces that straddle ranks.
GPU (@gpu): the pack / unpack / scatter kernels against the numpy
restatement (bytes exact); the owner path on one GPU at 2 x 10M spans (two
split-mode sources, both owners, decisions against the oracle on the
global batch); the round over RCCL at world 1 through torch.distributed and
through the C ABI (ose_exchange_sample).
"""
import os
import socket

import numpy as np
import pytest

from odigos_amd import native
from tests.exchange_emul import (REC_BYTES, CpuOps, HostCols, endpoint_bits, expand_for_oracle, owners, pack,
                                 synthetic_global_batch, unpack)
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


def test_record_bytes_abi():
    assert REC_BYTES == native.XREC_BYTES == 56


def test_pack_records_and_positions():
    tid, start, end, status, svc, svc_str, ep = synthetic_global_batch(1, 2000, 5)
    rec, counts, pos = pack(tid, start, end, status, svc, svc_str, ep, 4, cfg=CFG)
    assert counts.sum() == len(rec) < 2000            # records fold several spans
    r = rec.view(np.dtype([("hi", "<u8"), ("lo", "<u8"), ("rest", "V40")]))
    np.testing.assert_array_equal(r["hi"][pos], tid[:, 0])
    np.testing.assert_array_equal(r["lo"][pos], tid[:, 1])
    # buckets are contiguous and keep source order inside a bucket
    own = owners(rec["hi"], rec["lo"], 4)
    assert np.all(np.diff(own) >= 0)
    for d in range(4):
        p = pos[owners(tid[:, 0], tid[:, 1], 4) == d]
        assert np.all(np.diff(p) >= 0)
    # no record crosses a 64-span step
    for k in range(0, 2000, 64):
        if k:
            assert pos[k] != pos[k - 1]


def _oracle_keep(glob, cfg=CFG):
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import SamplingOracle
    hc = HostCols(*glob)
    ho = HostOutputs(hc.cols)
    assert SamplingOracle(cfg).process(hc.cols, ho.outs, native.GROUP_TRACE_ID, SEED, 4) == 0
    return ho.view("keep", np.uint8)[: hc.cols.n_spans].copy()


def _fractional(cfg):
    import copy
    cfg = copy.deepcopy(cfg)
    for k, r in enumerate(cfg["endpoint_rules"]):
        r["rule_details"]["fallback_sampling_ratio"] = 33.3 + k
    return cfg


@pytest.mark.parametrize("seed,world", [(5, 1), (6, 3), (7, 8)])
def test_records_fold_like_spans(seed, world):
    # the owner's fold over the records (expanded for the oracle) decides every
    # trace exactly as the oracle over the original spans (zero starts reset
    # minStart inside and across records; fractional ratios)
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import SamplingOracle
    cfg = _fractional(CFG)
    glob = synthetic_global_batch(1, 6000, seed)
    rec, counts, pos = pack(*glob, world, cfg=cfg)
    hc, main = expand_for_oracle(rec.view(np.uint8), cfg)
    ho = HostOutputs(hc.cols)
    assert SamplingOracle(cfg).process(hc.cols, ho.outs, native.GROUP_TRACE_ID, SEED, 2) == 0
    keep_rec = ho.view("keep", np.uint8)[main]
    np.testing.assert_array_equal(keep_rec[pos], _oracle_keep(glob, cfg))


def test_unpack_columns():
    glob = synthetic_global_batch(1, 3000, 9)
    rec, counts, pos = pack(*glob, 2, cfg=CFG)
    hc = unpack(rec.view(np.uint8))
    a = hc.a
    n = len(rec)
    assert np.all(a["res_svc_str"][:n] == 0xFFFFFFFF)
    assert np.all(a["resource"][:n] == np.arange(n))
    flags = (rec["w4"] >> np.uint64(24)).astype(np.int64)
    lat = (flags & 2) != 0
    np.testing.assert_array_equal(a["end_ns"][:n][~lat], 0)
    np.testing.assert_array_equal(a["svc_match"][:n], rec["svcb"])
    reset_first = lat & ((flags & 4) != 0) & (rec["m"] != np.uint64(2**64 - 1))
    np.testing.assert_array_equal((a["status"][:n] & 0x80) != 0, reset_first)


def _rank_main(rank, world, m, store_file, q):
    import torch.distributed as dist
    from odigos_amd.exchange import route_and_sample
    # a file rendezvous: no port to race for with tests running in parallel
    dist.init_process_group("gloo", init_method="file://" + store_file, rank=rank, world_size=world)
    try:
        glob = synthetic_global_batch(world, m, 11)
        lo, hi = rank * m, (rank + 1) * m
        local = HostCols(*(x[lo:hi] for x in glob))
        ops = CpuOps(local, CFG, SEED)
        route_and_sample(ops, world)
        want = _oracle_keep(glob)[lo:hi]
        q.put((rank, bool(np.array_equal(ops.keep, want)), int((ops.keep != want).sum()), ops.records_sent))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_protocol_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    import tempfile
    store = os.path.join(tempfile.mkdtemp(prefix="ose_gloo_"), "store")
    procs = [ctx.Process(target=_rank_main, args=(r, world, 3000, store, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    # partial records: fewer records than spans cross the exchange
    assert sum(r for _, _, _, r in res) < world * 3000


def test_straddling_traces_exist():
    glob = synthetic_global_batch(2, 3000, 11)
    tid = glob[0]
    a = {(int(h), int(l)) for h, l in tid[:3000]}
    b = {(int(h), int(l)) for h, l in tid[3000:]}
    assert len(a & b) > 50


# ---------------- GPU ----------------

def _shard_vs_emulation(cfg, with_attr, world=3):
    import ctypes as C
    import torch
    from odigos_amd.batch import DeviceBatch, Engine, Generator
    g = Generator("sampling", seed=0x0D160053, n_spans=120_000)
    n = g.cols.n_spans
    attr = None
    if with_attr:
        attr = np.random.default_rng(7).integers(0, 2**62, size=n, dtype=np.int64).astype(np.uint64)
        attr &= np.uint64(1)   # one span_attribute rule: bit 0
        g.cols.attr_match = attr.ctypes.data
    st = g.array("start_ns").view(np.uint64)
    st[np.random.default_rng(8).random(len(st)) < 0.02] = 0   # zero starts: records with a reset
    eng = Engine({"odigossampling": cfg})
    db = DeviceBatch(g.cols)
    L = native.lib()
    rb = L.ose_shard_record_bytes(eng.h)
    assert rb == REC_BYTES
    send = torch.empty(n * rb, dtype=torch.uint8, device="cuda")
    counts = torch.zeros(world, dtype=torch.int64, device="cuda")
    pos = torch.empty(n, dtype=torch.int32, device="cuda")
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
    rec, cnt, p = pack(tid, st[:n], g.array("end_ns").view(np.uint64)[:n], g.array("status")[:n], rsvc[res], rstr[res],
                       ep, world, attr, cfg=cfg)
    R = len(rec)
    np.testing.assert_array_equal(counts.cpu().numpy(), cnt)
    np.testing.assert_array_equal(pos.cpu().numpy(), p)
    np.testing.assert_array_equal(send[: R * rb].cpu().numpy(), rec.view(np.uint8))
    # unpack
    from odigos_amd.exchange import OWNER_COLS
    cols = {k: torch.empty(R * w, dtype=torch.uint8, device="cuda") for k, w in OWNER_COLS}
    native.check(L.ose_shard_unpack(send.data_ptr(), R, rb, *[cols[k].data_ptr() for k, _ in OWNER_COLS], None))
    torch.cuda.synchronize()
    hc = unpack(rec.view(np.uint8))
    for k in cols:
        np.testing.assert_array_equal(cols[k].cpu().numpy(), hc.a[k].view(np.uint8)[: cols[k].numel()])
    return R, n


@pytest.mark.gpu
def test_gpu_shard_kernels_vs_emulation():
    R, n = _shard_vs_emulation(CFG, False)
    assert R < n / 2


@pytest.mark.gpu
def test_gpu_shard_kernels_with_attr_bits():
    # span_attribute rules: their bits ride in the record's rule word
    cfg = dict(CFG)
    cfg["global_rules"] = list(CFG.get("global_rules") or []) + [
        {"name": "attr", "type": "span_attribute",
         "rule_details": {"service_name": "svc-attr", "attribute_key": "env", "condition_type": "string",
                          "operation": "equals", "expected_value": "prod", "sampling_ratio": 50.0}}]
    _shard_vs_emulation(cfg, True, world=8)


def _owner_path(sources, cfg, general=False):
    """The whole exchange on one GPU: pack every source batch for len(sources)
    owners, hand each owner its buckets in source-rank order, decide there
    (ose_shard_decide; general: unpack + SAMPLE), send the keep bytes back
    and scatter them."""
    import ctypes as C
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    from odigos_amd.exchange import DeviceExchange
    W = len(sources)
    eng = Engine({"odigossampling": cfg})
    L = native.lib()
    dbs, packs = [], []
    for g in sources:
        db = DeviceBatch(g.cols)
        n = g.cols.n_spans
        send = torch.empty(max(n, 1) * REC_BYTES, dtype=torch.uint8, device="cuda")
        counts = torch.zeros(W, dtype=torch.int64, device="cuda")
        pos = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
        native.check(L.ose_shard_pack(eng.h, C.byref(db.cols), W, send.data_ptr(), counts.data_ptr(), pos.data_ptr(), None))
        c = counts.cpu().numpy()
        packs.append((send, np.concatenate([[0], np.cumsum(c)]), pos))
        dbs.append(db)
    backs = [torch.empty(max(int(p[1][-1]), 1), dtype=torch.uint8, device="cuda") for p in packs]
    records = 0
    for o in range(W):
        parts = [p[0][p[1][o] * REC_BYTES: p[1][o + 1] * REC_BYTES] for p in packs]
        recv = torch.cat(parts)
        k = recv.numel() // REC_BYTES
        records += k
        ex = DeviceExchange.receiver(eng, REC_BYTES)
        keep_x = ex.unpack_sample(recv, k) if general else ex.decide(recv, k)
        off = 0
        for s, p in enumerate(packs):
            m = int(p[1][o + 1] - p[1][o])
            backs[s][p[1][o]: p[1][o + 1]] = keep_x[off: off + m]
            off += m
    for s, (db, p) in enumerate(zip(dbs, packs)):
        native.check(L.ose_shard_scatter_keep(backs[s].data_ptr(), p[2].data_ptr(), db.cols.n_spans, db.outs.keep, None))
    torch.cuda.synchronize()
    return [db.out_numpy("keep", n=db.cols.n_spans) for db in dbs], records


def _concat_keep_oracle(sources, cfg, threads=16):
    """The oracle on the global batch: the sources concatenated in rank order."""
    from tests.oracle_lib import concat_keep_oracle
    return concat_keep_oracle(sources, cfg, SEED, threads)


@pytest.mark.gpu
def test_gpu_owner_path_2x10M():
    # two split-mode sources of a 20M-span fused batch (the ResourceSpans of a
    # trace land on both): each owner folds the records it receives in source
    # order; every span's decision equals the oracle on the global batch
    from odigos_amd.batch import Generator
    sources = [Generator("fused", seed=0x0D160074, n_spans=20_000_000, threads=16, rank=r, world=2) for r in range(2)]
    assert min(g.cols.n_spans for g in sources) > 9_000_000
    got, records = _owner_path(sources, CFG)
    want = _concat_keep_oracle(sources, CFG)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert records < 0.6 * sum(g.cols.n_spans for g in sources)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [3, 8])
def test_gpu_owner_path_zero_starts(world):
    from odigos_amd.batch import Generator
    cfg = _fractional(CFG)
    sources = [Generator("zipf", seed=0x0D160075 + world, n_spans=400_000, rank=r, world=world) for r in range(world)]
    for k, g in enumerate(sources):
        st = g.array("start_ns").view(np.uint64)
        st[np.random.default_rng(k).random(len(st)) < 0.01] = 0
    got, _ = _owner_path(sources, cfg)
    want = _concat_keep_oracle(sources, cfg)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def _owner_recvs(sources, cfg):
    """Pack every source for len(sources) owners; each owner's received
    records (the source buckets in rank order) and the engine."""
    import ctypes as C
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    W = len(sources)
    eng = Engine({"odigossampling": cfg})
    L = native.lib()
    rb = int(L.ose_shard_record_bytes(eng.h))
    packs = []
    for g in sources:
        db = DeviceBatch(g.cols)
        n = g.cols.n_spans
        send = torch.empty(max(n, 1) * rb, dtype=torch.uint8, device="cuda")
        counts = torch.zeros(W, dtype=torch.int64, device="cuda")
        pos = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
        native.check(L.ose_shard_pack(eng.h, C.byref(db.cols), W, send.data_ptr(), counts.data_ptr(), pos.data_ptr(), None))
        packs.append((send, np.concatenate([[0], np.cumsum(counts.cpu().numpy())])))
    recvs = [torch.cat([p[0][p[1][o] * rb: p[1][o + 1] * rb] for p in packs]) for o in range(W)]
    return eng, recvs, rb


def _decide_both(eng, recv, rb):
    """ose_shard_decide's keep and the general path's on the same records,
    and whether the former fell back to the general path."""
    from odigos_amd.exchange import DeviceExchange
    import torch
    k = recv.numel() // rb
    ex = DeviceExchange.receiver(eng, rb)
    fold = ex.decide(recv, k)[:k].cpu().numpy().copy()
    torch.cuda.synchronize()
    general = bool(native.lib().osehost_owner_last_general(eng.h))
    ref = ex.unpack_sample(recv, k)[:k].cpu().numpy().copy()
    return fold, ref, general


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["fused", "fractional", "zipf", "latency_chunks", "attr100_chunks"])
def test_gpu_owner_decide_vs_general(case):
    # the owner's bucketed fold (ose_shard_decide: records bucketed by trace
    # hash, grouped, ordered and folded in LDS) against the general path
    # (unpack + the SAMPLE stage, itself checked against the oracle by the
    # tests above) on the same received records, byte for byte
    from odigos_amd.batch import Generator
    from tests.test_sampling_chunks import CONFIGS, _attr_bits, _chunks
    from tests.test_sampling_random import inject_zero_starts
    from tests.workloads import wide_attr100_config
    if case in ("fused", "fractional"):
        cfg = CFG if case == "fused" else _fractional(CFG)
        sources = [Generator("fused", seed=0x0D1600D1, n_spans=1_000_000, rank=r, world=4) for r in range(4)]
    elif case == "zipf":
        cfg = _fractional(CFG)
        sources = [Generator("zipf", seed=0x0D1600D2, n_spans=300_000, rank=r, world=3) for r in range(3)]
    else:
        cfg = CONFIGS["latency"]() if case == "latency_chunks" else wide_attr100_config()
        assert _chunks(cfg) >= 2
        sources = [Generator("sampling", seed=0x0D1600D3, n_spans=400_000, rank=r, world=3) for r in range(3)]
        for r, g in enumerate(sources):
            if case == "attr100_chunks":
                g.attr_bits = _attr_bits(g, 100, seed=60 + r, p=0.01)
    for r, g in enumerate(sources):
        inject_zero_starts(g, 0.01, 40 + r)
    eng, recvs, rb = _owner_recvs(sources, cfg)
    paths = []
    for recv in recvs:
        fold, ref, general = _decide_both(eng, recv, rb)
        np.testing.assert_array_equal(fold, ref)
        paths.append(general)
    if case != "zipf":
        assert not any(paths), paths   # these batches stay on the fold


@pytest.mark.gpu
def test_gpu_owner_decide_overflow_falls_back():
    # a trace received as 600 pieces overflows its bucket (512 records): the
    # whole batch takes the general path, with the same decisions
    import torch
    from odigos_amd.batch import Generator
    sources = [Generator("fused", seed=0x0D1600D4, n_spans=200_000, rank=r, world=2) for r in range(2)]
    eng, recvs, rb = _owner_recvs(sources, CFG)
    recv = recvs[0]
    one = recv[:rb]
    big = torch.cat([recv[: 100 * rb], one.repeat(600), recv[100 * rb:]])
    fold, ref, general = _decide_both(eng, big, rb)
    assert general
    np.testing.assert_array_equal(fold, ref)
    fold, ref, general = _decide_both(eng, recv, rb)
    assert not general
    np.testing.assert_array_equal(fold, ref)


@pytest.mark.gpu
def test_gpu_exchange_round_world1():
    # the full round on one GPU over RCCL: through torch.distributed
    # (route_and_sample) and through the C ABI (ose_exchange_sample)
    import torch
    import torch.distributed as dist
    from odigos_amd.batch import DeviceBatch, Engine, Generator, HostOutputs
    from odigos_amd.exchange import DeviceExchange, NcclComm, NcclExchange, route_and_sample
    from tests.oracle_lib import SamplingOracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        g = Generator("fused", seed=0x0D160064, n_spans=200_000, shuffle=True)
        eng = Engine({"odigossampling": CFG})
        ho = HostOutputs(g.cols)
        assert SamplingOracle(CFG).process(g.cols, ho.outs, native.GROUP_TRACE_ID, 0x5EED, 8) == 0
        n = g.cols.n_spans
        db = DeviceBatch(g.cols)
        ex = DeviceExchange(eng, db, stream=torch.cuda.current_stream().cuda_stream)
        route_and_sample(ex, 1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(db.out_numpy("keep")[:n], ho.view("keep", np.uint8)[:n])
        db2 = DeviceBatch(g.cols)
        comm = NcclComm(0, 1)
        nx = NcclExchange(eng, db2, comm, stream=torch.cuda.current_stream().cuda_stream)
        nx.round()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(db2.out_numpy("keep")[:n], ho.view("keep", np.uint8)[:n])
        assert nx.stats[2] == n and 0 < nx.stats[0] == nx.stats[1] < n
        # node counters: all-reduce of a local vector over one rank is the identity
        loc = torch.arange(1, 9, dtype=torch.int64, device="cuda")
        node = torch.zeros(8, dtype=torch.int64, device="cuda")
        nx.allreduce_counters(loc.data_ptr(), node.data_ptr(), 8)
        torch.cuda.synchronize()
        assert node.tolist() == list(range(1, 9))
        comm.close()
    finally:
        dist.destroy_process_group()


def _local_round(sources, cfg, rounds=1, stream_per_rank=True):
    """ose_exchange_sample's round (exchange_round) at world len(sources) on
    ONE GPU: one engine, stream and host thread per rank, the in-process
    transport (osehost_xgroup_*) moving the bytes with device copies where
    RCCL would send them over xGMI.  Returns each rank's keep bytes and
    round stats."""
    import ctypes as C
    import threading
    import torch
    from odigos_amd.batch import DeviceBatch, Engine
    L = native.lib()
    W = len(sources)
    grp = C.c_void_p()
    native.check(L.osehost_xgroup_create(W, C.byref(grp)))
    engs = [Engine({"odigossampling": cfg}) for _ in range(W)]
    dbs = [DeviceBatch(g.cols) for g in sources]
    streams = [torch.cuda.Stream() if stream_per_rank else torch.cuda.current_stream() for _ in range(W)]
    stats = [(C.c_uint64 * 3)() for _ in range(W)]
    errs = [None] * W
    torch.cuda.synchronize()

    def rank_main(r):
        try:
            rnd = native.Rand(SEED, 0.0)
            for _ in range(rounds):
                rc = L.osehost_exchange_sample_local(engs[r].h, C.byref(dbs[r].cols), C.byref(dbs[r].outs), grp, r,
                                                     C.byref(rnd), C.c_void_p(streams[r].cuda_stream), stats[r])
                if rc:
                    errs[r] = (rc, native.last_error() if hasattr(native, "last_error") else "")
                    return
        except Exception as ex:   # pragma: no cover
            errs[r] = repr(ex)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    torch.cuda.synchronize()
    L.osehost_xgroup_destroy(grp)
    assert all(e is None for e in errs), errs
    keeps = [db.out_numpy("keep", n=db.cols.n_spans).copy() for db in dbs]
    for e in engs:
        e.close()
    return keeps, [list(s) for s in stats]


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_total", [(2, 600_000), (3, 900_000), (8, 2_400_000)])
def test_gpu_exchange_round_local_world(world, n_total):
    # the product round (bucket offsets, the grouped all-to-all of counts and
    # records, owner unpack + SAMPLE, the reverse split, the scatter) at
    # world > 1, on split-mode C4 sources whose traces straddle ranks; every
    # rank's keep equals the oracle on the concatenated global batch
    from odigos_amd.batch import Generator
    sources = [Generator("fused", seed=0x0D1600B0 + world, n_spans=n_total, threads=8, rank=r, world=world)
               for r in range(world)]
    got, stats = _local_round(sources, CFG, rounds=2)
    want = _concat_keep_oracle(sources, CFG)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    sent = sum(s[0] for s in stats)
    recv = sum(s[1] for s in stats)
    assert sent == recv and 0 < sent < sum(g.cols.n_spans for g in sources)
    assert [s[2] for s in stats] == [g.cols.n_spans for g in sources]


@pytest.mark.gpu
def test_gpu_exchange_round_local_zipf_zero_starts():
    # Zipf trace sizes (long traces straddle every rank), zero starts and
    # fractional ratios through the same round at world 3, all ranks on one stream
    from odigos_amd.batch import Generator
    cfg = _fractional(CFG)
    sources = [Generator("zipf", seed=0x0D1600B9, n_spans=600_000, rank=r, world=3) for r in range(3)]
    for k, g in enumerate(sources):
        st = g.array("start_ns").view(np.uint64)
        st[np.random.default_rng(40 + k).random(len(st)) < 0.01] = 0
    got, _ = _local_round(sources, cfg, stream_per_rank=True)
    want = _concat_keep_oracle(sources, cfg)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.gpu
def test_gpu_exchange_round_local_empty_rank():
    # a rank with no spans still takes part in every collective
    from odigos_amd.batch import Generator
    sources = [Generator("fused", seed=0x0D1600BA, n_spans=200_000, rank=r, world=2) for r in range(2)]
    sources.append(Generator("fused", seed=0x0D1600BB, n_spans=0))
    got, stats = _local_round(sources, CFG)
    want = _concat_keep_oracle(sources, CFG)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert stats[2][0] == 0 and stats[2][2] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_total,one_stream", [(8, 2_400_000, False), (3, 900_000, True)])
def test_gpu_node_step_full(world, n_total, one_stream):
    # the whole N-GPU C4 step at world > 1 (tests/node_emul.py, what
    # bench.py runs per rank): TEMPLATE on the side stream, the exchange
    # round, SIZE | APPLY_KEEP on the decisions and the counter all-reduce,
    # two steps; every rank's keep, url_out and template bytes and the node's
    # counters against the oracle on the concatenated global batch
    import torch
    from odigos_amd.batch import Generator
    from tests.node_emul import LocalNode
    from tests.oracle_lib import node_parity
    from tests.workloads import c3_sampling_config
    keys = ["k8s.namespace.name", "k8s.deployment.name", "service.name"]
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": keys}}
    gens = [Generator("fused", seed=0x0D1600C0 + world, n_spans=n_total, threads=8, rank=r, world=world)
            for r in range(world)]
    for g in gens:
        g.cols.res_url_ok = None
    tform = native.STAGE_TEMPLATE_REFS
    node = LocalNode(cfg, gens, tmpl_form=tform, one_stream=torch.cuda.current_stream() if one_stream else None,
                     seed=0x5EED)
    try:
        for _ in range(2):
            node.step()
        torch.cuda.synchronize()
        stages = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | tform | native.STAGE_SIZE
        par = node_parity(gens, node.dbs, cfg, stages, 8, 2, node.node_counters())
        assert all(par.values()), par
        for d in node.dbs:
            assert int(d.out_numpy("device_status", np.uint32)[0]) == 0
    finally:
        node.close()
