"""Trace-id exchange across the GPUs of one node.

odigossampling needs every span of a trace on one GPU.  In the reference
that co-location is the node collector's loadbalancing exporter keyed by
trace id (autoscaler/controllers/nodecollector/collectorconfig/
traces.go:26-84).  Here, per step:

1. ``ose_shard_pack`` folds the batch into partial records (one per stretch
   of spans with one trace id and one latency service, 56 bytes: the error,
   endpoint and rule bits and the latency monoid element of the stretch) and
   buckets them by owner = hash(trace id) mod world, keeping source order;
2. an all-to-all of the record counts, then of the records (RCCL over xGMI);
3. ``ose_shard_decide`` on the received records: bucketed by trace-id hash,
   each bucket's traces grouped and folded in LDS in (source rank, source
   order) = global batch order (``ose_shard_unpack`` + the SAMPLE stage is
   the general path it falls back to, and stays callable);
4. the reverse all-to-all of the keep bytes and ``ose_shard_scatter_keep``.

Two drivers of the same round:
* ``NcclExchange`` — the product path: one C-ABI call per round
  (``ose_exchange_sample``) on an RCCL communicator the engine library
  creates (``ose_nccl_comm_init``; the 128-byte unique id travels over
  torch.distributed once), exactly what a cgo shim would call;
* ``route_and_sample`` — the protocol written against a small ops object
  over torch.distributed collectives, so the same code runs on the device ops
  below and, in tests, on CPU ops over gloo.
"""
from __future__ import annotations

import ctypes as C

from . import native


def route_and_sample(ops, world: int, group=None) -> None:
    """One exchange round; ops provides pack/alloc/decide/scatter."""
    import torch
    import torch.distributed as dist
    XREC = ops.rec_bytes                                # bytes per exchanged record
    send, counts, pos = ops.pack(world)                 # counts: int64 tensor [world] on ops.device
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    sc = [int(x) for x in counts.tolist()]              # host sync: split sizes
    rc = [int(x) for x in recv_counts.tolist()]
    n_send, n_recv = sum(sc), sum(rc)
    recv = ops.alloc(n_recv * XREC)
    dist.all_to_all_single(recv, send[: n_send * XREC], [c * XREC for c in rc], [c * XREC for c in sc], group=group)
    keep_x = ops.decide(recv, n_recv)                   # uint8 [n_recv]
    back = ops.alloc(n_send)
    dist.all_to_all_single(back, keep_x[:n_recv], sc, rc, group=group)
    ops.scatter(back, pos)


OWNER_COLS = (("trace_id", 16), ("start_ns", 8), ("end_ns", 8), ("status", 1), ("resource", 4), ("res_svc", 4),
              ("res_svc_str", 4), ("route_match", 8), ("svc_match", 8))


class DeviceExchange:
    """Device ops for route_and_sample over one HBM-resident batch."""

    seed = 0x5EED

    def __init__(self, engine, db, stream=None):
        import torch
        self.torch = torch
        self.eng, self.db = engine, db
        self.L = native.lib()
        self.stream = stream
        self.device = torch.device("cuda", torch.cuda.current_device())
        n = db.cols.n_spans
        self.n = n
        self.rec_bytes = int(self.L.ose_shard_record_bytes(engine.h))
        if not self.rec_bytes:
            raise RuntimeError("the trace-id exchange needs odigossampling on the engine")
        self.send = torch.empty(max(n, 1) * self.rec_bytes, dtype=torch.uint8, device=self.device)
        self.pos = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        self.counts = None
        self._recv_cap = 0
        self._x = None

    @classmethod
    def receiver(cls, engine, rec_bytes, stream=None):
        """Owner-side ops only (decide, unpack_sample), for a batch of records that
        arrived without a local source batch (bench.py's owner workload)."""
        import torch
        self = cls.__new__(cls)
        self.torch = torch
        self.eng, self.db = engine, None
        self.L = native.lib()
        self.stream = stream
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.n = 0
        self.rec_bytes = rec_bytes
        self.counts = None
        self._recv_cap = 0
        self._x = None
        return self

    def _s(self):
        return None if self.stream is None else C.c_void_p(self.stream)

    def pack(self, world):
        torch = self.torch
        self.counts = torch.zeros(world, dtype=torch.int64, device=self.device)
        native.check(self.L.ose_shard_pack(self.eng.h, C.byref(self.db.cols), world, self.send.data_ptr(),
                                           self.counts.data_ptr(), self.pos.data_ptr(), self._s()))
        return self.send, self.counts, self.pos

    def alloc(self, nbytes):
        return self.torch.empty(max(nbytes, 1), dtype=self.torch.uint8, device=self.device)[:nbytes]

    def _ensure(self, n):
        torch = self.torch
        if n <= self._recv_cap and self._x is not None:
            return self._x
        cap = max(int(n * 1.25), 1024)
        planes = self.planes()   # route_match / svc_match: one plane per rule chunk
        x = {k: torch.empty(cap * w * (planes if k in ("route_match", "svc_match") else 1) + 16, dtype=torch.uint8,
                            device=self.device) for k, w in OWNER_COLS}
        x["keep"] = torch.empty(cap, dtype=torch.uint8, device=self.device)
        x["status_word"] = torch.zeros(16, dtype=torch.uint8, device=self.device)
        self._x, self._recv_cap = x, cap
        return x

    def planes(self):
        """rule chunks of the engine's sampling config (records carry one
        endpoint and one rule word per chunk: 40 + 16 per chunk bytes)"""
        return (self.rec_bytes - 40) // 16

    def decide(self, recv, n):
        """The owner's decisions, one keep byte per record (ose_shard_decide)."""
        x = self._ensure(n)
        native.check(self.L.ose_shard_decide(self.eng.h, recv.data_ptr(), n, self.rec_bytes, x["keep"].data_ptr(),
                                             x["status_word"].data_ptr(), C.byref(native.Rand(self.seed, 0.0)),
                                             self._s()))
        return x["keep"]

    def unpack_sample(self, recv, n):
        """The general path: records unpacked into span columns + the SAMPLE stage."""
        x = self._ensure(n)
        p = {k: v.data_ptr() for k, v in x.items()}
        native.check(self.L.ose_shard_unpack(recv.data_ptr(), n, self.rec_bytes,
                                             *[p[k] for k, _ in OWNER_COLS], self._s()))
        cols = native.Columns()
        cols.n_spans = n
        cols.n_resources = n
        cols.match_planes = self.planes()
        for k, _ in OWNER_COLS:
            setattr(cols, k, p[k])
        outs = native.Outputs()
        outs.keep = p["keep"]
        outs.device_status = p["status_word"]
        rnd = native.Rand(self.seed, 0.0)
        native.check(self.L.ose_process_device(self.eng.h, C.byref(cols), C.byref(outs), native.STAGE_SAMPLE,
                                               native.GROUP_TRACE_ID, C.byref(rnd), self._s()))
        return x["keep"]

    def scatter(self, back, pos):
        native.check(self.L.ose_shard_scatter_keep(back.data_ptr(), pos.data_ptr(), self.n,
                                                   self.db.outs.keep, self._s()))


class NcclComm:
    """An RCCL communicator created by the engine library (ose_nccl_comm_init);
    the unique id is broadcast once over an existing torch.distributed group."""

    def __init__(self, rank: int, world: int, group=None):
        import torch
        import torch.distributed as dist
        self.L = native.lib()
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf = (C.c_uint8 * 128)()
            native.check(self.L.ose_nccl_unique_id(buf, 128))
            uid = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
        if world > 1:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
            t = uid.to(dev)
            dist.broadcast(t, 0, group=group)
            uid = t.cpu()
        ub = (C.c_uint8 * 128)(*uid.tolist())
        h = C.c_void_p()
        native.check(self.L.ose_nccl_comm_init(C.byref(h), world, ub, rank))
        self.h, self.rank, self.world = h, rank, world

    def close(self):
        if getattr(self, "h", None):
            self.L.ose_nccl_comm_destroy(self.h)
            self.h = None

    __del__ = close


class NcclExchange:
    """The product round: ``ose_exchange_sample`` (one C-ABI call per step)."""

    seed = 0x5EED

    def __init__(self, engine, db, comm: NcclComm, stream=None):
        self.eng, self.db, self.comm, self.stream = engine, db, comm, stream
        self.L = native.lib()
        self.stats = (C.c_uint64 * 3)()

    def round(self):
        rnd = native.Rand(self.seed, 0.0)
        s = None if self.stream is None else C.c_void_p(self.stream)
        native.check(self.L.ose_exchange_sample(self.eng.h, C.byref(self.db.cols), C.byref(self.db.outs),
                                                self.comm.h, self.comm.rank, self.comm.world, C.byref(rnd), s,
                                                self.stats))

    def allreduce_counters(self, local_ptr: int, node_ptr: int, n: int):
        s = None if self.stream is None else C.c_void_p(self.stream)
        native.check(self.L.ose_allreduce_counters(local_ptr, node_ptr, n, self.comm.h, s))
