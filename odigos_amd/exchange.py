"""Trace-id exchange across the GPUs of one node.

odigossampling needs every span of a trace on one GPU.  In the reference
that co-location is the node collector's loadbalancing exporter keyed by
trace id (autoscaler/controllers/nodecollector/collectorconfig/
traces.go:26-84).  Here, per step:

1. ``ose_shard_pack`` buckets, per span, the 48-byte record (56 with
   span_attribute bits) the trace stage
   reads (trace id, start, end, endpoint-match bits, service ids, status,
   span_attribute bits) by
   owner = hash(trace id) mod world, keeping batch order inside a bucket;
2. an all-to-all of the bucket sizes, then of the records (RCCL over xGMI:
   torch.distributed's "nccl" backend is RCCL on ROCm);
3. ``ose_shard_unpack`` + the SAMPLE stage on the received spans (source
   rank order, then batch order: a trace split over sources is found by the
   trace-id table and handled by the sort-based path);
4. the reverse all-to-all of the keep bytes and ``ose_shard_scatter_keep``.

The protocol (``route_and_sample``) is written against a small ops object
so the same code runs on the device ops below and, in tests, on CPU ops
over gloo.
"""
from __future__ import annotations

import ctypes as C

from . import native



def route_and_sample(ops, world: int, group=None) -> None:
    """One exchange round; ops provides pack/alloc/unpack_sample/scatter."""
    import torch
    import torch.distributed as dist
    XREC = ops.rec_bytes                                # bytes per exchanged span record
    send, counts, pos = ops.pack(world)                 # counts: int64 tensor [world] on ops.device
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    sc = [int(x) for x in counts.tolist()]              # host sync: split sizes
    rc = [int(x) for x in recv_counts.tolist()]
    n_send, n_recv = sum(sc), sum(rc)
    recv = ops.alloc(n_recv * XREC)
    dist.all_to_all_single(recv, send[: n_send * XREC], [c * XREC for c in rc], [c * XREC for c in sc], group=group)
    keep_x = ops.unpack_sample(recv, n_recv)            # uint8 [n_recv]
    back = ops.alloc(n_send)
    dist.all_to_all_single(back, keep_x[:n_recv], sc, rc, group=group)
    ops.scatter(back, pos)


class DeviceExchange:
    """Device ops for route_and_sample over one HBM-resident batch."""

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
        """Owner-side ops only (unpack_sample), for a batch of records that
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
        d = self.device
        x = {"trace_id": torch.empty(2 * cap, dtype=torch.int64, device=d),
             "start_ns": torch.empty(cap, dtype=torch.int64, device=d),
             "end_ns": torch.empty(cap, dtype=torch.int64, device=d),
             "status": torch.empty(cap, dtype=torch.uint8, device=d),
             "resource": torch.empty(cap, dtype=torch.int32, device=d),
             "res_svc": torch.empty(cap, dtype=torch.int32, device=d),
             "res_svc_str": torch.empty(cap, dtype=torch.int32, device=d),
             "route_match": torch.empty(cap, dtype=torch.int64, device=d),
             "attr_match": torch.empty(cap, dtype=torch.int64, device=d),
             "keep": torch.empty(cap, dtype=torch.uint8, device=d),
             "status_word": torch.zeros(4, dtype=torch.int32, device=d)}
        self._x, self._recv_cap = x, cap
        return x

    def unpack_sample(self, recv, n):
        x = self._ensure(n)
        p = {k: v.data_ptr() for k, v in x.items()}
        native.check(self.L.ose_shard_unpack(recv.data_ptr(), n, self.rec_bytes, p["trace_id"], p["start_ns"], p["end_ns"],
                                             p["status"], p["resource"], p["res_svc"], p["res_svc_str"],
                                             p["route_match"], p["attr_match"], self._s()))
        cols = native.Columns()
        cols.n_spans = n
        cols.n_resources = n
        for f in ("trace_id", "start_ns", "end_ns", "status", "resource", "res_svc", "res_svc_str", "route_match",
                  "attr_match"):
            setattr(cols, f, p[f])
        outs = native.Outputs()
        outs.keep = p["keep"]
        outs.device_status = p["status_word"]
        rnd = native.Rand(self.seed, 0.0)
        native.check(self.L.ose_process_device(self.eng.h, C.byref(cols), C.byref(outs), native.STAGE_SAMPLE,
                                               native.GROUP_TRACE_ID, C.byref(rnd), self._s()))
        return x["keep"]

    seed = 0x5EED

    def scatter(self, back, pos):
        native.check(self.L.ose_shard_scatter_keep(back.data_ptr(), pos.data_ptr(), self.n,
                                                   self.db.outs.keep, self._s()))

