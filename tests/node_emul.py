"""An N-GPU step of the C4 pipeline emulated on ONE GPU (test and bench
infrastructure): one engine, batch, stream pair and host thread per rank;
the exchange round and the counter all-reduce go through the in-process
transport (osehost_xgroup_*, shard_host.cpp) where RCCL would move the bytes
over xGMI.  The step is what bench.py runs per rank at N > 1: TEMPLATE on a
second stream (it needs no decision), ose_exchange_sample's round (pack,
all-to-all, owner unpack + SAMPLE, reverse split, scatter), then SIZE |
APPLY_KEEP on the decisions and the node's counters summed over the ranks
(ose_allreduce_counters)."""
from __future__ import annotations

import concurrent.futures as cf
import ctypes as C

from odigos_amd import native


class LocalNode:
    def __init__(self, cfg: dict, gens, fields=None, null_outputs=(), tmpl_form: int = 0, one_stream=None,
                 seed: int = 0x5EED, engine0=None):
        import torch
        from odigos_amd.batch import DeviceBatch, Engine
        self.L = native.lib()
        self.W = len(gens)
        self.seed = seed
        self.tform = tmpl_form
        self.grp = C.c_void_p()
        native.check(self.L.osehost_xgroup_create(self.W, C.byref(self.grp)))
        self.gens, self.engs, self.dbs, self.mains, self.sides, self.ctr = list(gens), [], [], [], [], []
        for r, g in enumerate(gens):
            d = DeviceBatch(g.cols, fields=fields)
            for f in null_outputs:
                setattr(d.outs, f, None)
            e = engine0 if (r == 0 and engine0 is not None) else Engine(cfg)
            e.reserve(g.cols.n_spans, g.cols.arena_bytes)
            self.engs.append(e)
            self.dbs.append(d)
            if one_stream is not None:
                # every rank's work on ONE stream: the GPU runs the kernels one at a time
                self.mains.append(one_stream)
                self.sides.append(one_stream)
            else:
                self.mains.append(torch.cuda.Stream())
                self.sides.append(torch.cuda.Stream())
            A = g.cols.n_attrsets
            self.ctr.append(torch.zeros(A + 1, dtype=torch.int64, device="cuda"))
        self.stats = [(C.c_uint64 * 3)() for _ in range(self.W)]
        self.size_on = "odigostrafficmetrics" in cfg
        self.pool = cf.ThreadPoolExecutor(self.W)

    def rank_step(self, r):
        e, d, m, s = self.engs[r], self.dbs[r], self.mains[r], self.sides[r]
        rnd = native.Rand(self.seed, 0.0)
        s.wait_stream(m)   # the previous step's SIZE has read this step's outputs
        e.process_device(d, native.STAGE_TEMPLATE | self.tform, native.GROUP_TRACE_ID, seed=self.seed,
                         stream=s.cuda_stream)
        native.check(self.L.osehost_exchange_sample_local(e.h, C.byref(d.cols), C.byref(d.outs), self.grp, r,
                                                          C.byref(rnd), C.c_void_p(m.cuda_stream), self.stats[r]))
        m.wait_stream(s)
        if self.size_on:
            e.process_device(d, native.STAGE_SIZE | native.STAGE_APPLY_KEEP | native.STAGE_APPLY_TEMPLATE,
                             native.GROUP_TRACE_ID, seed=self.seed, stream=m.cuda_stream)
            A = self.gens[r].cols.n_attrsets
            node = self.ctr[r].data_ptr()
            native.check(self.L.osehost_allreduce_counters_local(d.outs.attrset_bytes, node, A, self.grp, r,
                                                                 C.c_void_p(m.cuda_stream)))
            native.check(self.L.osehost_allreduce_counters_local(d.outs.accepted_spans, node + 8 * A, 1, self.grp,
                                                                 r, C.c_void_p(m.cuda_stream)))
        else:
            e.process_device(d, native.STAGE_APPLY_KEEP, native.GROUP_TRACE_ID, seed=self.seed, stream=m.cuda_stream)

    def step(self):
        for f in [self.pool.submit(self.rank_step, r) for r in range(self.W)]:
            f.result()

    def node_counters(self, r: int = 0):
        """(attrset_bytes, accepted_spans) of the node as rank r's all-reduce left them."""
        A = self.gens[r].cols.n_attrsets
        v = self.ctr[r].cpu().numpy()
        return v[:A], int(v[A])

    def close(self):
        self.pool.shutdown()
        self.L.osehost_xgroup_destroy(self.grp)
