#!/usr/bin/env python3
"""bench.py — spans/sec of the Odigos gateway hot path on MI355X.

One "step" = one pass of the configured processors over one device-resident
synthetic batch (BASELINE.json configs; seeds from SURVEY.md §8d).  With
--gpus N the driver launches one rank per GPU (torch.distributed.run); the
timed region is bracketed by barrier + synchronize, the max over ranks is
reported and rank 0 prints ONE JSON line.

Workloads:
  fused     C4 (configs[3], the default): odigossampling -> odigosurltemplate
            -> odigostrafficmetrics over 100M spans in total.  N = 1: all
            100M spans on one GPU.  N > 1: rank r holds the batch node
            collector r of N delivers (gen_batch.cpp split mode: the
            ResourceSpans of one trace land on different ranks), ~100M/N
            spans each (strong scaling); sampling partials go to each trace's
            owner GPU through an RCCL all-to-all (odigos_amd/exchange.py).
  url       C2 (configs[1]): odigosurltemplate, 10M spans/GPU, default rules
  sampling  C3 (configs[2]): odigossampling, 50M spans / ~5M traces per GPU
  zipf      C5 (configs[4]): odigossampling + odigosurltemplate on Zipf(1.1)
            trace sizes (1-50k spans) with 1M distinct routes and 64-bit ids
            in paths, 50M spans per GPU
  owner     diagnostic: on ONE GPU, the batch trace owner 0 receives in an
            8-GPU C4 step (the partial records of 8 source shards in rank
            order, so a trace arrives as several runs): unpack + the SAMPLE
            stage, which takes the sort-based path.

The CPU baseline (rank 0, N = 1) is the oracle (oracle/*.c, built with
-march=native on this host) on C1 = 1M spans of the fused mix, seed
0x0D160001, on this process's CPU share; the same oracle
then checks the timed GPU output at full size (parity_vs_oracle).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "spans/sec processed (whole node) at 1/2/4/8 MI355X; % of HBM roofline"

FUSED_FIELDS = ("arena", "trace_id", "start_ns", "end_ns", "status", "kind", "resource", "scope", "url_flags", "path",
                "route", "span_size", "name_len", "res_svc", "res_svc_str", "res_attrset", "res_size", "scope_size",
                "scope_resource")
SAMPLE_FIELDS = ("arena", "trace_id", "start_ns", "end_ns", "status", "resource", "route", "res_svc", "res_svc_str")
URL_KERNELS = ("url_plan_kernel", "url_plan_slow_kernel", "url_scan_kernel", "url_copy_kernel", "url_emit_slow_kernel")
TRACE_KERNELS = ("trace_eval_kernel", "trace_dup_check", "trace_long_kernel")   # trace_long_kernel: its HIP-event bracket holds trace_long_plan_kernel too
MULTI_KERNELS = ("trace_multi_kernel", "trace_dup_check")   # rule-chunked lists in one pass
# the repeated-trace-id paths, each timed as one span of launches (run lists,
# then the sort path for traces that overflow them)
SLOW_KERNELS = ("trace_run_list", "trace_sort_path")
SIZE_KERNELS = ("size_span_kernel", "size_tail_kernel", "size_fix_kernel")
PER_TRACE_OUTS = ("trace_count", "trace_first_span", "trace_keep", "trace_level", "trace_ratio")

WORKLOADS = {
    "url": dict(gen="url", seed=0x0D160002, spans=10_000_000, per_gpu=True,
                cfg={"odigosurltemplate": {}}, stages="TEMPLATE",
                # no include/exclude configured: the shim passes res_url_ok = NULL
                null_columns=("res_url_ok",), null_outputs=(),
                fields=("arena", "kind", "url_flags", "path"), kernels=URL_KERNELS,
                metric_config="C2: URL templatization only, 10M spans/GPU, C2 segment mix, default rules"),
    "sampling": dict(gen="sampling", seed=0x0D160003, spans=50_000_000, per_gpu=True,
                     cfg=None, stages="SAMPLE", null_columns=(), null_outputs=PER_TRACE_OUTS,
                     fields=SAMPLE_FIELDS, kernels=TRACE_KERNELS + SLOW_KERNELS,
                     metric_config="C3: trace-level sampling (1 error + 4 service + 16 latency rules), "
                                   "50M spans / ~5M traces per GPU, grouped by trace_id"),
    "sampling_wide": dict(gen="sampling", seed=0x0D160003, spans=50_000_000, per_gpu=True,
                          cfg="wide", stages="SAMPLE", null_columns=(), null_outputs=PER_TRACE_OUTS,
                          fields=SAMPLE_FIELDS, kernels=MULTI_KERNELS[:1] + TRACE_KERNELS + SLOW_KERNELS,
                          metric_config="diagnostic: C3's batch under 1 error + 4 service + 150 latency rules "
                                        "(three rule chunks, evaluated in one trace-stage pass)"),
    "zipf": dict(gen="zipf", seed=0x0D160005, spans=50_000_000, per_gpu=True,
                 cfg=None, stages="SAMPLE|TEMPLATE", null_columns=("res_url_ok",), null_outputs=PER_TRACE_OUTS,
                 fields=SAMPLE_FIELDS + ("kind", "url_flags", "path"), kernels=TRACE_KERNELS + SLOW_KERNELS + URL_KERNELS,
                 metric_config="C5: odigossampling + odigosurltemplate on Zipf(1.1) trace sizes (1 to 50k "
                               "spans/trace), 1M distinct routes, 64-bit user ids in paths, 50M spans per GPU"),
    "fused": dict(gen="fused", seed=0x0D160004, spans=100_000_000, per_gpu=False,
                  cfg=None, stages="SAMPLE|TEMPLATE|SIZE", null_columns=("res_url_ok",),
                  null_outputs=PER_TRACE_OUTS + ("res_bytes",), fields=FUSED_FIELDS,
                  kernels=TRACE_KERNELS + SLOW_KERNELS + URL_KERNELS + SIZE_KERNELS,
                  metric_config="C4: fused odigossampling -> odigosurltemplate -> odigostrafficmetrics, 100M spans "
                                "in total (all on one GPU at N=1; ~100M/N per GPU, trace-id all-to-all over RCCL "
                                "at N>1)"),
    "node8": dict(gen="fused", seed=0x0D160004, spans=100_000_000, per_gpu=False, ranks=8,
                  cfg=None, stages="SAMPLE|TEMPLATE|SIZE", null_columns=("res_url_ok",),
                  null_outputs=PER_TRACE_OUTS + ("res_bytes",), fields=FUSED_FIELDS,
                  kernels=("shard_pack", "owner_fold", "shard_unpack") + TRACE_KERNELS + SLOW_KERNELS + URL_KERNELS + SIZE_KERNELS,
                  metric_config="diagnostic: C4 at N=8 emulated on ONE GPU -- the 8 ranks' whole steps (pack, the "
                                "exchange round through the in-process transport, owner SAMPLE, reverse split, "
                                "TEMPLATE on a second stream, SIZE|APPLY_KEEP), one thread, engine and stream pair "
                                "per rank; the projected per-GPU step is the wall time / 8"),
    "owner": dict(gen="fused", seed=0x0D160004, spans=100_000_000, per_gpu=False, sources=8,
                  cfg=None, stages="SAMPLE", null_columns=(), null_outputs=PER_TRACE_OUTS,
                  fields=SAMPLE_FIELDS, kernels=("owner_fold", "shard_unpack") + TRACE_KERNELS + SLOW_KERNELS,
                  metric_config="C4 owner side on one GPU: the records trace owner 0 of 8 receives "
                                "(8 source shards of the 100M-span C4 batch, rank order), decided by ose_shard_decide "
                                "(the bucketed fold; unpack + SAMPLE when it overflows)"),
}

# node-collector res_attributes_keys (autoscaler/controllers/nodecollector/collectorconfig/ownmetrics-ui.go:33-47)
NODE_KEYS = ["k8s.namespace.name", "k8s.deployment.name", "k8s.statefulset.name", "k8s.daemonset.name",
             "k8s.cronjob.name", "k8s.job.name", "k8s.pod.name", "k8s.node.name", "service.name"]
C1 = dict(gen="fused", seed=0x0D160001, spans=1_000_000)   # SURVEY.md §8d CPU reference config


def _cfg(wl):
    if wl["cfg"] == "wide":
        from tests.workloads import wide_latency_config
        return {"odigossampling": wide_latency_config()}
    if wl["cfg"] is not None:
        return wl["cfg"]
    from tests.workloads import c3_sampling_config
    st = wl["stages"]
    cfg = {"odigossampling": c3_sampling_config()}
    if "TEMPLATE" in st:
        cfg["odigosurltemplate"] = {}
    if "SIZE" in st:
        cfg["odigostrafficmetrics"] = {"res_attributes_keys": NODE_KEYS}
    return cfg


def _stages(wl):
    from odigos_amd import native
    m = 0
    for s in wl["stages"].split("|"):
        m |= getattr(native, "STAGE_" + s)
    return m


# ---- algorithmic bytes -------------------------------
def algorithmic_bytes_url(gen, url_out, tmpl, n) -> int:
    """URL row: per span 8 B path ref + 1 B kind + 1 B url_flags read, 8 B
    template ref + 1 B url_out written; plus the path bytes of every span
    whose path is templatized (read) and the template bytes written (the
    lengths of the emitted templates: the packed arena's size, and what the
    refs form writes)."""
    path = gen.array("path").view(np.uint32).reshape(-1, 2)[:n]
    templ_read = int(path[(url_out[:n] & 1) != 0, 1].sum())
    written = int(tmpl.reshape(-1, 2)[:n][url_out[:n] != 0, 1].astype(np.int64).sum())
    return n * (8 + 1 + 1) + n * (8 + 1) + templ_read + written


def algorithmic_bytes_sampling(gen, n, cfg) -> int:
    """Sampling row: per span 16 B trace_id + 8 B start + 8 B end + 1 B
    status + 4 B resource + 8 B route ref read and 1 B keep written; per
    resource 8 B (res_svc, res_svc_str); plus min(len(route), longest rule
    route) route bytes per span that carries one."""
    rules = cfg["odigossampling"].get("endpoint_rules", []) + cfg["odigossampling"].get("service_rules", []) + \
        cfg["odigossampling"].get("global_rules", [])
    pmax = max([len(r["rule_details"].get("http_route", "")) for r in rules] + [0])
    route = gen.array("route").view(np.uint32).reshape(-1, 2)[:n]
    rb = int(np.minimum(route[:, 1], pmax).sum())
    return n * (16 + 8 + 8 + 1 + 4 + 8 + 1) + gen.cols.n_resources * 8 + rb


def algorithmic_bytes(wl, gen, db, n, cfg) -> int:
    st = wl["stages"]
    b = 0
    if "SAMPLE" in st:
        b += algorithmic_bytes_sampling(gen, n, cfg)
    if "TEMPLATE" in st:
        b += algorithmic_bytes_url(gen, db.out_numpy("url_out", n=n), db.out_numpy("tmpl", np.uint32, n=2 * n), n)
    if "SIZE" in st:
        # span_size, scope, name_len per span; 8 B per scope, 12 B per resource, 8 B per attribute set
        b += n * 12 + gen.cols.n_scopes * 8 + gen.cols.n_resources * 12 + gen.cols.n_attrsets * 8
    return b


# ---- CPU baseline (oracle) ----------------------------------------------------------
def cpu_share():
    """(threads this process may use, nproc, CPU model).  The GPU box gives a
    one-GPU job a share of the host (16 CPUs); nproc shows every CPU of the
    machine, so the share is read from the affinity mask, the cgroup quota
    and OMP_NUM_THREADS (set to the share on the box)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    share = aff
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            share = min(share, max(1, int(int(q) / int(p))))
    except Exception:
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        share = min(share, max(1, int(os.environ["OMP_NUM_THREADS"])))
    model = ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return share, os.cpu_count() or 1, model


def native_oracle() -> str:
    """Builds oracle/*.c with -march=native for this host (the checker and the
    CPU baseline; the in-tree liboracle.so is built for a generic x86-64)."""
    out = Path(tempfile.gettempdir()) / f"liboracle_native_{os.getpid()}.so"
    src = sorted(str(p) for p in (ROOT / "oracle").glob("*.c"))
    r = subprocess.run(["gcc", "-std=c11", "-O3", "-march=native", "-fPIC", "-pthread", "-shared", "-o", str(out),
                        *src, "-lm"], capture_output=True, text=True)
    if r.returncode != 0:
        return ""
    os.environ["OSE_ORACLE_LIB"] = str(out)
    return "-O3 -march=native"


def oracle_chain(cfg, stages):
    """The oracles chained in gateway order (sampling -> templating -> size)."""
    from odigos_amd import native
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import SamplingOracle, UrlOracle, size_process
    so = SamplingOracle(cfg["odigossampling"]) if stages & native.STAGE_SAMPLE else None
    uo = UrlOracle(cfg["odigosurltemplate"]) if stages & native.STAGE_TEMPLATE else None

    def chain(cols, nt):
        ho = HostOutputs(cols)
        if so:
            assert so.process(cols, ho.outs, native.GROUP_TRACE_ID, 0x5EED, nt) == 0
        if uo:
            assert uo.process(cols, ho.outs, nt) == 0
        if stages & native.STAGE_SIZE:
            assert size_process(cols, ho.outs, stages, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0, nt) == 0
        return ho
    return chain


def cpu_baseline(wl, cfg, stages, threads, budget_s=12.0):
    """C1 (1M spans of the fused mix, seed 0x0D160001) through the oracle
    chain of this workload's stages: `threads` pthreads repeated to about
    budget_s/2, then one single-thread pass."""
    from odigos_amd.batch import Generator
    chain = oracle_chain(cfg, stages)
    g = Generator(C1["gen"], seed=C1["seed"], n_spans=C1["spans"], threads=threads)
    n = g.cols.n_spans
    reps, t0 = 0, time.perf_counter()
    while True:
        chain(g.cols, threads)
        reps += 1
        if time.perf_counter() - t0 > budget_s / 2 or reps >= 200:
            break
    mt = n * reps / (time.perf_counter() - t0)
    t1 = time.perf_counter()
    chain(g.cols, 1)
    st = n / (time.perf_counter() - t1)
    return mt, st, f"C1: {n} spans of the fused mix (seed 0x0D160001) x {reps} passes, oracle chain " \
                   f"[{wl['stages']}] with {threads} pthreads"


def parity_full(wl, gen, db, cfg, stages, threads, calls):
    """The oracle chain on the whole timed batch against the GPU outputs:
    keep, url_out, template refs and bytes, attribute-set counters."""
    from odigos_amd import native
    chain = oracle_chain(cfg, stages)
    ho = chain(gen.cols, threads)
    n = gen.cols.n_spans
    res = {}
    if stages & native.STAGE_SAMPLE:
        res["keep"] = bool(np.array_equal(ho.view("keep", np.uint8)[:n], db.out_numpy("keep", n=n)))
    if stages & native.STAGE_TEMPLATE:
        uo = db.out_numpy("url_out", n=n)
        res["url_out"] = bool(np.array_equal(ho.view("url_out", np.uint8)[:n], uo))
        m = uo != 0
        used = db.used()
        if stages & native.STAGE_TEMPLATE_REFS:
            # per span: the bytes each ref names (the arena is sparse)
            from tests.oracle_lib import span_template_bytes
            gb, gl = span_template_bytes(db.out_numpy("tmpl", np.uint32, n=2 * n), db.out_numpy("tmpl_arena", n=used), m)
            ob, ol = span_template_bytes(ho.view("tmpl", np.uint32)[: 2 * n], ho.bufs["tmpl_arena"][: int(ho.used[0])], m)
            res["tmpl_lens"] = bool(np.array_equal(gl, ol))
            res["tmpl_bytes_per_span"] = bool(gb.size == ob.size and np.array_equal(gb, ob))
        else:
            res["tmpl_refs"] = bool(np.array_equal(ho.view("tmpl", np.uint64)[:n][m],
                                                   db.out_numpy("tmpl", np.uint64, n=n)[m]))
            res["tmpl_arena"] = bool(used == int(ho.used[0]) and
                                     np.array_equal(ho.bufs["tmpl_arena"][:used], db.out_numpy("tmpl_arena", n=used)))
    if stages & native.STAGE_SIZE:
        A = gen.cols.n_attrsets
        # the device counters were ADDED to by every timed and warm-up call
        res["attrset_bytes"] = bool(np.array_equal(calls * ho.view("attrset_bytes", np.int64)[:A],
                                                   db.out_numpy("attrset_bytes", np.int64, n=A)))
        res["accepted_spans"] = bool(calls * int(ho.view("accepted_spans", np.int64)[0]) ==
                                     int(db.out_numpy("accepted_spans", np.int64, n=1)[0]))
    return res


# ---- owner-side workload --------------------------------------------------------------
def build_owner_batch(eng, wl, threads):
    """Packs the 8 source shards of the C4 batch on this GPU and keeps what
    trace owner 0 receives, in source-rank order (what the all-to-all
    delivers).  Returns the device record buffer, its record count and the
    number of source spans those records stand for."""
    import ctypes as C

    import torch

    from odigos_amd import native
    from odigos_amd.batch import DeviceBatch, Generator
    L = native.lib()
    W = wl["sources"]
    rb = int(L.ose_shard_record_bytes(eng.h))
    parts, spans_repr = [], 0
    for s in range(W):
        g = Generator(wl["gen"], seed=wl["seed"], n_spans=wl["spans"], threads=threads, rank=s, world=W)
        db = DeviceBatch(g.cols, fields=SAMPLE_FIELDS)
        n = g.cols.n_spans
        send = torch.empty(max(n, 1) * rb, dtype=torch.uint8, device="cuda")
        counts = torch.zeros(W, dtype=torch.int64, device="cuda")
        pos = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
        native.check(L.ose_shard_pack(eng.h, C.byref(db.cols), W, send.data_ptr(), counts.data_ptr(),
                                      pos.data_ptr(), None))
        c0 = int(counts[0].item())
        parts.append(send[: c0 * rb].clone())
        # spans whose trace owner is rank 0
        pos_np = pos[:n].cpu().numpy()
        spans_repr += int((pos_np.astype(np.int64) < c0).sum())
        del db, send, pos, g
    recv = torch.cat(parts)
    return recv, recv.numel() // rb, spans_repr, rb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # default: the whole hot path (C4), which is also the configuration the
    # multi-GPU runs exercise (trace-id exchange when N > 1); DESIGN.md §6
    ap.add_argument("--workload", default="fused", choices=sorted(WORKLOADS))
    ap.add_argument("--spans", type=int, default=0, help="override the workload's span count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    # refs (OSE_STAGE_TEMPLATE_REFS): the templates stay where the GPU assembled
    # them and the device-resident consumer follows the refs; packed: the
    # compact arena a host copy needs (one more pass over the template bytes)
    ap.add_argument("--tmpl-form", default="refs", choices=("refs", "packed"))
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from odigos_amd import native
    from odigos_amd.batch import DeviceBatch, Engine, Generator

    wl = WORKLOADS[args.workload]
    stages = _stages(wl)
    tform = native.STAGE_TEMPLATE_REFS if args.tmpl_form == "refs" else 0
    if stages & native.STAGE_TEMPLATE:
        stages |= tform
    cfg = _cfg(wl)
    share, nproc, model = cpu_share()
    gen_threads = max(1, min(16, share))
    eng = Engine(cfg)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    total = args.spans or wl["spans"]
    gen = db = comm = None
    extra = {}

    if args.workload == "node8":
        assert world == 1, "the node8 workload emulates an 8-GPU step on one GPU"
        from tests.node_emul import LocalNode
        W = wl["ranks"]
        gens = []
        for r in range(W):
            g = Generator(wl["gen"], seed=wl["seed"], n_spans=total, threads=gen_threads, rank=r, world=W)
            for f in wl.get("null_columns", ()):
                setattr(g.cols, f, None)
            gens.append(g)
        one = os.environ.get("OSE_NODE8_ONE_STREAM")
        node = LocalNode(cfg, gens, fields=wl.get("fields"), null_outputs=wl.get("null_outputs", ()), tmpl_form=tform,
                         one_stream=stream if one else None, engine0=eng)
        dbs, stats = node.dbs, node.stats
        n_units = sum(g.cols.n_spans for g in gens)
        step = node.step
        extra = {"emulated_ranks": W, "one_stream": bool(one),
                 "kernel_times": "per-kernel HIP-event brackets are not reported at node8: the 8 ranks' host "
                                 "threads submit concurrently and their brackets overlap; per-kernel durations "
                                 "come from rocprofv3 --kernel-trace of the one-stream run (profiles/)"}
    elif args.workload == "owner":
        assert world == 1, "the owner workload emulates an 8-GPU step on one GPU"
        recv, n_rec, spans_repr, rb = build_owner_batch(eng, wl, gen_threads)
        from odigos_amd.exchange import DeviceExchange
        ex = DeviceExchange.receiver(eng, rb, stream=sh)
        n_units = spans_repr
        extra = {"records": n_rec, "record_bytes": rb, "spans_represented": spans_repr}
        eng.reserve(max(n_rec, 1))

        def step():
            ex.decide(recv, n_rec)
    else:
        if wl["per_gpu"]:
            gen = Generator(wl["gen"], seed=wl["seed"] + rank, n_spans=total, threads=gen_threads)
        else:
            gen = Generator(wl["gen"], seed=wl["seed"], n_spans=total, threads=gen_threads, rank=rank, world=world)
        for f in wl.get("null_columns", ()):
            setattr(gen.cols, f, None)   # columns the configured processors do not read
        db = DeviceBatch(gen.cols, fields=wl.get("fields"))
        for f in wl.get("null_outputs", ()):
            setattr(db.outs, f, None)    # outputs the shim does not read (per-trace diagnostics)
        n_units = gen.cols.n_spans
        eng.reserve(n_units, gen.cols.arena_bytes)
        if world > 1 and stages & native.STAGE_SAMPLE:
            # fold each rank's spans into partial records, route them
            # to each trace's owner GPU (RCCL over xGMI), decide there, bring keep
            # back (one C-ABI call: ose_exchange_sample), then template and size
            # locally on the decisions and sum the traffic counters over the node
            from odigos_amd.exchange import NcclComm, NcclExchange
            comm = NcclComm(rank, world)
            nx = NcclExchange(eng, db, comm, stream=sh)
            local_st = (stages & ~native.STAGE_SAMPLE) | native.STAGE_APPLY_KEEP
            A = gen.cols.n_attrsets
            node_ctr = torch.zeros(A + 1, dtype=torch.int64, device="cuda")

            # TEMPLATE reads nothing the exchange writes: it runs on a second
            # stream while the round packs, waits for the counts, moves the
            # records and decides on the owners (the exchange
            # overlapped with the URL stage); SIZE | APPLY_KEEP joins both
            side = torch.cuda.Stream()
            side_h = side.cuda_stream
            tmpl_st = local_st & (native.STAGE_TEMPLATE | native.STAGE_TEMPLATE_REFS)
            rest_st = local_st & ~(native.STAGE_TEMPLATE | native.STAGE_TEMPLATE_REFS)
            if tmpl_st:
                rest_st |= native.STAGE_APPLY_TEMPLATE   # SIZE counts what TEMPLATE wrote on the side stream

            def step():
                if tmpl_st:
                    side.wait_stream(stream)   # the previous step's SIZE has read this step's outputs
                    eng.process_device(db, tmpl_st, native.GROUP_TRACE_ID, seed=0x5EED, stream=side_h)
                nx.round()
                if tmpl_st:
                    stream.wait_stream(side)
                if rest_st & native.STAGE_SIZE:
                    eng.process_device(db, rest_st, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)
                    nx.allreduce_counters(db.outs.attrset_bytes, node_ctr.data_ptr(), A)
                    nx.allreduce_counters(db.outs.accepted_spans, node_ctr.data_ptr() + 8 * A, 1)
        else:
            def step():
                eng.process_device(db, stages, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    all_engs = [] if args.workload == "node8" else [eng]
    for e in all_engs:
        e.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = {}
    for e in all_engs:
        e.profile(False)
        for k, v in e.profile_read().items():
            acc = prof.setdefault(k, {"launches": 0, "ms": 0.0})
            acc["launches"] += v["launches"]
            acc["ms"] += v["ms"]
    for d in (dbs if args.workload == "node8" else [db] if db is not None else []):
        status = int(d.out_numpy("device_status", np.uint32)[0])
        if status:
            raise SystemExit(f"device status {status}: kernel reported a failure")
    units = torch.tensor([float(n_units)], dtype=torch.float64, device="cuda")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.all_reduce(units, op=dist.ReduceOp.SUM)
    total_units = float(units.item())

    per_k = {}
    for kn in wl["kernels"]:
        k = prof.get(kn, {"launches": 0, "ms": 0.0})
        per_k[kn] = k["ms"] / max(args.steps, 1)   # device ms per step (gated kernels: 0 when not launched)
    k_ms = sum(per_k.values())
    kname = "+".join(wl["kernels"])
    # SAMPLE + TEMPLATE by trace id: the URL planning kernels run on a second
    # stream beside the trace stage (engine.cpp run_stages; OSE_ONE_STREAM=1
    # serialises them for per-kernel profiles), so their HIP-event brackets
    # overlap and the roofline's time base is the step
    overlapped = (args.workload not in ("node8", "owner") and world == 1 and stages & native.STAGE_SAMPLE
                  and stages & native.STAGE_TEMPLATE and n_units >= (1 << 20) and not os.environ.get("OSE_ONE_STREAM"))
    if world > 1 and stages & native.STAGE_SAMPLE:
        st_ = [int(x) for x in nx.stats]
        extra.update({"exchange_records_sent": st_[0], "exchange_records_received": st_[1],
                      "exchange_record_bytes_per_span": native.XREC_BYTES * st_[0] / max(st_[2], 1)})
        out_kernels = dict(prof)
        extra["exchange_kernels_ms"] = {k: v["ms"] / max(args.steps, 1) for k, v in out_kernels.items()
                                        if k in ("shard_pack", "owner_fold", "shard_unpack", "owner_sample")}
    if args.workload == "node8":
        st_ = [[int(x) for x in st] for st in stats]
        extra.update({"exchange_records_sent": sum(x[0] for x in st_),
                      "exchange_record_bytes_per_span": native.XREC_BYTES * sum(x[0] for x in st_) / max(n_units, 1),
                      "projected_ms_per_gpu_step": elapsed / args.steps * 1e3 / W,
                      "projected_xgmi_ms": native.XREC_BYTES * max(x[0] for x in st_) * (W - 1) / W /
                                           (7 * 153e9) * 1e3 * 2})   # records + keep bytes back, 7 links of 153 GB/s
    if args.workload == "owner":
        b_alg = None
        achieved = 0.0
    else:
        if args.workload == "node8":
            # per-GPU algorithmic bytes over the projected per-GPU step (wall / 8)
            b_alg = sum(algorithmic_bytes(wl, g, d, g.cols.n_spans, cfg) for g, d in zip(gens, dbs))
            achieved = b_alg / (elapsed / args.steps) / 1e9
        else:
            b_alg = algorithmic_bytes(wl, gen, db, n_units, cfg)
            achieved = b_alg / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0
            if overlapped:   # the brackets overlap: the stage set's GPU time is at most the step
                achieved = b_alg / (elapsed / args.steps) / 1e9

    traffic = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            d = json.loads(tj.read_text())
            ent = d.get(args.workload, {}).get(kname)
            if ent and ent.get("spans") == n_units:
                traffic = ent["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    value = total_units * args.steps / elapsed
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "spans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if wl["per_gpu"] else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, SURVEY.md §8d mix)",
        "config": {"workload": wl["metric_config"], "spans_per_gpu": n_units, "spans_total": int(total_units),
                   "template_form": args.tmpl_form if stages & native.STAGE_TEMPLATE else None,
                   "seed": wl["seed"], "processors": list(cfg.keys()),
                   "parallelism": (f"dp{world}: trace-id all-to-all (RCCL) of sampling partials, local templating/size"
                                   if world > 1 and stages & native.STAGE_SAMPLE else
                                   f"dp{world}: independent span shards, no data-path collective"), **extra},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "kernel_ms": None if args.workload == "node8" else k_ms,
                     "time_base": "step (SAMPLE and the URL planning overlap on two streams; kernel_ms_each are "
                                  "overlapping brackets)" if overlapped else "kernel_ms",
                     "kernel_ms_each": None if args.workload == "node8" else per_k,
                     "algorithmic_bytes_per_launch": b_alg},
    }
    # measured HBM stream-copy bandwidth beside the spec peak (2 x 2 GiB copy,
    # read + written bytes over the kernel time)
    try:
        import ctypes as C
        a_ = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
        b_ = torch.empty_like(a_)
        bw = C.c_double()
        native.check(native.lib().osehost_stream_copy(b_.data_ptr(), a_.data_ptr(), a_.numel(), 10, C.c_void_p(sh),
                                                      C.byref(bw)))
        out["roofline"]["stream_copy_gbs"] = bw.value
        out["roofline"]["frac_of_stream_copy"] = achieved / bw.value if bw.value else None
        del a_, b_
    except Exception as ex:   # diagnostics only
        out["roofline"]["stream_copy_gbs"] = None
        print("stream copy measurement failed:", ex, file=sys.stderr)
    if world > 1 and not args.no_parity:
        # every rank's outputs against the oracle: split workloads (C4) on rank 0
        # over the W sources concatenated in rank order (the global batch the
        # trace-id exchange decides), per-GPU workloads on each rank's own batch
        # (tests/dist_parity.py; the checker only, after the timed region)
        from tests import dist_parity
        if rank == 0:
            native_oracle()
        n = gen.cols.n_spans
        if not wl["per_gpu"]:
            A = gen.cols.n_attrsets
            has_t = bool(stages & native.STAGE_TEMPLATE)
            has_s = bool(stages & native.STAGE_SIZE)
            dig = dist_parity.output_digest(
                n, stages, keep=db.out_numpy("keep", n=n),
                url_out=db.out_numpy("url_out", n=n) if has_t else None,
                tmpl=db.out_numpy("tmpl", np.uint32, n=2 * n) if has_t else None,
                tmpl_arena=db.out_numpy("tmpl_arena", n=db.used()) if has_t else None,
                attrset_bytes=db.out_numpy("attrset_bytes", np.int64, n=A) if has_s else None,
                accepted_spans=int(db.out_numpy("accepted_spans", np.int64, n=1)[0]) if has_s else None,
                node_counters=(node_ctr[:A].cpu().numpy(), int(node_ctr[A].item())) if has_s else None)

            def regen(s):
                g = Generator(wl["gen"], seed=wl["seed"], n_spans=total, threads=gen_threads, rank=s, world=world)
                for f in wl.get("null_columns", ()):
                    setattr(g.cols, f, None)
                return g
            par = dist_parity.split_parity(rank, world, dig, regen, cfg, stages, args.steps + args.warmup, share,
                                           own_source=gen)
        else:
            par = dist_parity.local_parity(rank, world, parity_full(wl, gen, db, cfg, stages, share,
                                                                   args.steps + args.warmup))
        if rank == 0:
            out["parity_vs_oracle"] = all(par.values())
            out["parity"] = par
    if rank == 0 and world == 1 and args.workload != "owner":
        orc = native_oracle()
        if not args.no_cpu_baseline:
            mt, st1, sample = cpu_baseline(wl, cfg, stages, share)
            out["cpu_baseline"] = {"value": mt, "unit": "spans/s", "cores": share, "kind": "port", "sample": sample,
                                   "value_1core": st1, "nproc": nproc, "cpu_model": model,
                                   "build": orc or "in-tree liboracle.so (-O3 -march=x86-64-v2)"}
        if not args.no_parity:
            # the oracle on the whole timed batch checks the GPU output
            if args.workload == "node8":
                from tests.oracle_lib import node_parity
                par = node_parity(gens, dbs, cfg, stages, share, args.steps + args.warmup, node.node_counters())
            else:
                par = parity_full(wl, gen, db, cfg, stages, share, args.steps + args.warmup)
            out["parity_vs_oracle"] = all(par.values())
            out["parity"] = par
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        if comm is not None:
            torch.cuda.synchronize()
            comm.close()   # the RCCL communicator goes before the process group and the HIP runtime
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
