#!/usr/bin/env python3
"""bench.py — spans/sec of the Odigos gateway hot path on MI355X.

One "step" = one pass of the configured processors over one device-resident
synthetic batch (BASELINE.json configs; seeds from SURVEY.md §8d).  With
--gpus N the driver launches one rank per GPU (torch.distributed.run); every
rank processes its own shard (weak scaling: the path partitions by trace,
SURVEY.md §8e), the timed region is bracketed by barrier + synchronize, and
the max over ranks is reported.  Rank 0 prints ONE JSON line.

Workloads (per GPU):
  url       C2  odigosurltemplate, 10M spans, default rules          (configs[1])
  sampling  C3  odigossampling, 50M spans / ~5M traces, C3 rules     (configs[2])
  zipf      C5  odigossampling on Zipf trace sizes (1-50k spans), 50M spans  (configs[4])
  fused     C4  all three processors, 12.5M spans/GPU (100M on 8)    (configs[3]);
                with N > 1 the sampling records go to each trace's owner
                GPU through an RCCL all-to-all (odigos_amd/exchange.py)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

WORKLOADS = {
    "url": dict(gen="url", seed=0x0D160002, spans=10_000_000,
                cfg={"odigosurltemplate": {}}, stages="TEMPLATE", group="TRACE_ID",
                # no include/exclude configured: the shim passes res_url_ok = NULL
                null_columns=("res_url_ok",), null_outputs=(),
                fields=("arena", "kind", "url_flags", "path"),
                kernels=("url_plan_kernel", "url_scan_kernel", "url_emit_kernel", "url_emit_slow_kernel"),
                metric_config="C2: URL templatization only, 10M spans/GPU, C2 segment mix, default rules"),
    "sampling": dict(gen="sampling", seed=0x0D160003, spans=50_000_000,
                     cfg=None, stages="SAMPLE", group="TRACE_ID",
                     null_columns=(), null_outputs=("trace_count", "trace_first_span", "trace_keep", "trace_level",
                                                    "trace_ratio"),
                     fields=("arena", "trace_id", "start_ns", "end_ns", "status", "resource", "route", "res_svc",
                             "res_svc_str"),
                     kernels=("trace_eval_kernel", "trace_long_kernel"),
                     metric_config="C3: trace-level sampling (1 error + 4 service + 16 latency rules), "
                                   "50M spans / ~5M traces per GPU, grouped by trace_id"),
    "zipf": dict(gen="zipf", seed=0x0D160005, spans=50_000_000,
                 cfg=None, stages="SAMPLE", group="TRACE_ID",
                 null_columns=(), null_outputs=("trace_count", "trace_first_span", "trace_keep", "trace_level",
                                                "trace_ratio"),
                 fields=("arena", "trace_id", "start_ns", "end_ns", "status", "resource", "route", "res_svc",
                         "res_svc_str"),
                 kernels=("trace_eval_kernel", "trace_long_kernel"),
                 metric_config="C5: trace-level sampling on Zipf(1.1) trace sizes (1 to 50k spans/trace), "
                               "50M spans per GPU, C3 rules, grouped by trace_id"),
    "fused": dict(gen="fused", seed=0x0D160004, spans=12_500_000,
                  cfg=None, stages="SAMPLE|TEMPLATE|SIZE", group="TRACE_ID",
                  null_columns=("res_url_ok",), null_outputs=("trace_count", "trace_first_span", "trace_keep",
                                                             "trace_level", "trace_ratio", "res_bytes"),
                  fields=("arena", "trace_id", "start_ns", "end_ns", "status", "kind", "resource", "scope",
                          "url_flags", "path", "route", "span_size", "name_len", "res_svc", "res_svc_str",
                          "res_attrset", "res_size", "scope_size", "scope_resource"),
                  kernels=("trace_eval_kernel", "trace_long_kernel", "url_plan_kernel", "url_scan_kernel", "url_emit_kernel", "url_emit_slow_kernel",
                           "size_span_kernel", "size_scope_kernel", "size_res_kernel"),
                  metric_config="C4: fused odigossampling -> odigosurltemplate -> odigostrafficmetrics, "
                                "12.5M spans/GPU (100M on 8), trace-id all-to-all over RCCL when N > 1"),
}

# node-collector res_attributes_keys (autoscaler/controllers/nodecollector/collectorconfig/ownmetrics-ui.go:33-47)
NODE_KEYS = ["k8s.namespace.name", "k8s.deployment.name", "k8s.statefulset.name", "k8s.daemonset.name",
             "k8s.cronjob.name", "k8s.job.name", "k8s.pod.name", "k8s.node.name", "service.name"]


def _cfg(wl):
    if wl["cfg"] is not None:
        return wl["cfg"]
    from tests.workloads import c3_sampling_config
    if wl["gen"] == "fused":
        return {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
                "odigostrafficmetrics": {"res_attributes_keys": NODE_KEYS}}
    return {"odigossampling": c3_sampling_config()}


def algorithmic_bytes_fused(gen, db, n, cfg) -> int:
    """SURVEY.md §8(d) fused row: the union of the three stages' columns, each
    read once (trace_id, start, end, status, resource, route ref + compared
    route bytes, kind, url_flags, path ref + templated path bytes, span_size,
    scope, name_len; per scope 8 B, per resource 20 B) and each output written
    once (keep, url_out, tmpl ref + bytes, attribute-set counters)."""
    samp = algorithmic_bytes_sampling(gen, db, n, cfg)          # includes the 1 B keep
    url = algorithmic_bytes_url(gen, db, n)
    size = n * (4 + 4 + 4) + gen.cols.n_scopes * 8 + gen.cols.n_resources * 12 + gen.cols.n_attrsets * 8
    return samp + url + size


def algorithmic_bytes_url(gen, db, n) -> int:
    """SURVEY.md §8(d) URL row: per span 8 B path ref + 1 B kind + 1 B url_flags
    read, 8 B template ref + 1 B url_out written; plus the path bytes of every
    span whose path is templatized (read) and the template bytes written."""
    url_out = db.out_numpy("url_out")[:n]
    path = gen.array("path").view(np.uint32).reshape(-1, 2)[:n]
    templ_read = int(path[(url_out & 1) != 0, 1].sum())
    return n * (8 + 1 + 1) + n * (8 + 1) + templ_read + db.used()


def algorithmic_bytes_sampling(gen, db, n, cfg) -> int:
    """SURVEY.md §8(d) sampling row: per span 16 B trace_id + 8 B start + 8 B
    end + 1 B status + 4 B resource + 8 B route ref read and 1 B keep written;
    per resource 8 B (res_svc, res_svc_str); plus min(len(route), longest
    rule route) route bytes per span that carries one."""
    rules = cfg["odigossampling"].get("endpoint_rules", []) + cfg["odigossampling"].get("service_rules", []) + \
        cfg["odigossampling"].get("global_rules", [])
    pmax = max([len(r["rule_details"].get("http_route", "")) for r in rules] + [0])
    route = gen.array("route").view(np.uint32).reshape(-1, 2)[:n]
    rb = int(np.minimum(route[:, 1], pmax).sum())
    return n * (16 + 8 + 8 + 1 + 4 + 8 + 1) + gen.cols.n_resources * 8 + rb


def cpu_baseline_url(gen, cfg, threads: int, budget_s: float = 12.0, calls: int = 1):
    """Oracle (oracle/url.c, -O3) on the same batch: `threads` pthreads over
    the whole batch, repeated until ~budget_s of wall time; plus one
    single-thread pass over a 1M-span prefix."""
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import UrlOracle
    orc = UrlOracle(cfg["odigosurltemplate"])
    ho = HostOutputs(gen.cols)
    n = gen.cols.n_spans
    reps, t0 = 0, time.perf_counter()
    while True:
        assert orc.process(gen.cols, ho.outs, threads) == 0
        reps += 1
        if time.perf_counter() - t0 > budget_s / 2 or reps >= 50:
            break
    dt = time.perf_counter() - t0
    mt = n * reps / dt
    c1 = _prefix(gen.cols, 1_000_000)
    ho1 = HostOutputs(c1)
    t1 = time.perf_counter()
    assert orc.process(c1, ho1.outs, 1) == 0
    st = c1.n_spans / (time.perf_counter() - t1)
    sample = f"{n} spans (the same C2 batch) x {reps} passes, oracle/url.c -O3 pthreads"

    def parity(db):
        return (int(ho.used[0]) == db.used() and
                np.array_equal(ho.view("url_out", np.uint8)[:n], db.out_numpy("url_out")[:n]))
    return mt, st, sample, parity


def cpu_baseline_fused(gen, cfg, threads: int, budget_s: float = 12.0, calls: int = 1):
    """The three oracles chained in gateway order (sampling -> templating ->
    size; oracle/{sampling,url,size}.c -O3, pthreads for the first two) on a
    2M-span prefix of the same batch, repeated to ~budget_s/2.  Parity: keep,
    url_out and the attribute-set counters of the full batch."""
    from odigos_amd import native
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import SamplingOracle, UrlOracle, size_process
    so, uo = SamplingOracle(cfg["odigossampling"]), UrlOracle(cfg["odigosurltemplate"])
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE

    def chain(cols, nt):
        ho = HostOutputs(cols)
        assert so.process(cols, ho.outs, native.GROUP_TRACE_ID, 0x5EED, nt) == 0
        assert uo.process(cols, ho.outs, nt) == 0
        assert size_process(cols, ho.outs, st, native.GROUP_TRACE_ID, ho.outs, 1, 1.0, 0.0) == 0
        return ho
    n = gen.cols.n_spans
    c2 = _prefix(gen.cols, min(n, 2_000_000))
    reps, t0 = 0, time.perf_counter()
    while True:
        chain(c2, threads)
        reps += 1
        if time.perf_counter() - t0 > budget_s / 2 or reps >= 20:
            break
    mt = c2.n_spans * reps / (time.perf_counter() - t0)
    c1 = _prefix(gen.cols, min(n, 500_000))
    t1 = time.perf_counter()
    chain(c1, 1)
    st1 = c1.n_spans / (time.perf_counter() - t1)
    sample = f"{c2.n_spans}-span prefix of the C4 shard x {reps} passes, oracle/{{sampling,url,size}}.c -O3"

    def parity(db):
        ho = chain(gen.cols, threads)
        A = gen.cols.n_attrsets
        return bool(np.array_equal(ho.view("keep", np.uint8)[:n], db.out_numpy("keep")[:n]) and
                    np.array_equal(ho.view("url_out", np.uint8)[:n], db.out_numpy("url_out")[:n]) and
                    # the device counters were ADDED to by every timed and warm-up call
                    np.array_equal(calls * ho.view("attrset_bytes", np.int64)[:A],
                                   db.out_numpy("attrset_bytes", np.int64)[:A]))
    return mt, st1, sample, parity


def cpu_baseline_sampling(gen, cfg, threads: int, budget_s: float = 12.0, calls: int = 1):
    """Oracle (oracle/sampling.c, -O3: trace_id grouping + per-trace rule
    fold) on a 5M-span prefix of the same batch, `threads` pthreads for the
    fold, repeated to ~budget_s/2; plus a single-thread pass over 1M spans.
    Parity: the full batch's keep column against the GPU's."""
    from odigos_amd import native
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import SamplingOracle
    orc = SamplingOracle(cfg["odigossampling"])
    n = gen.cols.n_spans
    c5 = _prefix(gen.cols, min(n, 5_000_000))
    ho5 = HostOutputs(c5)
    reps, t0 = 0, time.perf_counter()
    while True:
        assert orc.process(c5, ho5.outs, native.GROUP_TRACE_ID, 0x5EED, threads) == 0
        reps += 1
        if time.perf_counter() - t0 > budget_s / 2 or reps >= 20:
            break
    mt = c5.n_spans * reps / (time.perf_counter() - t0)
    c1 = _prefix(gen.cols, min(n, 1_000_000))
    ho1 = HostOutputs(c1)
    t1 = time.perf_counter()
    assert orc.process(c1, ho1.outs, native.GROUP_TRACE_ID, 0x5EED, 1) == 0
    st = c1.n_spans / (time.perf_counter() - t1)
    sample = f"{c5.n_spans}-span prefix of the same batch x {reps} passes, oracle/sampling.c -O3 pthreads"

    def parity(db):
        ho = HostOutputs(gen.cols)
        assert orc.process(gen.cols, ho.outs, native.GROUP_TRACE_ID, 0x5EED, threads) == 0
        return bool(np.array_equal(ho.view("keep", np.uint8)[:n], db.out_numpy("keep")[:n]))
    return mt, st, sample, parity


def _prefix(cols, k):
    import ctypes as C
    from odigos_amd import native
    c1 = native.Columns()
    C.memmove(C.addressof(c1), C.addressof(cols), C.sizeof(native.Columns))
    c1.n_spans = min(cols.n_spans, k)
    return c1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # default: the whole hot path (C4 shard), which is also the configuration the
    # multi-GPU runs exercise (trace-id exchange when N > 1); DESIGN.md §6
    ap.add_argument("--workload", default="fused", choices=sorted(WORKLOADS))
    ap.add_argument("--spans", type=int, default=0, help="override spans per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
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
    n_spans = args.spans or wl["spans"]
    stages = 0
    for s in wl["stages"].split("|"):
        stages |= getattr(native, "STAGE_" + s)
    cfg = _cfg(wl)
    gen = Generator(wl["gen"], seed=wl["seed"] + rank, n_spans=n_spans, threads=16)
    for f in wl.get("null_columns", ()):
        setattr(gen.cols, f, None)   # columns the configured processors do not read
    eng = Engine(cfg)
    db = DeviceBatch(gen.cols, fields=wl.get("fields"))
    for f in wl.get("null_outputs", ()):
        setattr(db.outs, f, None)    # outputs the shim does not read (per-trace diagnostics)
    eng.reserve(n_spans)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    group = getattr(native, "GROUP_" + wl["group"])

    if world > 1 and stages & native.STAGE_SAMPLE:
        # route every span's sampling record to its trace's owner
        # GPU (RCCL all-to-all), decide there, bring keep back, then template
        # and size locally on the decisions
        from odigos_amd.exchange import DeviceExchange, route_and_sample
        ex = DeviceExchange(eng, db, stream=sh)
        local = (stages & ~native.STAGE_SAMPLE) | native.STAGE_APPLY_KEEP

        def step():
            route_and_sample(ex, world)
            if local & (native.STAGE_TEMPLATE | native.STAGE_SIZE):
                eng.process_device(db, local, group, seed=0x5EED, stream=sh)
    else:
        def step():
            eng.process_device(db, stages, group, seed=0x5EED, stream=sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.profile(False)
    prof = eng.profile_read()
    status = int(db.out_numpy("device_status", np.uint32)[0])
    if status:
        raise SystemExit(f"device status {status}: kernel reported a failure")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if args.workload == "url":
        b_alg = algorithmic_bytes_url(gen, db, n_spans)
    elif args.workload == "fused":
        b_alg = algorithmic_bytes_fused(gen, db, n_spans, cfg)
    else:
        b_alg = algorithmic_bytes_sampling(gen, db, n_spans, cfg)
    knames = wl["kernels"]
    per_k = {}
    for kn in knames:
        k = prof.get(kn, {"launches": 0, "ms": 0.0})
        per_k[kn] = k["ms"] / max(k["launches"], 1)
    k_ms = sum(per_k.values())
    kname = "+".join(knames)
    achieved = b_alg / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0

    traffic = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            d = json.loads(tj.read_text())
            ent = d.get(args.workload, {}).get(kname)
            if ent and ent.get("spans") == n_spans:
                traffic = ent["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    total_spans = n_spans * world * args.steps
    value = total_spans / elapsed
    out = {
        "metric": "spans/sec processed (whole node) at 1/2/4/8 MI355X; % of HBM roofline",
        "value": value,
        "unit": "spans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, SURVEY.md §8d mix)",
        "config": {"workload": wl["metric_config"], "spans_per_gpu": n_spans, "seed": wl["seed"],
                   "processors": list(cfg.keys()),
                   "parallelism": (f"dp{world}: trace-id all-to-all (RCCL) of sampling records, local templating/size"
                                   if world > 1 and stages & native.STAGE_SAMPLE else
                                   f"dp{world}: independent span shards, no data-path collective")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "kernel_ms": k_ms, "kernel_ms_each": per_k,
                     "algorithmic_bytes_per_launch": b_alg},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        fn = {"url": cpu_baseline_url, "sampling": cpu_baseline_sampling, "zipf": cpu_baseline_sampling,
              "fused": cpu_baseline_fused}[args.workload]
        mt, st, sample, parity = fn(gen, cfg, threads, calls=args.steps + args.warmup)
        out["cpu_baseline"] = {"value": mt, "unit": "spans/s", "cores": threads, "kind": "port",
                               "sample": sample, "value_1core": st}
        # the CPU pass doubles as a parity spot-check of the timed GPU output
        out["parity_vs_oracle"] = bool(parity(db))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
