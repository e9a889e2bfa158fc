#!/usr/bin/env python3
"""bench.py — spans/sec of the Odigos gateway hot path on MI355X.

One "step" = one pass of the configured processors over one device-resident
synthetic batch (BASELINE.json configs; seeds from SURVEY.md §8d).  With
--gpus N the driver launches one rank per GPU (torch.distributed.run); every
rank processes its own shard (weak scaling: the path partitions by trace,
SURVEY.md §8e), the timed region is bracketed by barrier + synchronize, and
the max over ranks is reported.  Rank 0 prints ONE JSON line.

Workloads (per GPU):
  url   C2  odigosurltemplate, 10M spans, default rules          (configs[1])
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
                cfg={"odigosurltemplate": {}}, stages="TEMPLATE",
                # no include/exclude configured: the shim passes res_url_ok = NULL
                null_columns=("res_url_ok",),
                fields=("arena", "kind", "url_flags", "path"),
                metric_config="C2: URL templatization only, 10M spans/GPU, C2 segment mix, default rules"),
}


def algorithmic_bytes_url(cols, url_out: np.ndarray, tmpl_used: int, gen) -> int:
    """SURVEY.md §8(d) URL row: per span 8 B path ref + 1 B kind + 1 B url_flags
    read, 8 B template ref + 1 B url_out written; plus the path bytes of every
    span whose path is templatized (read) and the template bytes written."""
    n = cols.n_spans
    path = gen.array("path").view(np.uint32).reshape(-1, 2)[:n]
    templ_read = int(path[(url_out & 1) != 0, 1].sum())
    return n * (8 + 1 + 1) + n * (8 + 1) + templ_read + tmpl_used


def cpu_baseline(gen, cfg_url, threads: int, budget_s: float = 12.0):
    """Oracle (oracle/url.c, -O3) on the same batch: `threads` pthreads over
    the whole batch, repeated until ~budget_s of wall time; plus one
    single-thread pass over a 1M-span prefix."""
    from odigos_amd.batch import HostOutputs
    from tests.oracle_lib import UrlOracle
    orc = UrlOracle(cfg_url)
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
    # single core on a bounded prefix
    import ctypes as C
    from odigos_amd import native
    c1 = native.Columns()
    C.memmove(C.addressof(c1), C.addressof(gen.cols), C.sizeof(native.Columns))
    c1.n_spans = min(n, 1_000_000)
    ho1 = HostOutputs(c1)
    t1 = time.perf_counter()
    assert orc.process(c1, ho1.outs, 1) == 0
    st = c1.n_spans / (time.perf_counter() - t1)
    return mt, st, reps, ho


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="url", choices=sorted(WORKLOADS))
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
    stages = getattr(native, "STAGE_" + wl["stages"])
    gen = Generator(wl["gen"], seed=wl["seed"] + rank, n_spans=n_spans, threads=16)
    for f in wl.get("null_columns", ()):
        setattr(gen.cols, f, None)   # columns the configured processors do not read
    eng = Engine(wl["cfg"])
    db = DeviceBatch(gen.cols, fields=wl.get("fields"))
    eng.reserve(n_spans)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def step():
        eng.process_device(db, stages, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)

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

    url_out = db.out_numpy("url_out")[:n_spans]
    used = db.used()
    b_alg = algorithmic_bytes_url(gen.cols, url_out, used, gen)
    # the URL stage is three launches (plan, scan, emit); the roofline is taken over their sum
    knames = ("url_plan_kernel", "url_scan_kernel", "url_emit_kernel")
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
                   "processors": list(wl["cfg"].keys()), "parallelism": f"trace-sharded x{world}, no data-path collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "kernel_ms": k_ms, "kernel_ms_each": per_k,
                     "algorithmic_bytes_per_launch": b_alg},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        mt, st, reps, ho = cpu_baseline(gen, wl["cfg"]["odigosurltemplate"], threads)
        # the CPU pass doubles as a parity spot-check of the timed GPU output
        parity = (int(ho.used[0]) == used and
                  np.array_equal(ho.view("url_out", np.uint8)[:n_spans], url_out))
        out["cpu_baseline"] = {"value": mt, "unit": "spans/s", "cores": threads, "kind": "port",
                               "sample": f"{n_spans} spans (the same C2 batch) x {reps} passes, oracle/url.c -O3 pthreads",
                               "value_1core": st}
        out["parity_vs_oracle"] = bool(parity)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
