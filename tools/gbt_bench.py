"""GPU-resident groupbytrace in steady state on one GPU:
a C4-mix batch of --spans spans arrives every simulated second (fresh trace
ids each time), wait_duration 30 s, so each call adds one batch and, after
the first 30, releases the traces of the batch added 30 s earlier; the
three processors then run on the release (OSE_GROUP_TRACE_ID).  Wall time
per leg with device syncs; one JSON line on stdout and in --out.  Not a
bench.py `value`.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spans", type=int, default=2_000_000)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "gbt.json"))
    args = ap.parse_args()
    import torch
    from bench import NODE_KEYS, cpu_share
    from odigos_amd import native
    from odigos_amd.batch import DeviceBatch, DeviceView, Engine, Generator, GroupByTrace
    from tests.workloads import c3_sampling_config
    share, nproc, model = cpu_share()
    g = Generator("fused", seed=0x6B70001, n_spans=args.spans, threads=max(1, min(16, share)))
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": NODE_KEYS}}
    eng = Engine(cfg)
    db = DeviceBatch(g.cols)
    tid = db.t["trace_id"][: 16 * args.spans].view(torch.int64)
    hold = 32 * args.spans
    # num_traces sized for the stream (contrib's default 1,000,000 would evict
    # traces at this rate: 30 s of batches hold ~6M traces)
    store = GroupByTrace(eng, {"wait_duration": "30s", "num_traces": 16_000_000}, hold, hold * 48)
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    legs = []
    S = 1_000_000_000
    for step in range(args.steps):
        tid.bitwise_xor_(step * 0x9E3779B97F4A7C15 & 0x7FFFFFFFFFFFFFFF if step else 0)
        torch.cuda.synchronize()
        a = time.perf_counter()
        store.add(db.cols, step * S)
        torch.cuda.synchronize()
        b = time.perf_counter()
        rel, ntr = store.release(step * S)
        torch.cuda.synchronize()
        c = time.perf_counter()
        rel_ms = (c - b) * 1e3
        if rel.n_spans:
            view = DeviceView(rel)   # outputs for this release (allocation not timed)
            torch.cuda.synchronize()
            c = time.perf_counter()
            eng.process_device(view, st, native.GROUP_TRACE_ID, seed=step)
            torch.cuda.synchronize()
        d = time.perf_counter()
        legs.append({"step": step, "add_ms": (b - a) * 1e3, "release_ms": rel_ms, "stages_ms": (d - c) * 1e3,
                     "released_spans": rel.n_spans, "released_traces": ntr})
        print(json.dumps(legs[-1]), flush=True)
    steady = [x for x in legs if x["released_spans"]]
    med = lambda k: sorted(x[k] for x in steady)[len(steady) // 2]  # noqa: E731
    res = {"metric": "groupbytrace store: steady-state add + release (+ stages) per batch", "spans_per_batch": args.spans,
           "wait_duration_s": 30, "num_traces": 16_000_000, "held_spans": store.stats()["held_spans"], "steady_steps": len(steady),
           "add_ms": med("add_ms"), "release_ms": med("release_ms"), "stages_ms": med("stages_ms"),
           "store_spans_per_s": args.spans / ((med("add_ms") + med("release_ms")) * 1e-3),
           "with_stages_spans_per_s": args.spans / ((med("add_ms") + med("release_ms") + med("stages_ms")) * 1e-3),
           "stats": store.stats(), "host_cpu": model}
    line = json.dumps(res)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(line + "\n")
    print(line, flush=True)


if __name__ == "__main__":
    main()
