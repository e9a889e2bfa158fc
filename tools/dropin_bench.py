"""End-to-end timing of the drop-in path (SURVEY.md §8d "drop-in" figure;
VERDICT r1 item 7): what a collector pays per ConsumeTraces when the
processors call the C ABI instead of running in Go.

Legs (one JSON line on stdout, also written to --out):

  consume_per_trace   odigossampling, OSE_GROUP_BATCH: one trace per call,
                      as groupbytrace delivers (groupbytrace.go:3-9), from
                      1 / 8 / 16 caller threads on one processor.  Each call is
                      the C++ host mirror's ProcessTraces: columnarise pdata
                      -> fill the pinned batch -> ose_process (H2D + kernels +
                      D2H) -> read back -> apply (host.cpp).
  consume_batch       the three processors in gateway order ("pipeline"),
                      OSE_GROUP_TRACE_ID, 8192-span batches (the batch
                      processor's default send_batch_size) from 1 / 8 threads.
  process_pinned      ose_process alone on engine-owned pinned batches of the
                      C4 mix (1M / 10M / 50M spans): fill + H2D + kernels +
                      D2H, the PCIe-inclusive rate (never the bench `value`).
  copy_bandwidth      pinned H2D and D2H copy rate of 1 GiB (hipMemcpyAsync
                      through torch), the bound process_pinned runs against.

Synthetic pdata: services svc-00..svc-15 (the C3 rules name svc-00..13),
routes and paths of the generator's shape, ~1% error spans.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

WORDS = ["users", "orders", "items", "cart", "search", "auth", "files", "payments", "reviews", "stock"]


def _path(rng: random.Random) -> tuple[str, str]:
    v = rng.choice(["v1", "v2"])
    w = rng.choice(WORDS)
    r = rng.random()
    if r < 0.4:
        return f"/api/{v}/{w}/{rng.randrange(1, 10**9)}", f"/api/{v}/{w}/{{id}}"
    if r < 0.6:
        u = "%08x-%04x-4%03x-a%03x-%012x" % (rng.getrandbits(32), rng.getrandbits(16), rng.getrandbits(12),
                                             rng.getrandbits(12), rng.getrandbits(48))
        return f"/api/{v}/{w}/{u}/{rng.choice(WORDS)}", f"/api/{v}/{w}/{{id}}/x"
    return f"/api/{v}/{w}", f"/api/{v}/{w}"


def make_trace(rng: random.Random, n_spans: int, t0: int) -> list[dict]:
    """One trace as resource_spans over 1-3 services (OTLP/JSON dicts)."""
    from odigos_amd import host
    tid = "%032x" % rng.getrandbits(128)
    svcs = [rng.randrange(16) for _ in range(rng.randint(1, 3))]
    by_svc: dict[int, list] = {s: [] for s in svcs}
    for k in range(n_spans):
        s = svcs[k % len(svcs)]
        path, route = _path(rng)
        start = t0 + rng.randrange(0, 50_000_000)
        dur = int(rng.expovariate(1 / 40e6))
        kind = 2 if k % 2 == 0 else 3
        attrs = {"http.request.method": rng.choice(["GET", "POST"]), "url.path": path}
        if rng.random() < 0.7:
            attrs["http.route"] = route
        by_svc[s].append(host.span(name="op", kind=kind, attributes=attrs, trace_id=tid,
                                   span_id="%016x" % rng.getrandbits(64), start=start, end=start + dur,
                                   status=2 if rng.random() < 0.01 else 0))
    return [host.resource_spans({"service.name": f"svc-{s:02d}", "k8s.namespace.name": "default",
                                 "k8s.pod.name": f"pod-{s}"}, spans) for s, spans in by_svc.items() if spans]


def per_trace_items(n_traces: int, seed: int) -> list[dict]:
    from odigos_amd import host
    rng = random.Random(seed)
    return [host.traces(*make_trace(rng, max(1, min(60, int(rng.expovariate(1 / 9)) + 1)), 1_700_000_000_000_000_000))
            for _ in range(n_traces)]


def batch_items(n_batches: int, spans_per_batch: int, seed: int) -> list[dict]:
    from odigos_amd import host
    rng = random.Random(seed)
    out = []
    for _ in range(n_batches):
        rs, n = [], 0
        while n < spans_per_batch:
            k = min(spans_per_batch - n, max(1, int(rng.expovariate(1 / 9)) + 1))
            rs.extend(make_trace(rng, k, 1_700_000_000_000_000_000))
            n += k
        out.append(host.traces(*rs))
    return out


def consume_leg(ptype: str, cfg: dict, group_mode: int, items: list[dict], threads: int, reps: int) -> dict:
    from odigos_amd import host, native
    p = host.Processor(ptype, cfg)
    p.configure(group_mode=group_mode)
    L = native.lib()
    payload = host.dumps(items).encode()
    out = (C.c_double * 12)()
    # warm-up: engine creation, first allocations
    rc = L.osehost_bench(p.h, host.dumps(items[: max(threads, 1)]).encode(), 1, threads, out)
    if rc:
        raise native.OseError(rc, (L.osehost_last_error() or b"").decode())
    rc = L.osehost_bench(p.h, payload, reps, threads, out)
    if rc:
        raise native.OseError(rc, (L.osehost_last_error() or b"").decode())
    wall, calls, spans = out[0], out[1], out[2]
    ph = dict(zip(("columnarize", "fill", "ose_process", "readback", "apply"), out[3:8]))
    p.close()
    return {"threads": threads, "calls": int(calls), "spans": int(spans), "wall_s": wall,
            "calls_per_s": calls / wall, "spans_per_s": spans / wall,
            "latency_us": {"p50": out[8] * 1e6, "p90": out[9] * 1e6, "p99": out[10] * 1e6, "max": out[11] * 1e6},
            "phase_us_per_call": {k: v / calls * 1e6 for k, v in ph.items()}}


def process_leg(n_spans: int, reps: int, threads: int) -> dict:
    from odigos_amd import native
    from odigos_amd.batch import Engine, Generator, PinnedBatch
    from tests.workloads import c3_sampling_config
    sys.path.insert(0, str(ROOT))
    from bench import NODE_KEYS
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": NODE_KEYS}}
    eng = Engine(cfg)
    g = Generator("fused", seed=0x0D160001, n_spans=n_spans, threads=threads)
    b = PinnedBatch(eng, g.cols)
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    b.fill(g.cols)
    b.cols.res_url_ok = None   # no include/exclude configured
    for f in ("trace_count", "trace_first_span", "trace_keep", "trace_level", "trace_ratio", "res_bytes"):
        setattr(b.outs, f, None)   # outputs the shim does not read
    b.process(st)   # warm-up (workspace, tables)
    t_fill = t_proc = 0.0
    for _ in range(reps):
        a = time.perf_counter()
        b.fill(g.cols)
        m = time.perf_counter()
        b.process(st)
        t_fill += m - a
        t_proc += time.perf_counter() - m
    in_bytes = sum(getattr(g.cols, "n_spans") * sz for f, sz in
                   (("trace_id", 16), ("start_ns", 8), ("end_ns", 8), ("status", 1), ("kind", 1), ("resource", 4),
                    ("scope", 4), ("url_flags", 1), ("path", 8), ("route", 8), ("span_size", 4), ("name_len", 4),
                    ("attr_match", 8))) + g.cols.arena_bytes
    b.close()
    return {"spans": n_spans, "reps": reps, "fill_ms": t_fill / reps * 1e3, "ose_process_ms": t_proc / reps * 1e3,
            "spans_per_s_process": n_spans * reps / t_proc, "spans_per_s_fill_process": n_spans * reps / (t_fill + t_proc),
            "h2d_bytes": in_bytes}


def copy_leg(nbytes: int = 1 << 30) -> dict:
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        d.copy_(h, non_blocking=True)
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        a = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        res[name + "_GBps"] = 5 * nbytes / (time.perf_counter() - a) / 1e9
    return res


def main():
    from odigos_amd import native
    from tests.workloads import c3_sampling_config
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "dropin.json"))
    ap.add_argument("--traces", type=int, default=4096)
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--process-spans", default="1000000,10000000,50000000")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--batch-only", action="store_true", help="only the 8192-span pipeline leg (and its parity)")
    args = ap.parse_args()
    sys.path.insert(0, str(ROOT))
    from bench import NODE_KEYS, cpu_share
    share, nproc, model = cpu_share()
    res = {"metric": "drop-in ConsumeTraces end to end (C ABI, pinned H2D + kernels + D2H + apply)",
           "host_cpu": model, "cpu_share": share, "nproc": nproc}
    t = time.perf_counter()
    pt = per_trace_items(args.traces, 0x0D16D001) if not args.batch_only else []
    res["consume_per_trace"] = []
    for th in (() if args.batch_only else (1, 8) if args.quick else (1, 8, 16)):
        res["consume_per_trace"].append(consume_leg("odigossampling", c3_sampling_config(), native.GROUP_BATCH, pt, th, 2))
        print(f"per-trace threads={th} {time.perf_counter() - t:.1f}s {res['consume_per_trace'][-1]}", flush=True)
    pipe = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
            "odigostrafficmetrics": {"res_attributes_keys": NODE_KEYS}}
    bi = batch_items(args.batches, 8192, 0x0D16D002)
    # (the same 8192-span pipeline calls are checked against the oracle by
    # tests/test_dropin_parity.py in the GPU suite)
    res["consume_batch"] = []
    for th in (1, 8):
        res["consume_batch"].append(consume_leg("pipeline", pipe, native.GROUP_TRACE_ID, bi, th, 2))
        print(f"batch threads={th} {time.perf_counter() - t:.1f}s {res['consume_batch'][-1]}", flush=True)
    res["process_pinned"] = []
    for n in ([] if args.batch_only else args.process_spans.split(",")):
        if n:
            res["process_pinned"].append(process_leg(int(n), 3, max(1, min(16, share))))
            print(f"process {n} {time.perf_counter() - t:.1f}s {res['process_pinned'][-1]}", flush=True)
    res["copy_bandwidth"] = copy_leg()
    line = json.dumps(res)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(line + "\n")
    print(line, flush=True)


if __name__ == "__main__":
    main()
