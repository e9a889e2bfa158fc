"""OTLP protobuf ingest timed end to end on one GPU: a
serialized TracesData in host memory (the C4 mix as an HTTP instrumentation
would send it, odigos_amd/csrc/gen_otlp.cpp) → ose_otlp_decode (structural
walk on the host, H2D, the span decoder, the host pass) → the three stages
on the decoded columns.  PCIe-inclusive by construction: not a bench.py
`value`.  One JSON line on stdout and in --out.

Legs: decode from pinned memory (ose_host_alloc: a receiver reading into
engine buffers), decode from pageable memory, the stages after it, and the
output side (ose_otlp_encode: decisions D2H, routing to data-stream
pipelines, one TracesData per pipeline).
The span decoder's roofline: message bytes read + columns written per
launch over its HIP-event time, against 8 TB/s.
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
    ap.add_argument("--spans", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "otlp.json"))
    args = ap.parse_args()
    import torch
    from bench import NODE_KEYS, cpu_share
    from odigos_amd import native
    from odigos_amd.batch import Engine, Generator, OtlpBatch, PinnedBuffer, Router
    from tests.workloads import c3_sampling_config
    share, nproc, model = cpu_share()
    threads = max(1, min(16, share))
    t = time.perf_counter()
    g = Generator("fused", seed=0x0D16F0A1, n_spans=args.spans, threads=threads)
    pb = g.otlp(threads)
    print(f"generated {len(pb) / 1e9:.2f} GB for {args.spans} spans in {time.perf_counter() - t:.1f}s", flush=True)
    cfg = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
           "odigostrafficmetrics": {"res_attributes_keys": NODE_KEYS}}
    eng = Engine(cfg)
    pin = PinnedBuffer(pb)
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    sh = torch.cuda.current_stream().cuda_stream

    # outputs allocated once (the shim keeps its buffers); template arena 64 B/span
    from odigos_amd.batch import device_outputs
    dims = native.Columns()
    dims.n_spans, dims.n_resources, dims.n_attrsets = g.cols.n_spans, g.cols.n_resources, 4096
    outs = device_outputs(dims, tmpl_cap=64 * args.spans)
    phases = []

    # data streams over the generated services (k8s.deployment.name = svc-NN in
    # namespace default): two pipelines, one of them fed twice, the rest default
    streams = [{"name": "ds-a", "sources": [{"namespace": "default", "kind": "Deployment", "name": "svc-%02d" % k}
                                            for k in range(0, 12)],
                "destinations": [{"destinationname": "d1", "configuredsignals": ["TRACES"]}]},
               {"name": "ds-b", "sources": [{"namespace": "default", "kind": "Deployment", "name": "svc-%02d" % k}
                                            for k in range(8, 20)],
                "destinations": [{"destinationname": "d2", "configuredsignals": ["TRACES", "LOGS"]}]}]
    router = Router({"datastreams": streams})
    enc = []

    def one(pinned: bool, stages: bool):
        a = time.perf_counter()
        ob = (OtlpBatch(eng, pin.p, stream=sh, length=pin.n, outputs=outs) if pinned
              else OtlpBatch(eng, pb, stream=sh, outputs=outs))
        phases.append(ob.timings_ms)
        torch.cuda.synchronize()
        b = time.perf_counter()
        if stages:
            eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)
            torch.cuda.synchronize()
        c = time.perf_counter()
        if stages:
            out = ob.encode(st, native.GROUP_TRACE_ID, router, stream=sh, copy=False)
            enc.append((time.perf_counter() - c, out, ob.encode_ms))
        info = (ob.cols.n_spans, ob.host_spans, int(ob.out_numpy("device_status", n=1)[0]) if stages else 0)
        ob.close()
        return b - a, c - b, info

    for _ in range(2):
        one(True, True)
    res = {"metric": "OTLP protobuf ingest: host TracesData bytes -> decoded columns -> SAMPLE|TEMPLATE|SIZE",
           "spans": args.spans, "message_bytes": len(pb), "bytes_per_span": len(pb) / args.spans,
           "host_cpu": model, "cpu_share": share, "nproc": nproc}
    eng.profile(True)
    dec, stg = [], []
    for _ in range(args.reps):
        d, s, info = one(True, True)
        dec.append(d)
        stg.append(s)
        assert info[2] == 0, "device status"
    prof = eng.profile_read()
    eng.profile(False)
    n_dec = prof.get("otlp_span_kernel", {"ms": 0.0, "launches": 1})
    k_ms = n_dec["ms"] / max(n_dec["launches"], 1)
    stage_ms = sum(v["ms"] for k, v in prof.items() if k != "otlp_span_kernel") / args.reps
    dp = min(dec)
    res["decode_pinned_ms"] = dp * 1e3
    best = phases[2 + dec.index(dp)]
    res["decode_phases_ms"] = best
    res["stages_ms"] = min(stg) * 1e3
    res["stages_kernel_ms"] = stage_ms
    res["end_to_end_spans_per_s"] = args.spans / (dp + min(stg))
    res["decode_spans_per_s"] = args.spans / dp
    res["host_pass_spans"] = info[1]
    res["span_kernel_ms"] = k_ms
    e_best = min(enc[2:], key=lambda x: x[0])
    res["encode_ms"] = e_best[0] * 1e3
    res["encode_phases_ms"] = dict(zip(("decisions_d2h", "sizing", "buffers", "writing"), e_best[2]))
    res["encode_outputs"] = [{"pipeline": p, "bytes": nb, "resources": nr} for p, nb, nr in e_best[1]]
    out_bytes = sum(x["bytes"] for x in res["encode_outputs"])
    res["encode_out_GBps"] = out_bytes / e_best[0] / 1e9
    res["end_to_end_with_encode_spans_per_s"] = args.spans / (dp + min(stg) + e_best[0])
    # decoder roofline: the message bytes it reads + 60 B/span of columns (and flags) written
    alg = len(pb) + 8 * args.spans + 60 * args.spans
    res["span_kernel_roofline"] = {"bound": "hbm", "achieved": alg / (k_ms * 1e-3) / 1e9 if k_ms else 0.0,
                                   "peak": 8000.0, "unit": "GB/s", "algorithmic_bytes": alg}
    res["span_kernel_roofline"]["frac"] = res["span_kernel_roofline"]["achieved"] / 8000.0
    d, _, _ = one(False, False)
    res["decode_pageable_ms"] = d * 1e3
    # per-call latency at the batch processor's 8192 spans
    smallpb = Generator("fused", seed=0x0D16F0A2, n_spans=8192, threads=threads).otlp(threads)
    spin = PinnedBuffer(smallpb)
    sdims = native.Columns()
    sdims.n_spans, sdims.n_resources, sdims.n_attrsets = 8192, 8192, 4096
    souts = device_outputs(sdims, tmpl_cap=64 * 8192)
    lat, sph, leg = [], [], []
    for k in range(220):
        a = time.perf_counter()
        ob = OtlpBatch(eng, spin.p, stream=sh, length=spin.n, outputs=souts)
        sph.append(ob.timings_ms)
        b = time.perf_counter()
        eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)
        torch.cuda.synchronize()
        c = time.perf_counter()
        ob.encode(st, native.GROUP_TRACE_ID, router, stream=sh, copy=False)
        d = time.perf_counter()
        sph[-1].update({"enc_" + x: v for x, v in zip(("d2h", "sizing", "buffers", "writing"), ob.encode_ms)})
        ob.close()
        if k >= 20:
            lat.append(time.perf_counter() - a)
            leg.append(((b - a) * 1e3, (c - b) * 1e3, (d - c) * 1e3))
    lat.sort()
    res["batch8192_decode_stages_encode_us"] = {"p50": lat[len(lat) // 2] * 1e6, "p99": lat[int(len(lat) * 0.99)] * 1e6}
    res["batch8192_spans_per_s"] = 8192 / lat[len(lat) // 2]
    res["batch8192_legs_ms_median"] = {k: sorted(x[j] for x in leg)[len(leg) // 2]
                                       for j, k in enumerate(("decode", "stages", "encode"))}
    res["batch8192_decode_phases_ms_median"] = {k: sorted(x[k] for x in sph[20:])[len(sph[20:]) // 2] for k in sph[0]}
    # the same 8192-span request from several callers at once (a receiver's
    # concurrent export requests): one stream and one set of outputs per
    # caller, the engine and router shared; whole-job spans/s
    import threading
    for callers in (1, 4, 8, 16):
        per = 120
        ready = threading.Barrier(callers + 1)
        errs = []

        def caller(k):
            try:
                cs = torch.cuda.Stream()
                ch = cs.cuda_stream
                co = device_outputs(sdims, tmpl_cap=64 * 8192)
                ready.wait()
                for _ in range(per):
                    ob = OtlpBatch(eng, spin.p, stream=ch, length=spin.n, outputs=co)
                    eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=0x5EED, stream=ch)
                    ob.encode(st, native.GROUP_TRACE_ID, router, stream=ch, copy=False)
                    ob.close()
                cs.synchronize()
            except Exception as ex:   # pragma: no cover
                errs.append(repr(ex))

        th = [threading.Thread(target=caller, args=(k,)) for k in range(callers)]
        for t_ in th:
            t_.start()
        ready.wait()
        a = time.perf_counter()
        for t_ in th:
            t_.join()
        wall = time.perf_counter() - a
        assert not errs, errs
        res.setdefault("batch8192_callers", []).append(
            {"callers": callers, "calls": callers * per, "wall_s": wall,
             "spans_per_s": callers * per * 8192 / wall, "calls_per_s": callers * per / wall})
        print(f"otlp 8192-span calls, {callers} callers: {callers * per * 8192 / wall / 1e6:.1f} M spans/s", flush=True)
    # the same requests through ose_otlp_pipeline: concurrent callers'
    # requests coalesced into one device batch per wave of calls
    from odigos_amd.batch import OtlpPipeline
    pipe = OtlpPipeline(eng, router, st)
    import os
    if os.environ.get("OSE_PIPE_RUNNING"):   # diagnostics: the product defaults otherwise (4, 200 us, 8)
        pipe.tune(int(os.environ["OSE_PIPE_RUNNING"]), int(os.environ.get("OSE_PIPE_WINDOW_US", "200")),
                  int(os.environ.get("OSE_PIPE_TARGET", "8")))
    for callers in (1, 4, 8, 16):
        per = 150 if callers > 1 else 120
        ready = threading.Barrier(callers + 1)
        errs = []

        def pcaller(k):
            try:
                ready.wait()
                for _ in range(per):
                    pipe.consume(spin.p, spin.n, seed=0x5EED, copy=False)
            except Exception as ex:   # pragma: no cover
                errs.append(repr(ex))

        th = [threading.Thread(target=pcaller, args=(k,)) for k in range(callers)]
        for t_ in th:
            t_.start()
        pipe.counters()
        ready.wait()
        a = time.perf_counter()
        for t_ in th:
            t_.join()
        wall = time.perf_counter() - a
        assert not errs, errs
        cnt = pipe.counters()
        res.setdefault("pipeline8192_callers", []).append(
            {"callers": callers, "calls": callers * per, "wall_s": wall,
             "spans_per_s": callers * per * 8192 / wall, "calls_per_s": callers * per / wall,
             "batches": cnt["batches"], "largest_batch": cnt["largest_batch"], "alone": cnt["alone"],
             "batch_ms": cnt["batch_ms"]})
        print(f"otlp pipeline 8192-span requests, {callers} callers: {callers * per * 8192 / wall / 1e6:.1f} M spans/s "
              f"({cnt['batches']} batches, largest {cnt['largest_batch']}, alone {cnt['alone']}, ms {cnt['batch_ms']})", flush=True)
    pipe.close()
    spin.close()
    pin.close()
    line = json.dumps(res)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(line + "\n")
    print(line, flush=True)


if __name__ == "__main__":
    main()
