"""Phases of one decode -> stages -> encode call chain over a message of k
concatenated 8192-span requests (the OTLP pipeline's batches), k = 1..16:
where a batch's time goes (diagnostic for odigos_amd/csrc/otlp_pipeline.cpp)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from odigos_amd import native
    from odigos_amd.batch import Engine, Generator, OtlpBatch, PinnedBuffer, device_outputs
    from tests.test_otlp_pipeline import _cfg, _router
    eng, router = Engine(_cfg()), _router()
    st = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE
    reqs = [Generator("fused", seed=0x0D16F0B0 + k, n_spans=8192, threads=4).otlp(4) for k in range(16)]
    sh = torch.cuda.current_stream().cuda_stream
    out = []
    for k in (1, 2, 4, 8, 16):
        msg = b"".join(reqs[:k])
        pin = PinnedBuffer(msg)
        dims = native.Columns()
        dims.n_spans, dims.n_resources, dims.n_attrsets = 8192 * k, 8192 * k, 4096
        outs = device_outputs(dims, tmpl_cap=64 * 8192 * k + len(msg))
        rows = []
        for rep in range(25):
            a = time.perf_counter()
            ob = OtlpBatch(eng, pin.p, stream=sh, length=pin.n, outputs=outs)
            b = time.perf_counter()
            eng.process_device(ob, st, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)
            torch.cuda.synchronize()
            c = time.perf_counter()
            ob.encode(st, native.GROUP_TRACE_ID, router, stream=sh, copy=False)
            d = time.perf_counter()
            if rep >= 5:
                rows.append({"decode": (b - a) * 1e3, "stages": (c - b) * 1e3, "encode": (d - c) * 1e3,
                             "phases": ob.timings_ms, "enc": ob.encode_ms})
            ob.close()
        med = lambda key: sorted(r[key] for r in rows)[len(rows) // 2]   # noqa: E731
        ph = {x: sorted(r["phases"][x] for r in rows)[len(rows) // 2] for x in rows[0]["phases"]}
        en = [sorted(r["enc"][j] for r in rows)[len(rows) // 2] for j in range(4)]
        line = {"requests": k, "bytes": len(msg), "decode_ms": med("decode"), "stages_ms": med("stages"),
                "encode_ms": med("encode"), "decode_phases_ms": ph, "encode_phases_ms": en,
                "spans_per_s": 8192 * k / ((med("decode") + med("stages") + med("encode")) / 1e3)}
        out.append(line)
        print(json.dumps(line), flush=True)
        pin.close()


if __name__ == "__main__":
    main()
