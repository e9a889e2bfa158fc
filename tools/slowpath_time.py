"""Time the SAMPLE stage on a batch whose traces are split into several runs
(the sort-based path), e.g. the owner's view after the trace-id exchange."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from odigos_amd import native
from odigos_amd.batch import DeviceBatch, Engine, Generator
from tests.workloads import c3_sampling_config

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
for shuffle in (False, True):
    g = Generator("sampling", 0x0D160003, n, threads=16, shuffle=shuffle)
    eng = Engine({"odigossampling": c3_sampling_config()})
    db = DeviceBatch(g.cols, fields=("arena", "trace_id", "start_ns", "end_ns", "status", "resource", "route", "res_svc", "res_svc_str"))
    for f in ("trace_count", "trace_first_span", "trace_keep", "trace_level", "trace_ratio"):
        setattr(db.outs, f, None)
    sh = torch.cuda.current_stream().cuda_stream
    eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        eng.process_device(db, native.STAGE_SAMPLE, native.GROUP_TRACE_ID, seed=0x5EED, stream=sh)
    e.record()
    torch.cuda.synchronize()
    print(f"shuffle={shuffle} n={n}: {s.elapsed_time(e) / 5:.3f} ms per SAMPLE call", flush=True)
