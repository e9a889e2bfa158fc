"""Ablation timings of trace_eval_kernel on the C3 batch (diagnostic).
Each variant sets OSE_TRACE_ABLATE (read per call by sampling_host.cpp)."""
import os, sys
import os
os.environ.setdefault("OSE_LIB_VARIANT", "_diag")   # the diagnostics build (OSE_DIAG=1) reads the ablation switches
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from odigos_amd import native
from odigos_amd.batch import DeviceBatch, Engine, Generator
from tests.workloads import c3_sampling_config

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
wl = os.environ.get("OSE_ABLATE_WORKLOAD", "sampling")   # "sampling" (C3) or "zipf" (C5)
g = Generator(wl, 0x0D160003 if wl == "sampling" else 0x0D160005, n, threads=16)
eng = Engine({"odigossampling": c3_sampling_config()})
db = DeviceBatch(g.cols, fields=("arena", "trace_id", "start_ns", "end_ns", "status", "resource", "route", "res_svc", "res_svc_str"))
for f in ("trace_count", "trace_first_span", "trace_keep", "trace_level", "trace_ratio"):
    setattr(db.outs, f, None)
sh = torch.cuda.current_stream().cuda_stream
eng.reserve(n)

def timeit(label, ablate, reps=5):
    os.environ["OSE_TRACE_ABLATE"] = str(ablate)
    eng.process_device(db, native.STAGE_SAMPLE, stream=sh)
    torch.cuda.synchronize()
    eng.profile(True)
    for _ in range(reps):
        eng.process_device(db, native.STAGE_SAMPLE, stream=sh)
    torch.cuda.synchronize()
    eng.profile(False)
    pr = eng.profile_read()["trace_eval_kernel"]
    print(f"{label:44s} {pr['ms'] / pr['launches']:9.3f} ms", flush=True)

timeit("C3 baseline (lean instance)", 0)
timeit("general instance (64: unused bit)", 64)
timeit("no table insert (1)", 1)
timeit("no latency scans (2)", 2)
timeit("no decide (4)", 4)
timeit("no endpoint prefix match (8)", 8)
timeit("no dependent service-id loads (16)", 16)
timeit("no route head reads (32)", 32)
timeit("no dependent loads (48)", 48)
timeit("none of them (63)", 63)
