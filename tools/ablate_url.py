"""Ablation timings of the URL kernels on synthetic C2 batches (diagnostic)."""
import sys, time
import os
os.environ.setdefault("OSE_LIB_VARIANT", "_diag")   # the diagnostics build (OSE_DIAG=1) reads the ablation switches
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np
import torch
from odigos_amd import native
from odigos_amd.batch import DeviceBatch, Engine, Generator

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
g = Generator("url", 0x0D160002, n, threads=16)
g.cols.res_url_ok = None
eng = Engine({"odigosurltemplate": {}})
db = DeviceBatch(g.cols, fields=("arena", "kind", "url_flags", "path"))
sh = torch.cuda.current_stream().cuda_stream

def timeit(label, reps=5):
    eng.process_device(db, native.STAGE_TEMPLATE, stream=sh)
    torch.cuda.synchronize()
    eng.profile(True)
    for _ in range(reps):
        eng.process_device(db, native.STAGE_TEMPLATE, stream=sh)
    torch.cuda.synchronize()
    eng.profile(False)
    pr = eng.profile_read()
    ms = {k: pr[k]["ms"] / pr[k]["launches"] for k in ("url_plan_kernel", "url_scan_kernel", "url_copy_kernel")}
    print(f"{label:40s} {sum(ms.values()):9.3f} ms  (plan {ms['url_plan_kernel']:.3f} scan {ms['url_scan_kernel']:.3f} copy {ms['url_copy_kernel']:.3f})", flush=True)

orig = db.t["url_flags"].clone()
timeit("C2 baseline")
db.t["url_flags"].zero_()
timeit("no method (skeleton only)")
db.t["url_flags"].copy_(orig)
k = db.t["kind"]; korig = k.clone()
k.fill_(1)
timeit("all internal kind (skeleton only)")
k.copy_(korig)
# only RAW path spans, short path "/"
p = db.t["path"].view(torch.int32).view(-1, 2)
porig = p.clone()
p[:, 1].clamp_(max=1)
timeit("paths truncated to 1 byte")
p.copy_(porig)
p[:, 1].clamp_(max=8)
timeit("paths truncated to 8 bytes")
p.copy_(porig)
timeit("C2 baseline again")
import os
for v, label in ((1, "skip emission"), (2, "skip planning"), (3, "skip planning+emission"), (7, "stage only (no bitmaps/plan/emit)"),
                 (1 | 8, "no emit, skip date"), (1 | 16, "no emit, skip email"), (1 | 32, "no emit, skip fffd"),
                 (1 | 64, "no emit, long segs cut to 64"), (1 | 8 | 16 | 32 | 64, "no emit, skip all rare"), (1 | 1024, "no emit, per-lane planner (no list)")):
    os.environ["OSE_URL_ABLATE"] = str(v)
    timeit(label)
os.environ.pop("OSE_URL_ABLATE")
