"""Per-section shader-clock breakdown of the URL kernels (diagnostic;
OSE_URL_ABLATE bit 512 makes the engine print the per-wave sums)."""
import os, sys
import os
os.environ.setdefault("OSE_LIB_VARIANT", "_diag")   # the diagnostics build (OSE_DIAG=1) reads the ablation switches
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from odigos_amd import native
from odigos_amd.batch import DeviceBatch, Engine, Generator

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
wl = os.environ.get("OSE_CLOCKS_WORKLOAD", "url")   # "url" (C2) or "fused" (C4's mix)
g = Generator(wl, 0x0D160002, n, threads=16)
g.cols.res_url_ok = None
eng = Engine({"odigosurltemplate": {}})
db = DeviceBatch(g.cols, fields=("arena", "kind", "url_flags", "path"))
sh = torch.cuda.current_stream().cuda_stream
extra = [int(x, 0) for x in sys.argv[2:]] or [8 | 16 | 32 | 64]
for ab in [512] + [512 | x for x in extra]:
    os.environ["OSE_URL_ABLATE"] = str(ab)
    eng.process_device(db, native.STAGE_TEMPLATE, stream=sh)
    torch.cuda.synchronize()
    print("ablate", ab, flush=True)
