#!/bin/bash
# OTLP ingest with the ResourceSpans level on the GPU: its tests, then the
# OTLP bench with and without it
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3g
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_otlp.py tests/test_router_encode.py tests/test_lifetime.py tests/test_concurrency.py tests/test_size.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u tools/otlp_bench.py --out $OUT/otlp_gpu_res.json > $OUT/otlp_gpu_res.log 2>&1 || { tail -30 $OUT/otlp_gpu_res.log; exit 1; }
OSE_OTLP_HOST_RESOURCES=1 timeout -k 10 400 python -u tools/otlp_bench.py --out $OUT/otlp_host_res.json > $OUT/otlp_host_res.log 2>&1 || { tail -30 $OUT/otlp_host_res.log; exit 1; }
python3 - <<'PY'
import json
for f in ("otlp_gpu_res", "otlp_host_res"):
    d = json.load(open(f"gpurun_out/r3g/{f}.json"))
    print(f, "decode_pinned_ms", round(d["decode_pinned_ms"], 2), {k: round(v, 2) for k, v in d["decode_phases_ms"].items()},
          "b8192 decode", round(d["batch8192_legs_ms_median"]["decode"], 3), d["batch8192_decode_phases_ms_median"])
PY
