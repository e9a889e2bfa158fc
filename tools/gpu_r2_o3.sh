#!/bin/bash
# OTLP walk with the next record's resource lines prefetched: OTLP tests + ingest bench (two runs)
set -o pipefail
mkdir -p gpurun_out/o3
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_otlp.py > gpurun_out/o3/tests.log 2>&1 || { tail -30 gpurun_out/o3/tests.log; exit 1; }
tail -1 gpurun_out/o3/tests.log
for r in 1 2; do
timeout -k 10 500 python -u tools/otlp_bench.py --spans 10000000 --reps 4 --out gpurun_out/o3/otlp_$r.json > gpurun_out/o3/otlp_$r.log 2>&1 || { tail -30 gpurun_out/o3/otlp_$r.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/o3/otlp_$r.json'));print(d['decode_pinned_ms'], d['decode_phases_ms'], d['end_to_end_with_encode_spans_per_s'])"
done
