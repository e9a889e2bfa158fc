#!/bin/bash
# PMC HBM traffic of url, fused, zipf with the current kernels; OTLP ingest bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for wl in url fused zipf; do
  bash tools/pmc_traffic.sh $wl > gpurun_out/pmc_$wl.log 2>&1 || { tail -20 gpurun_out/pmc_$wl.log; exit 1; }
  echo "== $wl $(python3 -c "import json; d=json.load(open('gpurun_out/pmc_traffic_$wl.json')); print(d['hbm_bytes_per_launch'])")"
done
timeout -k 10 400 python3 -u tools/otlp_bench.py --spans 10000000 --reps 5 --out gpurun_out/otlp_r2d.json > gpurun_out/otlp_r2d.log 2>&1 || { tail -20 gpurun_out/otlp_r2d.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/otlp_r2d.json')); print('otlp stages_ms', d['stages_ms'], 'e2e', d['end_to_end_spans_per_s'])"
