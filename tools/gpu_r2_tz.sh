#!/bin/bash
# PMC HBM traffic of C5 with the current URL kernels, then its bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_traffic.sh zipf || exit 1
python3 - <<'PY'
import json
t = json.load(open("profiles/pmc_traffic.json"))
t.update(json.load(open("gpurun_out/pmc_traffic_zipf.json")))
json.dump(t, open("gpurun_out/pmc_traffic_merged.json", "w"), indent=1)
PY
cp gpurun_out/pmc_traffic_merged.json profiles/pmc_traffic.json
timeout -k 10 500 python -u bench.py --workload zipf --steps 20 --warmup 5 > gpurun_out/bench_zipf_tz.log 2>&1 || { tail -30 gpurun_out/bench_zipf_tz.log; exit 1; }
grep '"metric"' gpurun_out/bench_zipf_tz.log | cut -c1-300
grep -o '"traffic": [0-9.a-z]*' gpurun_out/bench_zipf_tz.log
