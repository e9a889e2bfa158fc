#!/bin/bash
# round-2 profile pass: kernel stats (rocprofv3 --kernel-trace --stats) for C4 and C2,
# PMC HBM traffic for C4 and C2, then the C4 and C2 bench lines (picking the traffic up)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
for wl in fused url; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/$wl -o ks -- python3 $R/bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $R/gpurun_out/prof/$wl.log 2>&1 || { echo "rocprof $wl failed"; tail -20 $R/gpurun_out/prof/$wl.log; exit 1; }
  db=$(find $R/gpurun_out/prof/$wl -name "*.db" | head -1)
  if [ -n "$db" ]; then python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/prof/${wl}_kernel_stats.csv > /dev/null; fi
  ls $R/gpurun_out/prof/$wl
done
cd $R
for wl in fused url; do bash tools/pmc_traffic.sh $wl || exit 1; done
python3 - <<'PY'
import json
from pathlib import Path
R = Path(".")
t = json.load(open(R / "profiles/pmc_traffic.json"))
for wl in ("fused", "url"):
    t.update({k: v for k, v in json.load(open(R / f"gpurun_out/pmc_traffic_{wl}.json")).items()})
json.dump(t, open(R / "gpurun_out/pmc_traffic_merged.json", "w"), indent=1)
PY
cp gpurun_out/pmc_traffic_merged.json profiles/pmc_traffic.json
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/prof/bench_fused.log 2>&1 || { tail -30 gpurun_out/prof/bench_fused.log; exit 1; }
grep '"metric"' gpurun_out/prof/bench_fused.log
timeout -k 10 300 python -u bench.py --workload url --steps 20 --warmup 5 > gpurun_out/prof/bench_url.log 2>&1 || { tail -30 gpurun_out/prof/bench_url.log; exit 1; }
grep '"metric"' gpurun_out/prof/bench_url.log
