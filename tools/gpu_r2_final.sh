#!/bin/bash
# round-2 closing pass: full GPU suite, smoke, kernel stats of C4, bench lines of every workload
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/final
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/final/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/final/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/prof -o ks -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $R/gpurun_out/final/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/final/prof.log; exit 1; }
db=$(find $R/gpurun_out/final/prof -name "*.db" | head -1)
python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/final/fused_kernel_stats.csv > /dev/null
cd $R
for wl in fused url sampling zipf owner; do
  st=20; wu=5; if [ $wl = owner ]; then st=10; wu=3; fi
  timeout -k 10 500 python -u bench.py --workload $wl --steps $st --warmup $wu > gpurun_out/final/bench_$wl.log 2>&1 || { tail -30 gpurun_out/final/bench_$wl.log; exit 1; }
  echo "== $wl $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/final/bench_$wl.log) $(grep -o '"frac": [0-9.]*' gpurun_out/final/bench_$wl.log) $(grep -o '"parity_vs_oracle": [a-z]*' gpurun_out/final/bench_$wl.log)"
done
