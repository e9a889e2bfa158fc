#!/bin/bash
# round-4 closing pass (after the one-pass rule chunks): GPU suite, smoke, the driver's default bench line
# (cpu baseline included), every other workload's line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/${TAG:-r4zz}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_default.log 2>&1 || { tail -30 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log | cut -c1-400
for wl in url sampling zipf owner node8 sampling_wide; do
  timeout -k 10 600 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$wl.log 2>&1 || { tail -30 $OUT/bench_$wl.log; exit 1; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"parity_vs_oracle": [a-z]*\|"projected_ms_per_gpu_step": [0-9.]*' $OUT/bench_$wl.log | tr '\n' ' ')"
done
# rocprof kernel stats of the sampling_wide line (the one-pass chunk kernel)
mkdir -p $OUT/wide
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/wide -o wide -- python3 $R/bench.py --workload sampling_wide --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/wide_prof.log 2>&1 || { tail -20 $OUT/wide_prof.log; exit 1; }
cd $R
f=$(ls $OUT/wide/*/*results.db $OUT/wide/*results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/wide_kernel_stats.csv > /dev/null
head -4 $OUT/wide_kernel_stats.csv | cut -d, -f1-4
