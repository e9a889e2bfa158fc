#!/bin/bash
# GPU pass: the GPU test suite (or the tests named by $TESTS), smoke, then the
# bench lines of the given workloads.  Every step time-limited; stops at the
# first failure.  usage: bash tools/gpu_check.sh <tag> [workload...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-chk}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" $OUT/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for wl in "$@"; do
  timeout -k 10 600 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$wl.log 2>&1 || { tail -30 $OUT/bench_$wl.log; exit 1; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"parity_vs_oracle": [a-z]*\|"projected_ms_per_gpu_step": [0-9.]*' $OUT/bench_$wl.log | tr '\n' ' ')"
  grep -o '"parity": {[^}]*}' $OUT/bench_$wl.log || true
  grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$wl.log || true
done
