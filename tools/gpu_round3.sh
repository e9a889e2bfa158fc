#!/bin/bash
# GPU pass: full GPU suite, smoke, default bench line, rocprof kernel stats of
# the default bench.  Every step time-limited; stops at the first failure.
# usage: bash tools/gpu_round3.sh <tag> [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" $OUT/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 "$@" > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"parity_vs_oracle": [a-z]*\|"kernel_ms_each": {[^}]*}' $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ks -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name "*.db" | head -1)
if [ -n "$db" ]; then python3 $R/tools/rocpd_stats.py $db $OUT/kernel_stats.csv > /dev/null && head -14 $OUT/kernel_stats.csv; fi
