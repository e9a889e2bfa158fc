#!/bin/bash
# gathered LDS stage for groups whose byte range overflows it: URL + OTLP GPU tests, C2/C4/C5 benches, OTLP bench + kernel stats
set -o pipefail
mkdir -p gpurun_out/ga
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_url_kats.py tests/test_url_random.py tests/test_otlp.py tests/test_size.py tests/test_concurrency.py > gpurun_out/ga/tests.log 2>&1
rc=$?
tail -3 gpurun_out/ga/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/ga/tests.log | head -30; exit $rc; fi
for wl in url fused zipf; do
  timeout -k 10 500 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ga/bench_$wl.log 2>&1 || { tail -30 gpurun_out/ga/bench_$wl.log; exit 1; }
  echo "== $wl"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ga/bench_$wl.log; grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/ga/bench_$wl.log; grep -o '"parity_vs_oracle": [a-z]*' gpurun_out/ga/bench_$wl.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ga/otlp_prof -o otlp -- python3 tools/otlp_bench.py --spans 10000000 --reps 3 --out gpurun_out/ga/otlp.json > gpurun_out/ga/otlp.log 2>&1 || { tail -20 gpurun_out/ga/otlp.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ga/otlp.json')); print('otlp stages_ms', d['stages_ms'], 'kernel', d['stages_kernel_ms'])"
true
