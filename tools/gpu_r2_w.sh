#!/bin/bash
# pipelined copy kernel: URL GPU tests, clocks on C4's mix, C2 and C4 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_url_kats.py tests/test_url_random.py > gpurun_out/r2w_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2w_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r2w_tests.log | head -30; exit $rc; fi
OSE_CLOCKS_WORKLOAD=fused timeout -k 10 200 python -u tools/url_clocks.py 10000000 > gpurun_out/r2w_clocks_c4.log 2>&1 || { tail -30 gpurun_out/r2w_clocks_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2w_clocks_c4.log
timeout -k 10 300 python -u bench.py --workload url --steps 20 --warmup 5 > gpurun_out/r2w_bench_url.log 2>&1 || { tail -30 gpurun_out/r2w_bench_url.log; exit 1; }
grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/r2w_bench_url.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2w_bench_fused.log 2>&1 || { tail -30 gpurun_out/r2w_bench_fused.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2w_bench_fused.log
grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/r2w_bench_fused.log
grep -o '"parity_vs_oracle": [a-z]*' gpurun_out/r2w_bench_fused.log
