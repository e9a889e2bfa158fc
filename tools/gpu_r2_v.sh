#!/bin/bash
# fused URL plan+assemble: URL/fused GPU tests, smoke, C2 and C4 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_url_kats.py tests/test_url_random.py tests/test_size.py tests/test_sampling_random.py > gpurun_out/r2v_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r2v_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r2v_tests.log | head -30; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2v_smoke.log 2>&1 || { tail -20 gpurun_out/r2v_smoke.log; exit 1; }
tail -1 gpurun_out/r2v_smoke.log
timeout -k 10 300 python -u bench.py --workload url --steps 20 --warmup 5 > gpurun_out/r2v_bench_url.log 2>&1 || { tail -30 gpurun_out/r2v_bench_url.log; exit 1; }
grep '"metric"' gpurun_out/r2v_bench_url.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2v_bench_fused.log 2>&1 || { tail -30 gpurun_out/r2v_bench_fused.log; exit 1; }
grep '"metric"' gpurun_out/r2v_bench_fused.log
