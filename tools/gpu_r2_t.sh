#!/bin/bash
# round 2 re-entry: full GPU suite, then the C4 bench (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
export OSE_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2t_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r2t_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r2t_pytest.log | head -20; exit $rc; fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2t_bench.log 2>&1 || { tail -30 gpurun_out/r2t_bench.log; exit 1; }
grep '"metric"' gpurun_out/r2t_bench.log
