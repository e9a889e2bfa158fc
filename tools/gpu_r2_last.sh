#!/bin/bash
# final check of the committed tree: full GPU suite, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out/last
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/last/pytest.log 2>&1
rc=$?
tail -2 gpurun_out/last/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/last/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1 || { tail -20 gpurun_out/last/smoke.log; exit 1; }
tail -1 gpurun_out/last/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/last/bench.log 2>&1 || { tail -30 gpurun_out/last/bench.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"traffic": [0-9.a-z]*\|"parity_vs_oracle": [a-z]*' gpurun_out/last/bench.log | tr '\n' ' '
