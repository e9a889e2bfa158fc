#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
OSE_CLOCKS_WORKLOAD=fused timeout -k 10 200 python -u tools/url_clocks.py 10000000 > gpurun_out/r2q_clocks_c4.log 2>&1 || { tail -30 gpurun_out/r2q_clocks_c4.log; exit 1; }
timeout -k 10 200 python -u tools/url_clocks.py 10000000 > gpurun_out/r2q_clocks_c2.log 2>&1 || { tail -30 gpurun_out/r2q_clocks_c2.log; exit 1; }
cat gpurun_out/r2q_clocks_c4.log gpurun_out/r2q_clocks_c2.log
