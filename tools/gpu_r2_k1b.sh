#!/bin/bash
# url_plan_slow_kernel diagnostics: slowest block clocks and group counts (C2, C4 mixes)
set -o pipefail
mkdir -p gpurun_out/k1b
timeout -k 10 200 python3 -u tools/url_clocks.py 10000000 > gpurun_out/k1b/clocks_c2.log 2>&1 || { tail -20 gpurun_out/k1b/clocks_c2.log; exit 1; }
OSE_CLOCKS_WORKLOAD=fused timeout -k 10 200 python3 -u tools/url_clocks.py 20000000 > gpurun_out/k1b/clocks_c4.log 2>&1 || { tail -20 gpurun_out/k1b/clocks_c4.log; exit 1; }
head -5 gpurun_out/k1b/clocks_c2.log; head -5 gpurun_out/k1b/clocks_c4.log
