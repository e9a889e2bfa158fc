#!/bin/bash
# diagnostics: URL per-section clocks on C4's mix, trace_eval ablations on C3
set -o pipefail
mkdir -p gpurun_out
OSE_CLOCKS_WORKLOAD=fused timeout -k 10 200 python -u tools/url_clocks.py 10000000 > gpurun_out/r2u_clocks_c4.log 2>&1 || { tail -30 gpurun_out/r2u_clocks_c4.log; exit 1; }
cat gpurun_out/r2u_clocks_c4.log
timeout -k 10 300 python -u tools/ablate_trace.py > gpurun_out/r2u_ablate_trace.log 2>&1 || { tail -30 gpurun_out/r2u_ablate_trace.log; exit 1; }
cat gpurun_out/r2u_ablate_trace.log
