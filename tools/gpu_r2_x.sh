#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ablate_trace.py > gpurun_out/r2x_ablate_trace.log 2>&1 || { tail -30 gpurun_out/r2x_ablate_trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2x_ablate_trace.log
