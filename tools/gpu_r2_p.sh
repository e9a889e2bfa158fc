#!/bin/bash
# round 2: groupbytrace steady state
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gbt_bench.py --spans 2000000 --steps 40 --out gpurun_out/r2p_gbt.json > gpurun_out/r2p_gbt.log 2>&1 || { tail -30 gpurun_out/r2p_gbt.log; exit 1; }
tail -3 gpurun_out/r2p_gbt.log
