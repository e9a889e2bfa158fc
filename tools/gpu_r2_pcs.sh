#!/bin/bash
# PC sampling (rocprofv3 beta, stochastic) of the URL plan kernel on C4's mix, 2M spans
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pcs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --kernel-trace --output-format csv -d $R/gpurun_out/pcs/run -o pcs -- python3 $R/bench.py --workload url --spans 2000000 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/pcs/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 $R/gpurun_out/pcs/run.log; ls -la $R/gpurun_out/pcs/run/* 2>/dev/null | head
exit 0
