#!/bin/bash
# PMC pass: HBM traffic (FETCH_SIZE / WRITE_SIZE) of the fused, url and
# sampling bench workloads, then the stall / issue counters of the C4 kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in fused url sampling; do
  bash tools/pmc_traffic.sh $wl || exit 1
done
bash tools/pmc_stall.sh 10000000 || exit 1
