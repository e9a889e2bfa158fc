#!/bin/bash
# url_plan A/B of the class order and the group-sum scan, then the HBM
# traffic of the fused workload (PMC, separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab.sh r3k_ab _nocls6,_nosum,_r2 fused url || exit 1
bash tools/pmc_traffic.sh fused || exit 1
