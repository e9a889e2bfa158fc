#!/bin/bash
# url_plan A/B (class order, group-sum scan, speculative classify reads) on
# C4, then the HBM traffic of the fused workload (PMC, separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab.sh r3k_ab _nocls6,_nosum,_spec fused || exit 1
bash tools/pmc_traffic.sh fused || exit 1
