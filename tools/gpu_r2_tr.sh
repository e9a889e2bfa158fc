#!/bin/bash
# URL clocks + slow/unplanned group counts (C2, C4 mixes), then PMC HBM traffic of url, fused, zipf
set -o pipefail
mkdir -p gpurun_out/tr
timeout -k 10 200 python3 -u tools/url_clocks.py 10000000 > gpurun_out/tr/clocks_c2.log 2>&1 || { tail -20 gpurun_out/tr/clocks_c2.log; exit 1; }
OSE_CLOCKS_WORKLOAD=fused timeout -k 10 200 python3 -u tools/url_clocks.py 20000000 > gpurun_out/tr/clocks_c4.log 2>&1 || { tail -20 gpurun_out/tr/clocks_c4.log; exit 1; }
head -4 gpurun_out/tr/clocks_c2.log; head -4 gpurun_out/tr/clocks_c4.log
for wl in url fused zipf; do
  bash tools/pmc_traffic.sh $wl > gpurun_out/tr/pmc_$wl.log 2>&1 || { tail -20 gpurun_out/tr/pmc_$wl.log; exit 1; }
  tail -3 gpurun_out/tr/pmc_$wl.log
done
