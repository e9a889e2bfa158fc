#!/bin/bash
# Round-3 pass: the GPU suite, then the deferred-classify A/B, URL clocks on
# C4's mix, the OTLP bench.  Each step time-limited; stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3i
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" $OUT/pytest.log | head -20; exit $rc; fi
bash tools/gpu_ab.sh r3i_ab _nodefer,_notail fused url || exit 1
OSE_CLOCKS_WORKLOAD=fused timeout -k 10 200 python -u tools/url_clocks.py 10000000 0 > $OUT/clocks_c4.log 2>&1 || { tail -5 $OUT/clocks_c4.log; exit 1; }
tail -6 $OUT/clocks_c4.log
timeout -k 10 300 python -u tools/otlp_bench.py --out $OUT/otlp.json > $OUT/otlp.log 2>&1 || { tail -5 $OUT/otlp.log; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/otlp.json'))
print('decode', round(d['decode_pinned_ms'],1), {k: round(v,1) for k,v in d['decode_phases_ms'].items()}, 'encode', round(d['encode_ms'],1), d['encode_phases_ms'], 'e2e', round(d['end_to_end_with_encode_spans_per_s']/1e6,1), 'M/s', 'b8192', d['batch8192_legs_ms_median'])"
