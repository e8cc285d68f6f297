#!/bin/bash
# Round 4: WCT fail-loud / original-method / factored-clamp / flash-attention tests, flash vs
# two-GEMM attention timing, then the round-4 PMC + SQ counter tables (tools/prof_pmc.sh)
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_adaptive.py -k "wct or whiten or matrix or factored or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for f in 1 0; do
  RPST_SANET_FLASH=$f timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/attn_flash$f.json 2>&1 || { tail $O/attn_flash$f.json; exit 1; }
  tail -1 $O/attn_flash$f.json
done
SKIP_TESTS=1 bash tools/prof_pmc.sh r04b_pmc > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -30 $O/prof.log
