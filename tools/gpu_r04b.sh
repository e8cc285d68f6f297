#!/bin/bash
# Round 4: WCT fail-loud / original-method / factored-clamp / flash-attention tests, flash vs
# two-GEMM attention timing, the stylize pipeline and forward() no-grad lines
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_adaptive.py -k "factored or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for f in 1 0; do
  RPST_SANET_FLASH=$f timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/attn_flash$f.json 2>&1 || { tail $O/attn_flash$f.json; exit 1; }
  tail -1 $O/attn_flash$f.json
done
timeout -k 10 300 python bench.py --model forward --no-cpu-baseline > $O/bench_forward.json 2> $O/bench_forward.err || { tail $O/bench_forward.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_forward.json'));print('forward', d['value'], d['ms_per_step'], d['roofline']['kernel'])"
timeout -k 10 300 python tools/bench_stylize.py --pairs 128 --batch 32 --workers 8 > $O/stylize.json 2> $O/stylize.err || { tail $O/stylize.err; exit 1; }
cat $O/stylize.json
