#!/bin/bash
# Round 4: flash attention variants (1 pipelined 4-wave = default, 2 8-wave, 3 plain 4-wave,
# 0 two-GEMM) tests + timing; GPU PNG filter tests; stylize pipeline line; training precision A/B
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
for f in 1 2; do
  RPST_SANET_FLASH=$f timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "attention" > $O/tests_flash$f.log 2>&1 || { tail -40 $O/tests_flash$f.log; exit 1; }
  echo "flash=$f $(grep -E 'passed|failed' $O/tests_flash$f.log | tail -1)"
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_imageio.py > $O/tests_io.log 2>&1 || { tail -40 $O/tests_io.log; exit 1; }
grep -E "passed|failed" $O/tests_io.log | tail -1
for f in 1 2 3 0; do
  RPST_SANET_FLASH=$f timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/attn_flash$f.json 2>&1 || { tail $O/attn_flash$f.json; exit 1; }
  echo "flash=$f $(tail -1 $O/attn_flash$f.json)"
done
timeout -k 10 300 python tools/bench_stylize.py --pairs 128 --batch 32 > $O/stylize.json 2> $O/stylize.err || { tail $O/stylize.err; exit 1; }
cat $O/stylize.json
for p in 1 0; do
  RPST_TRAIN_PRECISE=$p timeout -k 10 300 python tools/grad_precision_ab.py > $O/gradab_$p.log 2>&1 || { tail $O/gradab_$p.log; exit 1; }
  tail -1 $O/gradab_$p.log
done
for m in train train_sanet train_source; do
  RPST_TRAIN_PRECISE=0 timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_${m}_p0.json 2> $O/bench_${m}_p0.err || { tail $O/bench_${m}_p0.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${m}_p0.json'));print('$m precise=0', d['value'], d['ms_per_step'])"
done
