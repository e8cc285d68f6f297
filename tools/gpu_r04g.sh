#!/bin/bash
# Round 4: conv parity with the last-co-tile exchange (5 barriers per epilogue), its A/B on
# the AdaIN-RP layers; flash attention with the exp2 / row-swap softmax; the training tests
# and lines; the stylize pipeline with the rle thread split
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py > $O/tests_kernels.log 2>&1 || { tail -30 $O/tests_kernels.log; exit 1; }
tail -1 $O/tests_kernels.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "attention" > $O/tests_flash.log 2>&1 || { tail -30 $O/tests_flash.log; exit 1; }
tail -1 $O/tests_flash.log
timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/attn.json 2>&1 || { tail $O/attn.json; exit 1; }
echo "attn $(tail -1 $O/attn.json)"
LIBS="we0 pk0 pk1" bash tools/ab_libs.sh r04g_we > $O/we.log 2>&1 || { tail $O/we.log; exit 1; }
cat $O/we.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py > $O/tests_train.log 2>&1 || { tail -40 $O/tests_train.log; exit 1; }
tail -1 $O/tests_train.log
for m in train train_wct train_sanet train_source; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_$m.json 2> $O/bench_$m.err || { tail $O/bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', d['value'], d['ms_per_step'])"
done
timeout -k 10 400 python tools/bench_stylize.py > $O/stylize.json 2> $O/stylize.err || { tail $O/stylize.err; exit 1; }
tail -1 $O/stylize.json | cut -c1-300
