#!/bin/bash
# Round 4: flash attention with LDS operands read a group ahead (Q in AGPRs, O in VGPRs):
# tests + timing; training-step precision policy (F(4x4) for AdaIN-RP / MultiScale / WCT /
# SourceNet): the training gradient tests and the training bench lines
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "attention" > $O/tests_flash.log 2>&1 || { tail -40 $O/tests_flash.log; exit 1; }
grep -E "passed|failed" $O/tests_flash.log | tail -1
for f in 1 3 0; do
  RPST_SANET_FLASH=$f timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/attn_flash$f.json 2>&1 || { tail $O/attn_flash$f.json; exit 1; }
  echo "flash=$f $(tail -1 $O/attn_flash$f.json)"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train.py > $O/tests_train.log 2>&1 || { tail -40 $O/tests_train.log; exit 1; }
grep -E "passed|failed" $O/tests_train.log | tail -1
for m in train train_wct train_sanet train_source; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_$m.json 2> $O/bench_$m.err || { tail $O/bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_config3.err || { tail $O/bench_config3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_config3.json'));print('config3', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step'))"
