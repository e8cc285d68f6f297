#!/bin/bash
# reflect-pad border gradient with split-K ring copies: the dgrad / training tests, then the
# SAModel / AdaptiveSAModel / AdaIN-RP training lines
set -o pipefail
O=gpurun_out/${1:-ab_ring}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for m in train_sanet train_adaptive train; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_$m.json 2> $O/bench_$m.err || { tail $O/bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', d['value'], d['ms_per_step'])"
done
