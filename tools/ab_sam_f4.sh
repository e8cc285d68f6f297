#!/bin/bash
# A/B of F(4x4) on the first K slices of SAModel's frozen input VGG in training
# (RPST_SAM_F4_SLICES=K): the SAModel / AdaptiveSAModel gradient tests and the training line
set -o pipefail
O=gpurun_out/${1:-sam_f4}; mkdir -p $O
for k in ${KS:-1 2 3}; do
  RPST_SAM_F4_SLICES=$k timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "samodel or adaptive" > $O/tests_$k.log 2>&1
  echo "slices=$k tests: $(tail -1 $O/tests_$k.log)"
  grep -o "AssertionError: .*" $O/tests_$k.log | head -3
  RPST_SAM_F4_SLICES=$k timeout -k 10 300 python bench.py --model train_sanet --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_$k.json 2> $O/bench_$k.err || { tail $O/bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$k.json'));print('slices=$k train_sanet', d['value'], d['ms_per_step'])"
done
