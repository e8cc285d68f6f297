#!/bin/bash
# Round 3: ReLU backward fused into the dgrad (masked conv epilogue + masked border fold)
set -o pipefail
mkdir -p gpurun_out/r03o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dgrad_masked or conv2d_pair or conv1x1" tests/test_gpu_train.py > gpurun_out/r03o/tests.log 2>&1 &&
for m in train train_wct train_sanet train_adaptive train_source train_multiscale; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/r03o/$m.json 2> gpurun_out/r03o/$m.err || exit 1
done
