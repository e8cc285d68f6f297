#!/bin/bash
# Round 3: AEA clamp path without the affinity matrix (Z = cn^T (sn W1^T), dW1 = (cn du)^T sn)
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_timed.py -k "adaptive or aea or Adaptive" > $O/tests.log 2>&1 &&
for m in "--model adaptive" "--model train_adaptive"; do
  f=$(echo $m | tr -d ' -'); timeout -k 10 300 python bench.py $m --no-cpu-baseline > $O/$f.json 2> $O/$f.err || exit 1
done
