#!/bin/bash
# Round 3: max pool in the F(4x4) epilogue (VGG relu1_2 / 2_2 / 3_4 write pooled maps)
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pool or dgrad_masked" > $O/tests_k.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_timed.py > $O/tests_m.log 2>&1 &&
for m in "--config 3" "--model source" "--model adaptive"; do
  f=$(echo $m | tr -d ' -'); timeout -k 10 300 python bench.py $m --no-cpu-baseline > $O/$f.json 2> $O/$f.err || exit 1
done
