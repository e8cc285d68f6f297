#!/bin/bash
# Round 3: the pixel-split 1x1 weight gradient (test + SAModel / AdaptiveSAModel training)
set -o pipefail
mkdir -p gpurun_out/r03n
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "conv1x1_wgrad or sanet or samodel" > gpurun_out/r03n/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --model train_sanet > gpurun_out/r03n/train_sanet.json 2> gpurun_out/r03n/train_sanet.err &&
timeout -k 10 300 python bench.py --model train_adaptive > gpurun_out/r03n/train_adaptive.json 2> gpurun_out/r03n/train_adaptive.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03n/prof -o train_sanet -- python3 bench.py --model train_sanet --steps 3 --warmup 1 > gpurun_out/r03n/prof.log 2>&1
