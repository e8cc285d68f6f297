#!/bin/bash
# Round 3: wave-per-plane statistics (A/B) + the stats / SANet parity tests
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "mean_std or adain or mean_variance or stats or sanet" > $O/tests.log 2>&1 &&
for r in 1 2; do for v in 1 0; do
  RPST_STATS_WAVE=$v timeout -k 10 120 python tools/bench_stats.py >> $O/bench_stats.log 2>&1 || exit 1
done; done &&
for v in 1 0; do
  RPST_STATS_WAVE=$v timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 30 > $O/c3_w$v.json 2> $O/c3_w$v.err || exit 1
done
