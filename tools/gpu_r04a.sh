#!/bin/bash
# Round 4 baseline: per-algorithm timing of the AdaIN-RP layers and the default bench line
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 300 python tools/bench_conv.py --layers adain --default-only --rounds 2 > $O/conv_adain.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs > $O/bench_default.json 2> $O/bench_default.err
