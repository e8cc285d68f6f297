#!/bin/bash
# Round 4: knob sweep on the small-Cin F(4x4) layers (co-tile split, 8- vs 16-row blocks),
# then the round-4 PMC traffic + SQ counter tables of configs[1] (tools/prof_pmc.sh)
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
# every algorithm (direct tile variants, F(2x2), F(4x4)) on the small layers
for only in 16-\>32 32-\>64 64-\>32 32-\>16; do
  timeout -k 10 180 python tools/bench_conv.py --layers adain --rounds 2 --only "$only" > $O/algo.log 2>&1 || { tail $O/algo.log; exit 1; }
  tail -1 $O/algo.log
done
for only in 16-\>32 32-\>64 64-\>32 32-\>16; do
  for cs in 1 2; do
    for half in 512 2048 0; do
      RPST_WINO4_COSPLIT=$cs RPST_WINO4_HALF=$half timeout -k 10 120 python tools/bench_conv.py --layers adain --algo winograd4 --rounds 2 --only "$only" > $O/k.log 2>&1 || { tail $O/k.log; exit 1; }
      echo "cosplit=$cs half=$half $(grep -o '"wino4_ms": [0-9.]*' $O/k.log)  $only"
    done
  done
done
SKIP_TESTS=1 bash tools/prof_pmc.sh r04d_pmc > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -25 $O/prof.log
# where the F(4x4) time goes per layer: timing-only builds (RPST_W4DBG: 8 no input transform,
# 16 no barriers, 32 no epilogue, 3 no DMA, 48 neither barriers nor epilogue)
LIBS="w0 w8 w16 w32 w3 w48" bash tools/ab_libs.sh r04d_attr > $O/attr.log 2>&1 || { tail $O/attr.log; exit 1; }
cat $O/attr.log
