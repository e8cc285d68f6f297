#!/bin/bash
# Round 4: the small-Cin layers -- every algorithm (direct tile variants, F(2x2), F(4x4)) on
# 16->32, 32->64, 64->32, 32->16, then where the F(4x4) time goes per layer in timing-only
# builds (RPST_W4DBG: 8 no input transform, 16 no barriers, 32 no epilogue, 3 no DMA, 48
# neither barriers nor epilogue; var/w*, tools/build_variants.sh)
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
for only in 16-\>32 32-\>64 64-\>32 32-\>16; do
  timeout -k 10 180 python tools/bench_conv.py --layers adain --rounds 2 --only "$only" > $O/algo.log 2>&1 || { tail $O/algo.log; exit 1; }
  tail -1 $O/algo.log
done
LIBS="w0 w8 w16 w32 w3 w48" bash tools/ab_libs.sh r04d_attr > $O/attr.log 2>&1 || { tail $O/attr.log; exit 1; }
cat $O/attr.log
