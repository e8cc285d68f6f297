#!/bin/bash
# Round 4: where the flash attention kernel's time goes -- timing-only builds
# (RPST_FLDBG: 1 no softmax, 2 no waits/barriers, 4 no DMA, 8 no O update), two rounds
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
for rep in 1 2; do
  for v in fl0 fl1 fl2 fl4 fl8 fl6 fl7; do
    RPST_LIB=$GRAFT_REPO_ROOT/var/$v/librpst.so timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/$v.json 2>&1 || { tail $O/$v.json; exit 1; }
    echo "$v rep $rep $(tail -1 $O/$v.json | cut -c1-60)"
  done
done
# the stylize.py pipeline with the zlib strategies (rle: stylize.py's default)
timeout -k 10 400 python tools/bench_stylize.py > $O/stylize.json 2> $O/stylize.err || { tail $O/stylize.err; exit 1; }
tail -1 $O/stylize.json | cut -c1-600
