#!/bin/bash
# Round 3: A/B of the pooled-output F(4x4) epilogue on one box (alternating runs)
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    RPST_POOL_EPILOGUE=$v timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 30 > $O/c3_p${v}_r$r.json 2> $O/c3_p${v}_r$r.err || exit 1
  done
done
for v in 1 0; do
  RPST_POOL_EPILOGUE=$v timeout -k 10 300 python bench.py --model source --no-cpu-baseline --steps 30 > $O/src_p$v.json 2> $O/src_p$v.err || exit 1
done
