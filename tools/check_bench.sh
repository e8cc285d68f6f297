# Kernel iteration on one MI355X: the GPU test suite, an A/B of var/ builds
# (tools/ab_variants.sh; AB="old base", LAYERS=...), then the default bench line.
# Usage: AB="old base" bash tools/check_bench.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-check}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
if [ -n "$AB" ]; then
  ROUNDS=${ROUNDS:-2} LAYERS=${LAYERS:-"128->256 64->128 256->128"} bash tools/ab_variants.sh $AB > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
  cat $O/ab.log
fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
