# A/B of prebuilt library variants (tools/build_variants.sh -> var/<name>/librpst.so) on the
# AdaIN-RP conv layers (tools/bench_conv.py, F(4x4)), interleaved by process, two rounds.
# Usage: LIBS="base slow" bash tools/ab_libs.sh <tag> [bench_conv args]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ablib}
shift
ARGS=${*:---layers adain --algo winograd4 --rounds 2}
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in $LIBS; do
    RPST_LIB=$R/var/$v/librpst.so timeout -k 10 300 python tools/bench_conv.py $ARGS > $O/conv_${v}_$rep.log 2>&1 || { tail $O/conv_${v}_$rep.log; exit 1; }
    echo "$v rep $rep: $(grep -o '"layer": "[0-9]*->[0-9]*[^"]*", "wino4_ms": [0-9.]*' $O/conv_${v}_$rep.log | sed 's/"layer": //; s/ k3 512x512//; s/"wino4_ms"://' | tr '\n' ' ')"
  done
done
