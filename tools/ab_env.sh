# A/B of one environment switch on the AdaIN-RP layers (tools/bench_conv.py, F(4x4)), rounds
# interleaved by process. Usage: VAR=RPST_WINO4_NOPRIO VALUES="0 1" bash tools/ab_env.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab}
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 300 python tools/bench_conv.py --layers adain --algo winograd4 --rounds 2 > $O/conv_${v}_$rep.log 2>&1 || { tail $O/conv_${v}_$rep.log; exit 1; }
    echo "$VAR=$v rep $rep: $(grep -o '"layer": "[0-9]*->[0-9]*[^"]*", "wino4_ms": [0-9.]*' $O/conv_${v}_$rep.log | sed 's/"layer": //; s/ k3 512x512//; s/"wino4_ms"://' | tr '\n' ' ')"
  done
done
