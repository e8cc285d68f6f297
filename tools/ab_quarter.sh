# Quarter-kernel A/B (round 6): the AdaIN-RP layers on F(4x4) under the production rule
# (RPST_W4Q=1) and with the quarter kernel forced on the small-Cin layers (=2), for each
# prebuilt library variant (tools/build_variants.sh -> var/<name>/librpst.so), plus the
# statistics epilogue on 128->256 (tools/ab_stats.py), interleaved by process, two rounds.
# Usage: LIBS="base noepi" bash tools/ab_quarter.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-abq}
mkdir -p $O
cd $R
for rep in ${REPS:-1 2}; do
  for v in $LIBS; do
    for q in ${QS:-1 2}; do
      RPST_W4Q=$q RPST_LIB=$R/var/$v/librpst.so timeout -k 10 300 python tools/bench_conv.py --layers ${LAYERS:-adain} --algo winograd4 --rounds 2 > $O/conv_${v}_q${q}_$rep.log 2>&1 || { tail $O/conv_${v}_q${q}_$rep.log; exit 1; }
      echo "$v q$q rep $rep: $(grep -o '"layer": "[0-9]*->[0-9]*[^"]*", "wino4_ms": [0-9.]*' $O/conv_${v}_q${q}_$rep.log | sed 's/"layer": //; s/ k3 512x512//; s/"wino4_ms"://; s/"//g' | tr '\n' ' ')"
    done
    if [ -n "$STATS" ]; then
      RPST_LIB=$R/var/$v/librpst.so timeout -k 10 200 python tools/ab_stats.py --rounds 2 --reps 3 > $O/stats_${v}_$rep.log 2>&1 || { tail $O/stats_${v}_$rep.log; exit 1; }
      echo "$v stats rep $rep: $(cat $O/stats_${v}_$rep.log)"
    fi
  done
done
