# A/B of F(4x4) kernel variants (RPST_WINO4_VAR) on every AdaIN-RP layer, HIP-event timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-w4var}
mkdir -p $O
cd $R
for v in ${VARS:-0 1 2}; do
  echo "VAR=$v"
  RPST_WINO4_VAR=$v timeout -k 10 300 python tools/bench_conv.py --layers adain --algo winograd4 --rounds 2 > $O/conv_$v.log 2>&1 || { tail $O/conv_$v.log; exit 1; }
  grep layer $O/conv_$v.log
done
