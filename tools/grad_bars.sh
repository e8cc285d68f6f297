# training tests on the floor-derived gradient bars, then the worst err / bar per
# golden case under each training conv setting (tools/grad_bars_ab.py).
# Usage: bash tools/grad_bars.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-grads}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_imageio.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -12
[ $rc -gt 1 ] && exit $rc
ALL=adain,multiscale,wct,sanet,source
for v in "" "RPST_TRAIN_QUARTER=1" "RPST_TRAIN_F4=$ALL" "RPST_TRAIN_F4=$ALL RPST_TRAIN_QUARTER=1"; do
  env $v timeout -k 10 300 python tools/grad_bars_ab.py > $O/bars.log 2>&1 || { tail $O/bars.log; exit 1; }
  tail -1 $O/bars.log
done
