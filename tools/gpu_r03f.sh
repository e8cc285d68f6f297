# round 3: F(4x4) half-height blocks (NR = 2) for small-Cin layers.
# 1) every F(4x4) kernel test with all layers forced to NR = 2, 2) the full GPU suite at
# the default threshold, 3) A/B of the AdaIN-RP layers: NR = 4 everywhere vs default vs 64
R=$PWD; O=$R/gpurun_out/r03f; mkdir -p $O
if [ -z "$SKIP_NR2" ]; then export RPST_WINO4_HALF=100000
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "conv or adain or stats or wino" > $O/tests_nr2.log 2>&1; rc=$?; tail -3 $O/tests_nr2.log; [ $rc -eq 0 ] || exit $rc
fi
unset RPST_WINO4_HALF
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_all.log 2>&1; rc=$?; tail -3 $O/tests_all.log; [ $rc -eq 0 ] || exit $rc
VAR=RPST_WINO4_HALF VALUES="0 32 64" timeout -k 10 600 bash tools/ab_env.sh r03f/ab
