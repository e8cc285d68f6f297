# Position-quarter F(4x4) kernel (rpst_wino4q.hip): conv parity tests on every algorithm,
# then every AdaIN-RP / VGG layer timed with the quarter kernel on (RPST_W4Q=1) and off
# (the 32-channel kernel), interleaved by process. Usage: bash tools/ab_w4q.sh <tag> [layers]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-w4q}
L=${2:-adain}
mkdir -p $O
cd $R
RPST_W4Q=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for q in 1 0; do
    RPST_W4Q=$q timeout -k 10 300 python tools/bench_conv.py --layers $L --algo winograd4 --rounds 2 > $O/conv_q${q}_$rep.log 2>&1 || { tail $O/conv_q${q}_$rep.log; exit 1; }
    echo "W4Q=$q rep $rep: $(grep -o '"layer": "[0-9]*->[0-9]*[^"]*", "wino4_ms": [0-9.]*' $O/conv_q${q}_$rep.log | sed 's/"layer": //; s/ k3 [0-9]*x[0-9]*//; s/"wino4_ms"://' | tr '\n' ' ')"
  done
done
