# F(4x4,3x3) bring-up: conv parity tests (all algorithms), then per-layer timings, then
# the timing-only DBG variants of the dominant layer.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/w4_tests.log 2>&1 || { tail -30 gpurun_out/w4_tests.log; exit 1; }
tail -3 gpurun_out/w4_tests.log
timeout -k 10 400 python -u tools/bench_conv.py --layers ${LAYERS:-all} --default-only --rounds 2 ${BENCH_ARGS:-} > gpurun_out/w4_bench.log 2>&1
cat gpurun_out/w4_bench.log
if [ -n "$DBGS" ]; then bash tools/wino4_dbg.sh; fi
