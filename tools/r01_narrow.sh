# Narrow 3x3 layers on the VALU: conv parity tests, AdaIN-RP model tests, default bench with
# the narrow kernel (default) and without (RPST_CONV_NARROW=0).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/narrow_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_narrow.json 2> gpurun_out/bench_narrow.err
RPST_CONV_NARROW=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nonarrow.json 2> gpurun_out/bench_nonarrow.err
