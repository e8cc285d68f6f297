# Narrow kernel rows per thread (default: 4 for Cout <= 4, 2 otherwise): conv and model
# parity tests, default bench.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/narrow_rpt_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
