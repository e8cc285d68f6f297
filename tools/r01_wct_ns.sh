# WCT: parity tests (matrix powers, whiten_and_color, wct_fuse, WCT-RP), then the WCT bench.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "wct or whiten or matrix" --timeout 120 --timeout-method thread > gpurun_out/wct_tests.log 2>&1
timeout -k 10 300 python bench.py --model wct --no-cpu-baseline > gpurun_out/bench_wct_ns32.json 2> gpurun_out/bench_wct_ns32.err
