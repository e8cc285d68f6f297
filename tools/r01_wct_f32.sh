# WCT colour transform on the fp32 MFMA: WCT parity tests, then the WCT bench with the
# fp32 transform (default) and the fp64 one (RPST_WCT_T_F64=1).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "wct or whiten or matrix" --timeout 120 --timeout-method thread > gpurun_out/wct_tests.log 2>&1
timeout -k 10 300 python bench.py --model wct --no-cpu-baseline > gpurun_out/bench_wct_f32.json 2> gpurun_out/bench_wct_f32.err
RPST_WCT_T_F64=1 timeout -k 10 300 python bench.py --model wct --no-cpu-baseline > gpurun_out/bench_wct_f64.json 2> gpurun_out/bench_wct_f64.err
