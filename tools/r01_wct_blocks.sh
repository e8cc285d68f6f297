# Covariance split-K sizing: WCT bench at (RPST_WCT_BLOCKS, RPST_WCT_KMIN) settings, then
# the WCT parity tests at the default.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for cfg in 4096:4096 8192:4096 16384:2048 12288:2048; do
  b=${cfg%%:*}; k=${cfg##*:}
  RPST_WCT_BLOCKS=$b RPST_WCT_KMIN=$k timeout -k 10 300 python bench.py --model wct --no-cpu-baseline > gpurun_out/bench_wct_b${b}_k$k.json 2> gpurun_out/bench_wct_b${b}_k$k.err
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/bench_wct_b${b}_k$k.json'));print(d['value'], d['kernel_ms_per_step']['wct_fuse C256 262144px N16'])")" | tee -a gpurun_out/r01_wct_blocks.log
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "wct or whiten or matrix" --timeout 120 --timeout-method thread > gpurun_out/wct_tests.log 2>&1
