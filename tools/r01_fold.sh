# AdaIN folded into per-image F(4x4) weights: targeted parity, full GPU suite, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k adain -x -q --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || { tail -40 gpurun_out/fold_tests.log; exit 1; }
tail -2 gpurun_out/fold_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d['value'], d['kernel_ms_per_step'])"
for m in ${MODELS:-source}; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || { tail gpurun_out/bench_$m.err; exit 1; }
  echo "$m $(python -c "import json;d=json.load(open('gpurun_out/bench_$m.json'));print(d['value'])")"
done
