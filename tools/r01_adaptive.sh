set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py --model adaptive > gpurun_out/bench_adaptive.json 2> gpurun_out/bench_adaptive.err
timeout -k 10 300 python bench.py --model sanet --no-cpu-baseline > gpurun_out/bench_sanet.json 2> gpurun_out/bench_sanet.err
