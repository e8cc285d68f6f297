set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "adain or mean_variance or stats" > gpurun_out/adain_tests.log 2>&1
timeout -k 10 120 python tools/bench_adain.py > gpurun_out/bench_adain.jsonl 2>&1
