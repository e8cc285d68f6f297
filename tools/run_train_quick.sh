set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --model train --no-cpu-baseline > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_train -o train -- python3 $GRAFT_REPO_ROOT/bench.py --model train --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_train.log 2>&1
