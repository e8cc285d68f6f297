set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --model train > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_train -o train -- python3 $R/bench.py --model train --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_train.log 2>&1
