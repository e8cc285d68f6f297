# Conv kernel iteration: GPU conv/model parity tests, every AdaIN-RP layer on F(4x4) (HIP
# events, tools/bench_conv.py) and the default bench line. Usage: bash tools/run_conv_check.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-conv}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_conv.py --layers adain --algo winograd4 --rounds 2 > $O/conv.log 2>&1 || { tail $O/conv.log; exit 1; }
cat $O/conv.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac']); print(d['kernel_ms_per_step'])"
