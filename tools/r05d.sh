# quarter-kernel epilogue changes: conv tests (every algorithm, quarter forced on every shape
# it supports), the stats A/B, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05d}; mkdir -p $O
RPST_W4Q=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv or stats" --timeout 300 --timeout-method thread > $O/tests_w4q2.log 2>&1 || { tail -40 $O/tests_w4q2.log; exit 1; }
tail -1 $O/tests_w4q2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_adaptive.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/ab_stats.py --rounds 2 || exit 1
RPST_W4Q=1 timeout -k 10 300 python tools/bench_conv.py --layers adain --algo winograd4 --rounds 2 > $O/conv.log 2>&1 || { tail $O/conv.log; exit 1; }
grep -o '"layer": "[0-9]*->[0-9]*[^"]*", "wino4_ms": [0-9.]*' $O/conv.log
timeout -k 10 300 python bench.py --no-configs > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac']); print(d['kernel_ms_per_step'])"
