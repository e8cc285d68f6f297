# round 3: WCT / AdaIN-fold / training GPU tests, then the configs[2] (WCT-RP) bench under
# rocprofv3 --kernel-trace --stats and the per-shape WCT bench
R=$PWD; O=$R/gpurun_out/r03e; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_kernels.py tests/test_gpu_adaptive.py -x -q --timeout 200 --timeout-method thread -k "wct or matrix or whiten or mix or fold or adain or sam or sanet or adaptive" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 $R/bench.py --config 2 --steps 10 --warmup 3 --no-configs > $O/bench_c2.log 2>&1; rc=$?; tail -2 $O/bench_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/bench_wct.py --json $O/wct_shapes.json > $O/wct.log 2>&1; rc=$?; tail -5 $O/wct.log; exit $rc
