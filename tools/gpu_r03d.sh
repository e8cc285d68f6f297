R=$PWD; O=$R/gpurun_out/r03d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "wct or matrix or whiten or mix or sam or sanet or adaptive" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wct -- python3 $R/tools/bench_wct.py --json $O/wct_shapes.json > $O/prof.log 2>&1; rc=$?; tail -6 $O/prof.log; exit $rc
