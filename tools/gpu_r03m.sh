# after the verification: the multi-level WCT shapes (8-way covariance split) and the
# configs[2] PMC traffic table with the 16-wave covariance kernel
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03m; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_timed.py tests/test_gpu_fullsize.py -x -q -k "wct or whiten or matrix" --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_wct.py --json $O/wct_shapes.json > $O/wct_shapes.log 2>&1 || { tail $O/wct_shapes.log; exit 1; }
cat $O/wct_shapes.log
timeout -k 10 200 python -u tools/bench_cov.py > $O/bench_cov.log 2>&1 || { tail $O/bench_cov.log; exit 1; }
cat $O/bench_cov.log
bash tools/prof_pmc_configs.sh r03m_pmc 2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_adain -o adain -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs > $O/prof_adain.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs > $O/bench_for_prof.json 2>/dev/null || exit 1
echo done
