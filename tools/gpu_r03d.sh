# 1x1 convs on the batched GEMM: kernel / model / training parity, then configs[3] and the
# AdaptiveSAModel bench with and without it (RPST_CONV1X1_GEMM=0), interleaved
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03d; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_adaptive.py tests/test_gpu_train.py tests/test_gpu_widen.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    RPST_CONV1X1_GEMM=$v timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --no-configs > $O/b3_${v}_$rep.json 2> $O/b3_${v}_$rep.err || { tail $O/b3_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b3_${v}_$rep.json'));print('gemm1x1=$v', d['value'], d['ms_per_step'], {k:v for k,v in d['kernel_ms_per_step'].items() if '1x1' in k or 'gemm' in k})"
  done
done
RPST_CONV1X1_GEMM=1 timeout -k 10 300 python bench.py --model adaptive --steps 10 --warmup 3 --no-cpu-baseline > $O/badapt.json 2> $O/badapt.err || { tail $O/badapt.err; exit 1; }
python -c "import json;d=json.load(open('$O/badapt.json'));print('adaptive', d['value'], d['ms_per_step'])"
