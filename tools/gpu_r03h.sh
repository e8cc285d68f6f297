# store_n (statistics-only style half of the AdaIN-RP encoder output): kernel + model tests,
# then configs[1] with and without it (interleaved)
R=$PWD; O=$R/gpurun_out/r03h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_timed.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "stats or adain" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    RPST_ADAIN_STORE_ALL=$v timeout -k 10 300 python bench.py --config 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail $O/b_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));print('store_all=$v', d['value'], d['ms_per_step'], d['roofline']['launch_ms'] if 'launch_ms' in d['roofline'] else d['roofline'])"
  done
done
