# Round-1 verification (final, after the WCT fp32 transform): GPU parity suite, smoke, bench lines of every
# workload, rocprofv3 kernel stats of the default bench, PMC FETCH/WRITE passes (separate runs).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for m in ${MODELS:-wct sanet multiscale source adaptive train}; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || { tail gpurun_out/bench_$m.err; exit 1; }
  echo "$m $(python -c "import json;d=json.load(open('gpurun_out/bench_$m.json'));print(d['value'], d['roofline']['kernel'], d['roofline']['frac'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_adain -o adain -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_adain.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_wct -o wct -- python3 $R/bench.py --model wct --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_wct.log 2>&1 || exit 1
echo done
