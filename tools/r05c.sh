set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 120 ./tools/mfma_peak.bin > $O/mfma_peak.log 2>&1 || { cat $O/mfma_peak.log; exit 1; }
tail -6 $O/mfma_peak.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_adaptive.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/ab_stats.py --rounds 2 || exit 1
timeout -k 10 200 python tools/bench_attn.py --reps 5 > $O/attn.json 2>&1 || { tail $O/attn.json; exit 1; }
tail -1 $O/attn.json
timeout -k 10 300 python bench.py --config 2 --steps 3 --warmup 2 --no-cpu-baseline > $O/bench_wct.json 2> $O/bench_wct.err || { tail $O/bench_wct.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_wct.json'));print(d['value'], d.get('roofline_wct'))"
