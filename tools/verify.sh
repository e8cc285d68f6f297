# End-of-round verification on one MI355X, in two calls (each under gpurun's 20-minute cap):
#   PART=1: the whole GPU test suite, smoke(), the default bench line (BASELINE configs[1]
#           with configs[0], [2]-[4] as sub-records), the stylize pipeline and the rocprofv3
#           kernel summary of configs[1];
#   PART=2: every other bench line (configs[2]-[4] alone, the SURVEY 8(f) workloads, the
#           training steps), the attention micro-bench and rocprofv3 summaries of configs[2],
#           configs[3] and two training steps.
# Usage: PART=1|2 bash tools/verify.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-verify}
mkdir -p $O
cd $R
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
  cat $O/bench_default.json
  timeout -k 10 400 python tools/bench_stylize.py > $O/stylize.json 2> $O/stylize.err || { tail $O/stylize.err; exit 1; }
  cat $O/stylize.json
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_adain -o adain -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs > $O/prof_adain.log 2>&1 || exit 1
else
  # RUNS: '|'-separated bench.py argument sets (default: all of them)
  IFS='|' read -r -a LINES <<< "${RUNS:---config 2|--config 3|--config 4|--model forward|--model multiscale|--model source|--model adaptive|--model train|--model train_wct|--model train_sanet|--model train_multiscale|--model train_source|--model train_adaptive}"
  for m in "${LINES[@]}"; do
    f=$O/bench_$(echo $m | tr -d ' -').json
    timeout -k 10 400 python bench.py $m --no-cpu-baseline > $f 2> $f.err || { tail $f.err; exit 1; }
    python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$m', d['value'], d['ms_per_step'], r['kernel'], r['frac'])"
  done
  timeout -k 10 120 python tools/bench_attn.py --reps 5 > $O/attn.json 2>&1 || { tail $O/attn.json; exit 1; }
  tail -1 $O/attn.json
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_wct -o wct -- python3 $R/bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_wct.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sanet -o sanet -- python3 $R/bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --no-configs > $O/prof_sanet.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train -o train -- python3 $R/bench.py --model train --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_train.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train_sanet -o train_sanet -- python3 $R/bench.py --model train_sanet --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_train_sanet.log 2>&1 || exit 1
fi
echo done
