#!/bin/bash
# Round 4: training tests + lines with F(4x4) on the constant branches (VGG loss targets,
# WCT-RP's encoder, SourceNet's frozen VGG); the stylize pipeline with the rle thread split;
# configs[3] (flash attention) and the forward line
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py > $O/tests_train.log 2>&1 || { tail -40 $O/tests_train.log; exit 1; }
tail -1 $O/tests_train.log
for m in train train_wct train_sanet train_source train_multiscale train_adaptive; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_$m.json 2> $O/bench_$m.err || { tail $O/bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_config3.err || { tail $O/bench_config3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_config3.json'));print('config3', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --model forward --no-cpu-baseline > $O/bench_forward.json 2> $O/bench_forward.err || { tail $O/bench_forward.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_forward.json'));print('forward', d['value'], d['ms_per_step'])"
timeout -k 10 400 python tools/bench_stylize.py > $O/stylize.json 2> $O/stylize.err || { tail $O/stylize.err; exit 1; }
tail -1 $O/stylize.json | cut -c1-300
