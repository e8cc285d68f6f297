# paired first conv (no torch.cat): kernel + every model's GPU parity, smoke, then configs[1]
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03h; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --no-configs --steps 20 --warmup 5 > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
python -c "import json;d=json.load(open('$O/b1.json'));print('configs[1]', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
