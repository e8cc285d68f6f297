set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wctb
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --config 2 --no-cpu-baseline > $O/bench_wct.json 2> $O/bench_wct.err || { tail $O/bench_wct.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_wct.json'));print(d['value'], d['ms_per_step']); print(d['kernel_ms_per_step'])"
RPST_FUSE_WCT=0 timeout -k 10 300 python bench.py --config 2 --no-cpu-baseline > $O/bench_wct_unfused.json 2> $O/bench_wct.err || { tail $O/bench_wct.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_wct_unfused.json'));print('unfused', d['value'], d['ms_per_step']); print(d['kernel_ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_wct -o wct -- python3 $R/bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_wct.log 2>&1 || exit 1
head -25 $O/prof_wct/wct_kernel_stats.csv | cut -c1-200
