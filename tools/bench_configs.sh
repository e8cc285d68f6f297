# Bench lines of BASELINE.json configs[1]-[4] on this box (configs[4] at the GPU count the
# box has; the driver's 8-GPU node runs it with --gpus 8). Usage: bash tools/bench_configs.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-configs}
mkdir -p $O
cd $R
for c in ${CONFIGS:-1 2 3 4}; do
  timeout -k 10 600 python bench.py --config $c ${EXTRA:-} > $O/config$c.json 2> $O/config$c.err || { tail $O/config$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/config$c.json'));r=d['roofline'];print('config $c', d['value'], d['unit'], d['ms_per_step'], r['kernel'], r['frac'], d.get('cpu_baseline'))"
done
