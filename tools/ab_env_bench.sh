# configs[1] bench line per environment setting ("X=0" = none), interleaved twice: images/s
# and the per-layer ms per step. Usage: bash tools/ab_env_bench.sh <tag> "VAR=v" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abenv}; shift; mkdir -p $O
for rep in 1 2; do
  for e in "$@"; do
    f=$O/$(echo $e | tr '=' '_').$rep.json
    env $e timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline > $f 2> $f.err || { tail $f.err; exit 1; }
    python -c "import json;d=json.load(open('$f'));k=d['kernel_ms_per_step'];print('$e', d['value'], ' '.join(x.split()[1] + ':' + str(round(k[x], 3)) for x in k))"
  done
done
