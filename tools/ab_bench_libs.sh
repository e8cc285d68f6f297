# configs[1] bench line per library variant (var/<name>/librpst.so; "base" = the in-tree
# build), interleaved twice: images/s and the quarter-kernel layers' ms per step.
# Usage: bash tools/ab_bench_libs.sh <tag> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; shift; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset RPST_LIB; else export RPST_LIB=var/$v/librpst.so; fi
    timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail $O/$v.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$v.$rep.json'));k=d['kernel_ms_per_step'];print('$v', d['value'], ' '.join(x.split()[1] + ':' + str(round(k[x], 3)) for x in k))"
  done
done
