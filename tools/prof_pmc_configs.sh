# Per-config PMC traffic (FETCH_SIZE / WRITE_SIZE in separate rocprofv3 passes, attributed
# per launch by tools/pmc_traffic.py) for BASELINE configs[1]-[4]:
#   profiles/<tag>/pmc_traffic_config{k}.json. Usage: bash tools/prof_pmc_configs.sh <tag> [configs]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-pmc_cfg}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in ${2:-1 2 3 4}; do
  B="python3 $R/bench.py --config $k --steps 2 --warmup 1 --no-cpu-baseline --layer-order $O/order$k.json"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$k -o run -- $B > $O/fetch$k.log 2>&1 || { tail $O/fetch$k.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write$k -o run -- $B > $O/write$k.log 2>&1 || { tail $O/write$k.log; exit 1; }
  python3 $R/tools/pmc_traffic.py $O/fetch$k $O/write$k $O/order$k.json $O/pmc_traffic_config$k.json || exit 1
  rm -rf $O/fetch$k $O/write$k
done
echo done
