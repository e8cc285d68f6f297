# Measurement pass: GPU kernel tests of the changed conv paths, the default bench,
# per-dispatch PMC traffic (FETCH / WRITE in separate passes) attributed per layer, and two
# SQ counter passes on one bench step, attributed per layer. Usage: bash tools/prof_pmc.sh <tag> (SKIP_TESTS=1 skips the kernel tests)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-pmc}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/gpu_kernels.log 2>&1 || { tail -30 $O/gpu_kernels.log; exit 1; }
  tail -2 $O/gpu_kernels.log
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --layer-order $O/order.json"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
python3 $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/order.json $O/pmc_traffic.json
B1="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-configs --layer-order $O/order1.json"
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for p in A B; do
  eval "C=\$SQ$p"
  K=""
  for c in $C; do grep -qw "$c" $O/counters_list.txt && K="$K $c"; done
  echo "pass $p:$K"
  timeout -s KILL 240 rocprofv3 --pmc $K --output-format csv -d $O/sq_$p -o run -- $B1 > $O/sq_$p.log 2>&1 || { tail $O/sq_$p.log; exit 1; }
done
python3 $R/tools/pmc_layers.py $O/order1.json $O/sq_A $O/sq_B > $O/sq_layers.csv
cat $O/sq_layers.csv
echo done
