# Timing experiments for the Winograd kernel (results are wrong by design): one layer,
# each RPST_WINO_DBG variant. Usage: bash tools/wino_dbg.sh [layer]
L=${1:-128->256}
mkdir -p gpurun_out
for d in ${DBGS:-256 16 32 1 2 4 15}; do
  echo "DBG=$d $(RPST_WINO_DBG=$d timeout -k 10 120 python tools/bench_conv.py --layers adain --only "$L" --algo winograd --rounds 2 2>/dev/null | grep layer)"
done
