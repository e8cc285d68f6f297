# Timing experiments for the F(4x4) Winograd kernel (results are wrong by design): one
# layer, each RPST_WINO4_DBG variant. Usage: bash tools/wino4_dbg.sh [layer]
L=${1:-128->256}
mkdir -p gpurun_out
for d in ${DBGS:-256 1 2 4 8 16 32 64 7 23 87 95}; do
  echo "DBG=$d $(RPST_WINO4_DBG=$d timeout -k 10 120 python tools/bench_conv.py --layers adain --only "$L" --algo winograd4 --rounds 2 2>/dev/null | grep layer)"
done
