# SQ counters of one F(4x4) conv layer (tools/bench_conv.py --only), old kernel (RPST_W4Q=0)
# against the position-quarter kernel (RPST_W4Q=1), two rocprofv3 --pmc passes each.
# Usage: bash tools/sq_conv.sh <tag> <cin->cout> [layers]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for q in 0 1; do
  for p in A B; do
    eval "C=\$SQ$p"
    RPST_W4Q=$q timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/q${q}_$p -o run -- python3 $R/tools/bench_conv.py --layers ${3:-adain} --only "$2" --algo winograd4 --rounds 1 --reps 2 > $O/q${q}_$p.log 2>&1 || { tail $O/q${q}_$p.log; exit 1; }
  done
  echo "== RPST_W4Q=$q"
  python3 $R/tools/sq_kernel.py mfma_kernel $O/q${q}_A $O/q${q}_B
done
