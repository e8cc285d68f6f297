#!/bin/bash
# Round 4: SQ counter tables per conv layer for configs[1] (AdaIN-RP: 128->256, 256->128,
# 64->128 @512^2) and configs[3] (SAModel: the VGG 256->256 @128^2), one config per process
# so the dispatch-order attribution sees one step layout (tools/pmc_layers.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for k in 1 3; do
  B="python3 $R/bench.py --config $k --steps 1 --warmup 0 --no-cpu-baseline --layer-order $O/order$k.json"
  timeout -s KILL 240 rocprofv3 --pmc $SQA --output-format csv -d $O/sqA$k -o run -- $B > $O/sqA$k.log 2>&1 || { tail $O/sqA$k.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $SQB --output-format csv -d $O/sqB$k -o run -- $B > $O/sqB$k.log 2>&1 || { tail $O/sqB$k.log; exit 1; }
  python3 $R/tools/pmc_layers.py $O/order$k.json $O/sqA$k $O/sqB$k > $O/sq_layers_config$k.csv || exit 1
  cut -c1-200 $O/sq_layers_config$k.csv
  rm -rf $O/sqA$k $O/sqB$k
done
