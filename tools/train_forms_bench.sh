# training-step benches with the default training conv forms and with F(4x4) (the
# 32-channel kernel) on every chain (RPST_TRAIN_F4=all families). Usage: bash tools/train_forms_bench.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-tb}
mkdir -p $O
cd $R
ALL=adain,multiscale,wct,sanet,source
for m in train train_wct train_sanet train_multiscale train_source train_adaptive; do
  for v in "RPST_TRAIN_F4=" "RPST_TRAIN_F4=$ALL"; do
    env $v timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; continue; }
    python -c "import json;d=json.load(open('$O/b.json'));print('$m', '${v#RPST_TRAIN_F4=}' or 'default', d['value'], d['unit'], d['ms_per_step'])"
  done
done
