# which conv forms the training steps can take on the floor-derived gradient bars:
# the training test file under each setting (default: differentiated chains F(2x2), constant
# branches F(4x4) 32-channel; RPST_TRAIN_QUARTER=1: constant branches may take the quarter
# kernel; RPST_TRAIN_F4=...: F(4x4) on every chain of those families), then the training
# benches of the SAModel and SourceNet steps. Usage: bash tools/train_forms.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-forms}
mkdir -p $O
cd $R
ALL=adain,multiscale,wct,sanet,source
i=0
for v in ${FORMS:-"RPST_TRAIN_QUARTER=1" "RPST_TRAIN_F4=$ALL" "RPST_TRAIN_F4=$ALL RPST_TRAIN_QUARTER=1"}; do
  i=$((i+1))
  env $v timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests_$i.log 2>&1
  echo "$v: $(tail -1 $O/tests_$i.log)"
  grep -E "^FAILED" $O/tests_$i.log | head -8
done
[ -n "$NOBENCH" ] && exit 0
for m in train_sanet train_source; do
  for v in "" "RPST_TRAIN_QUARTER=1"; do
    env $v timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > $O/bench_$m.json 2> $O/bench_$m.err || { tail -3 $O/bench_$m.err; continue; }
    python -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', '$v', d['value'], d['unit'], d['ms_per_step'])"
  done
done
