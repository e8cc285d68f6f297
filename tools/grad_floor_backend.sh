set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gdbg; mkdir -p $O
T="tests/test_gpu_train.py::test_samodel_training_gradients_match_reference"
for cfg in "default:" "fast:MIOPEN_FIND_MODE=2" "nowino:MIOPEN_DEBUG_CONV_WINOGRAD=0" "normal:MIOPEN_FIND_MODE=1"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env RPST_GRAD_DEBUG=1 $e timeout -k 10 300 python -u -m pytest $T -q -s --timeout 280 --timeout-method thread > $O/$n.log 2>&1
  echo "== $n rc=$?"; grep GRADDBG $O/$n.log | sort -k6 -g -r | awk '{print $3,$4,$6,$8,$10}' | head -0
  python3 - $O/$n.log <<'PY'
import sys
rows=[l.split() for l in open(sys.argv[1]) if l.startswith('GRADDBG')]
rows=[(float(r[5])/max(float(r[7]),3*float(r[9])), r) for r in rows]
rows.sort(reverse=True)
for q,r in rows[:4]: print(round(q,3), r[2], r[3], 'rms', r[5], 'cpu_bar', r[7], 'gpu32', r[9])
PY
done
