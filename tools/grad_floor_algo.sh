# SAModel / AdaptiveSAModel gradient RMS against the floor bars under each conv algorithm of
# the training step (RPST_CONV_ALGO, per launch), with the GPU torch floor printed
# (RPST_GRAD_DEBUG). Usage: bash tools/grad_floor_algo.sh [algos]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/galgo; mkdir -p $O
T="tests/test_gpu_train.py::test_samodel_training_gradients_match_reference tests/test_gpu_train.py::test_adaptive_samodel_training_gradients_match_reference"
for a in ${1:-default direct}; do
  if [ "$a" = default ]; then e=""; else e="RPST_CONV_ALGO=$a"; fi
  env RPST_GRAD_DEBUG=1 $e timeout -k 10 400 python -u -m pytest $T -q -s --timeout 380 --timeout-method thread > $O/$a.log 2>&1
  echo "== $a rc=$? $(tail -1 $O/$a.log)"
  python3 - $O/$a.log <<'PY'
import sys
rows=[l.split() for l in open(sys.argv[1]) if l.startswith('GRADDBG')]
for fam in sorted(set(r[1] for r in rows)):
    rr=[(float(r[5])/float(r[7]), r) for r in rows if r[1]==fam]
    rr.sort(reverse=True)
    for q,r in rr[:3]: print(fam, 'rms/cpu_bar', round(q,3), r[3], 'rms', r[5], 'gpu32', r[9])
PY
done
