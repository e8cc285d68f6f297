# The attention models' gradient tests twice in separate processes under the suite's MIOpen
# setting (tests/conftest.py: MIOPEN_FIND_MODE=FAST): the GPU torch floor must repeat.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/grep; mkdir -p $O
T="tests/test_gpu_train.py::test_samodel_training_gradients_match_reference tests/test_gpu_train.py::test_adaptive_samodel_training_gradients_match_reference"
for r in 1 2; do
  RPST_GRAD_DEBUG=1 timeout -k 10 400 python -u -m pytest $T -q -s --timeout 380 --timeout-method thread > $O/r$r.log 2>&1
  echo "== run $r rc=$? $(tail -1 $O/r$r.log)"
  grep GRADDBG $O/r$r.log | awk '{print $2, $4, $6, $10}' | sort > $O/r$r.txt
done
cmp -s $O/r1.txt $O/r2.txt && echo "floors and errors identical across the two processes" || diff $O/r1.txt $O/r2.txt | head
python3 - $O/r1.log <<'PY'
import sys
rows=[l.split() for l in open(sys.argv[1]) if l.startswith('GRADDBG')]
for fam in sorted(set(r[1] for r in rows)):
    rr=[(float(r[5])/max(float(r[7]),3*float(r[9])), r) for r in rows if r[1]==fam]
    rr.sort(reverse=True)
    for q,r in rr[:3]: print(fam, 'rms/bar', round(q,3), r[3], 'rms', r[5], 'cpu_bar', r[7], 'gpu32', r[9])
PY
