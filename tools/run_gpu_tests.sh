# GPU test suite (optionally a subset): python -m pytest -m gpu, one process, per-test timeout.
# Usage: bash tools/run_gpu_tests.sh <tag> [pytest args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-tests}
shift
[ $# -eq 0 ] && set -- tests
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -25
exit $rc
