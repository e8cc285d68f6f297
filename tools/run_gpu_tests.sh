# GPU parity suite (optionally a subset: FILES="tests/x.py ..."), then optional extra command.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${TMO:-500} python -u -m pytest ${FILES:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
