set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_prefetch.py tests/test_state_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_prefetch.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_prefetch.log; exit $rc
