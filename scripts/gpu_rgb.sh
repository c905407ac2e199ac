# rgb_array GPU parity + the generated-assets suite (quick round-3 check)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rgb_array.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_rgb.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_rgb.log; exit $rc
