# round 2: new boundary / C5 parity tests, the full GPU suite, then a bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_c5.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -15 gpurun_out/pytest_new.log; tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
