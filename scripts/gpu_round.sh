# One GPU call: parity tests, default bench line, then rocprofv3 kernel stats + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/profile.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
