# Full -m gpu suite, then the default bench line; each step under its own limit, chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
