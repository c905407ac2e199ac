# Round-3 GPU call: parity suite, a short bench line, the occupancy census.
#   STEPS=tests,bench,census (default all); PYTEST_ARGS / BENCH_ARGS / CENSUS_GAMES override
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${STEPS:-tests,bench,census}
rc=0
if [[ $S == *tests* ]]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [[ $rc != 0 ]] && exit $rc
fi
if [[ $S == *bench* ]]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  [[ $rc != 0 ]] && exit $rc
fi
if [[ $S == *census* ]]; then
  timeout -k 10 300 python3 scripts/census.py ${CENSUS_GAMES:-coinrun} > gpurun_out/census.log 2>&1
  rc=$?; tail -60 gpurun_out/census.log
fi
exit $rc
