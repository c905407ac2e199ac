# Round-4 GPU call: smoke, the -m gpu parity suite (optionally a -k filter: K=...), then the driver's
# default bench line.  Each step runs under its own time limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 10; }
tail -1 gpurun_out/smoke.log
if [[ "${TESTS:-1}" == 1 ]]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [[ $rc != 0 ]] && exit $rc
fi
if [[ "${BENCH:-1}" == 1 ]]; then
  timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 11; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(round(d['value']/1e6,2), d['roofline'], d.get('host_path'), d['cpu_baseline'])"
fi
