# Round-3 closing check of the committed tree: smoke, the whole GPU parity suite, the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 10; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[[ $rc != 0 ]] && exit $rc
timeout -k 10 600 python3 bench.py --host-steps 0 --no-cpu-baseline > gpurun_out/bench_verify.json 2> gpurun_out/bench_verify.err || { tail -5 gpurun_out/bench_verify.err; exit 11; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_verify.json')); print(round(d['value']/1e6,2), d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic_source'])"
