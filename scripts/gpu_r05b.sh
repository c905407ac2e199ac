# Round-5 (b): the register-frame coinrun render -- smoke, the coinrun parity tests, the default bench
# line against PROCGEN_MI355X_RENDER_RF=0 (the LDS-frame kernel), then the state-test port for a few
# games (timing).  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/b
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/b/smoke.log 2>&1 || { tail -5 gpurun_out/b/smoke.log; exit 10; }
tail -1 gpurun_out/b/smoke.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_coinrun.py -x -v --timeout 300 --timeout-method thread > gpurun_out/b/pytest_coinrun.log 2>&1 || { tail -30 gpurun_out/b/pytest_coinrun.log; exit 11; }
tail -2 gpurun_out/b/pytest_coinrun.log
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/b/$1.json 2> gpurun_out/b/$1.err || { tail -5 gpurun_out/b/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
ab coinrun_rf "A=0" coinrun 100 || exit 12
ab coinrun_lds "PROCGEN_MI355X_RENDER_RF=0" coinrun 100 || exit 12
for v in ${VARIANTS:-}; do ab coinrun_$v "PROCGEN_MI355X_RENDER_RF=0 PROCGEN_MI355X_LIB=$v" coinrun 100 || exit 12; done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_state_rollouts.py -x -v --timeout 600 --timeout-method thread ${SK:+-k "$SK"} > gpurun_out/b/pytest_state.log 2>&1 || { tail -30 gpurun_out/b/pytest_state.log; exit 13; }
tail -25 gpurun_out/b/pytest_state.log
exit 0
