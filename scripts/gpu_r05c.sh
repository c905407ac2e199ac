# Round-5 (c): the register-frame render for every game -- parity forced on for all games
# (tests/test_gpu_render_rf.py), then per game a bench line with it (RENDER_RF=all) and without it
# (RENDER_RF=0) at 65,536 envs.  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c
if [[ "${TESTS:-1}" == 1 ]]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_render_rf.py -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/c/pytest_rf.log 2>&1 || { tail -40 gpurun_out/c/pytest_rf.log; exit 11; }
  tail -3 gpurun_out/c/pytest_rf.log
fi
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 10 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline > gpurun_out/c/$1.json 2> gpurun_out/c/$1.err || { tail -5 gpurun_out/c/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
for g in ${GAMES:-bigfish bossfight caveflyer chaser climber coinrun dodgeball fruitbot heist jumper leaper maze miner ninja plunder starpilot}; do
  ab ${g}_rf "PROCGEN_MI355X_RENDER_RF=all" $g ${STEPS:-40} || exit 12
  ab ${g}_lds "PROCGEN_MI355X_RENDER_RF=0" $g ${STEPS:-40} || exit 12
done
exit 0
