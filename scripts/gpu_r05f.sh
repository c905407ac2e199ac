# Round-5 (f): the state-test port for all 16 games, the rf parity file, then bench lines: the driver's
# default (coinrun), the all-16 mixed shard, and the games whose default render changed.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/f
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_state_rollouts.py tests/test_gpu_render_rf.py -x -v --durations=20 --timeout 600 --timeout-method thread > gpurun_out/f/pytest.log 2>&1 || { tail -40 gpurun_out/f/pytest.log; exit 11; }
tail -25 gpurun_out/f/pytest.log
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/f/$1.json 2> gpurun_out/f/$1.err || { tail -5 gpurun_out/f/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
ab coinrun "A=0" coinrun 100 || exit 12
ab mixed16 "A=0" bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot 100 || exit 12
ab mixed16_lds "PROCGEN_MI355X_RENDER_RF=0" bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot 100 || exit 12
exit 0
