# Round-5 (g): the state-test port for miner (states without an agent), bench lines (driver default,
# mixed 16 with and without the register-frame render), the per-game CPU baseline table on this box's
# cores, and render_mode="rgb_array" (bench + rocprofv3 stats + FETCH / WRITE passes of the hires kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/g
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_state_rollouts.py -x -v --timeout 600 --timeout-method thread -k miner > gpurun_out/g/pytest_miner.log 2>&1 || { tail -30 gpurun_out/g/pytest_miner.log; exit 11; }
tail -2 gpurun_out/g/pytest_miner.log
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/g/$1.json 2> gpurun_out/g/$1.err || { tail -5 gpurun_out/g/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
ab coinrun "A=0" coinrun 100 || exit 12
M=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
ab mixed16 "A=0" $M 100 || exit 12
ab mixed16_lds "PROCGEN_MI355X_RENDER_RF=0" $M 100 || exit 12
timeout -k 10 300 python3 scripts/cpu_baseline_table.py > gpurun_out/g/cpu_baseline_games.json 2> gpurun_out/g/cpu_baseline_games.err || { tail -5 gpurun_out/g/cpu_baseline_games.err; exit 13; }
cat gpurun_out/g/cpu_baseline_games.err
for g in coinrun bossfight; do
  timeout -k 10 300 python3 scripts/bench_rgb_array.py --env-name $g --num-envs 4096 --steps 4 > gpurun_out/g/rgb_$g.json 2> gpurun_out/g/rgb_$g.err || { tail -5 gpurun_out/g/rgb_$g.err; exit 14; }
  cat gpurun_out/g/rgb_$g.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g/rgbprof_$g -o run -- python3 scripts/bench_rgb_array.py --env-name $g --num-envs 4096 --steps 2 > gpurun_out/g/rgbprof_$g.log 2>&1 || exit 15
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/g/rgbfetch_$g -o run -- python3 scripts/bench_rgb_array.py --env-name $g --num-envs 4096 --steps 2 > gpurun_out/g/rgbfetch_$g.log 2>&1 || exit 16
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/g/rgbwrite_$g -o run -- python3 scripts/bench_rgb_array.py --env-name $g --num-envs 4096 --steps 2 > gpurun_out/g/rgbwrite_$g.log 2>&1 || exit 17
done
exit 0
