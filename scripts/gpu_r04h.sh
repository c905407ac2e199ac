# Round-4 closing call, by priority: smoke + the -m gpu suite on the current default build, the
# driver's default bench line, the coinrun counter passes, then A/Bs of the experiment builds
# (PROCGEN_MI355X_LIB=rows / aux / k2 / rb16) and of GPU_MAX_HW_QUEUES=8.  The first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/h
bash scripts/gpu_r04.sh || exit $?
GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 12; }
python3 -c "import json; d=json.load(open('gpurun_out/ctr/summary.json'))['coinrun']; print({k: (v.get('avg_ms'), v.get('hbm_bytes_per_part_act'), v.get('scratch')) for k, v in d.items()})"
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/h/$1.json 2> gpurun_out/h/$1.err || { tail -5 gpurun_out/h/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/h/$1.json')); print('$1', round(d['value']/1e6,2), d['roofline']['kernel_ms'].get('step_wall'), {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
ab coinrun_default "A=0" coinrun 200 || exit 13
ab coinrun_rows "PROCGEN_MI355X_LIB=rows" coinrun 200 || exit 13
ab coinrun_rb16 "PROCGEN_MI355X_LIB=rb16" coinrun 200 || exit 13
ab coinrun_k2 "PROCGEN_MI355X_LIB=k2" coinrun 200 || exit 13
ab coinrun_q8 "GPU_MAX_HW_QUEUES=8" coinrun 200 || exit 13
ab mixed16_default "A=0" $M 50 || exit 13
ab mixed16_q8s8 "GPU_MAX_HW_QUEUES=8 PROCGEN_MI355X_MIXED_STREAMS=8" $M 50 || exit 13
ab bossfight_default "A=0" bossfight 50 || exit 13
ab bossfight_aux "PROCGEN_MI355X_LIB=aux" bossfight 50 || exit 13
ab bossfight_k2 "PROCGEN_MI355X_LIB=k2" bossfight 50 || exit 13
ab fruitbot_aux "PROCGEN_MI355X_LIB=aux" fruitbot 50 || exit 13
ab maze_rb16 "PROCGEN_MI355X_LIB=rb16" maze 50 || exit 13
ab maze_default "A=0" maze 50 || exit 13
PROCGEN_MI355X_LIB=rows timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "hard_unbounded or test_gpu_coinrun" > gpurun_out/h/pytest_rows.log 2>&1; rc=$?; tail -2 gpurun_out/h/pytest_rows.log; [[ $rc != 0 ]] && exit $rc
exit 0
