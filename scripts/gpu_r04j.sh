# Round-4: verification of the default build (smoke, full -m gpu suite, the driver's default bench line,
# coinrun counters), then fruitbot's tight aux (default now) against the r04_d-era build (old), and the
# world-1 gather with 4 vs 8 hardware queues.  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/j
bash scripts/gpu_r04.sh || exit $?
GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 12; }
ab() { # name env-assignments game steps [extra bench args]
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline $5 > gpurun_out/j/$1.json 2> gpurun_out/j/$1.err || { tail -5 gpurun_out/j/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/j/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
ab fruitbot_default "A=0" fruitbot 50 || exit 13
ab fruitbot_old "PROCGEN_MI355X_LIB=old" fruitbot 50 || exit 13
ab bossfight_default "A=0" bossfight 50 || exit 13
W="WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1"
ab gather_q4 "$W MASTER_PORT=29541" coinrun 100 --gather || exit 13
ab gather_q8 "$W MASTER_PORT=29542 GPU_MAX_HW_QUEUES=8" coinrun 100 --gather || exit 13
ab coinrun_q8 "GPU_MAX_HW_QUEUES=8" coinrun 100 || exit 13
exit 0
