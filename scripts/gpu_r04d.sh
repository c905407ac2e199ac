# Round-4 verification call: the coinrun pixel diff, smoke + the -m gpu suite, every game alone and the
# mixed-16 shard (gpu_r03_games.sh), the mixed-16 shard without the per-game level prefetch (A/B), then
# the gather / host-path traces (gpu_r04_gather.sh).  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python3 scripts/diag_stamp.py coinrun 8 2>&1 | grep "diff px"
BENCH=0 bash scripts/gpu_r04.sh || exit $?
bash scripts/gpu_r03_games.sh > gpurun_out/games.log 2>&1 || { tail -5 gpurun_out/games.log; exit 14; }
cat gpurun_out/games.log
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
PROCGEN_MI355X_PREFETCH=0 timeout -k 10 200 python3 bench.py --env-name $M --steps 50 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > gpurun_out/games/mixed16_noprefetch.json 2> gpurun_out/games/mixed16_noprefetch.err || exit 15
python3 -c "import json; d=json.load(open('gpurun_out/games/mixed16_noprefetch.json')); print('mixed16 no prefetch', round(d['value']/1e6,2), d['roofline']['kernel_ms']['step_wall'])"
[[ "${GATHER:-1}" == 1 ]] && { bash scripts/gpu_r04_gather.sh || exit $?; }
exit 0
