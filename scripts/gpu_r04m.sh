# Round-4: mixed batches with the chains packed by LPT + swaps and only the used streams created,
# parity of every mixed-batch test, then the all-16 shard with the chains enqueued in game-id order (default) vs cheapest first (asc).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/m; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mixed or heist or prefetch or parts" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [[ $rc != 0 ]] && exit $rc
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']/1e6,2), d['ms_per_step'])"
}
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
ab mixed16_default "A=0" $M 200 || exit 13
ab mixed16_asc "PROCGEN_MI355X_MIXED_ORDER=asc" $M 200 || exit 13
ab mixed16_default2 "A=0" $M 200 || exit 13
ab maze_heist "A=0" maze,heist 100 || exit 13
ab coinrun "A=0" coinrun 200 || exit 13
exit 0
