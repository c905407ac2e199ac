# Round-5 (y): the mixed shard's level prefetch again after the round-5 generators (prefetch stream /
# in band, for the two slowest generators), alternating with the default on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/y
mkdir -p $O
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
M=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
for i in 1 2; do
  ab mixed16_$i "A=0" $M 100 || exit 13
  ab mixed16_pf_jl_$i "PROCGEN_MI355X_PREFETCH_GAMES=jumper,leaper" $M 100 || exit 13
  ab mixed16_ib_jl_$i "PROCGEN_MI355X_PREFETCH_GAMES=jumper,leaper PROCGEN_MI355X_PREFETCH_INBAND=1" $M 100 || exit 13
done
