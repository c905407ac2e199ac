# Round-4: the all-16 mixed shard against the stream count (mixed streams 3 / 4 / 5, the jumper +
# caveflyer level prefetch with and without a freed queue), and 2 parts for bossfight / leaper / dodgeball.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/l; mkdir -p $O
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']/1e6,2), d['ms_per_step'])"
}
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
ab mixed16_default "A=0" $M 100 || exit 13
ab mixed16_s3 "PROCGEN_MI355X_MIXED_STREAMS=3" $M 100 || exit 13
ab mixed16_s5 "PROCGEN_MI355X_MIXED_STREAMS=5" $M 100 || exit 13
ab mixed16_s3_pf "PROCGEN_MI355X_MIXED_STREAMS=3 PROCGEN_MI355X_PREFETCH_GAMES=caveflyer,jumper" $M 100 || exit 13
ab mixed16_s4_pf "PROCGEN_MI355X_PREFETCH_GAMES=caveflyer,jumper" $M 100 || exit 13
ab mixed16_default2 "A=0" $M 100 || exit 13
for g in bossfight leaper dodgeball; do
  ab ${g}_p1 "A=0" $g 50 || exit 13
  ab ${g}_p2 "PROCGEN_MI355X_PARTS=2" $g 50 || exit 13
done
exit 0
