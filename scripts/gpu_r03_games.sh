# Round-3 per-game + mixed-16 device-resident bench lines (no phase profile)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/games; mkdir -p $OUT
GAMES=${GAMES:-"bigfish bossfight caveflyer chaser climber coinrun dodgeball fruitbot heist jumper leaper maze miner ninja plunder starpilot"}
for g in $GAMES; do
  timeout -k 10 120 python3 bench.py --env-name $g --steps ${STEPS:-50} --warmup 20 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline > $OUT/$g.json 2> $OUT/$g.err || { tail -5 $OUT/$g.err; exit 12; }
  python3 -c "import json; d=json.load(open('$OUT/$g.json')); print('$g', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
done
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
timeout -k 10 200 python3 bench.py --env-name $M --steps ${STEPS:-50} --warmup 20 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline > $OUT/mixed16.json 2> $OUT/mixed16.err || { tail -5 $OUT/mixed16.err; exit 13; }
python3 -c "import json; d=json.load(open('$OUT/mixed16.json')); print('mixed16', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
