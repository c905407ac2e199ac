# Round-5 (r): the mixed shard's LPT packing under different chain-cost tables, on one box (box noise
# is a few %): the r04 table, the r05 measured table, render weighted 1.5x / 2x, reset weighted 0.5x.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r
mkdir -p $O
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
M=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
R04=0.21,0.85,1.13,0.67,0.46,0.50,0.66,0.74,0.49,1.45,0.99,0.51,0.51,0.47,0.35,0.67
R05=0.22,0.94,0.62,0.49,0.36,0.57,0.64,0.75,0.41,1.03,0.85,0.54,0.49,0.43,0.42,0.72
W15=0.26,1.29,0.77,0.59,0.44,0.69,0.77,0.97,0.48,1.29,1.03,0.63,0.60,0.54,0.56,0.85
W20=0.30,1.64,0.92,0.70,0.52,0.81,0.91,1.19,0.55,1.56,1.21,0.72,0.70,0.65,0.69,0.98
RS05=0.17,0.91,0.53,0.40,0.33,0.53,0.60,0.64,0.32,0.84,0.65,0.40,0.44,0.39,0.38,0.56
for i in 1 2; do
  for v in R04 R05 W15 W20 RS05; do ab mixed16_${v}_$i "PROCGEN_MI355X_MIXED_COSTS=${!v}" $M 100 || exit 13; done
done
