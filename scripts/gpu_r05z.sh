# Round-5 (z): mixed-shard packing with the r04 table and the heaviest chains (jumper, bossfight)
# weighted up so they share their streams with fewer chains; alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/z
mkdir -p $O
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'])"
}
M=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
R04=0.21,0.85,1.13,0.67,0.46,0.50,0.66,0.74,0.49,1.45,0.99,0.51,0.51,0.47,0.35,0.67
J20=0.21,0.85,1.13,0.67,0.46,0.50,0.66,0.74,0.49,2.00,0.99,0.51,0.51,0.47,0.35,0.67
JB=0.21,1.30,1.13,0.67,0.46,0.50,0.66,0.74,0.49,1.80,0.99,0.51,0.51,0.47,0.35,0.67
C08=0.21,0.85,0.80,0.67,0.46,0.50,0.66,0.74,0.49,1.45,0.99,0.51,0.51,0.47,0.35,0.67
for i in 1 2; do
  for v in R04 J20 JB C08; do ab mixed16_${v}_$i "PROCGEN_MI355X_MIXED_COSTS=${!v}" $M 100 || exit 13; done
done
