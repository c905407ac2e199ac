# Bench lines beyond the default: the all-16-game mixed shard of configs[4] (65,536 envs on one GPU),
# every game alone (65,536 envs), and the RCCL obs all-gather path through torchrun (1 rank).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/bench
S=${STEPS:-100}; W=${WARMUP:-20}
ALL=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
timeout -k 10 300 python3 bench.py --env-name $ALL --num-envs 65536 --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/mixed16.json 2> gpurun_out/bench/mixed16.err || exit $?
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gather --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/coinrun_gather.json 2> gpurun_out/bench/coinrun_gather.err || exit $?
for g in ${GAMES:-bigfish bossfight caveflyer chaser climber dodgeball fruitbot heist jumper leaper maze miner ninja plunder starpilot}; do
  timeout -k 10 300 python3 bench.py --env-name $g --num-envs 65536 --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/$g.json 2> gpurun_out/bench/$g.err || exit $?
done
for f in gpurun_out/bench/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('%-16s %12.0f' % ('$f'.split('/')[-1][:-5], d['value']), d['roofline']['kernel_ms'])"; done
