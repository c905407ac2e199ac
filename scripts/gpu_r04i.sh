# A/B of the current default build (obs-copy stream created lazily) against the r04_d build
# (PROCGEN_MI355X_LIB=old, commit 7f27173) on coinrun and the mixed-16 shard, then the host path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/i
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/i/$1.json 2> gpurun_out/i/$1.err || { tail -5 gpurun_out/i/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/i/$1.json')); print('$1', round(d['value']/1e6,2), {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
ab coinrun_default "A=0" coinrun 200 || exit 13
ab coinrun_old "PROCGEN_MI355X_LIB=old" coinrun 200 || exit 13
ab mixed16_default "A=0" $M 50 || exit 13
ab mixed16_old "PROCGEN_MI355X_LIB=old" $M 50 || exit 13
ab coinrun_default2 "A=0" coinrun 200 || exit 13
timeout -k 10 300 python3 bench.py --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/i/host_default.json 2> gpurun_out/i/host_default.err || { tail -5 gpurun_out/i/host_default.err; exit 14; }
python3 -c "import json; d=json.load(open('gpurun_out/i/host_default.json')); print('host', round(d['value']/1e6,2), d.get('host_path'))"
exit 0
