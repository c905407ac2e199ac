# Round-5 (k): in-band level prefetch for the mixed shard (parity, then mixed16 A/B: default, prefetch on
# a fifth stream for caveflyer/jumper/leaper, the same in band), coinrun register-frame render with LDS
# padding (occupancy cap) in 2 parts, rgb_array after the page-locked DMA, default coinrun counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/k
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefetch.py -x -v --timeout 120 --timeout-method thread -k mixed > $O/pytest_prefetch.log 2>&1 || { tail -30 $O/pytest_prefetch.log; exit 11; }
tail -2 $O/pytest_prefetch.log
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
M=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
ab mixed16 "A=0" $M 100 || exit 12
ab mixed16_pf3 "PROCGEN_MI355X_PREFETCH_GAMES=caveflyer,jumper,leaper" $M 100 || exit 12
ab mixed16_ib3 "PROCGEN_MI355X_PREFETCH_GAMES=caveflyer,jumper,leaper PROCGEN_MI355X_PREFETCH_INBAND=1" $M 100 || exit 12
ab mixed16_ib2 "PROCGEN_MI355X_PREFETCH_GAMES=caveflyer,jumper PROCGEN_MI355X_PREFETCH_INBAND=1" $M 100 || exit 12
ab mixed16_ib4 "PROCGEN_MI355X_PREFETCH_GAMES=caveflyer,jumper,leaper,starpilot PROCGEN_MI355X_PREFETCH_INBAND=1" $M 100 || exit 12
ab coinrun "A=0" coinrun 100 || exit 13
ab coinrun_rf2 "PROCGEN_MI355X_RENDER_RF=coinrun PROCGEN_MI355X_PARTS=2" coinrun 100 || exit 13
ab coinrun_rf2_pad2k "PROCGEN_MI355X_RENDER_RF=coinrun PROCGEN_MI355X_PARTS=2 PROCGEN_MI355X_LIB=rfpad2k" coinrun 100 || exit 13
ab coinrun_rf2_pad4k "PROCGEN_MI355X_RENDER_RF=coinrun PROCGEN_MI355X_PARTS=2 PROCGEN_MI355X_LIB=rfpad4k" coinrun 100 || exit 13
ab coinrun_cr16 "PROCGEN_MI355X_LIB=cr16" coinrun 100 || exit 13
ab coinrun_again "A=0" coinrun 100 || exit 13
for g in coinrun bossfight; do
  timeout -k 10 300 python3 scripts/bench_rgb_array.py --env-name $g --num-envs 4096 --steps 4 > $O/rgb_$g.json 2> $O/rgb_$g.err || { tail -5 $O/rgb_$g.err; exit 14; }
  cat $O/rgb_$g.json
done
GAMES=coinrun timeout -k 10 900 bash scripts/gpu_counters.sh > $O/counters.log 2>&1 || { tail -5 $O/counters.log; exit 15; }
tail -3 $O/counters.log
exit 0
