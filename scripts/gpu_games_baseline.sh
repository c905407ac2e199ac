# Per-game diagnostics: phase shares (PG_PROFILE build) + a short device-resident bench line per game.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/games; mkdir -p $OUT
GAMES=${GAMES:-"bigfish bossfight caveflyer chaser climber coinrun dodgeball fruitbot heist jumper leaper maze miner ninja plunder starpilot"}
if [ "${PHASE:-1}" = 1 ]; then timeout -k 10 400 python3 scripts/phase_profile.py $GAMES > $OUT/phase.json 2> $OUT/phase.err || { tail -5 $OUT/phase.err; exit 11; }; fi
for g in $GAMES; do
  timeout -k 10 120 python3 bench.py --env-name $g --steps ${STEPS:-50} --warmup 20 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline > $OUT/$g.json 2> $OUT/$g.err || { tail -5 $OUT/$g.err; exit 12; }
  python3 -c "import json; d=json.load(open('$OUT/$g.json')); print('$g', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
done
