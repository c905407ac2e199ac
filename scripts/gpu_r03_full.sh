# Round-3 GPU call: the whole parity suite, the default bench line, per-game + mixed-16 lines.
#   STEPS=tests,golden,bench,games (default: tests,bench,games); GAMES overrides the per-game list
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/games
S=${STEPS:-tests,bench,games}
if [[ $S == *tests* ]]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [[ $rc != 0 ]] && exit $rc
fi
if [[ $S == *golden* ]]; then
  timeout -k 10 300 python3 -u scripts/make_state_golden.py gpurun_out/upstream_states.npz > gpurun_out/golden.log 2>&1 || { tail -5 gpurun_out/golden.log; exit 11; }
fi
if [[ $S == *bench* ]]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --host-steps 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('coinrun', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  [[ $rc != 0 ]] && exit $rc
fi
if [[ $S == *games* ]]; then
  OUT=gpurun_out/games
  for g in ${GAMES:-jumper caveflyer leaper maze heist starpilot bossfight fruitbot}; do
    timeout -k 10 120 python3 bench.py --env-name $g --steps 50 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > $OUT/$g.json 2> $OUT/$g.err || { tail -5 $OUT/$g.err; exit 12; }
    python3 -c "import json; d=json.load(open('$OUT/$g.json')); print('$g', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  done
  M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
  timeout -k 10 200 python3 bench.py --env-name $M --steps 100 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > $OUT/mixed16.json 2> $OUT/mixed16.err || { tail -5 $OUT/mixed16.err; exit 13; }
  python3 -c "import json; d=json.load(open('$OUT/mixed16.json')); print('mixed16', round(d['value']/1e6,2), d['roofline']['kernel_ms']['step_wall'])"
fi
exit 0
