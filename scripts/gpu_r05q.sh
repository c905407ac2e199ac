# Round-5 (q): the reset RNG's register window (every game's level generation draws through it): parity
# over every game (test_gpu_games, the mixed / prefetch / state tests), phase stamps, bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/q
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_games.py tests/test_gpu_prefetch.py tests/test_gpu_c5.py tests/test_gpu_genassets.py tests/test_gpu_state.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 11; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 scripts/reset_phases.py jumper caveflyer leaper > $O/reset_phases.json 2> $O/reset_phases.err || { tail -5 $O/reset_phases.err; exit 12; }
python3 -c "
import json
for b in open('$O/reset_phases.json').read().split('}\n{'):
    b = b if b.startswith('{') else '{' + b
    b = b if b.rstrip().endswith('}') else b + '}'
    d = json.loads(b); print(d['game'], d['total_cycles_per_reset'], d['slowest_env_cycles_per_reset'], d['cycles_per_reset'])
" || true
ab() { # name env-assignments game steps
  env $2 timeout -k 10 200 python3 bench.py --env-name $3 --steps $4 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,2), d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms'].items() if k != 'per_game'})"
}
M=bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot
ab mixed16 "A=0" $M 100 || exit 13
python3 -c "import json; d=json.load(open('$O/mixed16.json'))['roofline']['kernel_ms']['per_game']; print(sorted(((round(v[1], 3), g) for g, v in d.items()), reverse=True))"
for g in leaper jumper caveflyer maze heist chaser coinrun; do ab $g "A=0" $g 100 || exit 13; done
