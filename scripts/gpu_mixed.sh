# mixed-16 bench + the C5 parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/games; mkdir -p $OUT
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
timeout -k 10 200 python3 bench.py --env-name $M --steps ${STEPS:-100} --warmup 20 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline > $OUT/mixed16.json 2> $OUT/mixed16.err || { tail -5 $OUT/mixed16.err; exit 13; }
python3 -c "import json; d=json.load(open('$OUT/mixed16.json')); print('mixed16', round(d['value']/1e6,2), d['roofline']['kernel_ms']['step_wall'])"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_c5.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_c5.log; exit $rc
