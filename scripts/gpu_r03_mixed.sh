# Mixed batches after packing the chains onto 4 streams: every mixed-batch parity test, the mixed-16 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_c5.py tests/test_gpu_prefetch.py tests/test_gpu_boundary.py tests/test_gpu_adapters.py tests/test_gpu_genassets.py tests/test_gpu_games.py -k "mixed or c5 or c4 or maze_heist or boundary or gym3 or prefetch or adapters or gen or sequence or offset or transfer or atlas or miner" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mixed.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_mixed.log
[[ $rc != 0 ]] && exit $rc
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
timeout -k 10 200 python3 bench.py --env-name $M --steps 200 --warmup 20 --settle 300 --host-steps 0 --no-cpu-baseline > gpurun_out/mixed16.json 2> gpurun_out/mixed16.err || { tail -5 gpurun_out/mixed16.err; exit 13; }
python3 -c "import json; d=json.load(open('gpurun_out/mixed16.json')); print('mixed16', round(d['value']/1e6,2))"
timeout -k 10 200 python3 bench.py --env-name maze,heist --steps 200 --warmup 20 --settle 300 --host-steps 0 --no-cpu-baseline > gpurun_out/maze_heist.json 2> gpurun_out/maze_heist.err || { tail -5 gpurun_out/maze_heist.err; exit 14; }
python3 -c "import json; d=json.load(open('gpurun_out/maze_heist.json')); print('maze+heist', round(d['value']/1e6,2))"
