# Round-3 final call: smoke, the parity suite, the driver's default bench line, the coinrun rocprofv3
# kernel stats + counter passes (the roofline's traffic), the all-16 mixed shard.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 10; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[[ $rc != 0 ]] && exit $rc
GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 21; }
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 11; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(round(d['value']/1e6,2), d['roofline'], d['host_path'], d['cpu_baseline'])"
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
timeout -k 10 200 python3 bench.py --env-name $M --steps 100 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > gpurun_out/mixed16.json 2> gpurun_out/mixed16.err || { tail -5 gpurun_out/mixed16.err; exit 13; }
python3 -c "import json; d=json.load(open('gpurun_out/mixed16.json')); print('mixed16', round(d['value']/1e6,2))"
PROCGEN_MI355X_MIXED_STREAMS=4 timeout -k 10 200 python3 bench.py --env-name $M --steps 100 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > gpurun_out/mixed16_ms4.json 2> gpurun_out/mixed16_ms4.err || { tail -5 gpurun_out/mixed16_ms4.err; exit 14; }
python3 -c "import json; d=json.load(open('gpurun_out/mixed16_ms4.json')); print('mixed16 4 streams', round(d['value']/1e6,2))"
