# Round-3 call after reverting the persistent-grid attempt: parity suite, the driver's default bench
# line (host path + cpu baseline included), the mixed-16 shard with / without level prefetch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[[ $rc != 0 ]] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 11; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(round(d['value']/1e6,2), d['roofline']['kernel_ms'], d['host_path'], d['cpu_baseline'])"
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
CFGS="PROCGEN_MI355X_PREFETCH=0 PROCGEN_MI355X_PREFETCH=1" STEPS=100 GAMES=$M bash scripts/gpu_ab.sh
CENSUS_WARM=350 timeout -k 10 300 python3 scripts/census.py coinrun > gpurun_out/census350.json 2> gpurun_out/census350.err || { tail -5 gpurun_out/census350.err; exit 14; }
python3 -c "
import json
d=json.load(open('gpurun_out/census350.json'))[0]
s=d['step']; print('census350 step span', s['span_us'], s['lifetime_us'], s['dispatch'], 'slowest starts', d['start_us_of_slowest'])
"
