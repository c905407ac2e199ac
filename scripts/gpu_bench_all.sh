# Bench lines for every BASELINE config that fits one GPU (configs[1..3] + the maze/heist mix).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/bench
S=${STEPS:-200}; W=${WARMUP:-50}
timeout -k 10 300 python3 bench.py --steps $S --warmup $W > gpurun_out/bench/coinrun.json 2> gpurun_out/bench/coinrun.err && \
timeout -k 10 300 python3 bench.py --env-name bigfish --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/bigfish.json 2> gpurun_out/bench/bigfish.err && \
timeout -k 10 300 python3 bench.py --env-name maze --num-envs 32768 --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/maze.json 2> gpurun_out/bench/maze.err && \
timeout -k 10 300 python3 bench.py --env-name heist --num-envs 32768 --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/heist.json 2> gpurun_out/bench/heist.err && \
timeout -k 10 300 python3 bench.py --env-name maze,heist --num-envs 65536 --steps $S --warmup $W --no-cpu-baseline > gpurun_out/bench/maze_heist.json 2> gpurun_out/bench/maze_heist.err
rc=$?
for f in gpurun_out/bench/*.json; do echo "== $f"; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['config']['env_name'], d['roofline']['kernel_ms'])" ; done
tail -2 gpurun_out/bench/*.err
exit $rc
