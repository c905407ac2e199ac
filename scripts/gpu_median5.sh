# coinrun 65,536 envs, 1000 timed steps, median of 5 runs (each run its own process).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/median5
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --steps 1000 --warmup 50 --settle 300 --host-steps 0 --no-cpu-baseline > gpurun_out/median5/run$i.json 2> gpurun_out/median5/run$i.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/median5/run$i.json')); print($i, d['value'], d['ms_per_step'])"
done
