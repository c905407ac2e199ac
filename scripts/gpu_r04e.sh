# Round-4: the -m gpu suite (the obs DMA moved to its own copy stream), the host-buffer path line, then
# an A/B of the HIP runtime's hardware queues (GPU_MAX_HW_QUEUES) against streams / parts for coinrun
# and the mixed-16 shard, and the world-1 gather under more queues.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/e
if [[ "${TESTS:-1}" == 1 ]]; then
  BENCH=0 bash scripts/gpu_r04.sh || exit $?
fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --settle 20 --host-steps 24 --no-cpu-baseline > gpurun_out/e/host.json 2> gpurun_out/e/host.err || { tail -5 gpurun_out/e/host.err; exit 11; }
python3 -c "import json; d=json.load(open('gpurun_out/e/host.json')); print('host', d['host_path'])"
M="bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,miner,ninja,plunder,starpilot"
for c in "-" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8,PROCGEN_MI355X_PARTS=4" "GPU_MAX_HW_QUEUES=16,PROCGEN_MI355X_PARTS=4"; do
  a=${c//,/ }; [[ $c == - ]] && a=""
  env $a timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --settle 300 --host-steps 0 --no-cpu-baseline > gpurun_out/e/coinrun.$c.json 2> gpurun_out/e/coinrun.$c.err || { tail -5 gpurun_out/e/coinrun.$c.err; exit 12; }
  python3 -c "import json; d=json.load(open('gpurun_out/e/coinrun.$c.json')); print('coinrun', '$c', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
done
for c in "-" "GPU_MAX_HW_QUEUES=8,PROCGEN_MI355X_MIXED_STREAMS=8" "GPU_MAX_HW_QUEUES=16,PROCGEN_MI355X_MIXED_STREAMS=16"; do
  a=${c//,/ }; [[ $c == - ]] && a=""
  env $a timeout -k 10 200 python3 bench.py --env-name $M --steps 50 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > gpurun_out/e/mixed16.$c.json 2> gpurun_out/e/mixed16.$c.err || { tail -5 gpurun_out/e/mixed16.$c.err; exit 13; }
  python3 -c "import json; d=json.load(open('gpurun_out/e/mixed16.$c.json')); print('mixed16', '$c', round(d['value']/1e6,2), d['roofline']['kernel_ms']['step_wall'])"
done
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --gather --host-steps 0 --no-cpu-baseline > gpurun_out/e/gather_q8.json 2> gpurun_out/e/gather_q8.err || { tail -5 gpurun_out/e/gather_q8.err; exit 14; }
python3 -c "import json; d=json.load(open('gpurun_out/e/gather_q8.json')); print('gather q8', round(d['value']/1e6,2), d['ms_per_step'])"
PROCGEN_MI355X_LIB=rows timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --settle 300 --host-steps 0 --no-cpu-baseline > gpurun_out/e/coinrun.rows.json 2> gpurun_out/e/coinrun.rows.err || { tail -5 gpurun_out/e/coinrun.rows.err; exit 16; }
python3 -c "import json; d=json.load(open('gpurun_out/e/coinrun.rows.json')); print('coinrun lib=rows', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
PROCGEN_MI355X_LIB=rows timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "coinrun or hard_unbounded or ninja or maze" > gpurun_out/e/pytest_rows.log 2>&1; rc=$?; tail -2 gpurun_out/e/pytest_rows.log; [[ $rc != 0 ]] && exit $rc
for g in bossfight fruitbot; do
  for L in "" aux; do
    PROCGEN_MI355X_LIB=$L timeout -k 10 200 python3 bench.py --env-name $g --steps 50 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > gpurun_out/e/$g.$L.json 2> gpurun_out/e/$g.$L.err || { tail -5 gpurun_out/e/$g.$L.err; exit 15; }
    python3 -c "import json; d=json.load(open('gpurun_out/e/$g.$L.json')); print('$g', 'lib=$L', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  done
done
for g in coinrun bossfight; do
  PROCGEN_MI355X_LIB=k2 timeout -k 10 200 python3 bench.py --env-name $g --steps 100 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/e/$g.k2.json 2> gpurun_out/e/$g.k2.err || { tail -5 gpurun_out/e/$g.k2.err; exit 18; }
  python3 -c "import json; d=json.load(open('gpurun_out/e/$g.k2.json')); print('$g', 'lib=k2', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
done
PROCGEN_MI355X_LIB=stamp timeout -k 10 300 python3 scripts/phase_profile.py bossfight fruitbot coinrun > gpurun_out/e/stamp.json 2> gpurun_out/e/stamp.err || { tail -3 gpurun_out/e/stamp.err; exit 17; }
exit 0
