# Round-4: the world-1 RCCL obs gather with 4 vs 8 hardware queues (bench lines + rocprofv3 kernel traces,
# overlap of the gather's copy with the engine's kernels from scripts/gather_overlap.py), and coinrun
# without the gather at 8 queues.  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/k; mkdir -p $O
last() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['value']/1e6,2), d['ms_per_step'])"; }
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
for q in 4 8; do
  MASTER_PORT=2955$q GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --gather --steps 100 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/gather_q$q.json 2> $O/gather_q$q.err || { tail -5 $O/gather_q$q.err; exit 11; }
  last $O/gather_q$q.json gather_q$q || exit 11
  MASTER_PORT=2956$q GPU_MAX_HW_QUEUES=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_q$q -o run -- python3 bench.py --gather --steps 20 --warmup 5 --settle 20 --host-steps 0 --no-cpu-baseline > $O/trace_q$q.json 2> $O/trace_q$q.err || { tail -5 $O/trace_q$q.err; exit 12; }
  python3 scripts/gather_overlap.py $(ls $O/trace_q$q/*kernel_trace.csv $O/trace_q$q/*/*kernel_trace.csv 2>/dev/null | head -1) $O/overlap_q$q.json || exit 13
done
unset WORLD_SIZE RANK LOCAL_RANK
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > $O/coinrun_q8.json 2> $O/coinrun_q8.err || { tail -5 $O/coinrun_q8.err; exit 14; }
last $O/coinrun_q8.json coinrun_q8
