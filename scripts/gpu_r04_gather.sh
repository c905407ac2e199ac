# Round-4: the obs gather at world 1 through RCCL (bench.py --gather under WORLD_SIZE=1: ObsGather's
# all_gather_into_tensor on its comm stream), a paired line without it, a rocprofv3 kernel + memory-copy
# trace of the gather run (does the comm-stream work overlap the next act?), and a runtime trace of the
# host-buffer path (where do host_path's milliseconds go beyond the 805 MB D2H copy?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/gather; mkdir -p $OUT
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531
timeout -k 10 300 python3 bench.py --gather --host-steps 0 --no-cpu-baseline > $OUT/gather.json 2> $OUT/gather.err || { tail -5 $OUT/gather.err; exit 11; }
python3 -c "import json; d=json.load(open('$OUT/gather.json')); print('gather', round(d['value']/1e6,2), d['ms_per_step'], d['config']['gather'])"
unset WORLD_SIZE RANK LOCAL_RANK
timeout -k 10 300 python3 bench.py --host-steps 0 --no-cpu-baseline > $OUT/nogather.json 2> $OUT/nogather.err || { tail -5 $OUT/nogather.err; exit 12; }
python3 -c "import json; d=json.load(open('$OUT/nogather.json')); print('no gather', round(d['value']/1e6,2), d['ms_per_step'])"
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_PORT=29532
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --gather --steps 20 --warmup 5 --settle 20 --host-steps 0 --no-cpu-baseline > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 13; }
unset WORLD_SIZE RANK LOCAL_RANK
timeout -k 10 300 rocprofv3 --runtime-trace --stats --output-format csv -d $OUT/host -o run -- python3 bench.py --steps 2 --warmup 1 --settle 1 --host-steps 6 --no-cpu-baseline > $OUT/host.json 2> $OUT/host.err || { tail -5 $OUT/host.err; exit 14; }
python3 -c "import json; d=json.load(open('$OUT/host.json')); print('host', d['host_path'])"
find $OUT -name "*.csv" | head -20
