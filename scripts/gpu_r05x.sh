# Round-5 (x): bench.py's stdout is the JSON line alone, also under torchrun with RCCL (--gather at
# world 1), and the driver's default command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/x
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gather --steps 50 --warmup 10 --no-cpu-baseline > $O/gather.json 2> $O/gather.err || { tail -5 $O/gather.err; exit 11; }
wc -l $O/gather.json
python3 -c "import json; d=json.load(open('$O/gather.json')); print('gather', round(d['value']/1e6,2), d['config'].get('gather'))"
timeout -k 10 600 python3 bench.py > $O/default.json 2> $O/default.err || { tail -5 $O/default.err; exit 12; }
wc -l $O/default.json
python3 -c "import json; d=json.load(open('$O/default.json')); print('default', round(d['value']/1e6,2), d['cpu_baseline']['value'], d['roofline']['traffic_source'])"
