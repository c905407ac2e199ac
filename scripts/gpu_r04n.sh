# Round-4: where the host-buffer path's time goes: kernel + memory-copy trace of bench.py's host_path
# (coinrun 65,536 envs, reuse_arrays and copy semantics), copies > 1 MB with their rates and gaps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/n; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/host -o run -- python3 bench.py --steps 2 --warmup 1 --settle 1 --host-steps 8 --no-cpu-baseline > $O/host.json 2> $O/host.err || { tail -5 $O/host.err; exit 11; }
python3 -c "import json; d=json.loads(open('$O/host.json').read().strip().splitlines()[-1]); print(d['host_path'])"
python3 scripts/host_copies.py $O/host > $O/copies.txt || exit 12
tail -60 $O/copies.txt
