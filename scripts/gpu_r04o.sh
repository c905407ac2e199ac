# Round-4: host-buffer path (part copies in finish order, part 0 behind part 1's render): parity of the host-path tests,
# two host_path bench lines, and a kernel + memory-copy trace of the same (scripts/host_copies.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/o; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "boundary or host or gym3 or adapters or buffers or parts or coinrun" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [[ $rc != 0 ]] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 10 --settle 20 --host-steps 40 --no-cpu-baseline > $O/host$i.json 2> $O/host$i.err || { tail -5 $O/host$i.err; exit 11; }
  python3 -c "import json; d=json.loads(open('$O/host$i.json').read().strip().splitlines()[-1]); h=d['host_path']; print('host$i', h['reuse_arrays'], h['reuse_obs_GBps'], h['value'], h['pcie_d2h_GBps'])"
done
PROCGEN_MI355X_HOST_SERIAL=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 10 --settle 20 --host-steps 40 --no-cpu-baseline > $O/host_noserial.json 2> $O/host_noserial.err || exit 13
python3 -c "import json; d=json.loads(open('$O/host_noserial.json').read().strip().splitlines()[-1]); h=d['host_path']; print('noserial', h['reuse_arrays'], h['reuse_obs_GBps'])"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 --settle 1 --host-steps 8 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 12; }
exit 0
