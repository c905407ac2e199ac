# (measured in round 4 and removed: the knob no longer exists; kept as the record of profiles/r04/r04_r_copy)
# Round-4: host-buffer obs copies on each part's own chain stream (PROCGEN_MI355X_COPY_ON_CHAIN=2)
# against the copy stream: host-path parity with the knob, host_path lines, and a kernel + memory-copy
# trace with the knob (blit or SDMA?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s; mkdir -p $O
PROCGEN_MI355X_COPY_ON_CHAIN=2 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "boundary or parts or coinrun" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [[ $rc != 0 ]] && exit $rc
h() { env $2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 10 --settle 20 --host-steps 40 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); h=d['host_path']; print('$1', h['reuse_arrays'], h['reuse_obs_GBps'], h['value'])"; }
h chain1 "PROCGEN_MI355X_COPY_ON_CHAIN=2" || exit 11
h cstream1 "A=0" || exit 11
h chain2 "PROCGEN_MI355X_COPY_ON_CHAIN=2" || exit 11
PROCGEN_MI355X_COPY_ON_CHAIN=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 --settle 1 --host-steps 8 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 12; }
exit 0
