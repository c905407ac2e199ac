# Round-5 (l): which engine carries the host-path D2H copy after kernels (scripts/d2h_probe2.hip under
# the kernel + memory-copy trace), and the level-generation phases of caveflyer / jumper (rprof build).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/l
mkdir -p $O
timeout -k 10 120 scripts/d2h_probe2 > $O/d2h_probe2.txt 2>&1 || exit 11
cat $O/d2h_probe2.txt
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/d2h -o run -- scripts/d2h_probe2 > $O/d2h_prof.log 2>&1 || { tail -5 $O/d2h_prof.log; exit 12; }
timeout -k 10 300 python3 scripts/reset_phases.py jumper caveflyer > $O/reset_phases.json 2> $O/reset_phases.err || { tail -5 $O/reset_phases.err; exit 13; }
cat $O/reset_phases.json
exit 0
