# Round-4 closing verification: smoke, the full -m gpu suite and the driver's default bench line
# (scripts/gpu_r04.sh), then the D2H engine probe (scripts/d2h_probe.hip) plain and under a kernel +
# memory-copy trace.  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_r04.sh || exit $?
mkdir -p gpurun_out/p
timeout -k 10 60 ./scripts/d2h_probe || exit 20
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/p/trace -o run -- ./scripts/d2h_probe > gpurun_out/p/probe.log 2>&1 || { tail -5 gpurun_out/p/probe.log; exit 21; }
exit 0
