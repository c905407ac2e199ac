# Diagnostic: the state tests (which met a sticky "illegal memory access" at the bossfight make in
# the full suite) with kernels serialized, so a fault names its launch; then the crate-pile tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_state.py -x -v --timeout 200 --timeout-method thread > gpurun_out/diag_state.log 2>&1
rc=$?; tail -5 gpurun_out/diag_state.log
[[ $rc != 0 ]] && exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_coinrun.py -x -q --timeout 200 --timeout-method thread -k "crate or full_size or fixture" > gpurun_out/crate.log 2>&1
rc=$?; tail -3 gpurun_out/crate.log
exit $rc
