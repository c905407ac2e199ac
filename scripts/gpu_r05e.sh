# Round-5 (e): the fused step + render kernel (pg_fused.hip, PROCGEN_MI355X_FUSED=1) -- coinrun parity
# with it on, then bench lines against the unfused register-frame render, 1 and 2 parts.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/e
PROCGEN_MI355X_FUSED=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_coinrun.py tests/test_gpu_parts.py -x -v --timeout 300 --timeout-method thread -k "coinrun or parts" > gpurun_out/e/pytest_fused.log 2>&1 || { tail -30 gpurun_out/e/pytest_fused.log; exit 11; }
tail -2 gpurun_out/e/pytest_fused.log
STEPS=100 SETTLE=200 CFGS="${CFGS:-PROCGEN_MI355X_PARTS=1 PROCGEN_MI355X_FUSED=1,PROCGEN_MI355X_PARTS=1 PROCGEN_MI355X_FUSED=1 PROCGEN_MI355X_FUSED=1,PROCGEN_MI355X_PARTS=3 -}" bash scripts/gpu_ab.sh || exit 12
exit 0
