# run the GPU parity file up to 3 times (separate processes), stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 1 2 3; do
  PG_FLAKE_DUMP=gpurun_out/flake.npz timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/flake_$k.log 2>&1
  rc=$?
  tail -2 gpurun_out/flake_$k.log
  [ $rc -eq 0 ] || { grep -A12 "AssertionError: rgb" gpurun_out/flake_$k.log | head -30; exit $rc; }
done
