# GPU parity run: the given pytest selections one after another; an assertion failure (rc 1)
# moves on to the next selection, anything else (fault, abort, timeout) stops the script.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rc=0
i=0
for sel in "$@"; do
  i=$((i+1))
  timeout -k 10 ${STEP_TIMEOUT:-600} python3 -m pytest $sel -x -q -m gpu ${PYTEST_ARGS} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$i.log 2>&1
  r=$?
  echo "== $sel rc=$r"; tail -25 gpurun_out/pytest_$i.log
  if [ $r -ne 0 ]; then rc=$r; fi
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then echo "stopping after rc=$r"; exit $r; fi
done
exit $rc
