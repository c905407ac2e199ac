# A/B of engine knobs over short bench lines: CFGS="A=1,B=2 A=0,B=0" [GAMES=...] (each config a
# comma-separated list of env assignments; "-" = defaults), then (TESTS=1) the GPU parity suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for g in ${GAMES:-coinrun}; do
  for c in ${CFGS:--}; do
    a=${c//,/ }; [[ $c == - ]] && a=""
    env $a timeout -k 10 200 python3 bench.py --env-name $g --steps ${STEPS:-200} --warmup 20 --settle ${SETTLE:-300} --host-steps 0 --no-cpu-baseline > gpurun_out/ab/$g.$c.json 2> gpurun_out/ab/$g.$c.err || { tail -5 gpurun_out/ab/$g.$c.err; exit 12; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$g.$c.json')); print('$g', '$c', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  done
done
if [[ -n "${TESTS:-}" ]]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  exit $rc
fi
