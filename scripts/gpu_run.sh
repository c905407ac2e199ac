# One parameterised GPU launcher (round 6): every stage runs under its own time limit, stages are
# chained so the first fault / abort / timeout ends the call, and nothing is retried.
#   DO="smoke tests ab counters bench"   stages, in this order
#   TESTS="tests/test_gpu_coinrun.py ..." pytest selections for `tests` (default: the whole -m gpu suite)
#   PYTEST_K=...                          -k filter for `tests`
#   VARIANTS="base rf"                    extra builds for `ab` (procgen_amd/libprocgen_mi355x_<v>.so)
#   GAMES="coinrun"  CFGS="A=1,B=2 -"     games and env-knob configs for `ab` (each config x variant)
#   STEPS=200 SETTLE=300                  bench length for `ab`
#   CGAMES="coinrun"                      games for `counters` (scripts/gpu_counters.sh)
#   CENSUS_GAMES="coinrun dodgeball"      games for `census` (smart-entity census, VARIANT=smart build)
#   SPEED_STEPS=1000                      round trips per line for `speed` (scripts/speed_shape.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for stage in ${DO:-smoke tests}; do
  case $stage in
  smoke)
    timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
  tests)
    timeout -k 10 ${TEST_TIMEOUT:-1100} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout ${PER_TEST:-300} \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc ;;
  ab)
    for g in ${GAMES:-coinrun}; do
      for v in default ${VARIANTS}; do
        for c in ${CFGS:--}; do
          a=${c//,/ }; [[ $c == - ]] && a=""
          lib=""; [ "$v" = default ] || lib=$v
          f=gpurun_out/ab/$g.$v.${c//=/_}
          env $a PROCGEN_MI355X_LIB=$lib timeout -k 10 240 python3 bench.py --env-name $g --steps ${STEPS:-200} --warmup 20 \
            --settle ${SETTLE:-300} --host-steps 0 --no-cpu-baseline > $f.json 2> $f.err || { tail -5 $f.err; exit 12; }
          python3 -c "import json; d=json.load(open('$f.json')); print('%-10s %-8s %-40s %6.2f M' % ('$g', '$v', '$c', d['value']/1e6), d['roofline']['kernel_ms'])"
        done
      done
    done ;;
  counters)
    GAMES="${CGAMES:-coinrun}" bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 13; }
    tail -3 gpurun_out/counters.log ;;
  census)  # smart-entity census (diagnostic build libprocgen_mi355x_smart.so), per game in CENSUS_GAMES
    for g in ${CENSUS_GAMES:-coinrun}; do
      PROCGEN_MI355X_LIB=smart timeout -k 10 300 python3 scripts/smart_census.py $g > gpurun_out/census_$g.json 2> gpurun_out/census_$g.err || { tail -5 gpurun_out/census_$g.err; exit 15; }
      cat gpurun_out/census_$g.json
    done ;;
  speed)  # the reference's speed-test shape (scripts/speed_shape.py)
    timeout -k 10 900 python3 scripts/speed_shape.py > gpurun_out/speed_shape.json 2> gpurun_out/speed_shape.err || { tail -5 gpurun_out/speed_shape.err; exit 16; }
    tail -16 gpurun_out/speed_shape.err ;;
  phase)  # per-phase cycle shares of step and render (PROFILE=1 build libprocgen_mi355x_prof.so), per game in PHASE_GAMES
    for g in ${PHASE_GAMES:-coinrun}; do
      timeout -k 10 300 python3 scripts/phase_profile.py $g > gpurun_out/phase_$g.json 2> gpurun_out/phase_$g.err || { tail -5 gpurun_out/phase_$g.err; exit 17; }
      cat gpurun_out/phase_$g.json
    done ;;
  probe)  # the host-path D2H probe inside a torch process under the memory-copy trace (teardown check)
    timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/probe -o run -- python3 scripts/d2h_probe_torch.py torch > gpurun_out/probe.log 2>&1
    rc=$?; grep -v "^W2026" gpurun_out/probe.log | tail -14; [ $rc -eq 0 ] || exit $rc ;;
  teardown)  # which process crashes at exit under the memory-copy trace: torch alone, then the probe without torch
    timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/td_torch -o run -- python3 -c "import torch; torch.zeros(1, device='cuda'); torch.cuda.synchronize(); print('torch alone ok')" > gpurun_out/td_torch.log 2>&1
    rc=$?; echo "torch alone under rocprofv3: rc=$rc"; grep -v "^W2026" gpurun_out/td_torch.log | tail -3; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/td_plain -o run -- python3 scripts/d2h_probe_torch.py plain > gpurun_out/td_plain.log 2>&1
    rc=$?; echo "probe without torch under rocprofv3: rc=$rc"; grep -v "^W2026" gpurun_out/td_plain.log | tail -3; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 14; }
    cat gpurun_out/bench.json ;;
  esac
done
