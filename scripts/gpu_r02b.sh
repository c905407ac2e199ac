set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_coinrun.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_b.log 2>&1 && \
timeout -k 10 400 python3 scripts/phase_profile.py bigfish bossfight caveflyer chaser climber coinrun dodgeball fruitbot heist jumper leaper maze miner ninja plunder starpilot > gpurun_out/phase_all.json 2> gpurun_out/phase.err && \
timeout -k 10 300 python3 bench.py --steps 50 --no-cpu-baseline > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
rc=$?
tail -3 gpurun_out/pytest_b.log; cat gpurun_out/bench_b.json; tail -3 gpurun_out/phase.err
exit $rc
