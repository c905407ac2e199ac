# Round-3 checkpoint call after a container rebuild: parity suite, bench, per-game + mixed16 lines,
# then the coinrun counter passes (kernel stats, SQ, FETCH, WRITE).
set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS=${STEPS:-tests,bench,games} GAMES="${GAMES:-}" bash scripts/gpu_r03_full.sh || exit $?
GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 21; }
tail -40 gpurun_out/counters.log
