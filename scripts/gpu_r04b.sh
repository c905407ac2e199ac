# Round-4 combined call: smoke + the -m gpu suite + the default bench line (gpu_r04.sh), the coinrun
# counter passes (gpu_r04_prof.sh counters), then the PG_PROFILE phase shares of the slow renders / steps
# (libprocgen_mi355x_prof.so, `make PROFILE=1`) and the coinrun census.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r04.sh || exit $?
STEPS=counters bash scripts/gpu_r04_prof.sh || exit $?
GAMES="${PGAMES:-bossfight fruitbot coinrun miner dodgeball}" bash scripts/gpu_phase2.sh || exit 15
STEPS=census bash scripts/gpu_r04_prof.sh || exit $?
