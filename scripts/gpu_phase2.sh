set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 scripts/phase_profile.py ${GAMES:-maze miner fruitbot bossfight ninja chaser leaper climber dodgeball jumper coinrun caveflyer heist starpilot plunder bigfish} > gpurun_out/phase2.json 2> gpurun_out/phase2.err
rc=$?
tail -3 gpurun_out/phase2.err
exit $rc
