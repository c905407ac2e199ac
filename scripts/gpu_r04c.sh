# Round-4 diagnostics: stamp_images' sub-phases (VARIANT=stamp build, written into the step slots of the
# phase profile: 0 prefetch of small images, 1 their in-order blends, 2 descriptor transform blits > 64 px,
# 3 in-order transform blits, 4 tile lists, 5 fills, 6 plain blits > 64 px, 7 outside stamp_images),
# the coinrun census (VARIANT=census), then every game alone and the mixed-16 shard.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PROCGEN_MI355X_LIB=stamp timeout -k 10 400 python3 scripts/phase_profile.py ${SGAMES:-bossfight fruitbot coinrun dodgeball} > gpurun_out/stamp.json 2> gpurun_out/stamp.err || { tail -3 gpurun_out/stamp.err; exit 11; }
STEPS=census bash scripts/gpu_r04_prof.sh || exit $?
[[ "${GAMESRUN:-1}" == 1 ]] && { bash scripts/gpu_r03_games.sh > gpurun_out/games.log 2>&1 || { tail -5 gpurun_out/games.log; exit 14; }; cat gpurun_out/games.log; }
exit 0
