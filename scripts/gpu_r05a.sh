# Round-5 (a): render-kernel sensitivity.  The counter list of this box, then coinrun bench lines of the
# default build against experiment builds: +4 KB LDS per render workgroup (occupancy sensitivity),
# 16- and 4-row texel batches (dependent-round sensitivity).  The first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/a
timeout -k 10 60 rocprofv3 -L > gpurun_out/a/counters_list.txt 2>&1 || echo "counter list rc=$?"
VARIANTS="${VARIANTS:-pad4k rb16 rb4}" GAMES=coinrun STEPS=60 bash scripts/gpu_variants.sh || exit 11
exit 0
