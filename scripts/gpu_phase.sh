set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/phase_profile.py 2>&1 | tee gpurun_out/phase.json | tail -30
