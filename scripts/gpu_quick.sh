set -o pipefail
cd $GRAFT_REPO_ROOT
rocm-smi --showproductname 2>&1 | head -5 || true
timeout -k 10 300 python -m pytest tests/test_gpu_coinrun.py -x -q -k "hard_200 or seeding" 2>&1 | tail -30
