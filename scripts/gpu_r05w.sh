# Round-5 (w): the final round-5 build's bench lines (all-16 mixed shard, the world-1 RCCL gather line,
# every game alone at 65,536 envs: scripts/gpu_bench_configs.sh), then the counter passes of the
# default coinrun bench (kernel stats, SQ, FETCH / WRITE: scripts/gpu_counters.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=100 WARMUP=20 timeout -k 10 1000 bash scripts/gpu_bench_configs.sh > gpurun_out/configs.log 2>&1 || { tail -5 gpurun_out/configs.log; exit 13; }
tail -20 gpurun_out/configs.log
GAMES=coinrun timeout -k 10 600 bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 14; }
exit 0
