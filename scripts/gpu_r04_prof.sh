# Round-4 profile call: coinrun parts A/B (1 / 2 / 3), the coinrun counter passes (bench traffic
# fields), the census of one step + render launch, every game alone and the mixed-16 shard.
#   STEPS=ab,counters,census,games (default: all)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${STEPS:-ab,counters,census,games}
if [[ $S == *ab* ]]; then
  CFGS="PROCGEN_MI355X_PARTS=1 PROCGEN_MI355X_PARTS=2 PROCGEN_MI355X_PARTS=3" bash scripts/gpu_ab.sh || exit 11
fi
if [[ $S == *counters* ]]; then
  GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 12; }
  python3 -c "import json; d=json.load(open('gpurun_out/ctr/summary.json'))['coinrun']; print({k: (v.get('avg_ms'), v.get('hbm_bytes_per_part_act'), v.get('scratch'), v.get('wait_any_frac')) for k, v in d.items()})"
fi
if [[ $S == *census* ]]; then
  timeout -k 10 300 python3 scripts/census.py coinrun > gpurun_out/census.log 2>&1 || { tail -5 gpurun_out/census.log; exit 13; }
  grep -v "^\s*[0-9]*,\?$" gpurun_out/census.log | tail -30
fi
if [[ $S == *games* ]]; then
  bash scripts/gpu_r03_games.sh > gpurun_out/games.log 2>&1 || { tail -5 gpurun_out/games.log; exit 14; }
  cat gpurun_out/games.log
fi
