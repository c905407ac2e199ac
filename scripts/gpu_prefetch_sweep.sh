# Level-prefetch sweep: per game, prefetch off / lag 2,3,4 (one stream) / lag 2,3 (two streams).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pf; mkdir -p $OUT
for g in ${GAMES:-jumper caveflyer leaper coinrun starpilot maze}; do
  for v in ${VARIANTS:-off 2:1 3:1 4:1 2:2 3:2}; do
    if [[ $v == off ]]; then export PROCGEN_MI355X_PREFETCH=0; else export PROCGEN_MI355X_PREFETCH=1 PROCGEN_MI355X_PREFETCH_LAG=${v%:*} PROCGEN_MI355X_PREFETCH_STREAMS=${v#*:}; fi
    timeout -k 10 120 python3 bench.py --env-name $g --steps 50 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > $OUT/$g.$v.json 2> $OUT/$g.$v.err || { tail -5 $OUT/$g.$v.err; exit 12; }
    python3 -c "import json; d=json.load(open('$OUT/$g.$v.json')); print('$g $v', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  done
done
