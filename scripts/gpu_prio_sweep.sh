# Reset/prefetch stream priorities: rp = reset stream high (1) / normal (0); pp = prefetch low (1) / normal (0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prio; mkdir -p $OUT
for g in ${GAMES:-jumper caveflyer leaper coinrun starpilot maze heist}; do
  for v in ${VARIANTS:-0:0:0 1:0:0 1:1:1 1:1:0 0:1:1}; do
    IFS=: read rp pf pp <<< "$v"
    export PROCGEN_MI355X_RESET_PRIO=$rp PROCGEN_MI355X_PREFETCH=$pf PROCGEN_MI355X_PREFETCH_PRIO=$pp
    timeout -k 10 120 python3 bench.py --env-name $g --steps 50 --warmup 20 --settle 100 --host-steps 0 --no-cpu-baseline > $OUT/$g.$v.json 2> $OUT/$g.$v.err || { tail -5 $OUT/$g.$v.err; exit 12; }
    python3 -c "import json; d=json.load(open('$OUT/$g.$v.json')); print('$g rp:pf:pp=$v', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  done
done
