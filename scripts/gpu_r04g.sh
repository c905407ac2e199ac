# Round-4 render experiments: RB=16 (16-row texel batches of the pixel-centric pass) and
# PG_RENDER_K=2 (two envs per workgroup) against the default build, coinrun and a few games.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/g
for g in ${GAMES:-coinrun maze bossfight}; do
  for L in "" rb16 k2; do
    PROCGEN_MI355X_LIB=$L timeout -k 10 200 python3 bench.py --env-name $g --steps 100 --warmup 20 --settle 200 --host-steps 0 --no-cpu-baseline > gpurun_out/g/$g.$L.json 2> gpurun_out/g/$g.$L.err || { tail -5 gpurun_out/g/$g.$L.err; exit 12; }
    python3 -c "import json; d=json.load(open('gpurun_out/g/$g.$L.json')); print('$g', 'lib=$L', round(d['value']/1e6,2), d['roofline']['kernel_ms'])"
  done
done
