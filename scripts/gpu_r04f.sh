# Round-4: coinrun counter passes (kernel stats, SQ, FETCH_SIZE, WRITE_SIZE) for the default build and
# the STEP_WAVES=4 experiment build (VARIANT=w4: no VGPR spills in the step kernel) -> is the step's
# write traffic scratch?  Then the driver's default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -5 gpurun_out/counters.log; exit 12; }
mv gpurun_out/ctr gpurun_out/ctr_default
if [[ "${W4:-1}" == 1 ]]; then
  PROCGEN_MI355X_LIB=w4 GAMES=coinrun bash scripts/gpu_counters.sh > gpurun_out/counters_w4.log 2>&1 || { tail -5 gpurun_out/counters_w4.log; exit 13; }
  mv gpurun_out/ctr gpurun_out/ctr_w4
fi
for d in gpurun_out/ctr_default gpurun_out/ctr_w4; do
  [[ -f $d/summary.json ]] && python3 -c "import json; d=json.load(open('$d/summary.json'))['coinrun']; print('$d', {k: (v.get('avg_ms'), v.get('fetch_bytes_per_launch'), v.get('write_bytes_per_launch'), v.get('scratch'), v.get('wait_any_frac')) for k, v in d.items()})"
done
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 11; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(round(d['value']/1e6,2), d['roofline']['render_kernel'], d['roofline']['end_to_end'], d.get('host_path'))"
