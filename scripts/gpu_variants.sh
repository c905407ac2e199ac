# bench every experiment build named in $VARIANTS (plus the default build) back to back
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then lib=""; else lib="$v"; fi
  PROCGEN_MI355X_LIB=$lib timeout -k 10 240 python bench.py --steps ${STEPS:-60} --warmup 10 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err
  rc=$?
  [ $rc -eq 0 ] || { echo "variant $v failed rc=$rc"; tail -5 gpurun_out/bench_$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_$v.json')); print('%-12s %.3fM env-steps/s' % ('$v', d['value']/1e6), d['roofline']['kernel_ms'])"
done
