# bench every experiment build named in $VARIANTS (plus the default build) back to back, per game in $GAMES
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in ${GAMES:-coinrun}; do
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then lib=""; else lib="$v"; fi
  PROCGEN_MI355X_LIB=$lib timeout -k 10 240 python bench.py --env-name $g --steps ${STEPS:-60} --warmup 10 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline > gpurun_out/bench_${g}_$v.json 2> gpurun_out/bench_${g}_$v.err
  rc=$?
  [ $rc -eq 0 ] || { echo "variant $v failed rc=$rc"; tail -5 gpurun_out/bench_${g}_$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${g}_$v.json')); print('%-10s %-12s %.3fM env-steps/s' % ('$g', '$v', d['value']/1e6), d['roofline']['kernel_ms'])"
done
done
