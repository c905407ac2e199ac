# Per-game rocprofv3 counter passes over a short device-resident bench (kernel trace only, one
# --pmc group per run, each under its own time limit):  kernel stats, SQ stall / instruction mix
# (2 passes), FETCH_SIZE, WRITE_SIZE.  GAMES="coinrun fruitbot" bash scripts/gpu_counters.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ctr
rm -rf $OUT; mkdir -p $OUT
for g in ${GAMES:-coinrun fruitbot bossfight}; do
  ARGS="--steps 10 --warmup 3 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline --env-name $g"
  D=$OUT/$g
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $ARGS > $D.trace.json 2> $D.trace.err || exit 11
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $D/p1 -o run -- python3 bench.py $ARGS > $D.p1.json 2> $D.p1.err || exit 12
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $D/p2 -o run -- python3 bench.py $ARGS > $D.p2.json 2> $D.p2.err || exit 13
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- python3 bench.py $ARGS > $D.fetch.json 2> $D.fetch.err || exit 14
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- python3 bench.py $ARGS > $D.write.json 2> $D.write.err || exit 15
done
python3 scripts/counter_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
