# Round-5 (d): memory-pipeline counters of the coinrun act with the register-frame render (RENDER_RF
# default) and the LDS-frame render (RENDER_RF=0): one --pmc group per run (TA 2, TCP 4, GRBM 2, SQ 5),
# kernel trace + stats in their own runs.  Summaries: scripts/counter_summary.py-style per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/d
rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --settle ${SETTLE:-100} --host-steps 0 --no-cpu-baseline --env-name ${GAME:-coinrun}"
for mode in ${MODES:-rf lds}; do
  if [ $mode = rf ]; then E="PROCGEN_MI355X_RENDER_RF=all"; else E="PROCGEN_MI355X_RENDER_RF=0"; fi
  export $E
  D=$OUT/$mode
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $ARGS > $D.trace.json 2> $D.trace.err || exit 11
  timeout -k 10 200 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $D/p1 -o run -- python3 bench.py $ARGS > $D.p1.json 2> $D.p1.err || exit 12
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $D/p2 -o run -- python3 bench.py $ARGS > $D.p2.json 2> $D.p2.err || exit 13
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- python3 bench.py $ARGS > $D.fetch.json 2> $D.fetch.err || exit 14
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- python3 bench.py $ARGS > $D.write.json 2> $D.write.err || exit 15
done
ls -R $OUT | head -50
exit 0
