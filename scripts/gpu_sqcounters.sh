# SQ instruction-mix / stall counters per kernel (separate --pmc passes, kernel trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sq
rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.json 2> $OUT/p1.err && \
timeout -k 10 300 rocprofv3 --pmc ${PASS2:-SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS} --kernel-trace --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.json 2> $OUT/p2.err
rc=$?
tail -3 $OUT/*.err
python3 scripts/sq_summary.py $OUT
exit $rc
