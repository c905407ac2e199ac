# rocprofv3 passes over a short bench run: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: TCC slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write.err
rc=$?
find $OUT -name "*.csv" | head -20
tail -3 $OUT/*.err
exit $rc
