# Round-5 (m): rgb_array chunked render overlapped with the DMA (parity, then the bench at 4,096 envs for
# 1 / 8 chunks), the D2H engine probe, the level-generation phases of caveflyer / jumper (rprof build).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/m
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rgb_array.py -x -v --timeout 200 --timeout-method thread -k "chunks or mixed or parity" > $O/pytest_rgb.log 2>&1 || { tail -30 $O/pytest_rgb.log; exit 11; }
tail -2 $O/pytest_rgb.log
for c in 1 8 16; do
  PROCGEN_MI355X_HR_CHUNKS=$c timeout -k 10 300 python3 scripts/bench_rgb_array.py --env-name coinrun --num-envs 4096 --steps 4 > $O/rgb_coinrun_c$c.json 2> $O/rgb_coinrun_c$c.err || { tail -5 $O/rgb_coinrun_c$c.err; exit 12; }
  cat $O/rgb_coinrun_c$c.json
done
timeout -k 10 300 python3 scripts/bench_rgb_array.py --env-name bossfight --num-envs 4096 --steps 4 > $O/rgb_bossfight_c8.json 2> $O/rgb_bossfight_c8.err || { tail -5 $O/rgb_bossfight_c8.err; exit 12; }
cat $O/rgb_bossfight_c8.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/rgbprof -o run -- python3 scripts/bench_rgb_array.py --env-name coinrun --num-envs 4096 --steps 2 > $O/rgbprof.log 2>&1 || exit 13
timeout -k 10 120 scripts/d2h_probe2 > $O/d2h_probe2.txt 2>&1 || exit 14
cat $O/d2h_probe2.txt
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/d2h -o run -- scripts/d2h_probe2 > $O/d2h_prof.log 2>&1 || { tail -5 $O/d2h_prof.log; exit 15; }
timeout -k 10 300 python3 scripts/reset_phases.py jumper caveflyer > $O/reset_phases.json 2> $O/reset_phases.err || { tail -5 $O/reset_phases.err; exit 16; }
cat $O/reset_phases.json
exit 0
