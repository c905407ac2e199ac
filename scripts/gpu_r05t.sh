# Round-5 (t): host-buffer observation copies as hipMemcpyDeviceToDeviceNoCU (PROCGEN_MI355X_D2H_NOCU=1):
# parity of the host-buffer tests with it on, then the host path and rgb_array rates off / on, and the
# copy engine in a kernel + memory-copy trace of the host path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t
mkdir -p $O
PROCGEN_MI355X_D2H_NOCU=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "host or rgb_array_chunks or boundary" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 11; }
tail -2 $O/pytest.log
for nocu in 0 1 0 1; do
  PROCGEN_MI355X_D2H_NOCU=$nocu timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --host-steps 40 --no-cpu-baseline > $O/host_$nocu.json 2> $O/host_$nocu.err || { tail -5 $O/host_$nocu.err; exit 12; }
  python3 -c "import json; d=json.load(open('$O/host_$nocu.json')); print('nocu=$nocu', round(d['value']/1e6,2), d['host_path'])"
done
for nocu in 0 1; do
  PROCGEN_MI355X_D2H_NOCU=$nocu timeout -k 10 300 python3 scripts/bench_rgb_array.py --env-name coinrun --num-envs 4096 --steps 4 > $O/rgb_$nocu.json 2> $O/rgb_$nocu.err || { tail -5 $O/rgb_$nocu.err; exit 13; }
  echo "nocu=$nocu $(cat $O/rgb_$nocu.json)"
done
PROCGEN_MI355X_D2H_NOCU=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --steps 10 --warmup 5 --host-steps 10 --no-cpu-baseline > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 14; }
python3 - <<'PY'
import csv
k = list(csv.DictReader(open("gpurun_out/t/tr/run_kernel_trace.csv")))
m = list(csv.DictReader(open("gpurun_out/t/tr/run_memory_copy_trace.csv")))
big = [r for r in k if "copyBuffer" in r["Kernel_Name"] and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 1000000]
d2h = [r for r in m if r["Direction"].endswith("DEVICE_TO_HOST") or "DEVICE_TO_DEVICE" in r["Direction"]]
print("copyBuffer kernels > 1 ms:", len(big), "SDMA copies:", len(d2h), sorted(set(r["Direction"] for r in m)))
PY
