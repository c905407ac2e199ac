# Round-5 (n): the D2H probe inside a Python process without / with torch's HIP context, and with a
# numpy destination (kernel + memory-copy traces: copyBuffer kernels = blits, memory copies = SDMA).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/n
mkdir -p $O
summ() {
  python3 - "$1" <<'PY'
import csv, sys, os
d = sys.argv[1]
k = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
m = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv")))) if os.path.exists(os.path.join(d, "run_memory_copy_trace.csv")) else []
blits = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in k if "copyBuffer" in r["Kernel_Name"]]
sdma = [(r["Direction"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in m if r["Direction"].endswith("DEVICE_TO_HOST")]
print(d, "blit D2H kernels:", [round(x) for x in blits], "SDMA D2H:", [round(x) for _, x in sdma])
PY
}
for mode in plain torch; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/$mode -o run -- python3 scripts/d2h_probe_torch.py $mode > $O/$mode.log 2>&1 || { tail -5 $O/$mode.log; exit 11; }
  cat $O/$mode.log | grep -v "^W\|rocprof" | head -20
  summ $O/$mode
done
exit 0
