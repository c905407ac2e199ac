# Round-5 (s): the D2H probe's engine-like variants (F-I) under the kernel + memory-copy trace: which
# condition turns a device -> page-locked host copy into a copyBuffer blit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- scripts/d2h_probe2 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 11; }
grep -E "^[A-I] |^base|^F |^G |^H |^I " $O/probe.log
python3 - <<'PY'
import csv
k = list(csv.DictReader(open("gpurun_out/s/tr/run_kernel_trace.csv")))
m = list(csv.DictReader(open("gpurun_out/s/tr/run_memory_copy_trace.csv")))
ev = [(int(r["Start_Timestamp"]), "K " + r["Kernel_Name"][:24], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in k]
ev += [(int(r["Start_Timestamp"]), "M " + r["Direction"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in m]
ev.sort()
for t, n, d in ev:
    if "busy" in n or "fill" in n:
        continue
    print("%-40s %8.1f us" % (n, d))
PY
