"""Copies > 1 MB (or > 100 us when the trace has no sizes) from a rocprofv3 --memory-copy-trace run, with their rate, stream and the gap to the
previous copy, plus the engine kernels between them (host-path analysis, scripts/gpu_r04n.sh)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
rows = list(csv.DictReader(open(mc[0])))
print("columns:", list(rows[0].keys()))
ev = []
for r in rows:
    size = int(r.get("Bytes") or r.get("Size") or 0)  # absent in rocprofv3 7.x: filter by duration
    if (size and size < (1 << 20)) or int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 100000:
        continue
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", size, r.get("Direction", ""),
               r.get("Stream_Id", r.get("Queue_Id", ""))))
for r in csv.DictReader(open(kt[0])):
    if r["Kernel_Name"].startswith("pg_") or "pg_" in r["Kernel_Name"][:20]:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:28], 0, "", r["Queue_Id"]))
ev.sort()
t0 = ev[0][0] if ev else 0
prev_end = None
for s, e, name, size, direc, st in ev:
    rate = size / (e - s) if name == "copy" and e > s else 0
    if name == "copy" and not size:
        name = "copy %s" % direc
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0
    print("%10.1f us  %8.1f us  gap %8.1f  %-28s %6s  q/s %s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, name,
          direc, st, ("%.1f MB %.1f GB/s" % (size / 1e6, rate)) if size else ""))
    prev_end = max(prev_end or 0, e)
