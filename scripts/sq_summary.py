#!/usr/bin/env python3
"""Average SQ counters per wave for each kernel from rocprofv3 --pmc csv output."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?").split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k in sorted(acc):
    a = acc[k]
    waves = a.get("SQ_WAVES", 0) / max(cnt[k].get("SQ_WAVES", 1), 1)
    print(k)
    for n in sorted(a):
        per_disp = a[n] / max(cnt[k][n], 1)
        print("   %-24s per dispatch %14.1f   per wave %10.1f" % (n, per_disp, per_disp / waves if waves else 0))
