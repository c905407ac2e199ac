#!/usr/bin/env python3
"""Turn the rocprofv3 output of scripts/gpu_profile.sh (gpurun_out/prof/) into the committed
summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_pmc.json           -- per-kernel average FETCH_SIZE / WRITE_SIZE per launch

Units: rocprofv3's FETCH_SIZE / WRITE_SIZE are KiB (x1024 -> bytes).  gfx950 correction
(MI355X_MICROARCH.md, HBM): FETCH_SIZE reads 1/2 of the bytes of WIDE (16 B/lane) coalesced
streaming reads; the render kernel's reads are 4-byte texel gathers, for which the guide
gives no calibration, so `traffic` uses the raw value and the x2 figure is kept as an upper
bound.  WRITE_SIZE is exact for 16-B/lane stores; the render kernel's 12-B/lane obs stores
measure exactly 65,536 x 12,288 B per launch (self-check below).
"""
import csv
import collections
import re
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def base_name(name):
    """'void (anonymous namespace)::pg_step_kernel<5>(PGDev, ...)' -> 'pg_step_kernel'"""
    m = re.search(r"(pg_\w+?_kernel)", name)
    return m.group(1) if m else name


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[base_name(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(tag, prof=os.path.join(REPO, "gpurun_out", "prof")):
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"),
                os.path.join(REPO, "profiles", "%s_kernel_stats.csv" % tag))
    stats = {}
    for r in csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))):
        k = base_name(r["Name"])
        if k in stats:  # several template instances (mixed batches): call-weighted average
            a, b = stats[k], r
            calls = int(a["Calls"]) + int(b["Calls"])
            avg = (float(a["AverageNs"]) * int(a["Calls"]) + float(b["AverageNs"]) * int(b["Calls"])) / calls
            stats[k] = {"Calls": calls, "AverageNs": avg}
        else:
            stats[k] = r
    fetch = per_kernel(os.path.join(prof, "fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(prof, "write", "run_counter_collection.csv"))
    out = {"tag": tag, "units": "bytes per launch", "kernels": {}}
    for k in ("pg_step_kernel", "pg_reset_kernel", "pg_render_kernel"):
        f = fetch.get(k, 0.0) * 1024
        w = write.get(k, 0.0) * 1024
        out["kernels"][k] = {"avg_ns": float(stats[k]["AverageNs"]) if k in stats else None,
                             "calls": int(stats[k]["Calls"]) if k in stats else None,
                             "fetch_bytes_raw": f, "fetch_bytes_x2_upper": 2 * f, "write_bytes": w,
                             "hbm_bytes": f + w}
    r = out["kernels"]["pg_render_kernel"]
    out["render_hbm_bytes_per_launch"] = r["hbm_bytes"]
    out["render_write_selfcheck"] = {"expected_obs_bytes": 65536 * 12288, "measured": r["write_bytes"]}
    with open(os.path.join(REPO, "profiles", "%s_pmc.json" % tag), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
