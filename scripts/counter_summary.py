#!/usr/bin/env python3
"""Summarise scripts/gpu_counters.sh output: per game and kernel, the average kernel duration
(rocprofv3 kernel trace), every counter per dispatch (and per wave for SQ_*), LDS / VGPR / scratch
of the dispatch, and derived figures: HBM bytes per launch = FETCH_SIZE + WRITE_SIZE (KB units,
x1024; no gfx950 FETCH correction applied: the engine's loads are 4-16 B gathers),
wait fraction = SQ_WAIT_ANY / SQ_WAVE_CYCLES."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ctr"


def kname(full):
    """'void (anonymous namespace)::pg_step_kernel<5>(PGDev, ...)' -> 'pg_step_kernel<5>' (None if not ours)."""
    head = full.split("(PGDev")[0].split("(int")[0]
    head = head.replace("void ", "").replace("(anonymous namespace)::", "").strip()
    return head if head.startswith("pg_") else None
out = {}
for gdir in sorted(glob.glob(os.path.join(root, "*"))):
    if not os.path.isdir(gdir):
        continue
    game = os.path.basename(gdir)
    kern = defaultdict(lambda: {"counters": defaultdict(list)})
    for f in glob.glob(os.path.join(gdir, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if not k:
                continue
            d = kern[k]
            d.setdefault("dur_ns", []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            d["lds_bytes"] = int(r.get("LDS_Block_Size", r.get("Lds_Size", 0)) or 0)
            d["vgpr"] = int(r.get("VGPR_Count", r.get("Arch_VGPR_Count", 0)) or 0)
            d["accum_vgpr"] = int(r.get("Accum_VGPR_Count", 0) or 0)
            d["sgpr"] = int(r.get("SGPR_Count", 0) or 0)
            d["scratch"] = int(r.get("Scratch_Size", r.get("Private_Segment_Size", 0)) or 0)
            d["workgroup"] = int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 0)) or 0)
            d["grid"] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    # per pass: (dispatch id, kernel, value) of every counter, for the per-act sums below
    seq = defaultdict(list)
    for f in glob.glob(os.path.join(gdir, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if not k:
                continue
            kern[k]["counters"][r["Counter_Name"]].append(float(r["Counter_Value"]))
            did = int(r.get("Dispatch_Id", r.get("Dispatch_ID", 0)) or 0)
            seq[r["Counter_Name"]].append((did, k, float(r["Counter_Value"])))
    # Per part-act sums: one act of a single game runs, per part, one step launch, the reset
    # launches and the render launches (mode 1 over the envs that did not finish + mode 2 over the
    # reset ones).  Over the last two thirds of the run's step launches (steady state), the bytes
    # of each kernel summed and divided by the number of step launches = that kernel's bytes per
    # part-act (for the step kernel: per launch; for the render: both modes).
    per_act = defaultdict(dict)
    for cname in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = sorted(seq.get(cname, []))
        steps = [i for i, (_, k, _) in enumerate(rows) if k.startswith("pg_step_kernel")]
        if len(steps) < 3:
            continue
        lo = steps[len(steps) // 3]
        n_steps = sum(1 for i in steps if i >= lo)
        tot = defaultdict(float)
        for did, k, v in rows[lo:]:
            tot[k] += v
        for k, v in tot.items():
            per_act[k][cname] = v * 1024 / n_steps
        for k in tot:
            per_act[k]["step_launches_in_window"] = n_steps
    res = {}
    for k, d in kern.items():
        c = {n: sum(v) / len(v) for n, v in d["counters"].items() if v}
        e = {x: d[x] for x in ("lds_bytes", "vgpr", "accum_vgpr", "sgpr", "scratch", "workgroup", "grid") if x in d}
        if d.get("dur_ns"):
            durs = d["dur_ns"][len(d["dur_ns"]) // 3:]  # skip the initial reset / warmup launches
            e["avg_ms"] = round(sum(durs) / len(durs) / 1e6, 4)
            e["launches"] = len(d["dur_ns"])
        e["counters_per_dispatch"] = {n: round(v, 1) for n, v in sorted(c.items())}
        waves = c.get("SQ_WAVES")
        if waves:
            e["per_wave"] = {n: round(v / waves, 1) for n, v in sorted(c.items()) if n.startswith("SQ_")}
        if "SQ_WAIT_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_launch"] = round((c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            e["fetch_bytes_per_launch"] = round(c["FETCH_SIZE"] * 1024)
            e["write_bytes_per_launch"] = round(c["WRITE_SIZE"] * 1024)
        pa = per_act.get(k, {})
        if "FETCH_SIZE" in pa and "WRITE_SIZE" in pa:
            e["hbm_bytes_per_part_act"] = round(pa["FETCH_SIZE"] + pa["WRITE_SIZE"])
            e["fetch_bytes_per_part_act"] = round(pa["FETCH_SIZE"])
            e["write_bytes_per_part_act"] = round(pa["WRITE_SIZE"])
            e["step_launches_in_window"] = pa["step_launches_in_window"]
        res[k] = e
    tot = [v["hbm_bytes_per_part_act"] for v in res.values() if "hbm_bytes_per_part_act" in v]
    if tot:
        res["_all_kernels"] = {"hbm_bytes_per_part_act": round(sum(tot)),
                               "what": "step + reset(s) + render(s) FETCH_SIZE + WRITE_SIZE per part-act"}
    out[game] = res
print(json.dumps(out, indent=1, sort_keys=True))
