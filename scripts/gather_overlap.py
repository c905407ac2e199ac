"""Overlap of the obs gather with the engine's kernels, from a rocprofv3 kernel trace.

usage: python3 scripts/gather_overlap.py <run_kernel_trace.csv> [out.json]

The gather's work is every dispatch that is not one of the engine's kernels (pg_*): at world 1
RCCL's all_gather_into_tensor is a copyBuffer blit, at world > 1 RCCL's own kernels.  For each
such dispatch the script measures how much of its [start, end) interval is covered by the union
of the pg_* kernel intervals, and reports the total and the fraction, plus the queues both ran on.
"""
import csv
import json
import sys


def union(intervals):
    out = []
    for s, e in sorted(intervals):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s, e, merged):
    tot = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    eng, other = [], []
    eng_q, other_q = set(), set()
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"]
        if name.startswith("pg_") or "pg_step" in name or "pg_render" in name or "pg_reset" in name:
            eng.append((s, e))
            eng_q.add(r["Queue_Id"])
        elif "copyBuffer" in name or "ncclDevKernel" in name or "rccl" in name.lower():
            other.append((s, e, name))
            other_q.add(r["Queue_Id"])
    merged = union(eng)
    lo = merged[0][0] if merged else 0
    # only the gathers inside the engine's active span (the warmup / settle before it aside)
    other = [o for o in other if o[0] >= lo]
    tot = sum(e - s for s, e, _ in other)
    ov = sum(covered(s, e, merged) for s, e, _ in other)
    res = {"gather_dispatches": len(other), "gather_ns": tot, "overlapped_ns": ov,
           "overlap_frac": round(ov / tot, 4) if tot else None,
           "gather_avg_us": round(tot / len(other) / 1e3, 1) if other else None,
           "gather_queues": sorted(other_q), "engine_queues": sorted(eng_q),
           "names": sorted({n for _, _, n in other})[:4]}
    print(json.dumps(res))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
