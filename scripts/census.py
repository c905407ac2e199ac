#!/usr/bin/env python3
"""Occupancy census of one step launch and one render launch (diagnostic PG_CENSUS build:
make -C procgen-1_amd/csrc VARIANT=census EXTRA=-DPG_CENSUS).

Every wave records its start / end on the 100 MHz constant clock and its HW_ID / XCC_ID
(pg_device.h Census).  From one launch's records this prints: the launch span, the mean wave
lifetime, the average and peak number of resident waves (chip, per CU, per SIMD), how fast waves
were dispatched, and how long the tail was -- i.e. whether the kernel ran at the occupancy its
resources allow or was bound by something else (dispatch, tail)."""
import json
import os
import sys

os.environ["PROCGEN_MI355X_LIB"] = "census"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def analyse(rec):
    t0, t1, hw = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64), rec[:, 2]
    ok = (t1 > t0) & (t0 > 0)
    t0, t1, hw = t0[ok], t1[ok], hw[ok]
    base = t0.min()
    t0 = (t0 - base) * 10.0  # ns (100 MHz)
    t1 = (t1 - base) * 10.0
    span = t1.max()
    life = t1 - t0
    hwid = (hw & 0xffffffff).astype(np.int64)
    xcc = (hw >> 32).astype(np.int64) & 0xf
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 15
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 7
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    n_cu = len(np.unique(cu_key))
    # resident waves over time (event sweep)
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    res = np.cumsum(ev[:, 1])
    peak = res.max()
    avg = life.sum() / span
    # per-CU peak residency
    per_cu_peak = []
    for k in np.unique(cu_key)[:64]:
        m = cu_key == k
        e = np.concatenate([np.stack([t0[m], np.ones(m.sum())], 1), np.stack([t1[m], -np.ones(m.sum())], 1)])
        e = e[np.lexsort((e[:, 1], e[:, 0]))]
        per_cu_peak.append(np.cumsum(e[:, 1]).max())
    q = np.percentile
    return {
        "waves": int(len(t0)), "cus_seen": int(n_cu), "span_us": round(span / 1e3, 2),
        "lifetime_us": {"mean": round(life.mean() / 1e3, 2), "p50": round(q(life, 50) / 1e3, 2),
                        "p90": round(q(life, 90) / 1e3, 2), "max": round(life.max() / 1e3, 2)},
        "resident_waves": {"avg": round(avg, 1), "peak": int(peak), "avg_per_simd": round(avg / (n_cu * 4), 2),
                           "peak_per_cu_sampled": int(max(per_cu_peak))},
        "dispatch": {"last_start_us": round(t0.max() / 1e3, 2), "p50_start_us": round(q(t0, 50) / 1e3, 2),
                     "tail_us": round((span - q(t1, 95)) / 1e3, 2)},
        "simd_share": [int((simd == s).sum()) for s in range(4)],
    }


def main(game="coinrun", num=65536, warm=60):
    torch.cuda.set_device(0)
    from procgen_amd import ProcgenGym3Env, _lib
    lib = _lib.load()
    env = ProcgenGym3Env(num=num, env_name=game, num_levels=200 if game == "coinrun" else 0, start_level=0,
                         rand_seed=0, device_buffers=True)
    for t in range(1, warm + 1):
        env.act_hashed(0x5EED, t)
    env.wait()
    raw = np.zeros((num, 16), np.uint64)
    lib.procgen_profile_raw(env._handle, raw.ctypes.data)
    out = {"game": game, "num_envs": num, "step": analyse(raw[:, 0:3]), "render": analyse(raw[:, 8:11])}
    # the slowest step waves of this launch and the state they left (PGEnv words: num_ents 27,
    # cur_time 2, action 1, rg_mti 64, sd_done 14, agent_erased 28)
    life = (raw[:, 1].astype(np.int64) - raw[:, 0].astype(np.int64)) * 10.0 / 1e3
    slow = []
    for e in np.argsort(-life)[:16]:
        w = env.debug_env(int(e))
        marks = [round((int(raw[e, 3 + k]) - int(raw[e, 0])) * 10.0 / 1e3, 1) for k in range(5)]
        slow.append({"env": int(e), "us": round(float(life[e]), 1), "marks_us": marks, "num_ents": int(w[27]), "cur_time": int(w[2]),
                     "action": int(w[1]), "rg_mti": int(w[64]), "done": int(w[14]), "agent_erased": int(w[28]), "grid8_ok": int(w[67])})
    dbg = [env.debug_env(int(e)) for e in range(0, num, 16)]
    ne = np.array([w[27] for w in dbg])
    g8 = np.array([w[67] for w in dbg])
    out["grid8_ok_frac"] = {"all": float(g8.mean()), "first4096": float(g8[:256].mean()), "rest": float(g8[256:].mean())}
    out["step_slowest"] = slow
    # phase split of a typical wave (median of the mark offsets over all waves)
    offs = (raw[:, 3:8].astype(np.int64) - raw[:, 0:1].astype(np.int64)) * 10.0 / 1e3
    out["marks_median_us"] = [round(float(np.median(offs[:, k])), 2) for k in range(5)]
    out["start_us_of_slowest"] = [round((int(raw[e, 0]) - int(raw[:, 0].min())) * 10.0 / 1e3, 1) for e in np.argsort(-life)[:16]]
    out["num_ents_sample"] = {"mean": float(ne.mean()), "p99": float(np.percentile(ne, 99)), "max": int(ne.max())}
    out["lifetime_hist_us"] = np.histogram(life, bins=[0, 20, 40, 60, 80, 120, 200, 400, 800, 2000])[0].tolist()
    env.close()
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    res = [main(g, warm=int(os.environ.get("CENSUS_WARM", "60"))) for g in (sys.argv[1:] or ["coinrun"])]
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "census.json"), "w") as f:
        json.dump(res, f, indent=1)
