"""Whole-population parity helpers (test infrastructure): the oracle leg of a full-size config run in
a host worker pool, and the digest both legs compare.

In the reference every env of a vec env is an independent Game with its own level-seed generator
(procgen/src/vecgame.cpp:349-378), so a 65,536-env config is 65,536 separate trajectories; these
helpers let a test check every one of them at every step instead of a sample.

Digest of one observation (include/procgen_mi355x.h procgen_read_outputs): the sum over k < 1,536 of
w_k * x_k mod 2^64, x_k the k-th little-endian 64-bit word of the 64x64x3 frame, w_k = splitmix64(k) | 1.
"""
import multiprocessing
import os
from concurrent.futures import ProcessPoolExecutor

import numpy as np

from oracle_lib import OracleEnv, hashed_actions

OBS_WORDS = 64 * 64 * 3 // 8
KEYS = ("obs_digest", "rew", "first", "prev_level_seed", "prev_level_complete", "level_seed")


def _weights():
    k = np.arange(OBS_WORDS, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = k + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x | np.uint64(1)


W = _weights()


def obs_digest(rgb):
    """uint8 [n, 64, 64, 3] -> uint64 [n] (wrapping arithmetic, as on the device)."""
    words = np.ascontiguousarray(rgb).reshape(len(rgb), -1).view("<u8")
    with np.errstate(over="ignore"):
        return (words * W).sum(axis=1, dtype=np.uint64)


def pool_size():
    """Worker processes for the oracle leg: the GPU box's CPU share is 16 (os.cpu_count() reports the
    whole machine there)."""
    return max(1, min(16, os.cpu_count() or 1))


def _oracle_chunk(job):
    game, count, offset, stride, steps, seed, kw = job
    o = OracleEnv(game, count, env_offset=offset, stride=stride, **kw)
    glob = offset + stride * np.arange(count, dtype=np.int64)
    out = {k: [] for k in KEYS}
    for t in range(steps + 1):
        if t:
            o.step(hashed_actions(seed, glob, t))
        r = o.observe()
        out["obs_digest"].append(obs_digest(r["rgb"]))
        for k in KEYS[1:]:
            out[k].append(r[k])
    o.close()
    return {k: np.stack(v) for k, v in out.items()}  # [steps + 1, count]


class OraclePopulation:
    """The oracle leg of `names` (a mixed batch plays names[n % len(names)] at env n) over global envs
    [offset, offset + num), started in a worker pool at construction so it runs while the GPU leg
    does.  result() -> dict of [steps + 1, num] arrays in env order."""

    def __init__(self, names, num, steps, seed, offset=0, chunk=1024, **kw):
        G = len(names)
        self.num, self.steps = num, steps
        self.ex = ProcessPoolExecutor(max_workers=pool_size(), mp_context=multiprocessing.get_context("spawn"))
        self.jobs = []  # (future, local env indices)
        for g, name in enumerate(names):
            first = (g - offset) % G  # local index of this game's first env
            local = np.arange(first, num, G)
            for a in range(0, len(local), chunk):
                idx = local[a:a + chunk]
                job = (name, len(idx), offset + int(idx[0]), G, steps, seed, kw)
                self.jobs.append((self.ex.submit(_oracle_chunk, job), idx))

    def result(self):
        out = None
        for fut, idx in self.jobs:
            r = fut.result()
            if out is None:
                out = {k: np.zeros((self.steps + 1, self.num), r[k].dtype) for k in KEYS}
            for k in KEYS:
                out[k][:, idx] = r[k]
        self.ex.shutdown()
        return out


def compare(engine, oracle, names, offset=0):
    """Raise with the first (step, env, field) that differs; engine / oracle: dicts of [steps + 1, num]."""
    for k in KEYS:
        a, b = engine[k], oracle[k]
        if a.shape != b.shape:
            raise AssertionError("%s: shape %s vs %s" % (k, a.shape, b.shape))
        bad = np.argwhere(a != b)
        if len(bad):
            t, e = (int(v) for v in bad[0])
            raise AssertionError("%s differs at step %d, local env %d = global env %d (%s): engine %s oracle %s; "
                                 "%d (step, env) pairs differ, %d envs" % (
                                     k, t, e, offset + e, names[(offset + e) % len(names)], a[t, e], b[t, e],
                                     len(bad), len(np.unique(bad[:, 1]))))
