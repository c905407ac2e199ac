"""CPU checks of the whole-population helpers (tests/population.py) that the GPU population tests
rely on: the strided oracle reproduces single-env oracles at the same global indices (one game's envs
of a mixed batch, vecgame.cpp:357-358), the worker-pool leg assembles envs in order, and the digest
is the documented wrapping sum."""
import numpy as np

from oracle_lib import OracleEnv, hashed_actions
from population import KEYS, OBS_WORDS, OraclePopulation, compare, obs_digest


def _single(name, n, steps, seed, **kw):
    o = OracleEnv(name, 1, env_offset=n, **kw)
    out = {k: [] for k in KEYS}
    for t in range(steps + 1):
        if t:
            o.step(hashed_actions(seed, [n], t))
        r = o.observe()
        out["obs_digest"].append(obs_digest(r["rgb"])[0])
        for k in KEYS[1:]:
            out[k].append(r[k][0])
    o.close()
    return {k: np.array(v) for k, v in out.items()}


def test_digest_definition():
    rng = np.random.RandomState(0)
    rgb = rng.randint(0, 256, size=(3, 64, 64, 3)).astype(np.uint8)
    got = obs_digest(rgb)

    def mix(x):
        m = (1 << 64) - 1
        x = (x + 0x9E3779B97F4A7C15) & m
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
        return x ^ (x >> 31)

    for e in range(3):
        b = rgb[e].tobytes()
        ref = sum(int.from_bytes(b[8 * k:8 * k + 8], "little") * (mix(k) | 1) for k in range(OBS_WORDS)) % (1 << 64)
        assert int(got[e]) == ref


def test_strided_oracle_matches_single_envs():
    o = OracleEnv("heist", 4, env_offset=1, stride=2, num_levels=0, rand_seed=5)
    glob = 1 + 2 * np.arange(4)
    singles = [_single("heist", int(n), 12, 0x77, num_levels=0, rand_seed=5) for n in glob]
    for t in range(13):
        if t:
            o.step(hashed_actions(0x77, glob, t))
        r = o.observe()
        for j in range(4):
            assert obs_digest(r["rgb"][j:j + 1])[0] == singles[j]["obs_digest"][t]
            assert r["level_seed"][j] == singles[j]["level_seed"][t]
    o.close()


def test_population_pool_assembles_mixed_batch_in_env_order():
    names, num, steps, seed = ["maze", "heist"], 10, 8, 0x99
    pop = OraclePopulation(names, num, steps, seed, offset=3, chunk=2, num_levels=0, rand_seed=2).result()
    ref = {k: np.zeros_like(v) for k, v in pop.items()}
    for e in range(num):
        s = _single(names[(3 + e) % 2], 3 + e, steps, seed, num_levels=0, rand_seed=2)
        for k in KEYS:
            ref[k][:, e] = s[k]
    compare(pop, ref, names, offset=3)
