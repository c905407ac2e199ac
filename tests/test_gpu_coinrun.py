"""GPU parity: the HIP engine (through the libenv C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): bit-exact reward / done(first) / level seeds and bit-exact
RGB for coinrun (its game logic has no transcendental libm call).  Cases mirror the
reference's own tests (procgen/env_test.py: seeding, determinism) plus option coverage
and sampled envs of the full 65,536-env configuration.
"""
import os

import numpy as np
import pytest

from oracle_lib import OracleEnv, hashed_actions

pytestmark = pytest.mark.gpu

KEYS = ["rew", "first", "prev_level_seed", "prev_level_complete", "level_seed"]


def make_gpu(num, **kw):
    from procgen_amd import ProcgenGym3Env
    return ProcgenGym3Env(num=num, env_name="coinrun", **kw)


def gpu_obs(env):
    rew, ob, first = env.observe()
    info = env.get_info()
    return dict(rgb=ob["rgb"], rew=rew, first=first.astype(np.uint8),
                prev_level_seed=np.array([i["prev_level_seed"] for i in info], np.int32),
                prev_level_complete=np.array([i["prev_level_complete"] for i in info], np.uint8),
                level_seed=np.array([i["level_seed"] for i in info], np.int32))


def assert_same(g, o, step, idx=None):
    sel = slice(None) if idx is None else idx
    for k in KEYS:
        np.testing.assert_array_equal(g[k][sel], o[k], err_msg="%s differs at step %d" % (k, step))
    if not np.array_equal(g["rgb"][sel], o["rgb"]):
        gg = g["rgb"][sel]
        diff = np.argwhere(np.any(gg != o["rgb"], axis=-1))
        vals = ["%s: %s vs %s" % (tuple(p), gg[tuple(p)].tolist(), o["rgb"][tuple(p)].tolist()) for p in diff[:8]]
        raise AssertionError("rgb differs at step %d (idx %s): %d pixels, (env,row,col): engine vs oracle\n  %s"
                             % (step, sel, len(diff), "\n  ".join(vals)))


PGENV_FIELDS = {1: "action", 2: "cur_time", 27: "num_ents", 28: "agent_erased", 33: "move_action",
                34: "special_action", 38: "action_vx", 39: "action_vy", 59: "has_support", 60: "facing_right",
                61: "is_on_crate", 64: "rg_mti", 67: "grid8_ok"}
FLOAT_FIELDS = {38, 39}


def describe_engine_env(env, i):
    """A few PGEnv members of engine env i (procgen_debug_env), for failure messages."""
    try:
        buf = env.debug_env(i)
    except Exception as e:  # pragma: no cover - diagnostics only
        return "debug_env failed: %s" % e
    out = []
    for k, name in PGENV_FIELDS.items():
        v = buf[k:k + 1].view(np.float32)[0] if k in FLOAT_FIELDS else int(buf[k])
        out.append("%s=%s" % (name, v))
    return " ".join(out)


def run_pair(num, steps, oracle_kw, gpu_kw, seed=0):
    env = make_gpu(num, **gpu_kw)
    orc = OracleEnv("coinrun", num, **oracle_kw)
    rng = np.random.RandomState(seed)
    assert_same(gpu_obs(env), orc.observe(), 0)
    episodes = 0
    for t in range(1, steps + 1):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        env.act(act)
        orc.step(act)
        g = gpu_obs(env)
        assert_same(g, orc.observe(), t)
        episodes += int(g["first"].sum())
    env.close()
    return episodes


def test_parity_hard_200_levels():
    n = run_pair(16, 400, dict(num_levels=200, start_level=0, rand_seed=0),
                 dict(num_levels=200, start_level=0, rand_seed=0))
    assert n > 0  # resets exercised


def test_parity_unbounded_levels_seed7():
    run_pair(8, 300, dict(num_levels=0, rand_seed=7), dict(num_levels=0, rand_seed=7), seed=3)


def test_parity_easy_no_center():
    run_pair(8, 200, dict(num_levels=50, rand_seed=1, distribution_mode=0, center_agent=0),
             dict(num_levels=50, rand_seed=1, distribution_mode="easy", center_agent=False), seed=5)


def test_parity_no_backgrounds_restrict_themes_sequential():
    run_pair(8, 300, dict(num_levels=10, rand_seed=2, use_backgrounds=0, restrict_themes=1, use_sequential_levels=1),
             dict(num_levels=10, rand_seed=2, use_backgrounds=False, restrict_themes=True, use_sequential_levels=True),
             seed=9)


def test_force_reset_action():
    # action -1 forces a reset (game.cpp:140-143)
    env = make_gpu(4, num_levels=100, rand_seed=4)
    orc = OracleEnv("coinrun", 4, num_levels=100, rand_seed=4)
    for t in range(1, 40):
        act = np.array([(t * 7 + k) % 15 if (t + k) % 11 else -1 for k in range(4)], np.int32)
        env.act(act)
        orc.step(act)
        assert_same(gpu_obs(env), orc.observe(), t)


def test_seeding_like_reference():
    # procgen/env_test.py:7-30
    def obs(level):
        e = make_gpu(1, num_levels=1, start_level=level)
        e.act(np.zeros(1))
        _, o, _ = e.observe()
        e.close()
        return o["rgb"]
    o1, o2, o3 = obs(0), obs(0), obs(1)
    assert np.array_equal(o1, o2)
    assert not np.array_equal(o1, o3)


def test_determinism_like_reference():
    # procgen/env_test.py:33-52
    def collect():
        rng = np.random.RandomState(0)
        env = make_gpu(2, rand_seed=23)
        _, obs, _ = env.observe()
        out = [obs["rgb"]]
        for _ in range(128):
            env.act(rng.randint(low=0, high=env.ac_space.eltype.n, size=(env.num,), dtype=np.int32))
            _, obs, _ = env.observe()
            out.append(obs["rgb"])
        env.close()
        return np.array(out)
    assert np.array_equal(collect(), collect())


def test_state_roundtrip():
    env = make_gpu(4, num_levels=20, rand_seed=11)
    rng = np.random.RandomState(1)
    for _ in range(30):
        env.act(rng.randint(0, 15, size=4))
        env.observe()
    states = env.get_state()
    acts = [rng.randint(0, 15, size=4) for _ in range(60)]
    a = []
    for ac in acts:
        env.act(ac)
        a.append(gpu_obs(env))
    env.set_state(states)
    for k, ac in enumerate(acts):
        env.act(ac)
        b = gpu_obs(env)
        for key in KEYS + ["rgb"]:
            np.testing.assert_array_equal(a[k][key], b[key])
    env.close()


def test_full_size_sampled_parity():
    """65,536 envs (BASELINE config 2), hashed actions; sampled envs against the oracle."""
    num = 65536
    env = make_gpu(num, num_levels=200, start_level=0, rand_seed=0)
    # includes the crate-pile envs (CRATE_PILE_ENVS: the slow-env launch path at scale) and both parts'
    # edges (the default 2-part split at 32,768)
    sample = [0, 1, 2, 56, 63, 64, 1000, 1551, 2240, 3056, 3350, 3868, 4095, 12345, 30000, 32767, 32768, 48596,
              50001, 65534, 65535]
    orcs = [OracleEnv("coinrun", 1, env_offset=i, num_levels=200, rand_seed=0) for i in sample]
    ids = np.arange(num)
    g = gpu_obs(env)
    for k, o in zip(sample, orcs):
        assert_same(g, o.observe(), 0, idx=slice(k, k + 1))
    for t in range(1, 151):
        act = hashed_actions(0x5EED, ids, t)
        env.act(act)
        g = gpu_obs(env)
        for k, o in zip(sample, orcs):
            o.step(act[k:k + 1])
            try:
                assert_same(g, o.observe(), t, idx=slice(k, k + 1))
            except AssertionError as e:
                dump = os.environ.get("PG_FLAKE_DUMP")
                if dump:  # diagnostics: frames + engine snapshot of the failing env
                    import ctypes
                    buf = ctypes.create_string_buffer(1 << 20)
                    nb = env._lib.get_state(env._handle, k, buf, 1 << 20)
                    np.savez(dump, engine=g["rgb"][k], oracle=o.observe()["rgb"][0], step=t, env=k,
                             state=np.frombuffer(buf.raw[:max(nb, 0)], np.uint8), odebug=o.debug(0))
                raise AssertionError("%s\n  global env %d, action %d\n  engine: %s\n  oracle debug: %s"
                                     % (e, k, act[k], describe_engine_env(env, k), o.debug(0).tolist()))
    env.close()


def test_gpu_vs_committed_fixture():
    """Engine vs the committed trajectory fixture (tests/golden/coinrun_oracle_traj.npz):
    global envs of the 65,536-env config (env_offset places a 1-env shard at that index)."""
    import os
    import zlib
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "coinrun_oracle_traj.npz"), allow_pickle=False)
    seed = int(z["action_seed"])
    frames_at = list(z["frame_steps"])
    for k, e in enumerate(z["envs"]):
        env = make_gpu(1, num_levels=200, start_level=0, rand_seed=0, env_offset=int(e))
        for t in range(int(z["steps"]) + 1):
            if t:
                env.act(hashed_actions(seed, [int(e)], t))
            g = gpu_obs(env)
            assert g["rew"][0] == z["rew"][t, k] and g["first"][0] == z["first"][t, k], (e, t)
            assert g["level_seed"][0] == z["level_seed"][t, k] and g["prev_level_seed"][0] == z["prev_level_seed"][t, k]
            assert zlib.crc32(g["rgb"][0].tobytes()) == z["rgb_crc32"][t, k], "env %d step %d" % (e, t)
            if t in frames_at:
                np.testing.assert_array_equal(g["rgb"][0], z["frames"][frames_at.index(t), k])
        env.close()


def test_gpu_determinism_two_engines():
    """Two identical engines driven with the same actions produce identical outputs
    (reference env_test.py determinism check, at scale: 16,384 envs, after other envs in
    this process have dirtied device memory)."""
    num = 16384
    a = make_gpu(num, num_levels=200, start_level=0, rand_seed=0)
    b = make_gpu(num, num_levels=200, start_level=0, rand_seed=0)
    rng = np.random.RandomState(7)
    for t in range(60):
        if t:
            act = rng.randint(0, 15, size=num).astype(np.int32)
            a.act(act)
            b.act(act)
        ga, gb = gpu_obs(a), gpu_obs(b)
        for k in KEYS + ["rgb"]:
            np.testing.assert_array_equal(ga[k], gb[k], err_msg="%s differs at step %d" % (k, t))
    a.close()
    b.close()


# Global env indices of the 200-level config whose levels hold crate piles (duplicate / stacked
# crates): with action seed 0, their steps reach 280-520 sub_step calls (the push recursion
# revisiting the same child up to 2^5 times) -- the steps the engine's push-chain memo
# (pg_step.hip memo_find) replays instead of walking.  Found with the oracle's diagnostic
# sub_step counter over envs 0..4095 (and 48596, the round-3 census tail env).
CRATE_PILE_ENVS = [56, 1551, 2240, 3056, 3350, 3868, 48596]


@pytest.mark.parametrize("e", CRATE_PILE_ENVS)
def test_crate_pile_push_chains(e):
    """Bit-exact through the deepest push chains: every step of 320, 1-env shard at global index e."""
    env = make_gpu(1, num_levels=200, start_level=0, rand_seed=0, env_offset=e)
    orc = OracleEnv("coinrun", 1, env_offset=e, num_levels=200, start_level=0, rand_seed=0)
    assert_same(gpu_obs(env), orc.observe(), 0)
    for t in range(320):
        act = hashed_actions(0, [e], t)
        env.act(act)
        orc.step(act)
        try:
            assert_same(gpu_obs(env), orc.observe(), t + 1)
        except AssertionError as err:
            raise AssertionError("%s\n  global env %d\n  engine: %s\n  oracle debug: %s"
                                 % (err, e, describe_engine_env(env, 0), orc.debug(0).tolist()))
    env.close()
