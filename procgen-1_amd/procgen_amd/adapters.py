"""Callers of the step path: the reference's baselines-VecEnv and gym adapters.

The reference builds these from gym3 (`procgen/env.py:276-290`: `ToBaselinesVecEnv`,
`ProcgenEnv`) and gym (`procgen/gym_registration.py:6-34`: `ExtractDictObWrapper` +
`ToGymEnv`, registered as ``procgen-<name>-v0``).  Neither gym nor gym3 is installed in this
image, so the adapters are restated here over any gym3-style env (``num``, ``act``,
``observe`` -> ``(rew, ob, first)``, ``get_info``, ``ob_space`` / ``ac_space``) with gym3's
published semantics (gym3 0.3.3 ``interop.py``):

* reset() only observes -- procgen envs reset themselves (auto-reset inside step,
  `game.cpp:160-171`); a reset() away from an episode start warns and does not reset.
* step() = act + observe; ``done`` is the ``first`` flag of the new observation, which is
  already the next episode's first frame.
* infos are ``env.get_info()``, one dict per env.

``render_mode="rgb_array"`` (the 512x512 antialiased ``info["rgb"]``) is built for all 16 games,
jumper's compass included in every distribution mode (drawn on the device, ``hc_draw_compass``);
``render_mode="human"`` needs gym3's ViewerWrapper window, which this build has not.
"""
import numpy as np

from .env import ENV_NAMES, ProcgenGym3Env


class ToBaselinesVecEnv:
    """gym3.ToBaselinesVecEnv + procgen's render() (procgen/env.py:276-286)."""

    # "human" needs gym3's viewer window; render("rgb_array") returns env 0's info["rgb"] (the 512x512
    # frame of render_mode="rgb_array") or else its 64x64 observation
    metadata = {"render.modes": ["rgb_array"], "video.frames_per_second": 15}

    def __init__(self, env):
        self.env = env
        self.num_envs = env.num
        self.observation_space = env.ob_space
        self.action_space = env.ac_space
        self._pending = False

    def reset(self):
        _rew, ob, first = self.env.observe()
        if not np.asarray(first).all():
            print("Warning: you called reset() with an env that was not at the start of an episode, "
                  "this will not reset the env")
        return ob

    def step_async(self, actions):
        self.env.act(actions)
        self._pending = True

    def step_wait(self):
        rew, ob, first = self.env.observe()
        self._pending = False
        return ob, rew, first, self.env.get_info()

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def render(self, mode="human"):
        info = self.env.get_info()[0]
        _, ob, _ = self.env.observe()
        if mode == "rgb_array":
            if "rgb" in info:
                return info["rgb"]
            return ob["rgb"][0]
        raise NotImplementedError("render(mode=%r): no viewer window in this build" % mode)

    def close(self):
        self.env.close()

    @property
    def unwrapped(self):
        return self


def ProcgenEnv(num_envs, env_name, **kwargs):  # procgen/env.py:289-290
    return ToBaselinesVecEnv(ProcgenGym3Env(num=num_envs, env_name=env_name, **kwargs))


class ToGymEnv:
    """gym3.ExtractDictObWrapper(key="rgb") + gym3.ToGymEnv over a num=1 env
    (procgen/gym_registration.py:24-26): single-env reset / step on the rgb frame."""

    metadata = {"render.modes": ["rgb_array"]}

    def __init__(self, env, key="rgb"):
        if env.num != 1:
            raise ValueError("ToGymEnv needs a num=1 env, got num=%d" % env.num)
        self.env = env
        self.key = key
        self.observation_space = env.ob_space[key]
        self.action_space = env.ac_space

    def reset(self):
        _rew, ob, _first = self.env.observe()
        return ob[self.key][0]

    def step(self, action):
        self.env.act(np.array([action], dtype=np.int32))
        rew, ob, first = self.env.observe()
        return ob[self.key][0], float(rew[0]), bool(first[0]), self.env.get_info()[0]

    def render(self, mode="rgb_array"):  # gym3 ToGymEnv.render: the info dict's "rgb" entry
        if mode != "rgb_array":
            raise NotImplementedError("render(mode=%r): no viewer window in this build" % mode)
        info = self.env.get_info()[0]
        if "rgb" in info:
            return info["rgb"]
        _, ob, _ = self.env.observe()
        return ob[self.key][0]

    def close(self):
        self.env.close()


def make_env(render_mode=None, render=False, **kwargs):  # procgen/gym_registration.py:6-26
    if render:
        render_mode = "human"
    if render_mode == "human":
        # the reference wraps the env in gym3's ViewerWrapper (a window fed by info["rgb"])
        raise NotImplementedError("make_env(render_mode='human'): no viewer window in this build; use "
                                  "render_mode='rgb_array' and env.render()")
    return ToGymEnv(ProcgenGym3Env(num=1, num_threads=0, render_mode=render_mode, **kwargs))


ENV_IDS = {"procgen-%s-v0" % name: name for name in ENV_NAMES}


def register_environments():  # procgen/gym_registration.py:29-34
    """Registers procgen-<name>-v0 with gym when gym is importable; returns the id -> name map."""
    try:
        from gym.envs.registration import register
    except ImportError:
        return dict(ENV_IDS)
    for env_id, name in ENV_IDS.items():
        register(id=env_id, entry_point="procgen_amd.adapters:make_env", kwargs={"env_name": name})
    return dict(ENV_IDS)
