"""``ProcgenGym3Env`` over the MI355X engine -- same constructor, options and
act/observe/get_info/callmethod surface as the reference (procgen/env.py:90-290),
without the gym3 dependency (absent here): the libenv C ABI is driven directly
through ctypes (procgen_amd/_lib.py).

Two modes:
* host mode (default, the reference's contract): observations land in numpy buffers
  after every ``observe()`` (a device->host copy per step);
* device mode (``device_buffers=True``): observations stay in HBM; ``device_ptrs()``
  exposes them and ``act_hashed`` steps with on-device synthetic actions.
"""
import ctypes
import random

import numpy as np

from . import _lib

MAX_STATE_SIZE = 2 ** 20  # procgen/env.py:13

ENV_NAMES = [
    "bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot",
    "heist", "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot",
]

# procgen/env.py:51-60
EXPLORATION_LEVEL_SEEDS = {
    "coinrun": 1949448038, "caveflyer": 1259048185, "leaper": 1318677581, "jumper": 1434825276,
    "maze": 158988835, "heist": 876640971, "climber": 1561126160, "ninja": 1123500215,
}

# procgen/env.py:64-70
DISTRIBUTION_MODE_DICT = {"easy": 0, "hard": 1, "extreme": 2, "memory": 10, "exploration": 20}

# procgen/env.py:179-196
COMBOS = [("LEFT", "DOWN"), ("LEFT",), ("LEFT", "UP"), ("DOWN",), (), ("UP",), ("RIGHT", "DOWN"), ("RIGHT",),
          ("RIGHT", "UP"), ("D",), ("A",), ("W",), ("S",), ("Q",), ("E",)]


_POOL = None


def _copy(a, chunk=64 << 20):
    """np.copy, split over threads when large (numpy releases the GIL while copying)."""
    if a.nbytes <= chunk or a.shape[0] < 2:
        return a.copy()
    global _POOL
    if _POOL is None:
        import os
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max(1, min(8, len(os.sched_getaffinity(0)))))
    out = np.empty_like(a)
    n = a.shape[0]
    k = min(n, max(2, a.nbytes // chunk))
    list(_POOL.map(lambda i: np.copyto(out[i * n // k:(i + 1) * n // k], a[i * n // k:(i + 1) * n // k]), range(k)))
    return out


def create_random_seed():  # procgen/env.py:73-82 (no mpi4py here)
    return random.SystemRandom().randint(0, 2 ** 31 - 1)


class Discrete:
    def __init__(self, n):
        self.n = n


class TensorType:
    def __init__(self, shape, eltype):
        self.shape = tuple(shape)
        self.eltype = eltype


class ProcgenError(RuntimeError):
    pass


def _check(lib, handle, rc=0):
    err = lib.procgen_last_error(handle)
    if rc < 0 or err:
        msg = lib.procgen_error_string(handle)
        raise ProcgenError("procgen_mi355x error %d: %s" % (err or -rc, msg.decode() if msg else ""))


class BaseProcgenEnv:
    """procgen/env.py:87-227 over libprocgen_mi355x.so."""

    def __init__(self, num, env_name, options, debug=False, rand_seed=None, num_levels=0, start_level=0,
                 use_sequential_levels=False, debug_mode=0, resource_root=None, num_threads=4, render_mode=None,
                 device_buffers=False, env_offset=0, upload_atlas=False, reuse_arrays=False):
        lib = _lib.load()
        self._lib = lib
        if render_mode is None:
            render_human = False
        elif render_mode == "rgb_array":
            render_human = True
        else:
            raise Exception(f"invalid render mode {render_mode}")
        if rand_seed is None:
            rand_seed = create_random_seed()
        self.combos = self.get_combos()
        options = dict(options)
        options.update({
            "env_name": env_name,
            "num_levels": num_levels,
            "start_level": start_level,
            "num_actions": len(self.combos),
            "use_sequential_levels": bool(use_sequential_levels),
            "debug_mode": debug_mode,
            "rand_seed": rand_seed,
            "num_threads": num_threads,
            "render_human": render_human,
        })
        if resource_root is not None:
            options["resource_root"] = resource_root
        if env_offset:
            options["env_offset"] = int(env_offset)
        self.options = options
        self.num = num
        self.env_name = env_name
        opts = _lib.OptionList(options)
        self._handle = lib.libenv_make(num, opts.struct)
        if not self._handle:
            msg = lib.procgen_error_string(None)
            raise ProcgenError("libenv_make failed: %s" % (msg.decode() if msg else "unknown"))
        # libenv_make loaded the images itself (the reference's images_load); a host-built atlas
        # can still replace them before the first reset (procgen_upload_atlas, tests only)
        if upload_atlas:
            from .assets import engine_atlas_for
            atlas = engine_atlas_for(tuple(env_name.split(",")))
            self._atlas = atlas
            rc = lib.procgen_upload_atlas(self._handle, atlas.pixels.ctypes.data, atlas.pixels.size,
                                          atlas.sprites.ctypes.data, atlas.backgrounds.ctypes.data,
                                          atlas.num_backgrounds.ctypes.data, atlas.num_themes.ctypes.data)
            _check(lib, self._handle, rc)

        self.ob_types = self._types(_lib.SPACE_OBSERVATION)
        self.ac_types = self._types(_lib.SPACE_ACTION)
        self.info_types = self._types(_lib.SPACE_INFO)
        act = self.ac_types[0]
        self.ac_space = TensorType((), Discrete(act[3] + 1))
        self.ob_space = {"rgb": TensorType(self.ob_types[0][2], Discrete(256))}
        self.device_buffers = device_buffers
        self.reuse_arrays = reuse_arrays  # gym3 CEnv(reuse_arrays=...): observe() returns the live buffers
        if device_buffers:
            rc = lib.procgen_start(self._handle)
            _check(lib, self._handle, rc)
            self._dev = _lib.pg_device_buffers()
            lib.procgen_device_buffers(self._handle, ctypes.byref(self._dev))
        else:
            self._alloc_host_buffers()

    # ------------------------------------------------------------------ buffers
    def _types(self, space):
        lib = self._lib
        n = lib.libenv_get_tensortypes(self._handle, space, None)
        arr = (_lib.libenv_tensortype * n)()
        lib.libenv_get_tensortypes(self._handle, space, arr)
        out = []
        for t in arr:
            shape = tuple(t.shape[i] for i in range(t.ndim))
            hi = t.high.uint8 if t.dtype == _lib.DTYPE_UINT8 else t.high.int32
            out.append((t.name.decode(), _lib.NP_DTYPE[t.dtype], shape, hi))
        return out

    def _alloc_host_buffers(self):
        n = self.num
        self._ob = {name: np.zeros((n,) + shape, dtype=dt) for name, dt, shape, _ in self.ob_types}
        self._ac = {name: np.zeros((n,) + shape, dtype=dt) for name, dt, shape, _ in self.ac_types}
        self._info = {name: np.zeros((n,) + shape, dtype=dt) for name, dt, shape, _ in self.info_types}
        self._rew = np.zeros(n, dtype=np.float32)
        self._first = np.zeros(n, dtype=np.uint8)

        def ptrs(bufs, types):
            arr = (ctypes.c_void_p * (len(types) * n))()
            for s, (name, dt, shape, _) in enumerate(types):
                b = bufs[name]
                stride = b.strides[0]
                for e in range(n):
                    arr[s * n + e] = b.ctypes.data + e * stride
            return arr

        self._ob_ptrs = ptrs(self._ob, self.ob_types)
        self._ac_ptrs = ptrs(self._ac, self.ac_types)
        self._info_ptrs = ptrs(self._info, self.info_types)
        bufs = _lib.libenv_buffers(self._ob_ptrs, self._ac_ptrs, self._info_ptrs, self._rew.ctypes.data,
                                   self._first.ctypes.data)
        self._lib.libenv_set_buffers(self._handle, ctypes.byref(bufs))
        _check(self._lib, self._handle)

    # ------------------------------------------------------------------ gym3 surface
    def get_combos(self):
        return list(COMBOS)

    def keys_to_act(self, keys_list):  # procgen/env.py:198-221
        result = []
        for keys in keys_list:
            action, max_len = None, -1
            for i, combo in enumerate(self.get_combos()):
                pressed = all(key in keys for key in combo)
                if pressed and max_len < len(combo):
                    action, max_len = i, len(combo)
            result.append(None if action is None else np.array([action]))
        return result

    def act(self, ac):
        # procgen/env.py:223-226: always cast actions to int32
        ac = np.asarray(ac).astype(np.int32).reshape(self.num)
        if self.device_buffers:
            raise ProcgenError("device-buffer env: use act_device / act_hashed")
        self._ac["action"][:] = ac
        self._lib.libenv_act(self._handle)
        _check(self._lib, self._handle)

    def observe(self):
        if self.device_buffers:
            rc = self._lib.procgen_wait(self._handle)
            _check(self._lib, self._handle, rc)
            return None
        self._lib.libenv_observe(self._handle)
        _check(self._lib, self._handle)
        if self.reuse_arrays:
            return self._rew, self._ob, self._first.view(bool)
        # gym3 CEnv._maybe_copy: fresh arrays every observe (a threaded copy for large batches)
        return self._rew.copy(), {k: _copy(v) for k, v in self._ob.items()}, self._first.astype(bool)

    def get_info(self):
        """gym3 contract: one dict per env (procgen/env.py via gym3 CEnv.get_info)."""
        if self.device_buffers:
            raise ProcgenError("device-buffer env: read device_ptrs() instead")
        items = list(self._info.items())
        return [{k: (v[i] if v.ndim == 1 else v[i].copy()) for k, v in items} for i in range(self.num)]

    def get_info_arrays(self):
        """The info tensors of the last observe() as arrays [num, ...] (no per-env dicts): the live
        buffers under reuse_arrays (as observe() returns them), else fresh copies -- the latent
        `grid` alone is 4.9 KB per env (declared for every game, vecgame.cpp:270-316), so large
        batches copy it over threads like the observations."""
        if self.device_buffers:
            raise ProcgenError("device-buffer env: read device_ptrs() instead")
        if self.reuse_arrays:
            return self._info
        return {k: _copy(v) for k, v in self._info.items()}

    def callmethod(self, method, *args, **kwargs):
        return getattr(self, method)(*args, **kwargs)

    def get_state(self):  # procgen/env.py:164-171
        buf = ctypes.create_string_buffer(MAX_STATE_SIZE)
        out = []
        for i in range(self.num):
            n = self._lib.get_state(self._handle, i, buf, MAX_STATE_SIZE)
            if n < 0:
                raise ProcgenError("get_state failed for env %d" % i)
            out.append(bytes(buf.raw[:n]))
        return out

    def set_state(self, states):  # procgen/env.py:173-177
        assert len(states) == self.num
        for i, s in enumerate(states):
            self._lib.set_state(self._handle, i, s, len(s))
        _check(self._lib, self._handle)
        if not self.device_buffers:
            self._lib.libenv_observe(self._handle)

    # ------------------------------------------------------------------ device extensions
    def act_hashed(self, seed, t):
        rc = self._lib.procgen_act_hashed(self._handle, seed, t)
        _check(self._lib, self._handle, rc)

    def act_device(self, ptr):
        rc = self._lib.procgen_act_device(self._handle, ptr)
        _check(self._lib, self._handle, rc)

    def wait(self):
        rc = self._lib.procgen_wait(self._handle)
        _check(self._lib, self._handle, rc)

    def read_envs(self, env_ids):
        """Outputs of a few envs (after the enqueued steps finish) without copying the batch:
        dict of rgb [k,64,64,3], rew, first, prev_level_seed, prev_level_complete, level_seed."""
        ids = np.ascontiguousarray(env_ids, dtype=np.int32).reshape(-1)
        k = ids.size
        out = dict(rgb=np.zeros((k, 64, 64, 3), np.uint8), rew=np.zeros(k, np.float32), first=np.zeros(k, np.uint8),
                   prev_level_seed=np.zeros(k, np.int32), prev_level_complete=np.zeros(k, np.uint8),
                   level_seed=np.zeros(k, np.int32))
        rc = self._lib.procgen_read_envs(self._handle, ids.ctypes.data, k, *[out[n].ctypes.data for n in (
            "rgb", "rew", "first", "prev_level_seed", "prev_level_complete", "level_seed")])
        _check(self._lib, self._handle, rc)
        return out

    def read_outputs(self):
        """Every env's outputs after the enqueued steps finish, with the observation as a 64-bit
        digest per env computed on the device (procgen_read_outputs): dict of obs_digest (uint64),
        rew, first, prev_level_seed, prev_level_complete, level_seed -- [num] each."""
        n = self.num
        out = dict(obs_digest=np.zeros(n, np.uint64), rew=np.zeros(n, np.float32), first=np.zeros(n, np.uint8),
                   prev_level_seed=np.zeros(n, np.int32), prev_level_complete=np.zeros(n, np.uint8),
                   level_seed=np.zeros(n, np.int32))
        rc = self._lib.procgen_read_outputs(self._handle, *[out[k].ctypes.data for k in (
            "obs_digest", "rew", "first", "prev_level_seed", "prev_level_complete", "level_seed")])
        _check(self._lib, self._handle, rc)
        return out

    def set_latent_state(self, env_idx, grid, agent_pos, exit_pos):
        """MinerGame::game_set_state (procgen/src/games/miner.cpp:423-449, the fork's JS setState):
        `grid` [h, w] (or flat with an explicit shape) of cell values, agent and exit cell positions.
        A DEAD_PLAYER (12) cell kills the agent.  The env's frame is re-rendered."""
        g = np.ascontiguousarray(grid, dtype=np.int32)
        h, w = (g.shape if g.ndim == 2 else (1, g.size))
        rc = self._lib.procgen_set_latent_state(self._handle, int(env_idx), g.ctypes.data, int(w), int(h),
                                                int(agent_pos[0]), int(agent_pos[1]), int(exit_pos[0]), int(exit_pos[1]))
        _check(self._lib, self._handle, rc)

    def set_obs_buffer(self, ptr):
        """Render later steps into the device buffer at `ptr` (uint8 [num,64,64,3]); None = own tensor.
        The engine keeps the raw pointer: unbind (None) before the buffer is freed.  A no-op once the
        env is closed (nothing holds the pointer any more)."""
        if not getattr(self, "_handle", None):
            return
        rc = self._lib.procgen_set_obs_buffer(self._handle, ptr)
        _check(self._lib, self._handle, rc)

    def device_ptrs(self):
        d = _lib.pg_device_buffers()
        self._lib.procgen_device_buffers(self._handle, ctypes.byref(d))
        return d

    def set_timing(self, on):
        self._lib.procgen_set_timing(self._handle, int(on))

    def kernel_times(self):
        """(timed steps, [step, reset, render, wall] ms, {game: [step, reset, render] ms}): the first
        three are sums over a mixed batch's games (concurrent streams), wall is the step's span."""
        names = self.env_name.split(",")
        k = 4 + 3 * len(names)
        out = (ctypes.c_float * k)()
        n = self._lib.procgen_kernel_times(self._handle, out, k)
        vals = list(out)
        per_game = {nm: vals[4 + 3 * g:7 + 3 * g] for g, nm in enumerate(names)}
        return n, vals[:4], per_game

    def num_parts(self):
        """Chains one act of this (single-game) env is split into (PROCGEN_MI355X_PARTS)."""
        return int(self._lib.procgen_num_parts(self._handle))

    def debug_env(self, i):
        buf = np.zeros(128, dtype=np.int32)
        self._lib.procgen_debug_env(self._handle, i, buf.ctypes.data, buf.nbytes)
        return buf

    def is_open(self):
        return bool(getattr(self, "_handle", None))

    def close(self):
        if getattr(self, "_handle", None):
            self._lib.libenv_close(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ProcgenGym3Env(BaseProcgenEnv):
    """procgen/env.py:229-273."""

    def __init__(self, num, env_name, center_agent=True, use_backgrounds=True, use_monochrome_assets=False,
                 restrict_themes=False, use_generated_assets=False, paint_vel_info=False, distribution_mode="hard",
                 **kwargs):
        assert distribution_mode in DISTRIBUTION_MODE_DICT, f'"{distribution_mode}" is not a valid distribution mode.'
        if distribution_mode == "exploration":
            assert env_name in EXPLORATION_LEVEL_SEEDS, f"{env_name} does not support exploration mode"
            distribution_mode = DISTRIBUTION_MODE_DICT["hard"]
            assert "num_levels" not in kwargs, "exploration mode overrides num_levels"
            kwargs["num_levels"] = 1
            assert "start_level" not in kwargs, "exploration mode overrides start_level"
            kwargs["start_level"] = EXPLORATION_LEVEL_SEEDS[env_name]
        else:
            distribution_mode = DISTRIBUTION_MODE_DICT[distribution_mode]
        options = {
            "center_agent": bool(center_agent),
            "use_generated_assets": bool(use_generated_assets),
            "use_monochrome_assets": bool(use_monochrome_assets),
            "restrict_themes": bool(restrict_themes),
            "use_backgrounds": bool(use_backgrounds),
            "paint_vel_info": bool(paint_vel_info),
            "distribution_mode": distribution_mode,
        }
        super().__init__(num, env_name, options, **kwargs)
