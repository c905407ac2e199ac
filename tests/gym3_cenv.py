"""A gym3 ``CEnv`` stand-in for tests: drives libprocgen_mi355x.so with exactly the call
sequence gym3's cffi binding makes for the reference (procgen/env.py:152-170 ->
gym3 libenv.CEnv): ``libenv_make`` -> ``libenv_get_tensortypes`` (count, then fill) for the
observation, action and info spaces -> ``libenv_set_buffers`` with per-env pointers at
``space_idx * num + env_idx`` (vecgame.cpp:30-40, 74-83) -> (``libenv_act``,
``libenv_observe``)* -> ``libenv_close``.  It resolves only the libenv symbols: no
``procgen_*`` extension is looked up or called (test infrastructure; gym3 is not installed).
"""
import ctypes

import numpy as np

LIBENV_SYMBOLS = ("libenv_version", "libenv_make", "libenv_get_tensortypes", "libenv_set_buffers",
                  "libenv_observe", "libenv_act", "libenv_close")


class RecordingLib:
    """Resolves symbols of a CDLL on demand and records every name looked up."""

    def __init__(self, path):
        self._dll = ctypes.CDLL(path)
        self.looked_up = []

    def __getattr__(self, name):
        self.looked_up.append(name)
        return getattr(self._dll, name)


def _bind(lib):
    from procgen_amd import _lib as L
    sig = {
        "libenv_version": (ctypes.c_int, []),
        "libenv_make": (ctypes.c_void_p, [ctypes.c_int, L.libenv_options]),
        "libenv_get_tensortypes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(L.libenv_tensortype)]),
        "libenv_set_buffers": (None, [ctypes.c_void_p, ctypes.POINTER(L.libenv_buffers)]),
        "libenv_observe": (None, [ctypes.c_void_p]),
        "libenv_act": (None, [ctypes.c_void_p]),
        "libenv_close": (None, [ctypes.c_void_p]),
    }
    fns = {}
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
        fns[name] = f
    return fns


class CEnv:
    def __init__(self, lib, num, options):
        from procgen_amd import _lib as L
        self.L = L
        self.f = _bind(lib)
        self.num = num
        self._opts = L.OptionList(options)
        self.handle = self.f["libenv_make"](num, self._opts.struct)
        if not self.handle:
            raise RuntimeError("libenv_make returned NULL")
        self.spaces = {}
        for name, code in (("ob", L.SPACE_OBSERVATION), ("ac", L.SPACE_ACTION), ("info", L.SPACE_INFO)):
            n = self.f["libenv_get_tensortypes"](self.handle, code, None)
            arr = (L.libenv_tensortype * n)()
            self.f["libenv_get_tensortypes"](self.handle, code, arr)
            self.spaces[name] = [(t.name.decode(), L.NP_DTYPE[t.dtype], tuple(t.shape[i] for i in range(t.ndim)))
                                 for t in arr]
        self.bufs = {s: {nm: np.zeros((num,) + sh, dt) for nm, dt, sh in types} for s, types in self.spaces.items()}
        self.rew = np.zeros(num, np.float32)
        self.first = np.zeros(num, np.uint8)
        self._ptrs = {}
        for s, types in self.spaces.items():
            arr = (ctypes.c_void_p * (len(types) * num))()
            for i, (nm, _, _) in enumerate(types):
                b = self.bufs[s][nm]
                for e in range(num):
                    arr[i * num + e] = b.ctypes.data + e * b.strides[0]
            self._ptrs[s] = arr
        self._c = L.libenv_buffers(self._ptrs["ob"], self._ptrs["ac"], self._ptrs["info"], self.rew.ctypes.data,
                                   self.first.ctypes.data)
        self.f["libenv_set_buffers"](self.handle, ctypes.byref(self._c))

    def observe(self):
        self.f["libenv_observe"](self.handle)
        return self.rew.copy(), {k: v.copy() for k, v in self.bufs["ob"].items()}, self.first.copy()

    def act(self, ac):
        self.bufs["ac"]["action"][:] = np.asarray(ac, np.int32)
        self.f["libenv_act"](self.handle)

    def info(self):
        return {k: v.copy() for k, v in self.bufs["info"].items()}

    def close(self):
        if self.handle:
            self.f["libenv_close"](self.handle)
            self.handle = None
